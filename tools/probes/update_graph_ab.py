"""Whole captured PPO update (Go2, 4096 envs x 24 steps, 5 epochs x 4 mini-batches: 20 fused
optimizer steps replayed as one HIP graph) under each GEMM staging mode
(pmlp_set_gemm_staging 0 / 1 / 2 / 3) and forward form (f = 1: the one-launch fused MLP
forward, 0: per-layer GEMMs), interleaved rounds in one process; graphs captured per mode.
Usage: update_graph_ab.py [staging:fused,...]   e.g. 0:0,2:0,2:1"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))
import torch  # noqa: E402

from rsl_rl.algorithms import PPO  # noqa: E402
from rsl_rl.modules import ActorCritic, mfma_mlp as mm  # noqa: E402

MODES = [tuple(int(v) for v in x.split(":")) if ":" in x else (int(x), 1)
         for x in (sys.argv[1] if len(sys.argv) > 1 else "0:0,2:0,2:1").split(",")]
N, T, O, A = 4096, 24, 48, 12
lib = mm.load()
lib.pmlp_set_gemm_staging.argtypes = [C.c_int32]
algs = {}
for mode in MODES:
    torch.manual_seed(0)
    ac = ActorCritic(O, O, A, [512, 256, 128], [512, 256, 128]).cuda()
    alg = PPO(ac, num_learning_epochs=5, num_mini_batches=4, device="cuda")
    alg.init_storage(N, T, [O], [None], [A])
    st = alg.storage
    g = torch.Generator(device="cuda").manual_seed(1)
    for k in ("observations", "actions", "values", "returns", "advantages", "mu"):
        getattr(st, k).copy_(torch.randn(getattr(st, k).shape, device="cuda", generator=g))
    st.sigma.fill_(1.0)
    st.actions_log_prob.copy_(-12.0 + torch.randn(st.actions_log_prob.shape, device="cuda", generator=g))
    lib.pmlp_set_gemm_staging(mode[0])
    alg._fused.fused_fwd = alg._fused.fused_fwd and bool(mode[1])
    for _ in range(3):  # eager, then capture + replay
        st.step = T
        alg.update()
    assert alg._fgraph is not None
    algs[mode] = alg
torch.cuda.synchronize()
res = {m: [] for m in MODES}
for rnd in range(5):
    for m in MODES:
        alg = algs[m]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            alg._fgraph.replay()
        e1.record()
        torch.cuda.synchronize()
        res[m].append(e0.elapsed_time(e1) / 5)
for m in MODES:
    v = sorted(res[m])
    print(f"staging {m[0]} fused-forward {m[1]}: update {v[len(v) // 2]:.3f} ms median, {v[0]:.3f} min  ({', '.join(f'{x:.3f}' for x in res[m])})")
