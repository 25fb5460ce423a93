"""Whole captured PPO update (Go2, 4096 envs x 24 steps, 5 epochs x 4 mini-batches: 20 fused
optimizer steps replayed as one HIP graph) with each layer's weight and input gradients in one
launch (pmlp_gemm_pair) and as two launches, interleaved rounds in one process."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))
import torch  # noqa: E402

from rsl_rl.algorithms import PPO  # noqa: E402
from rsl_rl.modules import ActorCritic  # noqa: E402

N, T, O, A = 4096, 24, 48, 12
algs = {}
for pair in (False, True):
    torch.manual_seed(0)
    ac = ActorCritic(O, O, A, [512, 256, 128], [512, 256, 128]).cuda()
    alg = PPO(ac, num_learning_epochs=5, num_mini_batches=4, device="cuda")
    alg.init_storage(N, T, [O], [None], [A])
    alg._fused.pair_backward = pair
    st = alg.storage
    g = torch.Generator(device="cuda").manual_seed(1)
    for k in ("observations", "actions", "values", "returns", "advantages", "mu"):
        getattr(st, k).copy_(torch.randn(getattr(st, k).shape, device="cuda", generator=g))
    st.sigma.fill_(1.0)
    st.actions_log_prob.copy_(-12.0 + torch.randn(st.actions_log_prob.shape, device="cuda", generator=g))
    for _ in range(3):  # eager, then capture + replay
        st.step = T
        alg.update()
    assert alg._fgraph is not None
    algs[pair] = alg
torch.cuda.synchronize()
res = {m: [] for m in algs}
for rnd in range(7):
    for m, alg in algs.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            alg._fgraph.replay()
        e1.record()
        torch.cuda.synchronize()
        res[m].append(e0.elapsed_time(e1) / 5)
for m in algs:
    v = sorted(res[m])
    print(f"paired backward {m}: update {v[len(v) // 2]:.3f} ms median, {v[0]:.3f} min  ({', '.join(f'{x:.3f}' for x in res[m])})")
