"""Captured Go2 PPO update (4096 envs x 24 steps, 5 x 4 mini-batches, one HIP graph) with the
first layer's split-K weight gradient at several slab counts (the shipped _ksplit: 32 slabs of
768 rows), interleaved rounds in one process.
usage: python tools/probes/update_ks0_ab.py [slabs ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))
import torch  # noqa: E402

from rsl_rl.algorithms import PPO  # noqa: E402
from rsl_rl.modules import ActorCritic  # noqa: E402

N, T, O, A = 4096, 24, 48, 12
variants = [int(x) for x in sys.argv[1:]] or [0, 16, 64, 96]
algs = {}
for v in variants:
    torch.manual_seed(0)
    ac = ActorCritic(O, O, A, [512, 256, 128], [512, 256, 128]).cuda()
    alg = PPO(ac, num_learning_epochs=5, num_mini_batches=4, device="cuda")
    alg.init_storage(N, T, [O], [None], [A])
    f = alg._fused
    M = N * T // 4
    if v:
        ks = (M + v - 1) // v
        f.ks[0] = (ks + 63) // 64 * 64
        nsl = (M + f.ks[0] - 1) // f.ks[0]
        f.slab[0] = [torch.empty(nsl, *s.shape[1:], device="cuda") for s in f.slab[0]]
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
    algs[(v, f.ks[0], f.slab[0][0].shape[0])] = alg
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
ref = None
for m, alg in algs.items():
    v = sorted(res[m])
    p = torch.cat([q.detach().flatten() for q in alg.actor_critic.parameters()])
    ref = p if ref is None else ref
    print(f"layer-0 slabs {m[2]:3d} ({m[1]} rows{' shipped' if m[0] == 0 else ''}): update {v[len(v) // 2]:.3f} ms median, "
          f"{v[0]:.3f} min; params max |diff| vs first {float((p - ref).abs().max()):.2e}", flush=True)
