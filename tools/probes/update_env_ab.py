"""A/B of one PPO update (20 fused optimizer steps replayed as a HIP graph) under two
values of an environment switch read when the fused step is built, interleaved in one
process (Go2 MLPs, 4096 envs x 24 steps).

    python tools/probes/update_env_ab.py PMLP_TN 1 0
    python tools/probes/update_env_ab.py PMLP_DW_SIDE_STREAM 0 1
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))
import torch  # noqa: E402

from rsl_rl.algorithms import PPO  # noqa: E402
from rsl_rl.modules import ActorCritic  # noqa: E402

N, T, O, A = 4096, 24, 48, 12


VAR, VALS = sys.argv[1], sys.argv[2:]


def make(val):
    os.environ[VAR] = val
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
    st.step = T
    for _ in range(3):
        alg.update()
        st.step = T
    return alg


algs = {f"{VAR}={v}": make(v) for v in VALS}
res = {k: [] for k in algs}
for rnd in range(5):
    for k, alg in algs.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(5):
            alg.update()
            alg.storage.step = T
        e1.record()
        torch.cuda.synchronize()
        res[k].append(e0.elapsed_time(e1) / 5)
for k, v in res.items():
    v = sorted(v)
    print(f"{k:24s} update ms: median {v[len(v) // 2]:.3f}  min {v[0]:.3f}  all {[round(x, 3) for x in v]}")
