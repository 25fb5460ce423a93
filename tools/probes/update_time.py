"""Captured Go2 PPO update (4096 envs x 24 steps, 5 epochs x 4 mini-batches) with the
libppomlp.so named by PPOMLP_LIB: median time of graph replays, and the parameters after
3 updates from a fixed seed saved to argv[1] (for a bitwise comparison of two builds).
Usage: PPOMLP_LIB=... python tools/probes/update_time.py out.npz   (tools/gpu_update_ab.sh)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))
import torch  # noqa: E402

from rsl_rl.algorithms import PPO  # noqa: E402
from rsl_rl.modules import ActorCritic  # noqa: E402

N, T, O, A = 4096, 24, 48, 12
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
for _ in range(3):  # eager, then capture + replay
    st.step = T
    alg.update()
assert alg._fgraph is not None
torch.cuda.synchronize()
np.savez(sys.argv[1], **{f"p{i}": p.detach().cpu().numpy() for i, p in enumerate(ac.parameters())})
ts = []
for rnd in range(7):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        alg._fgraph.replay()
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) / 5)
ts.sort()
print(f"{os.path.basename(os.environ.get('PPOMLP_LIB', 'libppomlp.so'))}: update {ts[len(ts) // 2]:.3f} ms median, "
      f"{ts[0]:.3f} min", flush=True)
