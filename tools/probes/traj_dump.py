"""Env trajectory of the build LEGGEDSIM_LIB names (task, envs, zero or random actions): the
root and DOF states after each of S steps into argv[1] (.npz), to compare two builds bitwise.
usage: LEGGEDSIM_LIB=... python tools/probes/traj_dump.py out.npz [task] [n] [steps] [zero|rand]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))
import torch  # noqa: E402
import isaacgym  # noqa: E402,F401
from legged_gym.envs import task_registry  # noqa: E402
from legged_gym.utils import get_args  # noqa: E402

out = sys.argv[1]
task = sys.argv[2] if len(sys.argv) > 2 else "go2"
n = int(sys.argv[3]) if len(sys.argv) > 3 else 256
S = int(sys.argv[4]) if len(sys.argv) > 4 else 40
mode = sys.argv[5] if len(sys.argv) > 5 else "zero"
env, _ = task_registry.make_env(name=task, args=get_args(["--task", task, "--num_envs", str(n), "--headless"]))
env.reset()
g = torch.Generator(device="cuda").manual_seed(0)
roots, dofs = [], []
for i in range(S):
    a = torch.zeros(n, env.num_actions, device="cuda") if mode == "zero" else \
        0.5 * torch.randn(n, env.num_actions, device="cuda", generator=g)
    env.step(a)
    roots.append(env.root_states.cpu().numpy().copy())
    dofs.append(env.dof_state.cpu().numpy().copy())
np.savez(out, root=np.stack(roots), dof=np.stack(dofs))
print("saved", out, flush=True)
