"""GPU bring-up probe: build an env on the HIP simulator, step it, compare one
step against the CPU oracle and time the fused step.  Prints a report."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import isaacgym  # noqa: F401,E402
from legged_gym.envs import *  # noqa: F401,F403,E402
from legged_gym.utils import get_args, task_registry  # noqa: E402
import bridge  # noqa: E402


def run(task, n, warm=50, timed=200):
    args = get_args(["--task", task, "--num_envs", str(n), "--headless"])
    env, cfg = task_registry.make_env(name=task, args=args)
    print(f"[{task}] bodies={env.num_bodies} dofs={env.num_dof} feet={env.feet_indices.tolist()}", flush=True)
    obs, _ = env.reset()
    torch.cuda.synchronize()
    g = torch.Generator(device="cuda").manual_seed(0)
    for i in range(warm):
        a = 0.5 * torch.randn(n, env.num_actions, device="cuda", generator=g)
        env.step(a)
    torch.cuda.synchronize()
    print(f"  after {warm} steps: base z mean={env.root_states[:, 2].mean().item():.4f} "
          f"min={env.root_states[:, 2].min().item():.4f} rew mean={env.rew_buf.mean().item():.4f} "
          f"resets={env.reset_buf.sum().item()} feetFz mean={env.contact_forces[:, env.feet_indices, 2].mean().item():.2f} "
          f"finite={bool(torch.isfinite(env.root_states).all())}", flush=True)
    # parity vs oracle on one step
    snap = bridge.snapshot(env)
    a = 0.5 * torch.randn(n, env.num_actions, device="cuda", generator=g)
    ctr = env.common_step_counter
    ref = bridge.step(env, snap, a.cpu().numpy(), ctr)
    env.step(a)
    torch.cuda.synchronize()
    got = {"root": env.root_states, "dofs": env.dof_state, "cforce": env._contact_forces, "obs": env.obs_buf,
           "rew": env.rew_buf, "reset": env.reset_buf, "commands": env.commands, "rbs": env.rigid_body_states,
           "torques": env.torques, "episode_length": env._episode_length}
    for k, v in got.items():
        v = v.detach().cpu().numpy()
        r = ref[k]
        if v.dtype == np.bool_:
            v = v.astype(np.uint8)
        d = np.abs(v.astype(np.float64) - r.astype(np.float64))
        scale = np.maximum(np.abs(r.astype(np.float64)), 1.0)
        rel = d / scale
        per_env = rel.reshape(n, -1).max(axis=1)
        print(f"  parity {k:15s} max|d|={d.max():.3e} max rel={rel.max():.3e} envs>1e-4: {(per_env > 1e-4).sum()}/{n}", flush=True)
    # timing
    acts = [0.5 * torch.randn(n, env.num_actions, device="cuda", generator=g) for _ in range(8)]
    for i in range(20):
        env.step(acts[i % 8])
    torch.cuda.synchronize()
    t0 = time.time()
    for i in range(timed):
        env.step(acts[i % 8])
    torch.cuda.synchronize()
    dt = time.time() - t0
    print(f"  timing: {dt / timed * 1e3:.3f} ms/step -> {n * timed / dt / 1e6:.2f} M env-steps/s", flush=True)
    return env


if __name__ == "__main__":
    tasks = sys.argv[1].split(",") if len(sys.argv) > 1 else ["go2"]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    for t in tasks:
        run(t, n)
