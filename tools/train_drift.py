"""Fused bf16 PPO path vs the fp32 torch path over a short Go2 training run: per-iteration
mean step reward of the rollout and the policy's mean action std (diagnostic for the drift
test in tests/test_gpu_training_drift.py).  usage: python tools/train_drift.py [iters] [envs]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))
import torch  # noqa: E402

import isaacgym  # noqa: F401,E402
from legged_gym.envs import task_registry  # noqa: E402
from legged_gym.utils import get_args  # noqa: E402
from legged_gym.utils.helpers import class_to_dict  # noqa: E402
from rsl_rl.runners import OnPolicyRunner  # noqa: E402


def run(fused, iters, n, seed=1):
    args = get_args(["--task", "go2", "--num_envs", str(n), "--headless", "--seed", str(seed)])
    env, _ = task_registry.make_env(name="go2", args=args)
    _, tc = task_registry.get_cfgs("go2")
    d = class_to_dict(tc)
    if not fused:
        d["policy"]["mixed_precision"] = False
        d["algorithm"]["fused_loss"] = False
    runner = OnPolicyRunner(env, d, log_dir=None, device="cuda:0")
    assert (runner.alg._fused is not None) == fused
    out = []
    for _ in range(iters):
        runner.learn(1)
        st = runner.alg.storage
        out.append((float(st.rewards.mean()), float(runner.alg.actor_critic.std.mean())))
    env.close()
    return out


if __name__ == "__main__":
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    for seed in (1, 2):
        a, b = run(True, iters, n, seed), run(False, iters, n, seed)
        for i, (x, y) in enumerate(zip(a, b)):
            print(f"seed {seed} it {i:3d}  fused rew {x[0]:+.5f} std {x[1]:.4f}   fp32 rew {y[0]:+.5f} std {y[1]:.4f}")
