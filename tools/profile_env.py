"""Env-only workload for rocprofv3 passes: Go2 x 4096 fused control steps.

Also runs a calibration copy of a known byte count (CAL_BYTES read + CAL_BYTES written,
float4 streaming, larger than the 256 MiB Infinity Cache) in the same process, so a PMC
pass carries its own reference: tools/pmc_summary.py scales the k_step FETCH_SIZE /
WRITE_SIZE by known / measured of that copy (MI355X_MICROARCH.md §HBM: calibrate on a
known byte count before trusting an absolute).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))

import torch  # noqa: E402

import isaacgym  # noqa: F401,E402
from legged_gym.envs import task_registry  # noqa: E402
from legged_gym.utils import get_args  # noqa: E402

CAL_BYTES = 1 << 30  # 1 GiB read + 1 GiB written per calibration copy


def calibrate(reps=3):
    src = torch.ones(CAL_BYTES // 4, device="cuda")
    dst = torch.empty_like(src)
    for _ in range(reps):
        dst.copy_(src)
    torch.cuda.synchronize()
    del src, dst
    torch.cuda.empty_cache()


def main(task="go2", n=4096, steps=100):
    calibrate()
    args = get_args(["--task", task, "--num_envs", str(n), "--headless"])
    env, _ = task_registry.make_env(name=task, args=args)
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(0)
    acts = [0.5 * torch.randn(n, env.num_actions, device="cuda", generator=g) for _ in range(8)]
    for i in range(steps):
        env.step(acts[i % 8])
    torch.cuda.synchronize()
    print(f"{task}: {steps} steps done")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "go2", int(sys.argv[2]) if len(sys.argv) > 2 else 4096,
         int(sys.argv[3]) if len(sys.argv) > 3 else 100)
