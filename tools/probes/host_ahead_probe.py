"""Is the host ahead of the device in OnPolicyRunner.learn (Go2 x 4096, no logging)?  Host
time to issue 20 iterations (no sync) against the device time to finish them.
usage: python tools/probes/host_ahead_probe.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))
import torch  # noqa: E402
import isaacgym  # noqa: F401,E402
from legged_gym.envs import task_registry  # noqa: E402
from legged_gym.utils import get_args  # noqa: E402
from legged_gym.utils.helpers import class_to_dict  # noqa: E402
from rsl_rl.runners import OnPolicyRunner  # noqa: E402

args = get_args(["--task", "go2", "--num_envs", "4096", "--headless"])
env, _ = task_registry.make_env(name="go2", args=args)
_, tc = task_registry.get_cfgs("go2")
runner = OnPolicyRunner(env, class_to_dict(tc), log_dir=None, device="cuda:0")
runner.learn(5, init_at_random_ep_len=True)
for rep in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    runner.learn(20)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"host issue {1e3 * (t1 - t0) / 20:.3f} ms per iteration, device done {1e3 * (t2 - t0) / 20:.3f} ms per iteration",
          flush=True)
