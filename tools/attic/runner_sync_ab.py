"""OnPolicyRunner.learn on Go2 x 4096 with and without the device sync after the collection
(runner.sync_phase_times), alternating rounds of 10 iterations in one process.
usage: python tools/probes/runner_sync_ab.py"""
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
res = {True: [], False: []}
for rnd in range(6):
    for sync in (True, False):
        runner.sync_phase_times = sync
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        runner.learn(10)
        torch.cuda.synchronize()
        res[sync].append((time.perf_counter() - t0) / 10 * 1e3)
for sync, v in res.items():
    v = sorted(v)
    print(f"sync after collection {sync}: {v[len(v) // 2]:.3f} ms per iteration median ({', '.join(f'{x:.3f}' for x in res[sync])})")
