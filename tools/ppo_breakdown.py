"""Collection vs update time of OnPolicyRunner iterations for any task (run under
rocprofv3 --kernel-trace --stats for the per-kernel split).
usage: python tools/ppo_breakdown.py task num_envs [iters]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))
import isaacgym  # noqa: F401,E402
from legged_gym.envs import task_registry  # noqa: E402
from legged_gym.utils import get_args  # noqa: E402
from legged_gym.utils.helpers import class_to_dict  # noqa: E402
from rsl_rl.runners import OnPolicyRunner  # noqa: E402

task, n = sys.argv[1], int(sys.argv[2])
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 3
args = get_args(["--task", task, "--num_envs", str(n), "--headless"])
env, _ = task_registry.make_env(name=task, args=args)
_, tc = task_registry.get_cfgs(task)
runner = OnPolicyRunner(env, class_to_dict(tc), log_dir=None, device="cuda:0")
runner.sync_phase_times = True  # device-exact phase times
runner.learn(2)
cs, ls = [], []
for _ in range(iters):
    runner.learn(1)
    c, l = runner.last_iteration_times
    cs.append(c)
    ls.append(l)
print(f"{task} x{n}: collection {1e3 * sum(cs) / iters:.2f} ms, learn {1e3 * sum(ls) / iters:.2f} ms", flush=True)
