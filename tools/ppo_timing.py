"""Time collection vs update of OnPolicyRunner on Go2 x 4096 (graph on/off)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
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
for use_graph in (False, True):
    runner = OnPolicyRunner(env, class_to_dict(tc), log_dir=None, device="cuda:0")
    runner.alg.use_graph = use_graph
    runner.learn(3)
    cs, ls = [], []
    for _ in range(5):
        runner.learn(1)
        c, l = runner.last_iteration_times
        cs.append(c); ls.append(l)
    print(f"graph={use_graph}: collection {1e3*sum(cs)/5:.2f} ms, learn {1e3*sum(ls)/5:.2f} ms", flush=True)
