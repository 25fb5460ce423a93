"""Profile target: a few graphed PPO iterations on Go2 x 4096."""
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

args = get_args(["--task", "go2", "--num_envs", "4096", "--headless"])
env, _ = task_registry.make_env(name="go2", args=args)
_, tc = task_registry.get_cfgs("go2")
runner = OnPolicyRunner(env, class_to_dict(tc), log_dir=None, device="cuda:0")
runner.sync_phase_times = True  # device-exact phase times
runner.learn(int(sys.argv[1]) if len(sys.argv) > 1 else 5)
torch.cuda.synchronize()
print("done", runner.last_iteration_times)
