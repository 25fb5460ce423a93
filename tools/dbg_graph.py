import os, sys, copy
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))
import torch
import isaacgym  # noqa
from legged_gym.envs import task_registry
from legged_gym.utils import get_args
from legged_gym.utils.helpers import class_to_dict
from rsl_rl.runners import OnPolicyRunner
n = int(sys.argv[1])
args = get_args(["--task", "go2", "--num_envs", str(n), "--headless"])
env, _ = task_registry.make_env(name="go2", args=args)
_, tc = task_registry.get_cfgs("go2")
for use_graph in (False, True):
    torch.manual_seed(0)
    runner = OnPolicyRunner(env, class_to_dict(tc), log_dir=None, device="cuda:0")
    runner.alg.use_graph = use_graph
    for it in range(6):
        runner.learn(1)
        ac = runner.alg.actor_critic
        print(f"graph={use_graph} it={it} std={ac.std.mean().item():.4f} min={ac.std.min().item():.4f} lr={runner.alg.learning_rate:.2e}", flush=True)
