import os, sys, copy
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))
import torch
import isaacgym  # noqa
from legged_gym.envs import task_registry
from legged_gym.utils import get_args
from legged_gym.utils.helpers import class_to_dict
from rsl_rl.runners import OnPolicyRunner
_, tc = task_registry.get_cfgs("go2")
for rep, n in enumerate([512, 256, 256]):
    args = get_args(["--task", "go2", "--num_envs", str(n), "--headless"])
    env, _ = task_registry.make_env(name="go2", args=args)
    runner = OnPolicyRunner(env, class_to_dict(tc), log_dir=None, device="cuda:0")
    for it in range(4):
        runner.learn(1)
        ac = runner.alg.actor_critic
        sd = ac.state_dict()
        print(f"rep={rep} n={n} it={it} std_min={ac.std.min().item():.4f} lr={runner.alg.learning_rate:.2e} "
              f"finite={all(torch.isfinite(v).all().item() for v in sd.values())} |w|max={max(v.abs().max().item() for v in sd.values()):.3f}", flush=True)
    del runner, env
