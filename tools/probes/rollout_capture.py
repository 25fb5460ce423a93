"""Which part of the rollout step breaks hipGraph capture?  usage: rollout_capture.py <case>"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "unitree-rl-gym_amd"))
import torch  # noqa: E402
import isaacgym  # noqa: F401,E402
from legged_gym.envs import task_registry  # noqa: E402
from legged_gym.utils import get_args  # noqa: E402
from legged_gym.utils.helpers import class_to_dict  # noqa: E402

case = sys.argv[1]
args = get_args(["--task", "go2", "--num_envs", "512", "--headless"])
env, _ = task_registry.make_env(name="go2", args=args)
_, train_cfg = task_registry.get_cfgs("go2")
from rsl_rl.runners import OnPolicyRunner  # noqa: E402
cfg = class_to_dict(train_cfg)
cfg["runner"]["rollout_graph"] = False
runner = OnPolicyRunner(env, cfg, log_dir=None, device="cuda:0")
runner.learn(1)
obs = env.get_observations()
ac = runner.alg.actor_critic
mean = torch.zeros(512, 12, device="cuda")
std = torch.ones(512, 12, device="cuda")
fns = {
    "normal": lambda: torch.normal(mean, std),
    "normal_expand": lambda: torch.normal(mean.expand(512, 12), (mean * 0 + ac.std).expand(512, 12)),
    "randn": lambda: torch.randn(512, 12, device="cuda"),
    "mean_value": lambda: ac.mean_and_value(obs, obs),
    "act_value": lambda: ac.act_and_value(obs, obs),
    "env_step": lambda: env.step(mean),
    "alg_act": lambda: runner.alg.act(obs, obs),
}
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
try:
    with torch.no_grad():
        with torch.cuda.graph(g):
            out = fns[case]()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    print(case, "OK", flush=True)
except Exception as e:  # report and exit non-zero: the next case runs in a fresh process
    print(case, "FAIL", type(e).__name__, str(e).splitlines()[0], flush=True)
    sys.exit(3)
