import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))
import torch
import isaacgym  # noqa
from legged_gym.envs import task_registry
from legged_gym.utils import get_args
from legged_gym.utils.helpers import class_to_dict
from rsl_rl.runners import OnPolicyRunner
_, tc = task_registry.get_cfgs("go2")
args = get_args(["--task", "go2", "--num_envs", "256", "--headless"])
env, _ = task_registry.make_env(name="go2", args=args)
for sched in ("adaptive", "fixed"):
    cfg = class_to_dict(tc)
    cfg["algorithm"]["schedule"] = sched
    runner = OnPolicyRunner(env, cfg, log_dir=None, device="cuda:0")
    alg = runner.alg
    orig_update = alg.update
    def upd():
        vl, sl = orig_update()
        fin = all(torch.isfinite(p).all().item() for p in alg.actor_critic.parameters())
        gfin = all(p.grad is None or torch.isfinite(p.grad).all().item() for p in alg.actor_critic.parameters())
        print(f"  sched={sched} call={alg._graph_calls} vl={vl:.5f} sl={sl:.5f} params_finite={fin} grads_finite={gfin} lr={alg.learning_rate:.2e}", flush=True)
        return vl, sl
    alg.update = upd
    runner.learn(4)
