"""Is the learning-curve gap between contact sweep counts the physics or the learning?  Trains Go2 x
4096 for `iters` PPO iterations at `train_sweeps`, then runs the trained policy (deterministic
actions, no updates) for `steps` control steps in envs built with each of `eval_sweeps`, same
seed, and prints the mean step reward and the fraction of envs that terminated early.
usage: python tools/probes/sweeps_policy_eval.py train_sweeps iters steps eval_sweeps..."""
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))
import torch  # noqa: E402

import isaacgym  # noqa: F401,E402
from legged_gym.envs import task_registry  # noqa: E402
from legged_gym.utils import get_args  # noqa: E402
from legged_gym.utils.helpers import class_to_dict  # noqa: E402
from rsl_rl.runners import OnPolicyRunner  # noqa: E402


def make(sweeps):
    env_cfg, tc = task_registry.get_cfgs("go2")
    env_cfg = copy.deepcopy(env_cfg)
    env_cfg.sim.physx.pgs_sweeps = sweeps
    env, _ = task_registry.make_env(name="go2", args=get_args(["--task", "go2", "--num_envs", "4096", "--headless"]),
                                    env_cfg=env_cfg)
    return env, tc


def main(train_sweeps, iters, steps, eval_sweeps):
    env, tc = make(train_sweeps)
    runner = OnPolicyRunner(env, class_to_dict(tc), log_dir=None, device="cuda:0")
    runner.learn(iters)
    policy = runner.get_inference_policy(device="cuda:0")
    env.close()
    for sw in eval_sweeps:
        env, _ = make(sw)
        obs = env.get_observations()
        rew = torch.zeros((), device="cuda")
        falls = torch.zeros((), device="cuda")
        with torch.inference_mode():
            for _ in range(steps):
                obs, _, r, d, x = env.step(policy(obs))
                rew += r.mean()
                falls += (d & ~x["time_outs"]).float().mean()
        print(f"trained at {train_sweeps} sweeps for {iters} iterations, evaluated at {sw} sweeps: mean step reward "
              f"{float(rew) / steps:+.5f}, terminations per env-step {float(falls) / steps:.5f}", flush=True)
        env.close()


if __name__ == "__main__":
    main(int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), [int(x) for x in sys.argv[4:]])
