"""Short training run of a task, printing the rollout's mean step reward and the mean
episode length per iteration (evidence that a config learns, e.g. H1 with and without
self-collision).  usage: python tools/learn_curve.py task iters envs [self_collisions(0/1|-)] [pgs_sweeps|-] [seed]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))
import copy  # noqa: E402

import torch  # noqa: E402

import isaacgym  # noqa: F401,E402
from legged_gym.envs import task_registry  # noqa: E402
from legged_gym.utils import get_args  # noqa: E402
from legged_gym.utils.helpers import class_to_dict  # noqa: E402
from rsl_rl.runners import OnPolicyRunner  # noqa: E402


def main(task, iters, n, selfc=None, sweeps=None, seed=None):
    args = get_args(["--task", task, "--num_envs", str(n), "--headless"])
    env_cfg, tc = task_registry.get_cfgs(task)
    env_cfg = copy.deepcopy(env_cfg)
    if selfc is not None and selfc != "-":
        env_cfg.asset.self_collisions = int(selfc)
    if sweeps is not None and sweeps != "-":
        env_cfg.sim.physx.pgs_sweeps = int(sweeps)
    if seed is not None:
        env_cfg.seed = int(seed)
    env, _ = task_registry.make_env(name=task, args=args, env_cfg=env_cfg)
    runner = OnPolicyRunner(env, class_to_dict(tc), log_dir=None, device="cuda:0")
    print(f"{task} x{n} sweeps={env._lgs_params.solver_iterations} self_collisions={env_cfg.asset.self_collisions} pairs="
          f"{0 if env.self_collision is None else len(env.self_collision.pairs)}", flush=True)
    for it in range(iters):
        runner.learn(1)
        st = runner.alg.storage
        ep = float(env._episode_length.float().mean())
        if it % 10 == 0 or it == iters - 1:
            print(f"it {it:4d} mean step reward {float(st.rewards.mean()):+.5f}  mean episode length {ep:7.1f}", flush=True)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4] if len(sys.argv) > 4 else None,
         sys.argv[5] if len(sys.argv) > 5 else None, sys.argv[6] if len(sys.argv) > 6 else None)
