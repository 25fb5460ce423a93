"""Train a registered task (reference scripts/train.py:11-18; same CLI)."""
import isaacgym  # noqa: F401  (kept: the reference imports it first)
from legged_gym.envs import *  # noqa: F401,F403
from legged_gym.utils import get_args, task_registry


def train(args):
    env, env_cfg = task_registry.make_env(name=args.task, args=args)
    ppo_runner, train_cfg = task_registry.make_alg_runner(env=env, name=args.task, args=args)
    ppo_runner.learn(num_learning_iterations=train_cfg.runner.max_iterations, init_at_random_ep_len=True)


if __name__ == "__main__":
    train(get_args())
