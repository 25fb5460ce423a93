"""Play-time state / episode-reward logger (reference ``legged_gym/utils/logger.py:5-38``).

Off the hot path: ``play.py`` imports it (reference ``scripts/play.py:9``) and user
scripts written against the reference call ``log_states`` / ``log_rewards`` /
``print_rewards`` from their play loops.  Same names, arguments and printed report.
"""
from collections import defaultdict

import numpy as np


class Logger:
    def __init__(self, dt):
        self.dt = dt
        self.state_log = defaultdict(list)  # key -> values, one per logged control step
        self.rew_log = defaultdict(list)  # 'rew_*' key -> episode mean x number of episodes
        self.num_episodes = 0
        self.plot_process = None  # the reference's plotting subprocess handle (never started here)

    def log_state(self, key, value):
        self.state_log[key].append(value)

    def log_states(self, states):
        for key, value in states.items():
            self.log_state(key, value)

    def log_rewards(self, infos, num_episodes):
        """``infos`` is ``extras["episode"]``: per-term means over the envs that ended.
        Weighted by the episode count so print_rewards averages over episodes."""
        for key, value in infos.items():
            if "rew" in key:
                v = value.item() if hasattr(value, "item") else float(value)
                self.rew_log[key].append(v * num_episodes)
        self.num_episodes += num_episodes

    def reset(self):
        self.state_log.clear()
        self.rew_log.clear()

    def print_rewards(self):
        print("Average rewards per second:")
        for key, values in self.rew_log.items():
            print(f" - {key}: {float(np.sum(np.asarray(values))) / self.num_episodes}")
        print(f"Total number of episodes: {self.num_episodes}")

    def __del__(self):
        if self.plot_process is not None:
            self.plot_process.kill()
