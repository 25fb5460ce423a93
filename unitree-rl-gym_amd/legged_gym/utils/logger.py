"""Play-time state/reward logger (reference utils/logger.py:5-38), text output only."""
from collections import defaultdict

import numpy as np


class Logger:
    def __init__(self, dt):
        self.state_log = defaultdict(list)
        self.rew_log = defaultdict(list)
        self.dt = dt
        self.num_episodes = 0

    def log_state(self, key, value):
        self.state_log[key].append(value)

    def log_states(self, d):
        for k, v in d.items():
            self.log_state(k, v)

    def log_rewards(self, d, num_episodes):
        for k, v in d.items():
            if "rew" in k:
                self.rew_log[k].append(v.item() * num_episodes)
        self.num_episodes += num_episodes

    def reset(self):
        self.state_log.clear()
        self.rew_log.clear()

    def print_rewards(self):
        print("Average rewards per second:")
        for k, vals in self.rew_log.items():
            print(f" - {k}: {np.sum(np.array(vals)) / max(self.num_episodes, 1)}")
        print(f"Total number of episodes: {self.num_episodes}")
