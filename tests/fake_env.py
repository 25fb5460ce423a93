"""A tiny pure-torch VecEnv for host-side rsl_rl tests (no simulator)."""
import torch

from rsl_rl.env import VecEnv


class FakeEnv(VecEnv):
    def __init__(self, num_envs=16, num_obs=6, num_actions=3, num_privileged_obs=None, device="cpu", ep_len=7):
        self.num_envs, self.num_obs, self.num_actions = num_envs, num_obs, num_actions
        self.num_privileged_obs = num_privileged_obs
        self.max_episode_length = ep_len
        self.device = device
        self.obs_buf = torch.zeros(num_envs, num_obs, device=device)
        self.privileged_obs_buf = None if num_privileged_obs is None else torch.zeros(num_envs, num_privileged_obs, device=device)
        self.rew_buf = torch.zeros(num_envs, device=device)
        self.reset_buf = torch.zeros(num_envs, dtype=torch.bool, device=device)
        self.episode_length_buf = torch.zeros(num_envs, dtype=torch.long, device=device)
        self.extras = {}
        self.g = torch.Generator(device=device).manual_seed(0)
        self.W = torch.randn(num_obs, num_actions, generator=self.g, device=device)

    def get_observations(self):
        return self.obs_buf

    def get_privileged_observations(self):
        return self.privileged_obs_buf

    def reset(self):
        self.obs_buf = torch.randn(self.num_envs, self.num_obs, generator=self.g, device=self.device)
        if self.privileged_obs_buf is not None:
            self.privileged_obs_buf = torch.randn(self.num_envs, self.num_privileged_obs, generator=self.g, device=self.device)
        return self.obs_buf, self.privileged_obs_buf

    def step(self, actions):
        target = self.obs_buf @ self.W
        self.rew_buf = -((actions - target) ** 2).sum(-1)
        self.episode_length_buf += 1
        dones = self.episode_length_buf >= self.max_episode_length
        self.episode_length_buf[dones] = 0
        self.obs_buf = torch.randn(self.num_envs, self.num_obs, generator=self.g, device=self.device)
        if self.privileged_obs_buf is not None:
            self.privileged_obs_buf = torch.cat([self.obs_buf, torch.zeros(self.num_envs, self.num_privileged_obs - self.num_obs)], 1)
        self.extras = {"time_outs": dones.clone(), "episode": {"rew_x": self.rew_buf.mean()}}
        return self.obs_buf, self.privileged_obs_buf, self.rew_buf, dones, self.extras
