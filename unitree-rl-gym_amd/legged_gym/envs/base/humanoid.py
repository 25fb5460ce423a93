"""Shared humanoid behaviour of the reference's H1/G1/H1_2 envs
(h1_env.py:8-123, g1_env.py:8-180, h1_2_env.py:8-123): gait-phase observations,
privileged obs = [base lin vel, obs], feet rigid-body state, and the five extra
reward terms.  All of it is computed inside the native step; this class only
selects the humanoid layout and exposes the same attributes."""
import torch

from leggedsim import cabi

from .legged_robot import LeggedRobot


class HumanoidRobot(LeggedRobot):
    obs_layout = cabi.OBS_HUMANOID
    max_contacts = 12
    max_rows = 48

    def _get_noise_scale_vec(self, cfg):
        """h1_env.py:10-31"""
        noise_vec = torch.zeros_like(self.obs_buf[0])
        self.add_noise = self.cfg.noise.add_noise
        ns = self.cfg.noise.noise_scales
        lvl = self.cfg.noise.noise_level
        A = self.num_actions
        noise_vec[:3] = ns.ang_vel * lvl * self.obs_scales.ang_vel
        noise_vec[3:6] = ns.gravity * lvl
        noise_vec[6:9] = 0.0
        noise_vec[9:9 + A] = ns.dof_pos * lvl * self.obs_scales.dof_pos
        noise_vec[9 + A:9 + 2 * A] = ns.dof_vel * lvl * self.obs_scales.dof_vel
        noise_vec[9 + 2 * A:9 + 3 * A] = 0.0
        noise_vec[9 + 3 * A:9 + 3 * A + 2] = 0.0
        return noise_vec

    def _init_buffers(self):
        super()._init_buffers()
        self._init_foot()

    def _init_foot(self):
        """h1_env.py:34-46: feet views into the rigid body state tensor."""
        self.feet_num = len(self.feet_indices)
        self.update_feet_state()

    def update_feet_state(self):
        self.feet_state = self.rigid_body_states_view[:, self.feet_indices, :]
        self.feet_pos = self.feet_state[:, :, :3]
        self.feet_vel = self.feet_state[:, :, 7:10]

    def step(self, actions):
        out = super().step(actions)
        self.update_feet_state()
        return out
