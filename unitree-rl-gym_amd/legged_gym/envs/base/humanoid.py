"""Shared humanoid behaviour of the reference's H1/G1/H1_2 envs
(h1_env.py:8-123, g1_env.py:8-180, h1_2_env.py:8-123): gait-phase observations,
privileged obs = [base lin vel, obs], feet rigid-body state, and the five extra
reward terms.  All of it is computed inside the native step; this class only
selects the humanoid layout and exposes the same attributes."""
from leggedsim import cabi

from .legged_robot import LeggedRobot


class HumanoidRobot(LeggedRobot):
    obs_layout = cabi.OBS_HUMANOID
    # 8 contact slots + 8 joint-limit rows = the 32-row variant, which runs two envs per
    # wave (H1 8192: 0.70 -> 0.38 ms per control step).  Slot order (include/leggedsim.h):
    # one slot per body on the ground first (a knee, hip or pelvis is never crowded out by
    # the soles), then up to 4 self contacts, then further sole corners (the feet's
    # candidates are dealt round-robin, Model.reorder_points: two planted soles share the
    # rest evenly).  Limits beyond the 8 limit rows use the rows of unused contact slots.
    max_contacts = 8
    max_rows = 32
    max_self_contacts = 4

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
