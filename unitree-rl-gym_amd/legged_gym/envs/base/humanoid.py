"""Shared humanoid behaviour of the reference's H1/G1/H1_2 envs
(h1_env.py:8-123, g1_env.py:8-180, h1_2_env.py:8-123): gait-phase observations,
privileged obs = [base lin vel, obs], feet rigid-body state, and the five extra
reward terms.  All of it is computed inside the native step; this class only
selects the humanoid layout and exposes the same attributes."""
from leggedsim import cabi

from .legged_robot import LeggedRobot

_OWN_FEET = ("_feet_state", "_feet_pos", "_feet_vel")


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
        """h1_env.py:34-46: the feet's rows of the rigid body state tensor."""
        self.feet_num = len(self.feet_indices)

    def update_feet_state(self):
        """h1_env.py:48-56 copies the feet rows after every step.  Here feet_state / feet_pos /
        feet_vel are gathered when read (the rows the step refreshed), so a training loop
        that never reads them (the rewards using them run in the native step) issues no
        gather launch per step; the values are the same as the reference's copies.  Copies a
        task assigned itself (the reference's _init_foot body) are dropped: the next read
        gathers the current rows."""
        for k in _OWN_FEET:
            self.__dict__.pop(k, None)

    def _refresh_task_views(self):
        """The reference refreshes the feet copies every step (h1_env.py:56, from the
        callback): a task holding its own copies (its _init_foot / update_feet_state assign
        them) gets its update_feet_state called at that point of every step."""
        d = self.__dict__
        if "_feet_state" in d or "_feet_pos" in d or "_feet_vel" in d:
            self.update_feet_state()

    # (a task subclass that assigns these attributes itself, as the reference's
    # _init_foot / update_feet_state do, gets its own tensors back until the next refresh)
    @property
    def feet_state(self):
        own = self.__dict__.get("_feet_state")
        return own if own is not None else self.rigid_body_states_view[:, self.feet_indices, :]

    @feet_state.setter
    def feet_state(self, v):
        self.__dict__["_feet_state"] = v

    @property
    def feet_pos(self):
        own = self.__dict__.get("_feet_pos")
        return own if own is not None else self.feet_state[:, :, :3]

    @feet_pos.setter
    def feet_pos(self, v):
        self.__dict__["_feet_pos"] = v

    @property
    def feet_vel(self):
        own = self.__dict__.get("_feet_vel")
        return own if own is not None else self.feet_state[:, :, 7:10]

    @feet_vel.setter
    def feet_vel(self, v):
        self.__dict__["_feet_vel"] = v
