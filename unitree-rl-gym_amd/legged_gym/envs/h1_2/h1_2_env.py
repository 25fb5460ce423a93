"""H1_2 (reference envs/h1_2/h1_2_env.py): hip_pos penalises DOFs [0, 2, 6, 8] (:123)."""
from legged_gym.envs.base.humanoid import HumanoidRobot


class H1_2Robot(HumanoidRobot):
    hip_dof_indices = (0, 2, 6, 8)
