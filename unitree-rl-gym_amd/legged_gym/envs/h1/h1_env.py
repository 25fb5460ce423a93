"""H1 (reference envs/h1/h1_env.py): hip_pos penalises DOFs [0, 1, 5, 6] (:123)."""
from legged_gym.envs.base.humanoid import HumanoidRobot


class H1Robot(HumanoidRobot):
    hip_dof_indices = (0, 1, 5, 6)
