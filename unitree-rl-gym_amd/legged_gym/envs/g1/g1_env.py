"""G1 (reference envs/g1/g1_env.py): hip_pos penalises DOFs [1, 2, 7, 8] (:180)."""
from legged_gym.envs.base.humanoid import HumanoidRobot


class G1Robot(HumanoidRobot):
    hip_dof_indices = (1, 2, 7, 8)
