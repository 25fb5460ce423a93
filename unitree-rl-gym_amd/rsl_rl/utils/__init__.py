from .utils import split_and_pad_trajectories, unpad_trajectories
