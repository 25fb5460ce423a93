import torch


def split_and_pad_trajectories(tensor, dones):
    """Split [T, N, ...] per env at dones into trajectories, pad them to T.

    Returns (padded [T, num_traj, ...], masks [T, num_traj]).  Trajectories are
    ordered env-major then time, as in rsl_rl v1.0.2.
    """
    T = tensor.shape[0]
    dones = dones.clone()
    dones[-1] = 1
    flat_dones = dones.transpose(1, 0).reshape(-1, 1)
    done_indices = torch.cat((flat_dones.new_tensor([-1], dtype=torch.int64), flat_dones.nonzero()[:, 0]))
    lengths = done_indices[1:] - done_indices[:-1]
    trajectories = torch.split(tensor.transpose(1, 0).flatten(0, 1), lengths.tolist())
    padded = torch.nn.utils.rnn.pad_sequence(trajectories)
    if padded.shape[0] < T:  # every trajectory shorter than T: pad to T explicitly
        pad = padded.new_zeros((T - padded.shape[0],) + tuple(padded.shape[1:]))
        padded = torch.cat((padded, pad), dim=0)
    masks = lengths > torch.arange(0, T, device=tensor.device).unsqueeze(1)
    return padded, masks


def unpad_trajectories(trajectories, masks):
    """Inverse of split_and_pad_trajectories for [T, num_traj, ...] outputs."""
    return trajectories.transpose(1, 0)[masks.transpose(1, 0)].view(-1, trajectories.shape[0], trajectories.shape[-1]).transpose(1, 0)
