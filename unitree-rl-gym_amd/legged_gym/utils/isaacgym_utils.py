"""Quaternion (xyzw) -> roll/pitch/yaw in (-pi, pi] (reference isaacgym_utils.py:11-29)."""
import numpy as np
import torch


def get_euler_xyz(q):
    qx, qy, qz, qw = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    roll = torch.atan2(2.0 * (qw * qx + qy * qz), qw * qw - qx * qx - qy * qy + qz * qz)
    sinp = 2.0 * (qw * qy - qz * qx)
    pitch = torch.where(sinp.abs() >= 1, torch.sign(sinp) * (np.pi / 2.0), torch.asin(sinp))
    yaw = torch.atan2(2.0 * (qw * qz + qx * qy), qw * qw + qx * qx - qy * qy - qz * qz)
    return torch.stack((roll, pitch, yaw), dim=-1)
