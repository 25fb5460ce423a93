"""env configuration -> ``lgs_task_params`` (everything post_physics_step reads).

Takes any env-like object (the live LeggedRobot, or a host-only namespace in
tests) exposing the attributes the reference env derives in _parse_cfg /
_init_buffers / _prepare_reward_function (legged_robot.py:52-186, 817-840).
"""
from __future__ import annotations

import os

import numpy as np

from . import cabi


def _np(x):
    if hasattr(x, "detach"):
        x = x.detach().cpu().numpy()
    return np.asarray(x)


def _put(arr, values):
    v = _np(values).astype(np.float32).reshape(-1)
    arr[: len(v)] = v.tolist()


def build_task_params(env) -> cabi.TaskParams:
    T = cabi.TaskParams()
    cfg = env.cfg
    A, D = env.num_actions, env.num_dof
    if A != D:
        raise ValueError("num_actions must equal the number of DOFs")
    T.obs_layout = env.obs_layout
    T.num_obs = env.num_obs
    T.num_privileged_obs = env.num_privileged_obs or 0
    T.num_actions = A
    T.decimation = cfg.control.decimation
    T.control_type = {"P": 0, "V": 1, "T": 2}.get(cfg.control.control_type, -1)
    if T.control_type < 0:
        raise NameError(f"Unknown controller type: {cfg.control.control_type}")
    T.action_scale = cfg.control.action_scale
    T.clip_actions = cfg.normalization.clip_actions
    T.clip_observations = cfg.normalization.clip_observations
    T.control_dt = env.dt
    _put(T.p_gains, env.p_gains)
    _put(T.d_gains, env.d_gains)
    _put(T.default_dof_pos, _np(env.default_dof_pos).reshape(-1))
    _put(T.torque_limits, env.torque_limits)
    lim = _np(env.dof_pos_limits)
    _put(T.soft_dof_pos_lower, lim[:, 0])
    _put(T.soft_dof_pos_upper, lim[:, 1])
    _put(T.dof_vel_limits, env.dof_vel_limits)
    s = env.obs_scales
    T.obs_scale_lin_vel, T.obs_scale_ang_vel = s.lin_vel, s.ang_vel
    T.obs_scale_dof_pos, T.obs_scale_dof_vel = s.dof_pos, s.dof_vel
    _put(T.commands_scale, env.commands_scale)
    T.add_noise = int(bool(env.add_noise))
    _put(T.noise_vec, env.noise_scale_vec)
    T.max_episode_length = float(env.max_episode_length)
    T.max_episode_length_s = float(env.max_episode_length_s)
    T.resample_interval = int(cfg.commands.resampling_time / env.dt)
    T.heading_command = int(bool(cfg.commands.heading_command))
    r = env.command_ranges
    _put(T.cmd_lin_vel_x, r["lin_vel_x"])
    _put(T.cmd_lin_vel_y, r["lin_vel_y"])
    _put(T.cmd_ang_vel_yaw, r["ang_vel_yaw"])
    _put(T.cmd_heading, r["heading"])
    T.push_robots = int(bool(cfg.domain_rand.push_robots))
    T.push_interval = int(cfg.domain_rand.push_interval)
    T.max_push_vel_xy = cfg.domain_rand.max_push_vel_xy
    _put(T.base_init_state, env.base_init_state)
    fi = [int(x) for x in _np(env.feet_indices).tolist()]
    if len(fi) > cabi.MAX_FEET:
        raise ValueError("too many feet bodies for the native step")
    T.num_feet = len(fi)
    T.feet_idx[: len(fi)] = fi
    pi_ = [int(x) for x in _np(env.penalised_contact_indices).tolist()][: cabi.MAX_CONTACT_BODIES]
    T.num_penalised = len(pi_)
    T.penalised_idx[: len(pi_)] = pi_
    ti = [int(x) for x in _np(env.termination_contact_indices).tolist()][: cabi.MAX_CONTACT_BODIES]
    T.num_termination = len(ti)
    T.termination_idx[: len(ti)] = ti
    hip = list(env.hip_dof_indices)
    T.num_hip = len(hip)
    T.hip_dofs[: len(hip)] = hip
    native = list(getattr(env, "_native_reward_names", env.reward_names))
    py = [n for n, _ in getattr(env, "_py_rewards", [])]
    hooks = getattr(env, "_hooks", frozenset())
    T.num_rewards = len(native)
    # the reward total (only_positive_rewards, the termination term) is finished in Python when
    # Python terms add to it or a Python check_termination decides the resets
    T.defer_reward_total = int(bool(py) or "check_termination" in hooks)
    T.num_extra_sums = len(py)
    for k, n in enumerate(native):
        T.reward_ids[k] = cabi.REWARD_ID[cabi.REWARD_ALIASES.get(n, n)]
        T.reward_scales[k] = float(env.reward_scales[n])
    T.has_termination_reward = int("termination" in env.reward_scales)
    T.termination_scale = float(env.reward_scales.get("termination", 0.0))
    rw = cfg.rewards
    T.only_positive_rewards = int(bool(rw.only_positive_rewards))
    T.tracking_sigma = rw.tracking_sigma
    T.base_height_target = rw.base_height_target
    T.max_contact_force = rw.max_contact_force
    T.soft_dof_vel_limit = rw.soft_dof_vel_limit
    T.soft_torque_limit = rw.soft_torque_limit
    # gait phase constants of the humanoid envs (h1_env.py:58-59, :101, :109)
    T.phase_period, T.phase_offset, T.stance_threshold, T.swing_height_target = 0.8, 0.5, 0.55, 0.08
    seed = int(getattr(cfg, "seed", 1))
    rank = int(os.environ.get("RANK", "0"))
    T.seed = (seed & 0xFFFFFFFF) | (rank << 32)
    # the rows the step refreshes: the feet (all the reference's humanoid envs read, h1_env.py:34-52)
    # unless the task asks for every body (rigid_body_state_bodies = "all"); by default every
    # body when the task has Python reward terms or step hooks, which may read any row
    bodies = getattr(env, "rigid_body_state_bodies", None)
    if bodies is None:
        bodies = "all" if (py or hooks) else "feet"
    if bodies not in ("all", "feet"):
        raise ValueError(f"rigid_body_state_bodies must be 'all', 'feet' or None, not {bodies!r}")
    T.write_body_states = int(bool(getattr(env, "uses_rigid_body_states", env.obs_layout == cabi.OBS_HUMANOID)) or
                              bool(py) or bool(hooks))
    if bodies == "all":
        T.body_state_mask = 0
    else:
        T.body_state_mask = sum(1 << b for b in fi) if fi else 0
    T.custom_origins = int(bool(getattr(env, "custom_origins", False)))
    return T
