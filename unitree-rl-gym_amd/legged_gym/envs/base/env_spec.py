"""Host-side derivation of every per-task constant the env uses.

One function shared by the GPU env (LeggedRobot) and the CPU tests, so the
constants the kernel receives are derived exactly once, the reference's way:
  _parse_cfg                     legged_robot.py:52-67
  dof limits / soft limits       legged_robot.py:456-469
  default pose + PD gains        legged_robot.py:168-186 (substring match, last wins)
  body index selection           legged_robot.py:346-407
  noise scale vector             legged_robot.py:188-219 / h1_env.py:10-31
  reward scale processing        legged_robot.py:817-840
"""
from types import SimpleNamespace

import numpy as np

from legged_gym.utils.helpers import class_to_dict
from leggedsim import cabi


def derive_env_spec(cfg, model, sim_dt, obs_layout, hip_dof_indices=(), verbose=True):
    s = SimpleNamespace()
    s.cfg = cfg
    s.obs_layout = obs_layout
    s.hip_dof_indices = tuple(hip_dof_indices)
    s.dt = cfg.control.decimation * sim_dt
    s.obs_scales = cfg.normalization.obs_scales
    s.reward_scales = class_to_dict(cfg.rewards.scales)
    s.command_ranges = class_to_dict(cfg.commands.ranges)
    s.max_episode_length_s = cfg.env.episode_length_s
    s.max_episode_length = np.ceil(s.max_episode_length_s / s.dt)
    cfg.domain_rand.push_interval = np.ceil(cfg.domain_rand.push_interval_s / s.dt)
    s.num_obs = cfg.env.num_observations
    s.num_privileged_obs = cfg.env.num_privileged_obs
    s.num_actions = cfg.env.num_actions
    s.num_dof = model.num_dofs
    s.num_bodies = model.num_bodies
    s.dof_names = list(model.dof_names)
    s.body_names = list(model.body_names)

    body_names = s.body_names
    feet = [n for n in body_names if cfg.asset.foot_name in n]
    pen = []
    for key in cfg.asset.penalize_contacts_on:
        pen.extend([n for n in body_names if key in n])
    term = []
    for key in cfg.asset.terminate_after_contacts_on:
        term.extend([n for n in body_names if key in n])
    s.feet_names = feet
    s.feet_indices = np.array([body_names.index(n) for n in feet], dtype=np.int64)
    s.penalised_contact_indices = np.array([body_names.index(n) for n in pen], dtype=np.int64)
    s.termination_contact_indices = np.array([body_names.index(n) for n in term], dtype=np.int64)

    lo = model.dof_lower.astype(np.float32)
    hi = model.dof_upper.astype(np.float32)
    m = (lo + hi) / 2
    r = hi - lo
    k = np.float32(cfg.rewards.soft_dof_pos_limit)
    s.dof_pos_limits = np.stack([m - 0.5 * r * k, m + 0.5 * r * k], axis=1).astype(np.float32)
    s.dof_vel_limits = model.dof_velocity.astype(np.float32)
    s.torque_limits = model.dof_effort.astype(np.float32)

    D = s.num_dof
    s.default_dof_pos = np.zeros((1, D), dtype=np.float32)
    s.p_gains = np.zeros(D, dtype=np.float32)
    s.d_gains = np.zeros(D, dtype=np.float32)
    for i, name in enumerate(s.dof_names):
        s.default_dof_pos[0, i] = cfg.init_state.default_joint_angles[name]
        found = False
        for key in cfg.control.stiffness.keys():
            if key in name:
                s.p_gains[i] = cfg.control.stiffness[key]
                s.d_gains[i] = cfg.control.damping[key]
                found = True
        if not found and cfg.control.control_type in ["P", "V"] and verbose:
            print(f"PD gain of joint {name} were not defined, setting them to zero")

    s.commands_scale = np.array([s.obs_scales.lin_vel, s.obs_scales.lin_vel, s.obs_scales.ang_vel], dtype=np.float32)
    s.add_noise = cfg.noise.add_noise
    s.noise_scale_vec = noise_scale_vec(cfg, s.num_obs, s.num_actions, obs_layout)
    init = cfg.init_state
    s.base_init_state = np.array(init.pos + init.rot + init.lin_vel + init.ang_vel, dtype=np.float32)

    for key in list(s.reward_scales.keys()):
        if s.reward_scales[key] == 0:
            s.reward_scales.pop(key)
        else:
            s.reward_scales[key] *= s.dt
    s.reward_names = [n for n in s.reward_scales if n != "termination"]
    s.sum_names = list(s.reward_names) + (["termination"] if "termination" in s.reward_scales else [])
    return s


def noise_scale_vec(cfg, num_obs, A, obs_layout):
    v = np.zeros(num_obs, dtype=np.float32)
    ns = cfg.noise.noise_scales
    lvl = cfg.noise.noise_level
    sc = cfg.normalization.obs_scales
    if obs_layout == cabi.OBS_QUADRUPED:
        v[:3] = ns.lin_vel * lvl * sc.lin_vel
        v[3:6] = ns.ang_vel * lvl * sc.ang_vel
        v[6:9] = ns.gravity * lvl
        v[12:12 + A] = ns.dof_pos * lvl * sc.dof_pos
        v[12 + A:12 + 2 * A] = ns.dof_vel * lvl * sc.dof_vel
    else:
        v[:3] = ns.ang_vel * lvl * sc.ang_vel
        v[3:6] = ns.gravity * lvl
        v[9:9 + A] = ns.dof_pos * lvl * sc.dof_pos
        v[9 + A:9 + 2 * A] = ns.dof_vel * lvl * sc.dof_vel
    return v
