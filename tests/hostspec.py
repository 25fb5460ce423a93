"""Host-only env specs for the CPU tests (no GPU): the same constant derivation
the GPU env uses (legged_gym.envs.base.env_spec) on the bundled robot models."""
import copy
import os

import numpy as np

import isaacgym  # noqa: F401
import legged_gym.envs  # noqa: F401  (task registration)
from legged_gym.envs.base.env_spec import derive_env_spec
from legged_gym.utils import task_registry
from leggedsim import cabi
from leggedsim.model import MODELS_DIR, Model
from leggedsim.selfcollision import build_self_collision
from leggedsim.task import build_task_params

MODEL_FILE = {"go2": "go2", "g1": "g1_12dof", "h1": "h1", "h1_2": "h1_2_12dof"}


def make_spec(task, cfg_edit=None):
    env_cfg, train_cfg = task_registry.get_cfgs(task)
    cfg = copy.deepcopy(env_cfg)
    if cfg_edit:
        cfg_edit(cfg)
    cls = task_registry.get_task_class(task)
    model = Model.load(os.path.join(MODELS_DIR, MODEL_FILE[task] + ".npz"))
    feet = {model.body_names.index(n) for n in model.body_names if cfg.asset.foot_name in n}
    model.reorder_points(feet)
    spec = derive_env_spec(cfg, model, cfg.sim.dt, cls.obs_layout, cls.hip_dof_indices, verbose=False)
    spec.model = model
    spec.task = build_task_params(spec)
    spec.sim_params = cabi.sim_params_from_cfg(cfg.sim, cfg.asset, max_contacts=cls.max_contacts,
                                               max_rows=cls.max_rows, ground_friction=float(cfg.terrain.static_friction))
    # the env's self-collision proxies/pairs (LeggedRobot.create_sim); the oracle only uses them
    # when a test hands them over (bridge.set_self_collision)
    spec.self_collision = None
    if int(getattr(cfg.asset, "self_collisions", 1)) == 0:
        spec.self_collision = build_self_collision(model, np.asarray(spec.default_dof_pos).reshape(-1),
                                                   max_self_contacts=cls.max_self_contacts)
    return spec


def host_buffers(spec, N):
    """Zeroed host arrays shaped like the env's device buffers."""
    D, B, A, F = spec.num_dof, spec.num_bodies, spec.num_actions, len(spec.feet_indices)
    nsum = len(spec.sum_names)
    f = np.float32
    b = dict(
        root=np.zeros((N, 13), f), dofs=np.zeros((N * D, 2), f), cforce=np.zeros((N * B, 3), f),
        rbs=np.zeros((N * B, 13), f), actions=np.zeros((N, A), f), last_actions=np.zeros((N, A), f),
        last_dof_vel=np.zeros((N, D), f), last_root_vel=np.zeros((N, 6), f), torques=np.zeros((N, D), f),
        commands=np.zeros((N, 4), f), feet_air_time=np.zeros((N, F), f), last_contacts=np.zeros((N, F), np.uint8),
        episode_length=np.zeros(N, np.int64), obs=np.zeros((N, spec.num_obs), f),
        priv_obs=np.zeros((N, spec.num_privileged_obs), f) if spec.num_privileged_obs else None,
        rew=np.zeros(N, f), reset=np.zeros(N, np.uint8), time_out=np.zeros(N, np.uint8),
        episode_sums=np.zeros((nsum, N), f), episode_acc=np.zeros(nsum + 1, f), base_lin_vel=np.zeros((N, 3), f),
        base_ang_vel=np.zeros((N, 3), f), projected_gravity=np.zeros((N, 3), f), rpy=np.zeros((N, 3), f),
        env_origins=np.zeros((N, 3), f), phase=np.zeros(N, f), leg_phase=np.zeros((N, 2), f),
        rew_terms=np.zeros((max(len(spec.reward_names), 1), N), f),
        friction=np.ones(N, f), added_mass=np.zeros(N, f),
    )
    num_cols = np.floor(np.sqrt(N))
    xx, yy = np.meshgrid(np.arange(np.ceil(N / num_cols)), np.arange(num_cols), indexing="ij")
    b["env_origins"][:, 0] = spec.cfg.env.env_spacing * xx.flatten()[:N]
    b["env_origins"][:, 1] = spec.cfg.env.env_spacing * yy.flatten()[:N]
    return b
