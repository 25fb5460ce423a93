"""ctypes mirror of ``include/leggedsim.h`` (structs + function prototypes).

Both the product library (``libleggedsim.so``, HIP) and the CPU oracle consume the
same descriptor structs, so one definition serves both.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

MAX_BODIES = 32
MAX_DOFS = 26
MAX_DEPTH = 10
MAX_FEET = 4
MAX_CONTACT_BODIES = 16
MAX_OBS = 128
MAX_REWARDS = 24
MAX_SELF_PROXIES = 64
MAX_SELF_PAIRS = 192
NUM_CONTACT_STATS = 3  # lgs_get_contact_stats: bodies without a slot, self contacts without one, limits without a row

OBS_QUADRUPED = 0
OBS_HUMANOID = 1

# lgs_reward_id, in the header's order
REWARD_IDS = [
    "action_rate", "alive", "ang_vel_xy", "base_height", "collision", "contact", "contact_no_vel",
    "dof_acc", "dof_pos_limits", "dof_vel", "dof_vel_limits", "feet_air_time", "feet_contact_forces",
    "feet_stumble", "feet_swing_height", "hip_pos", "lin_vel_z", "orientation", "stand_still",
    "torque_limits", "torques", "tracking_ang_vel", "tracking_lin_vel",
]
REWARD_ID = {n: i for i, n in enumerate(REWARD_IDS)}
# the reference names the stumble term `_reward_stumble` but the cfg key is `feet_stumble`
REWARD_ALIASES = {"stumble": "feet_stumble"}

STREAM_NOISE, STREAM_CMD, STREAM_RESET_DOF, STREAM_RESET_ROOT, STREAM_RESET_CMD, STREAM_PUSH = range(6)

f32p = C.POINTER(C.c_float)
i32p = C.POINTER(C.c_int32)


class ModelDesc(C.Structure):
    _fields_ = [
        ("num_bodies", C.c_int32), ("num_dofs", C.c_int32), ("num_points", C.c_int32),
        ("parent", i32p), ("dof", i32p), ("subtree_end", i32p), ("depth", i32p), ("chain", i32p),
        ("joint_rot", f32p), ("joint_pos", f32p), ("axis", f32p), ("mass", f32p), ("com", f32p),
        ("inertia", f32p), ("dof_body", i32p), ("dof_lower", f32p), ("dof_upper", f32p),
        ("dof_effort", f32p), ("dof_velocity", f32p), ("pt_body", i32p), ("pt_pos", f32p),
        ("pt_radius", f32p), ("body_names", C.POINTER(C.c_char_p)), ("dof_names", C.POINTER(C.c_char_p)),
    ]


class SimParams(C.Structure):
    _fields_ = [
        ("dt", C.c_float), ("gravity", C.c_float * 3), ("solver_iterations", C.c_int32),
        ("contact_offset", C.c_float), ("rest_offset", C.c_float), ("max_depenetration_velocity", C.c_float),
        ("baumgarte", C.c_float), ("ground_friction", C.c_float), ("armature", C.c_float),
        ("clamp_joint_velocity", C.c_int32), ("max_contacts", C.c_int32), ("max_rows", C.c_int32),
    ]


class SelfCollisionDesc(C.Structure):
    _fields_ = [
        ("num_proxies", C.c_int32), ("proxy_body", i32p), ("capsule", f32p),
        ("num_pairs", C.c_int32), ("pair", i32p), ("max_self_contacts", C.c_int32),
    ]


class SelfCollisionHandle:
    """Keeps the numpy arrays alive behind a SelfCollisionDesc (leggedsim.selfcollision.SelfCollision)."""

    def __init__(self, sc):
        self.body = np.ascontiguousarray(sc.proxy_body, dtype=np.int32)
        self.caps = np.ascontiguousarray(sc.capsules, dtype=np.float32).reshape(-1)
        self.pairs = np.ascontiguousarray(sc.pairs, dtype=np.int32).reshape(-1)
        self.desc = SelfCollisionDesc(len(self.body), self.body.ctypes.data_as(i32p), self.caps.ctypes.data_as(f32p),
                                      len(self.pairs) // 2, self.pairs.ctypes.data_as(i32p),
                                      int(sc.max_self_contacts))


class TaskParams(C.Structure):
    _fields_ = [
        ("obs_layout", C.c_int32), ("num_obs", C.c_int32), ("num_privileged_obs", C.c_int32),
        ("num_actions", C.c_int32), ("decimation", C.c_int32), ("control_type", C.c_int32),
        ("action_scale", C.c_float), ("clip_actions", C.c_float), ("clip_observations", C.c_float),
        ("control_dt", C.c_float),
        ("p_gains", C.c_float * MAX_DOFS), ("d_gains", C.c_float * MAX_DOFS),
        ("default_dof_pos", C.c_float * MAX_DOFS), ("torque_limits", C.c_float * MAX_DOFS),
        ("soft_dof_pos_lower", C.c_float * MAX_DOFS), ("soft_dof_pos_upper", C.c_float * MAX_DOFS),
        ("dof_vel_limits", C.c_float * MAX_DOFS),
        ("obs_scale_lin_vel", C.c_float), ("obs_scale_ang_vel", C.c_float), ("obs_scale_dof_pos", C.c_float),
        ("obs_scale_dof_vel", C.c_float), ("commands_scale", C.c_float * 3),
        ("add_noise", C.c_int32), ("noise_vec", C.c_float * MAX_OBS),
        ("max_episode_length", C.c_float), ("max_episode_length_s", C.c_float),
        ("resample_interval", C.c_int32), ("heading_command", C.c_int32),
        ("cmd_lin_vel_x", C.c_float * 2), ("cmd_lin_vel_y", C.c_float * 2), ("cmd_ang_vel_yaw", C.c_float * 2),
        ("cmd_heading", C.c_float * 2),
        ("push_robots", C.c_int32), ("push_interval", C.c_int32), ("max_push_vel_xy", C.c_float),
        ("base_init_state", C.c_float * 13),
        ("num_feet", C.c_int32), ("feet_idx", C.c_int32 * MAX_FEET),
        ("num_penalised", C.c_int32), ("penalised_idx", C.c_int32 * MAX_CONTACT_BODIES),
        ("num_termination", C.c_int32), ("termination_idx", C.c_int32 * MAX_CONTACT_BODIES),
        ("num_hip", C.c_int32), ("hip_dofs", C.c_int32 * 8),
        ("num_rewards", C.c_int32), ("reward_ids", C.c_int32 * MAX_REWARDS),
        ("reward_scales", C.c_float * MAX_REWARDS),
        ("has_termination_reward", C.c_int32), ("termination_scale", C.c_float),
        ("only_positive_rewards", C.c_int32),
        ("tracking_sigma", C.c_float), ("base_height_target", C.c_float), ("max_contact_force", C.c_float),
        ("soft_dof_vel_limit", C.c_float), ("soft_torque_limit", C.c_float),
        ("phase_period", C.c_float), ("phase_offset", C.c_float), ("stance_threshold", C.c_float),
        ("swing_height_target", C.c_float),
        ("seed", C.c_uint64),
        ("write_body_states", C.c_int32),
        ("custom_origins", C.c_int32),
        ("defer_reward_total", C.c_int32), ("num_extra_sums", C.c_int32),
        ("body_state_mask", C.c_uint32),
    ]


class EnvBuffers(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in (
        "actions", "last_actions", "last_dof_vel", "last_root_vel", "torques", "commands", "feet_air_time",
        "last_contacts", "episode_length", "obs", "priv_obs", "rew", "reset", "time_out", "episode_sums",
        "episode_acc", "base_lin_vel", "base_ang_vel", "projected_gravity", "rpy", "env_origins", "phase",
        "leg_phase", "rew_terms", "step_counter", "ep_means", "ep_snapshot", "time_outs_carry", "actions_in",
        "episode_acc_next")]


class ModelHandle:
    """Keeps the numpy arrays alive behind a ModelDesc."""

    def __init__(self, model):
        self.model = model
        m = model
        self._keep = {}

        def ip(name, a):
            a = np.ascontiguousarray(a, dtype=np.int32)
            self._keep[name] = a
            return a.ctypes.data_as(i32p)

        def fp(name, a):
            a = np.ascontiguousarray(a, dtype=np.float32)
            self._keep[name] = a
            return a.ctypes.data_as(f32p)

        self.desc = ModelDesc(
            m.num_bodies, m.num_dofs, m.num_points,
            ip("parent", m.parent), ip("dof", m.dof), ip("subtree_end", m.subtree_end), ip("depth", m.depth),
            ip("chain", m.chain), fp("joint_rot", m.joint_rot), fp("joint_pos", m.joint_pos), fp("axis", m.axis),
            fp("mass", m.mass), fp("com", m.com), fp("inertia", m.inertia), ip("dof_body", m.dof_body),
            fp("dof_lower", m.dof_lower), fp("dof_upper", m.dof_upper), fp("dof_effort", m.dof_effort),
            fp("dof_velocity", m.dof_velocity), ip("pt_body", m.pt_body), fp("pt_pos", m.pt_pos),
            fp("pt_radius", m.pt_radius), self._names("body_names", m.body_names),
            self._names("dof_names", m.dof_names))

    def _names(self, key, names):
        arr = (C.c_char_p * len(names))(*[n.encode() for n in names])
        self._keep[key] = arr
        return C.cast(arr, C.POINTER(C.c_char_p))


def sim_params_from_cfg(sim_cfg=None, asset_cfg=None, **over):
    """cfg.sim / cfg.sim.physx / cfg.asset -> SimParams (legged_robot_config.py:131-143,225-242)."""
    p = SimParams()
    p.dt = 0.005
    p.gravity[:] = (0.0, 0.0, -9.81)
    p.solver_iterations = 8
    p.contact_offset = 0.01
    p.rest_offset = 0.0
    p.max_depenetration_velocity = 1.0
    p.baumgarte = 0.2
    p.ground_friction = 1.0
    p.armature = 0.0
    p.clamp_joint_velocity = 1
    p.max_contacts = 8
    p.max_rows = 32
    if sim_cfg is not None:
        p.dt = float(sim_cfg.dt)
        p.gravity[:] = tuple(float(x) for x in sim_cfg.gravity)
        px = getattr(sim_cfg, "physx", None)
        if px is not None:
            # PhysX runs num_position_iterations TGS iterations; the budget here is two plain
            # Gauss-Seidel sweeps per position iteration.  A task's physx.pgs_sweeps (the fewest
            # sweeps that meet the convergence bar on its contacts, measured with
            # tools/pgs_sweeps: DESIGN 3.2) replaces it.
            sweeps = getattr(px, "pgs_sweeps", None)
            p.solver_iterations = int(sweeps) if sweeps else \
                max(1, 2 * int(px.num_position_iterations) + int(px.num_velocity_iterations))
            p.contact_offset = float(px.contact_offset)
            p.rest_offset = float(px.rest_offset)
            p.max_depenetration_velocity = float(px.max_depenetration_velocity)
    if asset_cfg is not None:
        p.armature = float(getattr(asset_cfg, "armature", 0.0))
    for k, v in over.items():
        if k == "gravity":
            p.gravity[:] = tuple(v)
        else:
            setattr(p, k, v)
    return p


def _find_lib(name, env_var):
    here = os.path.dirname(os.path.abspath(__file__))
    cands = [os.environ.get(env_var, "")]
    cands += [os.path.join(here, name)]
    for c in cands:
        if c and os.path.exists(c):
            return c
    return None


def oracle_path():
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    return os.path.join(root, "oracle", "_build", "liblgs_oracle.so")


def load_oracle(path=None):
    """The CPU oracle (test infrastructure only); path: another build of it (e.g. -march=native)."""
    p = path or oracle_path()
    if not os.path.exists(p):
        raise FileNotFoundError(f"oracle not built: {p} (run `make -C oracle`)")
    lib = C.CDLL(p)
    vp = C.c_void_p
    lib.orc_uniform.restype = C.c_float
    lib.orc_uniform.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]
    lib.orc_simulate.argtypes = [C.POINTER(ModelDesc), C.POINTER(SimParams), C.c_int, vp, vp, vp, vp, vp, vp, vp]
    lib.orc_step.argtypes = [C.POINTER(ModelDesc), C.POINTER(SimParams), C.POINTER(TaskParams), C.c_int,
                             vp, vp, vp, vp, vp, vp, C.POINTER(EnvBuffers), C.c_int64]
    lib.orc_step_physics.argtypes = [C.POINTER(ModelDesc), C.POINTER(SimParams), C.POINTER(TaskParams), C.c_int,
                                     vp, vp, vp, vp, vp, vp, C.POINTER(EnvBuffers)]
    lib.orc_reset_idx.argtypes = [C.POINTER(ModelDesc), C.POINTER(TaskParams), C.c_int, vp, vp,
                                  C.POINTER(EnvBuffers), vp, C.c_int64]
    lib.orc_post_physics.argtypes = [C.POINTER(ModelDesc), C.POINTER(TaskParams), C.c_int, vp, vp, vp, vp,
                                     C.POINTER(EnvBuffers), C.c_int64]
    lib.orc_compute_torques.argtypes = [C.POINTER(TaskParams), C.c_int, C.c_int, vp, vp, vp, C.c_float, vp]
    lib.orc_body_states_env.argtypes = [C.POINTER(ModelDesc), vp, vp, vp]
    lib.orc_set_heightfield.argtypes = [vp, C.c_int, C.c_int, C.c_float, C.c_float, C.c_float]
    lib.orc_set_heightfield.restype = None
    lib.orc_terrain_sample.argtypes = [C.c_float, C.c_float, vp]
    lib.orc_terrain_sample.restype = C.c_float
    lib.orc_set_self_collision.argtypes = [C.POINTER(SelfCollisionDesc)]
    lib.orc_set_self_collision.restype = None
    lib.orc_set_factor_chain.argtypes = [C.c_int]
    lib.orc_set_factor_chain.restype = None
    lib.orc_contact_stats.argtypes = [vp, C.c_int]
    lib.orc_contact_stats.restype = None
    return lib
