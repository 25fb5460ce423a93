"""Python side of the CPU ORACLE (test infrastructure only).

Runs ``oracle/lgs_oracle.c`` on host copies of a live env's buffers so tests,
``__graft_entry__.smoke()`` and bench.py's cpu_baseline leg can compare the HIP
product path against it.  Nothing in the product package imports this module.
"""
from __future__ import annotations

import ctypes as C
import os
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_PKG = os.path.join(_HERE, "..", "unitree-rl-gym_amd")
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)

from leggedsim import cabi  # noqa: E402

STATE_KEYS = ("root", "dofs", "cforce", "rbs")
ENV_KEYS = ("actions", "last_actions", "last_dof_vel", "last_root_vel", "torques", "commands", "feet_air_time",
            "last_contacts", "episode_length", "obs", "priv_obs", "rew", "reset", "time_out", "episode_sums",
            "episode_acc", "base_lin_vel", "base_ang_vel", "projected_gravity", "rpy", "env_origins", "phase",
            "leg_phase")


_made = False


def ensure_built():
    """(Re)build the oracle if its source changed (make is incremental), then load it."""
    global _made
    if not _made:
        import subprocess
        subprocess.check_call(["make", "-s", "-C", _HERE], stdout=subprocess.DEVNULL)
        _made = True
    return cabi.load_oracle()


def snapshot(env):
    """Host copies of every buffer lgs_step reads or writes."""
    import torch
    torch.cuda.synchronize()
    t = lambda x: None if x is None else x.detach().cpu().numpy().copy()  # noqa: E731
    i = env._buf_idx ^ 1  # the buffers the NEXT step writes
    snap = {
        "root": t(env.root_states), "dofs": t(env.dof_state), "cforce": t(env._contact_forces),
        "rbs": t(env.rigid_body_states), "actions": t(env.actions), "last_actions": t(env.last_actions),
        "last_dof_vel": t(env.last_dof_vel), "last_root_vel": t(env.last_root_vel), "torques": t(env.torques),
        "commands": t(env.commands), "feet_air_time": t(env.feet_air_time),
        "last_contacts": t(env.last_contacts).astype(np.uint8), "episode_length": t(env._episode_length),
        "obs": t(env._obs_bufs[i]), "priv_obs": t(env._priv_bufs[i]), "rew": t(env.rew_buf),
        "reset": t(env._reset_bufs[i]).astype(np.uint8), "time_out": t(env._timeout_bufs[i]).astype(np.uint8),
        "episode_sums": t(env._episode_sums), "episode_acc": np.zeros_like(t(env._episode_acc[0])),
        "base_lin_vel": t(env.base_lin_vel), "base_ang_vel": t(env.base_ang_vel),
        "projected_gravity": t(env.projected_gravity), "rpy": t(env.rpy), "env_origins": t(env.env_origins),
        "phase": t(env.phase), "leg_phase": t(env.leg_phase),
        "friction": np.ascontiguousarray(env.shape_friction, dtype=np.float32),
        "added_mass": np.ascontiguousarray(env.added_base_mass, dtype=np.float32),
    }
    return snap


def _env_struct(b):
    E = cabi.EnvBuffers()
    for k in ENV_KEYS:
        arr = b.get(k)
        setattr(E, k, None if arr is None else arr.ctypes.data)
    E.rew_terms = None if b.get("rew_terms") is None else b["rew_terms"].ctypes.data
    return E


_ground = None  # the heightfield array the oracle points at (kept alive here)


def set_ground(lib, terrain=None, terrain_cfg=None):
    """Point the oracle's contact ground at an env's heightfield (or the z = 0 plane)."""
    global _ground
    if terrain is None:
        lib.orc_set_heightfield(None, 0, 0, 0.0, 0.0, 0.0)
        _ground = None
        return
    _ground = np.ascontiguousarray(terrain.heightsamples, dtype=np.int16)
    lib.orc_set_heightfield(_ground.ctypes.data, _ground.shape[0], _ground.shape[1],
                            float(terrain_cfg.horizontal_scale), float(terrain_cfg.vertical_scale),
                            float(terrain_cfg.border_size))


_self = None  # the self-collision arrays the oracle points at (kept alive here)


def set_self_collision(lib, sc=None):
    """Give the oracle an env's self-collision proxies and pairs (None: off)."""
    global _self
    if sc is None or len(sc.pairs) == 0:
        lib.orc_set_self_collision(None)
        _self = None
        return
    _self = cabi.SelfCollisionHandle(sc)
    lib.orc_set_self_collision(C.byref(_self.desc))


def set_env(lib, env):
    """Ground, self-collision and Cholesky elimination order of a live env's sim."""
    set_ground(lib, getattr(env, "terrain", None), env.cfg.terrain)
    set_self_collision(lib, getattr(env, "self_collision", None))
    lib.orc_set_factor_chain(env.sim.factor_chain())


def step(env, snap, actions, step_counter, lib=None):
    """One fused control step of every env on the CPU oracle.  Returns new arrays."""
    lib = lib or ensure_built()
    set_env(lib, env)
    b = {k: (None if v is None else np.ascontiguousarray(v).copy()) for k, v in snap.items()}
    b["actions"] = np.ascontiguousarray(actions, dtype=np.float32).copy()
    b["episode_acc"][:] = 0
    mh = cabi.ModelHandle(env.model)
    E = _env_struct(b)
    p = lambda a: a.ctypes.data  # noqa: E731
    lib.orc_step(C.byref(mh.desc), C.byref(env._lgs_params), C.byref(env.task_params), env.num_envs,
                 p(b["root"]), p(b["dofs"]), p(b["cforce"]), p(b["rbs"]), p(b["added_mass"]), p(b["friction"]),
                 C.byref(E), int(step_counter))
    return b


def step_raw(model, sim_params, task, num_envs, bufs, step_counter, lib=None, terrain=None, terrain_cfg=None,
             self_collision=None):
    """orc_step on caller-provided host arrays (bench cpu_baseline / golden tests)."""
    lib = lib or ensure_built()
    set_ground(lib, terrain, terrain_cfg)
    set_self_collision(lib, self_collision)
    mh = cabi.ModelHandle(model)
    E = _env_struct(bufs)
    p = lambda a: a.ctypes.data  # noqa: E731
    lib.orc_step(C.byref(mh.desc), C.byref(sim_params), C.byref(task), num_envs, p(bufs["root"]), p(bufs["dofs"]),
                 p(bufs["cforce"]), p(bufs["rbs"]), p(bufs["added_mass"]), p(bufs["friction"]), C.byref(E),
                 int(step_counter))
    return bufs
