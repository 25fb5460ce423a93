"""Loader for the HIP simulator ``libleggedsim.so`` (the product path).

There is deliberately no CPU fallback: if the library or a GPU is missing the
env raises.  Build with ``make -C unitree-rl-gym_amd/csrc`` or
``__graft_entry__.build()``.
"""
from __future__ import annotations

import ctypes as C
import os

from . import cabi

_LIB = None
LIB_NAME = "libleggedsim.so"


def lib_path():
    env = os.environ.get("LEGGEDSIM_LIB")
    if env:
        return env
    here = os.path.dirname(os.path.abspath(__file__))
    return os.path.join(os.path.dirname(here), "csrc", "build", LIB_NAME)


class LeggedSimError(RuntimeError):
    pass


def load():
    """Load libleggedsim.so.  torch must be imported first so that the library
    binds to the same HIP runtime (same SONAME) torch already loaded."""
    global _LIB
    if _LIB is not None:
        return _LIB
    import torch  # noqa: F401  (HIP runtime first, see docstring)

    p = lib_path()
    if not os.path.exists(p):
        raise LeggedSimError(
            f"HIP simulator library not found at {p}; build it with `make -C unitree-rl-gym_amd/csrc` "
            "(no CPU fallback exists for the product path)")
    lib = C.CDLL(p)
    vp = C.c_void_p
    lib.lgs_last_error.restype = C.c_char_p
    lib.lgs_version.restype = C.c_int
    lib.lgs_uniform.restype = C.c_float
    lib.lgs_uniform.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]
    lib.lgs_create_sim.argtypes = [C.POINTER(cabi.ModelDesc), C.POINTER(cabi.SimParams), C.c_int32, C.c_int32,
                                   C.POINTER(vp)]
    lib.lgs_destroy_sim.argtypes = [vp]
    lib.lgs_set_stream.argtypes = [vp, vp]
    lib.lgs_synchronize.argtypes = [vp]
    lib.lgs_set_env_properties.argtypes = [vp, vp, vp]
    lib.lgs_bind_state.argtypes = [vp, vp, vp, vp, vp]
    lib.lgs_refresh.argtypes = [vp]
    lib.lgs_set_dof_actuation_force.argtypes = [vp, vp]
    lib.lgs_simulate.argtypes = [vp]
    lib.lgs_forward_kinematics.argtypes = [vp]
    lib.lgs_set_actor_root_state_indexed.argtypes = [vp, vp, vp, C.c_int32]
    lib.lgs_set_dof_state_indexed.argtypes = [vp, vp, vp, C.c_int32]
    lib.lgs_set_task.argtypes = [vp, C.POINTER(cabi.TaskParams)]
    lib.lgs_step.argtypes = [vp, C.POINTER(cabi.EnvBuffers), C.c_int64]
    lib.lgs_reset_all.argtypes = [vp, C.POINTER(cabi.EnvBuffers), C.c_int64]
    lib.lgs_step_physics.argtypes = [vp, C.POINTER(cabi.EnvBuffers), C.c_int64]
    lib.lgs_post_physics.argtypes = [vp, C.POINTER(cabi.EnvBuffers), C.c_int64]
    lib.lgs_reset_idx.argtypes = [vp, C.POINTER(cabi.EnvBuffers), vp, C.c_int64]
    lib.lgs_post_physics_rewards.argtypes = [vp, C.POINTER(cabi.EnvBuffers), C.c_int64]
    lib.lgs_post_physics_finish.argtypes = [vp, C.POINTER(cabi.EnvBuffers), C.c_int64]
    lib.lgs_post_physics_prepare.argtypes = [vp, C.POINTER(cabi.EnvBuffers), C.c_int64]
    lib.lgs_post_physics_term_rewards.argtypes = [vp, C.POINTER(cabi.EnvBuffers), C.c_int64]
    if hasattr(lib, "lgs_step_deferred"):  # (absent only from pre-round-6 builds used in A/B timing)
        lib.lgs_step_deferred.argtypes = [vp, C.POINTER(cabi.EnvBuffers), C.c_int64]
        lib.lgs_step_extras.argtypes = [vp, C.POINTER(cabi.EnvBuffers), C.c_int64]
        lib.lgs_get_push_state.argtypes = [vp, C.POINTER(vp), C.POINTER(vp)]
        for name in ("lgs_step_deferred", "lgs_step_extras", "lgs_get_push_state"):
            getattr(lib, name).restype = C.c_int
    lib.lgs_get_counts.argtypes = [vp, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
    lib.lgs_set_heightfield.argtypes = [vp, vp, C.c_int32, C.c_int32, C.c_float, C.c_float, C.c_float]
    lib.lgs_set_self_collision.argtypes = [vp, C.POINTER(cabi.SelfCollisionDesc)]
    if hasattr(lib, "lgs_get_contact_stats"):  # (absent only from pre-round-4 builds used in A/B timing)
        lib.lgs_get_contact_stats.argtypes = [vp, vp, C.c_int32]
        lib.lgs_get_contact_stats.restype = C.c_int
    if hasattr(lib, "lgs_get_instantiation"):  # (absent only from pre-round-4 builds used in A/B timing)
        lib.lgs_get_instantiation.argtypes = [vp, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
        lib.lgs_get_instantiation.restype = C.c_int
    if hasattr(lib, "lgs_get_factor_chain"):
        lib.lgs_get_factor_chain.argtypes = [vp, C.POINTER(C.c_int32)]
        lib.lgs_get_factor_chain.restype = C.c_int
    for name in ("lgs_get_body_name", "lgs_get_dof_name"):
        getattr(lib, name).argtypes = [vp, C.c_int32]
        getattr(lib, name).restype = C.c_char_p
    for name in ("lgs_find_body", "lgs_find_dof"):
        getattr(lib, name).argtypes = [vp, C.c_char_p]
        getattr(lib, name).restype = C.c_int32
    for name in ("lgs_create_sim", "lgs_destroy_sim", "lgs_set_stream", "lgs_synchronize", "lgs_set_env_properties",
                 "lgs_bind_state", "lgs_refresh", "lgs_set_dof_actuation_force", "lgs_simulate",
                 "lgs_forward_kinematics", "lgs_set_actor_root_state_indexed", "lgs_set_dof_state_indexed",
                 "lgs_set_task", "lgs_step", "lgs_reset_all", "lgs_get_counts", "lgs_set_heightfield",
                 "lgs_step_physics", "lgs_post_physics", "lgs_reset_idx", "lgs_post_physics_rewards",
                 "lgs_post_physics_finish", "lgs_post_physics_prepare", "lgs_post_physics_term_rewards",
                 "lgs_set_self_collision"):
        getattr(lib, name).restype = C.c_int
    _LIB = lib
    return lib


def check(lib, status, what):
    if status != 0:
        raise LeggedSimError(f"{what} failed ({status}): {lib.lgs_last_error().decode(errors='replace')}")


EXPORTED_SYMBOLS = [
    "lgs_last_error", "lgs_version", "lgs_create_sim", "lgs_destroy_sim", "lgs_set_stream", "lgs_synchronize",
    "lgs_set_env_properties", "lgs_bind_state", "lgs_refresh", "lgs_set_dof_actuation_force", "lgs_simulate",
    "lgs_forward_kinematics", "lgs_set_actor_root_state_indexed", "lgs_set_dof_state_indexed", "lgs_set_task",
    "lgs_step", "lgs_reset_all", "lgs_get_counts", "lgs_uniform", "lgs_set_heightfield",
    "lgs_step_physics", "lgs_post_physics", "lgs_reset_idx", "lgs_post_physics_rewards", "lgs_post_physics_finish",
    "lgs_post_physics_prepare", "lgs_post_physics_term_rewards",
    "lgs_step_deferred", "lgs_step_extras", "lgs_get_push_state",
    "lgs_set_self_collision", "lgs_get_body_name", "lgs_get_dof_name", "lgs_find_body", "lgs_find_dof",
    "lgs_get_contact_stats", "lgs_get_instantiation", "lgs_get_factor_chain",
]


class Sim:
    """Thin owner of an ``lgs_sim*`` bound to caller-owned torch state tensors."""

    def __init__(self, model, sim_params: cabi.SimParams, num_envs: int, device_id: int):
        self.lib = load()
        self.model = model
        self._mh = cabi.ModelHandle(model)
        self._sp = sim_params
        h = C.c_void_p()
        check(self.lib, self.lib.lgs_create_sim(C.byref(self._mh.desc), C.byref(sim_params), num_envs, device_id,
                                                C.byref(h)), "lgs_create_sim")
        self.handle = h
        self.num_envs = num_envs

    def set_stream(self, stream_ptr):
        check(self.lib, self.lib.lgs_set_stream(self.handle, C.c_void_p(stream_ptr)), "lgs_set_stream")

    def set_env_properties(self, friction=None, added_mass=None):
        import numpy as np
        f = None if friction is None else np.ascontiguousarray(friction, dtype=np.float32)
        m = None if added_mass is None else np.ascontiguousarray(added_mass, dtype=np.float32)
        check(self.lib, self.lib.lgs_set_env_properties(
            self.handle, None if f is None else f.ctypes.data, None if m is None else m.ctypes.data),
            "lgs_set_env_properties")

    def set_heightfield(self, heights, horizontal_scale, vertical_scale, border_size):
        """gym.add_heightfield: int16 [rows, cols] height samples (None: the z = 0 plane)."""
        import numpy as np
        if heights is None:
            check(self.lib, self.lib.lgs_set_heightfield(self.handle, None, 0, 0, 0.0, 0.0, 0.0), "lgs_set_heightfield")
            self._hf = None
            return
        hf = np.ascontiguousarray(heights, dtype=np.int16)
        self._hf = hf
        check(self.lib, self.lib.lgs_set_heightfield(self.handle, hf.ctypes.data, hf.shape[0], hf.shape[1],
                                                     float(horizontal_scale), float(vertical_scale),
                                                     float(border_size)), "lgs_set_heightfield")

    def set_self_collision(self, sc):
        """create_actor's self-collision filter (legged_robot.py:373-374): sc is a
        leggedsim.selfcollision.SelfCollision, or None to turn self-collision off."""
        if sc is None or len(sc.pairs) == 0:
            check(self.lib, self.lib.lgs_set_self_collision(self.handle, None), "lgs_set_self_collision")
            self._sc = None
            return
        self._sc = cabi.SelfCollisionHandle(sc)
        check(self.lib, self.lib.lgs_set_self_collision(self.handle, C.byref(self._sc.desc)), "lgs_set_self_collision")

    def bind(self, root, dofs, cforce, rbs):
        for t in (root, dofs, cforce, rbs):
            assert t.is_cuda and t.is_contiguous() and str(t.dtype) == "torch.float32"
        self._bound = (root, dofs, cforce, rbs)
        check(self.lib, self.lib.lgs_bind_state(self.handle, root.data_ptr(), dofs.data_ptr(), cforce.data_ptr(),
                                                rbs.data_ptr()), "lgs_bind_state")

    def set_task(self, task: cabi.TaskParams):
        self._task = task
        check(self.lib, self.lib.lgs_set_task(self.handle, C.byref(task)), "lgs_set_task")

    def step(self, env_bufs: cabi.EnvBuffers, step_counter: int):
        check(self.lib, self.lib.lgs_step(self.handle, C.byref(env_bufs), step_counter), "lgs_step")

    def step_deferred(self, env_bufs: cabi.EnvBuffers, step_counter: int):
        """lgs_step without its extras launch (its consumer does that work)."""
        check(self.lib, self.lib.lgs_step_deferred(self.handle, C.byref(env_bufs), step_counter), "lgs_step_deferred")

    def step_extras(self, env_bufs: cabi.EnvBuffers, step_counter: int):
        """The extras of a deferred step, on their own (what lgs_step launches after the step)."""
        check(self.lib, self.lib.lgs_step_extras(self.handle, C.byref(env_bufs), step_counter), "lgs_step_extras")

    def push_state(self):
        """(vsim, pushed) device pointers of the push bookkeeping (lgs_get_push_state)."""
        v, p = C.c_void_p(), C.c_void_p()
        check(self.lib, self.lib.lgs_get_push_state(self.handle, C.byref(v), C.byref(p)), "lgs_get_push_state")
        return v.value, p.value

    def step_physics(self, env_bufs: cabi.EnvBuffers, step_counter: int):
        check(self.lib, self.lib.lgs_step_physics(self.handle, C.byref(env_bufs), step_counter), "lgs_step_physics")

    def post_physics(self, env_bufs: cabi.EnvBuffers, step_counter: int):
        check(self.lib, self.lib.lgs_post_physics(self.handle, C.byref(env_bufs), step_counter), "lgs_post_physics")

    def post_physics_rewards(self, env_bufs: cabi.EnvBuffers, step_counter: int):
        check(self.lib, self.lib.lgs_post_physics_rewards(self.handle, C.byref(env_bufs), step_counter),
              "lgs_post_physics_rewards")

    def post_physics_prepare(self, env_bufs: cabi.EnvBuffers, step_counter: int):
        check(self.lib, self.lib.lgs_post_physics_prepare(self.handle, C.byref(env_bufs), step_counter),
              "lgs_post_physics_prepare")

    def post_physics_term_rewards(self, env_bufs: cabi.EnvBuffers, step_counter: int):
        check(self.lib, self.lib.lgs_post_physics_term_rewards(self.handle, C.byref(env_bufs), step_counter),
              "lgs_post_physics_term_rewards")

    def post_physics_finish(self, env_bufs: cabi.EnvBuffers, step_counter: int):
        check(self.lib, self.lib.lgs_post_physics_finish(self.handle, C.byref(env_bufs), step_counter),
              "lgs_post_physics_finish")

    def reset_idx(self, env_bufs: cabi.EnvBuffers, mask_u8, step_counter: int):
        assert mask_u8.is_cuda and mask_u8.numel() == self.num_envs and mask_u8.element_size() == 1
        check(self.lib, self.lib.lgs_reset_idx(self.handle, C.byref(env_bufs), mask_u8.data_ptr(), step_counter),
              "lgs_reset_idx")

    def reset_all(self, env_bufs: cabi.EnvBuffers, step_counter: int):
        check(self.lib, self.lib.lgs_reset_all(self.handle, C.byref(env_bufs), step_counter), "lgs_reset_all")

    def simulate(self, torques):
        self._tau = torques
        check(self.lib, self.lib.lgs_set_dof_actuation_force(self.handle, torques.data_ptr()), "set_dof_actuation_force")
        check(self.lib, self.lib.lgs_simulate(self.handle), "lgs_simulate")

    def forward_kinematics(self):
        check(self.lib, self.lib.lgs_forward_kinematics(self.handle), "lgs_forward_kinematics")

    def set_root_indexed(self, src, ids_i32, n):
        check(self.lib, self.lib.lgs_set_actor_root_state_indexed(self.handle, src.data_ptr(), ids_i32.data_ptr(), n),
              "set_actor_root_state_indexed")

    def set_dof_indexed(self, src, ids_i32, n):
        check(self.lib, self.lib.lgs_set_dof_state_indexed(self.handle, src.data_ptr(), ids_i32.data_ptr(), n),
              "set_dof_state_indexed")

    def contact_stats(self, reset=False):
        """Capacity drops summed over envs and substeps (lgs_get_contact_stats): a dict of
        touching bodies without a contact slot, self contacts without one, joint limits
        without a row.  Synchronises the sim's stream."""
        import numpy as np
        out = np.zeros(cabi.NUM_CONTACT_STATS, dtype=np.uint64)
        check(self.lib, self.lib.lgs_get_contact_stats(self.handle, out.ctypes.data, int(bool(reset))),
              "lgs_get_contact_stats")
        return {"bodies": int(out[0]), "self": int(out[1]), "limits": int(out[2])}

    def padded_shape(self):
        """(DOFs, bodies) of the compiled kernel the sim runs on (the model padded to it)."""
        d, b = C.c_int32(), C.c_int32()
        check(self.lib, self.lib.lgs_get_instantiation(self.handle, C.byref(d), C.byref(b), None),
              "lgs_get_instantiation")
        return d.value, b.value

    def factor_chain(self):
        """The chain length the kernel's Cholesky eliminates level by level (0: index order);
        pre-level-order builds (A/B timing only) report 0."""
        if not hasattr(self.lib, "lgs_get_factor_chain"):
            return 0
        ch = C.c_int32()
        check(self.lib, self.lib.lgs_get_factor_chain(self.handle, C.byref(ch)), "lgs_get_factor_chain")
        return ch.value

    # name queries (gym.get_asset_rigid_body_names / get_asset_dof_names /
    # find_actor_rigid_body_handle, legged_robot.py:342-343, 388-407)
    def body_names(self):
        n, b, d = C.c_int32(), C.c_int32(), C.c_int32()
        check(self.lib, self.lib.lgs_get_counts(self.handle, C.byref(n), C.byref(b), C.byref(d)), "lgs_get_counts")
        return [self.lib.lgs_get_body_name(self.handle, i).decode() for i in range(b.value)]

    def dof_names(self):
        n, b, d = C.c_int32(), C.c_int32(), C.c_int32()
        check(self.lib, self.lib.lgs_get_counts(self.handle, C.byref(n), C.byref(b), C.byref(d)), "lgs_get_counts")
        return [self.lib.lgs_get_dof_name(self.handle, i).decode() for i in range(d.value)]

    def find_body(self, name):
        return int(self.lib.lgs_find_body(self.handle, name.encode()))

    def find_dof(self, name):
        return int(self.lib.lgs_find_dof(self.handle, name.encode()))

    def close(self):
        if getattr(self, "handle", None):
            self.lib.lgs_destroy_sim(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
