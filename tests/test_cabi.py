"""The C-ABI library loads and exports every function include/leggedsim.h
declares, and the ctypes mirror has the C struct sizes (no GPU calls)."""
import ctypes as C
import os
import re

from conftest import ROOT
from leggedsim import cabi

HEADER = os.path.join(ROOT, "include", "leggedsim.h")


def declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"LGS_API\s+[\w\s\*]+?\b(lgs_\w+)\s*\(", src)))


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ("lgs_create_sim", "lgs_step", "lgs_simulate", "lgs_set_actor_root_state_indexed",
                 "lgs_set_dof_state_indexed", "lgs_bind_state", "lgs_reset_all", "lgs_last_error"):
        assert must in names


def test_library_exports_every_declared_symbol():
    import torch  # noqa: F401
    from leggedsim import native
    lib = C.CDLL(native.lib_path())
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    assert set(native.EXPORTED_SYMBOLS) <= set(declared_functions())


def test_ctypes_structs_match_c_layout(oracle_lib):
    oracle_lib.orc_sizeof.restype = C.c_long
    for i, st in enumerate((cabi.ModelDesc, cabi.SimParams, cabi.TaskParams, cabi.EnvBuffers,
                            cabi.SelfCollisionDesc)):
        assert C.sizeof(st) == oracle_lib.orc_sizeof(i), st.__name__


def test_error_path_without_gpu_is_a_status_not_a_crash():
    import torch
    from leggedsim import native
    lib = native.load()
    if torch.cuda.is_available():
        return
    h = C.c_void_p()
    rc = lib.lgs_create_sim(None, None, 0, 0, C.byref(h))
    assert rc != 0 and lib.lgs_last_error()


def test_name_queries_without_a_sim_are_null_not_a_crash():
    """lgs_get_body_name / lgs_get_dof_name / lgs_find_body / lgs_find_dof (the gym name
    queries of legged_robot.py:342-343, 388-407) on a NULL sim: NULL / -1 and an error text."""
    from leggedsim import native
    lib = native.load()
    assert lib.lgs_get_body_name(None, 0) is None and lib.lgs_last_error()
    assert lib.lgs_get_dof_name(None, 0) is None
    assert lib.lgs_find_body(None, b"base") == -1 and lib.lgs_find_dof(None, b"x") == -1


def test_deferred_step_entries_refuse_null_arguments():
    """lgs_step_deferred / lgs_step_extras / lgs_get_push_state (the rollout-consumed extras,
    include/leggedsim.h) on a NULL sim: a status and an error text, no launch."""
    from leggedsim import native
    lib = native.load()
    E = cabi.EnvBuffers()
    assert lib.lgs_step_deferred(None, C.byref(E), 0) != 0 and lib.lgs_last_error()
    assert lib.lgs_step_extras(None, C.byref(E), 0) != 0
    v, p = C.c_void_p(), C.c_void_p()
    assert lib.lgs_get_push_state(None, C.byref(v), C.byref(p)) != 0
