"""Runtime robot generality: a robot whose (DOFs, bodies) shape has no instantiation of its
own runs, with no rebuild, on a padded generic one (LGS_GENERIC_SHAPES in csrc/leggedsim.hip:
inert DOFs on massless bodies hinged to the base, M_jj = 1, then inert fixed bodies) and is
bit-exact with the oracle run on the UNPADDED model.

The robots are the reference's own with joints locked (the URDF joint made "fixed", its link
kept as a fixed body, as with collapse_fixed_joints=False for that joint):

* H1 with both ankles locked: 8 DOFs, 11 bodies -> padded to (16, 24);
* G1 23-DOF with both wrists locked: 21 DOFs, 24 bodies -> padded to (26, 32).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

import isaacgym  # noqa: F401,E402
import legged_gym.envs.base.legged_robot as lr  # noqa: E402
from test_gpu_parity import _register_g1_23dof, fused_vs_oracle, warm  # noqa: E402


def lock_dofs(model, names):
    """The model with the named joints fixed at q = 0 (their links stay as fixed bodies)."""
    gone = {model.dof_names.index(n) for n in names}
    keep = [j for j in range(model.num_dofs) if j not in gone]
    remap = -np.ones(model.num_dofs, np.int32)
    remap[keep] = np.arange(len(keep), dtype=np.int32)
    model.dof = np.where(model.dof >= 0, remap[np.maximum(model.dof, 0)], -1).astype(np.int32)
    model.dof_names = [model.dof_names[j] for j in keep]
    for k in ("dof_body", "dof_lower", "dof_upper", "dof_effort", "dof_velocity"):
        setattr(model, k, np.ascontiguousarray(getattr(model, k)[keep]))
    return model


@pytest.fixture
def locked(monkeypatch):
    def use(names):
        real = lr.load_model
        monkeypatch.setattr(lr, "load_model", lambda *a, **k: lock_dofs(real(*a, **k), names))
    return use


@pytest.mark.parametrize("n", [6, 512])
def test_h1_ankles_locked_runs_padded_and_matches_oracle_bitwise(locked, n):
    locked(["left_ankle_joint", "right_ankle_joint"])
    D = 8
    env, g = warm("h1", n, steps=8, seed=n, env__num_actions=D, env__num_observations=11 + 3 * D,
                  env__num_privileged_obs=14 + 3 * D)
    assert env.num_dof == D and env.num_bodies == 11
    assert env.sim.padded_shape() == (16, 24)
    assert env.sim.factor_chain() == 0  # dense instantiation: index-order Cholesky (the oracle's default)
    fused_vs_oracle(env, g, 3, f"h1 ankles locked x{n}")


@pytest.mark.parametrize("n", [37, 256])
def test_g1_23dof_wrists_locked_runs_padded_and_matches_oracle_bitwise(locked, n):
    _register_g1_23dof()
    locked(["left_wrist_roll_joint", "right_wrist_roll_joint"])
    D = 21
    env, g = warm("g1_23dof", n, steps=6, seed=n, env__num_actions=D, env__num_observations=9 + 3 * D + 2,
                  env__num_privileged_obs=12 + 3 * D + 2)
    assert env.num_dof == D and env.num_bodies == 24
    assert env.sim.padded_shape() == (26, 32)
    fused_vs_oracle(env, g, 2, f"g1_23dof wrists locked x{n}")


def test_padded_reset_and_forward_kinematics_match_oracle(locked):
    """gym.refresh_rigid_body_state_tensor (lgs_forward_kinematics) and reset_idx on the
    padded instantiation: every real body row equals the oracle's forward kinematics."""
    import ctypes as C
    import bridge
    from leggedsim import cabi
    locked(["left_ankle_joint", "right_ankle_joint"])
    D = 8
    env, g = warm("h1", 64, steps=5, env__num_actions=D, env__num_observations=11 + 3 * D,
                  env__num_privileged_obs=14 + 3 * D)
    env.reset_idx(torch.arange(0, 64, 3, device="cuda"))
    env.gym.refresh_rigid_body_state_tensor(env.sim)
    torch.cuda.synchronize()
    B = env.num_bodies
    got = env.rigid_body_states.view(64, B, 13).cpu().numpy()
    root = env.root_states.cpu().numpy()
    dofs = env.dof_state.cpu().numpy().reshape(64, -1)
    want = np.zeros((64, B, 13), np.float32)
    lib = bridge.ensure_built()
    mh = cabi.ModelHandle(env.model)
    for e in range(64):
        r, d = np.ascontiguousarray(root[e]), np.ascontiguousarray(dofs[e])
        lib.orc_body_states_env(C.byref(mh.desc), r.ctypes.data, d.ctypes.data, want[e].ctypes.data)
    np.testing.assert_array_equal(got, want)
