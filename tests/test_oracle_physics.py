"""Analytic checks of the oracle's rigid-body dynamics (the physics half of the
oracle is the build's own algorithm: PhysX is closed source, so parity vs
IsaacGym is unpinned and these properties pin it instead)."""
import ctypes as C

import numpy as np
import pytest

from hostspec import make_spec
from leggedsim import cabi


def sim(lib, spec, root, dofs, tau, params=None, n=1, steps=1):
    mh = cabi.ModelHandle(spec.model)
    sp = params or spec.sim_params
    B = spec.num_bodies
    cf = np.zeros((root.shape[0] * B, 3), np.float32)
    rbs = np.zeros((root.shape[0] * B, 13), np.float32)
    p = lambda a: a.ctypes.data  # noqa: E731
    for _ in range(steps):
        lib.orc_simulate(C.byref(mh.desc), C.byref(sp), root.shape[0], p(root), p(dofs), p(tau), p(cf), p(rbs),
                         None, None)
    return cf, rbs


def init_state(spec, N=1, z=5.0):
    root = np.zeros((N, 13), np.float32)
    root[:, 2] = z
    root[:, 6] = 1.0
    dofs = np.zeros((N * spec.num_dof, 2), np.float32)
    dofs[:, 0] = np.tile(spec.default_dof_pos[0], N)
    return root, dofs


@pytest.mark.parametrize("task", ["go2", "h1", "g1", "h1_2"])
def test_free_fall_is_rigid_and_matches_integrator(task, oracle_lib):
    s = make_spec(task)
    root, dofs = init_state(s, z=20.0)
    tau = np.zeros((1, s.num_dof), np.float32)
    n = 100
    sim(oracle_lib, s, root, dofs, tau, steps=n)
    dt, g = s.sim_params.dt, 9.81
    # semi-implicit Euler: v_n = -g dt n ; z_n = z0 - g dt^2 n(n+1)/2  (the COM of the whole body)
    assert abs(root[0, 9] - (-g * dt * n)) < 2e-3
    assert abs(root[0, 2] - (20.0 - g * dt * dt * n * (n + 1) / 2)) < 2e-3
    # no internal motion: gravity alone produces no joint acceleration
    np.testing.assert_allclose(dofs[:, 0], np.tile(s.default_dof_pos[0], 1), atol=2e-4)
    assert np.abs(dofs[:, 1]).max() < 2e-3
    np.testing.assert_allclose(root[0, 3:7], [0, 0, 0, 1], atol=1e-4)


def _momentum(spec, rbs):
    B = spec.num_bodies
    m = spec.model.mass
    v = rbs.reshape(-1, B, 13)[0, :, 7:10]
    return (m[:, None] * v).sum(0)


@pytest.mark.parametrize("task", ["go2", "h1"])
def test_zero_gravity_momentum_converges_first_order(task, oracle_lib):
    """No external force: total linear momentum is constant up to the semi-implicit
    Euler error, which must halve when dt halves (a wrong bias/Coriolis term would
    leave an O(1) residual instead)."""
    s = make_spec(task)
    rng = np.random.default_rng(0)
    qd0 = rng.normal(0, 3.0, s.num_dof).astype(np.float32)
    w0 = rng.normal(0, 0.5, 6).astype(np.float32)

    def drift(dt, T=0.05):
        params = cabi.sim_params_from_cfg(s.cfg.sim, s.cfg.asset, gravity=(0.0, 0.0, 0.0), clamp_joint_velocity=0,
                                          max_contacts=s.sim_params.max_contacts, max_rows=s.sim_params.max_rows,
                                          dt=dt)
        root, dofs = init_state(s, z=50.0)
        root[0, 7:13] = w0
        dofs[:, 1] = qd0
        tau = np.zeros((1, s.num_dof), np.float32)
        _, rbs0 = sim(oracle_lib, s, root, dofs, tau, params, steps=1)
        p0 = _momentum(s, rbs0)
        _, rbs = sim(oracle_lib, s, root, dofs, tau, params, steps=int(round(T / dt)) - 1)
        return np.abs(_momentum(s, rbs) - p0).max(), np.abs(p0).max()

    d1, pmag = drift(0.004)
    d2, _ = drift(0.002)
    assert d1 < 0.02 * max(pmag, 1.0)
    assert 0.35 < d2 / d1 < 0.65


def test_go2_stands_on_pd_and_feet_carry_weight(oracle_lib):
    s = make_spec("go2")
    N = 4
    root, dofs = init_state(s, N=N, z=0.42)
    d = s.default_dof_pos[0]
    kp, kd = s.p_gains, s.d_gains
    lim = s.torque_limits
    mh = cabi.ModelHandle(s.model)
    B = s.num_bodies
    cf = np.zeros((N * B, 3), np.float32)
    p = lambda a: a.ctypes.data  # noqa: E731
    for _ in range(1200):  # 6 s: Kd = 0.5 leaves a slowly decaying pitch rocking
        q = dofs[:, 0].reshape(N, -1)
        qd = dofs[:, 1].reshape(N, -1)
        tau = np.clip(kp * (d - q) - kd * qd, -lim, lim).astype(np.float32)
        oracle_lib.orc_simulate(C.byref(mh.desc), C.byref(s.sim_params), N, p(root), p(dofs), p(tau), p(cf), None,
                                None, None)
    weight = s.model.mass.sum() * 9.81
    fz = cf.reshape(N, B, 3)[:, :, 2]
    feet = s.feet_indices
    assert np.all(np.abs(fz[:, feet].sum(1) - weight) < 0.05 * weight)  # feet carry the robot
    assert np.all(fz[:, feet] > 1.0)                                     # all four feet touch
    assert np.all(np.abs(root[:, 7:13]) < 0.05)                          # at rest
    assert np.all((root[:, 2] > 0.15) & (root[:, 2] < 0.42))             # standing, not fallen


def test_joint_limits_hold(oracle_lib):
    s = make_spec("go2")
    root, dofs = init_state(s, z=30.0)
    params = cabi.sim_params_from_cfg(s.cfg.sim, s.cfg.asset, gravity=(0.0, 0.0, 0.0),
                                      max_contacts=s.sim_params.max_contacts, max_rows=s.sim_params.max_rows)
    tau = np.zeros((1, s.num_dof), np.float32)
    tau[0, 2] = -35.0  # FL calf driven hard into its lower limit
    sim(oracle_lib, s, root, dofs, tau, params, steps=400)
    lo = s.model.dof_lower[2]
    assert dofs[2, 0] > lo - 0.01


def test_rng_identical_in_product_and_oracle(oracle_lib):
    import torch  # noqa: F401  (shared HIP runtime before loading the product lib)
    from leggedsim import native
    lib = native.load()
    rng = np.random.default_rng(3)
    for _ in range(200):
        seed = int(rng.integers(0, 2 ** 63))
        args = [int(x) for x in rng.integers(0, 2 ** 31, 4)]
        a = lib.lgs_uniform(seed, *args)
        b = oracle_lib.orc_uniform(seed, *args)
        assert a == b and 0.0 <= a < 1.0


@pytest.mark.parametrize("task,ch", [("go2", 3), ("h1", 5), ("h1_2", 6)])
def test_level_order_factorisation_is_the_same_solve(task, ch, oracle_lib):
    """orc_set_factor_chain(CH): the chain-structured kernels eliminate the joint pivots level by
    level, so the base rows of L sum their leg terms in that order.  Only the rounding of those
    sums moves: PD-held standing from a drop, 40 substeps, agrees with the index-order
    factorisation to float noise (the GPU parity tests pin each order bit for bit)."""
    s = make_spec(task)
    out = []
    try:
        for c in (0, ch):
            oracle_lib.orc_set_factor_chain(c)
            root, dofs = init_state(s, N=2, z=0.6)
            tau = np.zeros((2, s.num_dof), np.float32)
            sim(oracle_lib, s, root, dofs, tau, n=2, steps=40)
            out.append((root.copy(), dofs.copy()))
    finally:
        oracle_lib.orc_set_factor_chain(0)
    np.testing.assert_allclose(out[1][0], out[0][0], atol=1e-4)
    np.testing.assert_allclose(out[1][1], out[0][1], atol=1e-3)
