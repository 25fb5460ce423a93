"""Self-collision (create_actor's self_collisions filter, reference legged_robot.py:373-374;
enabled by g1_config.py:65, h1_config.py:77, h1_2_config.py:86, off for Go2 go2_config.py:39).

PhysX is absent, so the contact model is the build's own (capsule proxies per URDF link,
leggedsim/selfcollision.py) and parity vs IsaacGym is unpinned; these tests pin its defining
properties on the CPU oracle.  HIP == oracle is tested on the GPU
(tests/test_gpu_self_collision.py)."""
import ctypes as C

import numpy as np
import pytest

import bridge
from hostspec import make_spec
from leggedsim import cabi
from leggedsim.selfcollision import body_frames, capsule_separation

HUMANOIDS = ["h1", "g1", "h1_2"]


@pytest.fixture
def oracle(oracle_lib):
    yield oracle_lib
    bridge.set_self_collision(oracle_lib, None)  # the oracle's pairs are process-global


def _points(model, group):
    sel = model.pt_shape == group
    return model.pt_body[sel][0], model.pt_pos[sel].astype(np.float64), model.pt_radius[sel].astype(np.float64)


@pytest.mark.parametrize("task", HUMANOIDS)
def test_capsule_proxies_enclose_their_shapes(task):
    s = make_spec(task)
    sc = s.self_collision
    groups = sorted(set(s.model.pt_shape.tolist()))
    assert len(groups) == len(sc.proxy_body)
    for k, g in enumerate(groups):
        b, P, rad = _points(s.model, g)
        assert sc.proxy_body[k] == b
        p0, p1, r = sc.capsules[k, 0:3].astype(np.float64), sc.capsules[k, 3:6].astype(np.float64), sc.capsules[k, 6]
        d = p1 - p0
        L2 = d @ d
        t = np.clip(((P - p0) @ d) / L2, 0, 1) if L2 > 0 else np.zeros(len(P))
        dist = np.linalg.norm(P - (p0 + t[:, None] * d), axis=1) + rad
        assert (dist <= r + 1e-5).all(), f"proxy {k} of body {b} leaves out a point by {(dist - r).max():.2e}"


@pytest.mark.parametrize("task", HUMANOIDS)
def test_pairs_follow_the_joint_filter_and_rest_pose(task):
    """PhysX never tests a link with itself or the link it is jointed to; pairs touching in
    the default pose are excluded (proxy slack) -- none of the tested pairs touch at rest."""
    s = make_spec(task)
    sc, m = s.self_collision, s.model
    assert len(sc.pairs) > 0
    R, p = body_frames(m, np.asarray(s.default_dof_pos).reshape(-1))
    for i, k in sc.pairs:
        a, b = sc.proxy_body[i], sc.proxy_body[k]
        assert a < b and m.parent[b] != a
        assert capsule_separation(sc.proxy_body, sc.capsules, R, p, i, k) >= 0.01


def test_go2_filters_self_collision():
    assert make_spec("go2").self_collision is None  # go2_config.py:39 self_collisions = 1


def crossed_pose(m, sc, q0, seed=0, tries=4000):
    """A joint vector near the default pose q0 in which exactly one tested pair overlaps by
    5-30 mm (its proxies interpenetrate), with the pair's index and separation."""
    q0 = np.asarray(q0, dtype=np.float64).reshape(-1)
    rng = np.random.default_rng(seed)
    for _ in range(tries):
        q = np.clip(q0 + rng.normal(0, 0.4, m.num_dofs), m.dof_lower, m.dof_upper)
        R, p = body_frames(m, q)
        seps = np.array([capsule_separation(sc.proxy_body, sc.capsules, R, p, i, k) for i, k in sc.pairs])
        hit = np.nonzero(seps < 0.012)[0]
        if len(hit) == 1 and -0.03 < seps[hit[0]] < -0.005:
            return q.astype(np.float32), int(hit[0]), float(seps[hit[0]])
    raise AssertionError("no single-pair self-contact pose found")


def _run(lib, s, q, substeps, with_self):
    bridge.set_self_collision(lib, s.self_collision if with_self else None)
    params = cabi.sim_params_from_cfg(s.cfg.sim, s.cfg.asset, gravity=(0.0, 0.0, 0.0),
                                      max_contacts=s.sim_params.max_contacts, max_rows=s.sim_params.max_rows)
    root = np.zeros((1, 13), np.float32)
    root[0, 2], root[0, 6] = 5.0, 1.0  # far above the ground, at rest
    dofs = np.zeros((s.num_dof, 2), np.float32)
    dofs[:, 0] = q
    tau = np.zeros((1, s.num_dof), np.float32)
    cf = np.zeros((s.num_bodies, 3), np.float32)
    rbs = np.zeros((s.num_bodies, 13), np.float32)
    mh = cabi.ModelHandle(s.model)
    P = lambda a: a.ctypes.data  # noqa: E731
    first = None
    for i in range(substeps):
        lib.orc_simulate(C.byref(mh.desc), C.byref(params), 1, P(root), P(dofs), P(tau), P(cf), P(rbs), None, None)
        if i == 0:
            first = cf.copy()
    return first, dofs[:, 0].copy()


@pytest.mark.parametrize("task", HUMANOIDS)
def test_self_contact_pushes_the_links_apart(task, oracle):
    """Legs crossed in the air, no gravity, no torque: the overlapping pair gets equal and
    opposite contact forces (internal: they sum to zero over the bodies) and the links are
    pushed apart; with self-collision off nothing touches and nothing moves."""
    s = make_spec(task)
    sc = s.self_collision
    q, pair, sep0 = crossed_pose(s.model, sc, s.default_dof_pos)
    i, k = sc.pairs[pair]
    a, b = int(sc.proxy_body[i]), int(sc.proxy_body[k])
    f, q_after = _run(oracle, s, q, 60, with_self=True)
    assert np.linalg.norm(f[a]) > 1.0, f"{s.model.body_names[a]} got no contact force"
    np.testing.assert_array_equal(f[a], -f[b])  # one contact: +F on the first body, -F on the second
    others = [x for x in range(s.num_bodies) if x not in (a, b)]
    assert not f[others].any()
    R, p = body_frames(s.model, q_after)
    sep1 = capsule_separation(sc.proxy_body, sc.capsules, R, p, i, k)
    assert sep1 > sep0 + 0.004, (sep0, sep1)
    f_off, q_off = _run(oracle, s, q, 60, with_self=False)
    assert not f_off.any()
    np.testing.assert_allclose(q_off, q, atol=1e-6)
