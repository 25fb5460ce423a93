"""Rough terrain: the height-map generator (legged_gym/utils/terrain.py over the
restated isaacgym.terrain_utils primitives) and the oracle's heightfield contact
ground (oracle/lgs_oracle.c orc_terrain_sample + contact frames), CPU only.

isaacgym.terrain_utils is absent from this image and no reference fixture covers
it (the reference never builds a heightfield): the generator's parity
is unpinned, so these tests check the defining properties of each primitive and
of the tile layout, and the contact ground against its own analytic statement.
"""
import copy
import ctypes as C

import numpy as np
import pytest

from hostspec import make_spec
from isaacgym import terrain_utils
from legged_gym.envs.base.legged_robot_config import LeggedRobotCfg
from legged_gym.utils.terrain import Terrain
from leggedsim import cabi


def tile(n=80, hs=0.1, vs=0.005):
    return terrain_utils.SubTerrain("t", width=n, length=n, vertical_scale=vs, horizontal_scale=hs)


def test_pyramid_stairs_rise_by_steps_to_a_flat_platform():
    t = terrain_utils.pyramid_stairs_terrain(tile(), step_width=0.31, step_height=0.1, platform_size=3.0)
    h = t.height_field_raw
    sw, sh = int(0.31 / 0.1), int(0.1 / 0.005)
    assert h[0, 0] == 0
    for k in range(1, 5):  # ring k sits k step heights up
        assert h[k * sw, 40] == k * sh
    centre = h[40, 40]
    assert centre == h.max() and centre % sh == 0
    assert (h[30:50, 30:50] == centre).all()  # the 3 m platform is flat
    d = terrain_utils.pyramid_stairs_terrain(tile(), step_width=0.31, step_height=-0.1, platform_size=3.0)
    assert d.height_field_raw[40, 40] == -centre


def test_pyramid_slope_gradient_and_platform():
    slope = 0.2
    t = terrain_utils.pyramid_sloped_terrain(tile(), slope=slope, platform_size=3.0)
    h = t.height_field_raw.astype(np.float64) * 0.005
    g = np.diff(h[40, :20]) / 0.1  # rise per metre along the centre line, below the platform clip
    assert abs(np.median(g) - slope) < 0.02
    assert h[40, 40] == h.max() and (h[30:50, 30:50] == h.max()).all()
    n = terrain_utils.pyramid_sloped_terrain(tile(), slope=-slope, platform_size=3.0)
    assert n.height_field_raw.max() == 0 and n.height_field_raw.min() < 0


def test_random_uniform_and_obstacles_stay_in_range():
    np.random.seed(3)
    t = terrain_utils.random_uniform_terrain(tile(), min_height=-0.05, max_height=0.05, step=0.005,
                                             downsampled_scale=0.2)
    assert t.height_field_raw.min() >= -10 and t.height_field_raw.max() <= 10
    assert len(np.unique(t.height_field_raw)) > 5
    o = terrain_utils.discrete_obstacles_terrain(tile(), 0.2, 1.0, 2.0, 20, platform_size=3.0)
    h = o.height_field_raw
    assert set(np.unique(h).tolist()) <= {-40, -20, 0, 20, 40}
    assert (h[25:55, 25:55] == 0).all()


def test_trimesh_uses_the_kernel_diagonal():
    h = np.arange(12, dtype=np.int16).reshape(3, 4)
    v, tri = terrain_utils.convert_heightfield_to_trimesh(h, 0.1, 0.005)
    assert v.shape == (12, 3) and tri.shape == (12, 3)
    # cell (0,0): triangles (0,0)-(1,1)-(0,1) and (0,0)-(1,0)-(1,1)
    assert list(tri[0]) == [0, 5, 1] and list(tri[1]) == [0, 4, 5]
    assert np.allclose(v[5], [0.1, 0.1, 5 * 0.005])


def terrain_cfg(**kw):
    cfg = copy.deepcopy(LeggedRobotCfg.terrain)
    cfg.mesh_type = "heightfield"
    for k, v in kw.items():
        setattr(cfg, k, v)
    return cfg


def test_curriculum_map_layout_and_origins():
    np.random.seed(1)
    cfg = terrain_cfg()
    t = Terrain(cfg, 4096)
    # 10 x 20 tiles of 8 m at 0.1 m with a 25 m border -> int16 1300 x 2100
    assert t.height_field_raw.shape == (1300, 2100) and t.height_field_raw.dtype == np.int16
    b = t.border
    assert (t.height_field_raw[:b] == 0).all() and (t.height_field_raw[:, :b] == 0).all()
    o = t.env_origins
    assert o.shape == (10, 20, 3)
    np.testing.assert_allclose(o[3, 7, :2], [3.5 * 8.0, 7.5 * 8.0])
    L = t.length_per_env_pixels
    for i, j in ((0, 0), (5, 12), (9, 19)):  # spawn height: highest sample within 1 m of the centre
        blk = t.height_field_raw[b + i * L:b + (i + 1) * L, b + j * L:b + (j + 1) * L]
        assert o[i, j, 2] == pytest.approx(blk[30:50, 30:50].max() * cfg.vertical_scale)
    col = 10  # choice 0.501: stairs; difficulty (the row) sets the step height
    span = [np.ptp(t.height_field_raw[b + i * L:b + (i + 1) * L, b + col * L:b + (col + 1) * L]) for i in range(10)]
    assert span[9] > span[1] > 0


def test_random_layout_is_seeded():
    np.random.seed(7)
    a = Terrain(terrain_cfg(curriculum=False, num_rows=3, num_cols=4), 16).height_field_raw.copy()
    np.random.seed(7)
    b = Terrain(terrain_cfg(curriculum=False, num_rows=3, num_cols=4), 16).height_field_raw
    assert np.array_equal(a, b)


# ------------------------------------------------------------ oracle ground --
def ref_sample(h, hs, vs, border, x, y):
    """numpy statement of the triangulated heightfield: height and unit normal."""
    u = np.clip((x + border) / hs, 0, h.shape[0] - 1)
    v = np.clip((y + border) / hs, 0, h.shape[1] - 1)
    i, j = min(int(u), h.shape[0] - 2), min(int(v), h.shape[1] - 2)
    fu, fv = u - i, v - j
    z = h.astype(np.float64) * vs
    if fu >= fv:  # triangle (i,j) (i+1,j) (i+1,j+1)
        P = [(i, j, z[i, j]), (i + 1, j, z[i + 1, j]), (i + 1, j + 1, z[i + 1, j + 1])]
    else:         # triangle (i,j) (i+1,j+1) (i,j+1)
        P = [(i, j, z[i, j]), (i + 1, j + 1, z[i + 1, j + 1]), (i, j + 1, z[i, j + 1])]
    P = np.array(P, dtype=np.float64)
    P[:, :2] = P[:, :2] * hs - border
    n = np.cross(P[1] - P[0], P[2] - P[0])
    n = n / np.linalg.norm(n) * np.sign(n[2])
    xc, yc = u * hs - border, v * hs - border
    return P[0, 2] - (n[0] * (xc - P[0, 0]) + n[1] * (yc - P[0, 1])) / n[2], n


@pytest.fixture()
def ground(oracle_lib):
    keep = []

    def set_hf(h, hs=0.1, vs=0.005, border=1.0):
        if h is None:
            oracle_lib.orc_set_heightfield(None, 0, 0, 0.0, 0.0, 0.0)
            return
        h = np.ascontiguousarray(h, dtype=np.int16)
        keep.append(h)
        oracle_lib.orc_set_heightfield(h.ctypes.data, h.shape[0], h.shape[1], hs, vs, border)

    yield set_hf
    oracle_lib.orc_set_heightfield(None, 0, 0, 0.0, 0.0, 0.0)


def sample(lib, x, y):
    n = (C.c_float * 3)()
    z = lib.orc_terrain_sample(x, y, C.cast(n, C.c_void_p))
    return z, np.array(n[:])


def test_oracle_ground_matches_the_triangulation(oracle_lib, ground):
    rng = np.random.default_rng(0)
    h = rng.integers(-60, 60, size=(20, 30)).astype(np.int16)
    ground(h, 0.1, 0.005, 1.0)
    for x, y in rng.uniform(-1.2, 2.1, size=(300, 2)):
        z, n = sample(oracle_lib, float(x), float(y))
        zr, nr = ref_sample(h, 0.1, 0.005, 1.0, float(x), float(y))
        assert z == pytest.approx(zr, abs=2e-5)
        np.testing.assert_allclose(n, nr, atol=2e-5)
    ground(None)
    z, n = sample(oracle_lib, 3.0, -2.0)
    assert z == 0.0 and list(n) == [0.0, 0.0, 1.0]


def _stand(lib, s, root, dofs, steps):
    """PD-hold the default pose for `steps` substeps (orc_simulate); returns forces, body states."""
    N, B = root.shape[0], s.num_bodies
    mh = cabi.ModelHandle(s.model)
    cf = np.zeros((N * B, 3), np.float32)
    rbs = np.zeros((N * B, 13), np.float32)
    d = s.default_dof_pos[0]
    p = lambda a: a.ctypes.data  # noqa: E731
    for _ in range(steps):
        q, qd = dofs[:, 0].reshape(N, -1), dofs[:, 1].reshape(N, -1)
        tau = np.clip(s.p_gains * (d - q) - s.d_gains * qd, -s.torque_limits, s.torque_limits).astype(np.float32)
        lib.orc_simulate(C.byref(mh.desc), C.byref(s.sim_params), N, p(root), p(dofs), p(tau), p(cf), p(rbs),
                         None, None)
    return cf, rbs


def _start(s, N, z):
    root = np.zeros((N, 13), np.float32)
    root[:, 0] = np.arange(N) * 0.7
    root[:, 2] = z
    root[:, 6] = 1.0
    dofs = np.zeros((N * s.num_dof, 2), np.float32)
    dofs[:, 0] = np.tile(s.default_dof_pos[0], N)
    return root, dofs


def test_flat_heightfield_is_exactly_the_plane(oracle_lib, ground):
    s = make_spec("go2")
    r1, d1 = _start(s, 3, 0.42)
    cf1, _ = _stand(oracle_lib, s, r1, d1, 200)
    ground(np.zeros((60, 60), np.int16), 0.1, 0.005, 3.0)
    r2, d2 = _start(s, 3, 0.42)
    cf2, _ = _stand(oracle_lib, s, r2, d2, 200)
    assert np.array_equal(r1, r2) and np.array_equal(d1, d2) and np.array_equal(cf1, cf2)
    assert (cf1.reshape(3, -1, 3)[:, s.feet_indices, 2] > 1.0).all()


def test_raised_ground_is_a_translation(oracle_lib, ground):
    s = make_spec("go2")
    r1, d1 = _start(s, 2, 0.42)
    cf1, _ = _stand(oracle_lib, s, r1, d1, 300)
    ground(np.full((60, 60), 40, np.int16), 0.1, 0.005, 3.0)  # ground at z = 0.2
    r2, d2 = _start(s, 2, 0.62)
    cf2, _ = _stand(oracle_lib, s, r2, d2, 300)
    np.testing.assert_allclose(r2[:, 2] - 0.2, r1[:, 2], atol=2e-4)
    np.testing.assert_allclose(r2[:, 3:], r1[:, 3:], atol=2e-3)
    np.testing.assert_allclose(d2, d1, atol=2e-3)
    np.testing.assert_allclose(cf2, cf1, atol=0.5)


def test_go2_stands_on_a_slope(oracle_lib, ground):
    """A 10 % slope along x: the contact normals tilt, static friction holds the robot,
    and the summed ground force balances its weight vertically."""
    s = make_spec("go2")
    h = (2 * np.arange(80)[:, None] * np.ones((1, 80))).astype(np.int16)  # 0.01 m per 0.1 m in x
    ground(h, 0.1, 0.005, 4.0)
    z0 = (0.0 + 4.0) * 0.1  # ground height under x = 0
    root, dofs = _start(s, 1, z0 + 0.44)
    cf, rbs = _stand(oracle_lib, s, root, dofs, 1400)
    W = s.model.mass.sum() * 9.81
    F = cf.reshape(-1, 3).sum(0)
    assert abs(F[2] - W) < 0.05 * W and abs(F[0]) < 0.05 * W and abs(F[1]) < 0.05 * W
    assert np.abs(root[0, 7:13]).max() < 0.05          # at rest, not sliding
    zf = rbs.reshape(-1, 13)[s.feet_indices]
    for f in zf:                                       # feet rest on the slope, not in it
        zg, n = sample(oracle_lib, float(f[0]), float(f[1]))
        assert -0.01 < f[2] - zg < 0.06
        np.testing.assert_allclose(n, [-0.1 / np.sqrt(1.01), 0.0, 1 / np.sqrt(1.01)], atol=1e-5)
    assert 0.15 < root[0, 2] - z0 < 0.45
