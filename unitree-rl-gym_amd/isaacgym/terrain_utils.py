"""Heightfield primitives of ``isaacgym.terrain_utils`` (IsaacGym Preview 4, public
Python module; absent from this image).

The reference's ``legged_gym/utils/terrain.py:5,65-115`` calls these by name;
this module restates their published algorithms so that ``Terrain`` builds the
same kind of int16 height map.  Heights are integers in units of
``vertical_scale``; the first array axis is x (``width`` samples), the second y
(``length`` samples).  Random draws use ``np.random`` exactly where the original
does (legged_gym seeds it through ``set_seed``), but no reference fixture covers
these functions: their parity is unpinned and the tests check
their defining properties instead.
"""
from __future__ import annotations

import numpy as np
from scipy.interpolate import RegularGridInterpolator


class SubTerrain:
    """One terrain tile: an int16 [width, length] height map plus its scales."""

    def __init__(self, terrain_name="terrain", width=256, length=256, vertical_scale=1.0, horizontal_scale=1.0):
        self.terrain_name = terrain_name
        self.vertical_scale = vertical_scale
        self.horizontal_scale = horizontal_scale
        self.width = int(width)
        self.length = int(length)
        self.height_field_raw = np.zeros((self.width, self.length), dtype=np.int16)


def _units(value, scale):
    return int(value / scale)


def random_uniform_terrain(terrain, min_height, max_height, step=1, downsampled_scale=None):
    """Uniform random heights in [min, max] (step `step`) on a coarse grid of pitch
    `downsampled_scale`, bilinearly upsampled to the tile and rounded."""
    if downsampled_scale is None:
        downsampled_scale = terrain.horizontal_scale
    lo, hi = _units(min_height, terrain.vertical_scale), _units(max_height, terrain.vertical_scale)
    st = max(_units(step, terrain.vertical_scale), 1)
    levels = np.arange(lo, hi + st, st)
    ext_x = terrain.width * terrain.horizontal_scale
    ext_y = terrain.length * terrain.horizontal_scale
    coarse = np.random.choice(levels, (int(ext_x / downsampled_scale), int(ext_y / downsampled_scale)))
    gx = np.linspace(0.0, ext_x, coarse.shape[0])
    gy = np.linspace(0.0, ext_y, coarse.shape[1])
    interp = RegularGridInterpolator((gx, gy), coarse.astype(np.float64), method="linear")
    fx = np.linspace(0.0, ext_x, terrain.width)
    fy = np.linspace(0.0, ext_y, terrain.length)
    px, py = np.meshgrid(fx, fy, indexing="ij")
    fine = np.rint(interp(np.stack([px.ravel(), py.ravel()], axis=1))).reshape(terrain.width, terrain.length)
    terrain.height_field_raw += fine.astype(np.int16)
    return terrain


def sloped_terrain(terrain, slope=1):
    """A plane rising along x with gradient `slope`."""
    x = np.arange(terrain.width).reshape(terrain.width, 1)
    rise = int(slope * (terrain.horizontal_scale / terrain.vertical_scale) * terrain.width)
    terrain.height_field_raw[:, :] += (rise * x / terrain.width).astype(terrain.height_field_raw.dtype)
    return terrain


def pyramid_sloped_terrain(terrain, slope=1, platform_size=1.0):
    """A four-sided pyramid (negative slope: a pit) with gradient `slope`, flattened
    to a square platform of side `platform_size` at the top (bottom)."""
    cx, cy = int(terrain.width / 2), int(terrain.length / 2)
    fx = (cx - np.abs(cx - np.arange(terrain.width))) / cx
    fy = (cy - np.abs(cy - np.arange(terrain.length))) / cy
    peak = int(slope * (terrain.horizontal_scale / terrain.vertical_scale) * (terrain.width / 2))
    terrain.height_field_raw += (peak * fx.reshape(-1, 1) * fy.reshape(1, -1)).astype(terrain.height_field_raw.dtype)
    half = int(platform_size / terrain.horizontal_scale / 2)
    corner = terrain.height_field_raw[terrain.width // 2 - half, terrain.length // 2 - half]
    terrain.height_field_raw = np.clip(terrain.height_field_raw, min(corner, 0), max(corner, 0))
    return terrain


def discrete_obstacles_terrain(terrain, max_height, min_size, max_size, num_rects, platform_size=1.0):
    """`num_rects` axis-aligned blocks of random size and height in
    {-h, -h/2, h/2, h}, on a 4-sample lattice, with a flat platform at the centre."""
    h = _units(max_height, terrain.vertical_scale)
    smin, smax = _units(min_size, terrain.horizontal_scale), _units(max_size, terrain.horizontal_scale)
    plat = _units(platform_size, terrain.horizontal_scale)
    nx, ny = terrain.height_field_raw.shape
    heights = [-h, -h // 2, h // 2, h]
    sizes = range(smin, smax, 4)
    for _ in range(num_rects):
        w = np.random.choice(sizes)
        ln = np.random.choice(sizes)
        i0 = np.random.choice(range(0, nx - w, 4))
        j0 = np.random.choice(range(0, ny - ln, 4))
        terrain.height_field_raw[i0:i0 + w, j0:j0 + ln] = np.random.choice(heights)
    x1, x2 = (terrain.width - plat) // 2, (terrain.width + plat) // 2
    y1, y2 = (terrain.length - plat) // 2, (terrain.length + plat) // 2
    terrain.height_field_raw[x1:x2, y1:y2] = 0
    return terrain


def wave_terrain(terrain, num_waves=1, amplitude=1.0):
    """Sum of a sine along x and a cosine along y with `num_waves` periods."""
    amp = int(0.5 * amplitude / terrain.vertical_scale)
    if num_waves > 0:
        div = terrain.length / (num_waves * np.pi * 2)
        x = np.arange(terrain.width).reshape(-1, 1)
        y = np.arange(terrain.length).reshape(1, -1)
        terrain.height_field_raw += (amp * np.cos(y / div) + amp * np.sin(x / div)).astype(terrain.height_field_raw.dtype)
    return terrain


def stairs_terrain(terrain, step_width, step_height):
    """Straight stairs along x."""
    sw, sh = _units(step_width, terrain.horizontal_scale), _units(step_height, terrain.vertical_scale)
    height = 0
    for k in range(terrain.width // sw):
        terrain.height_field_raw[k * sw:(k + 1) * sw, :] += height
        height += sh
    return terrain


def pyramid_stairs_terrain(terrain, step_width, step_height, platform_size=1.0):
    """Concentric square steps of width `step_width` rising (falling, for a negative
    height) by `step_height` towards a central platform of side >= `platform_size`."""
    sw, sh = _units(step_width, terrain.horizontal_scale), _units(step_height, terrain.vertical_scale)
    plat = _units(platform_size, terrain.horizontal_scale)
    x0, x1, y0, y1 = 0, terrain.width, 0, terrain.length
    level = 0
    while (x1 - x0) > plat and (y1 - y0) > plat:
        x0, x1, y0, y1 = x0 + sw, x1 - sw, y0 + sw, y1 - sw
        level += sh
        terrain.height_field_raw[x0:x1, y0:y1] = level
    return terrain


def stepping_stones_terrain(terrain, stone_size, stone_distance, max_height, platform_size=1.0, depth=-10):
    """Square stones of side `stone_size` separated by `stone_distance` over a pit of
    depth `depth`, heights uniform in [-max_height, max_height], central platform."""
    ss, sd = _units(stone_size, terrain.horizontal_scale), _units(stone_distance, terrain.horizontal_scale)
    h = _units(max_height, terrain.vertical_scale)
    plat = _units(platform_size, terrain.horizontal_scale)
    levels = np.arange(-h - 1, h, step=1)
    terrain.height_field_raw[:, :] = int(depth / terrain.vertical_scale)
    if terrain.length >= terrain.width:
        y = 0
        while y < terrain.length:
            y1 = min(terrain.length, y + ss)
            x = np.random.randint(0, ss)
            terrain.height_field_raw[0:max(0, x - sd), y:y1] = np.random.choice(levels)
            while x < terrain.width:
                x1 = min(terrain.width, x + ss)
                terrain.height_field_raw[x:x1, y:y1] = np.random.choice(levels)
                x += ss + sd
            y += ss + sd
    else:
        x = 0
        while x < terrain.width:
            x1 = min(terrain.width, x + ss)
            y = np.random.randint(0, ss)
            terrain.height_field_raw[x:x1, 0:max(0, y - sd)] = np.random.choice(levels)
            while y < terrain.length:
                y1 = min(terrain.length, y + ss)
                terrain.height_field_raw[x:x1, y:y1] = np.random.choice(levels)
                y += ss + sd
            x += ss + sd
    x1, x2 = (terrain.width - plat) // 2, (terrain.width + plat) // 2
    y1, y2 = (terrain.length - plat) // 2, (terrain.length + plat) // 2
    terrain.height_field_raw[x1:x2, y1:y2] = 0
    return terrain


def convert_heightfield_to_trimesh(height_field_raw, horizontal_scale, vertical_scale, slope_threshold=None):
    """Vertices [rows*cols, 3] and triangles [2*(rows-1)*(cols-1), 3] of the height map,
    each cell split along its (i,j)-(i+1,j+1) diagonal -- the triangulation the HIP
    contact kernel samples (lgs_set_heightfield).  With `slope_threshold`, samples
    next to a steeper rise are moved onto it (near-vertical walls)."""
    hf = height_field_raw
    nr, nc = hf.shape
    y = np.linspace(0, (nc - 1) * horizontal_scale, nc)
    x = np.linspace(0, (nr - 1) * horizontal_scale, nr)
    yy, xx = np.meshgrid(y, x)
    if slope_threshold is not None:
        thr = slope_threshold * horizontal_scale / vertical_scale
        mx, my, mxy = np.zeros((nr, nc)), np.zeros((nr, nc)), np.zeros((nr, nc))
        mx[:nr - 1, :] += (hf[1:, :] - hf[:nr - 1, :] > thr)
        mx[1:, :] -= (hf[:nr - 1, :] - hf[1:, :] > thr)
        my[:, :nc - 1] += (hf[:, 1:] - hf[:, :nc - 1] > thr)
        my[:, 1:] -= (hf[:, :nc - 1] - hf[:, 1:] > thr)
        mxy[:nr - 1, :nc - 1] += (hf[1:, 1:] - hf[:nr - 1, :nc - 1] > thr)
        mxy[1:, 1:] -= (hf[:nr - 1, :nc - 1] - hf[1:, 1:] > thr)
        xx = xx + (mx + mxy) * horizontal_scale
        yy = yy + (my + mxy) * horizontal_scale
    verts = np.zeros((nr * nc, 3), dtype=np.float32)
    verts[:, 0] = xx.ravel()
    verts[:, 1] = yy.ravel()
    verts[:, 2] = hf.ravel() * vertical_scale
    tris = np.zeros((2 * (nr - 1) * (nc - 1), 3), dtype=np.uint32)
    for i in range(nr - 1):
        i0 = np.arange(nc - 1) + i * nc
        i1, i2 = i0 + 1, i0 + nc
        i3 = i2 + 1
        s = 2 * i * (nc - 1)
        tris[s:s + 2 * (nc - 1):2] = np.stack([i0, i3, i1], axis=1)
        tris[s + 1:s + 2 * (nc - 1):2] = np.stack([i0, i2, i3], axis=1)
    return verts, tris
