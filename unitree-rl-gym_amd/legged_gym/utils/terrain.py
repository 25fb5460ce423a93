"""Rough-terrain height map (reference ``legged_gym/utils/terrain.py``).

The reference builds an int16 height map of ``num_rows x num_cols`` tiles
(``terrain_length x terrain_width`` metres each, ``border_size`` metres of flat
border) from ``isaacgym.terrain_utils`` primitives -- smooth/rough pyramid
slopes, pyramid stairs up/down and discrete obstacles, chosen by the cumulative
``terrain_proportions`` -- with one spawn origin per tile (:8-115).  The
reference's ``LeggedRobot.create_sim`` never calls it (it always adds a plane,
legged_robot.py:240-257); here ``mesh_type = 'heightfield'`` / ``'trimesh'``
hands the map to the simulator (``lgs_set_heightfield``), whose contact kernel
samples its triangulation.

Tile difficulty and type follow the reference: curriculum rows get difficulty
``row / num_rows`` and type ``col / num_cols + 0.001`` (:53-60); the random mode
draws ``choice ~ U(0,1)`` and ``difficulty in {0.5, 0.75, 0.9}`` per tile
(:44-51).  The spawn height of a tile is the highest sample within +-1 m of its
centre (:108-115).
"""
from __future__ import annotations

import numpy as np

from isaacgym import terrain_utils


def _tile_params(difficulty):
    """Per-difficulty primitive parameters (terrain.py:79-86)."""
    return dict(slope=difficulty * 0.4,
                step_height=0.05 + 0.18 * difficulty,
                obstacle_height=0.05 + difficulty * 0.2,
                stone_size=1.5 * (1.05 - difficulty),
                stone_distance=0.05 if difficulty == 0 else 0.1,
                gap_size=1.0 * difficulty,
                pit_depth=1.0 * difficulty)


def gap_terrain(terrain, gap_size, platform_size=1.0):
    """A -1000 (bottomless) square ring of width `gap_size` around the platform."""
    g = int(gap_size / terrain.horizontal_scale)
    p = int(platform_size / terrain.horizontal_scale)
    cx, cy = terrain.length // 2, terrain.width // 2
    x1, y1 = (terrain.length - p) // 2, (terrain.width - p) // 2
    x2, y2 = x1 + g, y1 + g
    terrain.height_field_raw[cx - x2:cx + x2, cy - y2:cy + y2] = -1000
    terrain.height_field_raw[cx - x1:cx + x1, cy - y1:cy + y1] = 0


def pit_terrain(terrain, depth, platform_size=1.0):
    """A square pit of depth `depth` and side `platform_size` at the tile centre."""
    d = int(depth / terrain.vertical_scale)
    half = int(platform_size / terrain.horizontal_scale / 2)
    x1, x2 = terrain.length // 2 - half, terrain.length // 2 + half
    y1, y2 = terrain.width // 2 - half, terrain.width // 2 + half
    terrain.height_field_raw[x1:x2, y1:y2] = -d


class Terrain:
    def __init__(self, cfg, num_robots) -> None:
        self.cfg = cfg
        self.num_robots = num_robots
        self.type = cfg.mesh_type
        if self.type in ("none", "plane"):
            return
        self.env_length, self.env_width = cfg.terrain_length, cfg.terrain_width
        self.proportions = list(np.cumsum(cfg.terrain_proportions))
        cfg.num_sub_terrains = cfg.num_rows * cfg.num_cols
        self.env_origins = np.zeros((cfg.num_rows, cfg.num_cols, 3))
        hs = cfg.horizontal_scale
        self.width_per_env_pixels = int(self.env_width / hs)
        self.length_per_env_pixels = int(self.env_length / hs)
        self.border = int(cfg.border_size / hs)
        self.tot_cols = int(cfg.num_cols * self.width_per_env_pixels) + 2 * self.border
        self.tot_rows = int(cfg.num_rows * self.length_per_env_pixels) + 2 * self.border
        self.height_field_raw = np.zeros((self.tot_rows, self.tot_cols), dtype=np.int16)
        if cfg.curriculum:
            self.curiculum()
        elif cfg.selected:
            self.selected_terrain()
        else:
            self.randomized_terrain()
        self.heightsamples = self.height_field_raw
        if self.type == "trimesh":
            self.vertices, self.triangles = terrain_utils.convert_heightfield_to_trimesh(
                self.height_field_raw, hs, cfg.vertical_scale, cfg.slope_treshold)

    # ------------------------------------------------------------ layouts --
    def _tiles(self):
        for k in range(self.cfg.num_rows * self.cfg.num_cols):
            yield np.unravel_index(k, (self.cfg.num_rows, self.cfg.num_cols))

    def randomized_terrain(self):
        for i, j in self._tiles():
            choice = np.random.uniform(0, 1)
            difficulty = np.random.choice([0.5, 0.75, 0.9])
            self.add_terrain_to_map(self.make_terrain(choice, difficulty), i, j)

    def curiculum(self):  # (sic) the reference's spelling
        for j in range(self.cfg.num_cols):
            for i in range(self.cfg.num_rows):
                self.add_terrain_to_map(self.make_terrain(j / self.cfg.num_cols + 0.001, i / self.cfg.num_rows), i, j)

    def selected_terrain(self):
        kwargs = dict(self.cfg.terrain_kwargs)
        fn = getattr(terrain_utils, kwargs.pop("type").split(".")[-1])
        for i, j in self._tiles():
            tile = self._new_tile()
            fn(tile, **kwargs.get("terrain_kwargs", kwargs))
            self.add_terrain_to_map(tile, i, j)

    def _new_tile(self):
        return terrain_utils.SubTerrain("terrain", width=self.width_per_env_pixels, length=self.width_per_env_pixels,
                                        vertical_scale=self.cfg.vertical_scale,
                                        horizontal_scale=self.cfg.horizontal_scale)

    # ---------------------------------------------------------------- tiles --
    def make_terrain(self, choice, difficulty):
        tile = self._new_tile()
        p = _tile_params(difficulty)
        bounds = self.proportions
        if choice < bounds[0]:  # smooth slope, down for the first half of the band
            slope = -p["slope"] if choice < bounds[0] / 2 else p["slope"]
            terrain_utils.pyramid_sloped_terrain(tile, slope=slope, platform_size=3.0)
        elif choice < bounds[1]:  # rough slope
            terrain_utils.pyramid_sloped_terrain(tile, slope=p["slope"], platform_size=3.0)
            terrain_utils.random_uniform_terrain(tile, min_height=-0.05, max_height=0.05, step=0.005,
                                                 downsampled_scale=0.2)
        elif choice < bounds[3]:  # stairs: down in band 2, up in band 3
            h = -p["step_height"] if choice < bounds[2] else p["step_height"]
            terrain_utils.pyramid_stairs_terrain(tile, step_width=0.31, step_height=h, platform_size=3.0)
        elif choice < bounds[4]:
            terrain_utils.discrete_obstacles_terrain(tile, p["obstacle_height"], 1.0, 2.0, 20, platform_size=3.0)
        elif choice < bounds[5]:
            terrain_utils.stepping_stones_terrain(tile, stone_size=p["stone_size"],
                                                  stone_distance=p["stone_distance"], max_height=0.0,
                                                  platform_size=4.0)
        elif choice < bounds[6]:
            gap_terrain(tile, gap_size=p["gap_size"], platform_size=3.0)
        else:
            pit_terrain(tile, depth=p["pit_depth"], platform_size=4.0)
        return tile

    def add_terrain_to_map(self, terrain, row, col):
        L, W, b = self.length_per_env_pixels, self.width_per_env_pixels, self.border
        x0, y0 = b + row * L, b + col * W
        self.height_field_raw[x0:x0 + L, y0:y0 + W] = terrain.height_field_raw
        hs = terrain.horizontal_scale
        x1, x2 = int((self.env_length / 2.0 - 1) / hs), int((self.env_length / 2.0 + 1) / hs)
        y1, y2 = int((self.env_width / 2.0 - 1) / hs), int((self.env_width / 2.0 + 1) / hs)
        z = np.max(terrain.height_field_raw[x1:x2, y1:y2]) * terrain.vertical_scale
        self.env_origins[row, col] = [(row + 0.5) * self.env_length, (col + 0.5) * self.env_width, z]
