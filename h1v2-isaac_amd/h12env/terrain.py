"""Heightfield terrain of the rough task (replaces IsaacLab's TerrainGenerator + TerrainImporter).

Restates the published algorithm of isaaclab.terrains (IsaacLab 2.1, not installed here -- parity of the
samples against it is unpinned, the layout and statistics follow it):

* ROUGH_TERRAINS_CFG (biped_tasks/utils/mdp/terrains.py:11-28): num_rows x num_cols sub-terrains of
  8 x 8 m, one type (HfRandomUniform, noise 0-2 cm in 5 mm steps), 20 m flat border, 0.1 m pixels,
  5 mm vertical scale.
* height_field_to_mesh: each sub-terrain is an (8/0.1 + 1)^2 pixel grid with a flat border of
  int(0.25/0.1) + 1 = 3 pixels; the inner pixels take random heights from {0, ..., 4} x 5 mm (the
  RectBivariateSpline up-sampling of random_uniform_terrain is the identity when the down-sampled scale
  equals the horizontal scale).  Sub-terrain origin: its centre at the maximum height of the central
  2 x 2 m.
* TerrainGenerator centres the whole grid on the world origin; TerrainImporter assigns env i the type
  floor(i / (N / num_cols)) and a random initial level in [0, max_init_terrain_level].

All sub-terrains are stitched into ONE heightfield (shared 0-height edges), which is what the kernels
sample (h12env_set_terrain).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .cfg import TerrainGeneratorCfg


@dataclass
class Terrain:
    heights: np.ndarray   # (nx, ny) float32 metres, heights[ix, iy] at (x0 + ix*hs, y0 + iy*hs)
    hscale: float
    x0: float
    y0: float
    origins: np.ndarray   # (rows, cols, 3) float32 sub-terrain origins (world)

    @property
    def shape(self):
        return self.heights.shape


def generate(cfg: TerrainGeneratorCfg, seed: int) -> Terrain:
    rng = np.random.default_rng(seed)
    hs, vs = cfg.horizontal_scale, cfg.vertical_scale
    sub_px = int(round(cfg.size[0] / hs))                 # 80 pixels per sub-terrain edge
    if int(round(cfg.size[1] / hs)) != sub_px:
        raise ValueError("square sub-terrains only")
    border_px = int(round(cfg.border_width / hs))         # 200
    inner_border = int(cfg.sub_border_width / hs) + 1     # 3 (height_field_to_mesh)
    nx = cfg.num_rows * sub_px + 1 + 2 * border_px
    ny = cfg.num_cols * sub_px + 1 + 2 * border_px
    hmin = int(cfg.noise_range[0] / vs)
    hmax = int(cfg.noise_range[1] / vs)
    hstep = max(1, int(cfg.noise_step / vs))
    levels = np.arange(hmin, hmax + hstep, hstep)
    H = np.zeros((nx, ny), dtype=np.int16)
    origins = np.zeros((cfg.num_rows, cfg.num_cols, 3), dtype=np.float32)
    x_grid0 = -0.5 * cfg.num_rows * cfg.size[0]
    y_grid0 = -0.5 * cfg.num_cols * cfg.size[1]
    c1 = int((cfg.size[0] * 0.5 - 1) / hs)
    c2 = int((cfg.size[0] * 0.5 + 1) / hs)
    for r in range(cfg.num_rows):
        for c in range(cfg.num_cols):
            sub = np.zeros((sub_px + 1, sub_px + 1), dtype=np.int16)
            n_in = sub_px + 1 - 2 * inner_border
            sub[inner_border:-inner_border, inner_border:-inner_border] = rng.choice(levels, size=(n_in, n_in))
            ix0 = border_px + r * sub_px
            iy0 = border_px + c * sub_px
            H[ix0:ix0 + sub_px + 1, iy0:iy0 + sub_px + 1] = np.maximum(H[ix0:ix0 + sub_px + 1, iy0:iy0 + sub_px + 1],
                                                                        sub)
            oz = float(sub[c1:c2, c1:c2].max()) * vs
            origins[r, c] = (x_grid0 + (r + 0.5) * cfg.size[0], y_grid0 + (c + 0.5) * cfg.size[1], oz)
    heights = (H.astype(np.float64) * vs).astype(np.float32)
    return Terrain(heights, hs, x_grid0 - border_px * hs, y_grid0 - border_px * hs, origins)


def initial_cells(num_envs: int, cfg: TerrainGeneratorCfg, max_init_level: int | None, seed: int):
    """TerrainImporter._compute_env_origins_curriculum: (levels, types) per env."""
    rng = np.random.default_rng(seed + 7919)
    max_lvl = cfg.num_rows - 1 if max_init_level is None else min(max_init_level, cfg.num_rows - 1)
    levels = rng.integers(0, max_lvl + 1, size=num_envs)
    types = np.floor(np.arange(num_envs) / (num_envs / cfg.num_cols)).astype(np.int64)
    return levels.astype(np.int32), np.minimum(types, cfg.num_cols - 1).astype(np.int32)


def ground_height(t: Terrain, x: np.ndarray, y: np.ndarray) -> np.ndarray:
    """Vectorised twin of the kernels' ground() (host-side checks and tools)."""
    u = np.clip((np.asarray(x) - t.x0) / t.hscale, 0, t.shape[0] - 1 - 1e-3)
    v = np.clip((np.asarray(y) - t.y0) / t.hscale, 0, t.shape[1] - 1 - 1e-3)
    ix, iy = u.astype(np.int64), v.astype(np.int64)
    fu, fv = u - ix, v - iy
    h = t.heights.astype(np.float64)
    h00, h01, h10, h11 = h[ix, iy], h[ix, iy + 1], h[ix + 1, iy], h[ix + 1, iy + 1]
    upper = fv >= fu
    a = np.where(upper, h11 - h01, h10 - h00)
    b = np.where(upper, h01 - h00, h11 - h10)
    return h00 + fu * a + fv * b
