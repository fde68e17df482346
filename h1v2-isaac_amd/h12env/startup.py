"""Host-side scene construction of the terrain tasks and the mode="startup" events, as workspace field
values (shared by the env and the parity tests so both sides start from the same state).

* TerrainImporter (velocity_env_cfg.py:40-56, curriculum origins): env i gets type floor(i / (N / cols))
  and a random initial level <= max_init_terrain_level; its origin is that sub-terrain's origin.  The
  pre-reset base position is set to the origin so the curriculum pass of the first reset is neutral.
* randomize_rigid_body_material (num_buckets buckets of (static, dynamic) friction, one bucket per env
  and sole; multiply-combined with the ground's material) and randomize_rigid_body_mass (added torso
  mass, "add" operation) -- velocity_env_cfg.py:146-166, cat_env_cfg.py:231-249.
Random streams: numpy / torch CPU generators seeded from cfg.seed and the shard's env offset.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np
import torch

from . import terrain as T


@dataclass
class StartupState:
    terrain: T.Terrain | None = None
    fields: dict = field(default_factory=dict)     # field name -> (count, n) float32
    terrain_cell: np.ndarray | None = None         # (n,) int32 level | type << 16


def startup_state(cfg, n: int, env_offset: int = 0) -> StartupState:
    st = StartupState()
    seed = int(cfg.seed or 0)
    tc = cfg.scene.terrain
    if tc.terrain_type == "generator":
        st.terrain = T.generate(tc.terrain_generator, seed)
        lv, ty = T.initial_cells(n, tc.terrain_generator, tc.max_init_terrain_level, seed + env_offset)
        st.terrain_cell = (lv | (ty << 16)).astype(np.int32)
        org = st.terrain.origins[lv, ty]                     # (n, 3)
        st.fields["ORIGIN"] = org.T.astype(np.float32).copy()
        pos = np.zeros((3, n), dtype=np.float32)
        pos[0:2] = org[:, 0:2].T
        pos[2] = org[:, 2] + cfg.robot.init_pos[2]
        st.fields["POS"] = pos
    ev = cfg.events
    g = torch.Generator(device="cpu").manual_seed(seed * 1_000_003 + 17 + env_offset)
    if ev.physics_material is not None:
        pm = ev.physics_material
        lo = torch.tensor([pm.static_friction_range[0], pm.dynamic_friction_range[0]])
        hi = torch.tensor([pm.static_friction_range[1], pm.dynamic_friction_range[1]])
        buckets = lo + (hi - lo) * torch.rand(pm.num_buckets, 2, generator=g)
        ids = torch.randint(0, pm.num_buckets, (n, 2), generator=g)
        ground = torch.tensor([tc.static_friction, tc.dynamic_friction])
        mu = (buckets[ids] * ground).reshape(n, 4)            # [mu_s L, mu_d L, mu_s R, mu_d R]
        st.fields["MU"] = mu.T.numpy().astype(np.float32).copy()
    if ev.add_base_mass is not None:
        am = ev.add_base_mass
        if am.operation != "add":
            raise ValueError("only the 'add' mass operation is implemented")
        a, b = am.mass_distribution_params
        st.fields["DMASS"] = (a + (b - a) * torch.rand(1, n, generator=g)).numpy().astype(np.float32)
    return st


def apply_to_arrays(st: StartupState, F: np.ndarray, I: np.ndarray) -> None:
    """Write a StartupState into host workspace arrays (F: (NF_FLOAT, n), I: (NF_INT, n))."""
    from ._abi import F as FIELDS
    from ._abi import I as IFIELDS

    for name, val in st.fields.items():
        o, c = FIELDS[name]
        F[o:o + c] = val
    if st.terrain_cell is not None:
        I[IFIELDS["TERRAIN"][0]] = st.terrain_cell
