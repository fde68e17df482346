"""H1-2 12-DoF model constants (from the committed model JSON) -> h12env_model struct."""
from __future__ import annotations

import json
from functools import lru_cache
from pathlib import Path

from ._abi import NJ, H12Model

MODEL_JSON = Path(__file__).resolve().parent / "assets" / "h12_12dof_model.json"

# IsaacLab init_state joint_pos (packages/biped_assets/biped_assets/robots/h12.py:39-53); equal to the MJCF keyframe.
DEFAULT_JOINT_POS = [0.0, -0.16, 0.0, 0.36, -0.2, 0.0, 0.0, -0.16, 0.0, 0.36, -0.2, 0.0]
ROOT_HEIGHT = 1.05  # h12.py:38


@lru_cache(maxsize=None)
def model_dict() -> dict:
    return json.loads(MODEL_JSON.read_text())


def joint_names() -> list[str]:
    return list(model_dict()["joint_names"])


def body_names() -> list[str]:
    return list(model_dict()["body_names"])


def build_model() -> H12Model:
    d = model_dict()
    m = H12Model()
    m.version = int(d["version"])
    for j, jd in enumerate(d["joints"]):
        m.parent[j] = int(jd["parent"])
        m.axis[j] = int(jd["axis"])
        for a in range(3):
            m.joint_pos[j][a] = jd["pos"][a]
            m.link_com[j][a] = jd["com"][a]
        m.link_mass[j] = jd["mass"]
        for a in range(6):
            m.link_inertia[j][a] = jd["inertia"][a]
        m.q_lower[j], m.q_upper[j] = jd["range"]
        m.mj_frc_limit[j] = jd["frcrange"]
        m.armature[j] = d["joint_defaults"]["armature"]
        m.damping[j] = d["joint_defaults"]["damping"]
        m.frictionloss[j] = d["joint_defaults"]["frictionloss"]
        m.q_default[j] = DEFAULT_JOINT_POS[j]
    for a in range(3):
        m.root_com[a] = d["root_com"][a]
    m.base_mass = d["base"]["mass"]
    for a in range(3):
        m.base_com[a] = d["base"]["com"][a]
    for a in range(6):
        m.base_inertia[a] = d["base"]["inertia"][a]
    m.root_height = ROOT_HEIGHT
    for p, pt in enumerate(d["foot"]["points"]):
        for a in range(3):
            m.foot_pts[p][a] = pt[a]
    m.foot_radius = d["foot"]["radius"]
    for a in range(3):
        m.knee_p0[a] = d["knee"]["p0"][a]
        m.knee_p1[a] = d["knee"]["p1"][a]
        m.torso_center[a] = d["torso_box"]["center"][a]
        m.torso_half[a] = d["torso_box"]["half"][a]
        m.torso_com[a] = d["torso_link"]["com"][a]
    m.knee_radius = d["knee"]["radius"]
    for r, seg in enumerate(d["foot"]["rods"]):
        for e in range(2):
            for a in range(3):
                m.foot_rods[r][e][a] = seg[e][a]
    m.gravity = d["gravity"]
    assert len(d["joints"]) == NJ
    return m
