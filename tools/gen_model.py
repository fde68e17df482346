#!/usr/bin/env python3
"""Model compiler: H1-2 12-DoF MJCF/URDF (data files) -> h12_12dof_model.json.

Reads only *data* files of the reference (XML), never imports its code:
  - dynamics constants from the 12-DoF MJCF
    ``packages/biped_assets/biped_assets/models/h12/scene/h12_12dof.xml:66-343``
    (pelvis + 12 leg bodies + 39 joint-less upper-body bodies; defaults :4-7;
    joint ranges :73-134; actuatorfrcrange; keyframe :362-368);
  - foot / knee / torso collision geometry from the URDF the IsaacLab USD was
    converted from ``packages/biped_assets/biped_assets/models/h12/h12_12dof.urdf:100-191``
    (4 sole rods r=0.005 at z=-0.04; knee cylinder r=0.02 l=0.2 at z=-0.2; torso box).

The 39 joint-less bodies (torso_link, arms, hands) are welded to the pelvis in
the MJCF, so they are folded into one composite base inertia: 52 bodies ->
13 moving bodies (1 floating base + 12 revolute leg links).

Run once in the build container (the GPU box never sees /root/reference); the
output JSON is committed and is the single source of model data for the HIP
library, the CPU oracle and the Python host.
"""
from __future__ import annotations

import json
import math
import sys
import xml.etree.ElementTree as ET
from pathlib import Path

import numpy as np

REF = Path("/root/reference/packages/biped_assets/biped_assets/models/h12")
MJCF = REF / "scene" / "h12_12dof.xml"
URDF = REF / "h12_12dof.urdf"
OUT = Path(__file__).resolve().parents[1] / "h1v2-isaac_amd" / "h12env" / "assets" / "h12_12dof_model.json"

JOINT_ORDER = [
    "left_hip_yaw_joint", "left_hip_pitch_joint", "left_hip_roll_joint",
    "left_knee_joint", "left_ankle_pitch_joint", "left_ankle_roll_joint",
    "right_hip_yaw_joint", "right_hip_pitch_joint", "right_hip_roll_joint",
    "right_knee_joint", "right_ankle_pitch_joint", "right_ankle_roll_joint",
]


def vec(s, n=3, default=None):
    if s is None:
        return np.array(default, dtype=np.float64)
    v = np.array([float(x) for x in s.split()], dtype=np.float64)
    assert v.size == n, s
    return v


def quat_to_mat(q):
    w, x, y, z = q / np.linalg.norm(q)
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
        [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
        [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)],
    ])


def inertial_of(body):
    """(mass, com(3), I_com(3x3)) of an MJCF <body> in its own frame."""
    ine = body.find("inertial")
    m = float(ine.get("mass"))
    c = vec(ine.get("pos"))
    R = quat_to_mat(vec(ine.get("quat"), 4, [1, 0, 0, 0]))
    D = np.diag(vec(ine.get("diaginertia")))
    return m, c, R @ D @ R.T


def body_frame(body):
    p = vec(body.get("pos"), 3, [0, 0, 0])
    R = quat_to_mat(vec(body.get("quat"), 4, [1, 0, 0, 0]))
    return p, R


def sym6(I):
    """xx, yy, zz, xy, xz, yz"""
    return [I[0, 0], I[1, 1], I[2, 2], I[0, 1], I[0, 2], I[1, 2]]


def fold_composite(root):
    """Mass, COM and COM-inertia (pelvis frame) of pelvis + every joint-less descendant."""
    items = []  # (m, com_in_pelvis, I_com_in_pelvis)
    m, c, I = inertial_of(root)
    items.append((m, c, I))

    def walk(body, p_par, R_par):
        for ch in body.findall("body"):
            if ch.find("joint") is not None:
                continue  # leg chain: a moving body
            p, R = body_frame(ch)
            p_w = p_par + R_par @ p
            R_w = R_par @ R
            if ch.find("inertial") is not None:
                mi, ci, Ii = inertial_of(ch)
                items.append((mi, p_w + R_w @ ci, R_w @ Ii @ R_w.T))
            walk(ch, p_w, R_w)

    walk(root, np.zeros(3), np.eye(3))
    M = sum(it[0] for it in items)
    com = sum(it[0] * it[1] for it in items) / M
    Itot = np.zeros((3, 3))
    for mi, ci, Ii in items:
        d = ci - com
        Itot += Ii + mi * (np.dot(d, d) * np.eye(3) - np.outer(d, d))
    return M, com, Itot, len(items)


def main():
    mj = ET.parse(MJCF).getroot()
    dflt_joint = mj.find("default/joint")
    damping = float(dflt_joint.get("damping"))
    armature = float(dflt_joint.get("armature"))
    frictionloss = float(dflt_joint.get("frictionloss"))
    pelvis = mj.find("worldbody/body[@name='pelvis']")

    base_m, base_c, base_I, n_folded = fold_composite(pelvis)

    links = {}

    def walk_legs(body, parent_name):
        for ch in body.findall("body"):
            j = ch.find("joint")
            if j is None:
                continue
            p, R = body_frame(ch)
            assert np.allclose(R, np.eye(3)), "leg bodies carry no rotation in the MJCF"
            m, c, I = inertial_of(ch)
            axis = vec(j.get("axis"))
            ax = int(np.argmax(np.abs(axis)))
            assert np.isclose(axis[ax], 1.0) and np.isclose(np.abs(axis).sum(), 1.0)
            rng = vec(j.get("range"), 2)
            frc = vec(j.get("actuatorfrcrange"), 2)
            links[j.get("name")] = dict(
                body=ch.get("name"), parent=parent_name, pos=p.tolist(), axis=ax,
                mass=m, com=c.tolist(), inertia=sym6(I), range=rng.tolist(), frcrange=float(frc[1]),
            )
            walk_legs(ch, j.get("name"))

    walk_legs(pelvis, None)
    assert list(links) == JOINT_ORDER, list(links)

    key = mj.find("keyframe/key")
    qpos0 = vec(key.get("qpos"), 19)

    # ---- URDF collision geometry (the USD used by IsaacLab was converted from it)
    ur = ET.parse(URDF).getroot()

    def coll(link):
        out = []
        for c in ur.findall(f"link[@name='{link}']/collision"):
            o = c.find("origin")
            g = c.find("geometry")[0]
            out.append((vec(o.get("xyz")), vec(o.get("rpy")), g.tag, g.attrib))
        return out

    rods = coll("left_ankle_roll_link")
    r_foot = float(rods[0][3]["radius"])
    # sole corner spheres: rod end points at the rod axis (z=-0.04), radius = rod radius
    pts = []
    for xyz, rpy, tag, a in rods:
        L = float(a["length"])
        if abs(rpy[0]) > 1:  # rotated about x: cylinder axis along y
            for s in (-1, 1):
                pts.append([xyz[0], xyz[1] + s * L / 2, xyz[2]])
    # transverse heel rod (x=-0.08, |y|<=0.038) and toe rod (x=0.17, |y|<=0.021)
    pts = sorted(pts, key=lambda p: (p[0], p[1]))
    assert len(pts) == 4
    # every sole rod as a segment (self-collision capsules): rotated about x -> axis y, about y -> axis x
    rod_segs = []
    for xyz, rpy, tag, a in rods:
        L = float(a["length"])
        ax = np.array([0.0, 1.0, 0.0]) if abs(rpy[0]) > 1 else np.array([1.0, 0.0, 0.0])
        rod_segs.append([(xyz - ax * L / 2).tolist(), (xyz + ax * L / 2).tolist()])
    knee = coll("left_knee_link")[0]
    knee_r = float(knee[3]["radius"])
    knee_L = float(knee[3]["length"])
    torso = coll("torso_link")[0]
    box = vec(torso[3]["size"])

    leg_mass = sum(l["mass"] for l in links.values())
    model = {
        "version": 1,
        "source": {"mjcf": "packages/biped_assets/biped_assets/models/h12/scene/h12_12dof.xml",
                   "urdf": "packages/biped_assets/biped_assets/models/h12/h12_12dof.urdf"},
        "joint_names": JOINT_ORDER,
        "body_names": ["pelvis"] + [links[j]["body"] for j in JOINT_ORDER],
        "base": {"mass": base_m, "com": base_c.tolist(), "inertia": sym6(base_I), "n_folded_bodies": n_folded},
        "total_mass": base_m + leg_mass,
        "joints": [
            dict(name=j, parent=(-1 if links[j]["parent"] is None else JOINT_ORDER.index(links[j]["parent"])),
                 **{k: v for k, v in links[j].items() if k != "parent"})
            for j in JOINT_ORDER
        ],
        "joint_defaults": {"damping": damping, "armature": armature, "frictionloss": frictionloss},
        "keyframe_qpos": qpos0.tolist(),
        "foot": {"body": ["left_ankle_roll_link", "right_ankle_roll_link"], "points": pts, "radius": r_foot,
                 "rods": rod_segs},
        "knee": {"body": ["left_knee_link", "right_knee_link"],
                 "p0": (knee[0] + np.array([0, 0, knee_L / 2])).tolist(),
                 "p1": (knee[0] - np.array([0, 0, knee_L / 2])).tolist(), "radius": knee_r},
        "torso_box": {"center": torso[0].tolist(), "half": (box / 2).tolist()},
        # torso_link is welded to the pelvis at the pelvis origin (no pos attribute, h12_12dof.xml:143)
        "torso_link": {"pos": [0.0, 0.0, 0.0], "com": inertial_of(pelvis.find(".//body[@name='torso_link']"))[1].tolist()},
        "gravity": 9.81,
        # the pelvis rigid body's own COM (pelvis frame): IsaacLab's root_com_* quantities (root_lin_vel_w / _b) are
        # those of the articulation's root body, and the USD keeps torso_link as a separate rigid body (the tasks
        # address it by name, cat_env_cfg.py:246,258)
        "root_com": inertial_of(pelvis)[1].tolist(),
    }
    OUT.parent.mkdir(parents=True, exist_ok=True)
    OUT.write_text(json.dumps(model, indent=1))
    print(f"wrote {OUT}: base {base_m:.4f} kg ({n_folded} bodies folded), legs {leg_mass:.4f} kg, "
          f"total {model['total_mass']:.4f} kg")


if __name__ == "__main__":
    sys.exit(main())
