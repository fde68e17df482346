#!/usr/bin/env python3
"""Quantify the model-level deviations of DESIGN.md §9 on the CPU oracle (build container; reads the reference's
MJCF for the pelvis body's own inertial): a random-action Flat rollout, then per env-step

  1. root_lin_vel: the pelvis rigid body's own COM velocity (what IsaacLab reports as root_lin_vel_w, the USD
     keeping torso_link as a separate body; the build's definition since round 2) vs the composite base COM
     (pelvis + the 40 welded upper-body bodies; the round-1 definition): |dv_xy| and the change of the
     track_lin_vel_xy_exp reward term between the two -- why the definition matters;
  2. joint limits: a stiff implicit limit spring (1e6 N m/rad on the predicted end-of-step position) plus the
     0.01 rad hard-limit projection instead of PhysX's hard limits -- how often and how far a joint sits beyond its
     range (all joint-env-steps, and the ones beyond);
  3. contact stiffness: sole-sphere penetration depth of the penalty springs (PhysX: rigid, ~0).

    python tools/deviations.py [--envs 1024] [--steps 300] [--out profiles/r3_deviations.json]
"""
from __future__ import annotations

import argparse
import json
import sys
import xml.etree.ElementTree as ET
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "h1v2-isaac_amd"), str(ROOT / "oracle"), str(ROOT / "tools")]
MJCF = Path("/root/reference/packages/biped_assets/biped_assets/models/h12/scene/h12_12dof.xml")


def quat_R(q):
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--out", type=str, default=None)
    ap.add_argument("--contact-k", type=float, default=None, help="experiment: ground contact stiffness override")
    a = ap.parse_args()
    import oracle as O
    from gen_model import inertial_of
    from h12env import H12FlatEnvCfg
    from h12env._abi import F
    from h12env.model import build_model

    pelvis = ET.parse(MJCF).getroot().find(".//worldbody/body[@name='pelvis']")
    _, c_pelvis, _ = inertial_of(pelvis)
    model = build_model()
    c_comp = np.asarray(model.base_com, dtype=np.float64)  # composite (model.root_com: the pelvis body)
    cfg = H12FlatEnvCfg()
    if a.contact_k:
        cfg.sim.contact_k = a.contact_k
    n = a.envs
    env = O.OracleEnv(model, cfg.to_c(), n)
    env.reset()
    rng = np.random.default_rng(0)
    ql, qu = np.asarray(model.q_lower, np.float64), np.asarray(model.q_upper, np.float64)
    dv, dr, excess, depth = [], [], [], []
    sl = lambda k: slice(F[k][0], F[k][0] + F[k][1])  # noqa: E731
    foot = np.array([[model.foot_pts[k][j] for j in range(3)] for k in range(4)], np.float64)
    for t in range(a.steps):
        env.step(rng.normal(size=(n, 12)).astype(np.float32), t + 1, n_threads=8)
        if t < 50:
            continue  # past the initial drop
        Fs = env.F.astype(np.float64)
        q, vl, w, cmd = Fs[sl("QUAT")].T, Fs[sl("VLIN")].T, Fs[sl("WANG")].T, Fs[sl("CMD")].T
        for i in range(n):
            R = quat_R(q[i])
            ww = R @ w[i]
            hx, hy = R[0, 0], R[1, 0]
            h = np.hypot(hx, hy)
            cy, sy = hx / h, hy / h

            def yaw_xy(v):
                return np.array([cy * v[0] + sy * v[1], -sy * v[0] + cy * v[1]])

            v_comp = yaw_xy(vl[i] + np.cross(ww, R @ c_comp))
            v_pel = yaw_xy(vl[i] + np.cross(ww, R @ c_pelvis))
            dv.append(np.hypot(*(v_comp - v_pel)))
            e_c, e_p = cmd[i, :2] - v_comp, cmd[i, :2] - v_pel
            dr.append(abs(np.exp(-(e_c @ e_c) / 0.25) - np.exp(-(e_p @ e_p) / 0.25)))
        jq = Fs[sl("Q")].T
        excess.append(np.maximum(np.maximum(ql - jq, jq - qu), 0.0))
        if t % 10 == 0 and foot is not None:  # sole-sphere penetration of the spheres in contact
            for i in range(0, n, 8):
                st = np.concatenate([Fs[sl("POS"), i], q[i], vl[i], w[i], Fs[sl("Q"), i], Fs[sl("QD"), i]])
                Rb, pb = O.body_poses(model, st)
                for f, b in ((0, 6), (1, 12)):
                    for k in range(4):
                        pl = foot[k].copy()
                        if f == 1:
                            pl[1] = -pl[1]
                        d = model.foot_radius - (Rb[b] @ pl + pb[b])[2]
                        if d > 0:
                            depth.append(d)
    dv, dr = np.asarray(dv), np.asarray(dr)
    excess = np.concatenate(excess)
    out = {
        "envs": n, "steps": a.steps, "window": "steps 51..%d, N(0,1) random actions (the bench workload)" % a.steps,
        "pelvis_com_minus_composite_com_m": (c_pelvis - c_comp).round(4).tolist(),
        "root_lin_vel_xy_yaw_frame_diff_m_s": {"median": float(np.median(dv)), "p95": float(np.percentile(dv, 95))},
        "track_lin_vel_xy_exp_abs_change": {"median": float(np.median(dr)), "p95": float(np.percentile(dr, 95))},
        "joint_env_steps_beyond_limit_fraction": float((excess > 0).mean()),
        "joint_limit_excess_rad": {"p99": float(np.percentile(excess, 99)), "max": float(excess.max())},
        "joint_limit_excess_rad_beyond_only": {"median": float(np.median(excess[excess > 0])) if (excess > 0).any() else 0.0,
                                               "p99": float(np.percentile(excess[excess > 0], 99)) if (excess > 0).any() else 0.0},
        "sim": {"contact_k": cfg.sim.contact_k, "limit_k": cfg.sim.limit_k, "limit_projection": cfg.sim.limit_projection,
                "max_depenetration_velocity": cfg.sim.max_depenetration_velocity},
    }
    if depth:
        d = np.asarray(depth)
        out["sole_penetration_mm_in_contact"] = {"median": float(1e3 * np.median(d)), "p95": float(1e3 * np.percentile(d, 95))}
    print(json.dumps(out, indent=1))
    if a.out:
        Path(a.out).write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main()
