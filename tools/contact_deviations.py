#!/usr/bin/env python3
"""Quantify the two contact deviations VERDICT round 3 listed on the CPU oracle, build container:

  1. Leg self-contact against the torso box (A/robots/h12.py:32 enables self-collision on every body; the URDF's
     colliders are the knee cylinders, the four sole rods per foot and the torso box -- the arm links carry visual
     meshes only, h12_12dof.urdf:403-733, so there is nothing to collide with on the welded arms).  Over a
     random-action rollout (the bench workload), per env-step, the signed distance from every leg collider (the
     capsule axis sampled at 21 points, minus the radius) to the torso box in the pelvis frame: how often a leg
     collider reaches the box (distance <= 0) and how close the legs come.

  2. Per-shape friction buckets for the knee and torso GROUND contacts under material randomisation (CaT / Rsl / C5:
     64 buckets of U(0.1, 1.25) per collision shape, C12/cat_env_cfg.py:231-239).  The build gives the soles their
     env's randomised coefficients and keeps the config's coefficients for knee and torso.  Both bodies are in every
     task's illegal-contact list (rough_env_cfg.py:95-100, rsl_env_cfg.py:418-430, cat_env_cfg.py:436-446), so their
     friction can act only inside the step in which the contact starts, before the reset.  Measured teacher-forced:
     each step the same pre-step state and actions through two oracles whose knee / torso ground friction sits at the
     two ends of the bucket range (0.1 and 1.25); the env-steps whose outputs differ, and by how much.

    python tools/contact_deviations.py [--envs 1024] [--steps 300] [--out profiles/r4_contact_deviations.json]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "h1v2-isaac_amd"), str(ROOT / "oracle")]


def box_dist(pts, c, h):
    """Signed distance of points (k, 3) to an axis-aligned box (center c, half extents h)."""
    d = np.abs(pts - c) - h
    out = np.linalg.norm(np.maximum(d, 0.0), axis=-1)
    inside = np.minimum(np.max(d, axis=-1), 0.0)
    return out + inside


def leg_colliders(m):
    """(body, p0, p1, radius) of every leg collider, in the link frame (left leg; the right one is its mirror and the
    colliders are symmetric about the link's xz-plane)."""
    out = []
    for leg in range(2):
        knee, foot = 4 + 6 * leg, 6 + 6 * leg
        out.append((knee, np.array(m.knee_p0[:]), np.array(m.knee_p1[:]), m.knee_radius))
        for r in range(4):
            out.append((foot, np.array(m.foot_rods[r][0][:]), np.array(m.foot_rods[r][1][:]), 0.005))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--out", type=str, default=None)
    a = ap.parse_args()
    import oracle as O
    from h12env import H12FlatEnvCfg
    from h12env._abi import F
    from h12env.model import build_model

    m = build_model()
    n = a.envs
    cfg = H12FlatEnvCfg()
    cfg.scene.num_envs = n
    c = cfg.to_c()
    env = O.OracleEnv(m, c, n)
    env.reset()
    rng = np.random.default_rng(0)
    colliders = leg_colliders(m)
    tc, th = np.array(m.torso_center[:]), np.array(m.torso_half[:])
    s_ = np.linspace(0.0, 1.0, 21)[:, None]
    dmin_all, hits, env_steps = [], 0, 0
    fields = [F[k] for k in ("POS", "QUAT", "VLIN", "WANG", "Q", "QD")]
    for t in range(a.steps):
        env.step(rng.normal(size=(n, 12)).astype(np.float32), t + 1)
        if t < 50:
            continue
        X = np.concatenate([env.F[o:o + k] for o, k in fields]).T.astype(np.float64)
        for i in range(n):
            R, p = O.body_poses(m, X[i])
            Rp, pp = R[0], p[0]
            dm = np.inf
            for body, p0, p1, rad in colliders:
                pts = (p0[None] + s_ * (p1 - p0)[None]) @ R[body].T + p[body]   # world
                loc = (pts - pp) @ Rp                                           # pelvis frame
                dm = min(dm, float(box_dist(loc, tc, th).min()) - rad)
            dmin_all.append(dm)
            hits += dm <= 0.0
            env_steps += 1
    d = np.array(dmin_all)
    res = {"envs": n, "steps": a.steps, "window": f"steps 51..{a.steps}, N(0,1) random actions (the bench workload)",
           "leg_torso_box": {
               "colliders": "knee cylinders (r 0.02) and 4 sole rods per foot (r 0.005) vs the torso box "
                            "(h12_12dof.urdf:116-190, 387-392); the arm links have no colliders",
               "env_steps": env_steps, "env_steps_in_contact": int(hits),
               "fraction_in_contact": hits / max(1, env_steps),
               "min_distance_m": {"min": float(d.min()), "p0.1": float(np.quantile(d, 0.001)),
                                  "p1": float(np.quantile(d, 0.01)), "median": float(np.median(d))}}}

    # 2. knee / torso ground friction at the two ends of the bucket range, teacher-forced, on the Rsl task (flat
    # plane, per-env sole materials drawn at startup, pushes; its illegal contacts include knees and torso)
    from h12env.cfg import H12RslEnvCfg
    from h12env.startup import apply_to_arrays, startup_state

    cfg2 = H12RslEnvCfg()
    cfg2.scene.num_envs = n
    lo, hi = cfg2.to_c(), cfg2.to_c()
    assert lo.per_env_friction and lo.illegal_contact_knees and lo.illegal_contact_torso
    lo.mu_static = lo.mu_dynamic = 0.1
    hi.mu_static = hi.mu_dynamic = 1.25
    # the soles keep each env's own randomised coefficients (H12_F_MU) in both
    A, B = O.OracleEnv(m, lo, n), O.OracleEnv(m, hi, n)
    apply_to_arrays(startup_state(cfg2, n), A.F, A.I)
    A.reset()
    rng = np.random.default_rng(1)
    diff_steps = diff_flags = knee_torso_steps = 0
    dphys, drew = [], []
    o_q = F["Q"][0]
    for t in range(a.steps):
        act = rng.normal(size=(n, 12)).astype(np.float32)
        B.F[:], B.I[:], B.obs[:] = A.F, A.I, A.obs
        _, ra, ta, tra, ia = A.step(act, t + 1)
        _, rb, tb, trb, ib = B.step(act, t + 1)
        if t < 50:
            continue
        knee_torso_steps += int(np.sum(ta))
        df = np.abs(A.F[:o_q + 24] - B.F[:o_q + 24]).max(axis=0)
        dr = np.abs(ra - rb)
        diff_flags += int(np.sum((ta != tb) | (tra != trb)))
        moved = (df > 1e-9) | (dr > 1e-9)
        diff_steps += int(np.sum(moved))
        dphys.extend(df[moved & ~ta].tolist())
        drew.extend(dr[moved].tolist())
    steps_w = (a.steps - 50) * n
    res["knee_torso_ground_friction"] = {
        "method": "teacher-forced: the same pre-step state and actions through two oracles with knee / torso ground "
                  "friction 0.1 vs 1.25 (the ends of the U(0.1, 1.25) bucket range), Rsl task (per-env sole materials)",
        "env_steps": steps_w, "terminating_env_steps": knee_torso_steps,
        "env_steps_with_any_output_difference": diff_steps, "termination_flag_differences": diff_flags,
        "max_abs_state_difference_non_terminating": float(max(dphys)) if dphys else 0.0,
        "reward_abs_difference": {"max": float(max(drew)) if drew else 0.0,
                                  "sum_over_window": float(np.sum(drew)) if drew else 0.0}}
    print(json.dumps(res, indent=1))
    if a.out:
        Path(a.out).write_text(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    main()
