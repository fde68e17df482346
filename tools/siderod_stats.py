#!/usr/bin/env python3
"""Quantify the foot's side-rod ground contacts the build leaves out (missing #2).

The URDF foot (h12_12dof.urdf:168-191) has four rods of radius 5 mm: a heel rod at x = -0.08 (|y| <= 0.038), a toe
rod at x = 0.17 (|y| <= 0.021) and two side rods along x from -0.078 to 0.132 at y = +-0.038.  The build's ground
contact uses 4 spheres at the transverse rods' ends (tools/gen_model.py; H12_NFOOT_PTS): the side rods' REAR ends sit
2 mm from the heel spheres, but their FRONT ends (0.132, +-0.038) are not colliders, so at x = 0.132 the support
polygon is 14.4 mm narrower per side (|y| 0.0236 instead of 0.038).  A side rod is a segment: its lowest point is one
of its ends, so a front end below the ground is exactly "the side rod touches where the model does not".

On the CPU oracle, the bench workload (N(0,1) random actions, Flat task, envs x steps, window after 50 steps), per
env-step and foot, from the oracle's body poses: the depth (radius - height) of the 4 modelled sole spheres and of the
2 side-rod front ends.  Reported: how often a front end penetrates, how often it penetrates while NO modelled sphere
does (PhysX would report a foot contact the build misses: the ContactSensor / air-time / feet_slide path), how often
it is the foot's deepest point, its depth distribution, and the foot's horizontal speed in those env-steps (the
feet_slide term's |v_xy| for a contact the build misses, V/mdp/rewards.py feet_slide).

    python tools/siderod_stats.py [--envs 1024] [--steps 300] [--out profiles/r5/siderod_contacts.json]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "h1v2-isaac_amd"), str(ROOT / "oracle")]


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
    env = O.OracleEnv(m, cfg.to_c(), n)
    env.reset()
    rng = np.random.default_rng(0)
    r = float(m.foot_radius)
    sph = np.array([m.foot_pts[q][:] for q in range(4)], dtype=np.float64)           # (4, 3) foot frame
    rods = np.array(m.foot_rods, dtype=np.float64).reshape(4, 2, 3)
    front = np.array([rods[2][1], rods[3][1]])                                           # side rods' front ends
    assert np.allclose(front[:, 0], 0.132, atol=1e-6) and np.allclose(np.abs(front[:, 1]), 0.038, atol=1e-6)
    fields = [F[k] for k in ("POS", "QUAT", "VLIN", "WANG", "Q", "QD")]
    stats = dict(foot_steps=0, sphere_contact=0, front_pen=0, front_only=0, front_deepest=0, first_contacts=0,
                 first_contacts_preceded_by_front_only=0)
    dfront, vfront_only, dsph_when_front = [], [], []
    slide_build = 0.0  # sum over modelled-contact foot-steps of the foot origin's horizontal speed
    prev = prev_foot = None
    prev_state = None  # per env and foot: 0 no contact, 1 front end only, 2 modelled contact
    for t in range(a.steps):
        env.step(rng.normal(size=(n, 12)).astype(np.float32), t + 1)
        X = np.concatenate([env.F[o:o + k] for o, k in fields]).T.astype(np.float64)
        poses = [O.body_poses(m, X[i]) for i in range(n)]
        cur = np.array([[(R[b] @ front.T).T + p[b] for b in (6, 12)] for R, p in poses])  # (n, 2, 2, 3)
        foot = np.array([[p[b] for b in (6, 12)] for R, p in poses])                      # (n, 2, 3)
        state = np.zeros((n, 2), np.int8)
        if t >= 50:
            for i, (R, p) in enumerate(poses):
                for f, b in enumerate((6, 12)):
                    zs = (R[b] @ sph.T).T[:, 2] + p[b][2]
                    zf = cur[i, f, :, 2]
                    ds, df = r - zs, r - zf
                    stats["foot_steps"] += 1
                    sc = bool((ds > 0).any())
                    stats["sphere_contact"] += sc
                    state[i, f] = 2 if sc else (1 if (df > 0).any() else 0)
                    if sc and prev_foot is not None:
                        slide_build += float(np.linalg.norm(foot[i, f, :2] - prev_foot[i, f, :2]) / 0.02)
                    if sc and prev_state is not None and prev_state[i, f] != 2:
                        stats["first_contacts"] += 1
                        stats["first_contacts_preceded_by_front_only"] += int(prev_state[i, f] == 1)
                    if (df > 0).any():
                        stats["front_pen"] += 1
                        dfront.append(float(df.max()))
                        dsph_when_front.append(float(ds.max()))
                        if not sc:
                            stats["front_only"] += 1
                            if prev is not None:  # horizontal speed of the touching front end over the env step
                                k = int(np.argmax(df))
                                vfront_only.append(float(np.linalg.norm(cur[i, f, k, :2] - prev[i, f, k, :2]) / 0.02))
                        if df.max() > ds.max():
                            stats["front_deepest"] += 1
        prev, prev_foot = cur, foot
        prev_state = state if t >= 50 else None
    fs = max(1, stats["foot_steps"])
    env_steps = fs / 2
    q = lambda x, p: float(np.quantile(np.array(x), p)) if x else None  # noqa: E731
    res = {"envs": n, "steps": a.steps, "window": f"env steps 51..{a.steps} (sampled once per env step), N(0,1) random "
                                                  "actions, Flat task (the bench workload), CPU oracle",
           "geometry": {"side_rod_front_ends_foot_frame": front.tolist(), "radius_m": r,
                        "support_width_lost_per_side_at_x0.132_m": 0.038 - (0.038 - (0.038 - 0.021) * (0.132 + 0.08) / 0.25)},
           "counts": stats,
           "fractions": {"front_end_penetrates": stats["front_pen"] / fs,
                         "front_end_only_contact (a foot contact the build misses)": stats["front_only"] / fs,
                         "front_end_is_the_deepest_point": stats["front_deepest"] / fs,
                         "sphere_contact (modelled)": stats["sphere_contact"] / fs},
           "front_end_depth_m": {"p50": q(dfront, 0.5), "p95": q(dfront, 0.95), "max": max(dfront) if dfront else None},
           "deepest_modelled_sphere_depth_when_front_penetrates_m": {"p50": q(dsph_when_front, 0.5)},
           "front_only_horizontal_speed_m_per_s": {"p50": q(vfront_only, 0.5), "p95": q(vfront_only, 0.95),
                                                   "n": len(vfront_only)},
           # feet_slide (weight -0.25, x step_dt 0.02; V/mdp/rewards.py feet_slide, C12 flat cfg): the contribution the
           # build misses in front-end-only contacts (the front end's speed standing in for the foot body's), against the
           # build's own (the foot origin's speed in its modelled-contact foot-steps); per env-step
           "feet_slide_per_env_step": {"build": -0.25 * 0.02 * slide_build / env_steps,
                                       "missed_front_only": -0.25 * 0.02 * float(np.sum(vfront_only)) / env_steps},
           # feet_air_time: a foot's first contact (ContactSensor first_contact) that the reference's side rod would have
           # made one or more env steps earlier (its front end alone touching in the preceding sample)
           "air_time_first_contacts": {"n": stats["first_contacts"],
                                       "preceded_by_front_only": stats["first_contacts_preceded_by_front_only"],
                                       "fraction": stats["first_contacts_preceded_by_front_only"] / max(1, stats["first_contacts"])}}
    s = json.dumps(res, indent=1)
    print(s)
    if a.out:
        Path(a.out).write_text(s + "\n")


if __name__ == "__main__":
    main()
