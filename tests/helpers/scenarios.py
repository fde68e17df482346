"""Well-conditioned forced-parity scenarios (test infrastructure; round 4).

The random-action Flat runs are dominated by ill-conditioned env-steps: stiff contacts (1e5 N/m) and stick / slip
switching amplify a 1e-7 relative perturbation of the pre-step state to ~1e-5 after one policy step (the
conditioning probe of tests/helpers/forced.py measures it per env-step), so a systematic error of 1e-5..1e-4
relative hides under amplified fp32 rounding there.  These scenarios put the env in states whose one-step map is
well-conditioned, so that the error quantiles of the teacher-forced comparison sit at the fp32 floor and a planted
1e-4-relative constant error stands out:

  flight   the robot 20 m above the floor, random base twist and joint motion: free-joint quaternion
           integration, the base row of the articulated-body solve, PD actuators and every inertia / mass
           without contact (M/h12_12dof.xml:68 free joint; A/robots/h12.py actuators)
  lying    robots resting on the torso box (h12_12dof.urdf:387), as test_torso_face_contacts_forced: the
           face's corner contacts carry the body with both contact spring and damper active, joints moving
           under small actions

Each function rewrites the physics rows of the field-major float state Fm [H12_NF_FLOAT, n] in place."""
from __future__ import annotations

import numpy as np

import oracle as O
from h12env._abi import F as FIELDS


def _set(Fm, name, i, v):
    o, c = FIELDS[name]
    Fm[o:o + c, i] = v


def _quat(roll, pitch, yaw):
    cy, sy, cp, sp, cr, sr = (np.cos(yaw / 2), np.sin(yaw / 2), np.cos(pitch / 2), np.sin(pitch / 2),
                              np.cos(roll / 2), np.sin(roll / 2))
    return np.array([cr * cp * cy + sr * sp * sy, sr * cp * cy - cr * sp * sy, cr * sp * cy + sr * cp * sy,
                     cr * cp * sy - sr * sp * cy])


def flight(model, Fm, rng, height=20.0):
    n = Fm.shape[1]
    q0 = np.asarray(model.q_default, dtype=np.float64)
    for i in range(n):
        _set(Fm, "POS", i, [rng.uniform(-1, 1), rng.uniform(-1, 1), height + rng.uniform(0, 1)])
        _set(Fm, "QUAT", i, _quat(*rng.uniform(-0.5, 0.5, 2), rng.uniform(-np.pi, np.pi)))
        _set(Fm, "VLIN", i, rng.normal(size=3) * 0.5)
        _set(Fm, "WANG", i, rng.normal(size=3) * 1.0)
        _set(Fm, "Q", i, q0 + rng.normal(size=12) * 0.1)
        _set(Fm, "QD", i, rng.normal(size=12) * 0.5)
    return Fm


def lying(model, Fm, rng):
    n = Fm.shape[1]
    ch = np.array(model.torso_center, dtype=np.float64)
    hh = np.array(model.torso_half, dtype=np.float64)
    signs = np.array([[sx, sy, sz] for sx in (-1, 1) for sy in (-1, 1) for sz in (-1, 1)], dtype=np.float64)
    for i in range(n):
        pitch = rng.uniform(np.deg2rad(80), np.deg2rad(100)) * (1 if i % 2 else -1)
        quat = _quat(rng.uniform(-0.2, 0.2), pitch, rng.uniform(-np.pi, np.pi))
        s = np.zeros(37)
        s[3:7] = quat
        s[13:25] = np.asarray(model.q_default) + rng.normal(size=12) * 0.05
        R, p = O.body_poses(model, s)
        z = (R[0] @ (ch[None] + signs * hh[None]).T)[2] + p[0][2]
        _set(Fm, "POS", i, [rng.uniform(-1, 1), rng.uniform(-1, 1), -z.min() - rng.uniform(0.0, 0.004)])
        _set(Fm, "QUAT", i, quat)
        _set(Fm, "VLIN", i, rng.normal(size=3) * 0.1)
        _set(Fm, "WANG", i, rng.normal(size=3) * 0.1)
        _set(Fm, "Q", i, s[13:25])
        _set(Fm, "QD", i, 0.0)
    return Fm


def lying_terrain(model, Fm, rng, terrain):
    """`lying` on the Rough heightfield: each robot at its env origin (H12_F_ORIGIN, +-0.5 m), the body placed so that
    the deepest of the torso box's 8 corners is 0-4 mm below the heightfield under it (h12env.terrain.ground_height,
    the kernels' triangle interpolation) -- the heightfield contact path (ground_local, torso_face on terrain)."""
    from h12env.terrain import ground_height

    n = Fm.shape[1]
    ch = np.array(model.torso_center, dtype=np.float64)
    hh = np.array(model.torso_half, dtype=np.float64)
    signs = np.array([[sx, sy, sz] for sx in (-1, 1) for sy in (-1, 1) for sz in (-1, 1)], dtype=np.float64)
    o, _ = FIELDS["ORIGIN"]
    for i in range(n):
        pitch = rng.uniform(np.deg2rad(80), np.deg2rad(100)) * (1 if i % 2 else -1)
        quat = _quat(rng.uniform(-0.2, 0.2), pitch, rng.uniform(-np.pi, np.pi))
        s = np.zeros(37)
        s[3:7] = quat
        s[13:25] = np.asarray(model.q_default) + rng.normal(size=12) * 0.05
        R, p = O.body_poses(model, s)
        c = (R[0] @ (ch[None] + signs * hh[None]).T).T + p[0]  # corners relative to the base position
        x, y = Fm[o, i] + rng.uniform(-0.5, 0.5), Fm[o + 1, i] + rng.uniform(-0.5, 0.5)
        g = ground_height(terrain, x + c[:, 0], y + c[:, 1])
        _set(Fm, "POS", i, [x, y, float(np.max(g - c[:, 2])) - rng.uniform(0.0, 0.004)])
        _set(Fm, "QUAT", i, quat)
        _set(Fm, "VLIN", i, rng.normal(size=3) * 0.1)
        _set(Fm, "WANG", i, rng.normal(size=3) * 0.1)
        _set(Fm, "Q", i, s[13:25])
        _set(Fm, "QD", i, 0.0)
    return Fm


SCENARIOS = dict(flight=flight, lying=lying)
