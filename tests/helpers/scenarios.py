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
  stance   (round 5) both feet flat on the floor at the default pose, the 8 sole spheres in persistent, STICKING
           contact (anchors at the spheres, contact flags set), PD holding the default targets under small actions:
           the sole-contact path the benchmark spends its time in -- normal spring / damper, the anchored stiction
           spring k_t / damper c_t (V/velocity_env_cfg.py:153-163 material, h12_12dof.urdf:168-191 sole geometry)
  single_stance  (round 5) the same on ONE foot: the other leg's hip and knee flexed so its foot is ~6 cm up, the
           pelvis placed over the stance foot's support polygon; the stance foot carries the whole weight
  slip     (round 5) stance with the base sliding at 1.5-2.5 m/s and every sole anchor 8 mm behind its sphere: the
           soles SLIP, dragged at mu_d fn (the dynamic friction coefficient shapes the force directly)

Each function rewrites the physics rows of the field-major float state Fm [H12_NF_FLOAT, n] in place (and, for the
sole-contact scenarios, the sole contact flags of the packed int row Im[H12_I_PACK] when Im is given, and the action
history; those return the (n, 12) hold action the steps are driven around)."""
from __future__ import annotations

import numpy as np

import oracle as O
from h12env._abi import F as FIELDS
from h12env._abi import I as IFIELDS

FOOT_BODY = (6, 12)  # ankle-roll bodies of the left / right leg in the oracle's body order
CMASK_BIT0 = 13      # H12_I_PACK bit of sole sphere 0 of the left foot (bit 13 + 4 foot + point)


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


def _soles(model, s):
    """World centres (2, 4, 3) of the 8 sole spheres for the 37-float physics state s (oracle kinematics)."""
    R, p = O.body_poses(model, s)
    pts = np.asarray(model.foot_pts, dtype=np.float64)
    return np.stack([(R[b] @ pts.T).T + p[b] for b in FOOT_BODY])


def _stance_state(model, rng, quat, q):
    s = np.zeros(37)
    s[3:7] = quat
    s[13:25] = q
    return s


def _place_on_soles(model, Fm, Im, i, s, feet, depth, anchor_shift=(0.0, 0.0), action_scale=0.5, preload=0.0):
    """Base height so that the lowest sole sphere of `feet` is `depth` deep; anchors at the spheres' current xy
    (world xy on the plane tasks) shifted by anchor_shift; contact flags of those feet's spheres set; the action
    history (ACT, ACT_PREV: the delayed-PD targets of the next steps) holding the joint angles.  Returns the hold
    action (JointPositionAction: target = q_default + scale a)."""
    r = float(model.foot_radius)
    sol = _soles(model, s)
    zmin = min(sol[f][:, 2].min() for f in feet)
    s[2] = r - depth - zmin
    sol = _soles(model, s)
    _set(Fm, "POS", i, s[0:3])
    _set(Fm, "QUAT", i, s[3:7])
    _set(Fm, "VLIN", i, s[7:10])
    _set(Fm, "WANG", i, s[10:13])
    _set(Fm, "Q", i, s[13:25])
    _set(Fm, "QD", i, s[25:37])
    oa, _ = FIELDS["ANCHOR"]
    org = 0.0  # plane tasks: anchors in world xy (only the heightfield kernels work relative to the env origin)
    # preload: each foot's anchors `preload` m beyond its spheres along the base's lateral axis, away from the other
    # foot -- the sticking stiction springs then carry k_t x preload each (the legs pushed apart), so the tangential
    # spring's constant shapes the step
    lat = np.array(O.body_poses(model, s)[0][0][:2, 1])
    lat = lat / max(np.linalg.norm(lat), 1e-12)
    for f in range(2):
        side = 1.0 if f == 0 else -1.0
        for q in range(4):
            Fm[oa + 8 * f + 2 * q:oa + 8 * f + 2 * q + 2, i] = (sol[f][q, :2] - org + np.asarray(anchor_shift)
                                                                + side * preload * lat)
    if Im is not None:
        op, _ = IFIELDS["PACK"]
        pk = int(Im[op, i]) & ~(0xFF << CMASK_BIT0)
        for f in feet:
            pk |= 0xF << (CMASK_BIT0 + 4 * f)
        Im[op, i] = pk
    hold = (s[13:25] - np.asarray(model.q_default, dtype=np.float64)) / action_scale
    _set(Fm, "ACT", i, hold)
    _set(Fm, "ACT_PREV", i, hold)
    return hold


def stance(model, Fm, rng, Im=None, action_scale=0.5, preload=0.0):
    """Both feet flat (default pose: hip pitch + knee + ankle pitch sum to 0), the 8 soles ~0.8 mm deep (the static
    load of 661 N over 8 spheres at 1e5 N/m), small velocities."""
    n = Fm.shape[1]
    q0 = np.asarray(model.q_default, dtype=np.float64)
    hold = np.zeros((n, 12))
    for i in range(n):
        s = _stance_state(model, rng, _quat(0.0, 0.0, rng.uniform(-np.pi, np.pi)), q0 + rng.normal(size=12) * 0.005)
        s[7:10] = rng.normal(size=3) * 0.01
        s[10:13] = rng.normal(size=3) * 0.01
        s[25:37] = rng.normal(size=12) * 0.02
        s[0:2] = rng.uniform(-1, 1, 2)  # near the world origin, as flight / lying: fp32 positions to ~1e-7 m
        hold[i] = _place_on_soles(model, Fm, Im, i, s, (0, 1), 0.8e-3, action_scale=action_scale, preload=preload)
    return hold


def single_stance(model, Fm, rng, Im=None, action_scale=0.5):
    """One foot flat on the floor carrying the robot (~1.6 mm deep); the other leg's hip pitch -0.3 rad, knee +0.6 rad
    and ankle pitch -0.3 rad (its foot ~6 cm up, level); the stance leg's hip roll / ankle roll / ankle pitch set so
    the stance foot is flat and the composite centre of mass is over it (to ~2 mm; found once with the oracle's
    kinematics), so the robot balances on that foot through the scenario's policy steps."""
    n = Fm.shape[1]
    q0 = np.asarray(model.q_default, dtype=np.float64)
    stance_leg = {0: (-0.21944, 0.21659, 0.00376), 1: (0.22135, -0.21848, 0.00382)}  # hip roll, ankle roll, pitch
    hold = np.zeros((n, 12))
    for i in range(n):
        f = i % 2  # stance foot
        q = q0 + rng.normal(size=12) * 0.003
        sw = 6 * (1 - f)
        q[sw + 1] += -0.3   # swing hip pitch
        q[sw + 3] += 0.6    # swing knee
        q[sw + 4] += -0.3   # swing ankle pitch: the swing foot stays level
        hr, ar, ap = stance_leg[f]
        q[6 * f + 2] += hr
        q[6 * f + 5] += ar
        q[6 * f + 4] += ap
        s = _stance_state(model, rng, _quat(0.0, 0.0, rng.uniform(-np.pi, np.pi)), q)
        s[7:10] = rng.normal(size=3) * 0.01
        s[10:13] = rng.normal(size=3) * 0.01
        s[25:37] = rng.normal(size=12) * 0.02
        s[0:2] = rng.uniform(-1, 1, 2)
        hold[i] = _place_on_soles(model, Fm, Im, i, s, (f,), 1.6e-3, action_scale=action_scale)
    return hold


def slip(model, Fm, rng, Im=None, action_scale=0.5):
    """stance, the base sliding horizontally at 1.5-2.5 m/s (random heading) with every sole anchor 8 mm behind its
    sphere: the anchored stiction spring's trial force (k_t 8 mm + c_t v = 240 N + 200 N) is far above mu_s fn, so
    every sole slips and is dragged at mu_d fn from the first physics step on."""
    n = Fm.shape[1]
    q0 = np.asarray(model.q_default, dtype=np.float64)
    hold = np.zeros((n, 12))
    for i in range(n):
        s = _stance_state(model, rng, _quat(0.0, 0.0, rng.uniform(-np.pi, np.pi)), q0 + rng.normal(size=12) * 0.005)
        hd = rng.uniform(-np.pi, np.pi)
        u = np.array([np.cos(hd), np.sin(hd)])
        s[7:9] = u * rng.uniform(1.5, 2.5)
        s[25:37] = rng.normal(size=12) * 0.02
        s[0:2] = rng.uniform(-1, 1, 2)
        hold[i] = _place_on_soles(model, Fm, Im, i, s, (0, 1), 0.8e-3, anchor_shift=tuple(-8e-3 * u),
                                  action_scale=action_scale)
    return hold


SCENARIOS = dict(flight=flight, lying=lying)
# the sole-contact scenarios (take the packed int rows too)
SOLE_SCENARIOS = dict(stance=stance, single_stance=single_stance, slip=slip)
