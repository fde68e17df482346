"""CPU: the oracle's self-collision model between the legs (ArticulationCfg enabled_self_collisions=True,
A/robots/h12.py:32; colliders h12_12dof.urdf:116,168-191,286,338-361).

The model is the build's (PhysX's contact solver is not available): knee cylinders and the four sole rods of each
foot as capsules, penalty contact between every left/right pair.  Checked here: the rod
segments come from the URDF, no force while the legs are apart, action = reaction (zero net force and moment on
the robot), a leg driven into the other is held off (and passes through without the model), random-action
rollouts stay finite, and knee self-contact is an illegal contact (C12/rough_env_cfg.py:95-109)."""
import xml.etree.ElementTree as ET
from pathlib import Path

import numpy as np
import pytest

import oracle as O
from h12env import H12FlatEnvCfg
from h12env._abi import F as FI

URDF = Path("/root/reference/packages/biped_assets/biped_assets/models/h12/h12_12dof.urdf")


def crossed_state(model, roll, z=2.0):
    s = np.zeros(37)
    s[2] = z
    s[3] = 1.0
    s[13:25] = np.asarray(model.q_default)
    s[13 + 2], s[13 + 8] = roll, -roll  # hip roll inward on both legs (mirror signs)
    return s


def world_wrench(model, state, fext):
    """Net world force and moment about the world origin of body-coordinate spatial forces."""
    R, p = O.body_poses(model, state)
    F = np.zeros(3)
    M = np.zeros(3)
    for b in range(13):
        fw = R[b] @ fext[b, 3:]
        nw = R[b] @ fext[b, :3]
        F += fw
        M += nw + np.cross(p[b], fw)
    return F, M


@pytest.mark.skipif(not URDF.exists(), reason="reference URDF not present (build container only)")
def test_rod_segments_follow_the_urdf(model):
    root = ET.parse(URDF).getroot()
    segs = []
    for c in root.findall("link[@name='left_ankle_roll_link']/collision"):
        xyz = np.array([float(v) for v in c.find("origin").get("xyz").split()])
        rpy = np.array([float(v) for v in c.find("origin").get("rpy").split()])
        L = float(c.find("geometry/cylinder").get("length"))
        ax = np.array([0, 1.0, 0]) if abs(rpy[0]) > 1 else np.array([1.0, 0, 0])
        segs.append(sorted([tuple(xyz - ax * L / 2), tuple(xyz + ax * L / 2)]))
    got = [sorted([tuple(np.array(model.foot_rods[r][e][:], dtype=np.float64)) for e in range(2)]) for r in range(4)]
    np.testing.assert_allclose(np.array(sorted(got)), np.array(sorted(segs)), atol=1e-6)


def test_no_force_when_apart(model):
    c = H12FlatEnvCfg().to_c()
    for roll in (0.0, -0.05, -0.1):
        f, rep = O.self_contacts(model, c, crossed_state(model, roll))
        assert np.abs(f).max() == 0.0


@pytest.mark.parametrize("roll", [-0.13, -0.15, -0.25, -0.35])
def test_action_equals_reaction(model, roll):
    c = H12FlatEnvCfg().to_c()
    rng = np.random.default_rng(int(-roll * 100))
    hit = 0
    for _ in range(10):
        s = crossed_state(model, roll)
        s[13:25] += rng.normal(size=12) * 0.05
        s[25:37] = rng.normal(size=12)
        f, rep = O.self_contacts(model, c, s)
        hit += np.abs(f).max() > 0
        F, M = world_wrench(model, s, f)
        scale = 1.0 + np.abs(f).max()
        np.testing.assert_allclose(F, 0.0, atol=1e-9 * scale)
        np.testing.assert_allclose(M, 0.0, atol=1e-9 * scale)
        # only the knees and feet receive self-contact wrenches
        assert np.abs(f[[0, 1, 2, 3, 5, 7, 8, 9, 11]]).max() == 0.0
    assert hit > 0


def _drive_crossing(model, self_collision, steps=100):
    cfg = H12FlatEnvCfg()
    cfg.fix_base = True
    cfg.sim.self_collision = self_collision
    c = cfg.to_c()
    ref = O.OracleEnv(model, c, 1)
    ref.reset()
    ref.F[0:7, 0] = [0, 0, 2.0, 1, 0, 0, 0]
    q = np.asarray(model.q_default, dtype=np.float64).copy()
    q[2], q[8] = -0.1, 0.1
    ref.F[FI["Q"][0]:FI["Q"][0] + 12, 0] = q
    ref.F[FI["QD"][0]:FI["QD"][0] + 12, 0] = 0.0
    qr = q.copy()
    qr[2], qr[8] = -0.43, 0.43  # drive both legs inward to the hip-roll limit: the feet would cross
    dy = []
    for _ in range(steps):
        ref.step_physics(qr[None].astype(np.float32), 1)
        s = np.zeros(37)
        s[0:7] = ref.F[0:7, 0]
        s[13:25] = ref.F[FI["Q"][0]:FI["Q"][0] + 12, 0]
        _, p = O.body_poses(model, s)
        dy.append(p[6][1] - p[12][1])  # left foot y - right foot y
    assert np.isfinite(ref.F).all()
    return np.array(dy)


def test_crossing_feet_are_held_apart(model):
    dy_on = _drive_crossing(model, True)
    dy_off = _drive_crossing(model, False)
    assert dy_off.min() < -0.2          # without the model the feet pass through each other
    assert dy_on.min() > 0.0            # with it the left foot stays left of the right one
    assert dy_on[-1] < 0.12             # ... while pressed against it


def test_random_action_rollout_finite_and_knee_contacts_terminate(model):
    n = 512
    out = {}
    for sc in (False, True):
        cfg = H12FlatEnvCfg()
        cfg.scene.num_envs = n
        cfg.sim.self_collision = sc
        ref = O.OracleEnv(model, cfg.to_c(), n)
        ref.reset()
        rng = np.random.default_rng(0)
        term = 0
        for t in range(1, 121):
            _, _, te, _, _ = ref.step(rng.normal(size=(n, 12)).astype(np.float32), t, n_threads=8)
            term += int(te.sum())
        assert np.isfinite(ref.F).all()
        assert np.abs(ref.F[FI["QD"][0]:FI["QD"][0] + 12]).max() < 500.0
        out[sc] = term
    # knee self-contacts are illegal contacts: more falls are declared with the model
    assert out[True] > out[False]


def test_self_jitter_hook(model):
    """The forced-parity harness's capsule jitter (oracle set_self_jitter): off by default and after reset to 0
    (bit-identical wrenches), and a 1e-6 m jitter moves a penetrating pair's force by about k * 1e-6 m."""
    c = H12FlatEnvCfg().to_c()
    s = crossed_state(model, -0.25)
    # a generic crossing (the symmetric state itself has exactly intersecting rod axes: no contact normal)
    s[13:25] += np.random.default_rng(3).normal(size=12) * 0.05
    f0, _ = O.self_contacts(model, c, s)
    assert np.abs(f0).max() > 0
    try:
        O.set_self_jitter(1e-6, 7)
        f1, _ = O.self_contacts(model, c, s)
    finally:
        O.set_self_jitter(0.0)
    f2, _ = O.self_contacts(model, c, s)
    np.testing.assert_array_equal(f2, f0)
    d = np.abs(f1 - f0).max()
    assert 0.0 < d < 10 * c.self_k * 1e-6


def test_self_friction_follows_randomised_materials(model):
    """With the startup material randomisation (C12/rsl_env_cfg.py:213-223) the leg-leg Coulomb cap is the
    product of the two legs' randomised dynamic coefficients (PhysX multiply combine), not the fixed 0.6 x 0.6."""
    c = H12FlatEnvCfg().to_c()
    s = crossed_state(model, -0.25)
    s[13:25] += np.random.default_rng(3).normal(size=12) * 0.05  # a generic crossing (test_self_jitter_hook)
    s[25:37] = np.random.default_rng(11).normal(size=12) * 4.0  # sliding: the tangential drag reaches its cap
    f_fixed, _ = O.self_contacts(model, c, s)
    assert np.abs(f_fixed).max() > 0
    c.per_env_friction = 1
    f_same, _ = O.self_contacts(model, c, s, mu=[0.6, 0.6, 0.6, 0.6])
    np.testing.assert_allclose(f_same, f_fixed, rtol=1e-6, atol=1e-9)  # self_mu is the fp32 0.36
    f_low, _ = O.self_contacts(model, c, s, mu=[0.1, 0.1, 0.2, 0.2])
    f_nofric, _ = O.self_contacts(model, c, s, mu=[0.0, 0.0, 0.0, 0.0])
    # the frictionless wrenches are the normal forces alone; a lower cap moves the result towards them
    assert np.abs(f_low - f_fixed).max() > 1e-3 * np.abs(f_fixed).max()
    assert np.abs(f_low - f_nofric).max() < np.abs(f_fixed - f_nofric).max()
    # without the randomisation flag the per-env values are ignored
    c.per_env_friction = 0
    f_off, _ = O.self_contacts(model, c, s, mu=[0.1, 0.1, 0.2, 0.2])
    np.testing.assert_array_equal(f_off, f_fixed)
