"""CPU: physical invariants of the oracle's rigid-body dynamics (test infrastructure self-checks).

The dynamics of record (PhysX, MuJoCo) are absent here, so the oracle is pinned by invariants:
CRBA+Cholesky == ABA, SPD mass matrix, energy and momentum conservation with first-order convergence
under semi-implicit Euler, yaw invariance, and exact left/right mirror symmetry (which the GPU
kernel's mirror-lane design relies on).
"""
import numpy as np
import pytest

import oracle as O
from h12env import H12FlatEnvCfg
from h12env.model import build_model


def rand_state(rng, height=2.0):
    s = np.zeros(37)
    s[0:3] = [rng.normal(), rng.normal(), height]
    q = rng.normal(size=4)
    s[3:7] = q / np.linalg.norm(q)
    s[7:13] = rng.normal(size=6)
    s[13:25] = rng.normal(size=12) * 0.3
    s[25:37] = rng.normal(size=12)
    return s


@pytest.fixture(scope="module")
def ccfg():
    c = H12FlatEnvCfg().to_c()
    return c


def test_aba_equals_crba(model, ccfg):
    rng = np.random.default_rng(0)
    for _ in range(20):
        s = rand_state(rng)
        tau = rng.normal(size=12) * 20
        a0, _ = O.forward_dynamics(model, ccfg, s, tau, algo=0, contact=False)
        a1, _ = O.forward_dynamics(model, ccfg, s, tau, algo=1, contact=False)
        np.testing.assert_allclose(a0, a1, rtol=1e-9, atol=1e-8)


def test_aba_equals_crba_with_contact(model, ccfg):
    rng = np.random.default_rng(1)
    n_contact = 0
    for _ in range(20):
        s = rand_state(rng, height=0.98)
        a0, r0 = O.forward_dynamics(model, ccfg, s, np.zeros(12), algo=0, contact=True)
        a1, _ = O.forward_dynamics(model, ccfg, s, np.zeros(12), algo=1, contact=True)
        n_contact += np.abs(np.array(r0.foot_force)).sum() > 0
        np.testing.assert_allclose(a0, a1, rtol=1e-9, atol=1e-7)
    assert n_contact > 0


def test_mass_matrix_spd_and_total_mass(model):
    rng = np.random.default_rng(2)
    d = O.Phys()  # noqa: F841
    for _ in range(10):
        M = O.mass_matrix(model, rand_state(rng))
        np.testing.assert_allclose(M, M.T, atol=1e-12)
        assert np.linalg.eigvalsh(M).min() > 0
        total = model.base_mass + sum(model.link_mass)
        np.testing.assert_allclose(np.diag(M)[3:6], total, rtol=1e-12)  # linear block = total mass
    assert abs(total - 67.3676) < 1e-3


def _free_cfg(dt):
    c = H12FlatEnvCfg().to_c()
    c.limit_k = 0.0
    c.limit_c = 0.0
    c.limit_projection = 0.0  # no joint limits at all: free-articulation invariants
    c.physics_dt = dt
    c.inner_steps = 1
    return c


def test_energy_conservation_converges(model):
    rng = np.random.default_rng(3)
    s0 = rand_state(rng, height=5.0)
    errs = []
    for dt in (4e-4, 2e-4, 1e-4):
        c = _free_cfg(dt)
        e0, _, _ = O.energy_momentum(model, s0)
        s = s0.copy()
        for _ in range(int(round(0.1 / dt))):
            s, _ = O.physics_step(model, c, s, np.zeros(12), contact=False)
        e1, _, _ = O.energy_momentum(model, s)
        errs.append(abs(e1 - e0) / abs(e0))
    assert errs[-1] < 2e-5
    assert errs[0] / errs[-1] > 2.5  # ~first order: error halves with dt


def test_momentum_conservation_zero_gravity(model):
    from h12env.model import build_model as bm

    m = bm()
    m.gravity = 0.0
    rng = np.random.default_rng(4)
    s0 = rand_state(rng)
    c = _free_cfg(1e-4)
    _, l0, a0 = O.energy_momentum(m, s0)
    s = s0.copy()
    for _ in range(500):
        s, _ = O.physics_step(m, c, s, rng.normal(size=12) * 5, contact=False)  # internal torques only
    _, l1, a1 = O.energy_momentum(m, s)
    np.testing.assert_allclose(l1, l0, rtol=0, atol=2e-3 * np.abs(l0).max())
    np.testing.assert_allclose(a1, a0, rtol=0, atol=2e-3 * np.abs(a0).max())


def test_yaw_invariance(model, ccfg):
    rng = np.random.default_rng(5)
    s = rand_state(rng, height=0.99)
    s[3:7] = [1, 0, 0, 0]
    tau = rng.normal(size=12) * 10
    a0, _ = O.forward_dynamics(model, ccfg, s, tau, algo=1)
    yaw = 0.7
    s2 = s.copy()
    s2[3:7] = [np.cos(yaw / 2), 0, 0, np.sin(yaw / 2)]
    Rz = np.array([[np.cos(yaw), -np.sin(yaw), 0], [np.sin(yaw), np.cos(yaw), 0], [0, 0, 1]])
    s2[7:10] = Rz @ s[7:10]  # world linear velocity rotates; body-frame quantities do not
    a1, _ = O.forward_dynamics(model, ccfg, s2, tau, algo=1)
    np.testing.assert_allclose(a1, a0, rtol=1e-9, atol=1e-8)


def test_left_right_mirror_symmetry(ccfg):
    """Reflect a state through the pelvis xz-plane: accelerations reflect exactly.  This is the identity
    the GPU kernel's mirror lanes use (right leg simulated with left-leg constants).  The legs are exact
    mirror images in the MJCF; the welded upper body is not (composite COM y = 1.3 mm), so the check
    symmetrises the base inertia only — the kernel itself treats the base in real coordinates."""
    model = build_model()
    model.base_com[1] = 0.0
    model.base_inertia[3] = 0.0
    model.base_inertia[5] = 0.0
    rng = np.random.default_rng(6)
    sign_j = np.array([-1, 1, -1, 1, 1, -1], float)  # x / z joints flip
    for height in (2.0, 0.99):
        s = rand_state(rng, height=height)
        tau = rng.normal(size=12) * 10
        m = s.copy()
        w, x, y, z = s[3:7]
        m[3:7] = [w, -x, y, -z]                  # M R M
        m[0:3] = s[0:3] * [1, -1, 1]
        m[7:10] = s[7:10] * [1, -1, 1]
        m[10:13] = s[10:13] * [-1, 1, -1]        # pseudo-vector
        for leg in range(2):
            src = slice(6 * leg, 6 * leg + 6)
            dst = slice(6 * (1 - leg), 6 * (1 - leg) + 6)
            m[13:25][dst] = sign_j * s[13:25][src]
            m[25:37][dst] = sign_j * s[25:37][src]
        mt = np.zeros(12)
        mt[0:6], mt[6:12] = sign_j * tau[6:12], sign_j * tau[0:6]
        a, _ = O.forward_dynamics(model, ccfg, s, tau, algo=0, contact=True)
        b, _ = O.forward_dynamics(model, ccfg, m, mt, algo=0, contact=True)
        exp = np.zeros(18)
        exp[0:3] = a[0:3] * [-1, 1, -1]
        exp[3:6] = a[3:6] * [1, -1, 1]
        exp[6:12], exp[12:18] = sign_j * a[12:18], sign_j * a[6:12]
        np.testing.assert_allclose(b, exp, rtol=1e-9, atol=1e-7)


def test_contact_standing_is_stable(model):
    """Default gains/contact parameters (cfg.sim): the robot dropped from the reset pose settles on
    its feet (no energy blow-up) for 0.5 s with PD holding the default pose."""
    cfg = H12FlatEnvCfg()
    c = cfg.to_c()
    s = np.zeros(54)
    s[2] = 1.05
    s[3] = 1.0
    s[13:25] = np.array(model.q_default)
    kp, kd = np.array(c.kp), np.array(c.kd)
    zs = []
    for _ in range(100):
        tau = np.clip(kp * (np.array(model.q_default) - s[13:25]) - kd * s[25:37], -np.array(c.effort_limit),
                      np.array(c.effort_limit))
        s, rep = O.physics_step(model, c, s, tau)
        zs.append(s[2])
    zs = np.array(zs)
    assert np.isfinite(s).all()
    assert 0.95 < zs[-1] < 1.03 and zs.max() < 1.06
    foot = np.array(rep.foot_force)
    assert 200 < foot[:, 2].sum() < 1300  # carries roughly the robot's weight (661 N)


def _near_contact_state(rng):
    s = rand_state(rng, height=rng.uniform(0.9, 0.97))
    s[13:25] *= 0.3
    q = np.array([1.0, 0.05 * rng.normal(), 0.05 * rng.normal(), 0.3 * rng.normal()])
    s[3:7] = q / np.linalg.norm(q)
    return s


def test_aba_equals_crba_with_implicit_penalty(model):
    """Implicit contact adds a point inertia per active contact (and the force cancelling its weight); both
    algorithms must solve the same augmented system."""
    cfg = H12FlatEnvCfg()
    assert cfg.sim.implicit_penalty and cfg.sim.inner_steps == 1
    c = cfg.to_c()
    rng = np.random.default_rng(11)
    n_contact = 0
    for _ in range(30):
        s = _near_contact_state(rng)
        tau = rng.normal(size=12) * 10
        a0, r0 = O.forward_dynamics(model, c, s, tau, algo=0, dt_impl=c.physics_dt, contact=True)
        a1, _ = O.forward_dynamics(model, c, s, tau, algo=1, dt_impl=c.physics_dt, contact=True)
        ae, _ = O.forward_dynamics(model, c, s, tau, algo=1, dt_impl=0.0, contact=True)
        n_contact += np.abs(np.array(r0.foot_force)).sum() > 0
        np.testing.assert_allclose(a0, a1, rtol=1e-9, atol=1e-7)
    assert n_contact >= 20


def test_implicit_single_step_tracks_the_converged_penalty_model(model):
    """Accuracy of the default integrator (one implicit step per 5 ms physics step) against the explicit
    penalty model at 16 substeps (converged): the drop-and-stand settling height and sole load agree within
    1 mm / 2 %; the round-1 explicit scheme at 2 substeps is further off (it needs the substeps for
    stability and still under-resolves the stiff sole contact)."""

    def settle(inner, impl):
        cfg = H12FlatEnvCfg()
        cfg.sim.inner_steps, cfg.sim.implicit_penalty = inner, impl
        c = cfg.to_c()
        s = np.zeros(54)
        s[2], s[3] = 1.05, 1.0
        q0 = np.array(model.q_default)
        s[13:25] = q0
        kp, kd, E = np.array(c.kp), np.array(c.kd), np.array(c.effort_limit)
        for _ in range(200):
            s, rep = O.physics_step(model, c, s, np.clip(kp * (q0 - s[13:25]) - kd * s[25:37], -E, E))
        return s[2], np.array(rep.foot_force)[:, 2].sum()

    z_ref, f_ref = settle(16, False)
    z_imp, f_imp = settle(1, True)
    z_exp2, _ = settle(2, False)
    assert abs(z_imp - z_ref) < 1e-3 and abs(f_imp - f_ref) < 0.02 * f_ref
    assert abs(z_imp - z_ref) < abs(z_exp2 - z_ref)


def test_implicit_single_step_is_stable_under_random_actions(model):
    cfg = H12FlatEnvCfg()
    c = cfg.to_c()
    n = 64
    env = O.OracleEnv(model, c, n)
    env.reset()
    rng = np.random.default_rng(3)
    for t in range(1, 151):
        env.step(rng.normal(size=(n, 12)).astype(np.float32), t, n_threads=4)
    assert np.isfinite(env.F).all()
    assert np.abs(env.F[25:37]).max() < 200.0  # joint velocities stay physical


def test_torso_box_rests_on_its_lowest_face(model):
    """The torso box collider (h12_12dof.urdf:387) lying on a face is carried by the face's four corners (the
    lowest corner through the implicit contact, the other three explicitly): with the
    explicit integrator's forces and the robot at rest, the reported torso force is k x the summed depths of the
    corners below the floor, and an edge (box tilted about the face's long axis) is carried by two corners."""
    c = H12FlatEnvCfg().to_c()
    c.self_collision = 0
    ch, hh = np.array(model.torso_center, dtype=np.float64), np.array(model.torso_half, dtype=np.float64)
    signs = np.array([[sx, sy, sz] for sx in (-1, 1) for sy in (-1, 1) for sz in (-1, 1)], dtype=np.float64)
    for ang, n_expect in ((np.pi / 2, 4), (np.pi / 2 + 0.05, 2)):
        s = np.zeros(37)
        s[3:7] = [np.cos(ang / 2), 0.0, np.sin(ang / 2), 0.0]  # pitched forward onto the chest face
        s[13:25] = np.asarray(model.q_default)
        R, p = O.body_poses(model, s)
        z = (R[0] @ (ch[None] + signs * hh[None]).T)[2] + p[0][2]
        s[2] = -z.min() - 0.002  # the lowest corner 2 mm below the floor
        depth = np.clip(-(z + s[2]), 0.0, None)
        assert (depth > 0).sum() == n_expect
        _, rep = O.forward_dynamics(model, c, s, np.zeros(12), algo=1, dt_impl=0.0, contact=True)
        np.testing.assert_allclose(rep.torso_force[2], c.contact_k * depth.sum(), rtol=1e-9)
