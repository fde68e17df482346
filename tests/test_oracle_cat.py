"""CPU: the CaT task (row f4, Isaac-Velocity-CaT-Flat-H12_12dof-v0; T/utils/cat/*, cat_env_cfg.py) -- the cfg ->
C-ABI mapping, the oracle's constraint values recomputed from the state (constraints.py), and its
ConstraintManager / CaTEnv.step pass checked against a numpy restatement of constraint_manager.py:23-123 +
cat_env.py:148-166 fed with the oracle's raw constraints: running maxima, probabilities, the no_move row remap,
reward scaling, dones, episode statistics and their log.

Parity against IsaacLab / PhysX is unpinned (not installed); ArticulationData.joint_vel_limits /
joint_effort_limits are taken as the URDF velocity limits and IsaacLab's 1e9 explicit-actuator effort limit
(RobotCfg, documented in DESIGN.md)."""
import numpy as np
import pytest

import oracle as O
from h12env._abi import CONSTRAINT_TERMS, NCSTR, NREW, REWARD_FUNCS
from h12env._abi import F as FIELDS
from h12env.cfg import ConstraintPTerm, H12CaTEnvCfg, H12RslEnvCfg
from h12env.startup import apply_to_arrays, startup_state

COL0 = [0, 1, 13, 25, 37, 39, 51, 52, 53, 54, 56]


def test_cat_cfg_maps_onto_the_kernel():
    cfg = H12CaTEnvCfg()
    c = cfg.to_c()
    assert c.cat_enable == 1 and c.cstr_mask == (1 << NCSTR) - 1
    assert [round(x, 6) for x in c.cstr_max_p] == [1.0] + [0.25] * 9
    assert c.cat_tau == pytest.approx(0.95) and c.cat_min_p == 0.0
    assert list(c.cstr_joint_vel_limit) == [23, 23, 23, 14, 9, 9] * 2
    assert c.cstr_foot_force_limit == 750 and c.cstr_nomove_vel == 6 and c.cstr_nomove_deadzone == pytest.approx(0.2)
    assert c.cstr_height == 1.0 and c.cstr_height_std == pytest.approx(0.05)
    assert c.cstr_clearance_min == pytest.approx(0.1) and c.cstr_orient_limit == pytest.approx(0.1)
    # 7 reward terms; joint_deviation_l1 over hip yaw/roll + ankle pitch/roll = two kernel ids at -0.1
    act = cfg.rewards.active()
    assert [k for k, _ in act] == ["track_lin_vel_xy_exp", "track_ang_vel_z_exp", "dof_torques_l2", "joint_acc_l2",
                                   "joint_vel_l2", "action_rate_l2", "joint_deviation_l1"]
    w = np.array(c.rew_w)
    assert w[REWARD_FUNCS.index("joint_deviation_l1:hip")] == pytest.approx(-0.1)
    assert w[REWARD_FUNCS.index("joint_deviation_l1:ankle")] == pytest.approx(-0.1)
    assert w[REWARD_FUNCS.index("joint_acc_l2")] == pytest.approx(-2.5e-7)
    assert (c.min_delay, c.max_delay) == (0, 5) and c.velocity_deadzone == pytest.approx(0.2)
    assert c.per_env_friction == 1 and c.per_env_mass == 1 and c.push_enable == 1 and c.history_length == 6
    # modify_constraint_p: max_p goes from 1/20 to init_max_p over num_steps
    t = cfg.curriculum.constraint_p[0]
    assert t.max_p(0) == pytest.approx(0.05) and t.max_p(10 ** 9) == pytest.approx(0.25)
    assert t.max_p(t.num_steps // 2) == pytest.approx(1 / 12)
    assert len(cfg.curriculum.constraint_p) == 9
    assert H12RslEnvCfg().to_c().cat_enable == 0


def cat_oracle(model, n, seed=0):
    cfg = H12CaTEnvCfg()
    cfg.scene.num_envs = n
    cfg.seed = seed
    c = cfg.to_c()
    env = O.OracleEnv(model, c, n)
    apply_to_arrays(startup_state(cfg, n), env.F, env.I)
    O.set_dz_count(0)
    O.cat_reset()
    return env, cfg, c


def field(F, k):
    o, cnt = FIELDS[k]
    return F[o:o + cnt]


def cat_pass_numpy(cs, run_prev, max_p, tau=float(np.float32(0.95)), min_p=0.0, mask=(1 << NCSTR) - 1):
    """constraint_manager.py:42-78 (CaT.add / get_probs) + no_move's row remap (constraints.py:202-238)."""
    n = cs.shape[1]
    still = np.nonzero(cs[56] != 0)[0]
    rows = cs[:56].copy()
    nm = slice(COL0[5], COL0[6])
    if len(still):
        rows[nm] = cs[nm][:, still[np.arange(n) % len(still)]]
    else:
        rows[nm] = 0.0
    cmax = np.maximum(rows.max(axis=1), 1e-6)
    run = cmax if run_prev is None else tau * run_prev + (1 - tau) * cmax
    pt = np.zeros((NCSTR, n))
    for t in range(NCSTR):
        if not (mask >> t) & 1:
            continue
        r = rows[COL0[t]:COL0[t + 1]]
        p = np.where(r > 0, min_p + np.clip(r / run[COL0[t]:COL0[t + 1], None], 0, 1) * (max_p[t] - min_p), 0.0)
        pt[t] = p.max(axis=0)
    return run, pt, pt.max(axis=0)


def test_cat_pass_matches_numpy_restatement(model):
    n = 96
    env, cfg, c = cat_oracle(model, n)
    plain = H12CaTEnvCfg()
    plain.constraints = None
    ref = O.OracleEnv(model, plain.to_c(), n)
    env.reset()
    # a mix of still envs (no_move active) and moving ones, some envs out of the base-height band
    cmd = FIELDS["CMD"][0]
    env.F[cmd:cmd + 3, : n // 3] = 0.0
    env.F[FIELDS["POS"][0] + 2, n // 2:n // 2 + 5] += 0.2
    rng = np.random.default_rng(1)
    run = None
    sums = np.zeros((NCSTR, n))
    psums = np.zeros((NCSTR, n))
    max_p = np.array(c.cstr_max_p, dtype=np.float64)
    for t in range(1, 4):
        ref.F[:], ref.I[:], ref.obs[:] = env.F, env.I, env.obs
        O.set_dz_count(0)
        a = (0.5 * rng.normal(size=(n, 12))).astype(np.float32)
        _, r_plain, *_ = ref.step(a, t)
        O.set_dz_count(0)
        _, rew, term, trunc, info = env.step(a, t)
        cs = O.cat_last_constraints(n)
        run, pt, pmax = cat_pass_numpy(cs, run, max_p)
        np.testing.assert_allclose(O.cat_running_max(), run, rtol=1e-12)
        reset = term | trunc
        np.testing.assert_allclose(info["cstr_prob"], np.where(reset, 1.0, pmax), rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(rew, r_plain * (1 - pmax), rtol=2e-6, atol=1e-8)
        sums += pt > 0
        psums += pt
        sums[:, reset] = 0
        psums[:, reset] = 0
        np.testing.assert_allclose(field(env.F, "CSTR_SUM"), sums, atol=1e-6)
        np.testing.assert_allclose(field(env.F, "CSTR_P"), psums, rtol=1e-6, atol=1e-6)
        assert pmax.max() > 0
    # the no_move remap is exercised: still envs exist and their rows land on every env
    assert (cs[56] != 0).sum() >= n // 3


def test_constraint_values_from_state(model):
    n = 64
    env, cfg, c = cat_oracle(model, n, seed=3)
    env.reset()
    rng = np.random.default_rng(2)
    _, _, term, trunc, info = env.step((0.8 * rng.normal(size=(n, 12))).astype(np.float32), 1)
    cs = O.cat_last_constraints(n)
    ok = ~(term | trunc)
    F = env.F
    q, qd = field(F, "Q"), field(F, "QD")
    lo, hi = np.asarray(model.q_lower)[:, None], np.asarray(model.q_upper)[:, None]
    mid, half = (lo + hi) / 2, (hi - lo) / 2 * 0.9
    np.testing.assert_allclose(cs[1:13][:, ok], np.maximum(mid - half - q, q - mid - half)[:, ok], atol=2e-6)
    vl = np.array([23, 23, 23, 14, 9, 9] * 2)[:, None]
    np.testing.assert_allclose(cs[13:25][:, ok], (np.abs(qd) - vl)[:, ok], atol=1e-5)
    tq = info["applied_torque"].T.astype(np.float64)
    np.testing.assert_allclose(cs[25:37][:, ok], (np.abs(tq) - 1e9)[:, ok], rtol=1e-12)
    np.testing.assert_allclose(cs[39:51][:, ok], (np.abs(qd) - 6.0)[:, ok], atol=1e-5)
    qw, qx, qy, qz = field(F, "QUAT")
    gx, gy = 2 * (qw * qy - qx * qz), -2 * (qw * qx + qy * qz)      # projected gravity xy
    np.testing.assert_allclose(cs[51][ok], (np.hypot(gx, gy) - 0.1)[ok], atol=1e-5)
    z = field(F, "POS")[2]
    np.testing.assert_array_equal(cs[52][ok], ((z < 0.95) | (z > 1.05))[ok].astype(float))
    np.testing.assert_array_equal(cs[0], term.astype(float))
    cm = field(F, "CMD")
    still = (np.abs(cm) < 0.2).all(axis=0)
    # commands may be resampled / deadzoned after the constraints; envs without a command change agree
    assert set(np.unique(cs[56])) <= {0.0, 1.0}
    assert (cs[57] >= 1).all()
    del still


def test_episode_statistics_logged_at_reset(model):
    n = 32
    env, cfg, c = cat_oracle(model, n)
    env.reset()
    E = FIELDS["EPSUM"][0]
    del E
    # push every env past the episode length in the next step: all reset, all logged
    env.I[0] = 999
    _, _, term, trunc, info = env.step(np.zeros((n, 12), np.float32), 1)
    assert trunc.all()
    np.testing.assert_array_equal(info["cstr_prob"], 1.0)
    log = info["log"]
    assert log[NREW] == n
    assert (log[NREW + 4:NREW + 4 + NCSTR] >= 0).all()
    np.testing.assert_allclose(field(env.F, "CSTR_SUM"), 0)
    np.testing.assert_allclose(field(env.F, "CSTR_P"), 0)


def test_constraint_curriculum_schedule():
    t = ConstraintPTerm("joint_position_limits", 24 * 5000, 0.25)
    steps = np.array([0, 1, 60000, 120000, 240000])
    got = np.array([t.max_p(int(s)) for s in steps])
    prog = np.minimum(steps / 120000, 1.0)
    np.testing.assert_allclose(got, 1 / (20 + prog * (4 - 20)))
    assert CONSTRAINT_TERMS.index("no_move") == 5
