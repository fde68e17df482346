"""extras["log"] semantics (CPU): the Metrics/base_velocity/* command metrics (IsaacLab 2.1
UniformVelocityCommand._update_metrics / CommandTerm.reset) in the oracle, and the persistence of extras["log"]
across steps without resets (the reference rebuilds it only in _reset_idx, cat_env.py:217-245)."""
import numpy as np
import torch

import oracle as O
from h12env import H12FlatEnvCfg
from h12env._abi import F as FIELDS
from h12env._abi import LOG_METRIC, NLOG, NREW
from h12env.env import _LazyLog


def _log(ring, slot, lookback=96):
    terms = [("track_lin_vel_xy_exp", [0]), ("track_ang_vel_z_exp", [1])]
    m = torch.zeros(2, NREW)
    m[0, 0] = m[1, 1] = 1.0
    return _LazyLog(ring, slot, 20.0, terms, m, lookback=lookback)


def test_log_keys_and_means():
    ring = torch.zeros(128, NLOG)
    acc = ring[5]
    acc[0], acc[1], acc[NREW], acc[NREW + 1], acc[NREW + 2] = 4.0, 2.0, 2.0, 1.0, 1.0
    acc[LOG_METRIC], acc[LOG_METRIC + 1] = 0.6, 0.2
    log = _log(ring, 5)
    assert set(log) == {"Episode_Reward/track_lin_vel_xy_exp", "Episode_Reward/track_ang_vel_z_exp",
                        "Metrics/base_velocity/error_vel_xy", "Metrics/base_velocity/error_vel_yaw",
                        "Episode_Termination/time_out", "Episode_Termination/base_contact"}
    assert abs(float(log["Episode_Reward/track_lin_vel_xy_exp"]) - 4.0 / 2 / 20.0) < 1e-7
    assert abs(float(log["Metrics/base_velocity/error_vel_xy"]) - 0.3) < 1e-7
    assert abs(float(log["Metrics/base_velocity/error_vel_yaw"]) - 0.1) < 1e-7
    assert float(log["Episode_Termination/time_out"]) == 1.0


def test_log_persists_over_steps_without_resets():
    """Slots 126, 127, 0 (the ring wraps): a step with resets, two without, then a step with resets again."""
    ring = torch.zeros(128, NLOG)
    ring[126, 0], ring[126, NREW], ring[126, LOG_METRIC] = 3.0, 1.0, 0.5
    ring[1, 0], ring[1, NREW] = 1.0, 1.0
    l1, l2, l3, l4 = (_log(ring, s) for s in (126, 127, 0, 1))
    for lg in (l2, l3):  # no reset: the last reset step's values
        assert list(lg) == list(l1)
        for k in l1:
            assert float(lg[k]) == float(l1[k])
    assert abs(float(l4["Episode_Reward/track_lin_vel_xy_exp"]) - 1.0 / 20.0) < 1e-7
    assert float(l4["Metrics/base_velocity/error_vel_xy"]) == 0.0
    # no reset within the lookback: zeros
    assert float(_log(ring, 0, lookback=2)["Episode_Reward/track_lin_vel_xy_exp"]) == 0.0


def test_oracle_command_metrics(model):
    """The oracle's per-step metric increment is |v*_xy - v_b,xy| / S and |w*_z - w_b,z| / S with S =
    resampling_time_range[1] / step_dt, on the post-step state (no env resets in this step)."""
    cfg = H12FlatEnvCfg()
    n = 8
    env = O.OracleEnv(model, cfg.to_c(), n)
    env.reset()
    rng = np.random.default_rng(0)
    for t in range(3):
        env.step(rng.normal(size=(n, 12)).astype(np.float32) * 0.3, t + 1)
    F0 = env.F.copy()
    _, _, term, trunc, info = env.step(rng.normal(size=(n, 12)).astype(np.float32) * 0.3, 4)
    assert not (term | trunc).any()
    o = FIELDS["METRIC"][0]
    q = env.F[FIELDS["QUAT"][0]:FIELDS["QUAT"][0] + 4].T.astype(np.float64)
    v = env.F[FIELDS["VLIN"][0]:FIELDS["VLIN"][0] + 3].T.astype(np.float64)
    w = env.F[FIELDS["WANG"][0]:FIELDS["WANG"][0] + 3].T.astype(np.float64)
    step_dt = cfg.sim.dt * cfg.decimation
    S = cfg.commands.base_velocity.resampling_time_range[1] / step_dt
    for i in range(n):
        qw, qx, qy, qz = q[i]
        R = np.array([[1 - 2 * (qy * qy + qz * qz), 2 * (qx * qy - qw * qz), 2 * (qx * qz + qw * qy)],
                      [2 * (qx * qy + qw * qz), 1 - 2 * (qx * qx + qz * qz), 2 * (qy * qz - qw * qx)],
                      [2 * (qx * qz - qw * qy), 2 * (qy * qz + qw * qx), 1 - 2 * (qx * qx + qy * qy)]])
        c = np.asarray(model.root_com, dtype=np.float64)
        vcom = v[i] + np.cross(R @ w[i], R @ c)  # root_lin_vel_w: the pelvis body COM velocity
        vb = R.T @ vcom
        cmd = F0[FIELDS["CMD"][0]:FIELDS["CMD"][0] + 3, i].astype(np.float64)
        d = env.F[o:o + 2, i] - F0[o:o + 2, i]
        np.testing.assert_allclose(d[0], np.hypot(cmd[0] - vb[0], cmd[1] - vb[1]) / S, rtol=1e-4, atol=1e-7)
        np.testing.assert_allclose(d[1], abs(cmd[2] - w[i, 2]) / S, rtol=1e-4, atol=1e-7)
    # CommandTerm.reset: a reset env logs its metrics and starts from zero
    env.F[FIELDS["EPSUM"][0]] = 0.0
    I = env.I.copy()
    env.I[0, 0] = 10 ** 6  # episode_length_buf past max: time-out on the next step
    _, _, term, trunc, info = env.step(np.zeros((n, 12), np.float32), 5)
    assert trunc[0]
    assert info["log"][LOG_METRIC] > 0.0
    env.I[:] = I
