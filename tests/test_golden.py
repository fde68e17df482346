"""CPU: the oracle against golden vectors produced by the reference's own code (tools/gen_golden.py):

  * CircularBuffer (utils/history/circular_buffer.py) as the ObservationManager history: term-major,
    oldest -> newest, first push after a reset fills the whole history;
  * CircularBuffer(max_delay + 1)[lag] as the DelayedPDActuator delay ring (one push per physics
    step, lag clamped to pushes - 1);
  * deploy ObservationHandler (biped_deploy/controllers/rl.py) with the Flat task's six terms:
    projected gravity, command pass-through, joint offsets, history layout;
  * ActionHandler: target = scale * a + q0 (JointPositionAction with use_default_offset).
All integer/index behaviour is bit-exact; float rows match to fp32 rounding.
"""
from pathlib import Path

import numpy as np

import oracle as O
from h12env import H12FlatEnvCfg

GOLD = Path(__file__).resolve().parent / "golden"


def test_history_matches_circular_buffer():
    z = np.load(GOLD / "circular_buffer.npz")
    for d, off, fo in ((3, 0, 0), (12, 90, 9)):
        frames, resets, hist = z[f"frames_d{d}"], z[f"resets_d{d}"], z[f"history_d{d}"]
        T, n = resets.shape
        rows = [np.zeros(450, np.float32) for _ in range(n)]
        for t in range(T):
            for i in range(n):
                fr = np.zeros(45)
                fr[fo:fo + d] = frames[t, i]
                fill = t == 0 or resets[t, i]
                rows[i] = O.history_write(fr, rows[i], fill)
                got = rows[i][off:off + 10 * d].reshape(10, d)
                np.testing.assert_array_equal(got, hist[t, i])


def test_delay_source_matches_circular_buffer_lag():
    z = np.load(GOLD / "delay_buffer.npz")
    lags, targets, resets, delayed, dec = z["lags"], z["targets"], z["resets"], z["delayed"], int(z["decimation"])
    T, n = targets.shape
    since = np.zeros(n, int)
    for t in range(T):
        since[resets[t]] = 0
        for s in range(dec):
            for i in range(n):
                src = O.delay_source(int(lags[i]), int(min(since[i], 2)), s, dec)
                assert src in (0, 1, 2)
                assert t - src >= 0
                np.testing.assert_array_equal(targets[t - src, i], delayed[t, s, i])
        since += 1


def test_observation_matches_deploy_handler(model):
    z = np.load(GOLD / "deploy_obs.npz")
    cfg = H12FlatEnvCfg()
    cfg.observations.policy.enable_corruption = False
    c = cfg.to_c()
    env = O.OracleEnv(model, c, 1)
    env.reset()
    from h12env._abi import F

    T = z["obs"].shape[0]
    for t in range(T):
        def put(name, vals):
            o, k = F[name]
            env.F[o:o + k, 0] = vals
        put("QUAT", z["quat"][t])
        put("WANG", z["wang"][t])
        put("CMD", z["cmd"][t])
        put("Q", z["q"][t])
        put("QD", z["qd"][t])
        put("ACT", z["act"][t])
        obs = env.observe(np.array([t == 0], np.uint8))
        np.testing.assert_allclose(obs[0], z["obs"][t], rtol=2e-6, atol=2e-6)


def test_action_scaling_matches_action_handler(model):
    z = np.load(GOLD / "deploy_obs.npz")
    q0 = np.array(model.q_default)
    np.testing.assert_allclose(float(z["action_scale"]) * z["action_in"] + q0, z["action_out"], rtol=0, atol=1e-7)  # q0 held in fp32
    # the env's JointPositionAction uses the same map with scale 0.5 (velocity_env_cfg.py:111)
    assert H12FlatEnvCfg().actions.joint_pos.scale == float(z["action_scale"])


def test_philox_known_answer():
    """Philox4x32-10 known-answer vectors (Salmon et al., SC'11 / Random123 kat_vectors)."""
    assert O.philox(0, 0, 0, 0, 0) == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    k = 0xA4093822299F31D0 & 0xFFFFFFFFFFFFFFFF
    # key (0xa4093822, 0x299f31d0) is (k0, k1): our uint64 seed packs k0 in the low word
    seed = 0xA4093822 | (0x299F31D0 << 32)
    assert O.philox(seed, 0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344) == [
        0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]
    del k
