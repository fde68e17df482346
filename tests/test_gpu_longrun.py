"""Long-horizon teacher-forced parity of the full Flat MDP step at the BASELINE size (4096 envs, 1100 steps).

Each step the GPU state is copied into the oracle and both step with the same actions (tests/helpers/forced.py
for the criteria and tolerances): per-term reward contributions, reward, terminated / truncated, the integer
state, the physics state and the newest observation frame of EVERY env are compared, and an env that leaves
tolerance must be shown threshold-sensitive by the oracle itself (perturbed re-runs), not by a percentage.
Episode lengths and command timers start randomised (rsl_rl's init_at_random_ep_len), so the window
reaches natural time-outs (V/velocity_env_cfg.py:264-268), 10 s command resampling (:92), standing envs,
falls (illegal contact, C12/rough_env_cfg.py:95-109) and the single-stance air-time reward path
(V/mdp/rewards.py:38-62); the test asserts each of these was exercised.  The episode-log accumulator of the
resetting envs (extras["log"], cat_env.py:217-245) is compared with the oracle's on every step whose resetting
envs all match.
"""
import numpy as np
import pytest
import torch

from forced import ForcedParity
from h12env import H12FlatEnvCfg
from h12env._abi import F as FIELDS
from h12env._abi import LOG_METRIC, NREW
from h12env.env import H12VelocityEnv

pytestmark = pytest.mark.gpu


def make(n, cfg=None):
    cfg = cfg or H12FlatEnvCfg()
    cfg.scene.num_envs = n
    cfg.sim.device = "cuda:0"
    return H12VelocityEnv(cfg)


@pytest.mark.timeout(600)
def test_teacher_forced_flat_4096x1100(gpu):
    n, steps = 4096, 1100
    env = make(n)
    env.reset()
    g = torch.Generator(device="cpu").manual_seed(21)
    env.episode_length_buf = torch.randint(0, int(env.max_episode_length), (n,), generator=g)
    ct = FIELDS["CMD_TIME"][0]
    env._fstate[ct].copy_(torch.rand(n, generator=g) * 10.0)
    fp = ForcedParity(env, seed=22)
    rng = np.random.default_rng(23)
    scale = rng.choice([0.15, 0.4, 1.0], size=(n, 1)).astype(np.float32)  # gentle envs stand and step longer
    o_ep = FIELDS["EPSUM"][0]
    cov = dict(time_outs=0, terminations=0, resamples=0, air_time_reward=0, log_steps=0)
    for t in range(steps):
        a = (rng.normal(size=(n, 12)).astype(np.float32) * scale)
        F0_ct = env._fstate[ct].cpu().numpy().copy()
        (Fg, Ig, og, rg, tg, trg), (Fo, Io, oo, ro, to, tro, info), ok, ex = fp.step(a)
        cov["time_outs"] += int(tro.sum())
        cov["terminations"] += int(to.sum())
        cov["resamples"] += int(((Fo[ct] > F0_ct + 1e-3) & ~(to | tro)).sum())
        done = to | tro
        cov["air_time_reward"] += int((((Fo[o_ep + 6] - fp.last_F0[o_ep + 6]) > 0) & ~done).sum())
        done_any = done | tg | trg  # envs resetting in either run (a threshold-sensitive flip resets one only)
        if done.any() and ok[done_any].all():
            # log accumulator of this step's resetting envs (episode sums, count, time-out / base-contact counts)
            env._flush_log()  # the fused step path defers its fold (h12env_flush_log)
            acc = env._log_ring[env.common_step_counter % len(env._log_ring)].cpu().numpy()
            lo = info["log"]
            k = list(range(NREW + 3)) + [LOG_METRIC, LOG_METRIC + 1]  # + the command metrics (ABI 7)
            np.testing.assert_allclose(acc[k], lo[k], rtol=1e-4, atol=1e-4 * max(1.0, float(np.abs(lo[k]).max())),
                                       err_msg=f"episode log at step {t + 1}")
            el = ex["log"]
            np.testing.assert_allclose(float(el["Metrics/base_velocity/error_vel_xy"]), lo[LOG_METRIC] / lo[NREW],
                                       rtol=1e-4, atol=1e-6)
            cov["log_steps"] += 1
        if (t + 1) % 100 == 0:
            print(f"[forced] step {t + 1}: {cov} explained {fp.explained} unexplained {len(fp.unexplained)}", flush=True)
    fp.check(max_bad_frac=0.01)
    print(fp.report(), cov)
    fp.check_quantiles()  # forced.RUN_GATE: the bulk of the error distribution stays at the measured floor
    assert cov["time_outs"] > 100, cov
    assert cov["terminations"] > 100, cov
    assert cov["resamples"] > 100, cov
    assert cov["log_steps"] > 100, cov
    assert cov["air_time_reward"] > 1000, cov
    env.close()

