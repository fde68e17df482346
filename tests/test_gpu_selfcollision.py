"""GPU parity of the self-collision model (knee cylinders and sole rods of the two legs, explicit penalty;
A/robots/h12.py:32 enabled_self_collisions=True) against the oracle's restatement (oracle self_contacts):
crossing-leg states in the air (self-contacts only), and teacher-forced MDP steps from crossed standing
states, where knee-knee contacts are illegal contacts (C12/rough_env_cfg.py:95-109) and the feet's
self-contacts feed the contact sensor.  Criteria as in tests/helpers/forced.py."""
import numpy as np
import pytest
import torch

import oracle as O
from forced import ForcedParity, phys_err, unexplained_envs
from h12env import H12FlatEnvCfg
from h12env._abi import F as FIELDS
from h12env.env import H12VelocityEnv

pytestmark = pytest.mark.gpu


def make(n, cfg=None):
    cfg = cfg or H12FlatEnvCfg()
    cfg.scene.num_envs = n
    cfg.sim.device = "cuda:0"
    return H12VelocityEnv(cfg)


def crossed_states(env, rng, z, roll=(-0.35, -0.12), qd=1.0):
    n = env.num_envs
    Fm = env._fstate.cpu().numpy().copy()
    o = FIELDS
    Fm[o["POS"][0]:o["POS"][0] + 3] = np.stack([rng.uniform(-1, 1, n), rng.uniform(-1, 1, n), np.full(n, z)])
    yaw = rng.uniform(-np.pi, np.pi, n)
    Fm[o["QUAT"][0]:o["QUAT"][0] + 4] = np.stack([np.cos(yaw / 2), 0 * yaw, 0 * yaw, np.sin(yaw / 2)])
    Fm[o["VLIN"][0]:o["VLIN"][0] + 6] = 0.0
    q = np.asarray(env._model.q_default)[:, None] + rng.normal(size=(12, n)) * 0.05
    r = rng.uniform(*roll, n)
    q[2], q[8] = r, -r
    q[3] += rng.uniform(0.0, 0.6, n)  # left knee bent by a random amount: knees and feet interleave
    Fm[o["Q"][0]:o["Q"][0] + 12] = q
    Fm[o["QD"][0]:o["QD"][0] + 12] = rng.normal(size=(12, n)) * qd
    return Fm


def count_self_contacts(env, Fm):
    c = env._ccfg
    hits = 0
    for i in range(env.num_envs):
        s = np.zeros(37)
        s[0:7] = Fm[0:7, i]
        s[7:13] = Fm[7:13, i]
        s[13:37] = Fm[13:37, i]
        f, _ = O.self_contacts(env._model, c, s)
        hits += np.abs(f).max() > 0
    return hits


def test_self_collision_physics_parity_in_air(gpu):
    """Fixed base 2 m up (no ground contact): only the legs' self-contacts act."""
    n = 1024
    cfg = H12FlatEnvCfg()
    cfg.fix_base = True
    env = make(n, cfg)
    env.reset()
    ref = O.OracleEnv(env._model, env._ccfg, n)
    rng = np.random.default_rng(41)
    Fm = crossed_states(env, rng, 2.0)
    env._fstate.copy_(torch.from_numpy(Fm))
    ref.F[:] = Fm
    ref.I[:] = env._istate.cpu().numpy()
    assert count_self_contacts(env, Fm) > n // 4
    q_ref = Fm[FIELDS["Q"][0]:FIELDS["Q"][0] + 12].T.astype(np.float32).copy()
    q_ref[:, 2] -= 0.2  # keep pressing the legs together
    q_ref[:, 8] += 0.2
    F0, I0 = ref.F.copy(), ref.I.copy()

    def rerun(Fs):
        ref.F[:], ref.I[:] = Fs, I0
        for _ in range(4):
            ref.step_physics(q_ref, 1)
        return ref.F.copy()

    for _ in range(4):
        env.step_physics(torch.from_numpy(q_ref).cuda(), 1)
    g = env._fstate.cpu().numpy()
    base = rerun(F0)
    assert np.isfinite(g).all()
    gerr = phys_err(g, base)
    bad = unexplained_envs(F0, gerr, 2e-3, rerun, phys_err, base, g)
    assert bad.size == 0, (bad[:10], gerr[bad[:10]])
    assert (gerr > 2e-3).mean() <= 0.01
    # the model acts: without it the same states end elsewhere
    cfg_off = H12FlatEnvCfg()
    cfg_off.fix_base = True
    cfg_off.sim.self_collision = False
    off = O.OracleEnv(env._model, cfg_off.to_c(), n)
    off.F[:], off.I[:] = F0, I0
    for _ in range(4):
        off.step_physics(q_ref, 1)
    assert (phys_err(off.F, base) > 1e-2).mean() > 0.2
    env.close()


def test_self_collision_mdp_forced_knee_contacts_terminate(gpu):
    """Crossed standing states, 30 teacher-forced MDP steps: knee self-contacts end episodes (illegal contact)
    exactly as in the oracle; every env matches or is shown threshold-sensitive."""
    n = 1024
    env = make(n)
    env.reset()
    rng = np.random.default_rng(42)
    Fm = crossed_states(env, rng, 1.02, roll=(-0.3, -0.15), qd=0.5)
    env._fstate.copy_(torch.from_numpy(Fm))
    fp = ForcedParity(env, seed=42)
    terms = 0
    for t in range(30):
        a = (rng.normal(size=(n, 12)) * 0.3).astype(np.float32)
        a[:, 2] -= 0.5  # policy keeps pulling the legs inward
        a[:, 8] += 0.5
        (_, _, _, rew, tg, _), (_, _, _, _, to, _, _), _, _ = fp.step(a)
        terms += int(to.sum())
        assert np.isfinite(rew).all()
    # every env is pressed into self-contact here: the fp32 self-contact allowance is per such env-step
    fp.check(max_bad_frac=0.02, self_rate=0.0)
    assert terms > 50, terms
    env.close()


@pytest.mark.parametrize("task", ["flat", "rsl"])
def test_self_contact_wrenches_match_oracle(gpu, task):
    """The kernel's self-contact wrenches (h12env_eval_self_contacts) on crossed states against the oracle's
    self_contacts, body by body: no dynamics in between, so this pins the contact geometry, law and the
    mirror-lane frame conversions directly.  rsl: the startup material randomisation is on
    (C12/rsl_env_cfg.py:213-223), so each env's leg-leg Coulomb cap is the product of its two legs' randomised
    dynamic coefficients (H12_F_MU) instead of the fixed 0.6 x 0.6."""
    from h12env.cfg import H12RslEnvCfg

    n = 2048
    env = make(n, H12RslEnvCfg() if task == "rsl" else None)
    env.reset()
    mu = env._fstate[FIELDS["MU"][0]:FIELDS["MU"][0] + 4].cpu().numpy().astype(np.float64) if task == "rsl" else None
    if task == "rsl":
        assert env._ccfg.per_env_friction == 1 and mu.std(axis=1).min() > 0.1
    rng = np.random.default_rng(43)
    Fm = crossed_states(env, rng, 1.0, roll=(-0.4, -0.1), qd=2.0)
    env._fstate.copy_(torch.from_numpy(Fm))
    g = env.eval_self_contacts().cpu().numpy()  # (n, leg, body, 6)
    bodies = [(0, 0, 4), (0, 1, 6), (1, 0, 10), (1, 1, 12)]
    hit = 0
    worst = []
    for i in range(n):
        s = np.zeros(37)
        s[0:37] = Fm[0:37, i]
        f, _ = O.self_contacts(env._model, env._ccfg, s, None if mu is None else mu[:, i])
        hit += np.abs(f).max() > 0
        scale = max(1.0, np.abs(f).max())
        worst.append(max(np.abs(g[i, leg, b] - f[body]).max() / scale for leg, b, body in bodies))
    worst = np.array(worst)
    # a pair at its contact onset (depth within the fp32 rounding of its pelvis-relative points, ~1e-7 m) switches
    # its force c |v_n| on or off: such an env is threshold-sensitive when the oracle with its capsule end points
    # jittered at that scale reproduces the kernel's wrenches (the harness's rule, tests/helpers/forced.py);
    # every other env is bounded by the fp32 error of the contact law itself
    BOUND = 2e-3
    flipped = 0
    for i in np.nonzero(worst > BOUND)[0]:
        s = Fm[0:37, i].astype(np.float64)
        for k, eps in enumerate((1e-7,) * 32 + (3e-7,) * 32 + (1e-6,) * 32):
            O.set_self_jitter(eps, 1000 + k)
            try:
                f, _ = O.self_contacts(env._model, env._ccfg, s, None if mu is None else mu[:, i])
            finally:
                O.set_self_jitter(0.0)
            scale = max(1.0, np.abs(f).max())
            if max(np.abs(g[i, leg, b] - f[body]).max() / scale for leg, b, body in bodies) <= 0.5 * worst[i]:
                flipped += 1
                worst[i] = 0.0  # explained
                break
    print("self-contact wrench error quantiles (0.5, 0.9, 0.99, max) of the non-flipped envs:",
          np.quantile(worst, [0.5, 0.9, 0.99, 1.0]), "envs in contact", hit, "onset flips", flipped)
    assert hit > n // 4
    assert worst.max() <= BOUND, np.sort(worst)[-10:]
    assert flipped <= 0.01 * hit, flipped
    env.close()


def test_self_contact_release_timeout_is_reported(gpu, monkeypatch):
    """the self wave's wait for the contact wave's release (the shared self-contact jobs of a block with
    more jobs than lanes) is bounded; a wait that ends at the bound unreleased must surface, not silently leave
    partial wrenches.  With the test hook H12_TEST_SKIP_SELF_RELEASE=1 the contact wave never releases, so every
    such inner step ends at the bound: h12env_check (env.check_device) must raise.  The same states without the
    hook report nothing."""
    from h12env._abi import H12EnvError

    n = 256
    for skip in (False, True):
        if skip:
            monkeypatch.setenv("H12_TEST_SKIP_SELF_RELEASE", "1")
        else:
            monkeypatch.delenv("H12_TEST_SKIP_SELF_RELEASE", raising=False)
        env = make(n)
        monkeypatch.delenv("H12_TEST_SKIP_SELF_RELEASE", raising=False)  # read at create only
        env.reset()
        rng = np.random.default_rng(44)
        Fm = crossed_states(env, rng, 1.02, roll=(-0.4, -0.2), qd=0.5)
        env._fstate.copy_(torch.from_numpy(Fm))
        a = np.zeros((n, 12), np.float32)
        a[:, 2] -= 0.5
        a[:, 8] += 0.5
        env.step(torch.from_numpy(a).cuda())
        if skip:
            with pytest.raises(H12EnvError, match="release"):
                env.check_device()
            env.check_device()  # the word is cleared by the read
        else:
            env.check_device()
        env.close()
