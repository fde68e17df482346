"""GPU edge cases of the C-ABI: ragged env counts (partial lane blocks and partial observation-assembly
blocks), observation buffers that alias or are not 16-byte aligned (the scalar assembly path), and
partial resets.  Oracle: oracle/h12_oracle.c; observation assembly rtol 1e-5; full MDP steps teacher-forced
with the criteria of tests/helpers/forced.py."""
import ctypes as C

import numpy as np
import pytest
import torch

import oracle as O
from h12env import H12FlatEnvCfg
from h12env._abi import NOBS
from h12env.env import H12VelocityEnv
from forced import ForcedParity

pytestmark = pytest.mark.gpu


def make(n):
    cfg = H12FlatEnvCfg()
    cfg.scene.num_envs = n
    cfg.sim.device = "cuda:0"
    return H12VelocityEnv(cfg)


@pytest.mark.parametrize("n", [1, 37, 97])
def test_ragged_env_counts_match_oracle(gpu, n):
    """Ragged env counts (partial lane blocks, partial assembly blocks, a single env): reset bit-compatible,
    then 40 teacher-forced MDP steps where EVERY env must match the oracle or be shown threshold-sensitive
    by it (tests/helpers/forced.py) -- no percentage slack, also for n = 1."""
    env = make(n)
    obs, _ = env.reset()
    ref = O.OracleEnv(env._model, env._ccfg, n)
    r = ref.reset()
    torch.cuda.synchronize()
    np.testing.assert_allclose(obs["policy"].cpu().numpy(), r, rtol=1e-5, atol=1e-6)
    fp = ForcedParity(env, seed=n)
    rng = np.random.default_rng(11)
    for t in range(40):
        a = rng.normal(size=(n, 12)).astype(np.float32)
        (_, _, _, rew, _, _), _, _, _ = fp.step(a)
        assert np.isfinite(rew).all()
    fp.check(max_bad_frac=0.02)
    env.close()


def _observe(env, prev, out, fill=None):
    lib = env._lib
    rc = lib.h12env_observe(env._h, C.c_void_p(prev.data_ptr()), C.c_void_p(out.data_ptr()),
                            None if fill is None else C.c_void_p(fill.data_ptr()), env._stream())
    assert rc == 0


@pytest.mark.parametrize("n", [64, 37])
def test_observe_aliasing_and_unaligned_buffers(gpu, n):
    """Same observe call three ways -- out of place, in place (obs == obs_prev) and into buffers offset
    by one float (no float4 path) -- must give bit-identical rows.  Each call is the first observe
    call of its handle (same noise counter) on identical state."""
    env = make(n)
    env.reset()
    rng = np.random.default_rng(12)
    for _ in range(3):
        env.step(torch.from_numpy(rng.normal(size=(n, 12)).astype(np.float32)).cuda())
    fill = torch.zeros(n, dtype=torch.uint8, device="cuda")
    fill[::5] = 1
    src = env._obs[env._k].clone()
    outs = []
    # (1) out of place (first observe call of this handle: counter 0)
    out1 = torch.empty_like(src)
    _observe(env, src, out1, fill)
    outs.append(out1)
    # (2) in place, on a fresh handle with the same state (its first observe call: counter 0 too)
    inplace = src.clone()
    env2 = make(n)
    env2._fstate.copy_(env._fstate)
    env2._istate.copy_(env._istate)
    _observe(env2, inplace, inplace, fill)
    outs.append(inplace)
    # (3) unaligned source and destination
    env3 = make(n)
    env3._fstate.copy_(env._fstate)
    env3._istate.copy_(env._istate)
    buf_in = torch.empty(n * NOBS + 1, device="cuda")
    buf_out = torch.empty(n * NOBS + 1, device="cuda")
    buf_in[1:].copy_(src.reshape(-1))
    _observe(env3, buf_in[1:], buf_out[1:], fill)
    outs.append(buf_out[1:].reshape(n, NOBS))
    torch.cuda.synchronize()
    assert torch.equal(outs[1], outs[2])
    # history part and new frame layout: the new frame sits in the newest slot of every term block
    o = outs[2].cpu().numpy()
    s = src.cpu().numpy()
    f = fill.cpu().numpy().astype(bool)
    for off, d in ((0, 3), (30, 3), (60, 3), (90, 12), (210, 12), (330, 12)):
        np.testing.assert_array_equal(o[~f, off:off + 9 * d], s[~f, off + d:off + 10 * d])
        for h in range(9):  # filled rows: every slot equals the newest
            np.testing.assert_array_equal(o[f, off + h * d:off + (h + 1) * d], o[f, off + 9 * d:off + 10 * d])
    assert torch.equal(outs[0], outs[1])
    for e in (env, env2, env3):
        e.close()


def test_partial_reset_ragged(gpu):
    n = 37
    env = make(n)
    env.reset()
    ref = O.OracleEnv(env._model, env._ccfg, n)
    ref.reset()
    before = env._obs[env._k].clone().cpu().numpy()
    mask = np.zeros(n, bool)
    mask[[0, 5, 36]] = True
    env.reset(env_ids=np.nonzero(mask)[0])
    r = ref.reset(mask)
    after = env._obs[env._k].cpu().numpy()
    np.testing.assert_array_equal(after[~mask], before[~mask])
    np.testing.assert_allclose(after[mask], r[mask], rtol=1e-5, atol=1e-6)
    env.close()


@pytest.mark.parametrize("task", ["rsl", "cat"])
@pytest.mark.parametrize("n", [1, 37, 100])
def test_ragged_env_counts_rsl_cat(gpu, task, n):
    """The Play configs run 100 envs: partial lane blocks, partial 4-row assembly blocks of the 270-float
    rows (270 * 4 bytes is not a multiple of 16 per row), CaT's chunked column maxima and compaction."""
    from h12env.cfg import H12CaTEnvCfg, H12RslEnvCfg

    cfg = H12RslEnvCfg() if task == "rsl" else H12CaTEnvCfg()
    cfg.scene.num_envs = n
    cfg.sim.device = "cuda:0"
    env = H12VelocityEnv(cfg)
    ref = O.OracleEnv(env._model, env._ccfg, n)
    ref.F[:] = env._fstate.cpu().numpy()
    ref.I[:] = env._istate.cpu().numpy()
    O.set_dz_count(0)
    O.cat_reset()
    obs, _ = env.reset()
    np.testing.assert_allclose(obs["policy"].cpu().numpy(), ref.reset(), rtol=1e-5, atol=2e-5)
    rng = np.random.default_rng(13)
    for t in range(1, 4):
        if task == "cat":
            for name, cid in cfg.constraints.active():
                if name != "contact":
                    ref.cfg.cstr_max_p[cid] = 1.0 / (20 + min((t - 1) / 120000, 1.0) * (4 - 20))
        a = (0.3 * rng.normal(size=(n, 12))).astype(np.float32)
        obs, rew, term, trunc, _ = env.step(torch.from_numpy(a).cuda())
        r_obs, r_rew, r_term, r_trunc, info = ref.step(a, t)
        go = obs["policy"].cpu().numpy()
        ok = (np.abs(go - r_obs) <= 2e-3 * np.maximum(1, np.abs(r_obs))).all(axis=1)
        assert ok.mean() >= 0.97, (t, ok.mean())
        okr = np.abs(rew.cpu().numpy() - r_rew) <= 2e-3 * np.maximum(1, np.abs(r_rew))
        assert okr.mean() >= 0.97, (t, okr.mean())
        if task == "cat":
            assert np.isfinite(term.cpu().numpy()).all()
    env.close()


@pytest.mark.parametrize("task", ["flat", "cat"])
@pytest.mark.parametrize("n", [1, 37, 4096])
def test_episode_log_fold_ragged(gpu, task, n):
    """The episode log (reward sums, reset / time-out / base-contact counts, command metrics and, for CaT, the
    constraint statistics) goes through per-block partial slots folded by the assembly kernel (log_load /
    log_fold; CaT) or, on the fused Flat path, by log_flush_kernel (deferred, h12env_flush_log): compare the step's accumulator with the oracle's on steps with forced time-outs, including grids
    smaller than the number of log values (n = 1, 37)."""
    from h12env._abi import F as FIELDS, LOG_METRIC, NLOG, NREW
    from h12env.cfg import H12CaTEnvCfg

    cfg = H12FlatEnvCfg() if task == "flat" else H12CaTEnvCfg()
    cfg.scene.num_envs = n
    cfg.sim.device = "cuda:0"
    env = H12VelocityEnv(cfg)
    env.reset()
    O.cat_reset()
    O.set_dz_count(0)
    ref = O.OracleEnv(env._model, env._ccfg, n)
    ref.F[:] = env._fstate.cpu().numpy()
    ref.I[:] = env._istate.cpu().numpy()
    ref.obs[:] = env._obs[env._k].cpu().numpy()
    rng = np.random.default_rng(5)
    checked = 0
    for t in range(1, 7):
        if t == 3:  # half of the envs (at least one) time out at step 4
            el = env.episode_length_buf.clone()
            el[: max(1, n // 2)] = int(env.max_episode_length) - 1
            env.episode_length_buf = el
            ref.I[:] = env._istate.cpu().numpy()
        if task == "cat":
            for name, cid in cfg.constraints.active():
                if name != "contact":
                    ref.cfg.cstr_max_p[cid] = 1.0 / (20 + min((t - 1) / 120000, 1.0) * (4 - 20))
        F0, I0 = env._fstate.cpu().numpy().copy(), env._istate.cpu().numpy().copy()
        a = (0.3 * rng.normal(size=(n, 12))).astype(np.float32)
        env.step(torch.from_numpy(a).cuda())
        ref.F[:], ref.I[:] = F0, I0  # teacher-forced: the oracle steps from the GPU's state
        _, _, r_term, r_trunc, info = ref.step(a, t)
        env._flush_log()  # the fused step path defers its fold (h12env_flush_log)
        acc = env._log_ring[env.common_step_counter % len(env._log_ring)].cpu().numpy()
        lo = info["log"]
        if (r_term | r_trunc).any():
            k = list(range(NREW + 3)) + [LOG_METRIC, LOG_METRIC + 1]
            if task == "cat":
                k += list(range(NREW + 4, NREW + 4 + 20))
            np.testing.assert_allclose(acc[k], lo[k], rtol=2e-3, atol=2e-4 * max(1.0, float(np.abs(lo[k]).max())),
                                       err_msg=f"{task} n={n} step {t}")
            assert acc[NREW] == lo[NREW] and acc[NREW] >= 1
            checked += 1
        else:
            assert not acc.any()
    assert checked >= 1
    env.close()
