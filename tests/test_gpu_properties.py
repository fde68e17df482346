"""GPU property tests (hypothesis, derandomised): generated batches of states, actions, observation
buffers and fill masks through the C-ABI against the oracle -- the "randomised states" layer of SURVEY.md
§4.  One env per task is built for the module and re-seeded per example.  Tolerances as in
test_gpu_parity.py: free-flight physics <= 2e-4 of the field scale for every env; contact physics >= 99 % of
envs at 2e-3; observation assembly (noise, history shift, fills, scales) rtol 1e-5."""
import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import oracle as O
from h12env import H12FlatEnvCfg
from h12env._abi import F as FIELDS
from h12env.cfg import H12RslEnvCfg
from h12env.env import H12VelocityEnv
from forced import phys_err, unexplained_envs

pytestmark = pytest.mark.gpu
GPU_PROP = settings(max_examples=8, deadline=None, derandomize=True,
                    suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture])
N = 256


@pytest.fixture(scope="module")
def flat_env():
    cfg = H12FlatEnvCfg()
    cfg.scene.num_envs = N
    cfg.sim.device = "cuda:0"
    env = H12VelocityEnv(cfg)
    env.reset()
    yield env
    env.close()


def write_states(env, ref, rng, height, vel):
    Fm = env._fstate.cpu().numpy().copy()
    put = lambda k, v: Fm.__setitem__(slice(FIELDS[k][0], FIELDS[k][0] + FIELDS[k][1]), v)  # noqa: E731
    put("POS", np.stack([rng.uniform(-1, 1, N), rng.uniform(-1, 1, N), rng.uniform(*height, N)]))
    q = rng.normal(size=(4, N)) * np.array([[4.0], [0.3], [0.3], [1.0]])
    put("QUAT", q / np.linalg.norm(q, axis=0))
    put("VLIN", rng.normal(size=(3, N)) * vel)
    put("WANG", rng.normal(size=(3, N)) * vel)
    put("Q", np.asarray(env._model.q_default)[:, None] + rng.normal(size=(12, N)) * 0.25)
    put("QD", rng.normal(size=(12, N)) * 2 * vel)
    env._fstate.copy_(torch.from_numpy(Fm))
    ref.F[:] = Fm
    ref.I[:] = env._istate.cpu().numpy()


def rel(a, b):
    return np.abs(a - b) / np.maximum(1.0, np.abs(b).max(axis=1, keepdims=True))


@GPU_PROP
@given(seed=st.integers(0, 2 ** 31 - 1), vel=st.floats(0.0, 1.5), spread=st.floats(0.05, 0.6))
def test_free_flight_physics_on_generated_states(gpu, flat_env, seed, vel, spread):
    env = flat_env
    ref = O.OracleEnv(env._model, env._ccfg, N)
    rng = np.random.default_rng(seed)
    write_states(env, ref, rng, (2.5, 3.0), vel)
    q_ref = (np.asarray(env._model.q_default)[None] + rng.normal(size=(N, 12)) * spread).astype(np.float32)
    env.step_physics(torch.from_numpy(q_ref).cuda(), 2)
    ref.step_physics(q_ref, 2)
    g = env._fstate.cpu().numpy()
    for k in ("POS", "QUAT", "VLIN", "WANG", "Q", "QD"):
        o, c = FIELDS[k]
        assert rel(g[o:o + c], ref.F[o:o + c]).max() < 2e-4, k


@GPU_PROP
@given(seed=st.integers(0, 2 ** 31 - 1), low=st.floats(0.94, 1.0))
def test_contact_physics_on_generated_states(gpu, flat_env, seed, low):
    env = flat_env
    ref = O.OracleEnv(env._model, env._ccfg, N)
    rng = np.random.default_rng(seed)
    write_states(env, ref, rng, (low, low + 0.08), 0.3)
    q_ref = (np.asarray(env._model.q_default)[None] + rng.normal(size=(N, 12)) * 0.2).astype(np.float32)
    F0, I0 = ref.F.copy(), ref.I.copy()

    def rerun(Fs):
        ref.F[:], ref.I[:] = Fs, I0
        for _ in range(3):
            ref.step_physics(q_ref, 1)
        return ref.F.copy()

    for _ in range(3):
        env.step_physics(torch.from_numpy(q_ref).cuda(), 1)
    g = env._fstate.cpu().numpy()
    base = rerun(F0)
    assert np.isfinite(g).all()
    gerr = phys_err(g, base)
    bad = unexplained_envs(F0, gerr, 2e-3, rerun, phys_err, base, g, seed=seed)
    assert bad.size == 0, (bad[:10], gerr[bad[:10]])
    assert (gerr > 2e-3).mean() <= 0.01


@GPU_PROP
@given(seed=st.integers(0, 2 ** 31 - 1), p_fill=st.floats(0.0, 1.0), rsl=st.booleans())
def test_observation_assembly_on_generated_buffers(gpu, seed, p_fill, rsl):
    """ObservationManager.compute outside step (h12env_observe): any previous observation buffer, any fill
    mask -> history shift / fill / noise / scale identical to the oracle (450 floats Flat, 270 Rsl)."""
    cfg = H12RslEnvCfg() if rsl else H12FlatEnvCfg()
    cfg.scene.num_envs = 97
    cfg.sim.device = "cuda:0"
    env = H12VelocityEnv(cfg)
    env.reset()
    ref = O.OracleEnv(env._model, env._ccfg, 97)
    ref.F[:] = env._fstate.cpu().numpy()
    ref.I[:] = env._istate.cpu().numpy()
    rng = np.random.default_rng(seed)
    prev = rng.normal(size=(97, env.obs_dim)).astype(np.float32)
    fill = (rng.random(97) < p_fill).astype(np.uint8)
    env._obs[env._k].copy_(torch.from_numpy(prev))
    ref.obs[:] = prev
    got = env.observe(torch.from_numpy(fill)).get("policy").cpu().numpy()
    want = ref.observe(fill)
    np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-6)
    env.close()
