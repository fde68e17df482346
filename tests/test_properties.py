"""CPU property tests (hypothesis, derandomised so every run checks the same examples): the oracle's dynamics
invariants over generated states, the history / delay-buffer semantics against small pure-Python models of
CircularBuffer (circular_buffer.py:84-170), Philox4x32-10 against a pure-Python restatement of the published
algorithm (Salmon et al., SC'11), and the cfg -> kernel reward-table mapping.  SURVEY.md §4 lists
"randomised states (hypothesis)" as the pin for the layers the reference does not test."""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import oracle as O
from h12env import H12FlatEnvCfg
from h12env._abi import NHIST, NREW, REWARD_FUNCS
from h12env.cfg import RewardsCfg, RewTerm

PROP = settings(max_examples=40, deadline=None, derandomize=True,
                suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture])
f64 = st.floats(-1.0, 1.0, allow_nan=False, allow_infinity=False)


@st.composite
def states(draw, height=(1.5, 3.0)):
    s = np.zeros(37)
    s[0:2] = draw(st.tuples(f64, f64))
    s[2] = draw(st.floats(*height))
    q = np.array(draw(st.tuples(f64, f64, f64, f64))) + np.array([1.5, 0, 0, 0])
    s[3:7] = q / np.linalg.norm(q)
    s[7:13] = np.array(draw(st.lists(f64, min_size=6, max_size=6))) * 2
    s[13:25] = np.array(draw(st.lists(f64, min_size=12, max_size=12))) * 0.6
    s[25:37] = np.array(draw(st.lists(f64, min_size=12, max_size=12))) * 3
    return s


@PROP
@given(s=states(), tau=st.lists(st.floats(-40, 40), min_size=12, max_size=12))
def test_aba_equals_crba_on_generated_states(model, s, tau):
    c = H12FlatEnvCfg().to_c()
    tau = np.array(tau)
    a, _ = O.forward_dynamics(model, c, s, tau, algo=0, contact=False)
    b, _ = O.forward_dynamics(model, c, s, tau, algo=1, contact=False)
    np.testing.assert_allclose(a, b, rtol=1e-8, atol=1e-8 * max(1.0, np.abs(a).max()))


@PROP
@given(s=states())
def test_mass_matrix_symmetric_positive_definite(model, s):
    M = O.mass_matrix(model, s)
    np.testing.assert_allclose(M, M.T, atol=1e-10)
    assert np.linalg.eigvalsh(M).min() > 0


def python_history(frames, fills, d, nh=NHIST):
    """CircularBuffer(max_len=nh) per term: the first push after a reset fills every slot, later pushes shift
    (oldest first)."""
    buf = None
    out = []
    for f, fill in zip(frames, fills):
        if buf is None or fill:
            buf = [f.copy() for _ in range(nh)]
        else:
            buf = buf[1:] + [f.copy()]
        out.append(np.stack(buf))
    return out


@PROP
@given(n=st.integers(1, 25), seed=st.integers(0, 2 ** 31 - 1), p_fill=st.floats(0.0, 0.5))
def test_history_write_equals_circular_buffer_model(n, seed, p_fill):
    rng = np.random.default_rng(seed)
    frames = [rng.normal(size=45) for _ in range(n)]
    fills = [True] + list(rng.random(n - 1) < p_fill)
    row = np.zeros(450, np.float32)
    blocks = [(0, 3), (3, 3), (6, 3), (9, 12), (21, 12), (33, 12)]
    models = [python_history([f[o:o + d].astype(np.float32) for f in frames], fills, d) for o, d in blocks]
    for t in range(n):
        row = O.history_write(frames[t], row, fills[t])
        off = 0
        for (o, d), m in zip(blocks, models):
            np.testing.assert_array_equal(row[off:off + NHIST * d].reshape(NHIST, d), m[t])
            off += NHIST * d


@PROP
@given(lag=st.integers(0, 5), since=st.integers(0, 2), dec=st.integers(3, 8))
def test_delay_source_equals_delay_buffer_model(lag, since, dec):
    """DelayBuffer: one push per physics step of the env step's held target; read at lag clamped to
    pushes - 1 (the first push after a reset fills the ring).  Source 0 = a_t, 1 = a_{t-1}, 2 = a_{t-2}."""
    for sub in range(dec):
        history = []  # env-step index of each push, newest last
        steps = since + 1
        for k in range(steps):
            n_sub = dec if k < steps - 1 else sub + 1
            history += [k] * n_sub
        if since < 2:
            pushes = len(history)
        else:
            pushes = 2 * dec + sub + 1
            history = [0] * (pushes - len(history)) + history
        L = min(lag, pushes - 1)
        src_step = history[-1 - L]
        want = (steps - 1) - src_step
        if lag > 2 * dec:
            continue
        assert O.delay_source(lag, since, sub, dec) == min(want, 2), (lag, since, sub, dec)


def philox_py(seed, c0, c1, c2, c3):
    M0, M1, W0, W1 = 0xD2511F53, 0xCD9E8D57, 0x9E3779B9, 0xBB67AE85
    k0, k1 = seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF
    c = [c0, c1, c2, c3]
    for _ in range(10):
        p0, p1 = M0 * c[0], M1 * c[2]
        c = [((p1 >> 32) ^ c[1] ^ k0) & 0xFFFFFFFF, p1 & 0xFFFFFFFF,
             ((p0 >> 32) ^ c[3] ^ k1) & 0xFFFFFFFF, p0 & 0xFFFFFFFF]
        k0, k1 = (k0 + W0) & 0xFFFFFFFF, (k1 + W1) & 0xFFFFFFFF
    return c


@PROP
@given(seed=st.integers(0, 2 ** 64 - 1), ctr=st.tuples(*[st.integers(0, 2 ** 32 - 1)] * 4))
def test_philox_equals_published_algorithm(seed, ctr):
    assert O.philox(seed, *ctr) == philox_py(seed, *ctr)


@PROP
@given(data=st.data())
def test_reward_table_mapping(data):
    """Any subset of kernel terms under any names and weights lands on its kernel ids; cfg order is the log order."""
    ids = data.draw(st.lists(st.integers(0, NREW - 1), unique=True, min_size=1, max_size=NREW))
    weights = data.draw(st.lists(st.floats(-5, 5, allow_nan=False).filter(lambda w: w != 0), min_size=len(ids),
                                 max_size=len(ids)))
    cfg = H12FlatEnvCfg()
    cfg.rewards = RewardsCfg({f"term_{i}": RewTerm(w, {}, REWARD_FUNCS[k]) for i, (k, w) in enumerate(zip(ids, weights))})
    c = cfg.to_c()
    w = np.array(c.rew_w)
    for k, wt in zip(ids, weights):
        assert w[k] == pytest.approx(wt, rel=1e-6)
    assert (w[[k for k in range(NREW) if k not in ids]] == 0).all()
    assert [k for _, (k,) in cfg.rewards.active()] == ids
