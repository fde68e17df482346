"""CPU: the compact rollout records of BASELINE config C4 (include/h12env.h "Rollout records", h12env.rollout).

* the closed-form row rebuild h12env_rollout_decode evaluates equals a step-by-step CircularBuffer model of the
  observation history (term-major, first push after a reset fills every slot: the semantics tests/golden/
  circular_buffer.npz pins from the reference's own circular_buffer.py), for history 10 (Flat) and 6 (Rsl), with
  resets at every position including the first step and back-to-back resets;
* the chunk-major gathered layout: what the chunked all-gathers produce is read back exactly, for chunk lengths that
  do and do not divide T;
* the library's record layout (256-B aligned sections) -- through the C-ABI, no GPU call.
The HIP decode itself is checked against these on the GPU (tests/test_gpu_rollout.py)."""
import numpy as np
import pytest

from rollout_ref import FRAME, decode_ref, history_model, pack_gathered, step_offset, unpack


@pytest.mark.parametrize("H", [10, 6, 1])
def test_closed_form_rebuild_equals_circular_buffer_model(H):
    rng = np.random.default_rng(H)
    T, N = 24, 9
    frames = rng.normal(size=(T, N, FRAME)).astype(np.float32)
    tail = rng.normal(size=(N, FRAME * H)).astype(np.float32)
    done = (rng.random((T, N)) < 0.15).astype(np.uint8)
    done[0, 0] = 1                  # reset on the first step
    done[5:8, 1] = 1                # back-to-back resets
    done[:, 2] = 0                  # never reset: every row reaches into the tail
    done[T - 1, 3] = 1              # reset on the last step
    np.testing.assert_array_equal(decode_ref(frames, done, tail, H), history_model(frames, done, tail, H))


@pytest.mark.parametrize("T,G,R", [(24, 4, 3), (24, 5, 2), (24, 24, 4), (7, 3, 1)])
def test_gathered_layout_round_trip(T, G, R):
    rng = np.random.default_rng(T * 100 + G)
    n = 5
    off = [0, 1024, 1280, 1536, 1792]   # frames 900 B, actions 240 B, rewards 20 B, flags 5 B each
    S = 2048
    shards = []
    truth = {k: [] for k in ("frames", "actions", "rewards", "terminated", "truncated")}
    for r in range(R):
        rec = np.zeros(T * S, np.uint8)
        f = rng.normal(size=(T, n, FRAME)).astype(np.float32)
        a = rng.normal(size=(T, n, 12)).astype(np.float32)
        w = rng.normal(size=(T, n)).astype(np.float32)
        te = (rng.random((T, n)) < 0.3).astype(np.uint8)
        tr = (rng.random((T, n)) < 0.3).astype(np.uint8)
        for s in range(T):
            b = s * S
            rec[b + off[0]:b + off[0] + 4 * n * FRAME] = f[s].view(np.uint8).reshape(-1)
            rec[b + off[1]:b + off[1] + 4 * n * 12] = a[s].view(np.uint8).reshape(-1)
            rec[b + off[2]:b + off[2] + 4 * n] = w[s].view(np.uint8)
            rec[b + off[3]:b + off[3] + n] = te[s]
            rec[b + off[4]:b + off[4] + n] = tr[s]
        shards.append(rec)
        for k, v in zip(truth, (f, a, w, te, tr)):
            truth[k].append(v)
    g = pack_gathered(shards, T, G, S)
    got = unpack(g, R, n, T, G, off, S)
    for k in truth:
        np.testing.assert_array_equal(got[k], np.concatenate(truth[k], axis=1), err_msg=k)
    # every step record of every shard has its own place
    offs = sorted(step_offset(r, s, R, T, G, S) for r in range(R) for s in range(T))
    assert offs == [i * S for i in range(R * T)]


def test_library_record_layout():
    from h12env.rollout import record_layout

    for n in (1, 37, 4096):
        off, S = record_layout(n)
        assert all(o % 256 == 0 for o in off) and S % 256 == 0
        assert off[1] >= 4 * n * FRAME and off[2] >= off[1] + 4 * n * 12 and off[3] >= off[2] + 4 * n
        assert off[4] >= off[3] + n and S >= off[4] + n
        assert S < 4 * n * FRAME + 4 * n * 12 + 6 * n + 5 * 256  # compact: ~238 B per env-step
