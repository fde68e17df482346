"""Test infrastructure for the compact rollout records (h12env.rollout, include/h12env.h "Rollout records"): numpy
restatements of the gathered-buffer layout and of the row rebuild, and a step-by-step CircularBuffer model of the
observation history (T/utils/history/circular_buffer.py:79-170 semantics, the same the oracle's history write is
pinned to by tests/golden/circular_buffer.npz: term-major rows, oldest slot first, the first push after a reset fills
every slot)."""
from __future__ import annotations

import numpy as np

FRAME = 45
TERM_DIMS = (3, 3, 3, 12, 12, 12)  # ang_vel, gravity, command, q - q0, qd, action


def chunk_len(c: int, T: int, G: int) -> int:
    return min(G, T - c * G)


def step_offset(r: int, s: int, n_shards: int, T: int, G: int, step_bytes: int) -> int:
    """Byte offset of shard r's step record s in the gathered buffer (chunk-major, then shard, then step)."""
    c = s // G
    return (c * G * n_shards + r * chunk_len(c, T, G) + (s - c * G)) * step_bytes


def pack_gathered(shard_records: list[np.ndarray], T: int, G: int, step_bytes: int) -> np.ndarray:
    """What the chunked all_gather_into_tensor calls produce from the shards' (T * step_bytes) uint8 records."""
    R = len(shard_records)
    out = np.zeros(R * T * step_bytes, np.uint8)
    for c in range((T + G - 1) // G):
        t0, gc = c * G, chunk_len(c, T, G)
        for r in range(R):
            a = step_offset(r, t0, R, T, G, step_bytes)
            out[a:a + gc * step_bytes] = shard_records[r][t0 * step_bytes:(t0 + gc) * step_bytes]
    return out


def unpack(gathered: np.ndarray, n_shards: int, n: int, T: int, G: int, off: list[int], step_bytes: int) -> dict:
    """Global (T, n_shards * n, ...) arrays of every section of the gathered records."""
    out = {"frames": np.zeros((T, n_shards * n, FRAME), np.float32), "actions": np.zeros((T, n_shards * n, 12), np.float32),
           "rewards": np.zeros((T, n_shards * n), np.float32), "terminated": np.zeros((T, n_shards * n), np.uint8),
           "truncated": np.zeros((T, n_shards * n), np.uint8)}
    for r in range(n_shards):
        for s in range(T):
            b = step_offset(r, s, n_shards, T, G, step_bytes)
            rec = gathered[b:b + step_bytes]
            g = slice(r * n, (r + 1) * n)
            out["frames"][s, g] = rec[off[0]:off[0] + 4 * n * FRAME].view(np.float32).reshape(n, FRAME)
            out["actions"][s, g] = rec[off[1]:off[1] + 4 * n * 12].view(np.float32).reshape(n, 12)
            out["rewards"][s, g] = rec[off[2]:off[2] + 4 * n].view(np.float32)
            out["terminated"][s, g] = rec[off[3]:off[3] + n]
            out["truncated"][s, g] = rec[off[4]:off[4] + n]
    return out


def _col_maps(H: int):
    """Per row column: frame component c, term width d, slot h (0 oldest)."""
    comp, width, slot = [], [], []
    c0 = 0
    for d in TERM_DIMS:
        for h in range(H):
            for k in range(d):
                comp.append(c0 + k)
                width.append(d)
                slot.append(h)
        c0 += d
    return np.array(comp), np.array(width), np.array(slot)


def decode_ref(frames: np.ndarray, done: np.ndarray, tail: np.ndarray, H: int) -> np.ndarray:
    """(T, N, 45H) rows from frames (T, N, 45), done (T, N) and the rows before step 0 (N, 45H): the closed form
    h12env_rollout_decode evaluates (slot h of row t = frame max(t - (H - 1 - h), last done <= t), else the tail's
    slot h + t + 1)."""
    T, N, _ = frames.shape
    comp, width, slot = _col_maps(H)
    cols = np.arange(FRAME * H)
    last = np.full((T, N), -1)
    cur = np.full(N, -1)
    for t in range(T):
        cur = np.where(done[t] != 0, t, cur)
        last[t] = cur
    out = np.zeros((T, N, FRAME * H), np.float32)
    for t in range(T):
        src = t - (H - 1 - slot)[None, :]                      # (1, C)
        src = np.maximum(src, last[t][:, None])                # (N, C)
        from_frame = src >= 0
        fr = frames[np.clip(src, 0, T - 1), np.arange(N)[:, None], comp[None, :]]
        tl = tail[np.arange(N)[:, None], np.clip(cols + (t + 1) * width, 0, FRAME * H - 1)[None, :]]
        out[t] = np.where(from_frame, fr, tl)
    return out


def history_model(frames: np.ndarray, done: np.ndarray, tail: np.ndarray, H: int) -> np.ndarray:
    """The same rows by pushing frames through a per-env CircularBuffer (term-major flattening), step by step."""
    T, N, _ = frames.shape
    bounds = np.cumsum((0,) + TERM_DIMS)
    hist = []  # per env: list of H frames, oldest first, rebuilt from the tail row
    for e in range(N):
        fr = np.zeros((H, FRAME), np.float32)
        col = 0
        for j, d in enumerate(TERM_DIMS):
            fr[:, bounds[j]:bounds[j + 1]] = tail[e, col:col + H * d].reshape(H, d)
            col += H * d
        hist.append([fr[h] for h in range(H)])
    out = np.zeros((T, N, FRAME * H), np.float32)
    for t in range(T):
        for e in range(N):
            f = frames[t, e]
            hist[e] = [f] * H if done[t, e] else hist[e][1:] + [f]
            b = np.stack(hist[e])
            out[t, e] = np.concatenate([b[:, bounds[j]:bounds[j + 1]].reshape(-1) for j in range(len(TERM_DIMS))])
    return out
