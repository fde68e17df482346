"""Compact rollout records and their all-gather (BASELINE config C4: "RCCL all-gather of rollout buffer over xGMI").

rsl_rl's RolloutStorage (rsl-rl-lib 2.3.3) keeps per iteration (T, N, 450) observations, T = num_steps_per_env = 24
(C12/agents/rsl_rl_ppo_cfg.py:12).  A 450-float row is 10 frames of 45 floats (CircularBuffer, term-major,
T/utils/history/circular_buffer.py:79-170), nine of which the previous row already holds.  So a shard records, per
env-step, only the new frame exactly as it enters the history (h12env_step_out.frame_out: noise and term scales
applied), the action, the reward and the two done flags -- 238 B instead of 1856 B -- the shards' records are
all-gathered in chunks of G steps on a side stream while the env keeps stepping, and every rank rebuilds the full
(T, N_global, 450) rows with ``h12env_rollout_decode`` (HIP), bit-identical to the rows the envs returned.

Layouts are the C library's (include/h12env.h, h12env_rollout_layout): a step record of one shard is
frames f32 [n][45] | actions f32 [n][12] | rewards f32 [n] | terminated u8 [n] | truncated u8 [n] (256-B aligned
sections); a shard's rollout is T step records back to back; the gathered buffer is chunk-major, then shard, then
step.
"""
from __future__ import annotations

import ctypes as C
import time

import torch

from . import distributed as Dist
from ._abi import NJ, OBS_FRAME, check, load_library


def record_layout(n: int):
    """(section byte offsets [5], step record bytes) of a shard of n envs."""
    lib = load_library()
    off = (C.c_size_t * 5)()
    sb = C.c_size_t()
    check(lib, lib.h12env_rollout_layout(int(n), off, C.byref(sb)), "h12env_rollout_layout")
    return [int(x) for x in off], int(sb.value)


class RolloutRecorder:
    """Device-resident compact rollout of one shard: T step records of n envs (one uint8 buffer).

    ``H12VelocityEnv.bind_rollout(rec)`` makes every env.step write its reward, done flags and new observation frame
    straight into step record ``rec.t`` (no extra copies) and advance the cursor; the caller writes the actions
    (``rec.actions[t]``), as a PPO runner stores its own actions."""

    def __init__(self, num_envs: int, T: int, device, history: int):
        self.n, self.T, self.history = int(num_envs), int(T), int(history)
        self.off, self.step_bytes = record_layout(self.n)
        self.record = torch.zeros(self.T * self.step_bytes, dtype=torch.uint8, device=device)
        steps = self.record.view(self.T, self.step_bytes)
        n, o = self.n, self.off

        def sec(i, count, dtype, shape):
            nb = count * torch.tensor([], dtype=dtype).element_size()
            return steps[:, o[i]:o[i] + nb].view(dtype).view(self.T, *shape)

        self.frames = sec(0, n * OBS_FRAME, torch.float32, (n, OBS_FRAME))
        self.actions = sec(1, n * NJ, torch.float32, (n, NJ))
        self.rewards = sec(2, n, torch.float32, (n,))
        self.terminated = sec(3, n, torch.bool, (n,))
        self.truncated = sec(4, n, torch.bool, (n,))
        self.t = 0  # next step record env.step writes

    def chunk_bytes(self, t0: int, t1: int) -> torch.Tensor:
        """The shard's records of steps [t0, t1) (contiguous)."""
        return self.record[t0 * self.step_bytes:t1 * self.step_bytes]


def decode(records: torch.Tensor, n_shards: int, n: int, T: int, G: int, history: int, t0: int, t1: int,
           tail: torch.Tensor, obs_out: torch.Tensor, stream=None) -> None:
    """Observation rows [t0, t1) of the gathered records (h12env_rollout_decode) into obs_out (T, n_shards*n, 45H);
    tail (n_shards*n, 45H): the rows before step 0 (may be obs_out[T - 1])."""
    row = OBS_FRAME * history
    ng = n_shards * n
    if obs_out.shape != (T, ng, row) or tail.shape != (ng, row) or obs_out.dtype != torch.float32 \
            or not obs_out.is_contiguous() or not tail.is_contiguous():
        raise ValueError(f"obs_out must be ({T}, {ng}, {row}) and tail ({ng}, {row}), contiguous fp32")
    lib = load_library()
    s = stream if stream is not None else torch.cuda.current_stream(obs_out.device)
    rc = lib.h12env_rollout_decode(records.data_ptr(), n_shards, n, T, G, history, t0, t1, tail.data_ptr(),
                                   obs_out.data_ptr(), s.cuda_stream)
    if rc:
        check(lib, rc, "h12env_rollout_decode")


class StreamFence:
    """Counters in signal memory ordering two streams without HIP events (h12env_fence_*): ``signal`` enqueues
    counter[slot] = value behind the stream's earlier work, ``wait`` holds the stream's later work until
    counter[slot] >= value."""

    def __init__(self, device, n_slots: int):
        self._lib = load_library()
        h = C.c_void_p()
        dev = torch.device(device)
        check(self._lib, self._lib.h12env_fence_create(dev.index or 0, n_slots, C.byref(h)), "h12env_fence_create")
        self._h = h

    def signal(self, slot: int, value: int, stream) -> None:
        rc = self._lib.h12env_fence_signal(self._h, slot, value, stream.cuda_stream)
        if rc:
            check(self._lib, rc, "h12env_fence_signal")

    def wait(self, slot: int, value: int, stream) -> None:
        rc = self._lib.h12env_fence_wait(self._h, slot, value, stream.cuda_stream)
        if rc:
            check(self._lib, rc, "h12env_fence_wait")

    def __del__(self):
        try:
            if self._h:
                self._lib.h12env_fence_destroy(self._h)
                self._h = None
        except Exception:
            pass


class RolloutGather:
    """Chunked all-gather of the shards' rollout records on a side stream, each chunk decoded into the global
    (T, N_global, 45H) observation rows right after it arrives -- while the env keeps stepping on its own stream.

    Per chunk of G steps: the compute stream records an event after the chunk's last step; the comm stream waits
    on it, all-gathers the chunk's bytes of every shard (one ``all_gather_into_tensor``) and decodes the chunk's
    rows.  Before the env writes a step record of the next iteration, the compute stream waits for the gather of
    that chunk (``before_step``), so the records are double-use safe with one buffer.  world == 1: the gather is a
    device copy (same code path, no collective)."""

    def __init__(self, rec: RolloutRecorder, world: int, G: int, tail: torch.Tensor, timing: bool = False,
                 sync: str = "fence", decode: bool = True):
        self.rec, self.world, self.G = rec, int(world), max(1, min(int(G), rec.T))
        dev = rec.record.device
        self.gathered = torch.empty(self.world * rec.record.numel(), dtype=torch.uint8, device=dev)
        ng, row = self.world * rec.n, OBS_FRAME * rec.history
        self.obs = torch.empty(rec.T, ng, row, device=dev)  # the decoded rollout rows handed to PPO
        if tail.shape != (ng, row):
            raise ValueError(f"tail must be ({ng}, {row})")
        self.tail = tail.contiguous().clone()   # rows before step 0 of the first iteration (all envs)
        self.comm = torch.cuda.Stream(device=dev)
        self.compute = torch.cuda.current_stream(dev)  # the stream the env steps on
        nchunks = (rec.T + self.G - 1) // self.G
        self.done_ev = [None] * nchunks          # per chunk: gathered (the records may be rewritten)
        self._ev = [(torch.cuda.Event(), torch.cuda.Event()) for _ in range(nchunks)]  # (ready, done), reused
        self._last_row = self.obs[rec.T - 1]     # the next iteration's tail
        self.prof = None                         # diagnostics: host seconds per _launch segment (dict)
        # stream ordering: "fence" (signal-memory counters: slot 0 = chunks recorded, slot 1 = chunks gathered) or
        # "event" (HIP events; ~100 us of host time per hand-off on this stack, tools/stream_diag.py)
        self.sync = sync
        self.fence = StreamFence(dev, 2) if sync == "fence" else None
        self.seq = 0                              # chunks launched so far
        self.chunk_seq = [0] * nchunks            # per chunk index: sequence number of its last gather
        self.timing = timing
        self.times: list[tuple] = []             # (chunk bytes, gather event pair, decode event pair)
        self.iterations = 0
        # decode=False: the gathered records are the product (a PPO learner rebuilds the rows of each minibatch it
        # draws; the full (T, N_global, 45H) rebuild is then never needed)
        self.decode_off = not decode

    def chunk_of(self, t: int) -> tuple[int, int, int]:
        c = t // self.G
        return c, c * self.G, min((c + 1) * self.G, self.rec.T)

    def before_step(self):
        """Call before env.step: the step record about to be written must have left in the previous gather."""
        t = self.rec.t
        c, t0, _ = self.chunk_of(t)
        if t != t0:
            return
        if self.fence is not None:
            if self.chunk_seq[c]:
                self.fence.wait(1, self.chunk_seq[c], self.compute)
        elif self.done_ev[c] is not None:
            self.compute.wait_event(self.done_ev[c])

    def after_step(self, t: int, actions=None):
        """Call after env.step wrote step record t: at a chunk's end, gather and decode it on the comm stream.
        actions: optional callable (t0, t1) -> None that writes the chunk's actions into rec.actions[t0:t1] (on the
        compute stream, before the gather)."""
        c, t0, t1 = self.chunk_of(t)
        if t + 1 != t1:
            return
        self._launch(c, t0, t1, self.rec.T, actions)
        if t1 == self.rec.T:
            self.iterations += 1

    def flush(self, t_end: int, actions=None):
        """Gather and decode the records of an unfinished chunk [chunk start, t_end) (end of a measurement window):
        decoded as a rollout of t_end steps (rows [0, t_end) of self.obs)."""
        if t_end <= 0:
            return
        c, t0, t1 = self.chunk_of(t_end - 1)
        if t_end == t1:
            return  # the chunk was complete (after_step gathered it)
        self._launch(c, t0, t_end, t_end, actions)

    def _launch(self, c: int, t0: int, t1: int, T_eff: int, actions):
        rec = self.rec
        prof = self.prof
        if prof is not None:
            p0 = time.perf_counter()
        if actions is not None:
            actions(t0, t1)
        self.seq += 1
        seq = self.seq
        ready, done = self._ev[c]
        if self.fence is not None:
            self.fence.signal(0, seq, self.compute)
            self.fence.wait(0, seq, self.comm)
        else:
            ready.record(self.compute)
            self.comm.wait_event(ready)
        if prof is not None:
            p1 = time.perf_counter()
        gc = t1 - t0
        S = rec.step_bytes
        out = self.gathered[t0 * self.world * S:(t0 + gc) * self.world * S]
        src = rec.record[t0 * S:t1 * S]
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)] if self.timing else None
        with torch.cuda.stream(self.comm):
            if ev:
                ev[0].record(self.comm)
            if self.world > 1:
                Dist.all_gather_into_tensor(out, src)
            else:
                out.copy_(src)
            if ev:
                ev[1].record(self.comm)
            if self.fence is not None:  # the records of this chunk may be rewritten from here on
                self.fence.signal(1, seq, self.comm)
                self.chunk_seq[c] = seq
            if prof is not None:
                p2 = time.perf_counter()
            tail = self.tail if self.iterations == 0 else self._last_row
            if not self.decode_off:
                decode(self.gathered, self.world, rec.n, T_eff, self.G, rec.history, t0, t1, tail,
                       self.obs if T_eff == rec.T else self.obs[:T_eff], stream=self.comm)
            if ev:
                ev[2].record(self.comm)
                self.times.append((out.numel(), ev))
            if self.fence is None:
                done.record(self.comm)
        if self.fence is None:
            self.done_ev[c] = done
        if prof is not None:
            p3 = time.perf_counter()
            for k, v in (("actions+events", p1 - p0), ("gather", p2 - p1), ("decode+done", p3 - p2)):
                prof[k] = prof.get(k, 0.0) + v
            prof["chunks"] = prof.get("chunks", 0) + 1

    def wait(self):
        torch.cuda.current_stream(self.rec.record.device).wait_stream(self.comm)

    def stats(self) -> dict:
        """Summed gather / decode milliseconds and gathered bytes of the timed chunks (synchronises)."""
        torch.cuda.synchronize(self.rec.record.device)
        g = d = 0.0
        nbytes = 0
        for b, ev in self.times:
            g += ev[0].elapsed_time(ev[1])
            d += ev[1].elapsed_time(ev[2])
            nbytes += b
        out = {"chunks": len(self.times), "gather_ms": g, "decode_ms": d, "gathered_bytes": nbytes}
        self.times = []
        return out
