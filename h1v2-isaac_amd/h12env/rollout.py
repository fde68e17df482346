"""Compact rollout records and their all-gather (BASELINE config C4: "RCCL all-gather of rollout buffer over xGMI").

rsl_rl's RolloutStorage (rsl-rl-lib 2.3.3) keeps per iteration (T, N, 450) observations, T = num_steps_per_env = 24
(C12/agents/rsl_rl_ppo_cfg.py:12).  A 450-float row is 10 frames of 45 floats (CircularBuffer, term-major,
T/utils/history/circular_buffer.py:79-170), nine of which the previous row already holds.  So a shard records, per
env-step, only the new frame exactly as it enters the history (h12env_step_out.frame_out: noise and term scales
applied), the action, the reward and the two done flags -- 234 B instead of 1856 B -- the shards' records are
all-gathered (one RCCL collective per rollout by default, asynchronous on RCCL's stream) while the env steps the next
rollout into the other half of a ring of 2T records, and every rank can rebuild the full (T, N_global, 450) rows
with ``h12env_rollout_decode`` (HIP), bit-identical to the rows the envs returned.

Layouts are the C library's (include/h12env.h, h12env_rollout_layout): a step record of one shard is
frames f32 [n][45] | actions f32 [n][12] | rewards f32 [n] | terminated u8 [n] | truncated u8 [n] (256-B aligned
sections); a shard's rollout is T step records back to back; the gathered buffer is chunk-major, then shard, then
step.
"""
from __future__ import annotations

import ctypes as C

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
    """Device-resident compact rollout of one shard: a ring of nbuf x T step records of n envs (one uint8 buffer).

    ``H12VelocityEnv.bind_rollout(rec)`` makes every env.step write its reward, done flags and new observation frame
    straight into ring slot ``rec.t`` (no extra copies) and advance the cursor (mod nbuf T); the caller writes the
    actions (``rec.actions[slot]``), as a PPO runner stores its own actions.  Rollout k occupies slots
    [(k mod nbuf) T, (k mod nbuf + 1) T): with nbuf = 2 the all-gather of one rollout has the whole next rollout to
    complete before its records are rewritten."""

    def __init__(self, num_envs: int, T: int, device, history: int, nbuf: int = 2):
        self.n, self.T, self.history, self.nbuf = int(num_envs), int(T), int(history), int(nbuf)
        self.slots = self.nbuf * self.T
        self.off, self.step_bytes = record_layout(self.n)
        self.record = torch.zeros(self.slots * self.step_bytes, dtype=torch.uint8, device=device)
        steps = self.record.view(self.slots, self.step_bytes)
        n, o = self.n, self.off

        def sec(i, count, dtype, shape):
            nb = count * torch.tensor([], dtype=dtype).element_size()
            return steps[:, o[i]:o[i] + nb].view(dtype).view(self.slots, *shape)

        self.frames = sec(0, n * OBS_FRAME, torch.float32, (n, OBS_FRAME))
        self.actions = sec(1, n * NJ, torch.float32, (n, NJ))
        self.rewards = sec(2, n, torch.float32, (n,))
        self.terminated = sec(3, n, torch.bool, (n,))
        self.truncated = sec(4, n, torch.bool, (n,))
        self.t = 0  # next ring slot env.step writes

    def chunk_bytes(self, s0: int, s1: int) -> torch.Tensor:
        """The shard's records of ring slots [s0, s1) (contiguous)."""
        return self.record[s0 * self.step_bytes:s1 * self.step_bytes]

    def rollout_bytes(self, buf: int) -> torch.Tensor:
        """The records of the rollout in ring half ``buf`` (T step records)."""
        return self.chunk_bytes(buf * self.T, (buf + 1) * self.T)


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
    """All-gather of the shards' rollout records, one collective per chunk of G steps (default G = T: one per
    rollout), issued asynchronously on RCCL's own stream right after the chunk's last step, so it runs while the env
    steps the next chunk into the other half of the recorder's ring; optionally every chunk's global
    (T, N_global, 45H) observation rows are rebuilt right after it arrives (``h12env_rollout_decode``).  The rebuild
    is SERIALISED with the env: it runs on the compute stream after ``work.wait()``, so with decode on the compute
    stream waits for every chunk's gather at once and the gather does not overlap the next steps (a side stream
    ordered by events cost ~95 us of host time per hand-off on this stack); bench figures
    taken with --rollout-decode are serialised figures.  Decode off (the default) keeps the overlap.

    Ordering uses the collectives' own stream semantics (torch.distributed Work): before the env rewrites a ring
    chunk, ``before_step`` makes the compute stream wait for that chunk's previous gather (``work.wait()``, a device-side
    wait; with the 2T ring it completed a whole rollout earlier).  world == 1: nothing to gather -- the records are
    read in place."""

    def __init__(self, rec: RolloutRecorder, world: int, G: int | None = None, tail: torch.Tensor | None = None,
                 timing: bool = False, decode: bool = True, collective: bool = False):
        self.rec, self.world = rec, int(world)
        # collective: issue the all-gather even at world 1 (a one-rank process group; exercises the RCCL path)
        self.coll = self.world > 1 or collective
        self.G = max(1, min(int(G or rec.T), rec.T))
        dev = rec.record.device
        S = rec.step_bytes
        self.gathered = (torch.empty(rec.nbuf * self.world * rec.T * S, dtype=torch.uint8, device=dev)
                         if self.coll else None)
        ng, row = self.world * rec.n, OBS_FRAME * rec.history
        self.obs = torch.empty(rec.T, ng, row, device=dev)  # the rebuilt rows of the latest rollout
        if tail is None or tail.shape != (ng, row):
            raise ValueError(f"tail must be ({ng}, {row})")
        self.tail = tail.contiguous().clone()   # rows before step 0 of the first rollout (all envs)
        self._last_row = self.obs[rec.T - 1]     # the next rollout's tail
        self._work = {}                          # (ring half, chunk) -> outstanding collective
        self.timing = timing
        self.times: list[tuple] = []             # (gathered bytes, (start, gathered, decoded) events)
        self.iterations = 0
        self.seq = 0                             # chunks launched so far
        # decode=False: the gathered records are the product (a PPO learner rebuilds the rows of each minibatch it
        # draws; the full (T, N_global, 45H) rebuild is then never needed)
        self.decode_off = not decode

    def chunk_of(self, t: int) -> tuple[int, int, int]:
        """(chunk, first step, end step) of rollout step t."""
        c = t // self.G
        return c, c * self.G, min((c + 1) * self.G, self.rec.T)

    def records(self, buf: int) -> torch.Tensor:
        """Every shard's records of the rollout in ring half ``buf``, chunk-major / shard / step."""
        if not self.coll:
            return self.rec.rollout_bytes(buf)
        n = self.world * self.rec.T * self.rec.step_bytes
        return self.gathered[buf * n:(buf + 1) * n]

    def before_step(self):
        """Call before env.step: a chunk's ring slots are rewritten only after their previous gather."""
        buf, t = divmod(self.rec.t, self.rec.T)
        c, t0, _ = self.chunk_of(t)
        if t == t0:
            w = self._work.pop((buf, c), None)
            if w is not None:
                w.wait()

    def after_step(self, slot: int, actions=None):
        """Call after env.step wrote ring slot ``slot``: at a chunk's end, gather it (and rebuild its rows).
        actions: optional callable (s0, s1) -> None writing the chunk's actions into rec.actions[s0:s1] first."""
        buf, t = divmod(slot, self.rec.T)
        c, t0, t1 = self.chunk_of(t)
        if t + 1 != t1:
            return
        self._launch(buf, c, t0, t1, self.rec.T, actions)
        if t1 == self.rec.T:
            self.iterations += 1

    def flush(self, slot_end: int, actions=None):
        """Gather (and rebuild) an unfinished chunk ending before ring slot ``slot_end`` (the cursor after the last
        step of a measurement window), as a rollout of that many steps."""
        s = (slot_end - 1) % self.rec.slots
        buf, t = divmod(s, self.rec.T)
        c, t0, t1 = self.chunk_of(t)
        if t + 1 == t1:
            return  # the chunk was complete (after_step gathered it)
        self._launch(buf, c, t0, t + 1, t + 1, actions)

    def _launch(self, buf: int, c: int, t0: int, t1: int, T_eff: int, actions):
        rec = self.rec
        T, S = rec.T, rec.step_bytes
        if actions is not None:
            actions(buf * T + t0, buf * T + t1)
        self.seq += 1
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)] if self.timing else None
        if ev:
            ev[0].record()
        work = None
        nbytes = (t1 - t0) * S
        if self.coll:
            base = buf * self.world * T * S
            out = self.gathered[base + t0 * self.world * S:base + t1 * self.world * S]
            work = Dist.all_gather_into_tensor(out, rec.chunk_bytes(buf * T + t0, buf * T + t1), async_op=True)
            nbytes *= self.world
        if ev:  # timing pass: the compute stream waits for the gather so that the event pair brackets it
            if work is not None:
                work.wait()
                work = None
            ev[1].record()
        if not self.decode_off:
            if work is not None:
                work.wait()
                work = None
            tail = self.tail if self.iterations == 0 else self._last_row
            decode(self.records(buf), self.world, rec.n, T_eff, self.G, rec.history, t0, t1, tail,
                   self.obs if T_eff == T else self.obs[:T_eff])
        if ev:
            ev[2].record()
            self.times.append((nbytes, ev))
        if work is not None:
            self._work[(buf, c)] = work

    def wait(self):
        """The compute stream waits for every outstanding gather."""
        for w in self._work.values():
            w.wait()
        self._work.clear()

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
