#!/usr/bin/env python3
"""Host-side cost of H12VelocityEnv.step (GPU box): the bench's timed loop is bound by max(GPU time, host time)
per step, so the Python path around the two kernel launches must stay well below the ~40 us GPU step.

    python tools/host_overhead.py [--envs 4096] [--steps 2000]

Prints the wall time per step of (a) env.step with the GPU running (the bench loop), (b) env.step with the
launches queued behind a long-running GPU wait (host time alone: the queue absorbs the launches), and a
cProfile of (b)'s top entries."""
from __future__ import annotations

import argparse
import cProfile
import io
import pstats
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "h1v2-isaac_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=2000)
    a = ap.parse_args()
    import torch

    from h12env import H12FlatEnvCfg
    from h12env.env import H12VelocityEnv

    cfg = H12FlatEnvCfg()
    cfg.scene.num_envs = a.envs
    cfg.sim.device = "cuda:0"
    env = H12VelocityEnv(cfg)
    env.reset()
    acts = torch.randn(64, a.envs, 12, device="cuda:0")
    for i in range(200):
        env.step(acts[i % 64])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        env.step(acts[i % 64])
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / a.steps * 1e6
    # host time alone: block the stream first so every launch of the loop only queues
    n_host = min(a.steps, 100)
    torch.cuda._sleep(int(2e9))  # ~1 s of GPU spin ahead of the launches
    t0 = time.perf_counter()
    for i in range(n_host):
        env.step(acts[i % 64])
    host = (time.perf_counter() - t0) / n_host * 1e6
    torch.cuda.synchronize()
    torch.cuda._sleep(int(2e9))
    pr = cProfile.Profile()
    pr.enable()
    for i in range(n_host):
        env.step(acts[i % 64])
    pr.disable()
    torch.cuda.synchronize()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(12)
    print(f"env.step: {wall:.1f} us per step with the GPU running; host alone {host:.1f} us per step")
    print(s.getvalue())
    env.close()


if __name__ == "__main__":
    main()
