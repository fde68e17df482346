#!/usr/bin/env python3
"""Diagnostic (GPU box): the price of a side stream beside the env step loop.  Every G steps the loop records an
event on the compute stream and does progressively more with it on a second stream; printed: wall ms per step
(after a final sync) and host us per G-step chunk of the side-stream calls.

    python tools/stream_diag.py [--envs 4096] [--steps 240] [--every 4]"""
import argparse
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "h1v2-isaac_amd"))

import torch  # noqa: E402

from h12env import H12FlatEnvCfg  # noqa: E402
from h12env.env import H12VelocityEnv  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=240)
    ap.add_argument("--every", type=int, default=4)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    cfg = H12FlatEnvCfg()
    cfg.scene.num_envs = a.envs
    cfg.sim.device = str(dev)
    env = H12VelocityEnv(cfg)
    env.reset()
    acts = torch.randn(64, a.envs, 12, device=dev)
    for i in range(100):
        env.step(acts[i % 64])
    torch.cuda.synchronize()
    comp = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(device=dev)
    side_hi = torch.cuda.Stream(device=dev, priority=-1)
    src = torch.zeros(4 << 20, dtype=torch.uint8, device=dev)
    dst = torch.zeros_like(src)
    evs = [torch.cuda.Event() for _ in range(8)]

    def run(name, fn):
        torch.cuda.synchronize()
        host = 0.0
        nch = 0
        t0 = time.perf_counter()
        for i in range(a.steps):
            env.step(acts[i % 64])
            if (i + 1) % a.every == 0:
                h0 = time.perf_counter()
                fn(nch)
                host += time.perf_counter() - h0
                nch += 1
        torch.cuda.synchronize()
        tw = time.perf_counter() - t0
        print(f"{name:34s} wall {1e3 * tw / a.steps:.4f} ms/step  side calls {1e6 * host / max(nch, 1):7.1f} us/chunk",
              flush=True)

    def record_only(c):
        evs[c % 8].record(comp)

    def record_wait(c):
        evs[c % 8].record(comp)
        side.wait_event(evs[c % 8])

    def record_wait_copy(c):
        evs[c % 8].record(comp)
        side.wait_event(evs[c % 8])
        with torch.cuda.stream(side):
            dst.copy_(src)

    def wait_stream_copy(c):
        side.wait_stream(comp)
        with torch.cuda.stream(side):
            dst.copy_(src)

    def record_wait_copy_hi(c):
        evs[c % 8].record(comp)
        side_hi.wait_event(evs[c % 8])
        with torch.cuda.stream(side_hi):
            dst.copy_(src)

    def same_stream_copy(c):
        dst.copy_(src)

    run("plain", lambda c: None)
    run("event record", record_only)
    run("event record + side wait", record_wait)
    run("record + wait + 4 MB copy on side", record_wait_copy)
    run("side.wait_stream + copy", wait_stream_copy)
    run("record + wait + copy (prio side)", record_wait_copy_hi)
    run("4 MB copy on the compute stream", same_stream_copy)
    run("plain", lambda c: None)
    env.close()


if __name__ == "__main__":
    main()
