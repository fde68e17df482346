#!/usr/bin/env python3
"""Diagnostic (GPU box): what the C4 rollout path costs per env step on one GPU, piece by piece.

    python tools/c4_diag.py [--envs 4096] [--steps 240] [--gather-every 4]

Modes: plain steps; steps recording into a bound RolloutRecorder; + the chunk's actions copied into the records;
+ the row rebuild (decode) per chunk.  For each: wall ms per step after a final sync, and the host-side ms per step of the
loop alone (launch-bound if it approaches the wall time)."""
import argparse
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "h1v2-isaac_amd"))

import torch  # noqa: E402

from h12env import H12FlatEnvCfg  # noqa: E402
from h12env.env import H12VelocityEnv  # noqa: E402
from h12env.rollout import RolloutGather, RolloutRecorder, decode  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=240)
    ap.add_argument("--gather-every", type=int, default=4)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    cfg = H12FlatEnvCfg()
    cfg.scene.num_envs = a.envs
    cfg.sim.device = str(dev)
    env = H12VelocityEnv(cfg)
    env.reset()
    n = a.envs
    acts = torch.randn(64, n, 12, device=dev)
    for i in range(100):
        env.step(acts[i % 64])
    torch.cuda.synchronize()

    def run(mode):
        rec = rg = None
        if mode != "plain":
            rec = RolloutRecorder(n, 24, dev, 10)
            rg = RolloutGather(rec, 1, a.gather_every, env.get_observations()["policy"].clone())
            mode_base = mode.split("-")[0]
            env.bind_rollout(rec)
            if mode_base == "record":
                rg = None
            elif mode_base == "acts":
                rg.decode_off = True
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.steps):
            if rg is not None:
                rg.before_step()
            tc = rec.t if rec is not None else 0
            env.step(acts[i % 64])
            if rg is not None:
                if mode.startswith("acts"):  # + the chunk's actions copied into the records (bench.py's put_actions)
                    rg.after_step(tc, lambda s0, s1: rec.actions[s0:s1].copy_(acts[:s1 - s0]))
                else:
                    rg.after_step(tc)
        th = time.perf_counter() - t0
        if rg is not None:
            rg.wait()
        torch.cuda.synchronize()
        tw = time.perf_counter() - t0
        if rec is not None:
            env.unbind_rollout()
        print(f"{mode:8s} wall {1e3 * tw / a.steps:.4f} ms/step   host loop {1e3 * th / a.steps:.4f} ms/step", flush=True)

    for mode in ("plain", "record", "acts", "decode", "plain"):
        run(mode)
    # the decode kernel alone: one chunk and one whole iteration of rows, back to back
    rec = RolloutRecorder(n, 24, dev, 10)
    g = torch.zeros(rec.record.numel(), dtype=torch.uint8, device=dev)
    out = torch.empty(24, n, 450, device=dev)
    tail = torch.zeros(n, 450, device=dev)
    for G, t1 in ((a.gather_every, a.gather_every), (24, 24)):
        for _ in range(3):
            decode(g, 1, n, 24, G, 10, 0, t1, tail, out)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            decode(g, 1, n, 24, G, 10, 0, t1, tail, out)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        print(f"decode {t1:2d} rows x {n} envs: {1e3 * ms:.1f} us  ({t1 * n * 1800 / ms / 1e6:.0f} GB/s written)", flush=True)
    env.close()


if __name__ == "__main__":
    main()
