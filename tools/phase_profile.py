#!/usr/bin/env python3
"""Per-phase shader-clock profile of step_kernel (experiment build, -DH12_PHASE_PROFILE).

    python tools/phase_profile.py --build [--tag NAME] [-D FLAG ...]   # here: compile tools/_variants/lib_NAME.so
    python tools/phase_profile.py [--tag NAME] [--steps K]            # GPU box: run the bench workload, print

The variant library records, per main (physics) wave and lane 0, the cycles between the PH / PHX marks of
csrc/h12env.hip into 16 global counters (h12env_phase_profile); printed here as cycles per wave and env
step.  Slots: 0 state loads, 1 physics loop, 2 contact-sensor replay, 3 rewards / terminations, 4 outputs +
episode log, 5 reset + commands + events, 6 observation frame, 7 state stores; inside each inner step
(summed over the step's inner steps): 10 pass 1 and the ground contacts, 8 the barrier R1 itself, 11 reading the
helper wave's joint terms, 12 the articulated-inertia chain, 9 the barrier R2 itself, 13 reading its bias forces /
self-contact wrenches, 14 the rest (bias-force chain, base solve, pass 3, integration, next state to the helper).  The marks' own atomics add a few hundred cycles per step.  Not the product
library: the variant is loaded through H12ENV_LIB and never built by __graft_entry__.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "h1v2-isaac_amd"))
VARIANTS = ROOT / "tools" / "_variants"
SLOTS = {0: "loads", 1: "physics", 2: "sensor", 3: "rewards", 4: "outputs+log", 5: "reset+cmd", 6: "frame",
         7: "stores", 10: "inner: pass 1 + ground contacts", 8: "inner: barrier R1 (waiting for the helpers)",
         11: "inner: joint terms from LDS", 12: "inner: inertia chain (pinned ahead of R2)",
         9: "inner: barrier R2 (waiting for the helpers)", 13: "inner: bias forces / self wrenches from LDS",
         14: "inner: bias chain .. integration + S"}


def build(tag: str, flags: list[str], plain: bool = False) -> Path:
    from h12env.build import ARCH, CSRC, hipcc

    VARIANTS.mkdir(parents=True, exist_ok=True)
    out = VARIANTS / f"lib_{tag}.so"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fno-slp-vectorize", "-Xarch_device",
           "-ffinite-math-only", "-Xarch_device", "-fno-signed-zeros", "-fPIC", "-shared", "-Wno-unused-function",
           *([] if plain else ["-DH12_PHASE_PROFILE"]), *[f"-D{f}" for f in flags], "-o", str(out),
           str(CSRC / "h12env.hip")]
    print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return out


def run(tag: str, steps: int, burn: int, envs: int, self_coll: bool) -> dict:
    os.environ["H12ENV_LIB"] = str(VARIANTS / f"lib_{tag}.so")
    import torch

    from h12env import H12FlatEnvCfg
    from h12env._abi import load_library
    from h12env.env import H12VelocityEnv

    lib = load_library()
    lib.h12env_phase_profile.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    lib.h12env_phase_profile.restype = C.c_int
    cfg = H12FlatEnvCfg()
    cfg.scene.num_envs = envs
    cfg.sim.device = "cuda:0"
    cfg.sim.self_collision = self_coll
    env = H12VelocityEnv(cfg)
    env.reset()
    g = torch.Generator(device="cuda:0").manual_seed(0)
    env.episode_length_buf = torch.randint(0, env.max_episode_length, (envs,), device="cuda:0", generator=g,
                                           dtype=env.episode_length_buf.dtype)
    acts = torch.randn(burn + steps, envs, 12, device="cuda:0", generator=g)
    buf = (C.c_ulonglong * 16)()
    for t in range(burn):
        env.step(acts[t])
    torch.cuda.synchronize()
    lib.h12env_phase_profile(buf, 1)
    for t in range(steps):
        env.step(acts[burn + t])
    torch.cuda.synchronize()
    lib.h12env_phase_profile(buf, 1)
    waves = (envs + 31) // 32
    res = {SLOTS[i]: round(buf[i] / waves / steps, 1) for i in SLOTS}
    if hasattr(lib, "h12env_wave_times"):  # per-wave realtime stamps (100 MHz) of single launches
        import numpy as np

        wt = (C.c_ulonglong * (11 * waves))()
        keys = ("span", "start_spread", "end_spread", "dur_mean", "dur_max", "drain_max")
        rows, raw, rsets, clk, bw, ends, light = [], [], [], [], [], [], []
        bws = []
        has_bw = hasattr(lib, "h12env_barrier_waits")
        bwbuf = (C.c_ulonglong * (64 * waves))()
        has_ks = hasattr(lib, "h12env_kernel_starts")
        ksbuf = (C.c_ulonglong * (4 * waves))()
        kss = []
        for t in range(40):
            env.step(acts[t])
            torch.cuda.synchronize()
            lib.h12env_wave_times(wt, waves)
            if has_bw:  # light build: per block, role (physics, helper, contact, self) and barrier (S, R1, R2, first S)
                lib.h12env_barrier_waits(bwbuf, waves)
                bws.append(np.frombuffer(bwbuf, dtype=np.uint64).reshape(waves, 4, 16).astype(np.float64) / 2370.0)
            if has_ks:  # every wave's first instruction (s_memrealtime ticks, 100 MHz)
                lib.h12env_kernel_starts(ksbuf, waves)
                kss.append(np.frombuffer(ksbuf, dtype=np.uint64).reshape(waves, 4).astype(np.float64) / 100.0)
            full = np.frombuffer(wt, dtype=np.uint64).reshape(waves, 11).astype(np.int64)
            bw.append(full[:, 9:11] / 2370.0)  # barrier-wait cycles -> us at the measured clock
            clk.append((full[:, 8] - full[:, 7]) / np.maximum(1, full[:, 2] - full[:, 0]) * 100.0)  # MHz
            if os.environ.get("H12_PHASE_LIGHT"):  # light build: columns 7 / 8 are the helper / self waves' end,
                # 9 / 10 the stamps after the rewards and after barrier L
                ends.append(np.stack([full[:, 2], full[:, 7], full[:, 8]], 1) - full[:, 0:1])
                light.append(np.stack([full[:, 3] - full[:, 0], full[:, 9] - full[:, 3], full[:, 10] - full[:, 9],
                                       full[:, 4] - full[:, 10], full[:, 6] - full[:, 4], full[:, 1] - full[:, 6]], 1))
            a = np.concatenate([full[:, :5], full[:, 6:7]], axis=1)
            a -= a[:, 0].min()
            # columns: 0 start, 1 end, 2 end after waitcnt, 3 after physics, 4 after reset, 5 XCC id
            # (s_getreg HW_REG_XCC_ID), 6 after barrier F
            a = np.concatenate([a[:, :5], full[:, 5:6], a[:, 5:6]], axis=1)
            raw.append(a.copy())
            rs = (env.reset_terminated | env.reset_time_outs).view(-1, 32).sum(1).cpu().numpy()
            rsets.append(rs)
            d = a[:, 1] - a[:, 0]
            rows.append([a[:, 2].max(), a[:, 0].max(), a[:, 1].max() - a[:, 1].min(), d.mean(), d.max(),
                         (a[:, 2] - a[:, 1]).max()])
        if os.environ.get("H12_WAVE_DUMP"):
            np.save(os.environ["H12_WAVE_DUMP"], np.asarray(raw))
            np.save(os.environ["H12_WAVE_DUMP"].replace(".npy", "_resets.npy"), np.asarray(rsets))
            if bws:  # (launches, blocks, role, barrier) waits in us: which role a slow block waited for
                np.save(os.environ["H12_WAVE_DUMP"].replace(".npy", "_bw.npy"), np.asarray(bws))
        res["wave_realtime_us_median"] = dict(zip(keys, (np.median(np.asarray(rows), axis=0) / 100.0).round(2).tolist()))
        R = np.asarray(raw)  # (launches, waves, 7)
        per = {}
        for x in range(8):
            m = R[:, :, 5] == x
            if not m.any():
                continue
            w = R[m]
            med = lambda v: round(float(np.median(v)) / 100.0, 2)  # noqa: E731
            per[f"xcc{x}"] = {"physics": med(w[:, 3] - w[:, 0]), "sensor..reset": med(w[:, 4] - w[:, 3]),
                              "frame+F wait": med(w[:, 6] - w[:, 4]), "store issue": med(w[:, 1] - w[:, 6]),
                              "store completion": med(w[:, 2] - w[:, 1]), "end": med(w[:, 2]),
                              "clock_MHz": round(float(np.median(np.asarray(clk)[m])), 0),
                              "barrier R1 wait": round(float(np.median(np.asarray(bw)[m][:, 0])), 2),
                              "barrier R2 wait": round(float(np.median(np.asarray(bw)[m][:, 1])), 2)}
        res["per_xcc_us_median"] = per
        if light:  # the physics wave's phases, medians over waves with / without a resetting env
            Lp = np.concatenate(light) / 100.0
            rw = np.concatenate(rsets) > 0
            names = ("physics loop", "sensor + rewards", "outputs + log + barrier L", "reset + command + events",
                     "frame + barrier F", "store issue")
            res["light_phases_us_median"] = {
                grp: {k: round(float(np.median(Lp[sel][:, i])), 2) for i, k in enumerate(names)}
                for grp, sel in (("waves_with_reset", rw), ("waves_without_reset", ~rw)) if sel.any()}
            res["light_phases_us_median"]["fraction_of_waves_with_reset"] = round(float(rw.mean()), 3)
        if bws and raw:  # round 6: the block tail -- each block's physics loop against its self-contact candidates
            # (the self wave's PHN marks: slot 8 = the most candidate envs of an inner step, slot 9 = their sum over the
            # launch), per launch the slowest block's loop against the median block's
            Bc = np.asarray(bws)  # (launches, blocks, role, 16) in us of 2370 cycles; the PHN slots hold counts
            ncmax = np.rint(Bc[:, :, 3, 8] * 2370.0).astype(int)
            ncsum = np.rint(Bc[:, :, 3, 9] * 2370.0).astype(int)
            Rw = np.asarray(raw)
            loop = (Rw[:, :, 3] - Rw[:, :, 0]) / 100.0  # us
            qq = lambda x: [round(float(np.quantile(x, p)), 2) for p in (0.5, 0.95, 1.0)]  # noqa: E731
            by = {}
            for k in range(int(ncmax.max()) + 1):
                m = ncmax == k
                if m.any():
                    by[str(k)] = {"blocks": int(m.sum()), "loop_us_median": round(float(np.median(loop[m])), 2)}
            res["block_tail"] = {
                "physics_loop_us_p50_p95_max": qq(loop.ravel()),
                "per_launch_max_minus_median_us": round(float(np.mean(loop.max(1) - np.median(loop, 1))), 2),
                "slowest_block_max_candidates_median": float(np.median(ncmax[np.arange(len(loop)), loop.argmax(1)])),
                "by_max_candidates": by,
                "candidate_sum_per_launch_p50_p95_max": qq(ncsum.ravel())}
        if bws:  # median over blocks and launches of the us each wave role waited per launch in each barrier kind
            B = np.concatenate(bws)  # (launches x blocks, 4, 4)
            res["barrier_wait_us_per_launch_median"] = {
                role: {bar: round(float(np.median(B[:, r, k])), 3) for k, bar in enumerate(("S", "R1", "R2", "S first"))}
                for r, role in enumerate(("physics", "helper", "contact", "self"))}
            # each role's own work before each barrier kind (summed over the launch's inner steps; "S first": the
            # work from the wave's start)
            res["work_before_barrier_us_per_launch_median"] = {
                role: {bar: round(float(np.median(B[:, r, 4 + k])), 3) for k, bar in enumerate(("S", "R1", "R2", "S first"))}
                for r, role in enumerate(("physics", "helper", "contact", "self"))}
            # the physics wave after R2, summed over the inner steps: from the barrier exit to the end of the bias
            # chain, of the base solve and of pass 3 (the rest up to S / the loop end: integration, state hand-off)
            res["physics_after_r2_marks_us_per_launch_median"] = {
                m: round(float(np.median(B[:, 0, 8 + i])), 3)
                for i, m in enumerate(("bias chain", "+ base combine / solve", "+ pass 3 / implicit reports"))}
            # the first inner step alone (slots 12-14: work before its S / R1 / R2; the instruction cache is cold at the
            # launch's start) against the mean inner step of the launch
            n_in = (3.0, 4.0, 4.0)  # barrier S between the 4 inner steps, R1 / R2 in each
            res["work_first_inner_step_us_median"] = {
                role: {bar: round(float(np.median(B[:, r, 12 + k])), 3) for k, bar in enumerate(("S", "R1", "R2"))}
                for r, role in enumerate(("physics", "helper", "contact", "self"))}
            res["work_mean_inner_step_us_median"] = {
                role: {bar: round(float(np.median(B[:, r, 4 + k])) / n_in[k], 3) for k, bar in enumerate(("S", "R1", "R2"))}
                for r, role in enumerate(("physics", "helper", "contact", "self"))}
            # each role's start after the block's first wave (slot 15: s_memrealtime at the wave's first stamp)
            St = B[:, :, 15] * 2370.0 / 100.0
            St = St - St.min(1, keepdims=True)
            res["wave_start_after_first_us_median"] = {
                role: round(float(np.median(St[:, r])), 3) for r, role in enumerate(("physics", "helper", "contact", "self"))}
            res["wave_start_after_first_us_p90"] = {
                role: round(float(np.quantile(St[:, r], 0.9)), 3) for r, role in enumerate(("physics", "helper", "contact", "self"))}
            if kss:
                K = np.concatenate(kss)  # (launches x blocks, 4) us
                q = lambda x: [round(float(np.quantile(x, p)), 3) for p in (0.05, 0.5, 0.95, 1.0)]
                n_l = len(kss)
                Kb = K.min(1).reshape(n_l, -1)
                res["block_first_instruction_after_first_block_us_q"] = q((Kb - Kb.min(1, keepdims=True)).ravel())
                res["wave_first_instruction_after_block_first_us_median"] = {
                    role: round(float(np.median(K[:, r] - K.min(1))), 3)
                    for r, role in enumerate(("physics", "helper", "contact", "self"))}
                # role start (slot 15: the physics wave's entry after its argument loads, the other roles' function
                # start) after the wave's own first instruction
                res["role_start_after_first_instruction_us_median"] = {
                    role: round(float(np.median(B[:, r, 15] * 2370.0 / 100.0 - K[:, r])), 3)
                    for r, role in enumerate(("physics", "helper", "contact", "self"))}
            # who arrives last at barrier F (slot 11: s_memrealtime at the arrival, 100 MHz): per block, each role's
            # arrival after the first one's
            Fa = B[:, :, 11] * 2370.0 / 100.0  # back to realtime ticks, then us
            Fa = Fa - Fa.min(1, keepdims=True)
            res["barrier_F_arrival_after_first_us_median"] = {
                role: round(float(np.median(Fa[:, r])), 3) for r, role in enumerate(("physics", "helper", "contact", "self"))}
            res["barrier_F_last_role_count"] = {
                role: int((Fa.argmax(1) == r).sum()) for r, role in enumerate(("physics", "helper", "contact", "self"))}
        if ends:
            E = np.concatenate(ends) / 100.0  # us from the physics wave's start: physics / helper / self wave ends
            res["wave_role_end_us"] = {"physics_median": round(float(np.median(E[:, 0])), 2),
                                       "helper_median": round(float(np.median(E[:, 1])), 2),
                                       "self_median": round(float(np.median(E[:, 2])), 2),
                                       "block_end_max_role": ["physics", "helper", "self"][
                                           int(np.bincount(np.argmax(E, 1), minlength=3).argmax())],
                                       "helper_after_physics_median": round(float(np.median(E[:, 1] - E[:, 0])), 2),
                                       "self_after_physics_median": round(float(np.median(E[:, 2] - E[:, 0])), 2)}
    env.close()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--tag", default="phase")
    ap.add_argument("-D", dest="defs", action="append", default=[])
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--burn-in", type=int, default=200)
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--no-self-collision", action="store_true")
    ap.add_argument("--plain", action="store_true", help="--build without the phase marks (an experiment variant "
                    "for H12ENV_LIB=tools/_variants/lib_TAG.so python bench.py)")
    a = ap.parse_args()
    if a.build:
        build(a.tag, a.defs, a.plain)
        return
    res = run(a.tag, a.steps, a.burn_in, a.envs, not a.no_self_collision)
    print(json.dumps({"tag": a.tag, "envs": a.envs, "cycles_per_wave_per_env_step": res}))


if __name__ == "__main__":
    main()
