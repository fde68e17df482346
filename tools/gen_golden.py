#!/usr/bin/env python3
"""Generate tests/golden/*.npz from the reference's own importable code (build container only).

  circular_buffer.npz : packages/biped_tasks/biped_tasks/utils/history/circular_buffer.py
                        (CircularBuffer.append / reset / buffer(), lines 79-137) driven like the
                        ObservationManager history of the Flat task (history 10, term dims 3 and 12)
  delay_buffer.npz    : the same CircularBuffer driven like IsaacLab's DelayBuffer inside
                        DelayedPDActuator (max_len = max_delay + 1 = 6, one push per physics step,
                        4 pushes per env step, per-env lags 0..5, __getitem__ lines 139-170)
  deploy_obs.npz      : packages/biped_deploy/biped_deploy/controllers/rl.py ObservationHandler
                        (projected_gravity :86-95, term-major history :60-81) with the Flat task's
                        terms, unit scales and an identity command map, plus ActionHandler (:124-130)

The reference is imported by file path with stubs only for modules the exercised classes never
call (onnxruntime at rl.py:7, the RL logger).  No reference source is copied into the repository:
only input/output arrays are written.
"""
from __future__ import annotations

import importlib.util
import sys
import types
from collections import deque  # noqa: F401  (used by the reference class)
from pathlib import Path

import numpy as np
import torch

REF = Path("/root/reference/packages")
OUT = Path(__file__).resolve().parents[1] / "tests" / "golden"


def load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def gen_circular_buffer(rng):
    cb_mod = load("ref_circular_buffer", REF / "biped_tasks/biped_tasks/utils/history/circular_buffer.py")
    out = {}
    for d in (3, 12):
        n, H, T = 5, 10, 16
        buf = cb_mod.CircularBuffer(max_len=H, batch_size=n, device="cpu")
        frames = rng.normal(size=(T, n, d)).astype(np.float32)
        resets = np.zeros((T, n), bool)
        resets[5, [1, 3]] = True
        resets[9, [0]] = True
        resets[12, [1, 2, 4]] = True
        hist = np.zeros((T, n, H, d), np.float32)
        for t in range(T):
            ids = np.nonzero(resets[t])[0]
            if len(ids):
                buf.reset(batch_ids=ids.tolist())
            buf.append(torch.from_numpy(frames[t]))
            hist[t] = buf.buffer().numpy()
        out[f"frames_d{d}"] = frames
        out[f"resets_d{d}"] = resets
        out[f"history_d{d}"] = hist
    np.savez_compressed(OUT / "circular_buffer.npz", **out)


def gen_delay_buffer(rng):
    cb_mod = load("ref_circular_buffer", REF / "biped_tasks/biped_tasks/utils/history/circular_buffer.py")
    n, dec, T, max_delay = 12, 4, 10, 5
    lags = np.tile(np.arange(max_delay + 1), 2)[:n].astype(np.int64)
    buf = cb_mod.CircularBuffer(max_len=max_delay + 1, batch_size=n, device="cpu")
    targets = rng.normal(size=(T, n)).astype(np.float32)
    resets = np.zeros((T, n), bool)   # reset BEFORE env step t (lags unchanged here)
    resets[4, [0, 5, 7]] = True
    resets[7, [2, 11]] = True
    delayed = np.zeros((T, dec, n), np.float32)
    for t in range(T):
        ids = np.nonzero(resets[t])[0]
        if len(ids):
            buf.reset(batch_ids=ids.tolist())
        for s in range(dec):
            buf.append(torch.from_numpy(targets[t][:, None]))
            delayed[t, s] = buf[torch.from_numpy(lags)].numpy()[:, 0]
    np.savez_compressed(OUT / "delay_buffer.npz", lags=lags, targets=targets, resets=resets, delayed=delayed,
                        decimation=dec)


def gen_deploy_obs(rng):
    sys.modules.setdefault("onnxruntime", types.ModuleType("onnxruntime"))
    logger = types.ModuleType("biped_deploy.utils.rl_logger")
    logger.RLLogger = object
    sys.modules.setdefault("biped_deploy", types.ModuleType("biped_deploy"))
    sys.modules.setdefault("biped_deploy.utils", types.ModuleType("biped_deploy.utils"))
    sys.modules["biped_deploy.utils.rl_logger"] = logger
    rl = load("ref_rl", REF / "biped_deploy/biped_deploy/controllers/rl.py")
    q0 = np.array([0.0, -0.16, 0.0, 0.36, -0.2, 0.0] * 2)
    terms = ["base_ang_vel", "projected_gravity", "generated_commands", "joint_pos_rel", "joint_vel_rel", "last_action"]
    H, T = 10, 14
    handler = rl.ObservationHandler(terms, [1] * 6, H, q0,
                                    {"lower": -np.ones(3), "upper": np.ones(3), "velocity_deadzone": 0.0})
    quats, wang, cmds, qs, qds, acts, obs = [], [], [], [], [], [], []
    for t in range(T):
        q = rng.normal(size=4)
        q /= np.linalg.norm(q)
        st = {"base_orientation": q, "base_angular_vel": rng.normal(size=3), "qpos": q0 + rng.normal(size=12) * 0.2,
              "qvel": rng.normal(size=12)}
        a = rng.normal(size=12)
        c = rng.uniform(-1, 1, size=3)
        o = handler.get_observations(st, a, c.copy())
        quats.append(q); wang.append(st["base_angular_vel"]); cmds.append(c); qs.append(st["qpos"])
        qds.append(st["qvel"]); acts.append(a); obs.append(o)
    act = rl.ActionHandler(0.5, q0)
    a_in = rng.normal(size=(8, 12))
    a_out = np.stack([act.get_scaled_action(x) for x in a_in])
    np.savez_compressed(OUT / "deploy_obs.npz", quat=np.array(quats), wang=np.array(wang), cmd=np.array(cmds),
                        q=np.array(qs), qd=np.array(qds), act=np.array(acts), obs=np.array(obs), history=H,
                        action_in=a_in, action_out=a_out, action_scale=0.5)


def gen_deploy_env_yaml():
    """deploy_env_yaml.json: the shipped deploy configs (scripts/deploy/policies/*/env.yaml, read as YAML
    data) -- top-level keys, observation entries, and the 12 leg joints' kp / kd / default_joint_pos."""
    import json

    import yaml

    out = {}
    for p in sorted((REF.parent / "scripts" / "deploy" / "policies").glob("*/env.yaml")):
        d = yaml.safe_load(p.read_text())
        legs = [j for j in d["joints"] if j["enabled"]]
        out[p.parent.name] = {"keys": list(d.keys()), "observations": d["observations"],
                              "history_length": d["history_length"], "action_scale": d["action_scale"],
                              "control_dt": d["control_dt"], "command_ranges": d["command_ranges"],
                              "velocity_deadzone": d["velocity_deadzone"], "history_step": d["history_step"],
                              "leg_joints": legs}
    (OUT / "deploy_env_yaml.json").write_text(json.dumps(out, indent=1))


def main():
    if sys.argv[1:] == ["--env-yaml"]:
        OUT.mkdir(parents=True, exist_ok=True)
        gen_deploy_env_yaml()
        return
    OUT.mkdir(parents=True, exist_ok=True)
    rng = np.random.default_rng(20251121)
    gen_circular_buffer(rng)
    gen_delay_buffer(rng)
    gen_deploy_obs(rng)
    gen_deploy_env_yaml()
    for f in sorted(OUT.glob("*.npz")):
        print(f, f.stat().st_size, "bytes")


if __name__ == "__main__":
    main()
