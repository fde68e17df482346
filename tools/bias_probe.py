#!/usr/bin/env python3
"""GPU probe of the kernel's signed bias against the fp64 oracle: the teacher-forced scenarios of
tests/test_gpu_sensitivity.py (flight, lying, stance, single_stance, slip) under configuration switches, one line of
per-field signed means (forced.ForcedParity.bias_fields) per run, so the source of the stance bias can be isolated
(which scenarios carry it, which switch removes it).

    python tools/bias_probe.py [--runs flight,lying,stance,stance:explicit,...] [--json out.json]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "h1v2-isaac_amd"), str(ROOT / "oracle"), str(ROOT / "tests" / "helpers"), str(ROOT / "tests")]

FIELDS_SHOWN = ("POS2", "VLIN2", "QUAT0", "Q1", "Q3", "Q4", "Q7", "Q9", "Q10", "WANG1")


def make_cfg(switches):
    from h12env import H12FlatEnvCfg

    cfg = H12FlatEnvCfg()
    cfg.terminations.base_contact_torso = False
    cfg.terminations.base_contact_knees = False
    for s in switches:
        if s == "explicit":
            cfg.sim.implicit_penalty = False
        elif s == "noself":
            cfg.sim.self_collision = False
        elif s.startswith("set."):  # set.<attr path>=<value>
            path, v = s[4:].split("=")
            obj = cfg
            parts = path.split(".")
            for p in parts[:-1]:
                obj = getattr(obj, p)
            setattr(obj, parts[-1], type(getattr(obj, parts[-1]))(float(v)))
        else:
            raise SystemExit(f"unknown switch {s}")
    return cfg


def run(spec, n, steps):
    import torch

    from forced import ForcedParity
    from h12env.env import H12VelocityEnv
    from scenarios import SCENARIOS, SOLE_SCENARIOS

    name, *sw = spec.split(":")
    cfg = make_cfg(sw)
    cfg.scene.num_envs = n
    cfg.sim.device = "cuda:0"
    env = H12VelocityEnv(cfg)
    env.reset()
    rng = np.random.default_rng(37)
    Fm = env._fstate.cpu().numpy().copy()
    Im = env._istate.cpu().numpy().copy()
    if name in SOLE_SCENARIOS:
        kw = dict(preload=1e-3) if name == "stance" else {}
        hold = SOLE_SCENARIOS[name](env._model, Fm, rng, Im=Im, action_scale=cfg.actions.joint_pos.scale, **kw)
        scale = 0.05
    else:
        SCENARIOS[name](env._model, Fm, rng)
        hold, scale = 0.0, dict(flight=1.0, lying=0.3)[name]
    env._fstate.copy_(torch.from_numpy(Fm))
    env._istate.copy_(torch.from_numpy(Im))
    fp = ForcedParity(env, seed=38)
    for _ in range(steps):
        fp.step((hold + rng.normal(size=(n, 12)) * scale).astype(np.float32))
    names, m, se = fp.bias_fields()
    env.close()
    return names, m, se, fp.quantiles()["phys"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", default="flight,lying,stance,single_stance,slip")
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--json")
    a = ap.parse_args()
    out = {}
    for spec in a.runs.split(","):
        names, m, se, q = run(spec, a.n, a.steps)
        z = m / (se + 1e-30)
        top = np.argsort(-np.abs(z))[:5]
        shown = " ".join(f"{f}={m[names.index(f)]:.2e}({z[names.index(f)]:.0f})" for f in FIELDS_SHOWN)
        print(f"{spec:28s} p50 {q['p50']:.2e} top " + " ".join(f"{names[i]}:{z[i]:.0f}" for i in top), flush=True)
        print(f"{'':28s} {shown}", flush=True)
        out[spec] = {"names": names, "mean": m.tolist(), "se": se.tolist(), "phys_quantiles": q}
    if a.json:
        Path(a.json).parent.mkdir(parents=True, exist_ok=True)
        Path(a.json).write_text(json.dumps(out))


if __name__ == "__main__":
    main()
