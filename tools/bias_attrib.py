#!/usr/bin/env python3
"""Attribution of the kernel's signed sole-contact bias, on the CPU.

The GPU sole scenarios (tests/test_gpu_sensitivity.py::test_forced_sole_contact_scenarios) measure a per-field signed
mean error of the kernel against the fp64 oracle far beyond its standard error (stance Q7 +2.5e-7, z = 167;
profiles/r5/bias_*.json).  This script runs the same scenarios with a CPU stand-in whose physics is the oracle's own
source evaluated in single precision (oracle/oracle_f32.c -> liboracle_f32.so) and prints, per field, its signed mean
against the fp64 oracle beside the kernel's.  An fp32 evaluation of the reference algorithm that carries the same
signature says the bias comes from evaluating the model in fp32, not from a kernel defect; the knobs below switch
single sources of fp32 error off in that stand-in (--exact-*) to name the operation.

    python tools/bias_attrib.py [--n 1024] [--steps 20] [--scen stance,single_stance,slip] [--json out.json]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "h1v2-isaac_amd"), str(ROOT / "oracle"), str(ROOT / "tests" / "helpers"), str(ROOT / "tests")]


def f32_lib(variant: str = ""):
    import subprocess

    so = ROOT / "oracle" / f"liboracle_f32{variant}.so"
    subprocess.run(["make", "-s", "-C", str(ROOT / "oracle"), so.name], check=True)
    import oracle as O

    L = C.CDLL(str(so))
    vp = C.c_void_p
    M, Cf = C.POINTER(O.H12Model), C.POINTER(O.H12Config)
    L.orc_env_reset.argtypes = [M, Cf, C.c_int, C.c_int64, vp, vp, vp, vp, C.c_uint64]
    L.orc_env_step.argtypes = [M, Cf, C.c_int, C.c_int64, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, C.c_int64,
                               C.c_int]
    return L


class F32Env:
    """OracleEnv's step / reset on the single-precision build."""

    def __init__(self, lib, model, cfg, n):
        import oracle as O

        self.O, self.L, self.model, self.cfg, self.n = O, lib, model, cfg, n
        self.F = np.zeros((O.NF_FLOAT, n), np.float32)
        self.I = np.zeros((O.NF_INT, n), np.int32)
        self.obs = np.zeros((n, O.lib().orc_obs_dim(C.byref(cfg))), np.float32)

    def reset(self):
        p = self.O._p
        self.L.orc_env_reset(C.byref(self.model), C.byref(self.cfg), self.n, 0, p(self.F), p(self.I), None,
                             p(self.obs), 0)

    def step(self, a, k):
        p, n = self.O._p, self.n
        a = np.ascontiguousarray(a, np.float32)
        obs, rew = np.empty_like(self.obs), np.empty(n, np.float32)
        term, trunc = np.empty(n, np.uint8), np.empty(n, np.uint8)
        log, tq = np.zeros(self.O.NLOG, np.float32), np.empty((n, 12), np.float32)
        ff, cp = np.empty((n, 2), np.float32), np.zeros(n, np.float32)
        rc = self.L.orc_env_step(C.byref(self.model), C.byref(self.cfg), n, 0, p(self.F), p(self.I), p(a), p(self.obs),
                                 p(obs), p(rew), p(term), p(trunc), p(log), p(tq), p(ff), p(cp), k, 8)
        assert rc == 0
        self.obs = obs
        return obs.copy(), rew, term.astype(bool), trunc.astype(bool)


class F32StandIn:
    """The surface ForcedParity drives, backed by the single-precision oracle (no added noise: its own rounding)."""

    def __init__(self, lib, n, cfg):
        import torch

        from h12env.model import build_model

        cfg.scene.num_envs = n
        self._model, self._ccfg = build_model(), cfg.to_c()
        self.num_envs, self.env_offset, self.device = n, 0, torch.device("cpu")
        self.core = F32Env(lib, build_model(), cfg.to_c(), n)
        self.core.reset()
        self._fstate, self._istate = torch.from_numpy(self.core.F), torch.from_numpy(self.core.I)
        self._obs = [torch.from_numpy(self.core.obs)]
        self._k, self.common_step_counter = 0, 0

    def step(self, a):
        import torch

        self.common_step_counter += 1
        obs, rew, term, trunc = self.core.step(a.numpy(), self.common_step_counter)
        self._fstate, self._istate = torch.from_numpy(self.core.F), torch.from_numpy(self.core.I)
        self._obs = [torch.from_numpy(obs)]
        return {"policy": self._obs[0]}, torch.from_numpy(rew), torch.from_numpy(term), torch.from_numpy(trunc), {}


def run(lib, name, n, steps, seed=37):
    from forced import ForcedParity
    from h12env import H12FlatEnvCfg
    from scenarios import SOLE_SCENARIOS

    cfg = H12FlatEnvCfg()
    cfg.terminations.base_contact_torso = False
    cfg.terminations.base_contact_knees = False
    env = F32StandIn(lib, n, cfg)
    kw = dict(preload=1e-3) if name == "stance" else {}
    hold = SOLE_SCENARIOS[name](env._model, env.core.F, np.random.default_rng(seed), Im=env.core.I, action_scale=0.5,
                                **kw)
    fp = ForcedParity(env, seed=seed + 1)
    rng = np.random.default_rng(seed + 2)
    for _ in range(steps):
        fp.step((hold + rng.normal(size=(n, 12)) * 0.05).astype(np.float32))
    return fp


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--scen", default="stance,single_stance,slip")
    ap.add_argument("--json")
    ap.add_argument("--seed", type=int, default=37)
    ap.add_argument("--variant", default="", help="'' = plain fp32 build, 'hw' = with the kernel's sin / cos prescale")
    a = ap.parse_args()
    lib = f32_lib(a.variant)
    out = {}
    for name in a.scen.split(","):
        fp = run(lib, name, a.n, a.steps, a.seed)
        names, m, se = fp.bias_fields()
        kern = json.loads((ROOT / "profiles" / "r5" / f"bias_{name}.json").read_text())
        km, kse = np.array(kern["mean"]), np.array(kern["se"])
        zk = km / kse
        print(f"== {name}: fp32 oracle vs fp64 oracle (this run) beside the kernel vs fp64 oracle (profiles/r5)")
        print(f"{'field':8s} {'f32 mean':>10s} {'f32 z':>7s} {'kern mean':>10s} {'kern z':>7s} {'diff z':>7s}")
        for i in np.argsort(-np.abs(zk))[:10]:
            dz = (km[i] - m[i]) / np.hypot(kse[i], se[i])
            print(f"{names[i]:8s} {m[i]:10.3g} {m[i] / (se[i] + 1e-30):7.1f} {km[i]:10.3g} {zk[i]:7.1f} {dz:7.1f}")
        out[name] = {"names": names, "mean": m.tolist(), "se": se.tolist(), "quantiles": fp.quantiles()}
    if a.json:
        Path(a.json).write_text(json.dumps(out))


if __name__ == "__main__":
    main()
