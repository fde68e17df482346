#!/usr/bin/env python3
"""GPU box: the MuJoCo-mode contact-phase error statistic (SURVEY.md §7 hard part 2).

The sim2sim path steps the free-floating robot standing on the floor (D/simulator/sim_mujoco.py:39-44,102-121; floor
M/scene_12dof.xml:20).  MuJoCo itself is not installed, so the comparison is the kernel's MuJoCo mode (fp32) against
the oracle's fp64 restatement of the same model, from identical states with identical joint targets:

* free-running: n envs, 1000 policy steps x 20 substeps (1 kHz), random joint targets q0 + 0.25 a (a ~ N(0, 0.6));
  relative joint-position error max_j |dq_j| / max(1, max_j |q_j|) per env, quantiles over envs at steps
  1, 10, 100, 1000 -- contact switching makes the two trajectories diverge chaotically, which is what this shows;
* teacher-forced: every policy step restarts the oracle from the GPU state, one-step error quantiles;
* both with the smooth frictionloss option off (default) and on.

    python tools/mujoco_contact_stats.py [--envs 64] [--steps 1000] [--out gpurun_out/mujoco_contact.json]
"""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "h1v2-isaac_amd"), str(ROOT / "oracle"), str(ROOT / "tests" / "helpers")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as O  # noqa: E402
from h12env import mujoco_cfg  # noqa: E402
from h12env._abi import F as FIELDS, I as IFIELDS  # noqa: E402
from h12env.env import H12VelocityEnv  # noqa: E402


def qerr(Fa, Fb):
    o, c = FIELDS["Q"]
    qa, qb = Fa[o:o + c].astype(np.float64), Fb[o:o + c].astype(np.float64)
    return np.abs(qa - qb).max(axis=0) / np.maximum(1.0, np.abs(qb).max(axis=0))


def run(n, steps, frictionloss, seed=11):
    cfg = mujoco_cfg()
    cfg.sim.frictionloss = frictionloss
    cfg.scene.num_envs = n
    cfg.sim.device = "cuda:0"
    env = H12VelocityEnv(cfg)
    env.reset()
    free = O.OracleEnv(env._model, env._ccfg, n)   # free-running twin
    forced = O.OracleEnv(env._model, env._ccfg, n)  # restarted from the GPU state every step
    free.F[:] = env._fstate.cpu().numpy()
    free.I[:] = env._istate.cpu().numpy()
    rng = np.random.default_rng(seed)
    q0 = np.asarray(env._model.q_default, np.float32)
    marks = {1, 10, 100, 1000, steps}
    out = {"free_running": {}, "teacher_forced_one_step": []}
    pack = IFIELDS["PACK"][0]
    contact = []
    for t in range(1, steps + 1):
        F0 = env._fstate.cpu().numpy().copy()
        I0 = env._istate.cpu().numpy().copy()
        q_ref = (q0[None] + 0.25 * 0.6 * rng.normal(size=(n, 12))).astype(np.float32)
        env.step_physics(torch.from_numpy(q_ref).cuda(), 20)
        g = env._fstate.cpu().numpy()
        free.step_physics(q_ref, 20)
        forced.F[:], forced.I[:] = F0, I0
        forced.step_physics(q_ref, 20)
        out["teacher_forced_one_step"].append(qerr(g, forced.F))
        contact.append(((free.I[pack] >> 13) & 0xFF) != 0)
        if t in marks:
            e = qerr(g, free.F)
            out["free_running"][str(t)] = {q: float(np.quantile(e, v)) for q, v in
                                           (("median", 0.5), ("p90", 0.9), ("max", 1.0))}
    tf = np.concatenate(out["teacher_forced_one_step"])
    out["teacher_forced_one_step"] = {"median": float(np.median(tf)), "p99": float(np.quantile(tf, 0.99)),
                                      "p99.9": float(np.quantile(tf, 0.999)), "max": float(tf.max())}
    out["sole_contact_fraction"] = float(np.mean(contact))
    o, _ = FIELDS["POS"]
    out["base_height_final_median_m"] = float(np.median(env._fstate.cpu().numpy()[o + 2]))
    env.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=64)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--out", default=str(ROOT / "gpurun_out" / "mujoco_contact.json"))
    a = ap.parse_args()
    res = {"workload": f"{a.envs} envs x {a.steps} policy steps x 20 substeps (1 ms), free base on the floor, random "
                       "joint targets q0 + 0.25 N(0, 0.6); error = max_j |dq_j| / max(1, max_j |q_j|) per env"}
    for fl in (False, True):
        res["frictionloss_" + ("on" if fl else "off")] = run(a.envs, a.steps, fl)
        print(json.dumps({k: v for k, v in res.items() if k.startswith("friction")}, indent=1), flush=True)
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    main()
