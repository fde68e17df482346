#!/usr/bin/env python3
"""Batched sim2sim on the MI355X: an exported policy (TorchScript policy.pt) + its env.yaml drive the env's
MuJoCo-mode physics (1 kHz PD x control_dt/0.001 substeps, MJCF torque clamps) for N envs at once, with the
deploy stack's observation / action handling (h12env.export.DeployController) -- the loop of the
reference's scripts/deploy/sim2sim.py (RLPolicy.step -> H12Mujoco.step), which runs one env in MuJoCo.

    python sim2sim.py <policy_dir> [--num_envs 64] [--episode_length 5] [--command 0.5 0 0] [--log_dir out]

policy_dir holds policy.pt and env.yaml (what play.py exports).  Commands are in the deploy convention
([-1, 1] per axis, scaled into env.yaml's command_ranges).  --log_dir writes env 0's trajectory in the
MJLogger metrics.json schema.
"""
from __future__ import annotations

import argparse
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("policy_dir", type=Path)
    ap.add_argument("--num_envs", type=int, default=64)
    ap.add_argument("--episode_length", type=float, default=5.0, help="seconds")
    ap.add_argument("--command", type=float, nargs=3, default=[0.0, 0.0, 0.0])
    ap.add_argument("--device", default="cuda:0")
    ap.add_argument("--log_dir", type=Path, default=None)
    args = ap.parse_args(argv)

    import torch
    import yaml

    from h12env import mujoco_cfg
    from h12env.env import H12VelocityEnv
    from h12env.export import DeployController, TrajectoryLogger, env_state

    pcfg = yaml.safe_load((args.policy_dir / "env.yaml").read_text())
    policy = torch.jit.load(str(args.policy_dir / "policy.pt"), map_location=args.device).eval()
    cfg = mujoco_cfg()
    cfg.scene.num_envs = args.num_envs
    cfg.sim.device = args.device
    cfg.decimation = int(round(pcfg["control_dt"] / cfg.sim.dt))
    env = H12VelocityEnv(cfg)
    env.reset()
    ctrl = DeployController(policy, pcfg, args.num_envs, args.device)
    cmd = torch.tensor(args.command, device=args.device).expand(args.num_envs, 3)
    log = TrajectoryLogger(env, 0) if args.log_dir else None
    if log:
        log.record_limits()
    steps = int(round(args.episode_length / pcfg["control_dt"]))
    for k in range(steps):
        q_ref = ctrl(env_state(env), cmd)
        env.step_physics(q_ref, cfg.decimation)
        if log:
            log.record_metrics((k + 1) * pcfg["control_dt"])
    z = env._field("POS")[2]
    print(f"[sim2sim] {args.num_envs} envs x {steps} control steps; base height mean {z.mean().item():.3f} m "
          f"(min {z.min().item():.3f})")
    if log:
        print(f"[sim2sim] trajectory of env 0: {log.save_data(args.log_dir)}")
    env.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
