#!/usr/bin/env python3
"""Play a trained checkpoint on the *-Play-v0 task and export it for deployment (the reference's
scripts/rsl_rl/play.py flow): <run>/exported/{policy.pt, env.yaml} (+ policy.onnx when the onnx package
is installed), then roll the policy out for --steps env steps.

    python play.py --task Isaac-Velocity-Flat-H12_12dof-Play-v0 --load_run <run dir name> [--checkpoint model_.*.pt]
"""
from __future__ import annotations

import argparse
import os
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
PKG = HERE.parent
for p in (PKG / "shims", PKG):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--task", default="Isaac-Velocity-Flat-H12_12dof-Play-v0")
    ap.add_argument("--num_envs", type=int, default=None)
    ap.add_argument("--experiment_name", default=None)
    ap.add_argument("--load_run", default=".*")
    ap.add_argument("--checkpoint", default="model_.*.pt")
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--device", default="cuda:0")
    args = ap.parse_args(argv)

    import gymnasium as gym
    import torch

    import biped_tasks.tasks  # noqa: F401
    from h12env.export import export_policy_as_jit, export_policy_as_onnx, write_env_yaml
    from isaaclab_rl.rsl_rl import RslRlVecEnvWrapper
    from isaaclab_tasks.utils import get_checkpoint_path
    from isaaclab_tasks.utils.parse_cfg import load_cfg_from_registry
    from rsl_rl.runners import OnPolicyRunner

    env_cfg = load_cfg_from_registry(args.task, "env_cfg_entry_point")
    agent_cfg = load_cfg_from_registry(args.task, "rsl_rl_cfg_entry_point")
    if args.num_envs:
        env_cfg.scene.num_envs = args.num_envs
    env_cfg.sim.device = agent_cfg.device = args.device
    root = os.path.abspath(os.path.join("logs", "rsl_rl", args.experiment_name or agent_cfg.experiment_name))
    path = get_checkpoint_path(root, args.load_run, args.checkpoint)
    print(f"[INFO]: Loading model checkpoint from: {path}")
    env = RslRlVecEnvWrapper(gym.make(args.task, cfg=env_cfg))
    runner = OnPolicyRunner(env, agent_cfg.to_dict(), log_dir=None, device=args.device)
    runner.load(path)
    policy = runner.get_inference_policy(device=args.device)
    out = os.path.join(os.path.dirname(path), "exported")
    export_policy_as_jit(runner.alg.policy, runner.obs_normalizer, out, "policy.pt")
    write_env_yaml(env_cfg, os.path.join(out, "env.yaml"))
    try:
        export_policy_as_onnx(runner.alg.policy, runner.obs_normalizer, out, "policy.onnx")
    except ImportError as e:
        print(f"[INFO]: skipping ONNX export ({e})")
    print(f"[INFO]: exported to {out}")
    obs, _ = env.get_observations()
    with torch.inference_mode():
        for _ in range(args.steps):
            obs, _, _, _ = env.step(policy(obs))
    env.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
