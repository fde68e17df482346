#!/usr/bin/env python3
"""PPO training of an H1-2 velocity task on the MI355X env.

Command line, configuration sources and log artefacts follow the reference's scripts/rsl_rl/train.py
(+ cli_args.py): task / num_envs / seed / max_iterations / experiment_name / run_name / resume /
load_run / checkpoint / logger flags, AppLauncher flags, Hydra-style ``env.*=`` / ``agent.*=``
overrides; runs land in logs/rsl_rl/<experiment>/<timestamp>[_<run>]/ with params/{env,agent}.{yaml,pkl},
metrics.jsonl and model_<it>.pt.  Everything is resolved through the same import surface the reference
script uses (h1v2-isaac_amd/shims), i.e. this is that call sequence exercised on this stack.

Multi-GPU (one rank per GPU):
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 train.py --distributed ...
Each rank steps its own env shard (global env ids rank*num_envs ...), the rollout is all-gathered over
RCCL and every rank applies the identical PPO update (h12env.ppo).
"""
from __future__ import annotations

import argparse
import os
import sys
from datetime import datetime
from pathlib import Path

HERE = Path(__file__).resolve().parent
PKG = HERE.parent
for p in (PKG / "shims", PKG):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))

from isaaclab.app import AppLauncher  # noqa: E402


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description="Train an RL agent with RSL-RL-style PPO on the MI355X env.")
    ap.add_argument("--video", action="store_true", default=False)
    ap.add_argument("--video_length", type=int, default=200)
    ap.add_argument("--video_interval", type=int, default=2000)
    ap.add_argument("--num_envs", type=int, default=None, help="envs per rank")
    ap.add_argument("--task", type=str, default="Isaac-Velocity-Flat-H12_12dof-v0")
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--max_iterations", type=int, default=None)
    rl = ap.add_argument_group("rsl_rl")
    rl.add_argument("--experiment_name", type=str, default=None)
    rl.add_argument("--run_name", type=str, default=None)
    rl.add_argument("--resume", type=bool, default=None)
    rl.add_argument("--load_run", type=str, default=None)
    rl.add_argument("--checkpoint", type=str, default=None)
    rl.add_argument("--logger", type=str, default=None, choices={"wandb", "tensorboard", "neptune"})
    rl.add_argument("--log_project_name", type=str, default=None)
    AppLauncher.add_app_launcher_args(ap)
    return ap


def apply_cli(agent_cfg, env_cfg, args):
    """cli_args.update_rsl_rl_cfg + the num_envs / seed / device / max_iterations overrides."""
    for flag, attr in (("seed", "seed"), ("resume", "resume"), ("load_run", "load_run"),
                       ("checkpoint", "load_checkpoint"), ("run_name", "run_name"), ("logger", "logger"),
                       ("experiment_name", "experiment_name"), ("max_iterations", "max_iterations")):
        v = getattr(args, flag, None)
        if v is not None:
            setattr(agent_cfg, attr, v)
    if agent_cfg.logger in {"wandb", "neptune"} and args.log_project_name:
        agent_cfg.wandb_project = agent_cfg.neptune_project = args.log_project_name
    if args.num_envs is not None:
        env_cfg.scene.num_envs = args.num_envs
    env_cfg.seed = agent_cfg.seed
    if args.device is not None:
        env_cfg.sim.device = args.device
        agent_cfg.device = args.device


def run_dir(agent_cfg) -> tuple[str, str]:
    root = os.path.abspath(os.path.join("logs", "rsl_rl", agent_cfg.experiment_name))
    name = datetime.now().strftime("%Y-%m-%d_%H-%M-%S") + (f"_{agent_cfg.run_name}" if agent_cfg.run_name else "")
    return root, os.path.join(root, name)


def main(argv=None) -> int:
    args, hydra_args = build_parser().parse_known_args(argv)
    if args.video:
        args.enable_cameras = True
    launcher = AppLauncher(args)

    import gymnasium as gym
    import torch
    import torch.distributed as dist

    import biped_tasks.tasks  # noqa: F401  (task registry)
    from isaaclab.utils.dict import print_dict
    from isaaclab.utils.io import dump_pickle, dump_yaml
    from isaaclab_rl.rsl_rl import RslRlVecEnvWrapper
    from isaaclab_tasks.utils import get_checkpoint_path
    from isaaclab_tasks.utils.hydra import apply_overrides
    from isaaclab_tasks.utils.parse_cfg import load_cfg_from_registry
    from rsl_rl.runners import OnPolicyRunner

    env_cfg = load_cfg_from_registry(args.task, "env_cfg_entry_point")
    agent_cfg = load_cfg_from_registry(args.task, "rsl_rl_cfg_entry_point")
    apply_overrides(env_cfg, agent_cfg, hydra_args)
    apply_cli(agent_cfg, env_cfg, args)
    rank = dist.get_rank() if dist.is_initialized() else 0

    root, log_dir = run_dir(agent_cfg)
    if rank == 0:
        print(f"[INFO] Logging experiment in directory: {root}")
    make_kw = {"cfg": env_cfg, "render_mode": "rgb_array" if args.video else None}
    if dist.is_initialized():
        make_kw["env_offset"] = rank * int(env_cfg.scene.num_envs)
    env = gym.make(args.task, **make_kw)
    if args.video:
        vk = {"video_folder": os.path.join(log_dir, "videos", "train"),
              "step_trigger": lambda s: s % args.video_interval == 0, "video_length": args.video_length}
        print_dict(vk, nesting=4)
        env = gym.wrappers.RecordVideo(env, **vk)
    env = RslRlVecEnvWrapper(env)
    runner = OnPolicyRunner(env, agent_cfg.to_dict(), log_dir=log_dir if rank == 0 else None, device=agent_cfg.device)
    runner.add_git_repo_to_log(__file__)
    if agent_cfg.resume:
        path = get_checkpoint_path(root, agent_cfg.load_run, agent_cfg.load_checkpoint)
        print(f"[INFO]: Loading model checkpoint from: {path}")
        runner.load(path)
    if rank == 0:
        for name, obj in (("env", env_cfg), ("agent", agent_cfg)):
            dump_yaml(os.path.join(log_dir, "params", f"{name}.yaml"), obj)
            dump_pickle(os.path.join(log_dir, "params", f"{name}.pkl"), obj)
    runner.learn(num_learning_iterations=agent_cfg.max_iterations, init_at_random_ep_len=True)
    env.close()
    launcher.app.close()
    del torch
    return 0


if __name__ == "__main__":
    sys.exit(main())
