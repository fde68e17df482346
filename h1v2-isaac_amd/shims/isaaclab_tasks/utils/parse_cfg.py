"""isaaclab_tasks.utils.parse_cfg: resolve a task's cfg entry points from the gym registry."""
from __future__ import annotations

import importlib
import os

import yaml


def load_cfg_from_registry(task_name: str, entry_point_key: str):
    import gymnasium as gym

    spec = gym.spec(task_name.split(":")[-1])
    ep = spec.kwargs.get(entry_point_key)
    if ep is None:
        raise ValueError(f"Could not find configuration for the environment: '{task_name}'. Please check that the "
                         f"gym registry has the entry point: '{entry_point_key}'.")
    if isinstance(ep, str) and ep.endswith(".yaml"):
        if os.path.exists(ep):
            path = ep
        else:
            mod, fname = ep.split(":")
            path = os.path.join(os.path.dirname(importlib.import_module(mod).__file__), fname)
        with open(path) as f:
            return yaml.safe_load(f)
    if callable(ep):
        return ep()
    mod, attr = ep.split(":")
    return getattr(importlib.import_module(mod), attr)()


def parse_env_cfg(task_name: str, device: str = "cuda:0", num_envs: int | None = None, use_fabric: bool | None = None):
    cfg = load_cfg_from_registry(task_name, "env_cfg_entry_point")
    cfg.sim.device = device
    if num_envs is not None:
        cfg.scene.num_envs = num_envs
    return cfg
