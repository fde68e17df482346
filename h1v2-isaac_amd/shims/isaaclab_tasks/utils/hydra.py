"""isaaclab_tasks.utils.hydra.hydra_task_config: load the task's env / agent cfgs from the registry and
apply Hydra-style command-line overrides (``env.scene.num_envs=1024 agent.max_iterations=10``)."""
from __future__ import annotations

import functools
import sys

import yaml

from .parse_cfg import load_cfg_from_registry


def _set(root, path: list[str], value):
    obj = root
    for k in path[:-1]:
        obj = obj[k] if isinstance(obj, dict) else getattr(obj, k)
    last = path[-1]
    if isinstance(obj, dict):
        obj[last] = value
    else:
        if not hasattr(obj, last):
            raise AttributeError(f"override: {type(obj).__name__} has no attribute {last!r}")
        setattr(obj, last, value)


def apply_overrides(env_cfg, agent_cfg, args: list[str]):
    for a in args:
        if "=" not in a or a.startswith("-"):
            continue
        key, raw = a.split("=", 1)
        key = key.lstrip("+")
        value = yaml.safe_load(raw)
        parts = key.split(".")
        if parts[0] == "env":
            _set(env_cfg, parts[1:], value)
        elif parts[0] == "agent":
            _set(agent_cfg, parts[1:], value)
        else:
            raise ValueError(f"override {a!r}: keys start with 'env.' or 'agent.'")


def hydra_task_config(task_name: str, agent_cfg_entry_point: str):
    def decorator(func):
        @functools.wraps(func)
        def wrapper(*args, **kwargs):
            env_cfg = load_cfg_from_registry(task_name, "env_cfg_entry_point")
            agent_cfg = load_cfg_from_registry(task_name, agent_cfg_entry_point) if agent_cfg_entry_point else None
            apply_overrides(env_cfg, agent_cfg, sys.argv[1:])
            return func(env_cfg, agent_cfg, *args, **kwargs)

        return wrapper

    return decorator
