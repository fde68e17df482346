"""isaaclab_tasks.utils: checkpoint discovery and registry cfg loading."""
from __future__ import annotations

import os
import re

from .parse_cfg import load_cfg_from_registry, parse_env_cfg


def get_checkpoint_path(log_path: str, run_dir: str = ".*", checkpoint: str = ".*", other_dirs: list[str] | None = None,
                        sort_alpha: bool = True) -> str:
    """Latest run directory under log_path matching run_dir, then its latest checkpoint matching
    checkpoint (numeric order of model_<it>.pt)."""
    try:
        runs = [os.path.join(log_path, d.name) for d in os.scandir(log_path)
                if d.is_dir() and re.match(run_dir, d.name)]
        if sort_alpha:
            runs.sort()
        else:
            runs = sorted(runs, key=os.path.getmtime)
        run_path = os.path.join(runs[-1], *other_dirs) if other_dirs else runs[-1]
    except IndexError:
        raise ValueError(f"No runs present in the directory: '{log_path}' match: '{run_dir}'.")
    ckpts = [f for f in os.listdir(run_path) if re.match(checkpoint, f)]
    if not ckpts:
        raise ValueError(f"No checkpoints in the directory: '{run_path}' match '{checkpoint}'.")
    ckpts.sort(key=lambda m: [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", m)])
    return os.path.join(run_path, ckpts[-1])


__all__ = ["get_checkpoint_path", "load_cfg_from_registry", "parse_env_cfg"]
