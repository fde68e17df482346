"""isaaclab.utils.io: dump_yaml / load_yaml / dump_pickle / load_pickle for cfg objects."""
from __future__ import annotations

import os
import pickle

import yaml

from .dict import class_to_dict


def _plain(x):
    if isinstance(x, tuple):
        return [_plain(v) for v in x]
    if isinstance(x, list):
        return [_plain(v) for v in x]
    if isinstance(x, dict):
        return {str(k): _plain(v) for k, v in x.items()}
    if isinstance(x, (int, float, str, bool)) or x is None:
        return x
    return str(x)


def dump_yaml(filename: str, data, sort_keys: bool = False):
    if not filename.endswith("yaml"):
        filename += ".yaml"
    os.makedirs(os.path.dirname(filename) or ".", exist_ok=True)
    d = data if isinstance(data, dict) else class_to_dict(data)
    with open(filename, "w") as f:
        yaml.safe_dump(_plain(d), f, default_flow_style=False, sort_keys=sort_keys)


def load_yaml(filename: str) -> dict:
    with open(filename) as f:
        return yaml.safe_load(f)


def dump_pickle(filename: str, data):
    if not filename.endswith("pkl"):
        filename += ".pkl"
    os.makedirs(os.path.dirname(filename) or ".", exist_ok=True)
    with open(filename, "wb") as f:
        pickle.dump(data, f)


def load_pickle(filename: str):
    """Loads a pickle this stack wrote itself (never use on untrusted files)."""
    with open(filename, "rb") as f:
        return pickle.load(f)
