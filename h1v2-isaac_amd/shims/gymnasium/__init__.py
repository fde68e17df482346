"""Minimal gymnasium 1.x surface for the reference scripts: registry (register / spec / make), Env,
spaces.Box / spaces.Dict, vector.utils.batch_space.  Only what train.py / play.py and the env use."""
from __future__ import annotations

import importlib
from dataclasses import dataclass, field
from typing import Any, Callable

from . import spaces, vector, wrappers  # noqa: F401

__version__ = "1.2.1+mi355x-shim"


@dataclass
class EnvSpec:
    id: str
    entry_point: Any = None
    kwargs: dict = field(default_factory=dict)
    disable_env_checker: bool = False
    max_episode_steps: int | None = None
    order_enforce: bool = True
    additional_wrappers: tuple = ()


registry: dict[str, EnvSpec] = {}


def register(id: str, entry_point: Any = None, kwargs: dict | None = None, disable_env_checker: bool = False, **extra):
    registry[id] = EnvSpec(id=id, entry_point=entry_point, kwargs=dict(kwargs or {}),
                           disable_env_checker=disable_env_checker,
                           max_episode_steps=extra.get("max_episode_steps"))


def spec(id: str) -> EnvSpec:
    if id not in registry:
        raise KeyError(f"Environment {id} doesn't exist (registered: {sorted(registry)})")
    return registry[id]


def _resolve(ep) -> Callable:
    if callable(ep):
        return ep
    mod, attr = ep.split(":")
    return getattr(importlib.import_module(mod), attr)


def make(id: str | EnvSpec, **kwargs):
    s = id if isinstance(id, EnvSpec) else spec(id)
    kw = dict(s.kwargs)
    kw.update(kwargs)
    env = _resolve(s.entry_point)(**kw)
    try:
        env.spec = s
    except Exception:
        pass
    return env


class Env:
    metadata: dict = {"render_modes": []}
    render_mode = None
    spec: EnvSpec | None = None

    @property
    def unwrapped(self):
        return self


class Wrapper(Env):
    def __init__(self, env):
        self.env = env

    def __getattr__(self, name):
        return getattr(self.env, name)

    @property
    def unwrapped(self):
        return self.env.unwrapped
