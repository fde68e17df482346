"""isaaclab.utils: configclass (dataclass with mutable defaults copied per instance)."""
from __future__ import annotations

import copy
import dataclasses


def configclass(cls):
    """Turn a class with annotated (or un-annotated) attributes into a dataclass; mutable defaults are
    deep-copied per instance (IsaacLab configclass semantics); adds to_dict / replace / copy."""
    for name, val in list(cls.__dict__.items()):
        if name.startswith("__") or callable(val) or isinstance(val, (property, classmethod, staticmethod)):
            continue
        if name not in cls.__dict__.get("__annotations__", {}):
            cls.__annotations__ = dict(cls.__dict__.get("__annotations__", {}))
            cls.__annotations__[name] = type(val)
    for name in list(cls.__dict__.get("__annotations__", {})):
        if name in cls.__dict__:
            val = cls.__dict__[name]
            if not isinstance(val, (int, float, str, bool, type(None), tuple)):
                setattr(cls, name, dataclasses.field(default_factory=lambda v=val: copy.deepcopy(v)))
    dc = dataclasses.dataclass(cls)
    if not hasattr(dc, "to_dict"):
        dc.to_dict = lambda self: class_to_dict(self)
    dc.replace = lambda self, **kw: dataclasses.replace(self, **kw)
    dc.copy = lambda self: copy.deepcopy(self)
    return dc


def class_to_dict(obj):
    from .dict import class_to_dict as f

    return f(obj)
