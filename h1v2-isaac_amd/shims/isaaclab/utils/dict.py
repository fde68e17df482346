"""isaaclab.utils.dict: print_dict, class_to_dict."""
from __future__ import annotations

import dataclasses


def class_to_dict(obj):
    if hasattr(obj, "to_dict") and not dataclasses.is_dataclass(obj) and not isinstance(obj, dict):
        return obj.to_dict()
    if dataclasses.is_dataclass(obj):
        out = {}
        for f in dataclasses.fields(obj):
            out[f.name] = class_to_dict(getattr(obj, f.name))
        return out
    if isinstance(obj, dict):
        return {k: class_to_dict(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(class_to_dict(v) for v in obj)
    if hasattr(obj, "items") and callable(obj.items):
        return {k: class_to_dict(v) for k, v in obj.items()}
    if callable(obj) and hasattr(obj, "__name__"):
        return f"{obj.__module__}:{obj.__name__}"
    return obj


def print_dict(val, nesting: int = -4, start: bool = True):
    if isinstance(val, dict):
        if not start:
            print("")
        nesting += 4
        for k in val:
            print(nesting * " ", end="")
            print(k, end=": ")
            print_dict(val[k], nesting, start=False)
    else:
        print(val.__name__ if callable(val) and hasattr(val, "__name__") else val)
