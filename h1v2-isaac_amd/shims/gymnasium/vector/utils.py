from __future__ import annotations

from ..spaces import Box, Dict


def batch_space(space, n: int = 1):
    if isinstance(space, Box):
        import numpy as np

        return Box(np.broadcast_to(space.low, (n, *space.shape)), np.broadcast_to(space.high, (n, *space.shape)),
                   (n, *space.shape), space.dtype)
    if isinstance(space, Dict):
        return Dict({k: batch_space(v, n) for k, v in space.items()})
    raise TypeError(f"batch_space: unsupported space {space!r}")
