"""Multi-GPU plumbing: one process per GPU, envs sharded contiguously by global id.

The env step itself has no exchange (each env is independent and its RNG is keyed by its global id,
so a shard's trajectories do not depend on the shard layout).  The only collective is the rollout
all-gather handed to PPO (BASELINE.json north_star): RCCL (`backend="nccl"` on ROCm)
over xGMI on GPUs, gloo on CPU for tests.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class Shard:
    rank: int
    world: int
    local_rank: int
    envs_per_rank: int

    @property
    def env_offset(self) -> int:
        return self.rank * self.envs_per_rank

    @property
    def global_envs(self) -> int:
        return self.world * self.envs_per_rank


def init(envs_per_rank: int, backend: str | None = None) -> Shard:
    """Read RANK / WORLD_SIZE / LOCAL_RANK (torchrun), bind the device, init the process group."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        kw = {}
        if backend == "nccl":
            torch.cuda.set_device(local)
            kw["device_id"] = torch.device(f"cuda:{local}")
        dist.init_process_group(backend, **kw)
    elif torch.cuda.is_available():
        torch.cuda.set_device(local)
    return Shard(rank, world, local, envs_per_rank)


def _staged() -> bool:
    """gloo handles CPU tensors: under gloo (CPU tests, or several ranks sharing one GPU, where RCCL refuses
    duplicate devices) device tensors go through host copies; RCCL works on the device tensors directly."""
    return dist.get_backend() == "gloo"


def all_reduce(t: torch.Tensor, op=dist.ReduceOp.SUM) -> None:
    if _staged() and t.is_cuda:
        h = t.cpu()
        dist.all_reduce(h, op=op)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=op)


def broadcast(t: torch.Tensor, src: int = 0) -> None:
    if _staged() and t.is_cuda:
        h = t.cpu()
        dist.broadcast(h, src=src)
        t.copy_(h)
    else:
        dist.broadcast(t, src=src)


def all_gather_into_tensor(out: torch.Tensor, x: torch.Tensor, async_op: bool = False):
    """async_op (RCCL): returns the collective's Work -- ``work.wait()`` makes the CURRENT stream wait for it (a
    device-side wait, the host does not block); staged (gloo) it completes before returning (None)."""
    if _staged() and x.is_cuda:
        h = torch.empty(out.shape, dtype=out.dtype)
        dist.all_gather_into_tensor(h, x.cpu())
        out.copy_(h)
        return None
    return dist.all_gather_into_tensor(out, x, async_op=async_op)


def allgather_envs(x: torch.Tensor, shard: Shard, env_dim: int = 0) -> torch.Tensor:
    """All-gather a per-shard tensor along its env dimension (rank order = global env order)."""
    if shard.world == 1:
        return x
    xt = x.movedim(env_dim, 0).contiguous()
    out = torch.empty((shard.world * xt.shape[0], *xt.shape[1:]), dtype=xt.dtype, device=xt.device)
    all_gather_into_tensor(out, xt)
    return out.movedim(0, env_dim)


def allgather_rollout(storage: dict[str, torch.Tensor], shard: Shard, env_dim: int = 1) -> dict[str, torch.Tensor]:
    """All-gather every (T, N_shard, ...) rollout tensor into (T, N_global, ...), one collective per
    dtype bucket (tensors of one dtype are packed into a single flat buffer to keep the number of RCCL
    launches per PPO iteration small)."""
    if shard.world == 1:
        return storage
    out: dict[str, torch.Tensor] = {}
    by_dtype: dict[torch.dtype, list[str]] = {}
    for k, v in storage.items():
        by_dtype.setdefault(v.dtype, []).append(k)
    for dt, keys in by_dtype.items():
        parts = [storage[k].movedim(env_dim, 0).contiguous() for k in keys]
        flat = torch.cat([p.reshape(p.shape[0], -1) for p in parts], dim=1)  # (N_shard, sum features)
        g = torch.empty((shard.world * flat.shape[0], flat.shape[1]), dtype=dt, device=flat.device)
        all_gather_into_tensor(g, flat)
        col = 0
        for k, p in zip(keys, parts):
            w = p[0].numel()
            out[k] = g[:, col:col + w].reshape(g.shape[0], *p.shape[1:]).movedim(0, env_dim)
            col += w
    return out


def max_over_ranks(value: float, device=None) -> float:
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier(device=None):
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()
    if device is not None and torch.device(device).type == "cuda":
        torch.cuda.synchronize(device)
