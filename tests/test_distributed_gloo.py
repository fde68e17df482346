"""CPU, world_size 2 (gloo): the multi-GPU path's sharding and rollout all-gather.

Each rank steps its contiguous shard of envs (the CPU oracle stands in for the per-GPU env: same
workspace layout, same global-id-keyed RNG), rollouts are all-gathered with h12env.distributed, and
rank 0 checks the gathered observations / rewards / dones bit-for-bit against one process stepping
all envs — the sharding-invariance contract the GPU bench relies on.
"""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import torch
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_per, steps, out_q):
    sys.path.insert(0, str(ROOT / "h1v2-isaac_amd"))
    sys.path.insert(0, str(ROOT / "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import oracle as O
    from h12env import H12FlatEnvCfg
    from h12env import distributed as D
    from h12env.model import build_model

    shard = D.init(n_per, backend="gloo")
    cfg = H12FlatEnvCfg()
    env = O.OracleEnv(build_model(), cfg.to_c(), n_per, env_offset=shard.env_offset)
    obs0 = env.reset()
    rng = np.random.default_rng(7)
    T = steps
    roll = {"obs": torch.zeros(T + 1, n_per, 450), "rew": torch.zeros(T, n_per),
            "done": torch.zeros(T, n_per, dtype=torch.uint8)}
    roll["obs"][0] = torch.from_numpy(obs0)
    for t in range(T):
        a_all = rng.normal(size=(shard.global_envs, 12)).astype(np.float32)  # same global batch on every rank
        a = a_all[shard.env_offset:shard.env_offset + n_per]
        obs, rew, term, trunc, _ = env.step(a, t + 1)
        roll["obs"][t + 1] = torch.from_numpy(obs)
        roll["rew"][t] = torch.from_numpy(rew)
        roll["done"][t] = torch.from_numpy((term | trunc).astype(np.uint8))
    g = D.allgather_rollout(roll, shard, env_dim=1)
    single = D.allgather_envs(torch.from_numpy(obs), shard, env_dim=0)
    if rank == 0:
        out_q.put({k: v.numpy() for k, v in g.items()} | {"last": single.numpy()})
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


def test_two_rank_sharding_and_allgather():
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle as O
    from h12env import H12FlatEnvCfg
    from h12env.model import build_model

    world, n_per, steps = 2, 24, 6
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_per, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single process, all envs
    env = O.OracleEnv(build_model(), H12FlatEnvCfg().to_c(), world * n_per)
    obs = [env.reset()]
    rews, dones = [], []
    rng = np.random.default_rng(7)
    for t in range(steps):
        a = rng.normal(size=(world * n_per, 12)).astype(np.float32)
        o, r, te, tr, _ = env.step(a, t + 1)
        obs.append(o)
        rews.append(r)
        dones.append((te | tr).astype(np.uint8))
    np.testing.assert_array_equal(got["obs"], np.stack(obs))
    np.testing.assert_array_equal(got["rew"], np.stack(rews))
    np.testing.assert_array_equal(got["done"], np.stack(dones))
    np.testing.assert_array_equal(got["last"], obs[-1])
