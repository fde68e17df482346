"""GPU, world_size 2: the multi-GPU path on the real HIP env.  Two ranks are started as child
processes (tests/helpers/dist_worker.py), both on cuda:0 of the one-GPU box with a gloo process group (RCCL refuses
two ranks on one device; h12env.distributed stages device tensors through the host under gloo).  Each rank steps its
contiguous shard of the Flat env; checked here:

  * the all-gathered rollout (observations, rewards, dones) equals one process stepping all 2N envs, bit for bit
    (env RNG keyed by global env id: shard-invariant trajectories);
  * after one PPO iteration of the runner (rollout all-gather, gradient / KL / normaliser all-reduces, rank-0
    parameter broadcast) both ranks hold bit-identical parameters, which moved and are finite.

RCCL itself (backend "nccl", one GPU per rank) runs in bench.py's N>1 path on the driver's 8-GPU node."""
import os
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

ROOT = Path(__file__).resolve().parents[1]
WORKER = ROOT / "tests" / "helpers" / "dist_worker.py"

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(420)
def test_two_rank_shards_allgather_and_ppo_update(tmp_path):
    n_per, steps, world = 256, 12, 2
    port = _free_port()
    procs = []
    for rank in range(world):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                   WORLD_SIZE=str(world), LOCAL_RANK="0")
        log = open(tmp_path / f"rank{rank}.log", "w")
        procs.append((subprocess.Popen([sys.executable, str(WORKER), str(tmp_path), str(n_per), str(steps)],
                                       env=env, stdout=log, stderr=subprocess.STDOUT), log))
    try:
        for p, _ in procs:
            p.wait(timeout=360)
    finally:
        for p, log in procs:
            if p.poll() is None:
                p.kill()
            log.close()
    for rank, (p, _) in enumerate(procs):
        assert p.returncode == 0, (tmp_path / f"rank{rank}.log").read_text()[-3000:]

    # ---- the same global rollout in one process
    sys.path.insert(0, str(ROOT / "tests" / "helpers"))
    from dist_worker import global_actions
    from h12env import H12FlatEnvCfg
    from h12env.env import H12VelocityEnv

    cfg = H12FlatEnvCfg()
    cfg.scene.num_envs = world * n_per
    cfg.sim.device = "cuda:0"
    env = H12VelocityEnv(cfg)
    obs, _ = env.reset()
    ref = {"obs": [obs["policy"].cpu().numpy()], "rew": [], "done": []}
    for t in range(steps):
        obs, rew, term, trunc, _ = env.step(global_actions(t, world * n_per).cuda())
        ref["obs"].append(obs["policy"].cpu().numpy())
        ref["rew"].append(rew.cpu().numpy())
        ref["done"].append((term | trunc).to(torch.uint8).cpu().numpy())
    env.close()
    got = np.load(tmp_path / "rollout.npz")
    for k in ("obs", "rew", "done"):
        np.testing.assert_array_equal(got[k], np.stack(ref[k]), err_msg=k)
    assert got["done"].any()  # some episodes end inside the window

    # ---- one PPO iteration: identical parameters on both ranks
    p = [np.load(tmp_path / f"params_{r}.npz") for r in range(world)]
    np.testing.assert_array_equal(p[0]["before"], p[1]["before"])
    np.testing.assert_array_equal(p[0]["after"], p[1]["after"])
    assert np.isfinite(p[0]["after"]).all()
    assert not np.array_equal(p[0]["before"], p[0]["after"])
