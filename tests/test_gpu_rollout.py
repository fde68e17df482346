"""GPU: the compact rollout records and their all-gather (BASELINE config C4; h12env.rollout, include/h12env.h
"Rollout records").

* single process (world 1: the records are read in place): the HIP row rebuild (h12env_rollout_decode) reproduces
  every observation row the env returned, bit for bit, over two whole iterations (the second one's tail aliases
  the first one's last row; the two halves of the recorder's ring) and a flushed partial chunk; Flat (history 10) and Rsl (history 6), ragged env counts
  (37: rows not float4-aligned) and a chunk length that does not divide T; the frames in the records are the newest
  slots of the returned rows, and the reward / done tensors the step returned are the records themselves;
* two ranks of bench.py's N > 1 path (child processes, both on cuda:0, gloo: RCCL refuses two ranks on one device):
  the line carries the c4_rollout_allgather split, and the decoded rows and gathered records equal one process
  stepping all 2N envs with the same actions, bit for bit."""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

from rollout_ref import decode_ref, unpack

ROOT = Path(__file__).resolve().parents[1]
pytestmark = pytest.mark.gpu


def _env(cfg, n):
    from h12env.env import H12VelocityEnv

    cfg.scene.num_envs = n
    cfg.sim.device = "cuda:0"
    env = H12VelocityEnv(cfg)
    env.reset()
    # random episode lengths: time-outs inside the window, plus natural falls
    g = torch.Generator(device="cpu").manual_seed(n)
    env.episode_length_buf = torch.randint(900, env.max_episode_length, (n,), generator=g, dtype=torch.int32)
    return env


@pytest.mark.parametrize("task,n", [("flat", 37), ("flat", 256), ("rsl", 64)])
def test_decoded_rows_equal_env_rows(gpu, task, n):
    from h12env import H12FlatEnvCfg
    from h12env.cfg import H12RslEnvCfg
    from h12env.rollout import RolloutGather, RolloutRecorder

    env = _env(H12FlatEnvCfg() if task == "flat" else H12RslEnvCfg(), n)
    H = env.obs_dim // 45
    T, G = 24, 5
    rec = RolloutRecorder(n, T, gpu, H)
    rg = RolloutGather(rec, 1, G, env.get_observations()["policy"].clone())
    env.bind_rollout(rec)
    gen = torch.Generator(device="cpu").manual_seed(7)
    rows, dones = [], 0
    for it in range(3):
        steps = T if it < 2 else 7
        rows = []
        for t in range(steps):
            rg.before_step()
            tc = rec.t
            assert tc == (it % 2) * T + t  # the recorder's ring of 2T slots
            a = torch.randn(n, 12, generator=gen).to(gpu)
            obs, rew, term, trunc, _ = env.step(a)
            rec.actions[tc].copy_(a)
            assert rew.data_ptr() == rec.rewards[tc].data_ptr() and term.data_ptr() == rec.terminated[tc].data_ptr()
            rows.append(obs["policy"].clone())
            # the frame in the record is the newest slot of every term of the returned row
            o = obs["policy"].view(n, -1)
            newest = torch.cat([o[:, 3 * H * k + 3 * (H - 1):3 * H * k + 3 * H] for k in range(3)] +
                               [o[:, 9 * H + 12 * H * k + 12 * (H - 1):9 * H + 12 * H * (k + 1)] for k in range(3)], 1)
            assert torch.equal(rec.frames[tc], newest)
            dones += int((term | trunc).sum())
            rg.after_step(tc)
        if it == 2:
            rg.flush(rec.t)
        rg.wait()
        torch.cuda.synchronize()
        got = rg.obs[:steps]
        want = torch.stack(rows)
        assert torch.equal(got, want), (it, (got != want).nonzero()[:5])
    assert dones > 0
    with pytest.raises(RuntimeError):  # only step() writes records: a reset mid-rollout would desync the rebuild
        env.reset()
    with pytest.raises(RuntimeError):
        env.observe()
    env.unbind_rollout()
    env.reset()
    env.close()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(600)
def test_two_rank_bench_rollout_allgather(tmp_path):
    world, n, K, B, W = 2, 64, 22, 40, 3
    port = _free_port()
    dump = tmp_path / "rollout.npz"
    procs = []
    for rank in range(world):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                   LOCAL_RANK=str(rank))
        log = open(tmp_path / f"rank{rank}.log", "w")
        cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", str(world), "--dist-backend", "gloo", "--envs", str(n),
               "--steps", str(K), "--warmup", str(W), "--burn-in", str(B), "--gather-every", "4",
               "--no-cpu-baseline", "--rollout-decode", "--dump-rollout", str(dump)]
        procs.append((subprocess.Popen(cmd, env=env, stdout=log, stderr=subprocess.STDOUT, cwd=str(ROOT)), log))
    try:
        for p, _ in procs:
            p.wait(timeout=540)
    finally:
        for p, log in procs:
            if p.poll() is None:
                p.kill()
            log.close()
    for rank, (p, _) in enumerate(procs):
        assert p.returncode == 0, (tmp_path / f"rank{rank}.log").read_text()[-3000:]
    line = [ln for ln in (tmp_path / "rank0.log").read_text().splitlines() if ln.startswith("{")][-1]
    out = json.loads(line)
    c4 = out["c4_rollout_allgather"]
    assert out["n_gpus"] == world and c4["chunks"] == 6 and c4["gather_every"] == 4
    for k in ("env_stream_ms_per_iter", "allgather_ms_per_iter", "decode_ms_per_iter", "gathered_bytes_per_iter",
              "received_bytes_per_rank_per_iter"):
        assert c4[k] is not None and c4[k] > 0, k
    assert "all-gather" in out["config"]["parallelism"]

    # ---- the same 2N envs in one process, same actions (each rank's generator) and episode lengths
    d = np.load(dump)
    from h12env import H12FlatEnvCfg
    from h12env.env import H12VelocityEnv

    cfg = H12FlatEnvCfg()
    cfg.scene.num_envs = world * n
    cfg.sim.device = "cuda:0"
    env = H12VelocityEnv(cfg)
    env.reset()
    pool = int(d["pool"])
    acts, eplen = [], []
    for r in range(world):
        g = torch.Generator(device="cuda:0").manual_seed(1234 + r)
        acts.append(torch.randn(pool, n, 12, device="cuda:0", generator=g))
        eplen.append(torch.randint(0, env.max_episode_length, (n,), device="cuda:0", generator=g, dtype=torch.int32))
    acts = torch.cat(acts, 1)
    env.episode_length_buf = torch.cat(eplen)
    for i in range(B + W):
        env.step(acts[i % pool])
    tail = env.get_observations()["policy"].clone()
    rows, rew, term, trunc, used = [], [], [], [], []
    for i in range(K):
        a = acts[(B + W + i) % pool]
        obs, r_, te, tr, _ = env.step(a)
        rows.append(obs["policy"].clone())
        rew.append(r_.clone())
        term.append(te.clone())
        trunc.append(tr.clone())
        used.append(a)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(d["tail"], tail.cpu().numpy())
    np.testing.assert_array_equal(d["obs"], torch.stack(rows).cpu().numpy())
    g = unpack(d["gathered"], world, n, int(d["T"]), int(d["G"]), list(d["off"]), int(d["step_bytes"]))
    np.testing.assert_array_equal(g["rewards"], torch.stack(rew).cpu().numpy())
    np.testing.assert_array_equal(g["terminated"], torch.stack(term).cpu().numpy().astype(np.uint8))
    np.testing.assert_array_equal(g["truncated"], torch.stack(trunc).cpu().numpy().astype(np.uint8))
    np.testing.assert_array_equal(g["actions"], torch.stack(used).cpu().numpy())
    # and the numpy restatement of the rebuild agrees with the HIP one on the gathered records
    done = g["terminated"] | g["truncated"]
    np.testing.assert_array_equal(decode_ref(g["frames"], done, d["tail"], 10), d["obs"])
    assert done.any()
    env.close()


@pytest.mark.timeout(400)
def test_rccl_rollout_allgather_one_rank(tmp_path):
    """The RCCL code path of the rollout all-gather (asynchronous all_gather_into_tensor on RCCL's stream, work.wait
    before a ring half is rewritten), on a one-rank NCCL process group (bench.py --force-collective): the 8-GPU run
    is the driver's, this keeps the same calls exercised on one GPU.  The line must carry the split, the window must
    replay bit-exactly, and the gathered records of the first rollout must rebuild the rows the env returned."""
    port = _free_port()
    dump = tmp_path / "rollout.npz"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1", "--master-addr",
           "127.0.0.1", "--master-port", str(port), str(ROOT / "bench.py"), "--gpus", "1", "--rollout", "on",
           "--force-collective", "--envs", "64", "--steps", "30", "--warmup", "3", "--burn-in", "20",
           "--gather-every", "8", "--no-cpu-baseline", "--dump-rollout", str(dump)]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run(cmd, env=env, cwd=str(ROOT), capture_output=True, text=True, timeout=360)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    c4 = out["c4_rollout_allgather"]
    assert out["replay_bit_exact"] and c4["backend"] == "nccl"
    assert c4["allgather_ms_per_iter"] is not None and c4["allgather_ms_per_iter"] > 0
    assert c4["gathered_bytes_per_iter"] > 0 and c4["chunks"] == 4
    d = np.load(dump)
    g = unpack(d["gathered"], 1, 64, int(d["T"]), int(d["G"]), list(d["off"]), int(d["step_bytes"]))
    done = g["terminated"] | g["truncated"]
    np.testing.assert_array_equal(decode_ref(g["frames"], done, d["tail"], 10), d["obs"])


@pytest.mark.timeout(900)
def test_c4_size_eight_rank_rehearsal(tmp_path):
    """BASELINE config C4 at its size, rehearsed on one GPU: 8 ranks of bench.py's N > 1 path (child processes, all
    on cuda:0, gloo: RCCL refuses several ranks on one device) x 4096 envs = 32 768 global envs (4096 per GPU,
    V/velocity_env_cfg.py:288), one full rollout of T = 24 steps (C12/agents/rsl_rl_ppo_cfg.py:12) recorded, all-gathered
    as one chunk and decoded into the global (24, 32768, 450) rows on every rank.  The gathered records and the
    decoded rows must equal one process stepping all 32 768 envs with the same actions, bit for bit.  (gloo stages
    the gather through the host, so no bandwidth figure is claimed; the ranks rendezvous in init_process_group before
    any of them touches the GPU.)"""
    world, n, K, B, W = 8, 4096, 24, 40, 3
    port = _free_port()
    dump = tmp_path / "rollout.npz"
    procs = []
    for rank in range(world):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                   LOCAL_RANK=str(rank), OMP_NUM_THREADS="2")
        log = open(tmp_path / f"rank{rank}.log", "w")
        cmd = [sys.executable, "-u", str(ROOT / "bench.py"), "--gpus", str(world), "--dist-backend", "gloo",
               "--envs", str(n), "--steps", str(K), "--warmup", str(W), "--burn-in", str(B), "--rollout", "on",
               "--no-cpu-baseline", "--rollout-decode", "--dump-rollout", str(dump)]
        procs.append((subprocess.Popen(cmd, env=env, stdout=log, stderr=subprocess.STDOUT, cwd=str(ROOT)), log))
    try:
        for p, _ in procs:
            p.wait(timeout=780)
    finally:
        for p, log in procs:
            if p.poll() is None:
                p.kill()
            log.close()
    for rank, (p, _) in enumerate(procs):
        assert p.returncode == 0, (tmp_path / f"rank{rank}.log").read_text()[-3000:]
    line = [ln for ln in (tmp_path / "rank0.log").read_text().splitlines() if ln.startswith("{")][-1]
    out = json.loads(line)
    print("C4 rehearsal line:", line[:400])
    c4 = out["c4_rollout_allgather"]
    assert out["n_gpus"] == world and out["config"]["global_envs"] == world * n
    assert c4["chunks"] == 1 and c4["gather_every"] == K and c4["rows_rebuilt"]
    assert c4["gathered_bytes_per_iter"] == pytest.approx(world * n * c4["record_bytes_per_env_step"] * K)

    d = np.load(dump)
    assert d["obs"].shape == (K, world * n, 450)
    from h12env import H12FlatEnvCfg
    from h12env.env import H12VelocityEnv

    cfg = H12FlatEnvCfg()
    cfg.scene.num_envs = world * n
    cfg.sim.device = "cuda:0"
    env = H12VelocityEnv(cfg)
    env.reset()
    pool = int(d["pool"])
    acts, eplen = [], []
    for r in range(world):  # each rank's generator: actions first, then the episode lengths (bench.py)
        g = torch.Generator(device="cuda:0").manual_seed(1234 + r)
        acts.append(torch.randn(pool, n, 12, device="cuda:0", generator=g))
        eplen.append(torch.randint(0, env.max_episode_length, (n,), device="cuda:0", generator=g, dtype=torch.int32))
    acts = torch.cat(acts, 1)
    env.episode_length_buf = torch.cat(eplen)
    for i in range(B + W):
        env.step(acts[i % pool])
    tail = env.get_observations()["policy"].clone()
    rows = torch.empty(K, world * n, 450, device="cuda:0")
    rew, term, trunc, used = [], [], [], []
    for i in range(K):
        a = acts[(B + W + i) % pool]
        obs, r_, te, tr, _ = env.step(a)
        rows[i].copy_(obs["policy"])
        rew.append(r_.clone())
        term.append(te.clone())
        trunc.append(tr.clone())
        used.append(a)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(d["tail"], tail.cpu().numpy())
    got = torch.from_numpy(d["obs"]).to("cuda:0")
    assert torch.equal(got, rows), (got != rows).nonzero()[:5]
    g = unpack(d["gathered"], world, n, int(d["T"]), int(d["G"]), list(d["off"]), int(d["step_bytes"]))
    np.testing.assert_array_equal(g["rewards"], torch.stack(rew).cpu().numpy())
    np.testing.assert_array_equal(g["terminated"], torch.stack(term).cpu().numpy().astype(np.uint8))
    np.testing.assert_array_equal(g["truncated"], torch.stack(trunc).cpu().numpy().astype(np.uint8))
    np.testing.assert_array_equal(g["actions"], torch.stack(used).cpu().numpy())
    assert (g["terminated"] | g["truncated"]).sum() > 100  # resets inside the rollout (random episode lengths + falls)
    env.close()
