#!/usr/bin/env python3
"""Benchmark: env-steps/s of Isaac-Velocity-Flat-H12_12dof-v0 random-action rollouts, 4096 envs per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

One step = one ManagerBasedRLEnv.step of every env on the GPU (4 physics steps of one implicit
integration step each, delayed PD, contact, sensor, rewards, terminations, resets, commands,
450-float observations).  Actions ~ N(0,1) are pre-generated and resident in HBM before timing.
Envs shard across ranks (4096 per GPU, weak scaling, RNG keyed by global env id).  With N > 1 the
timed region is BASELINE config C4: every rank records its shard's rollout compactly (per env-step
the new observation frame, action, reward, done flags: h12env.rollout) and all-gathers it over RCCL,
asynchronously on RCCL's stream, once per rollout of T = 24 steps (--gather-every: smaller chunks)
while it steps the next rollout; --rollout-decode also rebuilds the global (T, N_global, 450)
observation rows on every rank.  The line's c4_rollout_allgather splits env / all-gather / decode
time.  N = 1 is config C2 (no collective; --rollout on records on one GPU).

Steady state: episode_length_buf is randomised first (rsl_rl's init_at_random_ep_len) and a fixed
burn-in (--burn-in, untimed, on top of --warmup) lets falls and time-outs reach their steady rate, so
any --steps window sees representative resets.  After the timed window the workspace snapshot taken
before it is restored and the SAME window is replayed (bit-identical, checked) to count its resets
and to time each kernel with HIP events bound to the dispatches (the interval rocprofv3 reports).

Rank 0 prints ONE JSON line with the contract fields plus `roofline` (dominant kernel) and
`cpu_baseline` (the CPU oracle on host cores, bounded sample).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "h1v2-isaac_amd"))

METRIC = "env-steps/sec at 4096 envs, Velocity-Flat-H12_12dof, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP32_PEAK_TFLOPS = 157.3    # MI355X_MICROARCH.md: peak FP32 vector
CLOCK_GHZ = 2.4             # MI355X_MICROARCH.md: max clock
N_SIMD = 1024               # 256 CUs x 4 SIMDs


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=1000)
    p.add_argument("--warmup", type=int, default=50)
    p.add_argument("--burn-in", type=int, default=300,
                   help="untimed steps after randomising episode_length_buf, before --warmup (steady state)")
    p.add_argument("--envs", type=int, default=None, help="envs per GPU (the metric is quoted at 4096; C5 at 8192)")
    p.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--pmc-file", type=str, default=None,
                   help="tools/profile.sh summary with per-launch HBM bytes (default profiles/latest_pmc.json)")
    p.add_argument("--profile-only", action="store_true", help="timed loop only (for rocprofv3 runs)")
    p.add_argument("--mode", choices=("env", "train"), default="env",
                   help="env: the metric (random-action rollout); train: BASELINE configs C3/C4 (PPO iterations "
                        "of the train.py runner, rollout all-gathered over RCCL when N > 1)")
    p.add_argument("--iterations", type=int, default=5, help="train mode: timed PPO iterations")
    p.add_argument("--precision", choices=("fp32", "bf16"), default="fp32", help="train mode: learning-phase GEMM precision")
    p.add_argument("--tunableop", action="store_true",
                   help="train mode: PyTorch TunableOp GEMM selection for the learner (opt-in: the timed selection can "
                        "differ between runs and ranks, so runs are not bit-reproducible; h12env.ppo.enable_tunable_gemm)")
    p.add_argument("--task", choices=("flat", "rough", "c5", "rsl", "cat"), default="flat",
                   help="flat: the metric's task; rough: Isaac-Velocity-Rough-H12_12dof-v0; c5: BASELINE config C5 "
                        "(rough + per-env friction / torso mass, 8192 envs unless --envs); rsl: "
                        "Isaac-Velocity-Rsl-H12_12dof-v0; cat: Isaac-Velocity-CaT-Flat-H12_12dof-v0")
    p.add_argument("--dist-backend", choices=("nccl", "gloo"), default="nccl",
                   help="process-group backend for N > 1 (nccl = RCCL over xGMI; gloo only to rehearse several "
                        "ranks on one GPU: rank r uses GPU r mod device_count)")
    p.add_argument("--decimation", type=int, default=None, help="experiment override (not the metric config)")
    p.add_argument("--inner-steps", type=int, default=None, help="experiment override (not the metric config)")
    p.add_argument("--explicit-penalty", action="store_true",
                   help="experiment: round-1 explicit penalty contact (use with --inner-steps 2)")
    p.add_argument("--no-self-collision", action="store_true", help="experiment: legs do not collide (not the metric)")
    p.add_argument("--rollout", choices=("auto", "on", "off"), default="auto",
                   help="BASELINE config C4: record the compact rollout (frame, action, reward, dones per env-step) and "
                        "all-gather it over the ranks (asynchronous RCCL collective per rollout, or per --gather-every "
                        "steps) inside the timed region (auto: on when N > 1 for the flat / rsl tasks, whose rows the "
                        "records rebuild; N = 1 is config C2, the plain rollout)")
    p.add_argument("--rollout-steps", type=int, default=24,
                   help="rollout length T (num_steps_per_env, C12/agents/rsl_rl_ppo_cfg.py:12)")
    p.add_argument("--gather-every", type=int, default=None,
                   help="all-gather chunk length G in env steps (C4; default: the rollout length)")
    p.add_argument("--rollout-decode", action="store_true",
                   help="C4: also rebuild the global (T, N_global, 450) observation rows on every rank after each "
                        "gathered chunk (off: the gathered records are handed over; a learner rebuilds its minibatch rows)")
    p.add_argument("--force-collective", action="store_true",
                   help="test hook: with --rollout on, issue the rollout all-gather even on one rank (a one-rank "
                        "process group, launched by torch.distributed.run): exercises the RCCL code path on one GPU")
    p.add_argument("--dump-rollout", type=str, default=None,
                   help="test hook: rank 0 saves the decoded rows and the gathered records of the timed window (.npz)")
    args = p.parse_args()
    if args.rollout == "on" and args.task not in ROLLOUT_TASKS:
        p.error(f"--rollout on: the compact rollout records rebuild history rows of the flat / rsl layouts only "
                f"(--task {args.task} has {'no history' if args.task in ('rough', 'c5') else 'CaT dones'})")
    if args.dump_rollout and args.steps > args.rollout_steps * (1 if args.rollout_decode else 2):
        # the dump saves the first ring half's records and tail with the latest decoded rows: one rollout's data only
        # while the window has not wrapped the ring (decode: rows of the first rollout only while K <= T)
        p.error("--dump-rollout needs --steps <= rollout length (x2 without --rollout-decode)")
    return args


ROLLOUT_TASKS = ("flat", "rsl")


def kernel_source_sha256() -> str:
    """The key of the ISA / PMC summaries: every kernel source file, headers included (h12env.build.source_sha256)."""
    from h12env.build import source_sha256
    return source_sha256()


def load_pmc(path):
    """Per-launch PMC figures of step_kernel / obs_assemble_kernel from a tools/profile.sh summary, used
    only if they were measured on the current kernel: the same sources (kernel_source_sha256: csrc/*.hip, csrc/*.h, include/*.h), or the same
    device ISA (the summary's isa_sha256 equal to profiles/latest_isa.json's, itself made from the current source):
    HBM bytes (FETCH_SIZE doubled + WRITE_SIZE per MI355X_MICROARCH.md) and the SQ wave / VALU-instruction counts."""
    p = Path(path) if path else ROOT / "profiles" / "latest_pmc.json"
    if not p.exists():
        return {}, None
    d = json.loads(p.read_text())
    if d.get("source_sha256") != kernel_source_sha256():
        isa, _ = load_isa()
        if not (d.get("isa_sha256") and isa.get("isa_sha256") == d["isa_sha256"]):
            return {}, f"{p.name}: stale (kernel source changed)"
    where = p.relative_to(ROOT) if p.resolve().is_relative_to(ROOT) else p
    return d.get("kernels", {}), (f"{where} (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, FETCH doubled "
                                  f"per MI355X_MICROARCH.md; SQ_INSTS_VALU / SQ_WAVES)")


def load_isa():
    """tools/kernel_isa.py --json summary (physics-wave loop VALU count, registers) if it was made from the current
    kernel source."""
    p = ROOT / "profiles" / "latest_isa.json"
    if not p.exists():
        return {}, None
    d = json.loads(p.read_text())
    if d.get("source_sha256") != kernel_source_sha256():
        return {}, f"{p.name}: stale (kernel source changed)"
    return d, f"{p.relative_to(ROOT)} (static ISA, tools/kernel_isa.py --json)"


def cpu_model() -> str:
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def usable_cpus() -> dict:
    """The CPUs this process may actually run on: its affinity mask and the cgroup CPU quota (cpu.max), whichever is
    smaller -- os.cpu_count() is the whole machine's."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if q != "max":
            quota = float(q) / float(period)
    except (OSError, ValueError):
        pass
    usable = max(1, min(aff, int(quota) if quota else aff))
    return {"affinity": aff, "cgroup_quota": quota, "usable": usable}


def cpu_baseline(seconds: float):
    """The CPU oracle (C, fp64, OpenMP over envs) on this host, bounded sample of the same workload."""
    import numpy as np

    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle as O
    from h12env import H12FlatEnvCfg
    from h12env.model import build_model

    avail = usable_cpus()
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or avail["usable"]
    threads = max(1, min(threads, avail["usable"]))
    n = 4096
    cfg = H12FlatEnvCfg()
    cfg.scene.num_envs = n
    env = O.OracleEnv(build_model(), cfg.to_c(), n)
    env.reset()
    rng = np.random.default_rng(0)
    acts = rng.normal(size=(8, n, 12)).astype(np.float32)
    env.step(acts[0], 1, n_threads=threads)  # warm
    t0 = time.perf_counter()
    steps = 0
    while time.perf_counter() - t0 < seconds:
        env.step(acts[steps % 8], steps + 2, n_threads=threads)
        steps += 1
    dt = time.perf_counter() - t0
    # BASELINE config C1: the sim2sim MuJoCo loop, one env on one core -- 1000 policy steps of 20 substeps
    # (dt 1 ms, PD every substep, MJCF clamps; oracle MuJoCo mode, free base with ground contact)
    from h12env.cfg import mujoco_cfg

    mc = mujoco_cfg().to_c()
    model = build_model()
    s = np.zeros(37)
    s[2], s[3] = 1.05, 1.0
    s[13:25] = np.asarray(model.q_default)
    q0 = np.asarray(model.q_default)
    t1 = time.perf_counter()
    for k in range(1000):
        q_ref = q0 + 0.25 * rng.normal(size=12)  # q_ref = q0 + 0.25 a, a ~ N(0, 1)
        s, _ = O.mujoco_rollout(model, mc, s, q_ref, 20, contact=True, algo=1)
    dt1 = time.perf_counter() - t1
    mujoco = {"value": 1000 / dt1, "unit": "env-steps/s", "cores": 1,
              "sample": "C1: oracle MuJoCo mode (sim2sim semantics), 1 env x 1000 policy steps x 20 substeps, "
                        f"q_ref = q0 + 0.25 a with a ~ N(0, 1) per policy step, ground contact ({dt1:.2f} s)"}
    return {"value": n * steps / dt, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(), "host_cpus": os.cpu_count(), "cpus_available": avail,
            "single_env_sim2sim": mujoco,
            "sample": f"oracle/h12_oracle.c (fp64, OpenMP) on {n} envs x {steps} env steps "
                      f"({dt:.1f} s) of the same random-action Flat-H12 workload, {threads} host threads"}


def train_mode(args, world, rank, dev, torch, dist):
    """C3 / C4: PPO iterations (24 env steps per env + 5 epochs x 4 minibatches) of the rsl_rl-style
    runner that scripts/train.py drives, with the agent cfg of the Flat task."""
    sys.path.insert(0, str(ROOT / "h1v2-isaac_amd" / "shims"))
    from biped_tasks.tasks.agents import H12_12dof_FlatPPORunnerCfg
    from h12env import H12FlatEnvCfg
    from h12env.env import H12VelocityEnv
    from h12env.ppo import OnPolicyRunner
    from isaaclab_rl.rsl_rl import RslRlVecEnvWrapper

    cfg = H12FlatEnvCfg()
    cfg.scene.num_envs = args.envs
    cfg.sim.device = str(dev)
    env = RslRlVecEnvWrapper(H12VelocityEnv(cfg, env_offset=rank * args.envs))
    agent = H12_12dof_FlatPPORunnerCfg(device=str(dev))
    tcfg = agent.to_dict()
    tcfg["algorithm"]["precision"] = args.precision
    if args.tunableop:
        os.environ["H12_TUNABLEOP"] = "1"
    runner = OnPolicyRunner(env, tcfg, log_dir=None, device=str(dev))
    import io
    import contextlib

    with contextlib.redirect_stdout(io.StringIO()):
        runner.learn(max(1, args.warmup // 25), init_at_random_ep_len=True)
    coll = learn = 0.0
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.iterations):
        with contextlib.redirect_stdout(io.StringIO()):
            runner.learn(1)
        st = runner.last_iteration_stats
        coll += st["Perf/collection_time"]
        learn += st["Perf/learning_time"]
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt, coll, learn], device=dev)
    if world > 1:
        from h12env import distributed as D

        D.all_reduce(t, op=dist.ReduceOp.MAX)
    dt, coll, learn = (float(x) for x in t.tolist())
    steps = world * args.envs * agent.num_steps_per_env * args.iterations
    if rank == 0:
        print(json.dumps({
            "metric": "PPO env-steps/sec (train.py loop, collection + learning), Velocity-Flat-H12_12dof",
            "value": steps / dt, "unit": "env-steps/s", "n_gpus": world, "steps": args.iterations,
            "warmup": max(1, args.warmup // 25), "ms_per_step": 1e3 * dt / args.iterations, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32" if args.precision == "fp32" else "f32 env / bf16 learner",
            "data": "synthetic: on-policy rollouts",
            "config": {"workload": "C3/C4: PPO iterations, 24 steps/env/iter, 5 epochs x 4 minibatches, "
                                   "MLP 512-256-128", "envs_per_gpu": args.envs, "global_envs": world * args.envs,
                       "parallelism": f"env-shard x{world}" + (" + RCCL rollout all-gather + grad all-reduce"
                                                               if world > 1 else "")},
            "collection_env_steps_per_s": steps / coll, "collection_s_per_iter": coll / args.iterations,
            "learning_s_per_iter": learn / args.iterations, "tunableop": bool(args.tunableop)}), flush=True)
    env.close()


def main():
    args = parse()
    if args.envs is None:
        args.envs = 8192 if args.task == "c5" else 4096
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device(f"cuda:{local % max(1, torch.cuda.device_count())}")
    if world > 1 or args.force_collective:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    torch.cuda.set_device(dev)

    if args.mode == "train":
        train_mode(args, world, rank, dev, torch, dist)
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    from h12env import H12FlatEnvCfg
    from h12env.cfg import H12CaTEnvCfg, H12RoughEnvCfg, H12RslEnvCfg, c5_cfg
    from h12env.env import H12VelocityEnv

    n = args.envs
    if args.task == "flat":
        cfg = H12FlatEnvCfg()
    elif args.task == "rough":
        cfg = H12RoughEnvCfg()
    elif args.task == "rsl":
        cfg = H12RslEnvCfg()
    elif args.task == "cat":
        cfg = H12CaTEnvCfg()
    else:
        cfg = c5_cfg()
    cfg.scene.num_envs = n
    cfg.sim.device = str(dev)
    if args.decimation:
        cfg.decimation = args.decimation
    if args.inner_steps:
        cfg.sim.inner_steps = args.inner_steps
    if args.explicit_penalty:
        cfg.sim.implicit_penalty = False
    if args.no_self_collision:
        cfg.sim.self_collision = False
    env = H12VelocityEnv(cfg, env_offset=rank * n)
    env.reset()
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    K, W, B = args.steps, args.warmup, args.burn_in
    pool = min(K + W + B, 256)
    actions = torch.randn(pool, n, 12, device=dev, generator=g)  # resident in HBM before timing
    # rsl_rl OnPolicyRunner.learn(init_at_random_ep_len=True): spread the time-outs over the episode
    env.episode_length_buf = torch.randint(0, env.max_episode_length, (n,), device=dev, generator=g,
                                           dtype=torch.int32)
    for i in range(B + W):
        env.step(actions[i % pool])

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    rollout = args.rollout == "on" or (args.rollout == "auto" and world > 1 and args.task in ROLLOUT_TASKS)
    rg = None
    if rollout:  # C4: compact rollout records all-gathered on a side stream and decoded on every rank
        from h12env import distributed as D
        from h12env.rollout import RolloutGather, RolloutRecorder

        rec = RolloutRecorder(n, args.rollout_steps, dev, env.obs_dim // 45)
        tail = torch.empty(world * n, env.obs_dim, device=dev)  # every env's row before the first step
        if world > 1:
            D.all_gather_into_tensor(tail, env.get_observations()["policy"].contiguous())
        else:
            tail.copy_(env.get_observations()["policy"])
        # no timing events inside the timed window (each event record costs host time comparable to a step); the
        # all-gather / decode split is measured in an untimed pass right after it
        rg = RolloutGather(rec, world, args.gather_every, tail, timing=False, decode=args.rollout_decode,
                           collective=args.force_collective)
        pool_off = B + W  # actions[pool_off + i] is the action of timed step i
        env.bind_rollout(rec)

        def put_actions(i_end):
            def f(s0, s1):  # the chunk's actions (pool slices) into ring slots [s0, s1), one copy when contiguous
                span = s1 - s0
                a0 = (i_end - span) % pool
                if a0 + span <= pool:
                    rec.actions[s0:s1].copy_(actions[a0:a0 + span])
                else:
                    k = pool - a0
                    rec.actions[s0:s0 + k].copy_(actions[a0:])
                    rec.actions[s0 + k:s1].copy_(actions[:span - k])
            return f

    snap = env.snapshot()  # replayed below (reset count + kernel timing of the same window); copied before the barrier
    barrier()
    # the env-stream span of the rollout path (C4 split); no event records in the plain timed window (each costs
    # host time, which a 20-step window does not amortise)
    ev_c = [torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)] if rg is not None else None
    t0 = time.perf_counter()
    if ev_c:
        ev_c[0].record()
    for i in range(K):
        if rg is None:
            env.step(actions[(B + W + i) % pool])
            continue
        rg.before_step()
        tc = rec.t
        env.step(actions[(pool_off + i) % pool])
        rg.after_step(tc, put_actions(pool_off + i + 1))
    if rg is not None and K > 0:
        rg.flush(rec.t, put_actions(pool_off + K))
    if ev_c:
        ev_c[1].record()
    if rg is not None:
        rg.wait()
    barrier()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], device=dev)
    if world > 1:
        from h12env import distributed as D

        D.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    c4 = None
    if rg is not None and args.dump_rollout and rank == 0:
        import numpy as np

        te = min(K, args.rollout_steps)
        if not args.rollout_decode:  # the check rebuilds the rows of the gathered records once, untimed
            from h12env.rollout import decode as _decode

            _decode(rg.records(0), world, n, te, rg.G, rec.history, 0, te, rg.tail, rg.obs[:te])
        np.savez(args.dump_rollout, obs=rg.obs[:te].cpu().numpy(), gathered=rg.records(0).cpu().numpy(),
                 tail=rg.tail.cpu().numpy(), off=np.array(rec.off), step_bytes=rec.step_bytes, T=te, G=rg.G,
                 n=n, world=world, burn_in=B, warmup=W, steps=K, pool=pool)
    final_obs = env.get_observations()["policy"].clone()
    if rg is not None and not args.profile_only:
        # the split pass (untimed, after the window): two more rollouts with an event pair around every chunk's
        # gather and decode on the comm stream
        chunks_timed = rg.seq
        rg.timing = True
        for i in range(2 * args.rollout_steps):
            rg.before_step()
            tc = rec.t
            env.step(actions[(pool_off + K + i) % pool])
            rg.after_step(tc, put_actions(pool_off + K + i + 1))
        rg.wait()
        st = rg.stats()
        split_iters = 2
        env_span = ev_c[0].elapsed_time(ev_c[1])
        iters = K / args.rollout_steps
        rec_b = rec.step_bytes
        recv = st["gathered_bytes"] / split_iters * (world - 1) / world  # bytes each rank receives from the others
        c4 = {"rollout_steps": args.rollout_steps, "gather_every": rg.G, "chunks": chunks_timed,
              "split_pass_chunks": st["chunks"],
              "record_bytes_per_env_step": rec_b / n, "full_row_bytes_per_env_step": (env.obs_dim + 12 + 2) * 4,
              "gathered_bytes_per_iter": st["gathered_bytes"] / split_iters, "received_bytes_per_rank_per_iter": recv,
              "env_stream_ms_per_iter": env_span / iters, "allgather_ms_per_iter": st["gather_ms"] / split_iters,
              "decode_ms_per_iter": st["decode_ms"] / split_iters, "ms_per_iter": 1e3 * dt / iters,
              "allgather_algbw_gbs": st["gathered_bytes"] / (st["gather_ms"] * 1e-3) / 1e9 if st["gather_ms"] else None,
              "allgather_busbw_gbs": recv * split_iters / (st["gather_ms"] * 1e-3) / 1e9 if st["gather_ms"] and world > 1 else None,
              "rows_rebuilt": bool(args.rollout_decode),
              "decoded_rows_bytes_per_iter": args.rollout_steps * world * n * env.obs_dim * 4 if args.rollout_decode else 0,
              "decode_gbs": (args.rollout_decode and st["chunks"] and st["decode_ms"] and
                             rg.G * world * n * env.obs_dim * 4 * st["chunks"] / (st["decode_ms"] * 1e-3) / 1e9) or None,
              "overlap": "one asynchronous RCCL all-gather per chunk (default: per rollout) on RCCL's stream, concurrent "
                         "with the next rollout's env steps into the other half of a 2T-record ring; the split above "
                         "comes from an untimed pass that serialises each gather between an event pair",
              "backend": (args.dist_backend if rg.coll else "none (N = 1: the records are read in place)")}
        if not rg.coll:  # nothing is gathered: no all-gather time or bandwidth to report
            c4.update(allgather_ms_per_iter=None, allgather_algbw_gbs=None, gathered_bytes_per_iter=0)
        env.unbind_rollout()
    if args.profile_only:
        if rank == 0:
            print(json.dumps({"profile_only": True, "ms_per_step": 1e3 * dt / K}))
        return

    # replay of the timed window from the snapshot: count its resets and time each launch with HIP
    # events bound to the dispatches (kernel begin / end, as rocprofv3 reports them); the replay must
    # reproduce the timed window bit for bit
    env.restore(snap)
    resets = torch.zeros((), dtype=torch.int64, device=dev)
    env.set_kernel_timing(True)
    env_ms = obs_ms = 0.0
    n_timed = 0
    for i in range(K):
        env.step(actions[(B + W + i) % pool])
        resets += (env.reset_terminated | env.reset_time_outs).sum()
        if (i + 1) % 2048 == 0:  # the library keeps at most 4096 timed steps
            a_ms, b_ms, c = env.kernel_times()
            env_ms, obs_ms, n_timed = env_ms + a_ms, obs_ms + b_ms, n_timed + c
    a_ms, b_ms, c = env.kernel_times()
    env_ms, obs_ms, n_timed = env_ms + a_ms, obs_ms + b_ms, n_timed + c
    env.set_kernel_timing(False)
    replay_exact = bool(torch.equal(env.get_observations()["policy"], final_obs))
    resets_in_window = int(resets.item())
    kern_ms_avg = env_ms / n_timed
    obs_ms_avg = obs_ms / n_timed
    bytes_env, flops_env = env.kernel_cost(0)
    obs_bytes_env, _ = env.kernel_cost(1)
    step_bytes_env, _ = env.step_cost()

    value = world * n * K / dt
    if rank == 0:
        achieved = bytes_env * n / (kern_ms_avg * 1e-3) / 1e9
        pmc, pmc_src = load_pmc(args.pmc_file)
        if (args.task != "flat" or args.envs != 4096 or args.no_self_collision or args.decimation is not None
                or args.inner_steps is not None or args.explicit_penalty):  # tools/profile.sh: the default workload
            pmc, pmc_src = {}, "not collected for this workload (tools/profile.sh profiles the default flat line)"
        traffic = pmc.get("step_kernel", {}).get("hbm_bytes_per_launch")
        # algorithmic read / write split of the fused Flat step (h12env_kernel_cost(0): state fields read and written,
        # actions read, reward / flags / applied torque / foot force written, the row's H-1 old frames read and its H
        # frames written) beside the PMC's
        split = None
        if traffic is not None and env.obs_fused:
            row = float(env.obs_dim)  # floats per observation row (H frames of 45)
            fields4 = (bytes_env - 110.0 - (2.0 * row - 45.0) * 4.0) / 2.0
            rd = fields4 + 48.0 + (row - 45.0) * 4.0
            k = pmc.get("step_kernel", {})
            split = {"algorithmic_read": rd * n, "algorithmic_write": (bytes_env - rd) * n,
                     "pmc_read": k.get("hbm_read_bytes_per_launch"), "pmc_write": k.get("hbm_write_bytes_per_launch")}
        # kernel 1 of the timing / cost pairs: the observation assembly kernel, or -- when step_kernel assembles the
        # rows itself (env.obs_fused) -- the deferred episode-log fold, launched once per <= 32 steps
        fused = env.obs_fused
        sec_kernel = "log_flush_kernel" if fused else "obs_assemble_kernel"
        obs_traffic = None if fused else pmc.get(sec_kernel, {}).get("hbm_bytes_per_launch")
        # VALU issue roofline of step_kernel: one wave per SIMD issues at most one VALU instruction per
        # 4 cycles (MI355X_MICROARCH.md, 'vector-instruction ISSUE cost', one wave's stream on one SIMD), so
        # the kernel's floor is (VALU instructions per wave) x 4 cycles at the 2.4 GHz max clock
        sq = pmc.get("step_kernel", {}).get("SQ", {})
        isa, isa_src = load_isa()
        issue = None
        if isa and args.task == "flat" and n == 4096 and not (args.no_self_collision or args.decimation
                                                                or args.inner_steps or args.explicit_penalty):
            # the step time is the PHYSICS wave's serial chain (the helper / self-contact waves of a block finish
            # inside its window): its physics-step loop runs decimation x inner_steps times per env step
            # (tools/kernel_isa.py --json, static ISA of this kernel source); the loads / rewards / reset / stores
            # around the loop are not counted, so the floor is a lower bound
            per_step = isa["physics_step_loop"]["valu"] * cfg.decimation * cfg.sim.inner_steps
            floor_ms = per_step * 4.0 / (CLOCK_GHZ * 1e9) * 1e3
            issue = {"bound": "valu-issue, one wave per SIMD (the physics wave's chain)",
                     "physics_wave_loop_valu_per_env_step": per_step,
                     "floor_ms": floor_ms, "frac": floor_ms / kern_ms_avg, "isa_source": isa_src}
            if sq.get("SQ_WAVES") and sq.get("SQ_INSTS_VALU"):  # PMC: all three waves of every block averaged
                issue.update(pmc_valu_insts_per_wave_all_roles=sq["SQ_INSTS_VALU"] / sq["SQ_WAVES"],
                             waves=sq["SQ_WAVES"], simds_in_use_frac=sq["SQ_WAVES"] / N_SIMD,
                             wait_frac=sq.get("SQ_WAIT_ANY", 0.0) / sq.get("SQ_WAVE_CYCLES", 1.0), pmc_source=pmc_src)
        metric, workload = METRIC, "Isaac-Velocity-Flat-H12_12dof-v0 random-action rollout, 4096 envs per MI355X"
        if args.task in ("rsl", "cat"):
            tid = {"rsl": "Rsl-H12_12dof", "cat": "CaT-Flat-H12_12dof"}[args.task]
            metric = f"env-steps/sec at {n} envs, Velocity-{tid}"
            workload = f"Isaac-Velocity-{tid}-v0 random-action rollout, {n} envs per MI355X"
        elif args.task != "flat":
            metric = f"env-steps/sec at {n} envs, Velocity-Rough-H12_12dof" + (" + friction/mass randomisation (C5)"
                                                                               if args.task == "c5" else "")
            workload = f"Isaac-Velocity-Rough-H12_12dof-v0 random-action rollout, {n} envs per MI355X" + (
                ", CaT startup randomisation (BASELINE C5)" if args.task == "c5" else "")
        out = {
            "metric": metric,
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": 1e3 * dt / K,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: N(0,1) random actions, reset distribution of the Flat task (seeded)",
            "config": {
                "workload": workload,
                "envs_per_gpu": n,
                "global_envs": n * world,
                "decimation": cfg.decimation,
                "physics_dt": cfg.sim.dt,
                "inner_steps": cfg.sim.inner_steps,
                "implicit_penalty": bool(cfg.sim.implicit_penalty),
                "parallelism": f"env-shard x{world}" + (f" + RCCL all-gather of the rollout every {rg.G} steps"
                                                         if rg is not None and world > 1 else ""),
            },
            "c4_rollout_allgather": c4 if c4 is not None or args.task in ROLLOUT_TASKS else {
                "skipped": f"--task {args.task}: the compact records rebuild flat / rsl history rows only"},
            "burn_in": B,
            "resets_in_window": resets_in_window,
            "replay_bit_exact": replay_exact,
            "roofline": {
                # the contract prices the dominant kernel against HBM (the north_star's roofline); the
                # binding limit of step_kernel at 4096 envs is VALU issue latency ("issue" below)
                "bound": "hbm",
                "binding": ("valu-issue latency of the physics wave's serial chain (one wave per SIMD; 4096 envs fill "
                            "128 of the 256 CUs with one 4-wave block each)"),
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "traffic_split": split,
                "kernel": "step_kernel",
                "kernel_ms_avg": kern_ms_avg,
                "kernel_timing": "HIP event pair bound to each dispatch (hipExtLaunchKernelGGL), replayed window",
                "algorithmic_bytes_per_launch": bytes_env * n,
                "issue": issue,
                "traffic_source": pmc_src,
                "valu_flops_per_env_step": flops_env,
                "valu_tflops": flops_env * n / (kern_ms_avg * 1e-3) / 1e12,
                "valu_frac": flops_env * n / (kern_ms_avg * 1e-3) / 1e12 / FP32_PEAK_TFLOPS,
                "obs_assembly": "fused into step_kernel" if fused else "obs_assemble_kernel",
                "secondary": {
                    "kernel": sec_kernel,
                    "bound": "hbm",
                    "kernel_ms_avg": obs_ms_avg,
                    "timing": ("per env step: the launches' time summed over the window / steps (one launch folds "
                               "the steps since the last one)") if fused else "per launch (one per env step)",
                    "achieved": obs_bytes_env * n / (obs_ms_avg * 1e-3) / 1e9 if obs_ms_avg > 0 else None,
                    "frac": obs_bytes_env * n / (obs_ms_avg * 1e-3) / 1e9 / HBM_PEAK_GBS if obs_ms_avg > 0 else None,
                    "traffic": obs_traffic,
                },
                "step_bytes_per_env": step_bytes_env,
                "step_achieved_gbs": step_bytes_env * n * K / dt / 1e9,
            },
            "cpu_baseline": None,
        }
        if not args.no_cpu_baseline and args.task == "flat":
            out["cpu_baseline"] = cpu_baseline(args.cpu_baseline_seconds)
        print(json.dumps(out), flush=True)
    env.close()
    if world > 1 or args.force_collective:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
