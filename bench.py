#!/usr/bin/env python3
"""Benchmark: env-steps/s of Isaac-Velocity-Flat-H12_12dof-v0 random-action rollouts, 4096 envs per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

One step = one ManagerBasedRLEnv.step of every env on the GPU (4 physics steps x 2 inner integration
steps, delayed PD, contact, sensor, rewards, terminations, resets, commands, 450-float observations).
Actions ~ N(0,1) are pre-generated and resident in HBM before timing.  Envs shard across ranks
(4096 per GPU, weak scaling, RNG keyed by global env id); no collective inside the timed region.

Rank 0 prints ONE JSON line with the contract fields plus `roofline` (dominant kernel, measured with
HIP events on the env's stream) and `cpu_baseline` (the CPU oracle on host cores, bounded sample).
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


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=500)
    p.add_argument("--warmup", type=int, default=50)
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
    return p.parse_args()


def load_pmc(path):
    """HBM bytes per launch of step_kernel / obs_assemble_kernel from a tools/profile.sh summary, used
    only if it was measured on the current kernel source (sha256 of csrc/h12env.hip)."""
    import hashlib
    p = Path(path) if path else ROOT / "profiles" / "latest_pmc.json"
    if not p.exists():
        return None, None, None
    d = json.loads(p.read_text())
    src = hashlib.sha256((ROOT / "h1v2-isaac_amd" / "csrc" / "h12env.hip").read_bytes()).hexdigest()
    if d.get("source_sha256") != src:
        return None, None, f"{p.name}: stale (kernel source changed)"
    k = d.get("kernels", {})
    return (k.get("step_kernel", {}).get("hbm_bytes_per_launch"), k.get("obs_assemble_kernel", {}).get("hbm_bytes_per_launch"),
            f"{p.relative_to(ROOT)} (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, FETCH doubled per MI355X_MICROARCH.md)")


def cpu_baseline(seconds: float):
    """The CPU oracle (C, fp64, OpenMP over envs) on this host, bounded sample of the same workload."""
    import numpy as np

    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle as O
    from h12env import H12FlatEnvCfg
    from h12env.model import build_model

    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    threads = max(1, min(threads, 16))
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
        q_ref = q0 + 0.25 * rng.normal(size=12) * 0.2
        s, _ = O.mujoco_rollout(model, mc, s, q_ref, 20, contact=True, algo=1)
    dt1 = time.perf_counter() - t1
    mujoco = {"value": 1000 / dt1, "unit": "env-steps/s", "cores": 1,
              "sample": "C1: oracle MuJoCo mode (sim2sim semantics), 1 env x 1000 policy steps x 20 substeps, "
                        f"random q_ref, ground contact ({dt1:.2f} s)"}
    return {"value": n * steps / dt, "unit": "env-steps/s", "cores": threads, "kind": "port",
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
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
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
            "learning_s_per_iter": learn / args.iterations}), flush=True)
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
    if world > 1:
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
    env = H12VelocityEnv(cfg, env_offset=rank * n)
    env.reset()
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    K, W = args.steps, args.warmup
    pool = min(K + W, 256)
    actions = torch.randn(pool, n, 12, device=dev, generator=g)  # resident in HBM before timing

    for i in range(W):
        env.step(actions[i % pool])

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    barrier()
    t0 = time.perf_counter()
    for i in range(K):
        env.step(actions[(W + i) % pool])
    barrier()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    if args.profile_only:
        if rank == 0:
            print(json.dumps({"profile_only": True, "ms_per_step": 1e3 * dt / K}))
        return

    # per-launch kernel durations with HIP events recorded by the library on the env's stream around
    # each of its two kernels (separate pass, so the timed region above is not perturbed)
    M = min(K, 200)
    env.set_kernel_timing(True)
    for i in range(M):
        env.step(actions[i % pool])
    env_ms, obs_ms, n_timed = env.kernel_times()
    env.set_kernel_timing(False)
    kern_ms_avg = env_ms / n_timed
    obs_ms_avg = obs_ms / n_timed
    bytes_env, flops_env = env.kernel_cost(0)
    obs_bytes_env, _ = env.kernel_cost(1)
    step_bytes_env, _ = env.step_cost()

    value = world * n * K / dt
    if rank == 0:
        achieved = bytes_env * n / (kern_ms_avg * 1e-3) / 1e9
        traffic, obs_traffic, pmc_src = load_pmc(args.pmc_file)
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
                "parallelism": f"env-shard x{world}",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "kernel": "step_kernel",
                "kernel_ms_avg": kern_ms_avg,
                "algorithmic_bytes_per_launch": bytes_env * n,
                "traffic_source": pmc_src,
                "valu_flops_per_env_step": flops_env,
                "valu_tflops": flops_env * n / (kern_ms_avg * 1e-3) / 1e12,
                "valu_frac": flops_env * n / (kern_ms_avg * 1e-3) / 1e12 / FP32_PEAK_TFLOPS,
                "secondary": {
                    "kernel": "obs_assemble_kernel",
                    "bound": "hbm",
                    "kernel_ms_avg": obs_ms_avg,
                    "achieved": obs_bytes_env * n / (obs_ms_avg * 1e-3) / 1e9,
                    "frac": obs_bytes_env * n / (obs_ms_avg * 1e-3) / 1e9 / HBM_PEAK_GBS,
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
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
