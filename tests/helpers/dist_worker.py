"""One rank of tests/test_gpu_distributed.py (started as a child process by the test, RANK / WORLD_SIZE / MASTER_*
in the environment): the real HIP env sharded by global env id, the rollout all-gather, and one PPO iteration of the
runner under torch.distributed.  Both ranks share cuda:0 on the one-GPU box, so the process group is gloo (RCCL
refuses two ranks on one device); device tensors are staged through the host by h12env.distributed.

    python dist_worker.py OUT_DIR N_PER STEPS
"""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "h1v2-isaac_amd"), str(ROOT / "h1v2-isaac_amd" / "shims")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def global_actions(t: int, n_global: int) -> torch.Tensor:
    g = torch.Generator(device="cpu").manual_seed(1000 + t)
    return torch.randn(n_global, 12, generator=g)


def main():
    out, n_per, steps = Path(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    from h12env import H12FlatEnvCfg
    from h12env import distributed as D
    from h12env.env import H12VelocityEnv

    shard = D.init(n_per, backend="gloo")
    cfg = H12FlatEnvCfg()
    cfg.scene.num_envs = n_per
    cfg.sim.device = "cuda:0"
    env = H12VelocityEnv(cfg, env_offset=shard.env_offset)
    # ---- (1) the env shard: a rollout under one global action stream, all-gathered (rank order = env order)
    obs, _ = env.reset()
    roll = {"obs": torch.zeros(steps + 1, n_per, obs["policy"].shape[1], device="cuda:0"),
            "rew": torch.zeros(steps, n_per, device="cuda:0"),
            "done": torch.zeros(steps, n_per, dtype=torch.uint8, device="cuda:0")}
    roll["obs"][0] = obs["policy"]
    for t in range(steps):
        a = global_actions(t, shard.global_envs)[shard.env_offset:shard.env_offset + n_per].cuda()
        obs, rew, term, trunc, _ = env.step(a)
        roll["obs"][t + 1] = obs["policy"]
        roll["rew"][t] = rew
        roll["done"][t] = (term | trunc).to(torch.uint8)
    g = D.allgather_rollout(roll, shard, env_dim=1)
    if shard.rank == 0:
        np.savez(out / "rollout.npz", **{k: v.cpu().numpy() for k, v in g.items()})
    env.close()
    # ---- (2) one PPO iteration of the runner on the sharded env (rollout all-gather + gradient all-reduce)
    from biped_tasks.tasks.agents import H12_12dof_FlatPPORunnerCfg
    from h12env.ppo import OnPolicyRunner
    from isaaclab_rl.rsl_rl import RslRlVecEnvWrapper

    env = H12VelocityEnv(cfg, env_offset=shard.env_offset)
    env.shard = shard
    agent = H12_12dof_FlatPPORunnerCfg()
    agent.num_steps_per_env = 8
    runner = OnPolicyRunner(RslRlVecEnvWrapper(env), agent.to_dict(), log_dir=None, device="cuda:0")
    p0 = torch.cat([p.detach().reshape(-1) for p in runner.alg.policy.parameters()]).cpu().numpy()
    runner.learn(1, init_at_random_ep_len=True)
    p1 = torch.cat([p.detach().reshape(-1) for p in runner.alg.policy.parameters()]).cpu().numpy()
    np.savez(out / f"params_{shard.rank}.npz", before=p0, after=p1)
    env.close()
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
