"""PPO runner (h12env.ppo, rsl_rl 2.3 semantics) and the rsl_rl wrapper shim on a CPU toy env:
learning progress, GAE against a hand computation, checkpoint round trip, 2-rank gloo data
parallelism (rollout all-gather + gradient all-reduce keep ranks bit-identical)."""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "h1v2-isaac_amd", "shims"))
sys.path.insert(0, os.path.join(ROOT, "tests", "helpers"))

from h12env.ppo import OnPolicyRunner, RolloutStorage  # noqa: E402
from isaaclab_rl.rsl_rl import RslRlOnPolicyRunnerCfg, RslRlVecEnvWrapper  # noqa: E402
from toyenv import ToyEnv, ToyEnvCfg  # noqa: E402


def small_cfg(**kw):
    c = RslRlOnPolicyRunnerCfg(device="cpu", num_steps_per_env=16, save_interval=1000, experiment_name="toy")
    c.policy.actor_hidden_dims = [32, 32]
    c.policy.critic_hidden_dims = [32, 32]
    c.policy.init_noise_std = 0.5
    c.algorithm.num_mini_batches = 2
    c.algorithm.entropy_coef = 0.0
    for k, v in kw.items():
        setattr(c, k, v)
    return c


def test_gae_matches_hand_computation():
    st = RolloutStorage(2, 3, 1, None, 1, "cpu")
    r = torch.tensor([[1.0, 0.0], [0.5, 1.0], [2.0, -1.0]])
    d = torch.tensor([[0.0, 0.0], [0.0, 1.0], [0.0, 0.0]])
    v = torch.tensor([[0.1, 0.2], [0.3, 0.4], [0.5, 0.6]])
    st.t["rewards"][:, :, 0] = r
    st.t["dones"][:, :, 0] = d
    st.t["values"][:, :, 0] = v
    last = torch.tensor([[0.7], [0.8]])
    g, lam = 0.9, 0.8
    st.compute_returns(last, g, lam, normalize_advantage=False)
    for e in range(2):
        adv = 0.0
        exp = [0.0] * 3
        for s in reversed(range(3)):
            nv = last[e, 0] if s == 2 else v[s + 1, e]
            nd = 1.0 - d[s, e]
            delta = r[s, e] + nd * g * nv - v[s, e]
            adv = delta + nd * g * lam * adv
            exp[s] = adv + v[s, e]
        assert torch.allclose(st.t["returns"][:, e, 0], torch.tensor(exp), atol=1e-6)


def test_runner_learns_toy_task(tmp_path):
    torch.manual_seed(0)
    env = RslRlVecEnvWrapper(ToyEnv(ToyEnvCfg(scene=type(ToyEnvCfg().scene)(num_envs=128))))
    runner = OnPolicyRunner(env, small_cfg().to_dict(), log_dir=str(tmp_path), device="cpu")
    runner.learn(1, init_at_random_ep_len=True)
    first = runner.last_iteration_stats["Loss/value_function"]
    r0 = runner.last_iteration_stats.get("Episode_Reward/dist")
    runner.learn(40)
    r1 = runner.last_iteration_stats.get("Episode_Reward/dist")
    assert r1 > r0 + 0.2, (r0, r1)
    assert runner.last_iteration_stats["Loss/value_function"] < first
    # rsl_rl checkpoint layout, reload restores the policy exactly
    ck = sorted(p for p in os.listdir(tmp_path) if p.startswith("model_"))[-1]
    d = torch.load(tmp_path / ck, weights_only=True)
    assert set(d) >= {"model_state_dict", "optimizer_state_dict", "iter", "infos"}
    env2 = RslRlVecEnvWrapper(ToyEnv())
    r2 = OnPolicyRunner(env2, small_cfg().to_dict(), log_dir=None, device="cpu")
    r2.load(str(tmp_path / ck))
    x = torch.randn(5, 6)
    assert torch.equal(r2.get_inference_policy()(x), runner.get_inference_policy()(x))
    assert (tmp_path / "metrics.jsonl").exists()


def _dp_worker(rank, world, port, q):
    _dp_run(rank, world, port, q, empirical=False)


def _dp_worker_norm(rank, world, port, q):
    _dp_run(rank, world, port, q, empirical=True)


def _dp_run(rank, world, port, q, empirical):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(100 + rank)  # different per-rank init: the broadcast must unify them
    env = RslRlVecEnvWrapper(ToyEnv(ToyEnvCfg(seed=rank, scene=type(ToyEnvCfg().scene)(num_envs=32))))
    runner = OnPolicyRunner(env, small_cfg(empirical_normalization=empirical).to_dict(), log_dir=None, device="cpu")
    runner.learn(3)
    flat = torch.cat([p.detach().reshape(-1) for p in runner.alg.policy.parameters()])
    if empirical:
        # learner RNG seeded with seed + rank: the same observation draws different exploration noise on
        # each rank; the observation normaliser sees the union of the shards: identical statistics
        x = torch.zeros(4, 6)
        with torch.inference_mode():
            a = runner.alg.act(x, x).clone()
        stats = torch.cat([runner.obs_normalizer._mean.reshape(-1), runner.obs_normalizer._var.reshape(-1),
                           runner.obs_normalizer.count.reshape(-1).float()])
        q.put((rank, (flat.numpy().tobytes(), a.numpy().tobytes(), stats.numpy().tobytes())))
    else:
        q.put((rank, flat.numpy().tobytes()))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_data_parallel_ranks_stay_identical():
    import multiprocessing as mp
    import random

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = random.randint(20000, 40000)
    ps = [ctx.Process(target=_dp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0] == res[1]


def test_two_rank_noise_differs_and_normaliser_is_shared():
    import multiprocessing as mp
    import random

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = random.randint(20000, 40000)
    ps = [ctx.Process(target=_dp_worker_norm, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][0] == res[1][0]          # parameters identical
    assert res[0][1] != res[1][1]          # exploration noise differs between ranks
    assert res[0][2] == res[1][2]          # normaliser statistics identical



def _norm_worker(rank, world, port, q):
    import torch.distributed as dist

    from h12env.ppo import EmpiricalNormalization

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = torch.Generator().manual_seed(7)
    # per update: each rank's local batch size; rank 0 keeps 5 while rank 1 changes (the case a count cached per
    # local batch size got wrong)
    sizes = [(5, 3), (5, 9), (5, 1), (2, 9)]
    norm = EmpiricalNormalization(4)
    for s in sizes:
        xs = [torch.randn(n, 4, generator=g, dtype=torch.float64).float() for n in s]
        norm.update(xs[rank])
    q.put((rank, (norm._mean.numpy().tobytes(), norm._var.numpy().tobytes(), int(norm.count))))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_normaliser_union_with_changing_batch_sizes():
    """The normaliser's sample count and update rate follow the union size of every update, also when one rank's local
    batch size stays the same while another's changes: both ranks end identical and equal to one
    process updating with the concatenated batches."""
    import multiprocessing as mp
    import random

    import numpy as np

    from h12env.ppo import EmpiricalNormalization

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = random.randint(20000, 40000)
    ps = [ctx.Process(target=_norm_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0] == res[1]
    g = torch.Generator().manual_seed(7)
    ref = EmpiricalNormalization(4)
    for s in [(5, 3), (5, 9), (5, 1), (2, 9)]:
        xs = [torch.randn(n, 4, generator=g, dtype=torch.float64).float() for n in s]
        ref.update(torch.cat(xs))
    assert res[0][2] == int(ref.count) == 39
    np.testing.assert_allclose(np.frombuffer(res[0][0], np.float32), ref._mean.numpy().ravel(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(np.frombuffer(res[0][1], np.float32), ref._var.numpy().ravel(), rtol=1e-4, atol=1e-6)
