"""GPU: the train.py call sequence (h1v2-isaac_amd/scripts/train.py on the import shims) on the real
Isaac-Velocity-Flat-H12_12dof-v0 env, 512 envs x 2 PPO iterations; then the checkpoint drives the env
through get_inference_policy (play.py's path)."""
import json
import sys
from pathlib import Path

import pytest
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "h1v2-isaac_amd" / "shims"), str(ROOT / "h1v2-isaac_amd" / "scripts")]

pytestmark = pytest.mark.gpu


def test_train_flat_task_two_iterations(gpu, tmp_path, monkeypatch):
    import train

    monkeypatch.chdir(tmp_path)
    rc = train.main(["--task", "Isaac-Velocity-Flat-H12_12dof-v0", "--headless", "--num_envs", "512",
                     "--max_iterations", "2", "agent.save_interval=1"])
    assert rc == 0
    run = next((tmp_path / "logs" / "rsl_rl" / "h12_12dof_flat").iterdir())
    lines = [json.loads(x) for x in (run / "metrics.jsonl").read_text().splitlines()]
    assert len(lines) == 2
    for x in lines:
        assert all(v == v for v in x.values() if isinstance(v, float))  # no NaN
        assert x["Perf/collection_env_steps_per_s"] > 0
    ck = run / "model_2.pt"
    assert ck.exists()

    import gymnasium as gym
    from isaaclab_rl.rsl_rl import RslRlVecEnvWrapper
    from isaaclab_tasks.utils.parse_cfg import load_cfg_from_registry
    from rsl_rl.runners import OnPolicyRunner

    cfg = load_cfg_from_registry("Isaac-Velocity-Flat-H12_12dof-Play-v0", "env_cfg_entry_point")
    agent = load_cfg_from_registry("Isaac-Velocity-Flat-H12_12dof-Play-v0", "rsl_rl_cfg_entry_point")
    env = RslRlVecEnvWrapper(gym.make("Isaac-Velocity-Flat-H12_12dof-Play-v0", cfg=cfg))
    runner = OnPolicyRunner(env, agent.to_dict(), log_dir=None, device="cuda:0")
    runner.load(str(ck))
    policy = runner.get_inference_policy(device="cuda:0")
    obs, _ = env.get_observations()
    with torch.inference_mode():
        for _ in range(20):
            obs, rew, dones, _ = env.step(policy(obs))
    assert torch.isfinite(obs).all() and torch.isfinite(rew).all()
    env.close()


def test_train_rough_task_one_iteration(gpu, tmp_path, monkeypatch):
    import train

    monkeypatch.chdir(tmp_path)
    rc = train.main(["--task", "Isaac-Velocity-Rough-H12_12dof-v0", "--headless", "--num_envs", "256",
                     "--max_iterations", "1", "env.scene.terrain.terrain_generator.num_rows=4",
                     "env.scene.terrain.terrain_generator.num_cols=4"])
    assert rc == 0
    run = next((tmp_path / "logs" / "rsl_rl" / "h12_12dof_rough").iterdir())
    x = json.loads((run / "metrics.jsonl").read_text().splitlines()[-1])
    assert "Curriculum/terrain_levels" in x


def test_train_rsl_task_one_iteration(gpu, tmp_path, monkeypatch):
    import train

    monkeypatch.chdir(tmp_path)
    rc = train.main(["--task", "Isaac-Velocity-Rsl-H12_12dof-v0", "--headless", "--num_envs", "256",
                     "--max_iterations", "1"])
    assert rc == 0
    run = next((tmp_path / "logs" / "rsl_rl" / "h12_12dof_flat").iterdir())
    x = json.loads((run / "metrics.jsonl").read_text().splitlines()[-1])
    assert "Episode_Reward/joint_vel_l2" in x and "Episode_Reward/base_height_l2" in x


def test_split_k_linear_gradients_match_linear(gpu):
    """The learner's split-K weight gradient equals nn.Linear's (fp32; summation order differs)."""
    from h12env.ppo import SplitKLinear

    torch.manual_seed(0)
    lin = SplitKLinear(270, 512).cuda()
    ref = torch.nn.Linear(270, 512).cuda()
    ref.load_state_dict(lin.state_dict())
    x = torch.randn(24576, 270, device="cuda", requires_grad=True)
    xr = x.detach().clone().requires_grad_(True)
    gy = torch.randn(24576, 512, device="cuda")
    lin(x).backward(gy)
    ref(xr).backward(gy)
    for a, b in ((lin.weight.grad, ref.weight.grad), (lin.bias.grad, ref.bias.grad), (x.grad, xr.grad)):
        assert torch.allclose(a, b, rtol=1e-4, atol=1e-3 * b.abs().max().item() * 1e-2), (a - b).abs().max()


def test_graph_captured_update_equals_eager(gpu, monkeypatch):
    """PPO.update replayed from the captured HIP graph gives the eager update's parameters (same kernels; the
    capture's warm-up is undone bit-exactly), over two updates with the KL-adaptive learning rate."""
    import copy

    from h12env.ppo import PPO, ActorCritic

    def run(graph: bool):
        monkeypatch.setenv("H12_PPO_GRAPH", "1" if graph else "0")
        torch.manual_seed(7)
        pol = ActorCritic(270, 270, 12, [128, 64], [128, 64])
        alg = PPO(copy.deepcopy(pol), num_learning_epochs=2, num_mini_batches=4, learning_rate=1e-3,
                  schedule="adaptive", desired_kl=0.01, device="cuda:0")
        alg.init_storage(1024, 8, [270], None, [12])
        out = []
        for u in range(2):
            g = torch.Generator(device="cuda:0").manual_seed(100 + u)
            for k, v in alg.storage.t.items():
                v.copy_(torch.randn(v.shape, generator=g, device="cuda:0") * (0.1 if k == "sigma" else 1.0))
            alg.storage.t["sigma"].abs_().add_(0.5)
            out.append(alg.update())
        return alg, out

    a, la = run(True)
    b, lb = run(False)
    assert a._graph is not None and b._graph is None
    for p, q in zip(a.policy.parameters(), b.policy.parameters()):
        assert torch.equal(p, q), (p - q).abs().max()
    assert la == lb and a.learning_rate == b.learning_rate


@pytest.mark.timeout(400)
def test_c3_ppo_iteration_at_4096_envs_graph_equals_eager(gpu, monkeypatch):
    """BASELINE config C3 at its size: one PPO iteration of the runner (24 steps x 4096 envs, 5 epochs x 4
    minibatches) on the Flat task.  The HIP-graph collection (actor / critic forward, Gaussian sample and
    log-probability in one replay) and the graph-captured update must give the eager path's rollout and
    parameters, and everything must stay finite."""
    from biped_tasks.tasks.agents import H12_12dof_FlatPPORunnerCfg
    from h12env import H12FlatEnvCfg
    from h12env.env import H12VelocityEnv
    from h12env.ppo import OnPolicyRunner
    from isaaclab_rl.rsl_rl import RslRlVecEnvWrapper

    def run(graph: bool):
        monkeypatch.setenv("H12_PPO_GRAPH", "1" if graph else "0")
        cfg = H12FlatEnvCfg()
        cfg.scene.num_envs = 4096
        cfg.sim.device = "cuda:0"
        env = H12VelocityEnv(cfg)
        agent = H12_12dof_FlatPPORunnerCfg()
        runner = OnPolicyRunner(RslRlVecEnvWrapper(env), agent.to_dict(), log_dir=None, device="cuda:0")
        runner.learn(1, init_at_random_ep_len=True)
        st = {k: v.clone() for k, v in runner.alg.storage.t.items()}
        params = torch.cat([p.detach().reshape(-1) for p in runner.alg.policy.parameters()])
        env.close()
        return st, params

    sg, pg = run(True)
    se, pe = run(False)
    for k in ("observations", "actions", "rewards", "dones", "values", "actions_log_prob", "mu", "sigma"):
        if k in sg:
            assert torch.isfinite(sg[k].float()).all(), k
            assert torch.equal(sg[k], se[k]), (k, (sg[k].float() - se[k].float()).abs().max())
    assert sg["dones"].any()
    assert torch.isfinite(pg).all()
    assert torch.equal(pg, pe), (pg - pe).abs().max()
