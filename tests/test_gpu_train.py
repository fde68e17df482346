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
