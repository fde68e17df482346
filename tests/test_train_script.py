"""h1v2-isaac_amd/scripts/train.py (the reference train.py call sequence on the import shims), run in a
subprocess on the CPU toy env: CLI + Hydra overrides, run directory layout, params dumps, checkpoints,
resume from the latest checkpoint."""
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
TRAIN = ROOT / "h1v2-isaac_amd" / "scripts" / "train.py"

PRELUDE = r"""
import sys
sys.path[:0] = [{shims!r}, {pkg!r}, {helpers!r}, {scripts!r}]
import gymnasium as gym
from isaaclab_rl.rsl_rl import RslRlOnPolicyRunnerCfg
def toy_agent():
    c = RslRlOnPolicyRunnerCfg(device="cpu", num_steps_per_env=8, max_iterations=3, save_interval=1,
                               experiment_name="toy_train")
    c.policy.actor_hidden_dims = [16]
    c.policy.critic_hidden_dims = [16]
    return c
gym.register(id="Toy-Reach-v0", entry_point="toyenv:ToyEnv",
             kwargs={{"env_cfg_entry_point": "toyenv:ToyEnvCfg", "rsl_rl_cfg_entry_point": toy_agent}})
import train
sys.exit(train.main(sys.argv[1:]))
"""


def run(tmp_path, *extra):
    prelude = PRELUDE.format(shims=str(ROOT / "h1v2-isaac_amd" / "shims"), pkg=str(ROOT / "h1v2-isaac_amd"),
                             helpers=str(ROOT / "tests" / "helpers"), scripts=str(TRAIN.parent))
    cmd = [sys.executable, "-c", prelude, "--task", "Toy-Reach-v0", "--headless", "--device", "cpu",
           "--num_envs", "16", "--seed", "3", "env.episode_length=20", *extra]
    return subprocess.run(cmd, cwd=tmp_path, capture_output=True, text=True, timeout=300)


def test_train_script_end_to_end_and_resume(tmp_path):
    r = run(tmp_path, "--max_iterations", "2")
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "Learning iteration" in r.stdout and "Computation:" in r.stdout
    runs = sorted((tmp_path / "logs" / "rsl_rl" / "toy_train").iterdir())
    assert len(runs) == 1
    run_dir = runs[0]
    for f in ("env.yaml", "agent.yaml", "env.pkl", "agent.pkl"):
        assert (run_dir / "params" / f).exists(), f
    assert "episode_length: 20" in (run_dir / "params" / "env.yaml").read_text()
    assert (run_dir / "model_2.pt").exists()
    lines = [json.loads(x) for x in (run_dir / "metrics.jsonl").read_text().splitlines()]
    assert [x["iter"] for x in lines] == [0, 1]
    # resume continues the iteration count from the latest checkpoint of the latest run
    r2 = run(tmp_path, "--max_iterations", "1", "--resume", "1", "--run_name", "again")
    assert r2.returncode == 0, r2.stdout[-3000:] + r2.stderr[-3000:]
    assert "Loading model checkpoint from" in r2.stdout and "model_2.pt" in r2.stdout
    again = [p for p in (tmp_path / "logs" / "rsl_rl" / "toy_train").iterdir() if p.name.endswith("_again")]
    assert again and (again[0] / "model_3.pt").exists()
