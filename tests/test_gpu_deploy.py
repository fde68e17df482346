"""GPU: deploy artefacts end to end (row f3) -- export a policy (TorchScript) + env.yaml, drive the
MuJoCo-mode env with the batched deploy controller (sim2sim), write env 0's MJLogger-schema trajectory."""
import json
import sys
from pathlib import Path

import pytest
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "h1v2-isaac_amd" / "scripts"))

pytestmark = pytest.mark.gpu


def test_export_and_sim2sim(gpu, tmp_path):
    import sim2sim

    from h12env.cfg import H12FlatEnvCfg
    from h12env.export import export_policy_as_jit, write_env_yaml
    from h12env.ppo import ActorCritic

    torch.manual_seed(0)
    pol = ActorCritic(450, 450, 12, [64, 32], [64, 32])
    for p in pol.actor.parameters():
        p.data.mul_(0.01)  # near-zero actions: the robot should stand under the default-pose PD
    d = tmp_path / "policy"
    export_policy_as_jit(pol, None, str(d))
    write_env_yaml(H12FlatEnvCfg(), str(d / "env.yaml"))
    rc = sim2sim.main([str(d), "--num_envs", "16", "--episode_length", "1.0", "--log_dir", str(tmp_path / "log")])
    assert rc == 0
    m = json.loads((tmp_path / "log" / "metrics.json").read_text())
    assert set(m[0]) == {"joint_pos_limits", "total_mass_force"}
    assert len(m) == 1 + 50
    keys = {"timestamp", "base_lin_pos", "base_quat_pos", "joint_pos", "base_lin_vel", "base_quat_vel", "joint_vel",
            "applied_torques", "foot_contact_forces", "action_rate", "joint_pos_rate"}
    assert set(m[1]) == keys and len(m[1]["joint_pos"]) == 12
    assert 0.85 < m[-1]["base_lin_pos"][2] < 1.2   # still standing after 1 s
