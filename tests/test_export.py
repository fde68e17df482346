"""CPU: deploy artefacts (row f3) -- env.yaml exporter against the reference's shipped deploy configs
(tests/golden/deploy_env_yaml.json, read from scripts/deploy/policies/*/env.yaml by tools/gen_golden.py),
the batched deploy observation handler against the reference ObservationHandler's golden vectors
(tests/golden/deploy_obs.npz), and TorchScript / ONNX policy export round trips."""
import json
from pathlib import Path

import numpy as np
import pytest
import torch
import yaml

from h12env.cfg import H12FlatEnvCfg, H12RoughEnvCfg
from h12env.export import DeployObservations, deploy_config, export_policy_as_jit, export_policy_as_onnx, write_env_yaml
from h12env.ppo import ActorCritic, EmpiricalNormalization

GOLD = Path(__file__).resolve().parent / "golden"


def test_env_yaml_layout_and_joints_match_shipped_configs(tmp_path):
    ref = json.loads((GOLD / "deploy_env_yaml.json").read_text())
    p = write_env_yaml(H12FlatEnvCfg(), str(tmp_path / "params" / "env.yaml"))
    d = yaml.safe_load(open(p))
    for name, r in ref.items():
        assert list(d.keys()) == r["keys"], name
    # joints: the 12 enabled leg joints of every shipped config (order, gains, defaults)
    for name, r in ref.items():
        legs = r["leg_joints"]
        assert [j["name"] for j in d["joints"]] == [j["name"] for j in legs], name
        for a, b in zip(d["joints"], legs):
            assert a["kp"] == b["kp"] and a["kd"] == b["kd"], (name, a, b)
            assert a["default_joint_pos"] == pytest.approx(b["default_joint_pos"], abs=1e-9)
            assert a["enabled"] is True
    # observation names are the deploy handler's function names, Flat order (no lin vel / scan)
    assert [o["name"] for o in d["observations"]] == [o["name"] for o in ref["demo_rsl"]["observations"]]
    assert d["history_length"] == 10 and d["action_scale"] == 0.5 and d["control_dt"] == pytest.approx(0.02)
    assert d["command_ranges"] == {"lin_vel_x": [0.0, 1.0], "lin_vel_y": [-0.5, 0.5], "ang_vel_z": [-1.0, 1.0]}
    rough = deploy_config(H12RoughEnvCfg())
    assert rough["observations"][0]["name"] == "base_lin_vel" and rough["observations"][-1]["name"] == "height_scan"


def test_deploy_observations_match_reference_handler():
    z = np.load(GOLD / "deploy_obs.npz")
    q0 = [0.0, -0.16, 0.0, 0.36, -0.2, 0.0] * 2
    cfg = {"observations": [{"name": n} for n in ("base_ang_vel", "projected_gravity", "generated_commands",
                                                  "joint_pos_rel", "joint_vel_rel", "last_action")],
           "history_length": int(z["history"]), "action_scale": float(z["action_scale"]), "velocity_deadzone": 0.0,
           "command_ranges": {"lin_vel_x": [-1, 1], "lin_vel_y": [-1, 1], "ang_vel_z": [-1, 1]},
           "joints": [{"name": f"j{i}", "default_joint_pos": q, "enabled": True} for i, q in enumerate(q0)]}
    h = DeployObservations(cfg, 1, "cpu")
    for t in range(z["obs"].shape[0]):
        st = {"base_orientation": torch.tensor(z["quat"][t])[None], "base_angular_vel": torch.tensor(z["wang"][t])[None],
              "qpos": torch.tensor(z["q"][t])[None], "qvel": torch.tensor(z["qd"][t])[None]}
        o = h(st, torch.tensor(z["act"][t])[None], torch.tensor(z["cmd"][t])[None])
        np.testing.assert_allclose(o[0].numpy(), z["obs"][t], rtol=1e-6, atol=1e-6)


def test_policy_export_round_trips(tmp_path):
    torch.manual_seed(0)
    pol = ActorCritic(450, 450, 12, [64, 32], [64, 32])
    norm = EmpiricalNormalization([450])
    norm.train()
    norm(torch.randn(256, 450) * 3 + 1)
    norm.eval()
    x = torch.randn(7, 450)
    want = pol.actor(norm(x))
    p = export_policy_as_jit(pol, norm, str(tmp_path / "exported"))
    got = torch.jit.load(p)(x)
    torch.testing.assert_close(got, want)
    try:
        q = export_policy_as_onnx(pol, norm, str(tmp_path / "exported"))
    except (ImportError, ModuleNotFoundError) as e:  # the onnx package is optional
        pytest.skip(f"onnx export unavailable: {e}")
    assert Path(q).stat().st_size > 1000
