"""Deploy artefacts (row f3): env.yaml, exported policies, batched deploy controller, trajectory log.

* ``deploy_config`` / ``write_env_yaml``: the env.yaml the sim2sim / sim2real deploy stack reads, restating
  biped_tasks/utils/mdp/config_exporter.py:27-58 (control_dt, history_length/step, action_scale,
  velocity_deadzone, command_ranges, observations [name, scale], joints [name, kp, kd, default_joint_pos,
  enabled]) for this stack's cfg objects; layout of scripts/deploy/policies/*/env.yaml.
* ``export_policy_as_jit`` / ``export_policy_as_onnx``: the actor (+ observation normaliser) as TorchScript /
  ONNX, what scripts/rsl_rl/play.py:102-114 writes to <run>/exported/.
* ``DeployObservations`` + ``DeployController``: the deploy-side ObservationHandler / ActionHandler
  (biped_deploy/controllers/rl.py:35-134) batched over envs in torch, so an exported policy + env.yaml drive
  this env's MuJoCo-mode physics (the sim2sim loop, scripts/deploy/sim2sim.py) on the GPU.
* ``TrajectoryLogger``: the MJLogger metrics.json schema (biped_deploy/utils/mj_logger.py:17-150) for one env.
"""
from __future__ import annotations

import copy
import json
import os
import re
from dataclasses import asdict, dataclass

import numpy as np
import torch
import torch.nn as nn
import yaml

from .model import build_model, joint_names

_OBS_FUNCS = {  # cfg term -> isaaclab mdp function name (the env.yaml "name")
    "base_lin_vel": "base_lin_vel",
    "base_ang_vel": "base_ang_vel",
    "projected_gravity": "projected_gravity",
    "velocity_commands": "generated_commands",
    "joint_pos": "joint_pos_rel",
    "joint_vel": "joint_vel_rel",
    "actions": "last_action",
    "height_scan": "height_scan",
}


# ---------------------------------------------------------------------------------------------- env.yaml
def deploy_config(cfg) -> dict:
    """get_deploy_config restated for H12FlatEnvCfg / H12RoughEnvCfg."""
    po = cfg.observations.policy
    observations = []
    for term, fn in _OBS_FUNCS.items():
        if term in ("base_lin_vel", "height_scan") and getattr(po, term, None) is None:
            continue
        ent = {"name": fn}
        scale = getattr(po, "scales", {}).get(term, 1.0) if hasattr(po, "scales") else 1.0
        if scale != 1.0:
            ent["scale"] = float(scale)
        observations.append(ent)
    joints = []
    names = joint_names()
    q0 = build_model().q_default
    for j, name in enumerate(names):
        ent = {"name": name}
        for g in cfg.robot.actuators.values():
            if any(re.fullmatch(p, name) for p in g.joint_names_expr):
                ent["kp"] = float(g.stiffness)
                ent["kd"] = float(g.damping)
        ent["default_joint_pos"] = float(round(q0[j], 6))
        ent["enabled"] = True
        joints.append(ent)
    r = cfg.commands.base_velocity.ranges
    return {
        "control_dt": float(cfg.sim.dt * cfg.decimation),
        "history_length": int(po.history_length or 1),
        "history_step": 1,
        "action_scale": float(cfg.actions.joint_pos.scale),
        "velocity_deadzone": float(getattr(cfg.commands.base_velocity, "velocity_deadzone", 0.0)),
        "command_ranges": {"lin_vel_x": [float(x) for x in r.lin_vel_x], "lin_vel_y": [float(x) for x in r.lin_vel_y],
                           "ang_vel_z": [float(x) for x in r.ang_vel_z]},
        "observations": observations,
        "joints": joints,
    }


def write_env_yaml(cfg, path: str) -> str:
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    with open(path, "w") as f:
        yaml.safe_dump(deploy_config(cfg), f, sort_keys=False, default_flow_style=False)
    return path


# ---------------------------------------------------------------------------------------------- policy export
class _ExportedPolicy(nn.Module):
    def __init__(self, actor: nn.Module, normalizer: nn.Module | None):
        super().__init__()
        from .ppo import plain_linear

        self.actor = plain_linear(actor).cpu().eval()
        self.normalizer = copy.deepcopy(normalizer).cpu().eval() if normalizer is not None else nn.Identity()

    def forward(self, x):
        return self.actor(self.normalizer(x))


def export_policy_as_jit(policy, normalizer, path: str, filename: str = "policy.pt") -> str:
    """TorchScript of actor(normalizer(obs)) (play.py:102-108)."""
    os.makedirs(path, exist_ok=True)
    m = torch.jit.script(_ExportedPolicy(policy.actor, normalizer))
    out = os.path.join(path, filename)
    m.save(out)
    return out


def export_policy_as_onnx(policy, normalizer, path: str, filename: str = "policy.onnx", verbose: bool = False) -> str:
    """ONNX of actor(normalizer(obs)), input "obs" (1, num_obs), output "actions" (play.py:109-114)."""
    try:
        import onnx  # noqa: F401  (torch's exporter serialises through it)
    except ImportError as e:
        raise ImportError("ONNX export needs the onnx package (not installed here); "
                          "export_policy_as_jit works without it") from e
    os.makedirs(path, exist_ok=True)
    m = _ExportedPolicy(policy.actor, normalizer)
    n_in = next(p for p in m.actor.parameters()).shape[1]
    out = os.path.join(path, filename)
    torch.onnx.export(m, torch.zeros(1, n_in), out, input_names=["obs"], output_names=["actions"], opset_version=17,
                      verbose=verbose, dynamo=False)
    return out


# ---------------------------------------------------------------------------------------------- deploy side
class DeployObservations:
    """ObservationHandler (rl.py:35-116) over N envs: per-term histories (first call fills), term-major."""

    def __init__(self, config: dict, num_envs: int, device):
        self.cfg = config
        self.n = num_envs
        self.dev = torch.device(device)
        en = [j for j in config["joints"] if j["enabled"]]
        self.q0 = torch.tensor([j["default_joint_pos"] for j in en], device=self.dev)
        self.terms = [o["name"] for o in config["observations"]]
        self.scales = [float(o.get("scale", 1.0)) for o in config["observations"]]
        self.H = int(config["history_length"])
        cr = config["command_ranges"]
        self.lower = torch.tensor([v[0] for v in cr.values()], device=self.dev)
        self.upper = torch.tensor([v[1] for v in cr.values()], device=self.dev)
        self.deadzone = float(config.get("velocity_deadzone", 0.0))
        self.hist: list[torch.Tensor | None] = [None] * len(self.terms)

    def _term(self, name, st, actions, command):
        if name == "base_ang_vel":
            return st["base_angular_vel"]
        if name == "projected_gravity":
            qw, qx, qy, qz = st["base_orientation"].unbind(-1)
            return torch.stack([2 * (-qz * qx + qw * qy), -2 * (qz * qy + qw * qx), 1 - 2 * (qw * qw + qz * qz)], -1)
        if name == "generated_commands":
            c = (command + 1) / 2 * (self.upper - self.lower) + self.lower
            return torch.where(c.abs() < self.deadzone, torch.zeros_like(c), c)
        if name == "joint_pos_rel":
            return st["qpos"] - self.q0
        if name == "joint_vel_rel":
            return st["qvel"]
        if name == "last_action":
            return actions
        raise KeyError(f"deploy observation term {name!r} is not available on this stack")

    def __call__(self, st: dict, actions: torch.Tensor, command: torch.Tensor) -> torch.Tensor:
        parts = []
        for i, name in enumerate(self.terms):
            x = (self._term(name, st, actions, command) * self.scales[i]).float()
            if self.hist[i] is None:
                self.hist[i] = x.unsqueeze(1).repeat(1, self.H, 1)
            else:
                self.hist[i] = torch.cat([self.hist[i][:, 1:], x.unsqueeze(1)], dim=1)
            parts.append(self.hist[i].reshape(self.n, -1))
        return torch.cat(parts, dim=1)


class DeployController:
    """RLPolicy: observations -> policy -> q_ref = default + action_scale * a (ActionHandler, rl.py:119-134)."""

    def __init__(self, policy, config: dict, num_envs: int, device):
        self.policy = policy
        self.obs = DeployObservations(config, num_envs, device)
        self.scale = float(config["action_scale"])
        self.actions = torch.zeros(num_envs, len(self.obs.q0), device=device)

    def __call__(self, st: dict, command: torch.Tensor) -> torch.Tensor:
        o = self.obs(st, self.actions, command)
        with torch.inference_mode():
            self.actions = self.policy(o).float()
        return self.scale * self.actions + self.obs.q0


def env_state(env) -> dict:
    """The deploy state dict (sim_mujoco.py get_state) from the env workspace, batched."""
    return {"base_orientation": env._field("QUAT").T, "base_angular_vel": env._field("WANG").T,
            "qpos": env._field("Q").T, "qvel": env._field("QD").T}


# ---------------------------------------------------------------------------------------------- trajectory log
def _json(obj):
    if isinstance(obj, (np.ndarray, np.generic)):
        return obj.tolist()
    raise TypeError(f"Object of type {type(obj)} is not JSON serializable")


@dataclass
class Metrics:
    timestamp: float
    base_lin_pos: np.ndarray
    base_quat_pos: np.ndarray
    joint_pos: dict
    base_lin_vel: np.ndarray
    base_quat_vel: np.ndarray
    joint_vel: dict
    applied_torques: dict
    foot_contact_forces: dict
    action_rate: dict
    joint_pos_rate: dict


@dataclass
class Limits:
    joint_pos_limits: dict
    total_mass_force: float


class TrajectoryLogger:
    """MJLogger's metrics.json for env `index` (records limits once, then one Metrics per call)."""

    def __init__(self, env, index: int = 0):
        self.env, self.i = env, index
        self.names = joint_names()
        self.data: list = []
        self.prev_q: dict = {}
        self.prev_tau: dict = {}

    def record_limits(self):
        m = build_model()
        lim = {n: np.array([m.q_lower[j], m.q_upper[j]]) for j, n in enumerate(self.names)}
        total = (m.base_mass + sum(m.link_mass)) * m.gravity
        self.data.append(Limits(lim, float(total)))

    def record_metrics(self, t: float, applied_torque: torch.Tensor | None = None, foot_force: torch.Tensor | None = None):
        e, i = self.env, self.i
        q = e._field("Q")[:, i].cpu().numpy()
        qd = e._field("QD")[:, i].cpu().numpy()
        tau = (applied_torque if applied_torque is not None else e._applied_torque)[i].cpu().numpy()
        jp, jv, at, ar, jr = {}, {}, {}, {}, {}
        for j, n in enumerate(self.names):
            jp[n] = float(q[j])
            jr[n] = float(q[j] - self.prev_q.get(n, q[j]))
            self.prev_q[n] = float(q[j])
            jv[n] = float(qd[j])
            at[n] = float(tau[j])
            ar[n] = float(tau[j] - self.prev_tau.get(n, tau[j]))
            self.prev_tau[n] = float(tau[j])
        ff = {"left_ankle_roll_link": 0.0, "right_ankle_roll_link": 0.0}
        if foot_force is not None:
            f = foot_force[i].cpu().numpy()
            ff = {"left_ankle_roll_link": float(f[0]), "right_ankle_roll_link": float(f[1])}
        self.data.append(Metrics(float(t), e._field("POS")[:, i].cpu().numpy(), e._field("QUAT")[:, i].cpu().numpy(), jp,
                                 e._field("VLIN")[:, i].cpu().numpy(), e._field("WANG")[:, i].cpu().numpy(), jv, at, ff,
                                 ar, jr))

    def save_data(self, log_dir) -> str:
        os.makedirs(log_dir, exist_ok=True)
        p = os.path.join(log_dir, "metrics.json")
        with open(p, "w") as f:
            json.dump([asdict(m) for m in self.data], f, indent=2, default=_json)
        return p
