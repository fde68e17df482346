#!/usr/bin/env python3
"""Generate tests/golden/ref_*.npz from the reference's own MDP term code (build container only).

The reference's reward / constraint / command / curriculum / observation-manager functions are imported by
file path from /root/reference with TYPE-ONLY stubs for the IsaacLab modules they name (IsaacLab is not
installed).  Every function is then driven with duck-typed env objects built from seeded random states, and
only input / output arrays are written -- no reference source enters the repository.

  ref_rewards.npz     velocity/mdp/rewards.py:38-62 feet_air_time_positive_biped,
                      utils/mdp/rewards.py:23-30 action_rate_l2
  ref_constraints.npz utils/cat/constraints.py (the ten terms of cat_env_cfg.py:336-425) fed through
                      constraint_manager.py ConstraintManager.compute (:212-228, the CaT class :23-123) and
                      ConstraintManager.reset (:195-210) over a multi-step sequence
  ref_commands.npz    utils/mdp/commands.py:83-138 UniformVelocityCommandWithDeadzone._update_command
                      (randperm -> identity, bernoulli -> fixed uniforms; both recorded)
  ref_curriculum.npz  velocity/mdp/curriculums.py:27-58 terrain_levels_vel, utils/cat/curriculums.py:21-42
                      modify_constraint_p
  ref_obs_manager.npz utils/history/observation_manager.py:271-355 ObservationManager.compute_group with the
                      reference CircularBuffer: noise -> clip -> scale -> history (Flat, Rsl and Rough layouts)

What the stubs restate (IsaacLab code absent here, named so it can be audited): SceneEntityCfg (a name + the
resolved ids), ContactSensor.compute_first_contact (current_contact_time > 0 and < dt + 1e-8),
math_utils.wrap_to_pi (IsaacLab 2.1 formula), Unoise (value + n_min + (n_max - n_min) u with u recorded),
configclass (identity).  Model-dependent inputs the reference receives from PhysX (projected gravity, heading,
foot link heights) are computed here from the sampled state -- foot heights through the oracle's kinematics
(oracle/oracle.py), so the foot_clearance fixture pins the touchdown / swing-max / deadzone logic, not FK.

    python tools/gen_golden_terms.py
"""
from __future__ import annotations

import importlib.util
import math
import sys
import types
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
REF = Path("/root/reference/packages")
BT = REF / "biped_tasks/biped_tasks"
OUT = ROOT / "tests" / "golden"
sys.path.insert(0, str(ROOT / "h1v2-isaac_amd"))
sys.path.insert(0, str(ROOT / "oracle"))


# ------------------------------------------------------------------------------------------------ stubs
def _mod(name, **attrs):
    m = types.ModuleType(name)
    m.__dict__.update(attrs)
    if "." not in name or True:
        m.__path__ = []  # importable as a package
    sys.modules[name] = m
    return m


class SceneEntityCfg:
    def __init__(self, name, body_names=None, joint_names=None, body_ids=slice(None), joint_ids=slice(None)):
        self.name, self.body_names, self.joint_names = name, body_names, joint_names
        self.body_ids, self.joint_ids = body_ids, joint_ids


def _wrap_to_pi(angles):  # isaaclab.utils.math.wrap_to_pi (IsaacLab 2.1)
    wrapped = torch.remainder(angles + torch.pi, 2 * torch.pi)
    return torch.where((wrapped == 0) & (angles > 0), torch.tensor(torch.pi, dtype=angles.dtype), wrapped - torch.pi)


def install_stubs():
    class _Any:
        def __init__(self, *a, **k):
            pass

    def configclass(cls):
        return cls

    _mod("isaaclab")
    _mod("isaaclab.managers", SceneEntityCfg=SceneEntityCfg, ManagerTermBase=_Any, ManagerBase=_Any)
    _mod("isaaclab.managers.manager_base", ManagerBase=_Any, ManagerTermBase=_Any)
    _mod("isaaclab.managers.manager_term_cfg", ManagerTermBaseCfg=object)
    _mod("isaaclab.sensors", ContactSensor=_Any)
    _mod("isaaclab.utils", configclass=configclass, modifiers=types.SimpleNamespace())
    _mod("isaaclab.utils.math", wrap_to_pi=_wrap_to_pi, matrix_from_quat=None, sample_uniform=None)
    _mod("isaaclab.utils.noise", NoiseModelCfg=_Any)
    _mod("isaaclab.assets", Articulation=_Any, RigidObject=_Any)
    _mod("isaaclab.terrains", TerrainImporter=_Any)
    _mod("isaaclab.envs", ManagerBasedRLEnv=_Any, ManagerBasedEnv=_Any, RLTaskEnv=_Any)
    _mod("prettytable", PrettyTable=_Any)

    class UniformVelocityCommand:  # base class of the deadzone command; only attributes are used
        pass

    class UniformVelocityCommandCfg:
        pass

    for n in ("isaaclab_tasks", "isaaclab_tasks.manager_based", "isaaclab_tasks.manager_based.locomotion",
              "isaaclab_tasks.manager_based.locomotion.velocity"):
        _mod(n)
    _mod("isaaclab_tasks.manager_based.locomotion.velocity.mdp", UniformVelocityCommand=UniformVelocityCommand,
         UniformVelocityCommandCfg=UniformVelocityCommandCfg)
    for n in ("biped_tasks", "biped_tasks.utils", "biped_tasks.utils.history"):
        _mod(n)
    cb = load("biped_tasks.utils.history.circular_buffer", BT / "utils/history/circular_buffer.py")
    sys.modules["biped_tasks.utils.history"].circular_buffer = cb
    _mod("biped_tasks.utils.history.manager_term_cfg", ObservationGroupCfg=object, ObservationTermCfg=object)


def load(name, path, package=None):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    if package:
        mod.__package__ = package
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


# ------------------------------------------------------------------------------------------------ helpers
def quat_random(rng, n, tilt):
    """unit quaternions (w, x, y, z): a yaw in (-pi, pi) and a tilt about a random horizontal axis."""
    yaw = rng.uniform(-math.pi, math.pi, n)
    ang = rng.uniform(0, tilt, n)
    ax = rng.uniform(0, 2 * math.pi, n)
    qy = np.stack([np.cos(yaw / 2), np.zeros(n), np.zeros(n), np.sin(yaw / 2)], 1)
    qt = np.stack([np.cos(ang / 2), np.sin(ang / 2) * np.cos(ax), np.sin(ang / 2) * np.sin(ax), np.zeros(n)], 1)
    w1, x1, y1, z1 = qy.T
    w2, x2, y2, z2 = qt.T
    return np.stack([w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2, w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                     w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2, w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2], 1)


def rot(q):
    w, x, y, z = q.T
    return np.stack([np.stack([1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)], -1),
                     np.stack([2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)], -1),
                     np.stack([2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)], -1)], 1)


def ns(**kw):
    return types.SimpleNamespace(**kw)


def f32(x):
    return torch.as_tensor(np.array(x), dtype=torch.float32)


# ------------------------------------------------------------------------------------------------ rewards
def gen_rewards(rng):
    R = load("ref_vel_rewards", BT / "tasks/locomotion/velocity/mdp/rewards.py")
    U = load("ref_utils_rewards", BT / "utils/mdp/rewards.py")
    n = 512
    # contact / air times with the edge cases: both in contact, one, none; times 0, sub-step, > threshold
    con = rng.choice([0.0, 0.005, 0.02, 0.15, 0.6], size=(n, 2)) * (rng.random((n, 2)) < 0.6)
    air = np.where(con > 0, 0.0, rng.choice([0.0, 0.005, 0.1, 0.35, 0.45, 1.2], size=(n, 2)))
    cmd = rng.uniform(-1, 1, (n, 3))
    k = rng.random(n)
    cmd[k < 0.2, :2] *= 0.0
    near = (k >= 0.2) & (k < 0.4)  # |cmd_xy| around the 0.1 gate
    ang = rng.uniform(0, 2 * math.pi, near.sum())
    r = 0.1 + rng.choice([-1e-3, 1e-3, -1e-5, 1e-5], near.sum())
    cmd[near, 0], cmd[near, 1] = r * np.cos(ang), r * np.sin(ang)
    cmd = cmd.astype(np.float32)
    act = rng.normal(size=(n, 12)).astype(np.float32)
    act_prev = rng.normal(size=(n, 12)).astype(np.float32)
    act_prev[: n // 8] = act[: n // 8]
    sensor = ns(data=ns(current_air_time=f32(air), current_contact_time=f32(con)))
    env = ns(scene=ns(sensors={"contact_forces": sensor}),
             command_manager=ns(get_command=lambda name: f32(cmd)),
             action_manager=ns(action=f32(act), prev_action=f32(act_prev)))
    cfg = SceneEntityCfg("contact_forces", body_names=".*ankle_roll_link", body_ids=[0, 1])
    fat = R.feet_air_time_positive_biped(env, command_name="base_velocity", threshold=0.4, sensor_cfg=cfg)
    arl = U.action_rate_l2(env, asset_cfg=SceneEntityCfg("robot", joint_ids=slice(None)))
    np.savez_compressed(OUT / "ref_rewards.npz", air=air.astype(np.float32), con=con.astype(np.float32), cmd=cmd,
                        act=act, act_prev=act_prev, threshold=0.4, feet_air_time_positive_biped=fat.numpy(),
                        action_rate_l2=arl.numpy())


# ------------------------------------------------------------------------------------------------ CaT
def gen_constraints(rng):
    import oracle as O
    from h12env.cfg import H12CaTEnvCfg
    from h12env.model import build_model

    _mod("ref_cat")
    sys.modules["ref_cat"].__path__ = [str(BT / "utils/cat")]
    Cn = load("ref_cat.constraints", BT / "utils/cat/constraints.py", package="ref_cat")
    M = load("ref_cat.constraint_manager", BT / "utils/cat/constraint_manager.py", package="ref_cat")
    model = build_model()
    cfg = H12CaTEnvCfg()
    n, T, dt = 48, 6, 0.005
    step_dt = dt * 4
    lo, hi = np.array(model.q_lower), np.array(model.q_upper)
    mid, half = (lo + hi) / 2, (hi - lo) / 2 * 0.9
    soft = np.stack([mid - half, mid + half], -1)
    q0 = np.array(model.q_default)
    vel_lim = np.array([23.0, 23, 23, 14, 9, 9] * 2)
    eff_lim = np.array([220.0, 220, 220, 360, 45, 45] * 2)  # finite, so joint_torque_limits carries signal
    max_p = {"contact": 1.0, "joint_position_limits": 0.25, "joint_velocity_limits": 0.2, "joint_torque_limits": 0.15,
             "foot_contact_force": 0.3, "no_move": 0.22, "base_orientation": 0.12, "base_height": 0.18,
             "foot_contact": 0.28, "foot_clearance": 0.24}
    terms = [
        ("contact", Cn.contact, {"asset_cfg": SceneEntityCfg("contact_forces", body_ids=[0, 1, 2, 5])}),
        ("joint_position_limits", Cn.joint_position_limits, {"asset_cfg": SceneEntityCfg("robot")}),
        ("joint_velocity_limits", Cn.joint_velocity_limits, {"asset_cfg": SceneEntityCfg("robot")}),
        ("joint_torque_limits", Cn.joint_torque_limits, {"asset_cfg": SceneEntityCfg("robot")}),
        ("foot_contact_force", Cn.foot_contact_force,
         {"limit": 750.0, "asset_cfg": SceneEntityCfg("contact_forces", body_ids=[3, 4])}),
        ("no_move", Cn.no_move, {"velocity_deadzone": 0.2, "joint_vel_limit": 6.0, "asset_cfg": SceneEntityCfg("robot")}),
        ("base_orientation", Cn.base_orientation, {"limit": 0.1, "asset_cfg": SceneEntityCfg("robot")}),
        ("base_height", Cn.base_height, {"height": 1.0, "std": 0.05, "asset_cfg": SceneEntityCfg("robot")}),
        ("foot_contact", Cn.foot_contact, {"asset_cfg": SceneEntityCfg("contact_forces", body_ids=[3, 4])}),
        ("foot_clearance", Cn.foot_clearance,
         {"min_height": 0.1, "velocity_deadzone": 0.2, "pos_asset_cfg": SceneEntityCfg("robot", body_ids=[0, 1]),
          "contact_asset_cfg": SceneEntityCfg("contact_forces", body_ids=[3, 4])}),
    ]
    # the manager as the reference runs it (compute :212-228, reset :195-210) on a duck-typed self
    mgr = types.SimpleNamespace(cat=M.CaT(tau=0.95, min_p=0.0), _term_names=[t[0] for t in terms],
                                _term_cfgs=[ns(func=f, params=p, max_p=max_p[nm]) for nm, f, p in terms],
                                _class_term_cfgs=[],
                                _episode_sums={t[0]: torch.zeros(n) for t in terms},
                                _cstr_mean_values={t[0]: torch.zeros(n) for t in terms})
    robot_data = ns()
    rec = {k: [] for k in ("pos", "quat", "q", "qd", "tau", "cmd", "con", "forces", "foot_z", "eplen", "raw", "runmax",
                           "prob", "pterm", "reset", "log_violation", "log_probability")}
    eplen = rng.integers(1, 400, n)
    sw = np.zeros((n, 2))
    for t in range(T):
        quat = quat_random(rng, n, tilt=rng.choice([0.02, 0.3]))
        pos = np.stack([rng.uniform(-1, 1, n), rng.uniform(-1, 1, n), rng.uniform(0.9, 1.1, n)], 1)
        q = q0 + rng.normal(size=(n, 12)) * 0.35
        qd = rng.normal(size=(n, 12)) * rng.choice([2.0, 8.0, 15.0], size=(n, 1))
        tau = rng.normal(size=(n, 12)) * rng.choice([50.0, 150.0, 300.0], size=(n, 1))
        cmd = rng.uniform(-1, 1, (n, 3))
        still = rng.random(n) < 0.3
        cmd[still] *= 0.15
        # bodies: 0/1 knees, 2 torso, 3/4 feet, 5 pelvis (no collider in the build model: zero force)
        forces = rng.normal(size=(n, 3, 6, 3)) * rng.choice([0.1, 0.5, 50.0, 400.0], size=(n, 3, 6, 1))
        forces[:, :, 0:3] *= (rng.random((n, 1, 3, 1)) < 0.3)
        forces[:, :, 5] = 0.0
        con = np.where(rng.random((n, 2)) < 0.5, rng.choice([0.005, 0.01, 0.02, 0.0201, 0.1], size=(n, 2)), 0.0)
        state = np.zeros((n, 37))
        state[:, 0:3], state[:, 3:7], state[:, 13:25], state[:, 25:37] = pos, quat, q, qd
        foot_z = np.zeros((n, 2))
        for i in range(n):  # body_link_pos_w z of the ankle-roll links (oracle kinematics)
            ti = O.term_in(state[i], np.zeros(12), np.zeros(12), np.zeros(3), np.zeros(2), np.zeros(2), np.zeros(12),
                           np.zeros(12), np.zeros(2), np.zeros(2), 0.0, 0)
            foot_z[i] = _foot_z(O, model, ti)
        gb = np.einsum("nji,j->ni", rot(quat), np.array([0.0, 0.0, -1.0]))
        eplen = eplen + 1
        robot_data.joint_pos = f32(q)
        robot_data.soft_joint_pos_limits = f32(np.broadcast_to(soft, (n, 12, 2)))
        robot_data.joint_vel = f32(qd)
        robot_data.joint_vel_limits = f32(np.broadcast_to(vel_lim, (n, 12)))
        robot_data.applied_torque = f32(tau)
        robot_data.joint_effort_limits = f32(np.broadcast_to(eff_lim, (n, 12)))
        robot_data.projected_gravity_b = f32(gb)
        robot_data.root_pos_w = f32(pos)
        robot_data.body_link_pos_w = f32(np.stack([np.zeros((n, 2)), np.zeros((n, 2)), foot_z], -1))
        cs_t = f32(np.zeros((n, 6)))
        cs_t[:, 3:5] = f32(con)
        sensor = ns(data=ns(net_forces_w_history=f32(forces), current_contact_time=cs_t),
                    compute_first_contact=lambda dt_, c=cs_t: ((c > 0) & (c < dt_ + 1e-8)).float())
        scene = {"robot": ns(data=robot_data), "contact_forces": sensor}
        env = ns(scene=scene, num_envs=n, device="cpu", step_dt=step_dt,
                 command_manager=ns(get_command=lambda name, c=f32(cmd): c),
                 action_manager=ns(action_term_dim=[12]), episode_length_buf=torch.as_tensor(eplen))
        mgr._env = env
        prob = M.ConstraintManager.compute(mgr)
        raw = mgr.cat.get_raw_constraints().numpy()
        runmax = mgr.cat.get_running_maxes().numpy()[0]
        pterm = np.stack([mgr.cat.probs[nm].max(1).values.numpy() for nm, _, _ in terms])
        reset = rng.random(n) < 0.25
        ids = np.nonzero(reset)[0]
        logs = M.ConstraintManager.reset(mgr, torch.as_tensor(ids)) if len(ids) else {}
        rec["log_violation"].append([float(logs.get(f"Episode_Constraint_violation/{nm}", np.nan)) for nm, _, _ in terms])
        rec["log_probability"].append([float(logs.get(f"Episode_Constraint_probability/{nm}", np.nan))
                                       for nm, _, _ in terms])
        for k, v in (("pos", pos), ("quat", quat), ("q", q), ("qd", qd), ("tau", tau), ("cmd", cmd), ("con", con),
                     ("forces", forces), ("foot_z", foot_z), ("eplen", eplen.copy()), ("raw", raw), ("runmax", runmax),
                     ("prob", prob.numpy()), ("pterm", pterm), ("reset", reset)):
            rec[k].append(v)
        eplen = np.where(reset, 0, eplen)
    out = {k: np.array(v) for k, v in rec.items()}
    out["swing_max_height_final"] = robot_data.swing_max_height.numpy()
    out["max_p"] = np.array([max_p[nm] for nm, _, _ in terms])
    out["term_names"] = np.array([nm for nm, _, _ in terms])
    out["soft_limits"], out["vel_limits"], out["effort_limits"] = soft, vel_lim, eff_lim
    np.savez_compressed(OUT / "ref_constraints.npz", **out)


def _foot_z(O, model, ti):
    from h12env.cfg import H12CaTEnvCfg

    c = H12CaTEnvCfg().to_c()
    c.cstr_clearance_deadzone = -1.0  # every env active, min 0: the output is min_height - swing_h ...
    sw = np.array([-1e9, -1e9])
    # ... with touchdown false the swing height becomes max(-1e9, foot z) = foot z
    ti.con[:] = [0.0, 0.0]
    O.cat_row(model, c, ti, False, sw)
    return sw


# ------------------------------------------------------------------------------------------------ commands
class _TorchProxy:
    """module-level `torch` of commands.py with randperm -> identity and bernoulli -> (u < p), u recorded."""

    def __init__(self, u):
        self._u = u

    def __getattr__(self, k):
        return getattr(torch, k)

    def randperm(self, n, *a, **k):
        return torch.arange(n)

    def bernoulli(self, p, *a, **k):
        return (self._u < p).to(p.dtype)


def gen_commands(rng):
    Cm = load("ref_commands", BT / "utils/mdp/commands.py")
    out = {}
    for case, (n, dz, heading) in enumerate([(64, 0.0, True), (64, 0.3, True), (65, 0.3, False), (64, 1.5, True)]):
        cmd = rng.uniform(-1, 1, (n, 3)).astype(np.float32)
        if case == 1:
            cmd[: n // 3, :2] *= 0.1  # fewer than half in the deadzone
        if case == 3:
            cmd[:, :2] *= 0.2        # all in the deadzone: activation path
        quat = quat_random(rng, n, tilt=0.2)
        R = rot(quat)
        heading_w = np.arctan2(R[:, 1, 0], R[:, 0, 0]).astype(np.float32)
        target = rng.uniform(-math.pi, math.pi, n).astype(np.float32)
        target[:4] = heading_w[:4] + np.array([2 * math.pi + 0.1, -2 * math.pi - 0.1, math.pi - 1e-3, 1e-3])
        is_heading = rng.random(n) < 0.7
        u = torch.as_tensor(rng.random(n), dtype=torch.float32)
        u[: n // 10] = 0.0  # some flips
        self = object.__new__(Cm.UniformVelocityCommandWithDeadzone)
        resampled = []
        self.cfg = ns(heading_command=heading, heading_control_stiffness=0.5, ranges=ns(ang_vel_z=(-1.0, 1.0)))
        self.is_heading_env = torch.as_tensor(is_heading)
        self.heading_target = torch.as_tensor(target)
        self.robot = ns(data=ns(heading_w=torch.as_tensor(heading_w)))
        self.vel_command_b = torch.as_tensor(cmd.copy())
        self.velocity_deadzone = dz
        self.dt = 0.005
        self.max_episode_length_s = 20.0
        self._resample = lambda ids: resampled.extend(int(i) for i in ids)
        Cm.torch = _TorchProxy(u)
        try:
            Cm.UniformVelocityCommandWithDeadzone._update_command(self)
        finally:
            Cm.torch = torch
        act = np.zeros(n, bool)
        act[resampled] = True
        out.update({f"c{case}_cmd_in": cmd, f"c{case}_quat": quat, f"c{case}_heading_w": heading_w,
                    f"c{case}_target": target, f"c{case}_is_heading": is_heading, f"c{case}_u": u.numpy(),
                    f"c{case}_deadzone": dz, f"c{case}_heading_command": heading,
                    f"c{case}_cmd_out": self.vel_command_b.numpy(), f"c{case}_activated": act,
                    f"c{case}_p_flip": 0.005 / 20.0})
    out["n_cases"] = 4
    np.savez_compressed(OUT / "ref_commands.npz", **out)


# ------------------------------------------------------------------------------------------------ curricula
def gen_curriculum(rng):
    Cv = load("ref_curriculums", BT / "tasks/locomotion/velocity/mdp/curriculums.py")
    Cc = load("ref_cat_curriculums", BT / "utils/cat/curriculums.py")
    n = 256
    origins = rng.uniform(-40, 40, (n, 3)).astype(np.float32)
    d = rng.choice([0.5, 3.9, 4.0, 4.1, 7.0, 9.5, 10.5, 20.0], n) + rng.uniform(-0.05, 0.05, n)
    ang = rng.uniform(0, 2 * math.pi, n)
    pos = origins.copy()
    pos[:, 0] += d * np.cos(ang)
    pos[:, 1] += d * np.sin(ang)
    pos[:, 2] += rng.uniform(0.5, 1.2, n)
    pos = pos.astype(np.float32)
    cmd = (rng.uniform(-1, 1, (n, 3)) * rng.choice([0.0, 0.3, 1.0], (n, 1))).astype(np.float32)
    rec = {}
    terrain = ns(cfg=ns(terrain_generator=ns(size=(8.0, 8.0))), terrain_levels=torch.zeros(n),
                 update_env_origins=lambda ids, up, down: rec.update(up=up.numpy(), down=down.numpy()))
    class Scene(types.SimpleNamespace):  # InteractiveScene: scene["robot"], scene.env_origins, scene.terrain
        def __getitem__(self, k):
            return self.entities[k]

    scene = Scene(entities={"robot": ns(data=ns(root_pos_w=torch.as_tensor(pos)))},
                  env_origins=torch.as_tensor(origins), terrain=terrain)
    env = ns(scene=scene, command_manager=ns(get_command=lambda name: torch.as_tensor(cmd)), max_episode_length_s=20.0)
    Cv.terrain_levels_vel(env, torch.arange(n), asset_cfg=SceneEntityCfg("robot"))
    # modify_constraint_p over a counter sweep
    counters = np.array([0, 1, 24, 1000, 12000, 59999, 60000, 120000, 240000, 10 ** 7])
    mps = []
    for init in (0.25, 0.05, 1.0):
        row = []
        for cnt in counters:
            term = ns(max_p=None)
            cm = ns(get_term_cfg=lambda name, t=term: t, set_term_cfg=lambda name, t: None)
            e = ns(common_step_counter=int(cnt), constraint_manager=cm)
            row.append(Cc.modify_constraint_p(e, None, term_name="x", num_steps=120000, init_max_p=init))
        mps.append(row)
    np.savez_compressed(OUT / "ref_curriculum.npz", pos=pos, origins=origins, cmd=cmd, terrain_size=8.0,
                        max_episode_length_s=20.0, move_up=rec["up"], move_down=rec["down"], counters=counters,
                        init_max_p=np.array([0.25, 0.05, 1.0]), num_steps=120000, max_p=np.array(mps))


# ------------------------------------------------------------------------------------------------ observations
def gen_obs_manager(rng):
    install = sys.modules["biped_tasks.utils.history.circular_buffer"]
    OM = load("ref_observation_manager", BT / "utils/history/observation_manager.py")
    out = {}
    layouts = {
        # name: (term dims, noise n_max per term (None = no noise), scale per term, clip per term, history)
        "flat": ([3, 3, 3, 12, 12, 12], [0.2, 0.05, None, 0.01, 1.5, None], [None] * 6, [None] * 6, 10),
        "rsl": ([3, 3, 3, 12, 12, 12], [0.2, 0.05, None, 0.01, 1.5, None], [0.25, None, None, None, 0.05, None],
                [None] * 6, 6),
        "rough": ([3, 3, 3, 3, 12, 12, 12, 187], [0.1, 0.2, 0.05, None, 0.01, 1.5, None, 0.1], [None] * 8,
                  [None] * 7 + [(-1.0, 1.0)], 0),
    }
    for name, (dims, noise, scale, clip, H) in layouts.items():
        n, T = 8, 13
        raw = [rng.normal(size=(T, n, d)).astype(np.float32) * (2.0 if d == 187 else 1.0) for d in dims]
        us = [rng.random((T, n, d)).astype(np.float32) for d in dims]
        resets = np.zeros((T, n), bool)
        resets[4, [1, 5]] = True
        resets[9, [0, 1, 7]] = True
        cur = {"t": 0}
        cfgs = []
        for k, d in enumerate(dims):
            nz = None
            if noise[k] is not None:
                nm = noise[k]
                nz = ns(n_min=-nm, n_max=nm,
                        func=lambda data, c, k=k: data + f32(us[k][cur["t"]]) * (c.n_max - c.n_min) + c.n_min)
            cfgs.append(ns(func=lambda env, k=k: f32(raw[k][cur["t"]]), params={}, modifiers=None, noise=nz,
                           clip=clip[k], scale=scale[k], history_length=H, flatten_history_dim=True,
                           history_step=1))
        names = [f"t{k}" for k in range(len(dims))]
        bufs = {nm: install.CircularBuffer(max_len=H, batch_size=n, device="cpu") for nm in names} if H > 0 else {}
        self = ns(_group_obs_term_names={"policy": names}, _group_obs_term_cfgs={"policy": cfgs},
                  _group_obs_term_history_buffer={"policy": bufs}, _group_obs_concatenate={"policy": True},
                  _env=ns(num_envs=n))
        obs = []
        for t in range(T):
            cur["t"] = t
            ids = np.nonzero(resets[t])[0]
            if len(ids) and H > 0:  # ObservationManager.reset -> CircularBuffer.reset of the reset envs
                for b in bufs.values():
                    b.reset(batch_ids=ids.tolist())
            obs.append(OM.ObservationManager.compute_group(self, "policy").numpy())
        for k in range(len(dims)):
            out[f"{name}_raw{k}"] = raw[k]
            out[f"{name}_u{k}"] = us[k]
        out[f"{name}_resets"] = resets
        out[f"{name}_obs"] = np.array(obs)
        out[f"{name}_history"] = H
    np.savez_compressed(OUT / "ref_obs_manager.npz", **out)


def main():
    OUT.mkdir(parents=True, exist_ok=True)
    install_stubs()
    rng = np.random.default_rng(20261016)
    gen_rewards(rng)
    gen_constraints(rng)
    gen_commands(rng)
    gen_curriculum(rng)
    gen_obs_manager(rng)
    for f in sorted(OUT.glob("ref_*.npz")):
        print(f, f.stat().st_size, "bytes")


if __name__ == "__main__":
    main()
