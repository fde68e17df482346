"""Configuration tree of `Isaac-Velocity-Flat-H12_12dof-v0`, restated as plain dataclasses.

Attribute paths mirror the IsaacLab cfg objects the reference composes, so scripts that poke at
`env_cfg.scene.num_envs`, `env_cfg.seed`, `env_cfg.sim.device`, `env_cfg.rewards.<term>.weight`,
`env_cfg.commands.base_velocity.ranges.lin_vel_x` ... keep working.  Values are the merged Flat
config:

  - sim / decimation / episode: velocity_env_cfg.py:299-315 (dt 0.005, decimation 4, 20 s)
  - actions: velocity_env_cfg.py:111 (JointPositionAction, scale 0.5, default offset)
  - actuators: packages/biped_assets/biped_assets/robots/h12.py:58-112 (DelayedPD, Kp/Kd/E, 0-5 delay)
  - commands: velocity_env_cfg.py:90-104 + flat_env_cfg.py:46-48
  - observations: velocity_env_cfg.py:124-132, flat_env_cfg.py:25-27 (no lin vel, history 10, noise on)
  - events: rough_env_cfg.py:77-92 (x,y +-0.5, yaw +-3.14, joints x1.0, no push, no mass)
  - rewards: rough_env_cfg.py:19-62 (term table), 111-120 (weights) + flat_env_cfg.py:35-44
  - terminations: velocity_env_cfg.py:264-268 + rough_env_cfg.py:95-109 (illegal-contact bodies)
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field, replace

from ._abi import (ABI_VERSION, CONSTRAINT_TERMS, MODE_ISAACLAB, MODE_MUJOCO, NCSTR, NHIST, NJ, NREW, REWARD_FUNCS,
                   REWARD_TERMS, TASK_FLAT, TASK_ROUGH, H12Config)
from .model import DEFAULT_JOINT_POS


@dataclass
class SimCfg:
    dt: float = 0.005
    device: str = "cuda:0"
    render_interval: int = 4
    # contact / integration parameters of the build's penalty model (DESIGN.md "Physics model")
    # one integration step per 5 ms physics step (PhysX's sim.dt) with the contact springs integrated
    # implicitly; inner_steps = 2 / implicit_penalty = False is the round-1 explicit scheme
    inner_steps: int = 1
    implicit_penalty: bool = True
    # PhysX enforces the articulation's max joint velocities (RobotCfg.joint_vel_limits, from the USD);
    # here: a stiff joint damper above the limit, integrated implicitly
    joint_velocity_limit: bool = True
    joint_velocity_limit_damping: float = 1.0e3
    # self-collision between the legs (h12.py:32 enabled_self_collisions=True): knee and sole-rod capsules,
    # explicit penalty: the ground contact's stiffness, damping below the explicit
    # stability bound c h / m_eff < 2 of the lightest contact DOF (toe about the ankle pitch, ~0.35 kg)
    self_collision: bool = True
    self_k: float = 3.0e4
    self_c: float = 50.0
    self_ct: float = 50.0
    self_mu: float = 0.36
    # ground contact: sole spheres / knee / torso, active on the predicted end-of-step depth, implicit.  PhysX's
    # contacts are rigid; 1e5 N/m gives a median sole penetration of 3.7 mm under random actions, 7e5 would give
    # 1.8 mm at 4x the fp32 threshold sensitivity
    contact_k: float = 1.0e5
    contact_c: float = 100.0
    # the explicit integrator (implicit_penalty = False: MuJoCo mode, the round-1 scheme) keeps the soft contact it is
    # stable with
    contact_k_explicit: float = 3.0e4
    contact_c_explicit: float = 100.0
    # RigidBodyPropertiesCfg.max_depenetration_velocity (A/robots/h12.py:29): the contact spring pushes a penetration
    # out at most this fast (implicit scheme)
    max_depenetration_velocity: float = 1.0
    friction_k: float = 3.0e4
    friction_c: float = 100.0
    # joint limits: PhysX holds the URDF ranges as hard limits; here a stiff spring on the predicted end-of-step
    # position, integrated implicitly.  The explicit integrator (implicit_penalty = False:
    # MuJoCo mode, the round-1 scheme) keeps the soft limit_k_explicit, all it is stable with
    limit_k: float = 1.0e6
    limit_k_explicit: float = 1.0e3
    limit_c: float = 2.0
    # a joint still carried further than this past its range within a step is projected back (hard-limit residual;
    # implicit scheme only)
    limit_projection: float = 0.01
    # MuJoCo mode: the MJCF joints' frictionloss (0.1 N m, a dry-friction constraint in MuJoCo) as a smooth
    # -f tanh(100 qd) torque; off by default
    frictionloss: bool = False
    static_friction: float = 0.8   # randomize_rigid_body_material startup (velocity_env_cfg.py:153-163)
    dynamic_friction: float = 0.6


@dataclass
class TerrainGeneratorCfg:
    """ROUGH_TERRAINS_CFG (biped_tasks/utils/mdp/terrains.py:11-28): one HfRandomUniform sub-terrain type."""
    size: tuple = (8.0, 8.0)
    border_width: float = 20.0
    num_rows: int = 10
    num_cols: int = 20
    horizontal_scale: float = 0.1
    vertical_scale: float = 0.005
    slope_threshold: float = 0.75
    curriculum: bool = True
    # HfRandomUniformTerrainCfg
    noise_range: tuple = (0.0, 0.02)
    noise_step: float = 0.005
    sub_border_width: float = 0.25


@dataclass
class TerrainCfg:
    """TerrainImporterCfg (velocity_env_cfg.py:40-56)."""
    terrain_type: str = "plane"            # "plane" | "generator"
    terrain_generator: TerrainGeneratorCfg | None = None
    max_init_terrain_level: int | None = 5
    static_friction: float = 1.0           # ground material, multiply-combined
    dynamic_friction: float = 1.0


@dataclass
class HeightScannerCfg:
    """RayCasterCfg at torso_link, offset z 20, yaw only, GridPatternCfg(0.1, (1.6, 1.0)) (velocity_env_cfg.py:58-66)."""
    prim_path: str = "{ENV_REGEX_NS}/Robot/torso_link"
    resolution: float = 0.1
    size: tuple = (1.6, 1.0)
    attach_yaw_only: bool = True


@dataclass
class SceneCfg:
    num_envs: int = 4096
    env_spacing: float = 2.5
    lazy_sensor_update: bool = True
    terrain: TerrainCfg = field(default_factory=TerrainCfg)
    height_scanner: HeightScannerCfg | None = None


@dataclass
class ActuatorGroupCfg:
    joint_names_expr: list
    effort_limit: float
    stiffness: float
    damping: float
    armature: float = 0.01
    friction: float = 0.0
    min_delay: int = 0
    max_delay: int = 5


@dataclass
class RobotCfg:
    init_pos: tuple = (0.0, 0.0, 1.05)
    joint_pos: tuple = tuple(DEFAULT_JOINT_POS)
    soft_joint_pos_limit_factor: float = 0.9
    # ArticulationData.joint_vel_limits / joint_effort_limits as the sim holds them: the URDF velocity limits
    # (h12_12dof.urdf:53-198, USD import keeps them) and, for explicit actuator models, IsaacLab's 1e9 effort
    # limit in the solver; read by the CaT joint_velocity_limits / joint_torque_limits constraints
    joint_vel_limits: tuple = (23.0, 23.0, 23.0, 14.0, 9.0, 9.0) * 2
    joint_effort_limits_sim: tuple = (1.0e9,) * 12
    actuators: dict = field(default_factory=lambda: {
        "legs": ActuatorGroupCfg([".*_hip_yaw_joint", ".*_hip_roll_joint", ".*_hip_pitch_joint"], 220.0, 200.0, 2.5),
        "knees": ActuatorGroupCfg([".*_knee_joint"], 360.0, 300.0, 4.0),
        "feet": ActuatorGroupCfg([".*_ankle_pitch_joint", ".*_ankle_roll_joint"], 45.0, 40.0, 2.0),
    })


@dataclass
class JointPositionActionCfg:
    asset_name: str = "robot"
    joint_names: tuple = (".*",)
    scale: float = 0.5
    use_default_offset: bool = True


@dataclass
class ActionsCfg:
    joint_pos: JointPositionActionCfg = field(default_factory=JointPositionActionCfg)


@dataclass
class Ranges:
    lin_vel_x: tuple = (0.0, 1.0)
    lin_vel_y: tuple = (-0.5, 0.5)
    ang_vel_z: tuple = (-1.0, 1.0)
    heading: tuple = (-math.pi, math.pi)


@dataclass
class UniformVelocityCommandCfg:
    asset_name: str = "robot"
    resampling_time_range: tuple = (10.0, 10.0)
    rel_standing_envs: float = 0.02
    rel_heading_envs: float = 1.0
    heading_command: bool = True
    heading_control_stiffness: float = 0.5
    debug_vis: bool = False
    ranges: Ranges = field(default_factory=Ranges)


@dataclass
class UniformVelocityCommandWithDeadzoneCfg(UniformVelocityCommandCfg):
    """biped_tasks/utils/mdp/commands.py:99-104: half of the envs kept in |cmd_xy| < velocity_deadzone,
    random cmd_z sign flips, no standing-env zeroing (the kernel's deadzone command mode)."""
    velocity_deadzone: float = 0.1


@dataclass
class CommandsCfg:
    base_velocity: UniformVelocityCommandCfg = field(default_factory=UniformVelocityCommandCfg)


@dataclass
class Unoise:
    n_min: float
    n_max: float


@dataclass
class PolicyObsCfg:
    enable_corruption: bool = True
    concatenate_terms: bool = True
    history_length: int = 10
    # term order preserved (velocity_env_cfg.py:118-137; base_lin_vel and height_scan removed for Flat)
    base_lin_vel: Unoise | None = None
    base_ang_vel: Unoise = field(default_factory=lambda: Unoise(-0.2, 0.2))
    projected_gravity: Unoise = field(default_factory=lambda: Unoise(-0.05, 0.05))
    velocity_commands: None = None
    joint_pos: Unoise = field(default_factory=lambda: Unoise(-0.01, 0.01))
    joint_vel: Unoise = field(default_factory=lambda: Unoise(-1.5, 1.5))
    actions: None = None
    height_scan: Unoise | None = None
    height_scan_clip: tuple = (-1.0, 1.0)
    height_scan_offset: float = 0.5
    # ObsTerm(scale=...) per term (applied after noise); missing terms are unscaled
    scales: dict = field(default_factory=dict)


@dataclass
class ObservationsCfg:
    policy: PolicyObsCfg = field(default_factory=PolicyObsCfg)


@dataclass
class RewTerm:
    """RewardTermCfg: weight, params and `func` -- the kernel term it maps to (one of _abi.REWARD_FUNCS: the
    isaaclab mdp function, qualified by its joint set / frame where the kernel hard-codes one)."""
    weight: float
    params: dict = field(default_factory=dict)
    func: "str | tuple | None" = None   # one kernel term, or several summed (one joint set split over ids)


def _funcs(v) -> tuple:
    return tuple(v) if isinstance(v, (tuple, list)) else (v,)


_FLAT_FUNCS = dict(zip(REWARD_TERMS, REWARD_FUNCS[:len(REWARD_TERMS)]))


def _rewards():
    T = RewTerm
    return {
        "track_lin_vel_xy_exp": T(1.0, {"command_name": "base_velocity", "std": 0.5}, "track_lin_vel_xy_yaw_frame_exp"),
        "track_ang_vel_z_exp": T(1.0, {"command_name": "base_velocity", "std": 0.5}, "track_ang_vel_z_world_exp"),
        "ang_vel_xy_l2": T(-0.05, {}, "ang_vel_xy_l2"),
        "dof_torques_l2": T(-2.0e-6, {}, "joint_torques_l2"),
        "dof_acc_l2": T(-1.0e-7, {}, "joint_acc_l2"),
        "action_rate_l2": T(-0.005, {}, "action_rate_l2"),
        "feet_air_time": T(0.75, {"command_name": "base_velocity", "threshold": 0.4}, "feet_air_time_positive_biped"),
        "flat_orientation_l2": T(-1.0, {}, "flat_orientation_l2"),
        "dof_pos_limits": T(-1.0, {}, "joint_pos_limits:ankle"),
        "termination_penalty": T(-200.0, {}, "is_terminated"),
        "feet_slide": T(-0.25, {}, "feet_slide"),
        "joint_deviation_hip": T(-0.2, {}, "joint_deviation_l1:hip"),
    }


def _rsl_rewards():
    """rsl_env_cfg.py:279-407, in its RewardManager order."""
    T = RewTerm
    return {
        "track_lin_vel_xy_exp": T(1.0, {"command_name": "base_velocity", "std": 0.5}, "track_lin_vel_xy_exp"),
        "track_ang_vel_z_exp": T(0.5, {"command_name": "base_velocity", "std": 0.5}, "track_ang_vel_z_exp"),
        "feet_air_time": T(0.75, {"command_name": "base_velocity", "threshold": 0.4}, "feet_air_time_positive_biped"),
        "feet_slide": T(-0.25, {}, "feet_slide"),
        "flat_orientation": T(-1.0, {}, "flat_orientation_l2"),
        "base_height_l2": T(-0.2, {"target_height": 1.0}, "base_height_l2"),
        "joint_torques_l2": T(-1.0e-5, {}, "joint_torques_l2"),
        "joint_vel_l2": T(-1.0e-3, {}, "joint_vel_l2"),
        "dof_acc_l2": T(-1.0e-7, {}, "joint_acc_l2"),
        "joint_deviation_hip": T(-0.2, {}, "joint_deviation_l1:hip"),
        "joint_deviation_ankle": T(-0.2, {}, "joint_deviation_l1:ankle"),
        "joint_pos_limits_ankle": T(-0.2, {}, "joint_pos_limits:ankle"),
        "joint_pos_limits_hip": T(-0.2, {}, "joint_pos_limits:hip"),
        "action_rate_l2": T(-0.01, {}, "action_rate_l2"),
        "contact_forces": T(-1.0e-3, {"threshold": 800.0}, "contact_forces"),
        "termination_penalty": T(-200.0, {}, "is_terminated"),
    }


class RewardsCfg:
    """Attribute-access container keeping the cfg's RewardManager term order.  A term set to None is
    removed (as in IsaacLab); a new RewTerm must name the kernel term it maps to (`func`)."""

    def __init__(self, terms=None):
        object.__setattr__(self, "_terms", terms or _rewards())

    def __getattr__(self, name):
        if name.startswith("__") or name == "_terms":
            raise AttributeError(name)
        try:
            return self._terms[name]
        except KeyError as e:
            raise AttributeError(name) from e

    def __getstate__(self):
        return {"_terms": self._terms}

    def __setstate__(self, st):
        object.__setattr__(self, "_terms", st["_terms"])

    def __setattr__(self, name, value):
        if value is not None:
            if not isinstance(value, RewTerm):
                raise TypeError(f"reward term {name!r} must be a RewTerm or None")
            func = value.func or (self._terms[name].func if self._terms.get(name) is not None else _FLAT_FUNCS.get(name))
            if func is None or any(f not in REWARD_FUNCS for f in _funcs(func)):
                raise AttributeError(f"reward term {name!r}: func {func!r} is not a kernel term {REWARD_FUNCS}")
            value.func = func
        self._terms[name] = value

    def items(self):
        return list(self._terms.items())

    def active(self):
        """(name, kernel ids) of the terms the RewardManager holds (None terms removed), in cfg order."""
        out, seen = [], {}
        for k, v in self._terms.items():
            if v is None:
                continue
            ids = tuple(REWARD_FUNCS.index(f) for f in _funcs(v.func))
            for kid in ids:
                if kid in seen:
                    raise ValueError(f"reward terms {seen[kid]!r} and {k!r} map to the same kernel term "
                                     f"{REWARD_FUNCS[kid]!r}")
                seen[kid] = k
            out.append((k, ids))
        return out

    def to_dict(self):
        return {k: (None if v is None else {"weight": v.weight, "params": dict(v.params), "func": v.func})
                for k, v in self.items()}


@dataclass
class TerminationsCfg:
    time_out: bool = True
    base_contact_threshold: float = 1.0
    # bodies of the illegal-contact list that carry colliders in the USD's source URDF
    base_contact_knees: bool = True
    base_contact_torso: bool = True


@dataclass
class PushEventCfg:
    """push_by_setting_velocity, mode "interval" (rsl_env_cfg.py:262-273)."""
    interval_range_s: tuple = (5.0, 8.0)
    velocity_range: dict = field(default_factory=lambda: {"x": (-1.0, 1.0), "y": (-1.0, 1.0)})


@dataclass
class EventsCfg:
    reset_base_pose_range: dict = field(default_factory=lambda: {"x": (-0.5, 0.5), "y": (-0.5, 0.5), "yaw": (-3.14, 3.14)})
    reset_joints_position_range: tuple = (1.0, 1.0)
    push_robot: "PushEventCfg | None" = None
    # startup randomisation (randomize_rigid_body_material / _mass, velocity_env_cfg.py:146-166,
    # cat_env_cfg.py:231-249); None = the constant material of the Flat task / no added mass
    physics_material: "MaterialEventCfg | None" = None
    add_base_mass: "MassEventCfg | None" = None


@dataclass
class MaterialEventCfg:
    static_friction_range: tuple = (0.8, 0.8)
    dynamic_friction_range: tuple = (0.6, 0.6)
    num_buckets: int = 64


@dataclass
class MassEventCfg:
    body_names: str = ".*torso_link"
    mass_distribution_params: tuple = (0.0, 6.0)
    operation: str = "add"


@dataclass
class ConstraintTerm:
    """ConstraintTermCfg (T/utils/cat/manager_constraint_cfg.py): `func` names the kernel constraint
    (one of _abi.CONSTRAINT_TERMS), max_p its maximum termination probability, params its limits."""
    func: str
    max_p: float
    params: dict = field(default_factory=dict)


def _cat_constraints():
    """cat_env_cfg.py:336-427 (ConstraintsCfg order)."""
    T = ConstraintTerm
    return {
        "contact": T("contact", 1.0),
        "joint_position_limits": T("joint_position_limits", 0.25),
        "joint_velocity_limits": T("joint_velocity_limits", 0.25),
        "joint_torque_limits": T("joint_torque_limits", 0.25),
        "foot_contact_force": T("foot_contact_force", 0.25, {"limit": 750.0}),
        "no_move": T("no_move", 0.25, {"velocity_deadzone": 0.2, "joint_vel_limit": 6.0}),
        "base_orientation": T("base_orientation", 0.25, {"limit": 0.1}),
        "base_height": T("base_height", 0.25, {"height": 1.0, "std": 0.05}),
        "foot_contact": T("foot_contact", 0.25),
        "foot_clearance": T("foot_clearance", 0.25, {"min_height": 0.1, "velocity_deadzone": 0.2}),
    }


class ConstraintsCfg:
    """Attribute-access container of the ConstraintManager's terms (cfg order); a term set to None is removed."""

    def __init__(self, terms=None):
        object.__setattr__(self, "_terms", terms if terms is not None else _cat_constraints())

    def __getattr__(self, name):
        if name.startswith("__") or name == "_terms":
            raise AttributeError(name)
        try:
            return self._terms[name]
        except KeyError as e:
            raise AttributeError(name) from e

    def __getstate__(self):
        return {"_terms": self._terms}

    def __setstate__(self, st):
        object.__setattr__(self, "_terms", st["_terms"])

    def __setattr__(self, name, value):
        if value is not None and (not isinstance(value, ConstraintTerm) or value.func not in CONSTRAINT_TERMS):
            raise AttributeError(f"constraint {name!r} must be a ConstraintTerm on one of {CONSTRAINT_TERMS}")
        self._terms[name] = value

    def items(self):
        return list(self._terms.items())

    def active(self):
        """(name, kernel constraint id) in cfg order."""
        out, seen = [], set()
        for k, v in self._terms.items():
            if v is None:
                continue
            cid = CONSTRAINT_TERMS.index(v.func)
            if cid in seen:
                raise ValueError(f"two constraints map to the kernel term {v.func!r}")
            seen.add(cid)
            out.append((k, cid))
        return out

    def to_dict(self):
        return {k: (None if v is None else {"func": v.func, "max_p": v.max_p, "params": dict(v.params)})
                for k, v in self.items()}


@dataclass
class ConstraintPTerm:
    """modify_constraint_p (T/utils/cat/curriculums.py:16-42): max_p = 1 / (20 + progress (1 / init_max_p - 20)),
    progress = min(common_step_counter / num_steps, 1)."""
    term_name: str
    num_steps: int
    init_max_p: float

    def max_p(self, step: int) -> float:
        progress = min(step / self.num_steps, 1.0)
        return 1.0 / (20 + progress * (1 / self.init_max_p - 20))


@dataclass
class RewardWeightTerm:
    """modify_reward_weight (isaaclab mdp.curriculums): once common_step_counter > num_steps, the
    reward term's weight becomes `weight`."""
    term_name: str
    weight: float
    num_steps: int


@dataclass
class CurriculumCfg:
    terrain_levels: bool = False  # terrain_levels_vel (velocity_env_cfg.py:271-275)
    reward_weights: list = field(default_factory=list)  # [RewardWeightTerm] (rsl_env_cfg.py:448-501)
    constraint_p: list = field(default_factory=list)    # [ConstraintPTerm] (cat_env_cfg.py:466-520)


@dataclass
class H12FlatEnvCfg:
    """Merged cfg of `Isaac-Velocity-Flat-H12_12dof-v0` (H12_12dof_FlatEnvCfg, flat_env_cfg.py:13-48)."""

    seed: int | None = 42
    decimation: int = 4
    episode_length_s: float = 20.0
    mode: int = MODE_ISAACLAB
    sim: SimCfg = field(default_factory=SimCfg)
    scene: SceneCfg = field(default_factory=SceneCfg)
    robot: RobotCfg = field(default_factory=RobotCfg)
    actions: ActionsCfg = field(default_factory=ActionsCfg)
    commands: CommandsCfg = field(default_factory=CommandsCfg)
    observations: ObservationsCfg = field(default_factory=ObservationsCfg)
    rewards: RewardsCfg = field(default_factory=RewardsCfg)
    terminations: TerminationsCfg = field(default_factory=TerminationsCfg)
    events: EventsCfg = field(default_factory=EventsCfg)
    curriculum: CurriculumCfg = field(default_factory=CurriculumCfg)
    constraints: "ConstraintsCfg | None" = None   # the CaT task's ConstraintManager terms
    fix_base: bool = False

    @property
    def task(self) -> int:
        """Rough layout (235-float obs with height scan) when the scene has a height scanner."""
        return TASK_ROUGH if self.scene.height_scanner is not None else TASK_FLAT

    @property
    def step_dt(self) -> float:
        return self.sim.dt * self.decimation

    @property
    def max_episode_length(self) -> int:
        return math.ceil(self.episode_length_s / self.step_dt)

    def to_c(self) -> H12Config:
        from .model import joint_names

        names = joint_names()
        c = H12Config()
        c.abi_version = ABI_VERSION
        c.mode = self.mode
        c.physics_dt = self.sim.dt
        c.decimation = self.decimation
        c.inner_steps = self.sim.inner_steps
        c.implicit_penalty = int(self.sim.implicit_penalty)
        if self.mode == MODE_ISAACLAB and self.sim.joint_velocity_limit:
            c.max_joint_vel[:] = self.robot.joint_vel_limits
            c.max_joint_vel_damping = self.sim.joint_velocity_limit_damping
        c.self_collision = int(self.sim.self_collision and self.mode == MODE_ISAACLAB)
        c.self_k, c.self_c = self.sim.self_k, self.sim.self_c
        c.self_ct, c.self_mu = self.sim.self_ct, self.sim.self_mu
        c.max_episode_length = self.max_episode_length
        c.action_scale = self.actions.joint_pos.scale
        import re

        groups = list(self.robot.actuators.items())
        for j, name in enumerate(names):
            hit = None
            for gi, (gname, g) in enumerate(groups):
                if any(re.fullmatch(p, name) for p in g.joint_names_expr):
                    hit = (gi, g)
                    break
            if hit is None:
                raise ValueError(f"joint {name} has no actuator group")
            gi, g = hit
            c.kp[j] = g.stiffness
            c.kd[j] = g.damping
            c.effort_limit[j] = g.effort_limit
            c.delay_group[j] = gi
        g0 = groups[0][1]
        c.min_delay, c.max_delay = g0.min_delay, g0.max_delay
        if any((g.min_delay, g.max_delay) != (g0.min_delay, g0.max_delay) for _, g in groups):
            raise ValueError("all actuator groups must share the delay range")
        if c.max_delay > 2 * self.decimation:
            raise ValueError("max_delay must be <= 2 * decimation (delay ring holds two env steps)")
        c.fix_base = int(self.fix_base)
        c.use_frictionloss = int(self.sim.frictionloss)
        s = self.sim
        c.contact_k, c.contact_c = ((s.contact_k, s.contact_c) if s.implicit_penalty
                                    else (s.contact_k_explicit, s.contact_c_explicit))
        c.friction_k, c.friction_c = s.friction_k, s.friction_c
        c.mu_static, c.mu_dynamic = s.static_friction, s.dynamic_friction
        c.limit_k, c.limit_c = (s.limit_k if s.implicit_penalty else s.limit_k_explicit), s.limit_c
        c.limit_projection = s.limit_projection if s.implicit_penalty else 0.0
        c.max_depenetration_velocity = s.max_depenetration_velocity if s.implicit_penalty else 0.0
        c.contact_threshold = self.terminations.base_contact_threshold
        bv = self.commands.base_velocity
        c.cmd_resample_time, c.cmd_resample_time_max = bv.resampling_time_range
        if isinstance(bv, UniformVelocityCommandWithDeadzoneCfg):
            c.cmd_deadzone = 1
            c.velocity_deadzone = bv.velocity_deadzone
            c.ang_flip_prob = self.sim.dt / self.episode_length_s   # commands.py:86-87: physics_dt / episode s
        r = bv.ranges
        c.cmd_lin_x[:] = r.lin_vel_x
        c.cmd_lin_y[:] = r.lin_vel_y
        c.cmd_ang_z[:] = r.ang_vel_z
        c.cmd_heading[:] = r.heading
        c.rel_standing_envs = bv.rel_standing_envs
        c.rel_heading_envs = bv.rel_heading_envs if bv.heading_command else -1.0
        c.heading_stiffness = bv.heading_control_stiffness
        pr = self.events.reset_base_pose_range
        c.reset_x[:] = pr["x"]
        c.reset_y[:] = pr["y"]
        c.reset_yaw[:] = pr["yaw"]
        po = self.observations.policy
        c.task = self.task
        c.history_length = max(1, int(po.history_length or 0))
        if c.task == TASK_FLAT and c.history_length > NHIST:
            raise ValueError(f"observation history is at most {NHIST} frames")
        for i, k in enumerate(("base_ang_vel", "projected_gravity", "velocity_commands", "joint_pos", "joint_vel",
                               "actions")):
            c.obs_scale[i] = float(po.scales.get(k, 1.0))
        if set(po.scales) - {"base_ang_vel", "projected_gravity", "velocity_commands", "joint_pos", "joint_vel",
                             "actions"}:
            raise ValueError(f"observation scales for unsupported terms: {sorted(po.scales)}")
        if c.task == TASK_ROUGH:
            if po.history_length not in (0, 1, None):
                raise ValueError("the rough observation has no history (history_length 0)")
            if po.base_lin_vel is None or po.height_scan is None:
                raise ValueError("the rough layout needs base_lin_vel and height_scan terms")
            c.noise_lin_vel = po.base_lin_vel.n_max
            c.noise_height_scan = po.height_scan.n_max
            c.scan_offset = po.height_scan_offset
            c.scan_clip = po.height_scan_clip[1]
            hs = self.scene.height_scanner
            if tuple(hs.size) != (1.6, 1.0) or abs(hs.resolution - 0.1) > 1e-9:
                raise ValueError("the kernel's height scan grid is 17 x 11 rays at 0.1 m")
            c.scan_resolution = hs.resolution
        else:
            if po.base_lin_vel is not None or po.height_scan is not None:
                raise ValueError("base_lin_vel / height_scan need the rough layout (scene.height_scanner)")
            c.noise_lin_vel, c.noise_height_scan, c.scan_offset, c.scan_clip, c.scan_resolution = 0.1, 0.1, 0.5, 1.0, 0.1
        t = self.scene.terrain
        c.terrain = 1 if t.terrain_type == "generator" else 0
        c.terrain_curriculum = int(bool(self.curriculum.terrain_levels) and c.terrain == 1)
        c.terrain_size = t.terrain_generator.size[0] if t.terrain_generator is not None else 8.0
        c.per_env_friction = int(self.events.physics_material is not None)
        c.per_env_mass = int(self.events.add_base_mass is not None)
        c.enable_corruption = int(po.enable_corruption)
        c.noise_ang_vel = po.base_ang_vel.n_max
        c.noise_gravity = po.projected_gravity.n_max
        c.noise_joint_pos = po.joint_pos.n_max
        c.noise_joint_vel = po.joint_vel.n_max
        terms = dict(self.rewards.items())
        for t in range(NREW):
            c.rew_w[t] = 0.0
        stds = set()
        c.track_std, c.air_time_threshold, c.base_height_target, c.contact_force_threshold = 0.5, 0.4, 1.0, 800.0
        for name, kids in self.rewards.active():
            term = terms[name]
            for kid in kids:
                c.rew_w[kid] = term.weight
                f = REWARD_FUNCS[kid]
                if f.startswith("track_"):
                    stds.add(float(term.params.get("std", 0.5)))
                elif f == "feet_air_time_positive_biped":
                    c.air_time_threshold = term.params.get("threshold", 0.4)
                elif f == "base_height_l2":
                    c.base_height_target = term.params.get("target_height", 1.0)
                elif f == "contact_forces":
                    c.contact_force_threshold = term.params.get("threshold", 1.0)
        if len(stds) > 1:
            raise ValueError(f"the tracking terms must share one std (got {sorted(stds)})")
        if stds:
            c.track_std = stds.pop()
        pe = self.events.push_robot
        c.push_interval[:], c.push_vel_x[:], c.push_vel_y[:] = (5.0, 8.0), (-1.0, 1.0), (-1.0, 1.0)  # C defaults
        if pe is not None:
            c.push_enable = 1
            c.push_interval[:] = pe.interval_range_s
            vr = pe.velocity_range
            if set(vr) - {"x", "y"}:
                raise ValueError("push velocity ranges other than x / y are not implemented")
            c.push_vel_x[:] = vr.get("x", (0.0, 0.0))
            c.push_vel_y[:] = vr.get("y", (0.0, 0.0))
        c.soft_limit_factor = self.robot.soft_joint_pos_limit_factor
        c.illegal_contact_knees = int(self.terminations.base_contact_knees)
        c.illegal_contact_torso = int(self.terminations.base_contact_torso)
        c.seed = (self.seed if self.seed is not None else 0) & 0xFFFFFFFFFFFFFFFF
        self._constraints_to_c(c)
        assert NJ == 12
        return c

    def _constraints_to_c(self, c):
        # C defaults (h12env_config_default) when the task has no ConstraintManager
        c.cat_enable, c.cstr_mask, c.cat_tau, c.cat_min_p = 0, (1 << NCSTR) - 1, 0.95, 0.0
        for t in range(NCSTR):
            c.cstr_max_p[t] = 1.0 if t == 0 else 0.25
        c.cstr_joint_vel_limit[:] = self.robot.joint_vel_limits
        c.cstr_joint_effort_limit[:] = self.robot.joint_effort_limits_sim
        c.cstr_foot_force_limit, c.cstr_nomove_deadzone, c.cstr_nomove_vel = 750.0, 0.2, 6.0
        c.cstr_orient_limit, c.cstr_height, c.cstr_height_std = 0.1, 1.0, 0.05
        c.cstr_clearance_min, c.cstr_clearance_deadzone = 0.1, 0.2
        if self.constraints is None:
            return
        c.cat_enable = 1
        c.cstr_mask = 0
        terms = dict(self.constraints.items())
        for name, cid in self.constraints.active():
            t = terms[name]
            c.cstr_mask |= 1 << cid
            c.cstr_max_p[cid] = t.max_p
            p = t.params
            f = CONSTRAINT_TERMS[cid]
            if f == "foot_contact_force":
                c.cstr_foot_force_limit = p.get("limit", 750.0)
            elif f == "no_move":
                c.cstr_nomove_deadzone = p.get("velocity_deadzone", 0.2)
                c.cstr_nomove_vel = p.get("joint_vel_limit", 6.0)
            elif f == "base_orientation":
                c.cstr_orient_limit = p.get("limit", 0.1)
            elif f == "base_height":
                c.cstr_height, c.cstr_height_std = p.get("height", 1.0), p.get("std", 0.05)
            elif f == "foot_clearance":
                c.cstr_clearance_min = p.get("min_height", 0.1)
                c.cstr_clearance_deadzone = p.get("velocity_deadzone", 0.2)


@dataclass
class H12RoughEnvCfg(H12FlatEnvCfg):
    """Isaac-Velocity-Rough-H12_12dof-v0 (H12_12dof_RoughEnvCfg, rough_env_cfg.py:65-125 on
    LocomotionVelocityRoughEnvCfg): generated heightfield + terrain curriculum, height scanner, base_lin_vel
    in the 235-float observation (no history), rough reward weights, lin_vel_y command 0."""

    def __post_init__(self):
        self.scene.terrain = TerrainCfg(terrain_type="generator", terrain_generator=TerrainGeneratorCfg(),
                                        max_init_terrain_level=5)
        self.scene.height_scanner = HeightScannerCfg()
        po = self.observations.policy
        po.history_length = 0
        po.base_lin_vel = Unoise(-0.1, 0.1)
        po.height_scan = Unoise(-0.1, 0.1)
        self.curriculum.terrain_levels = True
        r = self.rewards
        r.feet_air_time.weight = 0.25              # rough_env_cfg.py:34-42
        r.dof_torques_l2.weight = -1.5e-7          # :114
        r.dof_acc_l2.weight = -1.25e-7             # :116
        r.action_rate_l2.weight = -0.005           # :115
        r.flat_orientation_l2.weight = -1.0        # :113
        self.commands.base_velocity.ranges.lin_vel_x = (0.0, 1.0)   # :123-125
        self.commands.base_velocity.ranges.lin_vel_y = (0.0, 0.0)
        self.commands.base_velocity.ranges.ang_vel_z = (-1.0, 1.0)


@dataclass
class H12RoughEnvCfg_PLAY(H12RoughEnvCfg):
    """rough_env_cfg.py:128-154: 50 envs, 40 s episodes, random initial levels, 5 x 5 terrain, no noise."""

    def __post_init__(self):
        super().__post_init__()
        self.scene.num_envs = 50
        self.episode_length_s = 40.0
        self.scene.terrain.max_init_terrain_level = None
        g = self.scene.terrain.terrain_generator
        g.num_rows, g.num_cols, g.curriculum = 5, 5, False
        self.commands.base_velocity.ranges.lin_vel_x = (1.0, 1.0)
        self.commands.base_velocity.ranges.lin_vel_y = (0.0, 0.0)
        self.commands.base_velocity.ranges.ang_vel_z = (-1.0, 1.0)
        self.commands.base_velocity.ranges.heading = (0.0, 0.0)
        self.observations.policy.enable_corruption = False


def c5_cfg(num_envs: int = 8192) -> H12RoughEnvCfg:
    """BASELINE config C5: the rough task with CaT's startup randomisation (cat_env_cfg.py:231-249):
    sole friction U(0.1, 1.25) in 64 buckets, torso mass + U(0, 6) kg, 8192 envs."""
    c = H12RoughEnvCfg()
    c.scene.num_envs = num_envs
    c.events.physics_material = MaterialEventCfg((0.1, 1.25), (0.1, 1.25), 64)
    c.events.add_base_mass = MassEventCfg(".*torso_link", (0.0, 6.0), "add")
    return c


@dataclass
class H12RslEnvCfg(H12FlatEnvCfg):
    """Isaac-Velocity-Rsl-H12_12dof-v0 (H12_12dof_EnvCfg, rsl_env_cfg.py:504-540): IdealPD actuators (no
    delay), action scale 0.25, deadzone velocity commands resampled every U(5, 8) s, 270-float observation
    (history 6, ang_vel x 0.25, joint_vel x 0.05), sole friction U(0.1, 1.25) in 64 buckets, pushes every
    U(5, 8) s, the 16-term reward table and its modify_reward_weight curriculum.  The shipped deploy
    env.yamls (scripts/deploy/policies/*) are this task's."""

    def __post_init__(self):
        MAX_CURRICULUM_ITERATIONS = 5000
        self.sim.static_friction = self.sim.dynamic_friction = 1.0   # sim.physics_material = ground (1.0 / 1.0)
        for g in self.robot.actuators.values():                      # H12_12DOF_IDEAL (h12.py:117-196)
            g.min_delay = g.max_delay = 0
        self.actions.joint_pos.scale = 0.25                          # rsl_env_cfg.py:124
        self.commands.base_velocity = UniformVelocityCommandWithDeadzoneCfg(
            resampling_time_range=(5.0, 8.0), rel_standing_envs=0.02, rel_heading_envs=1.0, heading_command=False,
            heading_control_stiffness=1.0, ranges=Ranges((-1.0, 1.0), (-1.0, 1.0), (-1.0, 1.0)),
            velocity_deadzone=0.0)                                   # rsl_env_cfg.py:83-100
        po = self.observations.policy
        po.history_length = 6                                        # rsl_env_cfg.py:199
        po.scales = {"base_ang_vel": 0.25, "joint_vel": 0.05}        # rsl_env_cfg.py:142, 192
        self.events.physics_material = MaterialEventCfg((0.1, 1.25), (0.1, 1.25), 64)   # :213-223
        self.events.push_robot = PushEventCfg((5.0, 8.0), {"x": (-1.0, 1.0), "y": (-1.0, 1.0)})  # :262-273
        self.rewards = RewardsCfg(_rsl_rewards())
        n = 24 * MAX_CURRICULUM_ITERATIONS                           # rsl_env_cfg.py:448-501
        self.curriculum.reward_weights = [
            RewardWeightTerm(k, w, n) for k, w in (
                ("flat_orientation", -1.0), ("joint_torques_l2", -1.0e-5), ("joint_vel_l2", -1.0e-3),
                ("dof_acc_l2", -1.0e-7), ("joint_deviation_hip", -0.2), ("joint_deviation_ankle", -0.2),
                ("joint_pos_limits_ankle", -0.2), ("joint_pos_limits_hip", -0.2), ("contact_forces", -1.0e-3),
                ("feet_air_time", 0.75), ("feet_slide", -0.25), ("base_height_l2", -0.2))]


@dataclass
class H12RslEnvCfg_PLAY(H12RslEnvCfg):
    """rsl_env_cfg.py:543-563: 100 envs, no pushes / material randomisation, no noise, vx 0.5."""

    def __post_init__(self):
        super().__post_init__()
        self.scene.num_envs = 100
        self.events.push_robot = None
        self.events.physics_material = None
        self.observations.policy.enable_corruption = False
        r = self.commands.base_velocity.ranges
        r.lin_vel_x, r.lin_vel_y, r.ang_vel_z = (0.5, 0.5), (0.0, 0.0), (0.0, 0.0)


@dataclass
class H12CaTEnvCfg(H12FlatEnvCfg):
    """Isaac-Velocity-CaT-Flat-H12_12dof-v0 (H12_12dof_EnvCfg, cat_env_cfg.py:528-565): Constraints as
    Terminations on the delayed-PD robot -- deadzone commands (0.2), 270-float observation (history 6,
    scales), friction + torso-mass randomisation, pushes, a 7-term reward and the 10 constraints whose
    termination probability scales the reward and is returned as dones (CaTEnv.step, cat_env.py:95-193)."""

    def __post_init__(self):
        MAX_CURRICULUM_ITERATIONS = 5000
        self.sim.static_friction = self.sim.dynamic_friction = 1.0
        self.actions.joint_pos.scale = 0.25                                   # cat_env_cfg.py:141
        self.commands.base_velocity = UniformVelocityCommandWithDeadzoneCfg(
            resampling_time_range=(5.0, 8.0), rel_standing_envs=0.02, rel_heading_envs=1.0, heading_command=False,
            heading_control_stiffness=1.0, ranges=Ranges((-1.0, 1.0), (-1.0, 1.0), (-1.0, 1.0)),
            velocity_deadzone=0.2)                                            # :99-116
        po = self.observations.policy
        po.history_length = 6                                                 # :216
        po.scales = {"base_ang_vel": 0.25, "joint_vel": 0.05}                 # :159, 188
        self.events.physics_material = MaterialEventCfg((0.1, 1.25), (0.1, 1.25), 64)   # :231-240
        self.events.add_base_mass = MassEventCfg(".*torso_link", (0.0, 6.0), "add")     # :242-251
        self.events.push_robot = PushEventCfg((5.0, 8.0), {"x": (-1.0, 1.0), "y": (-1.0, 1.0)})  # :288-293
        T = RewTerm
        self.rewards = RewardsCfg({                                           # :300-331
            "track_lin_vel_xy_exp": T(1.0, {"command_name": "base_velocity", "std": math.sqrt(0.25)},
                                      "track_lin_vel_xy_exp"),
            "track_ang_vel_z_exp": T(0.5, {"command_name": "base_velocity", "std": math.sqrt(0.25)},
                                     "track_ang_vel_z_exp"),
            "dof_torques_l2": T(-1.0e-5, {}, "joint_torques_l2"),
            "joint_acc_l2": T(-2.5e-7, {}, "joint_acc_l2"),
            "joint_vel_l2": T(-1.0e-3, {}, "joint_vel_l2"),
            "action_rate_l2": T(-0.01, {}, "action_rate_l2"),
            "joint_deviation_l1": T(-0.1, {}, ("joint_deviation_l1:hip", "joint_deviation_l1:ankle")),
        })
        self.constraints = ConstraintsCfg()
        n = 24 * MAX_CURRICULUM_ITERATIONS                                    # :466-520
        self.curriculum.constraint_p = [ConstraintPTerm(k, n, 0.25) for k in (
            "joint_position_limits", "joint_velocity_limits", "joint_torque_limits", "foot_contact_force", "no_move",
            "base_orientation", "base_height", "foot_contact", "foot_clearance")]


@dataclass
class H12CaTEnvCfg_PLAY(H12CaTEnvCfg):
    """cat_env_cfg.py:568-583: 100 envs, zero commands."""

    def __post_init__(self):
        super().__post_init__()
        self.scene.num_envs = 100
        r = self.commands.base_velocity.ranges
        r.lin_vel_x, r.lin_vel_y, r.ang_vel_z = (0.0, 0.0), (0.0, 0.0), (0.0, 0.0)


def mujoco_cfg(**kw) -> H12FlatEnvCfg:
    """sim2sim semantics (scripts/deploy/config.yaml:7, policies/demo_rsl/env.yaml): dt 1 ms x 20,
    PD every physics step, no delay, MJCF clamps, q_ref = q0 + 0.25 a."""
    c = H12FlatEnvCfg(mode=MODE_MUJOCO, decimation=20)
    c.sim = replace(c.sim, dt=0.001, inner_steps=1, implicit_penalty=False)
    c.actions.joint_pos.scale = 0.25
    for k, v in kw.items():
        setattr(c, k, v)
    return c
