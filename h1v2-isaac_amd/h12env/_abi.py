"""ctypes mirror of include/h12env.h (the C-ABI of libh12env.so).

Kept field-for-field identical to the header; tests/test_abi.py checks struct sizes against
the library's own sizeof via h12env_state_bytes / h12env_config_default round-trips.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

NJ = 12
NHIST = 10
OBS_FRAME = 45
NOBS = OBS_FRAME * NHIST
NFOOT_PTS = 4
NREW = 20        # reward terms the kernel implements (REWARD_FUNCS)
NREW_FLAT = 12   # terms 0-11: the Flat / Rough tables
NCSTR = 10       # CaT constraint terms (CONSTRAINT_TERMS)
NCSTR_COLS = 56
NLOG = 46        # log accumulator: NREW episode sums, count, time-out count, base-contact count, spare,
                 # then per constraint term the summed violation rates (10) and mean probabilities (10),
                 # then the summed command metrics error_vel_xy, error_vel_yaw (LOG_METRIC)
LOG_METRIC = 44
ABI_VERSION = 9

MODE_ISAACLAB = 0
MODE_MUJOCO = 1
TASK_FLAT = 0
TASK_ROUGH = 1
ROUGH_FRAME = 48
SCAN_NX, SCAN_NY = 17, 11
NSCAN = SCAN_NX * SCAN_NY
NOBS_ROUGH = ROUGH_FRAME + NSCAN

# state field offsets (H12_F_* / H12_I_*)
F = dict(POS=(0, 3), QUAT=(3, 4), VLIN=(7, 3), WANG=(10, 3), Q=(13, 12), QD=(25, 12), ACT=(37, 12),
         ACT_PREV=(49, 12), CMD=(61, 3), HEADING=(64, 1), CMD_TIME=(65, 1), AIR=(66, 2), CONTACT=(68, 2),
         LAST_AIR=(70, 2), LAST_CONTACT=(72, 2), EPSUM=(74, 12), ANCHOR=(86, 16), ORIGIN=(102, 3), MU=(105, 4),
         DMASS=(109, 1), EPSUM2=(110, 8), PUSH_TIME=(118, 1), CSTR_SUM=(119, 10), CSTR_P=(129, 10),
         SWING_H=(139, 2), METRIC=(141, 2))
NF_FLOAT = 143
I = dict(EPLEN=(0, 1), PACK=(1, 1), TERRAIN=(2, 1))
NF_INT = 3

# the Flat task's reward term names, in RewardManager order (kernel ids 0-11)
REWARD_TERMS = [
    "track_lin_vel_xy_exp", "track_ang_vel_z_exp", "ang_vel_xy_l2", "dof_torques_l2", "dof_acc_l2",
    "action_rate_l2", "feet_air_time", "flat_orientation_l2", "dof_pos_limits", "termination_penalty",
    "feet_slide", "joint_deviation_hip",
]
# kernel reward ids (H12_R_*): the isaaclab mdp function each computes, with its joint / frame variant
REWARD_FUNCS = [
    "track_lin_vel_xy_yaw_frame_exp", "track_ang_vel_z_world_exp", "ang_vel_xy_l2", "joint_torques_l2",
    "joint_acc_l2", "action_rate_l2", "feet_air_time_positive_biped", "flat_orientation_l2",
    "joint_pos_limits:ankle", "is_terminated", "feet_slide", "joint_deviation_l1:hip",
    "track_lin_vel_xy_exp", "track_ang_vel_z_exp", "base_height_l2", "joint_vel_l2", "joint_deviation_l1:ankle",
    "joint_pos_limits:hip", "contact_forces", "lin_vel_z_l2",
]
assert len(REWARD_FUNCS) == NREW
# CaT constraint terms (H12_C_*), ConstraintsCfg order of cat_env_cfg.py:336-427
CONSTRAINT_TERMS = ["contact", "joint_position_limits", "joint_velocity_limits", "joint_torque_limits",
                    "foot_contact_force", "no_move", "base_orientation", "base_height", "foot_contact",
                    "foot_clearance"]
assert len(CONSTRAINT_TERMS) == NCSTR

f32 = C.c_float
i32 = C.c_int32


class H12Model(C.Structure):
    _fields_ = [
        ("version", i32),
        ("parent", i32 * NJ),
        ("axis", i32 * NJ),
        ("joint_pos", (f32 * 3) * NJ),
        ("link_mass", f32 * NJ),
        ("link_com", (f32 * 3) * NJ),
        ("link_inertia", (f32 * 6) * NJ),
        ("base_mass", f32),
        ("base_com", f32 * 3),
        ("base_inertia", f32 * 6),
        ("q_lower", f32 * NJ),
        ("q_upper", f32 * NJ),
        ("armature", f32 * NJ),
        ("damping", f32 * NJ),
        ("frictionloss", f32 * NJ),
        ("mj_frc_limit", f32 * NJ),
        ("q_default", f32 * NJ),
        ("root_height", f32),
        ("foot_pts", (f32 * 3) * NFOOT_PTS),
        ("foot_radius", f32),
        ("knee_p0", f32 * 3),
        ("knee_p1", f32 * 3),
        ("knee_radius", f32),
        ("torso_center", f32 * 3),
        ("torso_half", f32 * 3),
        ("gravity", f32),
        ("torso_com", f32 * 3),
        ("foot_rods", f32 * 3 * 2 * 4),
        ("root_com", f32 * 3),
    ]


class H12Config(C.Structure):
    _fields_ = [
        ("abi_version", i32),
        ("mode", i32),
        ("physics_dt", f32),
        ("decimation", i32),
        ("inner_steps", i32),
        ("max_episode_length", i32),
        ("action_scale", f32),
        ("kp", f32 * NJ),
        ("kd", f32 * NJ),
        ("effort_limit", f32 * NJ),
        ("delay_group", i32 * NJ),
        ("min_delay", i32),
        ("max_delay", i32),
        ("fix_base", i32),
        ("use_frictionloss", i32),
        ("contact_k", f32),
        ("contact_c", f32),
        ("mu_static", f32),
        ("mu_dynamic", f32),
        ("friction_k", f32),
        ("friction_c", f32),
        ("limit_k", f32),
        ("limit_c", f32),
        ("contact_threshold", f32),
        ("cmd_resample_time", f32),
        ("cmd_lin_x", f32 * 2),
        ("cmd_lin_y", f32 * 2),
        ("cmd_ang_z", f32 * 2),
        ("cmd_heading", f32 * 2),
        ("rel_standing_envs", f32),
        ("rel_heading_envs", f32),
        ("heading_stiffness", f32),
        ("reset_x", f32 * 2),
        ("reset_y", f32 * 2),
        ("reset_yaw", f32 * 2),
        ("enable_corruption", i32),
        ("noise_ang_vel", f32),
        ("noise_gravity", f32),
        ("noise_joint_pos", f32),
        ("noise_joint_vel", f32),
        ("rew_w", f32 * NREW),
        ("track_std", f32),
        ("air_time_threshold", f32),
        ("soft_limit_factor", f32),
        ("illegal_contact_knees", i32),
        ("illegal_contact_torso", i32),
        ("seed", C.c_uint64),
        ("task", i32),
        ("terrain", i32),
        ("terrain_curriculum", i32),
        ("per_env_friction", i32),
        ("per_env_mass", i32),
        ("noise_lin_vel", f32),
        ("noise_height_scan", f32),
        ("scan_offset", f32),
        ("scan_clip", f32),
        ("scan_resolution", f32),
        ("terrain_size", f32),
        ("cmd_resample_time_max", f32),
        ("cmd_deadzone", i32),
        ("velocity_deadzone", f32),
        ("ang_flip_prob", f32),
        ("push_enable", i32),
        ("push_interval", f32 * 2),
        ("push_vel_x", f32 * 2),
        ("push_vel_y", f32 * 2),
        ("history_length", i32),
        ("obs_scale", f32 * 6),
        ("base_height_target", f32),
        ("contact_force_threshold", f32),
        ("cat_enable", i32),
        ("cstr_mask", C.c_uint32),
        ("cstr_max_p", f32 * NCSTR),
        ("cat_tau", f32),
        ("cat_min_p", f32),
        ("cstr_joint_vel_limit", f32 * NJ),
        ("cstr_joint_effort_limit", f32 * NJ),
        ("cstr_foot_force_limit", f32),
        ("cstr_nomove_deadzone", f32),
        ("cstr_nomove_vel", f32),
        ("cstr_orient_limit", f32),
        ("cstr_height", f32),
        ("cstr_height_std", f32),
        ("cstr_clearance_min", f32),
        ("cstr_clearance_deadzone", f32),
        ("implicit_penalty", i32),
        ("max_joint_vel", f32 * NJ),
        ("max_joint_vel_damping", f32),
        ("self_collision", i32),
        ("self_k", f32),
        ("self_c", f32),
        ("self_ct", f32),
        ("self_mu", f32),
        ("limit_projection", f32),
        ("max_depenetration_velocity", f32),
    ]


class H12StepOut(C.Structure):
    _fields_ = [
        ("obs", C.c_void_p),
        ("rew", C.c_void_p),
        ("terminated", C.c_void_p),
        ("truncated", C.c_void_p),
        ("log_acc", C.c_void_p),
        ("applied_torque", C.c_void_p),
        ("foot_force", C.c_void_p),
        ("cstr_prob", C.c_void_p),
        ("frame_out", C.c_void_p),
    ]


PKG_DIR = Path(__file__).resolve().parent
LIB_PATH = PKG_DIR / "libh12env.so"

_lib = None


class H12EnvError(RuntimeError):
    pass


def load_library(path: str | os.PathLike | None = None):
    """Load libh12env.so (built in-tree by __graft_entry__.build()).  Fails loudly: there is no
    CPU fallback for the product path."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = Path(path) if path is not None else Path(os.environ.get("H12ENV_LIB", LIB_PATH))
    if not p.exists():
        raise H12EnvError(f"HIP extension {p} is missing; build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    # torch's bundled libamdhip64.so.7 must be the one the library binds to (same soname):
    # importing torch first guarantees it is already resident in the process.
    try:
        import torch  # noqa: F401
    except Exception:  # pragma: no cover - torch is always present in this image
        pass
    lib = C.CDLL(str(p), mode=C.RTLD_GLOBAL)
    vp = C.c_void_p
    lib.h12env_config_default.argtypes = [C.POINTER(H12Config)]
    lib.h12env_config_default.restype = C.c_int
    lib.h12env_state_bytes.argtypes = [C.c_int]
    lib.h12env_state_bytes.restype = C.c_size_t
    lib.h12env_create.argtypes = [C.POINTER(H12Model), C.POINTER(H12Config), C.c_int, C.c_int64, C.c_int, vp,
                                  C.POINTER(vp)]
    lib.h12env_create.restype = C.c_int
    lib.h12env_destroy.argtypes = [vp]
    lib.h12env_destroy.restype = None
    lib.h12env_reset.argtypes = [vp, vp, vp, vp]
    lib.h12env_reset.restype = C.c_int
    lib.h12env_step.argtypes = [vp, vp, vp, C.POINTER(H12StepOut), C.c_int64, vp]
    lib.h12env_step.restype = C.c_int
    lib.h12env_flush_log.argtypes = [vp, vp]
    lib.h12env_flush_log.restype = C.c_int
    if hasattr(lib, "h12env_step_lds"):  # round 6 (a round-5 library, loaded as an A/B baseline, lacks these)
        lib.h12env_step_lds.argtypes = [vp, C.POINTER(C.c_size_t), C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)]
        lib.h12env_step_lds.restype = C.c_int
        lib.h12env_check.argtypes = [vp, vp]
        lib.h12env_check.restype = C.c_int
    lib.h12env_obs_fused.argtypes = [vp]
    lib.h12env_obs_fused.restype = C.c_int
    if hasattr(lib, "h12env_cat_inline"):  # (a round-5 library, loaded as an A/B baseline, lacks it)
        lib.h12env_cat_inline.argtypes = [vp]
        lib.h12env_cat_inline.restype = C.c_int
    lib.h12env_observe.argtypes = [vp, vp, vp, vp, vp]
    lib.h12env_observe.restype = C.c_int
    lib.h12env_set_terrain.argtypes = [vp, vp, C.c_int, C.c_int, C.c_float, C.c_float, C.c_float, vp, C.c_int, C.c_int]
    lib.h12env_set_terrain.restype = C.c_int
    lib.h12env_step_physics.argtypes = [vp, vp, C.c_int, vp]
    lib.h12env_step_physics.restype = C.c_int
    lib.h12env_rollout_layout.argtypes = [C.c_int, C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)]
    lib.h12env_rollout_layout.restype = C.c_int
    lib.h12env_rollout_decode.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, vp, vp, vp]
    lib.h12env_rollout_decode.restype = C.c_int
    lib.h12env_fence_create.argtypes = [C.c_int, C.c_int, C.POINTER(vp)]
    lib.h12env_fence_create.restype = C.c_int
    lib.h12env_fence_destroy.argtypes = [vp]
    lib.h12env_fence_destroy.restype = None
    lib.h12env_fence_signal.argtypes = [vp, C.c_int, C.c_uint64, vp]
    lib.h12env_fence_signal.restype = C.c_int
    lib.h12env_fence_wait.argtypes = [vp, C.c_int, C.c_uint64, vp]
    lib.h12env_fence_wait.restype = C.c_int
    lib.h12env_field_ptr.argtypes = [vp, C.c_int, C.c_int]
    lib.h12env_field_ptr.restype = vp
    lib.h12env_eval_terms.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp]
    lib.h12env_eval_terms.restype = C.c_int
    lib.h12env_eval_self_contacts.argtypes = [vp, vp, vp]
    lib.h12env_eval_self_contacts.restype = C.c_int
    lib.h12env_num_envs.argtypes = [vp]
    lib.h12env_num_envs.restype = C.c_int
    lib.h12env_obs_dim.argtypes = [vp]
    lib.h12env_obs_dim.restype = C.c_int
    lib.h12env_set_reward_weights.argtypes = [vp, C.POINTER(C.c_float), C.c_int]
    lib.h12env_set_reward_weights.restype = C.c_int
    lib.h12env_set_constraint_max_p.argtypes = [vp, C.POINTER(C.c_float), C.c_int]
    lib.h12env_set_constraint_max_p.restype = C.c_int
    lib.h12env_step_cost.argtypes = [vp, C.POINTER(C.c_double), C.POINTER(C.c_double)]
    lib.h12env_step_cost.restype = C.c_int
    lib.h12env_kernel_cost.argtypes = [vp, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double)]
    lib.h12env_kernel_cost.restype = C.c_int
    lib.h12env_set_kernel_timing.argtypes = [vp, C.c_int]
    lib.h12env_set_kernel_timing.restype = C.c_int
    lib.h12env_kernel_times.argtypes = [vp, C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_int)]
    lib.h12env_kernel_times.restype = C.c_int
    lib.h12env_last_error.argtypes = []
    lib.h12env_last_error.restype = C.c_char_p
    lib.h12env_abi_version.argtypes = []
    lib.h12env_abi_version.restype = C.c_int
    lib.h12env_sizeof_struct.argtypes = [C.c_int]
    lib.h12env_sizeof_struct.restype = C.c_size_t
    for i, st in enumerate((H12Model, H12Config, H12StepOut)):
        if lib.h12env_sizeof_struct(i) != C.sizeof(st):
            raise H12EnvError(f"{st.__name__}: ctypes size {C.sizeof(st)} != C size {lib.h12env_sizeof_struct(i)}")
    if lib.h12env_abi_version() != ABI_VERSION:
        raise H12EnvError(f"libh12env ABI {lib.h12env_abi_version()} != python mirror {ABI_VERSION}")
    if path is None:
        _lib = lib
    return lib


def check(lib, rc: int, what: str):
    if rc != 0:
        msg = lib.h12env_last_error()
        raise H12EnvError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")


EXPORTED_SYMBOLS = [
    "h12env_config_default", "h12env_state_bytes", "h12env_create", "h12env_destroy", "h12env_reset",
    "h12env_step", "h12env_flush_log", "h12env_obs_fused", "h12env_cat_inline", "h12env_observe", "h12env_step_physics", "h12env_field_ptr", "h12env_num_envs", "h12env_step_cost",
    "h12env_last_error", "h12env_abi_version", "h12env_sizeof_struct", "h12env_kernel_cost",
    "h12env_set_kernel_timing", "h12env_kernel_times", "h12env_set_terrain", "h12env_obs_dim",
    "h12env_set_reward_weights", "h12env_set_constraint_max_p", "h12env_eval_terms", "h12env_eval_self_contacts",
    "h12env_rollout_layout", "h12env_rollout_decode", "h12env_fence_create", "h12env_fence_destroy",
    "h12env_fence_signal", "h12env_fence_wait", "h12env_step_lds", "h12env_check",
]
