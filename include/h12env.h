/*
 * h12env.h — C-ABI of the MI355X-native H1-2 12-DoF velocity-tracking environment
 * (the hot path of `Isaac-Velocity-Flat-H12_12dof-v0`, reference repo
 * olivier-stasse/h1v2-Isaac; paths below are relative to that repository).
 *
 * What each entry point replaces on the reference side (the reference reaches all of
 * this through IsaacLab 2.1 / PhysX; the in-repo mirrors are cited):
 *
 *   h12env_create      ManagerBasedRLEnv.__init__ -> load_managers + scene cloning
 *                      (packages/biped_tasks/biped_tasks/utils/cat/cat_env.py:31-93; task cfg
 *                      .../velocity/config/h12_12dof/flat_env_cfg.py:13-48, rough_env_cfg.py:65-125;
 *                      robot cfg packages/biped_assets/biped_assets/robots/h12.py:18-114)
 *   h12env_reset       ManagerBasedRLEnv._reset_idx + reset events + ObservationManager.compute
 *                      (cat_env.py:195-248; rough_env_cfg.py:77-92; observation_manager.py:271-355)
 *   h12env_step        ManagerBasedRLEnv.step (cat_env.py:95-193): action processing, 4 x (delayed PD
 *                      actuator -> PhysX step -> sensor update), terminations, rewards, resets,
 *                      commands, observations with 10-frame history (circular_buffer.py:79-170)
 *   h12env_step_physics  parity hook: the MuJoCo sim2sim substep loop
 *                      (packages/biped_deploy/biped_deploy/robots/h12_mujoco.py:55-67,
 *                      packages/biped_deploy/biped_deploy/simulator/sim_mujoco.py:102-121)
 *
 * Conventions
 *   - Every function returns 0 on success or a negative H12_E* code; the message of the last
 *     failure on the calling thread is h12env_last_error().
 *   - All array arguments are DEVICE pointers on the handle's device unless named *_host.
 *   - Calls are stream-ordered on the hipStream_t passed in (NULL = default stream) and never
 *     synchronise the host.  One handle per device; calls on one handle are not re-entrant.
 *   - Persistent per-env state lives in ONE device workspace of h12env_state_bytes(n) bytes,
 *     field-major structure-of-arrays (field f of env i at offset f*n + i).  The caller may
 *     supply the workspace (e.g. a torch uint8 tensor) so that it can view fields in place
 *     (episode_length_buf is writable from Python, as rsl_rl's OnPolicyRunner requires).
 */
#ifndef H12ENV_H
#define H12ENV_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define H12ENV_ABI_VERSION 9
#define H12_NJ 12          /* actuated joints (L leg 6, R leg 6; MJCF depth-first order) */
#define H12_NHIST 10       /* observation history length of the Flat task (flat_env_cfg.py:26); max */
#define H12_OBS_FRAME 45   /* ang_vel 3, gravity 3, command 3, q-q0 12, qd 12, action 12 */
#define H12_NOBS (H12_OBS_FRAME * H12_NHIST) /* 450 */
#define H12_NFOOT_PTS 4    /* sole contact spheres per foot (URDF rods, h12_12dof.urdf:168-191) */
#define H12_NREW 20        /* reward terms the kernel implements (union of the Flat / Rough / Rsl tables) */
#define H12_NREW_FLAT 12   /* terms 0-11: the Flat / Rough tables */
#define H12_NCSTR 10       /* CaT constraint terms (cat_env_cfg.py:336-427, ConstraintsCfg order) */
#define H12_NCSTR_COLS 56  /* their columns: 1 + 12 + 12 + 12 + 2 + 12 + 1 + 1 + 1 + 2 */
#define H12_NLOG 46        /* log accumulator: 20 episode reward sums, reset count, time-out / base-contact counts,
                              spare, then per constraint term the sums over reset envs of the episode's
                              violation rate (10) and mean probability (10), then (ABI 7) the sums over reset
                              envs of the command metrics error_vel_xy, error_vel_yaw (H12_LOG_METRIC) */
#define H12_LOG_METRIC 44  /* UniformVelocityCommand._update_metrics accumulators, logged by CommandTerm.reset */
/* Rough task (Isaac-Velocity-Rough-H12_12dof-v0, rough_env_cfg.py:65-125): no history, base_lin_vel
 * first, height scan last (velocity_env_cfg.py:118-137) */
#define H12_ROUGH_FRAME 48 /* lin_vel 3, ang_vel 3, gravity 3, command 3, q-q0 12, qd 12, action 12 */
#define H12_SCAN_NX 17     /* GridPatternCfg(resolution 0.1, size (1.6, 1.0)), velocity_env_cfg.py:60-66 */
#define H12_SCAN_NY 11
#define H12_NSCAN (H12_SCAN_NX * H12_SCAN_NY) /* 187 */
#define H12_NOBS_ROUGH (H12_ROUGH_FRAME + H12_NSCAN) /* 235 */

/* max-joint-velocity damper: over the first H12_VLIM_RAMP rad/s of excess e the torque is -c e^2 / (2 ramp)
 * (its slope, and with it the implicit joint inertia h dtau/dqd, grows from 0 to c), beyond it -c (e - ramp/2),
 * so the dynamics stay continuous where a joint crosses its limit */
#define H12_VLIM_RAMP 1.0f

/* error codes */
#define H12_OK 0
#define H12_E_ARG (-1)
#define H12_E_HIP (-2)
#define H12_E_STATE (-3)
#define H12_E_ALLOC (-4)

/* simulation modes */
#define H12_MODE_ISAACLAB 0 /* explicit PD once per physics step with per-group delay + effort clip */
#define H12_MODE_MUJOCO 1   /* PD every substep, no delay, MJCF actuatorfrcrange clamp (sim2sim) */

/* tasks (observation layout) */
#define H12_TASK_FLAT 0     /* 45 x history_length floats, term-major history (flat_env_cfg.py:25-27: 450) */
#define H12_TASK_ROUGH 1    /* 235 floats: 48-float frame + 187-ray height scan, no history */
/* (the Rsl task, rsl_env_cfg.py, is H12_TASK_FLAT with history_length 6 and per-term obs_scale) */

/* reward terms the kernel implements; h12env_config.rew_w[term] weights them (0 = off).  Terms 0-11 are
 * the Flat table in its RewardManager order; 12-19 complete the Rsl table (rsl_env_cfg.py:279-407).
 * The host maps each cfg term (name, mdp function, joint set) onto one of these ids. */
enum {
  H12_R_TRACK_LIN_VEL_XY = 0, /* track_lin_vel_xy_yaw_frame_exp, std 0.5   rough_env_cfg.py:24-28 */
  H12_R_TRACK_ANG_VEL_Z,      /* track_ang_vel_z_world_exp, std 0.5       rough_env_cfg.py:29-33 */
  H12_R_ANG_VEL_XY_L2,        /* ang_vel_xy_l2                            velocity_env_cfg.py:237 */
  H12_R_DOF_TORQUES_L2,       /* joint_torques_l2                         flat_env_cfg.py:40-44 */
  H12_R_DOF_ACC_L2,           /* joint_acc_l2                             flat_env_cfg.py:37 */
  H12_R_ACTION_RATE_L2,       /* action_rate_l2                           flat_env_cfg.py:36 */
  H12_R_FEET_AIR_TIME,        /* feet_air_time_positive_biped, thr 0.4    rough_env_cfg.py:34-42 */
  H12_R_FLAT_ORIENTATION_L2,  /* flat_orientation_l2                      rough_env_cfg.py:113 */
  H12_R_DOF_POS_LIMITS,       /* joint_pos_limits (ankles)                rough_env_cfg.py:52-56 */
  H12_R_TERMINATION,          /* is_terminated                            rough_env_cfg.py:22 */
  H12_R_FEET_SLIDE,           /* feet_slide                               rough_env_cfg.py:43-50 */
  H12_R_JOINT_DEV_HIP,        /* joint_deviation_l1 (hip yaw/roll)        rough_env_cfg.py:58-62 */
  H12_R_TRACK_LIN_VEL_XY_BASE,/* track_lin_vel_xy_exp (base frame)        rsl_env_cfg.py:283-287 */
  H12_R_TRACK_ANG_VEL_Z_BASE, /* track_ang_vel_z_exp (base frame)         rsl_env_cfg.py:288-292 */
  H12_R_BASE_HEIGHT_L2,       /* base_height_l2, (z - target)^2           rsl_env_cfg.py:322-328 */
  H12_R_JOINT_VEL_L2,         /* joint_vel_l2 (all joints)                rsl_env_cfg.py:335-338 */
  H12_R_JOINT_DEV_ANKLE,      /* joint_deviation_l1 (ankle pitch/roll)    rsl_env_cfg.py:358-372 */
  H12_R_DOF_POS_LIMITS_HIP,   /* joint_pos_limits (hip yaw/roll)          rsl_env_cfg.py:380-386 */
  H12_R_CONTACT_FORCES,       /* contact_forces: sum_f max(max_h|F|-thr,0) rsl_env_cfg.py:395-405 */
  H12_R_LIN_VEL_Z_L2          /* lin_vel_z_l2 (v_b,z^2)                   velocity_env_cfg.py:236 */
};

/* CaT constraint terms (Constraints-as-Terminations, T/utils/cat/constraints.py; cfg cat_env_cfg.py:336-427) */
enum {
  H12_C_CONTACT = 0,          /* contact: any illegal body in contact (max_p 1.0)            1 column */
  H12_C_JOINT_POS_LIMITS,     /* max(soft_lo - q, q - soft_hi)                              12 columns */
  H12_C_JOINT_VEL_LIMITS,     /* |qd| - joint_vel_limits                                    12 columns */
  H12_C_JOINT_TORQUE_LIMITS,  /* |applied_torque| - joint_effort_limits                     12 columns */
  H12_C_FOOT_CONTACT_FORCE,   /* max_h |F_foot| - 750                                        2 columns */
  H12_C_NO_MOVE,              /* |qd| - 6 while all |cmd| < deadzone (rows remapped, see DESIGN) 12 columns */
  H12_C_BASE_ORIENTATION,     /* |g_b,xy| - 0.1                                              1 column */
  H12_C_BASE_HEIGHT,          /* z outside height +- std                                     1 column */
  H12_C_FOOT_CONTACT,         /* number of feet in contact not in {1, 2}                     1 column */
  H12_C_FOOT_CLEARANCE        /* (min_height - swing max height) at touchdown, command active 2 columns */
};

/* Model constants (filled from h12env/assets/h12_12dof_model.json, generated from the MJCF). */
typedef struct h12env_model {
  int32_t version;
  int32_t parent[H12_NJ];        /* -1 = floating base */
  int32_t axis[H12_NJ];          /* 0=x 1=y 2=z (all H1-2 leg axes are coordinate axes) */
  float joint_pos[H12_NJ][3];    /* joint frame origin in parent frame at q=0 (no rotation) */
  float link_mass[H12_NJ];
  float link_com[H12_NJ][3];
  float link_inertia[H12_NJ][6]; /* about COM, link frame: xx yy zz xy xz yz */
  float base_mass;
  float base_com[3];
  float base_inertia[6];         /* pelvis + 39 welded upper-body bodies, about composite COM */
  float q_lower[H12_NJ], q_upper[H12_NJ];
  float armature[H12_NJ], damping[H12_NJ], frictionloss[H12_NJ];
  float mj_frc_limit[H12_NJ];    /* MJCF actuatorfrcrange (MuJoCo mode clamp) */
  float q_default[H12_NJ];       /* keyframe / init_state joint_pos (h12.py:39-53) */
  float root_height;             /* init_state pos z = 1.05 */
  float foot_pts[H12_NFOOT_PTS][3]; /* sole sphere centres in ankle-roll frame */
  float foot_radius;
  float knee_p0[3], knee_p1[3];  /* knee capsule segment in knee frame */
  float knee_radius;
  float torso_center[3], torso_half[3]; /* torso collision box in base frame */
  float gravity;                 /* 9.81 */
  float torso_com[3];            /* torso_link COM in base frame (h12_12dof.xml:144): where the
                                    randomize_rigid_body_mass event adds mass (cat_env_cfg.py:240-249) */
  /* ABI 6: the four sole rods (URDF cylinders r = foot_radius, h12_12dof.urdf:168-191) as segments in the
   * ankle-roll frame: heel, toe, two side rods (self-collision capsules) */
  float foot_rods[4][2][3];
  /* ABI 7: COM of the pelvis rigid body alone (base frame, h12_12dof.xml pelvis <inertial>): IsaacLab's
   * root_lin_vel_w is the root body's COM velocity, and the USD keeps torso_link / arms as separate bodies */
  float root_com[3];
} h12env_model;

/* Task / simulation configuration. h12env_config_default() fills the Flat-H12_12dof values. */
typedef struct h12env_config {
  int32_t abi_version;
  int32_t mode;                /* H12_MODE_* */
  float physics_dt;            /* 0.005 (velocity_env_cfg.py:305); MuJoCo mode: 0.001 */
  int32_t decimation;          /* 4 (velocity_env_cfg.py:302); MuJoCo mode: 20 */
  int32_t inner_steps;         /* contact/dynamics integration substeps per physics step (>=1) */
  int32_t max_episode_length;  /* ceil(20 s / step_dt) = 1000 */
  float action_scale;          /* 0.5 (velocity_env_cfg.py:111) */
  float kp[H12_NJ], kd[H12_NJ], effort_limit[H12_NJ]; /* h12.py:58-112 */
  int32_t delay_group[H12_NJ]; /* 0 legs, 1 knees, 2 feet */
  int32_t min_delay, max_delay;/* 0, 5 physics steps */
  int32_t fix_base;            /* parity hook: base welded in place (scene_12dof.xml:23-25) */
  int32_t use_frictionloss;    /* smooth MJCF frictionloss (off by default) */
  /* penalty contact + joint limits */
  float contact_k, contact_c;  /* normal spring [N/m] / damper [N s/m] */
  float mu_static, mu_dynamic; /* 0.8 / 0.6 (velocity_env_cfg.py:153-163, multiply with ground 1.0) */
  float friction_k, friction_c;/* sole stiction spring [N/m] / damper [N s/m] (anchored, Coulomb-capped) */
  float limit_k, limit_c;      /* joint-limit penalty [Nm/rad], [Nm s/rad] */
  float contact_threshold;     /* ContactSensorCfg.force_threshold = 1.0 N */
  /* commands: UniformVelocityCommandCfg (velocity_env_cfg.py:90-104, flat_env_cfg.py:46-48) */
  float cmd_resample_time;
  float cmd_lin_x[2], cmd_lin_y[2], cmd_ang_z[2], cmd_heading[2];
  float rel_standing_envs, rel_heading_envs, heading_stiffness;
  /* reset events (rough_env_cfg.py:77-92) */
  float reset_x[2], reset_y[2], reset_yaw[2];
  /* observation corruption: AdditiveUniformNoise half-widths (velocity_env_cfg.py:124-131) */
  int32_t enable_corruption;
  float noise_ang_vel, noise_gravity, noise_joint_pos, noise_joint_vel;
  /* rewards */
  float rew_w[H12_NREW];
  float track_std;             /* 0.5 */
  float air_time_threshold;    /* 0.4 */
  float soft_limit_factor;     /* 0.9 (h12.py:56) */
  int32_t illegal_contact_knees, illegal_contact_torso; /* bodies with colliders among the list */
  uint64_t seed;
  /* rough task / terrain / startup randomisation (ABI 2) */
  int32_t task;                /* H12_TASK_* */
  int32_t terrain;             /* 0 plane z = 0, 1 heightfield (h12env_set_terrain) */
  int32_t terrain_curriculum;  /* terrain_levels_vel on reset (velocity/mdp/curriculums.py:21-52) */
  int32_t per_env_friction;    /* sole friction from H12_F_MU (randomize_rigid_body_material buckets) */
  int32_t per_env_mass;        /* added torso mass from H12_F_DMASS (randomize_rigid_body_mass) */
  float noise_lin_vel;         /* 0.1 (velocity_env_cfg.py:118) */
  float noise_height_scan;     /* 0.1 (velocity_env_cfg.py:131-136) */
  float scan_offset;           /* 0.5: height = sensor z - hit z - offset (isaaclab mdp.height_scan) */
  float scan_clip;             /* 1.0 */
  float scan_resolution;       /* 0.1 m grid spacing */
  float terrain_size;          /* 8.0 m sub-terrain edge (terrains.py:12) */
  /* Rsl task (ABI 3; rsl_env_cfg.py) */
  float cmd_resample_time_max; /* resampling_time_range = (cmd_resample_time, this); Rsl (5, 8) s */
  int32_t cmd_deadzone;        /* UniformVelocityCommandWithDeadzone._update_command (utils/mdp/commands.py:41-96) */
  float velocity_deadzone;     /* |cmd_xy| < this counts as in the deadzone (Rsl 0.0) */
  float ang_flip_prob;         /* per-step probability of cmd_z *= -1 (physics_dt / episode_length_s) */
  int32_t push_enable;         /* push_by_setting_velocity interval event (rsl_env_cfg.py:262-273) */
  float push_interval[2];      /* interval_range_s (5, 8) */
  float push_vel_x[2], push_vel_y[2]; /* velocity_range x / y (-1, 1) m/s added to the root velocity */
  int32_t history_length;      /* observation history (flat layout): 10 Flat, 6 Rsl; 1..H12_NHIST */
  float obs_scale[6];          /* per-term scale after noise: ang_vel, gravity, command, q-q0, qd, action */
  float base_height_target;    /* base_height_l2 target (1.0) */
  float contact_force_threshold; /* contact_forces threshold (800 N) */
  /* CaT task (ABI 4; T/utils/cat, cat_env_cfg.py): constraint probabilities scale the reward and are
   * returned as dones (h12env_step_out.cstr_prob) */
  int32_t cat_enable;
  uint32_t cstr_mask;          /* bit t: constraint term t (H12_C_*) active */
  float cstr_max_p[H12_NCSTR]; /* per-term maximum termination probability (curriculum: h12env_set_constraint_max_p) */
  float cat_tau, cat_min_p;    /* running-max Polyak factor 0.95, minimum probability 0 (constraint_manager.py:26) */
  float cstr_joint_vel_limit[H12_NJ];    /* ArticulationData.joint_vel_limits (URDF velocity 23 / 14 / 9 rad/s) */
  float cstr_joint_effort_limit[H12_NJ]; /* ArticulationData.joint_effort_limits (explicit actuators: 1e9) */
  float cstr_foot_force_limit;  /* 750 N */
  float cstr_nomove_deadzone;   /* 0.2 */
  float cstr_nomove_vel;        /* 6.0 rad/s */
  float cstr_orient_limit;      /* 0.1 */
  float cstr_height, cstr_height_std; /* 1.0, 0.05 */
  float cstr_clearance_min;     /* 0.1 m */
  float cstr_clearance_deadzone;/* 0.2 */
  /* ABI 5: the penalty springs / dampers (ground contacts, joint limits) integrated implicitly over the
   * integration substep h: the force at the end of the substep, f(x + h v', v'), linearised in the
   * acceleration -> an added point inertia h (c + h k) at each active contact and an added joint
   * inertia h (c + h k) at each active limit in the dynamics solve */
  int32_t implicit_penalty;
  /* ABI 5: PhysX maxJointVelocity (the USD's joint velocity limits, converted from the URDF: 23 / 14 / 9 rad/s,
   * IsaacLab write_joint_velocity_limit_to_sim).  Enforced like the other penalties, through the dynamics
   * solve (so the reaction reaches the whole articulation): above the limit a joint damper
   * -max_joint_vel_damping (|qd| - max) sign(qd), integrated implicitly; 0 = no limit (MuJoCo mode) */
  float max_joint_vel[H12_NJ];
  float max_joint_vel_damping; /* [N m s / rad]; C1 ramp-in over the first H12_VLIM_RAMP of excess (see below) */
  /* ABI 6: self-collision between the two legs (ArticulationCfg enabled_self_collisions=True, h12.py:32):
   * capsules of the knee cylinders (knee_p0/p1, knee_radius) and the four sole rods of each foot (foot_rods,
   * foot_radius), every left/right pair.  Penalty law, explicit: f_n = max(0, k d - c v_n) along the
   * closest-point normal, viscous friction -c_t v_t capped at mu f_n, applied equal and opposite at the
   * midpoint of the closest points; reported into the bodies' net contact forces (ContactSensor: foot timers,
   * illegal knee contact). */
  int32_t self_collision;
  float self_k, self_c;        /* normal stiffness [N/m], damping [N s/m] */
  float self_ct, self_mu;      /* tangential damping [N s/m], Coulomb cap (0.6 x 0.6, material multiply; with
                                  per_env_friction: left x right leg H12_F_MU dynamic coefficient) */
  /* ABI 8: hard joint limits (PhysX holds the URDF ranges, A/robots/h12.py:18-35).  The stiff implicit limit spring
   * (limit_k, activated on the predicted end-of-step position) stops a joint at its range inside the solve, with
   * the reaction on the whole articulation; a joint that other forces (a foot slammed into the ground) still carry
   * further than limit_projection past its range within a step is projected back to that tolerance and its outward
   * velocity zeroed (PhysX's position-level limit correction; 0 = off, MuJoCo mode: its limits are soft) */
  float limit_projection;      /* [rad] */
  /* ABI 8: PhysX's max_depenetration_velocity (RigidBodyPropertiesCfg, A/robots/h12.py:29: 1.0 m/s): the
   * implicit ground-contact spring pushes a penetration out at most this fast -- its elastic term uses
   * min(depth, h * v) -- so a deep initial penetration is resolved over several steps instead of launching the
   * body (0 = off; explicit integration: off) */
  float max_depenetration_velocity; /* [m/s] */
} h12env_config;

/* Persistent per-env state fields (field-major SoA in the workspace). */
enum {
  H12_F_POS = 0,        /* 3  base position, env-local frame [m] */
  H12_F_QUAT = 3,       /* 4  base orientation w x y z */
  H12_F_VLIN = 7,       /* 3  base-origin linear velocity, world frame (MuJoCo qvel[0:3]) */
  H12_F_WANG = 10,      /* 3  base angular velocity, base frame (MuJoCo qvel[3:6]) */
  H12_F_Q = 13,         /* 12 joint positions */
  H12_F_QD = 25,        /* 12 joint velocities */
  H12_F_ACT = 37,       /* 12 action_manager.action  (a_t, raw) */
  H12_F_ACT_PREV = 49,  /* 12 action_manager.prev_action (a_{t-1}) */
  H12_F_CMD = 61,       /* 3  vel_command_b */
  H12_F_HEADING = 64,   /* 1  heading_target */
  H12_F_CMD_TIME = 65,  /* 1  command time_left */
  H12_F_AIR = 66,       /* 2  current_air_time (feet) */
  H12_F_CONTACT = 68,   /* 2  current_contact_time (feet) */
  H12_F_LAST_AIR = 70,  /* 2  last_air_time */
  H12_F_LAST_CONTACT = 72, /* 2 last_contact_time */
  H12_F_EPSUM = 74,     /* 12 episode reward sums */
  H12_F_ANCHOR = 86,    /* 16 sole-sphere stiction anchors: [foot][pt][x,y] world axes, relative to the env origin */
  H12_F_ORIGIN = 102,   /* 3  env origin (terrain origin of the env's level / type; 0 on the plane) */
  H12_F_MU = 105,       /* 4  static, dynamic friction of the left / right sole (per_env_friction) */
  H12_F_DMASS = 109,    /* 1  mass added at the torso COM (per_env_mass) */
  H12_F_EPSUM2 = 110,   /* 8  episode sums of reward terms 12-19 */
  H12_F_PUSH_TIME = 118,/* 1  push_robot interval time left */
  H12_F_CSTR_SUM = 119, /* 10 CaT: episode count of steps with the term violated (max prob > 0) */
  H12_F_CSTR_P = 129,   /* 10 CaT: episode sum of the term's max probability */
  H12_F_SWING_H = 139,  /* 2  CaT foot_clearance: max foot height of the current swing (left, right) */
  H12_F_METRIC = 141,   /* 2  (ABI 7) command metrics error_vel_xy, error_vel_yaw of the episode (base_velocity) */
  H12_NF_FLOAT = 143
};
enum {
  H12_I_EPLEN = 0,      /* episode_length_buf (int32) */
  H12_I_PACK = 1,       /* bits 0-8 lags (3 x 3 bits), 9-10 steps since reset (sat. 2), 11 heading env,
                           12 standing env, 13-20 sole-sphere contact flags (bit 13 + 4*foot + pt) */
  H12_I_TERRAIN = 2,    /* terrain level (bits 0-15) and terrain type / column (bits 16-31) */
  H12_NF_INT = 3
};

/* Optional per-step outputs; any pointer may be NULL. */
typedef struct h12env_step_out {
  float* obs;              /* N x h12env_obs_dim: 45 x history (flat layout) or 235 (rough) (required) */
  float* rew;              /* N       (required) */
  uint8_t* terminated;     /* N       (required) */
  uint8_t* truncated;      /* N       (required) */
  float* log_acc;          /* H12_NLOG floats, accumulated into (caller zeroes).  (ABI 9) The step's additions may
                              be deferred: they are complete, in step order, once h12env_flush_log has run on the
                              stream (later steps flush by themselves when 64 steps are pending or an accumulator
                              is reused) */
  float* applied_torque;   /* N x 12, last physics step (ArticulationData.applied_torque) */
  float* foot_force;       /* N x 2,  |net contact force| of the feet, last physics step */
  float* cstr_prob;        /* N, CaT task: the dones CaTEnv.step returns (constraint termination probability,
                              1 for envs reset this step); the reward is already scaled by 1 - p */
  float* frame_out;        /* (ABI 8) N x 45, flat layout only: the step's new observation frame exactly as it
                              enters the history (noise added, term scales applied) -- the newest slot of every
                              term of obs.  With terminated / truncated it is the rollout record of the step from
                              which h12env_rollout_decode rebuilds the observation rows bit for bit */
} h12env_step_out;

typedef struct h12env h12env;

int h12env_config_default(h12env_config* cfg);
size_t h12env_state_bytes(int n_envs);
/* device: HIP ordinal; env_offset: global id of this shard's first env (RNG keying, sharding
 * invariance); state_dev: caller workspace of h12env_state_bytes(n_envs) bytes or NULL. */
int h12env_create(const h12env_model* model, const h12env_config* cfg, int n_envs, int64_t env_offset,
                  int device, void* state_dev, h12env** out);
void h12env_destroy(h12env* h);
/* Reset the envs flagged in mask (N bytes, NULL = all) and write their first observation
 * (history filled with the first frame) into obs (N x h12env_obs_dim); other rows are left untouched. */
int h12env_reset(h12env* h, const uint8_t* mask, float* obs, void* stream);
/* One env step (decimation x physics).  obs_prev: previous obs (history source), may equal
 * out->obs.  step_index: common_step_counter after increment (>= 1). */
int h12env_step(h12env* h, const float* actions, const float* obs_prev, const h12env_step_out* out,
                int64_t step_index, void* stream);
/* (ABI 9) Complete every deferred episode-log addition of earlier h12env_step calls (one kernel on stream; nothing
 * when none is pending).  Call it before reading a step's log_acc. */
int h12env_flush_log(h12env* h, void* stream);
/* (ABI 9) 1 when h12env_step assembles the observation rows inside the env kernel (history layouts -- Flat, Rsl,
 * CaT -- with 16-byte aligned obs / obs_prev; environment variable H12_FUSE_OBS=0 at h12env_create selects the two-kernel
 * path), else 0.  Results are bit-identical either way; the kernel timing / cost pairs name different kernels. */
int h12env_obs_fused(const h12env* h);
/* (ABI 9, round 6) 1 when a CaT handle's h12env_step applies the constraint probabilities inside the env kernel (the
 * fused path, with the kernel's whole grid resident on the device; environment variable H12_CAT_INLINE=0 at
 * h12env_create selects the two-kernel path), else 0.  Results are bit-identical either way.  Replaces the separate
 * probability pass of CaT.compute (biped_tasks/utils/cat/cat_env.py:95-193, constraint_manager.py:126-269). */
int h12env_cat_inline(const h12env* h);
/* ObservationManager.compute() outside step(): appends one frame of the current state to every
 * env's history (obs_prev -> obs, may alias); fill_mask[i] != 0 fills env i's history with the frame
 * (the first push after a reset).  fill_mask may be NULL. */
int h12env_observe(h12env* h, const float* obs_prev, float* obs, const uint8_t* fill_mask, void* stream);
/* Heightfield terrain (cfg.terrain = 1), device arrays owned by the caller and kept alive while the
 * handle uses them: heights[ix * ny + iy] is the ground height at (x0 + ix*hscale, y0 + iy*hscale),
 * triangulated like isaaclab.terrains.utils.convert_height_field_to_mesh (cells split along the
 * (ix, iy) -> (ix+1, iy+1) diagonal); origins[(level * cols + type) * 3 + k] are the sub-terrain
 * origins the curriculum moves envs between.  Replaces TerrainImporter (velocity_env_cfg.py:40-56). */
int h12env_set_terrain(h12env* h, const float* heights, int nx, int ny, float hscale, float x0, float y0,
                       const float* origins, int rows, int cols);
/* Parity hook: n_substeps physics steps with a held joint target q_ref (N x 12) using the
 * configured mode (PD, limits, contact), no MDP.  Mirrors H12Mujoco.step. */
int h12env_step_physics(h12env* h, const float* q_ref, int n_substeps, void* stream);
/* Parity hook: the MDP term code of h12env_step (unweighted reward terms [H12_NREW][N], terminated, truncated
 * and, on a CaT env, the constraint rows [H12_NCSTR_COLS + 4][N] into cstr: the 56 raw columns, the no_move flag,
 * the pre-reset episode length, and foot_clearance's updated swing height (left, right)) evaluated on the workspace state as
 * it stands (post-physics, pre-reset; EPLEN already counted) with injected tau (N x 12, applied torque), jacc
 * (N x 12, joint acceleration) and fmax (N x 5: max over the contact history of |F| on the left / right foot,
 * left / right knee, torso).  Read-only on the workspace: foot_clearance is evaluated on the stored swing height,
 * which (unlike a step) is not updated -- the updated value goes to cstr's last two rows -- so calls between
 * steps do not change the env.  Replaces nothing in the
 * reference: it exposes RewardManager / TerminationManager / ConstraintManager term functions
 * (velocity/mdp/rewards.py, utils/cat/constraints.py) for the reference-fixture tests. */
int h12env_eval_terms(h12env* h, const float* tau, const float* jacc, const float* fmax, float* terms,
                      uint8_t* terminated, uint8_t* truncated, float* cstr, void* stream);

/* Parity hook (tests only): the self-contact wrenches between the legs (h12env_config.self_collision) that the
 * physics step applies on the workspace state as it stands; out (device, n x 2 x 2 x 6): per env, leg (left,
 * right), body (knee, foot): moment xyz, force xyz in body coordinates.  Replaces nothing in the reference (its
 * self-collisions live inside PhysX, ArticulationCfg enabled_self_collisions, A/robots/h12.py:32). */
int h12env_eval_self_contacts(h12env* env, float* out, void* stream);
/* ---- Rollout records (ABI 8; BASELINE config C4: the rollout buffer all-gathered over xGMI for PPO).
 * rsl_rl's RolloutStorage keeps (T, N, 450) observations per iteration (T = num_steps_per_env 24,
 * C12/agents/rsl_rl_ppo_cfg.py:12).  A 450-float row is 10 frames of 45 floats, nine of them already in the previous
 * row (CircularBuffer, T/utils/history/circular_buffer.py:79-170), so a shard's rollout is recorded compactly --
 * per env-step the new frame (h12env_step_out.frame_out), the action, the reward and the two done flags: 238 B
 * instead of 1856 B -- gathered over the ranks, and the full rows are rebuilt on every receiving GPU.
 * Step record of one shard of n envs (byte offsets from h12env_rollout_layout, each section 256-B aligned):
 *   [0] frames f32 [n][45]   [1] actions f32 [n][12]   [2] rewards f32 [n]   [3] terminated u8 [n]
 *   [4] truncated u8 [n]
 * A shard's rollout is T step records back to back ([T][step_bytes]).  It is all-gathered in chunks of G steps
 * (the last chunk may be shorter): chunk c (steps [cG, cG + Gc)) is one all_gather_into_tensor of the shards'
 * bytes [cG, cG + Gc) x step_bytes, so the gathered buffer is, per chunk in order, n_shards runs of Gc step
 * records (G = T: n_shards whole rollouts back to back).  Global env id = shard * n + local id. */
int h12env_rollout_layout(int n, size_t offsets[5], size_t* step_bytes);
/* Rebuild observation rows from gathered rollout records: obs_out[t][g][:] (T x n_shards*n x 45*history) is the
 * observation the env returned after step t for global env g, for t in [t0, t1) (the records of steps < t1 must be
 * present).  tail (n_shards*n x 45*history) holds each env's observation before step 0 of the records (the last
 * row of the previous iteration); it may alias obs_out's row T - 1 (every block reads its envs' tail rows before
 * it writes any of their rows).  Rows are bit-identical to the env's own: slot h of row t is the frame of step
 * t - (history - 1 - h), or of the env's last done step <= t if that is later (a reset refills the history), or,
 * before step 0, the tail row's slot h + t + 1. */
int h12env_rollout_decode(const void* records, int n_shards, int n, int T, int G, int history, int t0, int t1,
                          const float* tail, float* obs_out, void* stream);
/* Stream fences (ABI 8): 64-bit counters in signal memory for ordering two streams without HIP events --
 * h12env_fence_signal enqueues "counter[slot] = value" behind all earlier work of the stream
 * (hipStreamWriteValue64), h12env_fence_wait makes every later command of the stream wait until
 * counter[slot] >= value (hipStreamWaitValue64).  The rollout all-gather orders its side stream against the env
 * stream with these (an event record + cross-stream wait cost ~100 us of host time per hand-off here; DESIGN.md
 * section 6).  Counters start at 0; values must increase per slot. */
typedef struct h12env_fence h12env_fence;
int h12env_fence_create(int device, int n_slots, h12env_fence** out);
void h12env_fence_destroy(h12env_fence* f);
int h12env_fence_signal(h12env_fence* f, int slot, uint64_t value, void* stream);
int h12env_fence_wait(h12env_fence* f, int slot, uint64_t value, void* stream);
/* Device pointer of a state field (see H12_F_* / H12_I_*), NULL on error. */
void* h12env_field_ptr(h12env* h, int is_int, int field);
int h12env_num_envs(const h12env* h);
/* Observation row length: 45 x history_length (flat layout; 450 Flat, 270 Rsl) or 235 (rough). */
int h12env_obs_dim(const h12env* h);
/* Replace the reward weights (n <= H12_NREW floats, indexed by H12_R_*) for the following steps:
 * CurriculumManager's modify_reward_weight (rsl_env_cfg.py:448-501) without recreating the handle. */
int h12env_set_reward_weights(h12env* h, const float* w, int n);
/* Replace the constraint terms' max_p (n <= H12_NCSTR) for the following steps: the CaT curriculum
 * modify_constraint_p (T/utils/cat/curriculums.py:16-42). */
int h12env_set_constraint_max_p(h12env* h, const float* max_p, int n);
/* Algorithmic accounting of one env step for the roofline report (both kernels of h12env_step). */
int h12env_step_cost(const h12env* h, double* bytes_per_env, double* flops_per_env);
/* Per-kernel accounting: kernel 0 = the env kernel of h12env_step (physics + MDP), 1 = the observation
 * assembly kernel (history shift + noise + fills).  Compulsory HBM bytes and counted FLOPs per env. */
int h12env_kernel_cost(const h12env* h, int kernel, double* bytes_per_env, double* flops_per_env);
/* Instrumentation (off by default): while enabled, h12env_step launches step_kernel and the observation
 * kernel with HIP event pairs bound to their dispatches (hipExtLaunchKernelGGL: begin / end of the kernel's
 * execution, the interval rocprofv3's kernel trace reports; at most 4096 steps are kept).
 * h12env_kernel_times synchronises on the last event, returns the summed milliseconds of each kernel and
 * the number of timed steps, and clears the record. */
int h12env_set_kernel_timing(h12env* h, int enable);
/* step_kernel's LDS budget (round 6): static hand-off bytes, the fused observation path's dynamic bytes and the
 * limit per CU.  With h = NULL the values compiled into the library (a compile-time assert holds static + dynamic
 * <= 160 KiB); with a handle the compiled kernel's static size (hipFuncGetAttributes), the dynamic bytes its step
 * launches use and the device's LDS per CU -- h12env_create refuses a configuration over the limit with
 * H12_E_STATE instead of letting the dispatch abort the queue.  No reference counterpart (PhysX sizes its own). */
int h12env_step_lds(const h12env* h, size_t* static_bytes, size_t* dynamic_bytes, size_t* limit_bytes);
/* Synchronises the stream and reads / clears the device diagnostic word: H12_E_STATE with a message when a
 * self-contact wait in step_kernel ended at its bound since the last check (that inner step's self-contact
 * wrenches may be partial), or (round 6) a CaT block's wait for the last block's fold did (that step's constraint
 * probabilities may be stale), else 0.  The Python host calls it when it already synchronises (episode-log reads,
 * close).  No reference counterpart (PhysX reports solver failures through its own error callback). */
int h12env_check(h12env* h, void* stream);
int h12env_kernel_times(h12env* h, double* env_ms, double* obs_ms, int* n_steps);
const char* h12env_last_error(void);
int h12env_abi_version(void);
/* sizeof of the ABI structs as compiled (0 = h12env_model, 1 = h12env_config, 2 = h12env_step_out),
 * so bindings can verify their mirrors; 0 for an unknown id. */
size_t h12env_sizeof_struct(int which);

#ifdef __cplusplus
}
#endif
#endif /* H12ENV_H */
