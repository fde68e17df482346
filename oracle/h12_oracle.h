/*
 * h12_oracle.h — CPU restatement (TEST INFRASTRUCTURE ONLY) of the H1-2 Flat velocity env step.
 *
 * This is the parity oracle for the HIP library: only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.  The product path (h12env python package -> libh12env.so)
 * never links or calls it.
 *
 * It restates, in double precision and with deliberately different algorithms from the
 * GPU kernel where that strengthens the check:
 *   - rigid-body dynamics: CRBA + RNEA + dense Cholesky (MuJoCo's own formulation, the
 *     sim2sim oracle path packages/biped_deploy/biped_deploy/simulator/sim_mujoco.py:39-44,109)
 *     and, separately, Featherstone ABA (cross-checked against CRBA in tests);
 *   - the explicit delayed PD actuator (packages/biped_assets/biped_assets/robots/h12.py:58-112;
 *     delay indexing = CircularBuffer.__getitem__, .../utils/history/circular_buffer.py:139-170);
 *   - the MDP terms of Isaac-Velocity-Flat-H12_12dof-v0 (rewards, terminations, resets,
 *     commands, observations + 10-frame history) as restated in SURVEY.md §8(a);
 *   - the rough task's additions (heightfield contact, height scan, base_lin_vel, terrain
 *     curriculum, per-env friction / added torso mass) as restated in DESIGN.md (row f2);
 *   - the Rsl task's additions (rsl_env_cfg.py: reward terms 12-19, deadzone commands with
 *     sign flips, push_by_setting_velocity interval event, observation history 6 + term scales,
 *     resampling-time range) as restated in DESIGN.md (row f4).
 *
 * Parity status: the algorithm of record (PhysX / MuJoCo / IsaacLab managers) is not present
 * in this container, so physics parity against it is UNPINNED; the oracle itself is pinned
 * by the reference's importable pieces (CircularBuffer, deploy ObservationHandler) through
 * tests/golden fixtures, and by physical invariants (energy, momentum, ABA == CRBA).
 */
#ifndef H12_ORACLE_H
#define H12_ORACLE_H
#include <stdint.h>
#include "../include/h12env.h"

#ifdef __cplusplus
extern "C" {
#endif

/* physics state in double (MuJoCo layout: pos, quat(wxyz), v_world, w_body, q, qd) */
typedef struct orc_phys {
  double pos[3], quat[4], vlin[3], wang[3], q[H12_NJ], qd[H12_NJ];
  double anchor[2][H12_NFOOT_PTS][2]; /* sole-sphere stiction anchors (world x, y) */
  int32_t cmask;                      /* bit 4f+p: sole sphere p of foot f was in contact */
  int32_t env_params;                 /* 1: mu / dmass below apply (per-env startup randomisation) */
  double mu[2][2];                    /* static, dynamic friction of the left / right sole */
  double dmass;                       /* mass added at the torso COM */
} orc_phys;

/* per physics-step contact report */
typedef struct orc_contact_report {
  double foot_force[2][3];   /* net world force on each foot */
  double knee_force[2][3];
  double torso_force[3];
} orc_contact_report;

/* ---- single-env physics (double) ---- */
/* Forward dynamics: generalised acceleration nudot = (wdot_b, vdot_b (spatial), qdd).
 * tau: joint torques; algo 0 = CRBA+Cholesky, 1 = ABA.  dt_impl: implicit damping dt (0 = none).
 * with_contact: evaluate penalty contact forces (report may be NULL). */
int orc_forward_dynamics(const h12env_model* m, const h12env_config* c, const orc_phys* s,
                         const double tau[H12_NJ], int algo, double dt_impl, int with_contact,
                         double nudot[18], orc_contact_report* rep);
/* Joint-space mass matrix (18 x 18, row major, base coords (w_b, v_b)), armature included. */
int orc_mass_matrix(const h12env_model* m, const orc_phys* s, double M[18 * 18]);
/* Total mechanical energy (kinetic + potential), linear + angular momentum about the world origin. */
int orc_self_contacts(const h12env_model* m, const h12env_config* c, const orc_phys* s, double* fext,
                      orc_contact_report* rep);
int orc_body_poses(const h12env_model* m, const orc_phys* s, double* R, double* p);
int orc_energy_momentum(const h12env_model* m, const orc_phys* s, double* energy, double lin_mom[3],
                        double ang_mom[3]);
/* One physics step of length c->physics_dt split into c->inner_steps, holding tau_pd;
 * joint limits (+ contact unless disabled) re-evaluated per inner step.  Averaged contact
 * forces are written to rep (may be NULL). */
int orc_physics_step(const h12env_model* m, const h12env_config* c, orc_phys* s, const double tau_pd[H12_NJ],
                     int with_contact, int algo, orc_contact_report* rep);
/* MuJoCo sim2sim loop (h12_mujoco.py:55-67): n_steps physics steps, PD to q_ref recomputed
 * every step, clamp at MJCF actuatorfrcrange.  traj (may be NULL) gets q after every step. */
int orc_mujoco_rollout(const h12env_model* m, const h12env_config* c, orc_phys* s, const double* q_ref,
                       int n_steps, int with_contact, int algo, double* traj_q);

/* ---- batched env API on the GPU workspace layout (field-major SoA floats / ints) ----
 * These mirror h12env_reset / h12env_step on host arrays so tests can feed both sides the
 * same state.  Compute is double; state storage is float (same as the workspace). */
int orc_env_reset(const h12env_model* m, const h12env_config* c, int n, int64_t env_offset,
                  float* fstate, int32_t* istate, const uint8_t* mask, float* obs, uint64_t reset_counter);
int orc_env_step(const h12env_model* m, const h12env_config* c, int n, int64_t env_offset, float* fstate,
                 int32_t* istate, const float* actions, const float* obs_prev, float* obs, float* rew,
                 uint8_t* terminated, uint8_t* truncated, float* log_acc, float* applied_torque,
                 float* foot_force, float* cstr_prob, int64_t step_index, int n_threads);
/* ---- MDP terms on a post-physics snapshot (the code orc_env_step runs; fixture-pinned in tests/) ---- */
typedef struct orc_term_in {
  orc_phys p;                      /* post-physics state of the env step */
  double act[H12_NJ], act_prev[H12_NJ]; /* ActionManager action / prev_action */
  double cmd[3];                   /* base_velocity command (pre-reset) */
  double air[2], con[2];           /* ContactSensor current_air_time / current_contact_time of the feet */
  double tau[H12_NJ];              /* applied_torque */
  double jacc[H12_NJ];             /* joint_acc */
  double fmax_foot[2], fmax_knee[2], fmax_torso; /* max over net_forces_w_history (3) of |F| */
  int eplen;                       /* episode_length_buf after this step's increment */
} orc_term_in;
/* terminations + the H12_NREW unweighted reward terms */
int orc_mdp_terms(const h12env_model* m, const h12env_config* c, const orc_term_in* in, double terms[H12_NREW],
                  int* terminated, int* time_out);
/* CaT constraint values of one env (+ still flag, episode length): out[col * stride], col < H12_NCSTR_COLS + 2;
 * swing_h = foot_clearance's swing_max_height (in / out) */
int orc_cat_row(const h12env_model* m, const h12env_config* c, const orc_term_in* in, int terminated,
                double swing_h[2], double* out, size_t stride);
/* CaT.add / get_probs over a batch of rows [H12_NCSTR_COLS + 2][n] (no_move remap included); run_max / run_init
 * carry the running maxima; pmax [n], pterm [H12_NCSTR][n] and ceff [H12_NCSTR_COLS][n] (may be NULL) out */
int orc_cat_probs(const h12env_config* c, int n, const double* cs, double run_max[H12_NCSTR_COLS], int* run_init,
                  double* pmax, double* pterm, double* ceff);

/* ConstraintManager episode statistics + their reset into the log accumulator; sum_v / sum_p [H12_NCSTR][n] */
void orc_cat_stats(const h12env_config* c, int n, const double* pterm, const double* eplen, const uint8_t* reset,
                   float* sum_v, float* sum_p, float* log_acc);
/* commands: the update given its decisions (returns 1 = resample this env); terrain curriculum decision */
int orc_cmd_update_decided(const h12env_config* c, double cmd[3], double heading_target, const double quat[4],
                           int is_heading, int is_standing, int deactivate, int activate, int flip);
void orc_terrain_move(const h12env_config* c, const double pos[3], const double origin[3], const double cmd[3], int* up,
                      int* down);
/* observations from explicit noise draws: the 45-float frame (noise + scale), the rough row (noise + clip),
 * and one history update with nh frames per term */
void orc_obs_frame_from(const h12env_config* c, const double raw[H12_OBS_FRAME], const double u[30],
                        double fr[H12_OBS_FRAME]);
void orc_rough_row_from(const h12env_config* c, const double raw[H12_NOBS_ROUGH], const double u[H12_NOBS_ROUGH - 15],
                        float* out);
void orc_history_write_n(const double frame[H12_OBS_FRAME], const float* prev_row, float* out_row, int fill, int nh);

/* CaT running maxima carried between steps (process-global): forget them / read them. */
void orc_cat_reset(void);
void orc_cat_running_max(double out[H12_NCSTR_COLS]);
/* The last orc_env_step's raw constraint values, [H12_NCSTR_COLS + 2][n] (+ no_move flag, pre-reset
 * episode length); -1 if n differs. */
int orc_cat_last_constraints(double* out, int n);
/* Physics-only batched step (h12env_step_physics): n_substeps with held q_ref per env. */
int orc_env_step_physics(const h12env_model* m, const h12env_config* c, int n, float* fstate, int32_t* istate,
                         const float* q_ref, int n_substeps);

/* Observation of the current state (ObservationManager.compute outside step), fill_mask may be NULL. */
int orc_env_observe(const h12env_model* m, const h12env_config* c, int n, int64_t env_offset, float* fstate,
                    int32_t* istate, const float* obs_prev, float* obs, const uint8_t* fill_mask, uint64_t counter);
/* Delayed-target source of substep `substep`: 0 = a_t, 1 = a_{t-1}, 2 = a_{t-2}. */
int orc_delay_source(int lag, int since_reset, int substep, int decimation);
/* One history update of a 450-float observation row (term-major, oldest -> newest). */
void orc_history_write(const double frame[H12_OBS_FRAME], const float* prev_row, float* out_row, int fill);

/* Heightfield used while c->terrain = 1 (same layout as h12env_set_terrain; host arrays, kept alive by the
 * caller).  Process-global: the oracle is single-terrain test infrastructure. */
void orc_set_terrain(const float* heights, int nx, int ny, double hscale, double x0, double y0,
                     const float* origins, int rows, int cols);
/* Ground height and slope at (x, y) (plane z = 0 when c->terrain = 0). */
double orc_ground(const h12env_config* c, double x, double y, double* gx, double* gy);
/* Observation row length of the configured task: 45 x history_length (flat layout) or 235 (rough). */
int orc_obs_dim(const h12env_config* c);
/* Deadzone command count carried from one orc_env_step to the next (the kernel's rotating counter);
 * process-global like the terrain. */
void orc_set_dz_count(int v);
/* test hook: jitter of the self-contact capsule end points (m), see h12_oracle.c capsule_world */
void orc_set_self_jitter(double eps, uint64_t seed);
/* test hook: jitter the joint-limit (rad) / ground-contact (m) switching decisions (forced.py only) */
void orc_set_threshold_jitter(double lim_eps, double contact_eps, uint64_t seed);
int orc_dz_count(void);

/* RNG shared by both sides (Philox4x32-10). */
void orc_philox(uint64_t seed, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t out[4]);

#ifdef __cplusplus
}
#endif
#endif
