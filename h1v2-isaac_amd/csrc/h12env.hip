// h12env.hip — MI355X (gfx950) implementation of the Isaac-Velocity-Flat-H12_12dof-v0 env step.
//
// One fused kernel per env step: delayed explicit PD (h12.py:58-112) -> decimation x inner_steps x
// (penalty contact + Featherstone ABA over the 13-body tree + semi-implicit Euler) -> contact sensor
// (history 3, air time) -> terminations -> 12 reward terms -> masked in-kernel resets -> command
// update -> observation frame + 10-frame history (ManagerBasedRLEnv.step, cat_env.py:95-193).
//
// Thread mapping: a LANE PAIR per env (lanes 2e, 2e+1 of a wave64 own the left / right leg).
// Mirror lanes: the H1-2 right leg is the exact mirror image of the left one about the pelvis
// xz-plane, so the right-leg lane runs the very same code and literal constants in MIRRORED
// coordinates (y -> -y; x/z joint angles negated).  The two legs meet only at the floating base:
// each lane un-mirrors its leg's articulated inertia / bias force, one DPP lane swap exchanges them,
// and both lanes solve the same 6x6 base system (fixed left+right summation order keeps the two
// copies bit-identical).  State is structure-of-arrays so each field access of a wave is one
// contiguous segment; the 450-float observation rows are written cooperatively through LDS so each
// wave stores its 32 consecutive rows as one contiguous, coalesced block.
//
// Register budget (one wave per SIMD, latency-bound): ABA keeps only the link spatial velocities
// between passes (bias forces and velocity-product accelerations are recomputed from them), MDP state
// is loaded after the physics loop, and the contact-sensor timers are replayed from per-substep flags.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <new>
#include <algorithm>
#include <vector>

#include "../../include/h12env.h"
#include "h12_math.h"
#include "h12_model_gen.h"

using namespace h12;

namespace {

constexpr int NJ = H12_NJ;
constexpr int NL = 6;               // links per leg
constexpr int ENVS_PER_BLOCK = 32;  // 64 lanes = 32 lane pairs
// episode-log values accumulated per block (partial slots, folded by the assembly kernel): step_kernel's reward sums,
// reset count, time-out / base-contact counts, command metrics, then cat_prob_kernel's constraint violation rates
// and mean probabilities.  Partial slot pv -> log slot:
constexpr int LOG_NSTEP = H12_NREW + 3 + 2, LOG_NPART = LOG_NSTEP + 2 * H12_NCSTR;
__host__ __device__ constexpr int log_slot(int pv) {
  return pv < H12_NREW + 3 ? pv : (pv < LOG_NSTEP ? H12_LOG_METRIC + (pv - H12_NREW - 3) : H12_NREW + 4 + (pv - LOG_NSTEP));
}
constexpr int BLOCK = 64;
// joint axes per leg link: hip yaw z, hip pitch y, hip roll x, knee y, ankle pitch y, ankle roll x
constexpr int AX[NL] = {2, 1, 0, 1, 1, 0};
constexpr int MAX_DEC = 32;         // contact flags of one env step are kept in a 32-bit mask
constexpr int FRAME_ROWS = H12_ROUGH_FRAME + 5;
// Kernel feature level K (template): 0 = plain flat task (no per-env parameters, plane, 45-row frame:
// the hot path compiles none of the rough-task code), 1 = extended features on the plane (rough layout,
// per-env friction / mass; runtime flags), 2 = extended + heightfield.
template <int K> struct Feat {
  static constexpr bool ext = K >= 1;
  static constexpr bool terrain = K == 2;
};  // frame scratch rows (rough: + base position, yaw cos / sin)

// experiment builds only (-DH12_PHASE_PROFILE): per-phase shader-clock cycles of step_kernel, summed
// over waves (lane 0), read back with h12env_phase_profile.  Not part of the product library.
#ifdef H12_PHASE_PROFILE
__device__ unsigned long long g_phase[16];
// per physics wave of the last launch, realtime: [0] start, [1] end, [2] end after waitcnt, [3] after the physics
// loop, [4] after reset + command, [5] XCC id, [6] after the frame + barrier F (before the state stores),
// [7] / [8] the shader-clock counter (s_memtime) at the start / at [2] -> the XCD's clock rate over the wave,
// [9] / [10] the cycles this wave waited in barriers R1 / R2 over the launch
__device__ unsigned long long g_wave[1024][11];
#ifdef H12_PHASE_LIGHT
// light mode (-DH12_PHASE_PROFILE -DH12_PHASE_LIGHT): the realtime stamps only, kept in registers and stored once at
// the wave's end (no per-phase atomics): the least perturbed view of the product kernel's per-XCD timing
// (columns 9 / 10: after the rewards, after barrier L)
#define PH_INIT() const unsigned long long _ph_rt0 = __builtin_amdgcn_s_memrealtime(); \
  unsigned long long _ph_s1 = 0, _ph_s3 = 0, _ph_s4 = 0, _ph_s5 = 0, _ph_s6 = 0
#define PH_WAVE_END()                                                          \
  do {                                                                         \
    const unsigned long long _r1 = __builtin_amdgcn_s_memrealtime();           \
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                           \
    const unsigned long long _r2 = __builtin_amdgcn_s_memrealtime();           \
    unsigned _xcc;                                                             \
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(_xcc));        \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 1024) {                        \
      g_wave[blockIdx.x][0] = _ph_rt0; g_wave[blockIdx.x][1] = _r1; g_wave[blockIdx.x][2] = _r2; \
      g_wave[blockIdx.x][3] = _ph_s1; g_wave[blockIdx.x][4] = _ph_s5; g_wave[blockIdx.x][6] = _ph_s6; \
      g_wave[blockIdx.x][5] = _xcc & 15u;                                      \
      g_wave[blockIdx.x][9] = _ph_s3; g_wave[blockIdx.x][10] = _ph_s4;          \
    }                                                                          \
  } while (0)
#define PH(i)                                                                       \
  do {                                                                              \
    if (i == 1) _ph_s1 = __builtin_amdgcn_s_memrealtime();                         \
    if (i == 3) _ph_s3 = __builtin_amdgcn_s_memrealtime();                         \
    if (i == 4) _ph_s4 = __builtin_amdgcn_s_memrealtime();                         \
    if (i == 5) _ph_s5 = __builtin_amdgcn_s_memrealtime();                         \
    if (i == 6) _ph_s6 = __builtin_amdgcn_s_memrealtime();                         \
  } while (0)
#define PHX_INIT() (void)0
#define PHX(i) (void)0
// the helper / self-contact waves' end (after their stores completed): columns 7 / 8
#define PH_HELPER_END()                                                        \
  do {                                                                         \
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                           \
    const unsigned long long _he = __builtin_amdgcn_s_memrealtime();           \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 1024)                          \
      g_wave[blockIdx.x][threadIdx.x < 2 * BLOCK ? 7 : 8] = _he;               \
  } while (0)
#else
#define PH_HELPER_END() (void)0
#define PH_INIT() unsigned long long _ph_t = __builtin_readcyclecounter(); \
  const unsigned long long _ph_c0 = _ph_t;                                \
  const unsigned long long _ph_rt0 = __builtin_amdgcn_s_memrealtime();    \
  if ((threadIdx.x & 63) == 0 && blockIdx.x < 1024) g_wave[blockIdx.x][9] = g_wave[blockIdx.x][10] = 0
#define PH_WAVE_END()                                                          \
  do {                                                                         \
    const unsigned long long _r1 = __builtin_amdgcn_s_memrealtime();           \
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                           \
    const unsigned long long _r2 = __builtin_amdgcn_s_memrealtime();           \
    const unsigned long long _c2 = __builtin_readcyclecounter();               \
    unsigned _xcc;                                                             \
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(_xcc));        \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 1024) {                        \
      g_wave[blockIdx.x][0] = _ph_rt0; g_wave[blockIdx.x][1] = _r1; g_wave[blockIdx.x][2] = _r2; \
      g_wave[blockIdx.x][5] = _xcc & 15u;                                      \
      g_wave[blockIdx.x][7] = _ph_c0; g_wave[blockIdx.x][8] = _c2;             \
    }                                                                          \
  } while (0)
#define PH(i)                                                                       \
  do {                                                                              \
    unsigned long long _t = __builtin_readcyclecounter();                           \
    if ((threadIdx.x & 63) == 0) atomicAdd(&g_phase[i], _t - _ph_t);                \
    if ((i == 1 || i == 5 || i == 6) && (threadIdx.x & 63) == 0 && blockIdx.x < 1024) \
      g_wave[blockIdx.x][i == 1 ? 3 : i == 5 ? 4 : 6] = __builtin_amdgcn_s_memrealtime(); \
    _ph_t = _t;                                                                     \
  } while (0)
// inside inner_step (its own clock mark): slots 10.. split the inner step around the helper hand-off
#define PHX_INIT() unsigned long long _phx_t = __builtin_readcyclecounter()
#define PHX(i)                                                                      \
  do {                                                                              \
    unsigned long long _t = __builtin_readcyclecounter();                           \
    if ((threadIdx.x & 63) == 0) atomicAdd(&g_phase[i], _t - _phx_t);               \
    if ((i == 8 || i == 9) && (threadIdx.x & 63) == 0 && blockIdx.x < 1024)         \
      atomicAdd(&g_wave[blockIdx.x][i + 1], _t - _phx_t);                           \
    _phx_t = _t;                                                                    \
  } while (0)
#endif
#else
#define PH_HELPER_END() (void)0
#define PH_INIT() (void)0
#define PH_WAVE_END() (void)0
#define PH(i) (void)0
#define PHX_INIT() (void)0
#define PHX(i) (void)0
#endif
// experiment builds only (-DH12_PHASE_PROFILE -DH12_PHASE_LIGHT): the shader-clock cycles each wave of step_kernel waits
// in the inner steps' barriers S / R1 / R2 (and separately the first S, index 3), accumulated in registers and stored once per wave ([block][role][barrier];
// roles 0 physics, 1 helper, 2 contact, 3 self): the wave that waits ~0 at a barrier is the one the block waited for
#if defined(H12_PHASE_PROFILE) && defined(H12_PHASE_LIGHT)
// [4..7]: the cycles each role spends between its previous barrier and barrier k (its own work before k)
// [12..14]: the same work times of the first inner step alone (from the first barrier S on; the instruction cache
// starts every launch cold), [13 of _bw]: set once the first inner step's barrier S has passed; [15] (_bw[17]): the
// wave's start (s_memrealtime, 100 MHz)
__device__ unsigned long long g_bw[1024][4][16];
#define H12_BW_DECL                                                                                                   \
  unsigned long long _bw[18] = {0ull, 0ull, 0ull, 0ull, 0ull, 0ull, 0ull, 0ull, __builtin_readcyclecounter(),       \
                                0ull, 0ull, 0ull, 0ull, 0ull, 0ull, 0ull, 0ull, __builtin_amdgcn_s_memrealtime()}
#define H12_BW_PARAM , unsigned long long (&_bw)[18]
// every wave's very first instruction (s_memrealtime; before any kernel-argument load), [block][wave]
__device__ unsigned long long g_kstart[1024][4];
#define H12_BW_KSTART()                                                          \
  do {                                                                           \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 1024)                            \
      g_kstart[blockIdx.x][threadIdx.x >> 6] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
// the physics wave's start stamp taken at its entry (its H12_BW_DECL follows the state loads)
#define H12_BW_ENTRY() const unsigned long long _bw_entry = __builtin_amdgcn_s_memrealtime()
#define H12_BW_SET_ENTRY() (_bw[17] = _bw_entry)
#define H12_BW_ARG , _bw
#define SYNC_W(k)                                                                \
  do {                                                                           \
    const unsigned long long _t0 = __builtin_readcyclecounter();                \
    _bw[4 + (k)] += _t0 - _bw[8];                                                \
    if ((k) != 3 && _bw[13] == 0) _bw[14 + (k)] += _t0 - _bw[8];                 \
    __syncthreads();                                                             \
    _bw[8] = __builtin_readcyclecounter();                                       \
    _bw[k] += _bw[8] - _t0;                                                      \
    if ((k) == 0) _bw[13] = 1;                                                   \
  } while (0)
// [9 + i]: the physics wave's time from its last barrier exit to mark i (PHL), summed: offsets inside a segment
#define PHL(i) (_bw[9 + (i)] += __builtin_readcyclecounter() - _bw[8])
// the self wave: the most candidate envs of an inner step (in its mark slot 0) and their sum (slot 1)
#define PHN(n) (_bw[9] = max(_bw[9], (unsigned long long)(n)), _bw[10] += (unsigned long long)(n))
#define H12_BW_STORE()                                                           \
  do {                                                                           \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 1024)                            \
      for (int _k = 0; _k < 11; ++_k) g_bw[blockIdx.x][threadIdx.x >> 6][_k] = _bw[_k + (_k >= 8)]; \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 1024)                            \
      for (int _k = 0; _k < 3; ++_k) g_bw[blockIdx.x][threadIdx.x >> 6][12 + _k] = _bw[14 + _k]; \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 1024) g_bw[blockIdx.x][threadIdx.x >> 6][15] = _bw[17];  \
  } while (0)
// slot 11: the wave's arrival at barrier F (s_memrealtime, 100 MHz: comparable across the waves of a block)
#define H12_BW_F_ARRIVAL()                                                       \
  do {                                                                           \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 1024)                            \
      g_bw[blockIdx.x][threadIdx.x >> 6][11] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define H12_BW_DECL (void)0
#define H12_BW_ENTRY() (void)0
#define H12_BW_KSTART() (void)0
#define H12_BW_SET_ENTRY() (void)0
#define H12_BW_PARAM
#define H12_BW_ARG
#define PHL(i) (void)0
#define PHN(n) (void)0
#define SYNC_W(k) __syncthreads()
#define H12_BW_STORE() (void)0
#define H12_BW_F_ARRIVAL() (void)0
#endif

thread_local char g_err[512] = "";
int set_err(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int set_err(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
  return code;
}
#define HIP_TRY(expr)                                                                        \
  do {                                                                                       \
    hipError_t _e = (expr);                                                                  \
    if (_e != hipSuccess) {                                                                  \
      (void)hipGetLastError(); /* no sticky error left for the caller's next HIP call */     \
      return set_err(H12_E_HIP, "%s: %s", #expr, hipGetErrorString(_e));                     \
    }                                                                                        \
  } while (0)

// ------------------------------------------------------------------ runtime parameters (kernarg)
struct KParams {
  float kp[NL], kd[NL], elim[NL], dimpl[NL];  // per leg link (leg-symmetric)
  float vmax[NL];         // PhysX max joint velocity (h12env_config.max_joint_vel; 0 -> no limit = 3e38)
  float cv;               // its damper (h12env_config.max_joint_vel_damping)
  int dgroup[NL];
  float g;
  int mode, fix_base, decimation, inner, max_len, min_delay, max_delay, use_fl;
  int corrupt, ill_knees, ill_torso;
  float dt, h, step_dt, action_scale, soft_f;
  float ck, cc, fk, fc, mus, mud, lk, lc, cthr;
  // implicit contact (h12env_config.implicit_penalty): cc / fc already include the
  // extra damping h k; impl != 0 adds the point inertia h cc (normal) / h fc (tangential, sticking or
  // below the drag cap) of every active contact to its body in the dynamics solve
  int impl;
  float fc_v;             // viscous tangential coefficient of the knee / torso contacts
  int self_coll;          // self-collision between the legs (h12env_config.self_collision)
  float sk, sc, sct, smu; // its normal stiffness / damping, tangential damping, Coulomb cap
  float dl;               // implicit joint-limit inertia h (lc + h lk) (lc already includes h lk)
  float lproj;            // hard-limit projection tolerance (h12env_config.limit_projection; 3e38: off)
  float dcap;             // depth cap of the contact spring, h * max_depenetration_velocity (3e38: off)
  float cmd_T, cmd_x0, cmd_x1, cmd_y0, cmd_y1, cmd_w0, cmd_w1, cmd_h0, cmd_h1;
  float rel_stand, rel_head, head_k;
  float rx0, rx1, ry0, ry1, ryaw0, ryaw1, root_z;
  float n_w, n_g, n_q, n_qd;
  float rew_w[H12_NREW];
  float std2_inv, air_thr;
  uint32_t seed_lo, seed_hi;
  // rough task / terrain / startup randomisation
  int task, terrain, curriculum, env_mu, env_mass;
  float n_lin, n_scan, scan_off, scan_clip, scan_res, terrain_size, ep_len_s;
  const float* t_h;       // heightfield [nx][ny] (device)
  const float* t_origin;  // [rows][cols][3]
  int t_nx, t_ny, t_rows, t_cols;
  float t_x0, t_y0, t_inv_hs;
  // Rsl task (rsl_env_cfg.py): reward terms 12-19, deadzone commands, pushes, history / scales
  int rsl;                // reward terms 12-19 are weighted (computed only then)
  float cmd_T1;           // resampling_time_range upper bound
  int dz;                 // UniformVelocityCommandWithDeadzone
  float dz_v, flip_p;
  int* dz_cnt;            // 3 rotating deadzone counters (handle-owned)
  int push;               // push_by_setting_velocity interval event
  float push_t0, push_t1, push_x0, push_x1, push_y0, push_y1;
  int hist;               // observation history length (flat layout)
  float oscale[6];        // per-term observation scale
  float h_target, cf_thr;
  // CaT task (T/utils/cat/*): constraints -> termination probabilities
  int cat;
  uint32_t cmask;
  float cmaxp[H12_NCSTR], ctau, cminp;
  float cvlim[NL], celim[NL];  // joint velocity / effort limits (leg-symmetric)
  float c_ff, c_nm_dz, c_nm_v, c_or, c_h, c_hstd, c_clr, c_clr_dz;
  float* cscr;            // [CAT_ROWS][n] raw constraints of the step (+ no_move flag, pre-reset episode length)
  float* crun;            // [2][H12_NCSTR_COLS] running maxima (CaT.running_maxes) and their reciprocals; 512 B after
                          // it, cat_inline's published fold (cat_cpub: no field of its own -- one more kernel argument
                          // shifted step_kernel's kernarg layout and measured 0.7 % slower on the Flat window)
  int* clist;             // [n] no_move-active envs in ascending order (the reference's row remap)
  int* cmeta;             // [0] = number of no_move-active envs, [1] = running maxima initialised, [2] = step_kernel
                          // blocks done with their CaT hand-off this launch (cat_fold); [64, 64 + 8 x 56) = the step's
                          // column maxima (eight sets) as order-preserving integer
                          // encodings, maxed by every block (cat_cmax); from [64 + 448] on: each env chunk's still
                          // (no_move-active) envs as a 32-bit mask (cat_cstill)
  // device diagnostic word (handle-owned, read and cleared by h12env_check): bit 0 = a self-contact wait for the
  // contact wave's release ended at its bound (self_finish), so that inner step's self-contact wrenches may be partial;
  // bit 1 = a CaT wait for the last block's fold ended at its bound (cat_prob_inline)
  int* diag;
  int dbg_norel;          // test hook (H12_TEST_SKIP_SELF_RELEASE=1 at h12env_create): the contact wave never releases
};

// CaT constraint columns (ConstraintsCfg order, cat_env_cfg.py:336-427) and the scratch rows after them
constexpr int C_COL0[H12_NCSTR + 1] = {0, 1, 13, 25, 37, 39, 51, 52, 53, 54, 56};
constexpr int CAT_ROW_NOMOVE = H12_NCSTR_COLS;      // 1 if all |cmd| < no_move deadzone
constexpr int CAT_ROW_EPLEN = H12_NCSTR_COLS + 1;   // episode length before the reset of this step
constexpr int CAT_ROWS = H12_NCSTR_COLS + 2;
static_assert(C_COL0[H12_NCSTR] == H12_NCSTR_COLS, "constraint columns");
constexpr float CAT_NEG = -3.0e38f;  // "no value" in the column maxima (finite: device code is finite-math)
static_assert(sizeof(KParams) < 1024, "kernarg budget");

struct Workspace {
  float* F;    // [H12_NF_FLOAT][n]
  int32_t* I;  // [H12_NF_INT][n]
  int n;
};

enum { ST_RESET = 1, ST_CMD = 2, ST_OBS = 3, ST_PUSH = 4 };

// joint-angle sign of leg link k in the lane's frame (x / z joints flip under the y-mirror)
H12_DEV float jsign(int k, float sg) { return AX[k] == 1 ? 1.f : sg; }
// soft joint limits (ArticulationCfg.soft_joint_pos_limit_factor) in the left-leg frame
H12_DEV float soft_lo(const KParams& P, int k) {
  return 0.5f * (h12m::QLO[k] + h12m::QHI[k]) - 0.5f * (h12m::QHI[k] - h12m::QLO[k]) * P.soft_f;
}
H12_DEV float soft_hi(const KParams& P, int k) {
  return 0.5f * (h12m::QLO[k] + h12m::QHI[k]) + 0.5f * (h12m::QHI[k] - h12m::QLO[k]) * P.soft_f;
}
// spatial sign of the y-mirror for component i of a motion / force 6-vector (ang x,y,z, lin x,y,z)
H12_DEV float s6(int i, float sg) { return (i % 2 == 0) ? sg : 1.f; }

// Heightfield ground (real coordinates): height at (x, y) and its slope (dh/dx, dh/dy) on the
// triangle mesh isaaclab.terrains.utils.convert_height_field_to_mesh builds (cell (ix, iy) split along
// its (ix, iy) -> (ix+1, iy+1) diagonal).  Outside the grid the edge cells extend (flat border).
H12_DEV float ground(const KParams& P, float x, float y, float& gx, float& gy) {
  float u = fminf(fmaxf((x - P.t_x0) * P.t_inv_hs, 0.f), (float)(P.t_nx - 1) - 1e-3f);
  float v = fminf(fmaxf((y - P.t_y0) * P.t_inv_hs, 0.f), (float)(P.t_ny - 1) - 1e-3f);
  int ix = (int)u, iy = (int)v;
  float fu = u - (float)ix, fv = v - (float)iy;
  const float* hp = P.t_h + (size_t)ix * P.t_ny + iy;
  float h00 = hp[0], h01 = hp[1], h10 = hp[P.t_ny], h11 = hp[P.t_ny + 1];
  float a, b;
  if (fv >= fu) { a = h11 - h01; b = h01 - h00; }  // triangle (00, 11, 01)
  else { a = h10 - h00; b = h11 - h10; }           // triangle (00, 10, 11)
  gx = a * P.t_inv_hs;
  gy = b * P.t_inv_hs;
  return h00 + fu * a + fv * b;
}

// The same ground at the env-local point (xl, yl) (real axes) of an env whose origin is org: the contact
// geometry runs in env-local coordinates (|x| of a few m) and only the per-env cell base (org - x0) / hs is
// formed at the terrain's magnitude -- its rounding is one rigid shift shared by every contact point of the
// env, where world coordinates (up to ~100 m on the C5 terrain, fp32 ulp 8e-6 m) would round each point
// independently (independent sub-10-micron errors on stiff contacts).  Returns the height relative to org.z.
H12_DEV float ground_local(const KParams& P, const float* org, float xl, float yl, float& gx, float& gy) {
  const float cu = (org[0] - P.t_x0) * P.t_inv_hs, cv = (org[1] - P.t_y0) * P.t_inv_hs;
  const float iu0 = floorf(cu), iv0 = floorf(cv);
  const float u = (cu - iu0) + xl * P.t_inv_hs, v = (cv - iv0) + yl * P.t_inv_hs;
  const float fu0 = floorf(u), fv0 = floorf(v);
  int ix = (int)iu0 + (int)fu0, iy = (int)iv0 + (int)fv0;
  float fu = u - fu0, fv = v - fv0;
  // clamp to [0, n - 1 - 1e-3] in cell units as ground() does (flat border outside the grid)
  if (ix < 0) { ix = 0; fu = 0.f; }
  if (ix > P.t_nx - 2) { ix = P.t_nx - 2; fu = 1.f - 1e-3f; }
  if (iy < 0) { iy = 0; fv = 0.f; }
  if (iy > P.t_ny - 2) { iy = P.t_ny - 2; fv = 1.f - 1e-3f; }
  const float* hp = P.t_h + (size_t)ix * P.t_ny + iy;
  float h00 = hp[0], h01 = hp[1], h10 = hp[P.t_ny], h11 = hp[P.t_ny + 1];
  float a, b;
  if (fv >= fu) { a = h11 - h01; b = h01 - h00; }  // triangle (00, 11, 01)
  else { a = h10 - h00; b = h11 - h10; }           // triangle (00, 10, 11)
  gx = a * P.t_inv_hs;
  gy = b * P.t_inv_hs;
  return (h00 - org[2]) + fu * a + fv * b;
}

// ------------------------------------------------------------------ per-lane simulation state
struct Base {               // shared floating base, REAL coordinates (identical in both lanes)
  float pos[3], quat[4], vlin[3], wang[3];
};
// A diverged floating base (round 6): any component of the base's angular velocity above 200 rad/s or of its linear
// velocity above 50 m/s, or not finite, terminates the episode like an illegal contact (the env resets in the same
// step).  The penalty contacts can blow up (a base spinning at 100+ rad/s for a few steps, then 1e5 rad/s and NaN in
// a random-action Rsl / CaT run at 8192 envs; PhysX's contact solver does not); IsaacLab has no such term -- DESIGN.md
// section 9.  Integer compares on the magnitudes' bits: NaN / inf sort above every finite threshold, and no
// finite-math assumption can fold them away.  The oracle applies the same rule (orc_mdp_terms).
constexpr float H12_DIV_W = 200.f, H12_DIV_V = 50.f;
template <typename B>
H12_DEV bool base_diverged(const B& b) {
  bool d = false;
#pragma unroll
  for (int a = 0; a < 3; ++a)
    d = d || (__float_as_uint(b.wang[a]) & 0x7fffffffu) > __float_as_uint(H12_DIV_W) ||
        (__float_as_uint(b.vlin[a]) & 0x7fffffffu) > __float_as_uint(H12_DIV_V);
  return d;
}
struct Leg {                // this lane's leg in the lane frame (mirrored for the right leg)
  float q[NL], qd[NL];
  float anc[H12_NFOOT_PTS][2];
  int cmask;                // 4 bits: sole sphere (lane-frame index) in contact
  float mus, mud;           // sole Coulomb coefficients (per env and foot, or the config's)
  float dmass;              // mass added at the torso COM (lane 0 applies it)
};
struct Forces {             // net contact force on this lane's bodies (body coords; only norms are used), summed
  float foot[3], knee[3], torso[3];
};

// Added point inertia of an implicit contact at body point p: mass tensor M = beta I + gamma u u^T (body
// coords, u = the ground normal in body coords) -> C += M, B += [p]x M, A += -[p]x M [p]x
// (= beta (|p|^2 I - p p^T) + gamma w w^T with w = p x u).
H12_DEV void ai_add_contact(AInertia& I, const float* p, const float* u, float beta, float gamma) {
  float w[3];
  cross(p, u, w);
  const float gu[3] = {gamma * u[0], gamma * u[1], gamma * u[2]};
  const float gw[3] = {gamma * w[0], gamma * w[1], gamma * w[2]};
  I.C[0] += beta + gu[0] * u[0]; I.C[1] += beta + gu[1] * u[1]; I.C[2] += beta + gu[2] * u[2];
  I.C[3] += gu[0] * u[1]; I.C[4] += gu[0] * u[2]; I.C[5] += gu[1] * u[2];
  I.B[0][1] -= beta * p[2]; I.B[0][2] += beta * p[1];
  I.B[1][0] += beta * p[2]; I.B[1][2] -= beta * p[0];
  I.B[2][0] -= beta * p[1]; I.B[2][1] += beta * p[0];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) I.B[i][j] += gw[i] * u[j];
  const float p2 = p[0] * p[0] + p[1] * p[1] + p[2] * p[2];
  I.A[0] += beta * (p2 - p[0] * p[0]) + gw[0] * w[0];
  I.A[1] += beta * (p2 - p[1] * p[1]) + gw[1] * w[1];
  I.A[2] += beta * (p2 - p[2] * p[2]) + gw[2] * w[2];
  I.A[3] += gw[0] * w[1] - beta * p[0] * p[1];
  I.A[4] += gw[0] * w[2] - beta * p[0] * p[2];
  I.A[5] += gw[1] * w[2] - beta * p[1] * p[2];
}

// implicit-contact linearisation of one active contact (zero when P.impl == 0 or out of contact)
struct ImplC {
  float beta, gamma, u[3];
};
// implicit part of a contact's force, -M a'_p (body coords): a = the body's spatial acceleration in the
// gravity-shifted frame of the solve, p the contact point, M = beta I + gamma u u^T (oracle implicit_report)
H12_DEV void impl_force(const float* a, const float* p, const float* u, float beta, float gamma, float* f) {
  float ap[3];
  cross(a, p, ap);
  ap[0] += a[3]; ap[1] += a[4]; ap[2] += a[5];
  const float gn = gamma * (u[0] * ap[0] + u[1] * ap[1] + u[2] * ap[2]);
  f[0] -= beta * ap[0] + gn * u[0];
  f[1] -= beta * ap[1] + gn * u[1];
  f[2] -= beta * ap[2] + gn * u[2];
}

// one penalty contact (sphere centre pl in body coords, body world pose Rb/pb, body spatial velocity
// vb in body coords); adds the body-frame spatial force into f[6]; anchored stiction for sole spheres
// sg: the lane's mirror sign (the heightfield is looked up at the real y = sg * y); org: the env origin (real
// axes; positions are env-local on terrain, see ground_local); mus / mud: Coulomb
// coefficients of this contact (per-env sole friction or the config's).  With P.impl, ic receives the
// added point inertia of the contact (oracle contact_point) and f the force that cancels its weight
// under the gravity-as-base-acceleration formulation.  EXPL: the force only (its implicit part -- the added point
// inertia and its weight -- left out; the torso face's secondary corners, torso_face).
template <bool ANCHOR, bool TERRAIN, bool EXPL = false>
H12_DEV bool contact_sphere(const KParams& P, const float Rb[3][3], const float* pb, const float* vb,
                            const float* pl, float rad, float* f, float* fw, float* anc, bool was_in, float sg,
                            const float* org, float mus, float mud, ImplC& ic, bool expl_rt = false) {
  ic.beta = 0.f;
  ic.gamma = 0.f;
  float xw[3];
  mv(Rb, pl, xw);
  xw[0] += pb[0]; xw[1] += pb[1]; xw[2] += pb[2];
  float nrm[3] = {0.f, 0.f, 1.f}, depth;
  if constexpr (TERRAIN) {  // unit normal (-h_x, -h_y, 1)/|.| of the ground triangle
    float gx, gy;
    float hg = ground_local(P, org, xw[0], sg * xw[1], gx, gy);
    float in = __builtin_amdgcn_rsqf(1.f + gx * gx + gy * gy);
    nrm[0] = -gx * in; nrm[1] = -sg * gy * in; nrm[2] = in;
    depth = rad - (xw[2] - hg) * in;
  } else {
    depth = rad - xw[2];
  }
  float vl[3];
  cross(vb, pl, vl);
  vl[0] += vb[3]; vl[1] += vb[4]; vl[2] += vb[5];
  float vw[3];
  mv(Rb, vl, vw);
  float vn = TERRAIN ? nrm[0] * vw[0] + nrm[1] * vw[1] + nrm[2] * vw[2] : vw[2];
  // active when the point is predicted below the ground at the end of the step (implicit: depth - h vn; oracle
  // contact_point), so a point arriving at speed is caught within the step instead of one step deep
  if (!(depth - (P.impl ? P.h * vn : 0.f) > 0.f)) return false;
  // a sole contact that opens with a penetration is pushed out at most at PhysX's max_depenetration_velocity
  // (elastic term capped at h v_max); a persistent one carries any load (oracle contact_point)
  float fn = P.ck * ((ANCHOR && !was_in) ? fminf(depth, P.dcap) : depth) - P.cc * vn;
  if (!(fn > 0.f)) return false;
  float ft0, ft1;
  bool stick;
  if constexpr (ANCHOR) {
    float ax = was_in ? anc[0] : xw[0], ay = was_in ? anc[1] : xw[1];
    ft0 = -P.fk * (xw[0] - ax) - P.fc * vw[0];
    ft1 = -P.fk * (xw[1] - ay) - P.fc * vw[1];
    float ftn2 = ft0 * ft0 + ft1 * ft1, cap = mus * fn;
    stick = !(ftn2 > cap * cap);
    if (!stick) {
      float sc = mud * fn * __builtin_amdgcn_rsqf(ftn2);
      ft0 *= sc;
      ft1 *= sc;
      float ik = frcp(P.fk);
      ax = xw[0] + ft0 * ik;
      ay = xw[1] + ft1 * ik;
    }
    anc[0] = ax;
    anc[1] = ay;
  } else {
    ft0 = -P.fc_v * vw[0];
    ft1 = -P.fc_v * vw[1];
    float ftn2 = ft0 * ft0 + ft1 * ft1, cap = mud * fn;
    stick = !(ftn2 > cap * cap);
    if (!stick) { float sc = cap * __builtin_amdgcn_rsqf(ftn2); ft0 *= sc; ft1 *= sc; }
  }
  float Fw[3] = {ft0, ft1, fn}, fl[3], nl[3];
  if constexpr (TERRAIN) { Fw[0] += fn * nrm[0]; Fw[1] += fn * nrm[1]; Fw[2] = fn * nrm[2]; }
  if (P.impl && !EXPL && !expl_rt) {  // expl_rt: EXPL decided per lane (helper_torso's split corners)
    const float h = P.h;
    const float alpha = h * P.cc;
    const float beta = stick ? h * (ANCHOR ? P.fc : P.fc_v) : 0.f;
    ic.beta = beta;
    ic.gamma = alpha - beta;
    mtv(Rb, nrm, ic.u);
    // g Mw e_z = g (beta e_z + gamma n n_z)
    const float gb = P.g * beta, gg = P.g * ic.gamma * nrm[2];
    Fw[0] += gg * nrm[0]; Fw[1] += gg * nrm[1]; Fw[2] += gb + gg * nrm[2];
  }
  mtv(Rb, Fw, fl);
  cross(pl, fl, nl);
  f[0] += nl[0]; f[1] += nl[1]; f[2] += nl[2];
  f[3] += fl[0]; f[4] += fl[1]; f[5] += fl[2];
  fw[0] += fl[0]; fw[1] += fl[1]; fw[2] += fl[2];  // reported in body coords (only its norm is used)
  return true;
}

// The rotation increment r = (cos a, w sin(a) / |w|), a = |w| h / 2, as Taylor polynomials in a^2 (round 6): the
// hardware sine of these small angles (1e-5 .. 0.05) is +3.7 ulp high on average (profiles/r6/r6d_hw_math_bias.txt),
// a signed error that turned every orientation increment 3e-7 (relative) too large; the series is exact to fp32 for
// a <= 0.5 (|w| <= 200 rad/s at h = 5 ms; the truncation error there is 2.4e-11 in sin a / a, 2.7e-10 in cos a) and
// needs no square root or reciprocal.  (Far beyond that range -- a diverging state -- the polynomials can overflow; such
// a base is terminated by base_diverged at the end of the env step.)  w = 0 leaves q as it is (the oracle's rule)
H12_DEV void quat_integrate(float* q, const float* w, float h) {
  const float w2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
  if (w2 > 0.f) {
    const float a2 = w2 * (0.25f * h * h);
    // sin(a) / a and cos(a) to a^8
    const float sa = __builtin_fmaf(a2, __builtin_fmaf(a2, __builtin_fmaf(a2, __builtin_fmaf(a2, 1.f / 362880.f,
                              -1.f / 5040.f), 1.f / 120.f), -1.f / 6.f), 1.f);
    const float ch = __builtin_fmaf(a2, __builtin_fmaf(a2, __builtin_fmaf(a2, __builtin_fmaf(a2, 1.f / 40320.f,
                              -1.f / 720.f), 1.f / 24.f), -0.5f), 1.f);
    const float sh = sa * (0.5f * h);
    float r[4] = {ch, w[0] * sh, w[1] * sh, w[2] * sh};
    float o[4] = {q[0] * r[0] - q[1] * r[1] - q[2] * r[2] - q[3] * r[3],
                  q[0] * r[1] + q[1] * r[0] + q[2] * r[3] - q[3] * r[2],
                  q[0] * r[2] - q[1] * r[3] + q[2] * r[0] + q[3] * r[1],
                  q[0] * r[3] + q[1] * r[2] - q[2] * r[1] + q[3] * r[0]};
    float inv = __builtin_amdgcn_rsqf(o[0] * o[0] + o[1] * o[1] + o[2] * o[2] + o[3] * o[3]);
    q[0] = o[0] * inv; q[1] = o[1] * inv; q[2] = o[2] * inv; q[3] = o[3] * inv;
  }
}

// Solve the 6x6 SPD system I x = b (LDL^T, fully unrolled)
H12_DEV void solve6(const AInertia& I, const float* b, float* x) {
  float M[6][6];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      M[i][j] = sget(I.A, i, j);
      M[i][3 + j] = I.B[i][j];
      M[3 + i][j] = I.B[j][i];
      M[3 + i][3 + j] = sget(I.C, i, j);
    }
  // T[i][j] = L[i][j] D[j] is the un-normalised column entry itself: one fma per term
  float L[6][6], T[6][6], Dinv[6];
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    float d = M[j][j];
#pragma unroll
    for (int k = 0; k < j; ++k) d -= L[j][k] * T[j][k];
    Dinv[j] = frcp(d);
#pragma unroll
    for (int i = j + 1; i < 6; ++i) {
      float t = M[i][j];
#pragma unroll
      for (int k = 0; k < j; ++k) t -= L[i][k] * T[j][k];
      T[i][j] = t;
      L[i][j] = t * Dinv[j];
    }
  }
  float y[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    float t = b[i];
#pragma unroll
    for (int k = 0; k < i; ++k) t -= L[i][k] * y[k];
    y[i] = t;
  }
#pragma unroll
  for (int i = 5; i >= 0; --i) {
    float t = y[i] * Dinv[i];
#pragma unroll
    for (int k = i + 1; k < 6; ++k) t -= L[k][i] * x[k];
    x[i] = t;
  }
}

// velocity-product acceleration c = v x (e_A qd)
template <int A>
H12_DEV void vprod(const float* v, float qd, float* c) {
  float e[3] = {0.f, 0.f, 0.f};
  e[A] = qd;
  cross(v, e, c);
  cross(v + 3, e, c + 3);
}
// rigid-body bias force v x* (I v) of leg link LINK (I = (Ibar, m c, m) in link coords)
template <int LINK>
H12_DEV void bias(const float* v, float* p) {
  const float* Ibar = h12m::IBAR[LINK];
  const float* mc = h12m::MC[LINK];
  const float m = h12m::M[LINK];
  const float* w = v;
  const float* vl = v + 3;
  float n[3], f[3], a1[3], a2[3];
  for (int i = 0; i < 3; ++i) n[i] = sget(Ibar, i, 0) * w[0] + sget(Ibar, i, 1) * w[1] + sget(Ibar, i, 2) * w[2];
  cross(mc, vl, a1);
  n[0] += a1[0]; n[1] += a1[1]; n[2] += a1[2];
  cross(mc, w, a2);
  f[0] = m * vl[0] - a2[0]; f[1] = m * vl[1] - a2[1]; f[2] = m * vl[2] - a2[2];
  float x1[3], x2[3], x3[3];
  cross(w, n, x1);
  cross(vl, f, x2);
  cross(w, f, x3);
  p[0] = x1[0] + x2[0]; p[1] = x1[1] + x2[1]; p[2] = x1[2] + x2[2];
  p[3] = x3[0]; p[4] = x3[1]; p[5] = x3[2];
}

// ---- ABA pass 1 for leg link LINK: spatial velocity v[LINK] from the parent's vp, world pose
// the spatial velocity alone
template <int LINK>
H12_DEV void link_vel(const Leg& lg, const float (&cs)[NL][2], const float* vp, float (&v)[NL][6]) {
  constexpr int A = AX[LINK];
  const float* r = h12m::R[LINK];
  const float c = cs[LINK][0], s = cs[LINK][1];
  float t[3];
  cross(r, vp, t);
  float lin[3] = {vp[3] - t[0], vp[4] - t[1], vp[5] - t[2]};
  rotT<A>(c, s, vp, v[LINK]);
  rotT<A>(c, s, lin, v[LINK] + 3);
  v[LINK][A] += lg.qd[LINK];
}
template <int LINK>
H12_DEV void link_pass1(const Leg& lg, float (&cs)[NL][2], const float* vp, float (&v)[NL][6], float (&R)[3][3],
                        float* p) {
  constexpr int A = AX[LINK];
  const float* r = h12m::R[LINK];
  float s, c;
  fsincos(lg.q[LINK], &s, &c);
  cs[LINK][0] = c;
  cs[LINK][1] = s;
  link_vel<LINK>(lg, cs, vp, v);
  float Rr[3];
  mv(R, r, Rr);
  p[0] += Rr[0]; p[1] += Rr[1]; p[2] += Rr[2];
  rmul_axis<A>(R, c, s);
}

// ---- ABA pass 2 for leg link LINK (leaf -> root), split in two chains: the articulated-inertia chain
// (link_ia: depends on the joint angles, the link velocities and the implicit contact / limit inertias only) and
// the bias-force chain (link_p: linear in the applied forces).  The split lets the forces of the step --
// actuator + limit torques, rigid-body bias forces, self-contact wrenches -- arrive after the inertia chain
// (step_kernel computes them in the block's helper wave meanwhile).
// link_ia: on entry IA is the articulated inertia of LINK in its own frame; on exit that of the parent (rigid part
// included; for LINK == 0 the leg's contribution to the base, at the base origin).  Keeps U, 1/D and
// Ic = Ia c (c = the velocity-product acceleration) for link_p and pass 3.
// AV (step_kernel's physics wave, round 5): the velocity-product accelerations are carried by the rigid-body bias forces
// instead (b_i = I_i a^v_i + v_i x* I_i v_i, a^v the accelerations of the links at zero joint and base acceleration,
// link_av; computed by the helper / contact waves), so the articulated-body recursion runs with c = 0: no Ic = Ia c
// here, no c in link_p / link_pass3 (exact algebra: the accelerations a~ = a - a^v obey a~_i = X_i a~_parent + S qdd_i;
// DESIGN.md section 2)
// AV: U kept as (angular, linear) pairs U[LINK][k] = (U_k, U_3+k) (f32x2 [NL][3]) for the packed link_p_pk /
// link_pass3_pk; otherwise float [NL][6]
template <int LINK, bool AV = false, typename UT>
H12_DEV void link_ia(const KParams& P, const Leg& lg, const float (&cs)[NL][2], const float (&v)[NL][6],
                     const ImplC& ick, float knee_pz, const float* dl, AInertia& IA, UT& U,
                     float (&Dinv)[NL], float (&Ic)[NL][6], float h) {
  constexpr int A = AX[LINK];
  float Ua[3] = {sget(IA.A, 0, A), sget(IA.A, 1, A), sget(IA.A, 2, A)};
  float Ul[3] = {IA.B[A][0], IA.B[A][1], IA.B[A][2]};
  float D = IA.A[A] + h12m::ARM[LINK] + h * P.dimpl[LINK] + dl[LINK];
  float di = frcp(D);
  Dinv[LINK] = di;
  // Ia = IA - U U^T / D; the A and C blocks share the index pattern: packed (A, C) pairs
  const f32x2 u2[3] = {pk2(Ua[0], Ul[0]), pk2(Ua[1], Ul[1]), pk2(Ua[2], Ul[2])};
  if constexpr (AV) {
    U[LINK][0] = u2[0]; U[LINK][1] = u2[1]; U[LINK][2] = u2[2];
  } else {
    U[LINK][0] = Ua[0]; U[LINK][1] = Ua[1]; U[LINK][2] = Ua[2];
    U[LINK][3] = Ul[0]; U[LINK][4] = Ul[1]; U[LINK][5] = Ul[2];
  }
  const f32x2 ud2[3] = {u2[0] * di, u2[1] * di, u2[2] * di};
  constexpr int SI[6] = {0, 1, 2, 0, 0, 1}, SJ[6] = {0, 1, 2, 1, 2, 2};
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    f32x2 ac = pk2(IA.A[k], IA.C[k]);
    ac -= u2[SI[k]] * ud2[SJ[k]];
    IA.A[k] = ac.x;
    IA.C[k] = ac.y;
  }
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) IA.B[i][j] -= Ua[i] * ud2[j].y;
  if constexpr (!AV) {
    float cb[6];
    vprod<A>(v[LINK], lg.qd[LINK], cb);
    ai_mul(IA, cb, Ic[LINK]);
  }
  // to the parent: rotate into parent axes, then shift the reference point by r
  ai_rotate<A>(IA, cs[LINK][0], cs[LINK][1]);
  ai_shift(IA, h12m::R[LINK]);
  if constexpr (LINK > 0) {
    AInertia Rg;
    ai_rigid(Rg, h12m::IBAR[LINK - 1], h12m::MC[LINK - 1], h12m::M[LINK - 1]);
    ai_add(IA, Rg);
    if constexpr (LINK - 1 == 3) {
      if (P.impl && ick.gamma + ick.beta > 0.f) {
        const float pk[3] = {0.f, 0.f, knee_pz};
        ai_add_contact(IA, pk, ick.u, ick.beta, ick.gamma);
      }
    }
  }
}
// link_p: on entry pAcc is the bias force of LINK (own frame, applied forces subtracted); on exit the parent's
// (its rigid-body bias force pbias[LINK - 1] included, the knee's external wrench subtracted), u[LINK] set.
template <int LINK, bool AV = false>
H12_DEV void link_p(const float (&cs)[NL][2], const float (&U)[NL][6], const float (&Dinv)[NL], const float (&Ic)[NL][6],
                    const float* tau, const float (&pbias)[NL][6], const float* fext_knee, float* pAcc, float (&u)[NL]) {
  constexpr int A = AX[LINK];
  const float uu = tau[LINK] - pAcc[A];
  u[LINK] = uu;
  const float ud = uu * Dinv[LINK];
  float pa[6];
  for (int i = 0; i < 6; ++i) pa[i] = AV ? pAcc[i] + U[LINK][i] * ud : pAcc[i] + Ic[LINK][i] + U[LINK][i] * ud;
  const float c = cs[LINK][0], s = cs[LINK][1];
  const float* r = h12m::R[LINK];
  float nr[3], fr[3], rf[3];
  rot<A>(c, s, pa, nr);
  rot<A>(c, s, pa + 3, fr);
  cross(r, fr, rf);
  pAcc[0] = nr[0] + rf[0]; pAcc[1] = nr[1] + rf[1]; pAcc[2] = nr[2] + rf[2];
  pAcc[3] = fr[0]; pAcc[4] = fr[1]; pAcc[5] = fr[2];
  if constexpr (LINK > 0) {
    for (int i = 0; i < 6; ++i) pAcc[i] += pbias[LINK - 1][i];
    if constexpr (LINK - 1 == 3)
      for (int i = 0; i < 6; ++i) pAcc[i] -= fext_knee[i];
  }
}

// rot<A> of (angular, linear) pairs: both halves of a spatial vector turn alike, one packed op per pair of scalar ones
template <int A>
H12_DEV void rot_pk(float c, float s, const f32x2* in, f32x2* out) {
  const f32x2 x = in[0], y = in[1], z = in[2];
  if constexpr (A == 0) { out[0] = x; out[1] = c * y - s * z; out[2] = s * y + c * z; }
  else if constexpr (A == 1) { out[0] = c * x + s * z; out[1] = y; out[2] = -s * x + c * z; }
  else { out[0] = c * x - s * y; out[1] = s * x + c * y; out[2] = z; }
}
// link_p of the AV form on (angular, linear) pairs p[k] = (pAcc_k, pAcc_3+k), U as pairs (link_ia<.., true>)
template <int LINK>
H12_DEV void link_p_pk(const float (&cs)[NL][2], const f32x2 (&U)[NL][3], const float (&Dinv)[NL], const float* tau,
                       const f32x2 (&pb)[NL][3], f32x2 (&p)[3], float (&u)[NL]) {
  constexpr int A = AX[LINK];
  const float uu = tau[LINK] - p[A].x;
  u[LINK] = uu;
  const float ud = uu * Dinv[LINK];
  f32x2 pa[3], q[3];
  for (int k = 0; k < 3; ++k) pa[k] = p[k] + U[LINK][k] * ud;
  rot_pk<A>(cs[LINK][0], cs[LINK][1], pa, q);
  const float* r = h12m::R[LINK];
  const float fr[3] = {q[0].y, q[1].y, q[2].y};
  float rf[3];
  cross(r, fr, rf);
  for (int k = 0; k < 3; ++k) p[k] = pk2(q[k].x + rf[k], q[k].y);
  if constexpr (LINK > 0)
    for (int k = 0; k < 3; ++k) p[k] += pb[LINK - 1][k];
}
// link_pass1 on pairs (leg_pass1: step_kernel's helper waves, whose pass 1 and contacts set barrier R1): the spatial
// velocity as (angular, linear) pairs (link_pass3_pk's transform, the joint rate for qdd), the world rotation's rows 0 / 1
// as column pairs C[j] = (R_0j, R_1j) with row 2 apart (R2), the position as (p01, p2): a joint rotation turns two
// columns, one packed op per pair of rows
template <int LINK, bool HWTRIG = false>
H12_DEV void link_pass1_pk(const Leg& lg, float (&cs)[NL][2], const f32x2* vp, f32x2 (&V)[NL][3], f32x2 (&C)[3],
                           float (&R2)[3], f32x2& p01, float& p2) {
  constexpr int A = AX[LINK], J = (A + 1) % 3, Q = (A + 2) % 3;
  const float* r = h12m::R[LINK];
  float s, c;
  if constexpr (HWTRIG) fsincos_hw(lg.q[LINK], &s, &c);  // the self-contact wave (fsincos_hw)
  else fsincos(lg.q[LINK], &s, &c);
  cs[LINK][0] = c;
  cs[LINK][1] = s;
  const float aw[3] = {vp[0].x, vp[1].x, vp[2].x};
  float t[3];
  cross(r, aw, t);
  f32x2 in[3];
  for (int k = 0; k < 3; ++k) in[k] = pk2(vp[k].x, vp[k].y - t[k]);
  rot_pk<A>(c, -s, in, V[LINK]);
  V[LINK][A].x += lg.qd[LINK];
  // the joint origin (the parent's rotation): p += R r, r sparse
  for (int k = 0; k < 3; ++k)
    if (r[k] != 0.f) {
      p01 += C[k] * r[k];
      p2 += R2[k] * r[k];
    }
  // R <- R R_A(q): columns J, Q turn (rotT<A> of every row)
  const f32x2 cj = C[J], cq = C[Q];
  C[J] = c * cj + s * cq;
  C[Q] = c * cq - s * cj;
  const float rj = R2[J], rq = R2[Q];
  R2[J] = c * rj + s * rq;
  R2[Q] = c * rq - s * rj;
}
// link_pass3 of the AV form on (angular, linear) pairs a[k] = (a_k, a_3+k)
template <int LINK>
H12_DEV void link_pass3_pk(const float (&cs)[NL][2], const f32x2 (&U)[NL][3], const float (&Dinv)[NL],
                           const float (&u)[NL], f32x2 (&a)[3], float* qdd) {
  constexpr int A = AX[LINK];
  const float* r = h12m::R[LINK];
  const float aw[3] = {a[0].x, a[1].x, a[2].x};
  float t[3];
  cross(r, aw, t);
  f32x2 in[3];
  for (int k = 0; k < 3; ++k) in[k] = pk2(a[k].x, a[k].y - t[k]);
  rot_pk<A>(cs[LINK][0], -cs[LINK][1], in, a);
  f32x2 ua = U[LINK][0] * a[0];
  ua += U[LINK][1] * a[1];
  ua += U[LINK][2] * a[2];
  const float x = (u[LINK] - (ua.x + ua.y)) * Dinv[LINK];
  qdd[LINK] = x;
  a[A].x += x;
}

// ---- ABA pass 3 for leg link LINK (root -> leaf)
template <int LINK, bool AV = false>
H12_DEV void link_pass3(const Leg& lg, const float (&cs)[NL][2], const float (&v)[NL][6], const float (&U)[NL][6],
                        const float (&Dinv)[NL], const float (&u)[NL], float* a, float* qdd) {
  constexpr int A = AX[LINK];
  const float* r = h12m::R[LINK];
  float c = cs[LINK][0], s = cs[LINK][1];
  float t[3];
  cross(r, a, t);
  float lin[3] = {a[3] - t[0], a[4] - t[1], a[5] - t[2]};
  float w[3], l[3];
  rotT<A>(c, s, a, w);
  rotT<A>(c, s, lin, l);
  if constexpr (AV) {
    a[0] = w[0]; a[1] = w[1]; a[2] = w[2];
    a[3] = l[0]; a[4] = l[1]; a[5] = l[2];
  } else {
    float cb[6];
    vprod<A>(v[LINK], lg.qd[LINK], cb);
    a[0] = w[0] + cb[0]; a[1] = w[1] + cb[1]; a[2] = w[2] + cb[2];
    a[3] = l[0] + cb[3]; a[4] = l[1] + cb[4]; a[5] = l[2] + cb[5];
  }
  float ua = 0.f;
  for (int i = 0; i < 6; ++i) ua += U[LINK][i] * a[i];
  float x = (u[LINK] - ua) * Dinv[LINK];
  qdd[LINK] = x;
  a[A] += x;
}

// ---- velocity-product accelerations a^v (round 5, the AV form of the ABA): the links' spatial accelerations when every
// joint and the base have zero acceleration, a^v_i = X_i a^v_parent + v_i x (e_A qd_i), a^v_base = 0 (link coords, lane
// frame).  av: on entry the parent's, on exit link LINK's.
template <int LINK>
H12_DEV void link_av(const Leg& lg, const float (&cs)[NL][2], const float (&v)[NL][6], float* av) {
  constexpr int A = AX[LINK];
  const float* r = h12m::R[LINK];
  const float c = cs[LINK][0], s = cs[LINK][1];
  float t[3];
  cross(r, av, t);
  float lin[3] = {av[3] - t[0], av[4] - t[1], av[5] - t[2]};
  float w[3], l[3], cb[6];
  rotT<A>(c, s, av, w);
  rotT<A>(c, s, lin, l);
  vprod<A>(v[LINK], lg.qd[LINK], cb);
  av[0] = w[0] + cb[0]; av[1] = w[1] + cb[1]; av[2] = w[2] + cb[2];
  av[3] = l[0] + cb[3]; av[4] = l[1] + cb[4]; av[5] = l[2] + cb[5];
}
// b += I_LINK a: the rigid inertia of leg link LINK (Ibar, m c, m; link origin, link coords) times a spatial acceleration
template <int LINK>
H12_DEV void rigid_mul_add(const float* a, float* b) {
  const float* Ibar = h12m::IBAR[LINK];
  const float* mc = h12m::MC[LINK];
  const float m = h12m::M[LINK];
  float x1[3], x2[3];
  cross(mc, a + 3, x1);
  cross(mc, a, x2);
  for (int i = 0; i < 3; ++i) {
    b[i] += sget(Ibar, i, 0) * a[0] + sget(Ibar, i, 1) * a[1] + sget(Ibar, i, 2) * a[2] + x1[i];
    b[3 + i] += m * a[3 + i] - x2[i];
  }
}
// b += M a at a body point p (the implicit contact's added point inertia M = beta I + gamma u u^T, body coords): the
// force M a_p at p (a_p = a_lin + a_ang x p) and its moment p x M a_p
H12_DEV void point_inertia_mul_add(const float* a, const float* p, const float* u, float beta, float gamma, float* b) {
  float ap[3];
  cross(a, p, ap);
  ap[0] += a[3]; ap[1] += a[4]; ap[2] += a[5];
  const float gn = gamma * (u[0] * ap[0] + u[1] * ap[1] + u[2] * ap[2]);
  const float f[3] = {beta * ap[0] + gn * u[0], beta * ap[1] + gn * u[1], beta * ap[2] + gn * u[2]};
  float n[3];
  cross(p, f, n);
  b[0] += n[0]; b[1] += n[1]; b[2] += n[2];
  b[3] += f[0]; b[4] += f[1]; b[5] += f[2];
}

// ---- flat ground: the 4 sole spheres of the foot in one pass.  On a plane every sphere has the same ground
// normal (u = R^T e_z in foot coords), so the forces are summed in world axes (one rotation back for the
// force, one for the moment: sum_q p_q x R^T F_q = R^T sum_q (R p_q) x F_q) and the implicit point
// inertias M_q = beta_q I + gamma_q u u^T enter through their moments: sum beta, sum gamma, sum beta p,
// sum gamma p, sum beta (|p|^2 I - p p^T), sum gamma p p^T (the p_q are model constants).  Same contact law
// as contact_sphere<true, false> + ai_add_contact per sphere; only the summation order differs.
struct SoleSums {
  float sb, sg, pb[3], pg[3];  // sum beta, sum gamma, sum beta p, sum gamma p (foot coords)
};
constexpr float sole_j(int q, int k) {  // |p|^2 I - p p^T of sole sphere q, symmetric packing
  const float* f = h12m::FOOT[q];
  const float p2 = f[0] * f[0] + f[1] * f[1] + f[2] * f[2];
  return k < 3 ? p2 - f[k] * f[k] : -(k == 3 ? f[0] * f[1] : (k == 4 ? f[0] * f[2] : f[1] * f[2]));
}
constexpr float sole_pp(int q, int k) {  // p p^T, symmetric packing
  const float* f = h12m::FOOT[q];
  return k < 3 ? f[k] * f[k] : (k == 3 ? f[0] * f[1] : (k == 4 ? f[0] * f[2] : f[1] * f[2]));
}

// Q0..Q1: the sole spheres this call evaluates (step_kernel splits them over two waves; the single-wave step all 4)
template <int Q0 = 0, int Q1 = H12_NFOOT_PTS>
H12_DEV void sole_contacts_flat(const KParams& P, const float R[3][3], const float* pf, const float* vb, Leg& lg,
                                AInertia& IA, float* pAcc, float* fw, SoleSums& ss) {
  float ww[3], v0[3];  // foot angular velocity and origin velocity, world axes
  mv(R, vb, ww);
  mv(R, vb + 3, v0);
  float F[3] = {0.f, 0.f, 0.f}, T[3] = {0.f, 0.f, 0.f};
  float J[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, G[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  ss = {};
  int nmask = 0;
  const float alpha = P.h * P.cc, hb = P.h * P.fc;
#pragma unroll
  for (int q = Q0; q < Q1; ++q) {
    float r[3];
    mv(R, h12m::FOOT[q], r);
    const float depth = h12m::FOOT_R - (r[2] + pf[2]);
    float vw[3];
    cross(ww, r, vw);
    vw[0] += v0[0]; vw[1] += v0[1]; vw[2] += v0[2];
    // branch-free (round 5): an inactive sphere contributes zeros -- the early-out branches made the compiler re-zero
    // the ~26 accumulators on every skip path (~95 v_mov per call); the same float operations on the active ones
    const bool was = (lg.cmask >> q) & 1;
    // an opening contact is pushed out at most at max_depenetration_velocity (contact_sphere)
    const float fn0 = P.ck * (was ? depth : fminf(depth, P.dcap)) - P.cc * vw[2];
    // active when predicted below the ground at the end of the step (contact_sphere) and pushing
    const bool on = (depth - (P.impl ? P.h * vw[2] : 0.f) > 0.f) && fn0 > 0.f;
    const float fn = on ? fn0 : 0.f;
    const float x0 = r[0] + pf[0], x1 = r[1] + pf[1];
    float ax = was ? lg.anc[q][0] : x0, ay = was ? lg.anc[q][1] : x1;
    float ft0 = -P.fk * (x0 - ax) - P.fc * vw[0];
    float ft1 = -P.fk * (x1 - ay) - P.fc * vw[1];
    const float ftn2 = ft0 * ft0 + ft1 * ft1, cap = lg.mus * fn;
    const bool stick = !(ftn2 > cap * cap);
    {
      const float sc = lg.mud * fn * __builtin_amdgcn_rsqf(ftn2);
      const float ik = frcp(P.fk);
      const float s0 = ft0 * sc, s1 = ft1 * sc;
      ax = stick ? ax : x0 + s0 * ik;
      ay = stick ? ay : x1 + s1 * ik;
      ft0 = on ? (stick ? ft0 : s0) : 0.f;
      ft1 = on ? (stick ? ft1 : s1) : 0.f;
    }
    lg.anc[q][0] = on ? ax : lg.anc[q][0];
    lg.anc[q][1] = on ? ay : lg.anc[q][1];
    nmask |= (on ? 1 : 0) << q;
    float Fw[3] = {ft0, ft1, fn};
    // the implicit terms unconditionally, zero without them (beta = gamma = 0): a P.impl branch left every
    // accumulator (the added inertia, the sums) zero-initialised ahead of it (~40 v_mov in the helper waves)
    {  // g M_w e_z = g (beta + gamma) e_z on a plane
      const bool im = P.impl && on;
      const float beta = (im && stick) ? hb : 0.f, gam = im ? alpha - beta : 0.f;
      Fw[2] += im ? P.g * alpha : 0.f;
      ss.sb += beta;
      ss.sg += gam;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        ss.pb[i] += beta * h12m::FOOT[q][i];
        ss.pg[i] += gam * h12m::FOOT[q][i];
      }
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        J[k] += beta * sole_j(q, k);
        G[k] += gam * sole_pp(q, k);
      }
    }
    float rf[3];
    cross(r, Fw, rf);
    F[0] += Fw[0]; F[1] += Fw[1]; F[2] += Fw[2];
    T[0] += rf[0]; T[1] += rf[1]; T[2] += rf[2];
  }
  constexpr int OWN = ((1 << Q1) - 1) & ~((1 << Q0) - 1);
  lg.cmask = (lg.cmask & ~OWN) | nmask;
  float fl[3], tl[3];
  mtv(R, F, fl);
  mtv(R, T, tl);
  pAcc[0] -= tl[0]; pAcc[1] -= tl[1]; pAcc[2] -= tl[2];
  pAcc[3] -= fl[0]; pAcc[4] -= fl[1]; pAcc[5] -= fl[2];
  fw[0] += fl[0]; fw[1] += fl[1]; fw[2] += fl[2];
  {  // zero without the implicit terms (the sums are)
    const float u[3] = {R[2][0], R[2][1], R[2][2]};
    // C += sum beta I + sum gamma u u^T
    const float gu[3] = {ss.sg * u[0], ss.sg * u[1], ss.sg * u[2]};
    IA.C[0] += ss.sb + gu[0] * u[0]; IA.C[1] += ss.sb + gu[1] * u[1]; IA.C[2] += ss.sb + gu[2] * u[2];
    IA.C[3] += gu[0] * u[1]; IA.C[4] += gu[0] * u[2]; IA.C[5] += gu[1] * u[2];
    // B += [sum beta p]x + (sum gamma p x u) u^T
    IA.B[0][1] -= ss.pb[2]; IA.B[0][2] += ss.pb[1];
    IA.B[1][0] += ss.pb[2]; IA.B[1][2] -= ss.pb[0];
    IA.B[2][0] -= ss.pb[1]; IA.B[2][1] += ss.pb[0];
    float c[3];
    cross(ss.pg, u, c);
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) IA.B[i][j] += c[i] * u[j];
    // A += sum beta (|p|^2 I - p p^T) + [u]x G [u]x^T, G = sum gamma p p^T ((p x u)(p x u)^T = [u]x p p^T [u]x^T)
    float Gf[3][3], Kx[3][3];
    sym_full(G, Gf);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      Kx[0][j] = -u[2] * Gf[1][j] + u[1] * Gf[2][j];
      Kx[1][j] = u[2] * Gf[0][j] - u[0] * Gf[2][j];
      Kx[2][j] = -u[1] * Gf[0][j] + u[0] * Gf[1][j];
    }
    auto mx = [&](int i, int j) {
      return j == 0 ? -u[2] * Kx[i][1] + u[1] * Kx[i][2]
                    : (j == 1 ? u[2] * Kx[i][0] - u[0] * Kx[i][2] : -u[1] * Kx[i][0] + u[0] * Kx[i][1]);
    };
    IA.A[0] += J[0] + mx(0, 0); IA.A[1] += J[1] + mx(1, 1); IA.A[2] += J[2] + mx(2, 2);
    IA.A[3] += J[3] + mx(0, 1); IA.A[4] += J[4] + mx(0, 2); IA.A[5] += J[5] + mx(1, 2);
  }
}

// implicit part of the sole forces from the moments of SoleSums (sum over q of impl_force)
H12_DEV void sole_impl_force_flat(const float* a, const float R[3][3], const SoleSums& ss, float* f) {
  const float u[3] = {R[2][0], R[2][1], R[2][2]};
  float xb[3], xg[3];
  cross(a, ss.pb, xb);
  cross(a, ss.pg, xg);
  const float gn = u[0] * xg[0] + u[1] * xg[1] + u[2] * xg[2] + ss.sg * (u[0] * a[3] + u[1] * a[4] + u[2] * a[5]);
  f[0] -= xb[0] + ss.sb * a[3] + gn * u[0];
  f[1] -= xb[1] + ss.sb * a[4] + gn * u[1];
  f[2] -= xb[2] + ss.sb * a[5] + gn * u[2];
}

// ---- self-collision between the legs (oracle self_contacts; h12env_config.self_collision).  Capsules: the knee
// cylinder (KNEE0-KNEE1, KNEE_R) and the four sole rods (ROD, FOOT_R) of each leg; every left/right pair (25).
//  * broad phase, every physics step, split over the lane pair: a knee segment and a foot bounding capsule
//    (FB0-FB1, FB_R) per leg, four capsule tests (knee-knee, knee-foot x2, foot-foot), two per lane;
//  * narrow phase only in waves where some env has a candidate group, and COMPACTED across the wave: the
//    lanes stage their leg's capsules and body kinematics in LDS, then the 25 pair jobs of every candidate env
//    are spread over all 64 lanes (one pass for up to 2 such envs), each job adding its pair force and moment
//    to the two bodies' LDS accumulators with no-return LDS float atomics (one wave per block: order fixed
//    by the single wave's instruction stream), and each lane reads back its own knee / foot wrench.
// Real (un-mirrored) coordinates throughout; the pair force acts +F on the left body, -F on the right one.

// Contact points of two capsule axes p1-q1, p2-q2 (the oracle's seg_points): general pairs (sin^2 of the angle
// >= 1e-3) one closest point, with the normal from d1 x d2 when both parameters are interior (well-conditioned where
// the axes nearly intersect); nearly parallel pairs a line contact, two points at the ends of the overlap along the
// first segment with half weight each (one point, the nearest ends, without overlap).  Parameters only: the
// points are p + d s, and the caller loops over them.
struct SegPts {
  float d1[3], d2[3], s0, s1, t0, t1, ncx, ncy, ncz, w;
  int n;
  bool has_nc;
};
H12_DEV void seg_points(const float* p1, const float* q1, const float* p2, const float* q2, SegPts& o) {
  // branch-free (every field written once, from selects: per-branch stores let the compiler re-form the two
  // points into a scratch array)
  float r[3];
  for (int a = 0; a < 3; ++a) { o.d1[a] = q1[a] - p1[a]; o.d2[a] = q2[a] - p2[a]; r[a] = p1[a] - p2[a]; }
  const float A = dot3(o.d1, o.d1), E = dot3(o.d2, o.d2), F = dot3(o.d2, r), C = dot3(o.d1, r), B = dot3(o.d1, o.d2);
  const float den = A * E - B * B, iA = frcp(A), iE = frcp(E);
  const bool par = !(den > 1e-3f * A * E);
  // nearly parallel: segment 2's ends projected onto segment 1; the overlap [lo, hi]
  const float u0 = -C * iA, u1 = (B - C) * iA;
  const float lo = fmaxf(0.f, fminf(u0, u1)), hi = fminf(1.f, fmaxf(u0, u1));
  const bool line = par && hi > lo;
  // one point: the clamped closest-point construction (from the unconstrained s, or for parallel axes without
  // overlap from the middle of the empty overlap = the nearest ends)
  float s = par ? fminf(fmaxf(0.5f * (lo + hi), 0.f), 1.f) : fminf(fmaxf((B * F - C * E) * frcp(den), 0.f), 1.f);
  float t = (B * s + F) * iE;
  const bool tlo = t < 0.f, thi = t > 1.f;
  s = tlo ? fminf(fmaxf(u0, 0.f), 1.f) : (thi ? fminf(fmaxf(u1, 0.f), 1.f) : s);
  t = fminf(fmaxf(t, 0.f), 1.f);
  o.has_nc = !par && !tlo && !thi && s > 0.f && s < 1.f;
  float c[3];
  cross(o.d1, o.d2, c);
  const float cn = o.has_nc ? __builtin_amdgcn_rsqf(dot3(c, c)) : 0.f;
  o.ncx = c[0] * cn; o.ncy = c[1] * cn; o.ncz = c[2] * cn;
  o.n = line ? 2 : 1;
  o.w = line ? 0.5f : 1.f;
  o.s0 = line ? lo : s;
  o.t0 = line ? fminf(fmaxf((B * lo + F) * iE, 0.f), 1.f) : t;
  o.s1 = hi;
  o.t1 = fminf(fmaxf((B * hi + F) * iE, 0.f), 1.f);
}
// broad phase: true when the capsules' axes may come within rr.  The segment distance is Lipschitz in the first
// segment's parameter with constant |d1| sin(angle) (while the second's stays interior), so for nearly parallel
// axes the midpoint of the overlap bounds the minimum from below by half the overlap's length times that constant
H12_DEV bool capsules_near(const float* p1, const float* q1, const float* p2, const float* q2, float rr) {
  float d1[3], d2[3], r[3];
  for (int a = 0; a < 3; ++a) { d1[a] = q1[a] - p1[a]; d2[a] = q2[a] - p2[a]; r[a] = p1[a] - p2[a]; }
  const float A = dot3(d1, d1), E = dot3(d2, d2), F = dot3(d2, r), C = dot3(d1, r), B = dot3(d1, d2);
  // branch-free (both cases evaluated, then selected): the broad phase runs every inner step, and standing legs
  // (parallel knees) put both cases in most waves
  const float den = A * E - B * B, iA = frcp(A), iE = frcp(E);
  const bool gen = den > 1e-3f * A * E;
  const float sgen = fminf(fmaxf((B * F - C * E) * frcp(gen ? den : 1.f), 0.f), 1.f);
  const float t0 = -C * iA, t1 = (B - C) * iA;
  const float lo = fmaxf(0.f, fminf(t0, t1)), hi = fminf(1.f, fmaxf(t0, t1));
  const float spar = fminf(fmaxf(0.5f * (lo + hi), 0.f), 1.f);
  const float slack = gen ? 0.f : 0.5f * fmaxf(hi - lo, 0.f) * fsqrt(fmaxf(den, 0.f) * iE) + 1e-4f;
  float s = gen ? sgen : spar;
  float t = (B * s + F) * iE;
  const float s_lo = fminf(fmaxf(t0, 0.f), 1.f), s_hi = fminf(fmaxf(t1, 0.f), 1.f);
  s = t < 0.f ? s_lo : (t > 1.f ? s_hi : s);
  t = fminf(fmaxf(t, 0.f), 1.f);
  const float dv[3] = {r[0] + d1[0] * s - d2[0] * t, r[1] + d1[1] * s - d2[1] * t, r[2] + d1[2] * s - d2[2] * t};
  const float reach = rr + slack;
  return dot3(dv, dv) < reach * reach;
}
H12_DEV void swap3(const float* a, float* b) { b[0] = pair_swap(a[0]); b[1] = pair_swap(a[1]); b[2] = pair_swap(a[2]); }

// LDS staging of one wave (block = one wave): per env and leg 16 float4 -- knee segment (2), sole rods (8),
// knee w / v / origin (3), foot w / v / origin (3), real frame -- and the per-body wrench accumulators
// (F, moment about the world origin).  Field-major ([field][env][leg], lane 2 env + leg): the staging writes and the
// own-body reads are lane-consecutive (an [env][leg][field] layout put every lane of a ds_write_b128 on the same
// banks; light stamps: the staging cost the self wave ~0.5 us per inner step)
constexpr int SG_KNEE = 0, SG_ROD = 2, SG_KKIN = 10, SG_FKIN = 13, SG_N = 16;
struct SelfLds {
  float4 geo[SG_N][ENVS_PER_BLOCK][2];
  // [set: 0 self wave, 1 contact wave (self_jobs_shared)][body: 0 knee, 1 foot][F xyz, m xyz][env][leg]: one set per
  // wave, summed in fixed order, so the float atomics' order stays deterministic
  float acc[2][2][6][ENVS_PER_BLOCK][2];
  int slot[ENVS_PER_BLOCK], flags[ENVS_PER_BLOCK];
  int ncand;  // step_kernel: the candidate envs of this inner step (the contact wave shares the jobs, self_jobs)
  int done;   // step_kernel: the inner steps whose jobs the contact wave has finished (its release to the self wave)
};

// LDS hand-off among the lanes of ONE wave (the compiler's lowering of a one-wave block's __syncthreads without
// the s_barrier): self_contacts runs inside a wave that may share its block with another wave (step_kernel's
// helper wave), so it must not wait at a workgroup barrier.
H12_DEV void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

H12_DEV SelfLds& self_lds() {
  __shared__ SelfLds L;
  return L;
}
// The contact wave's release count as an LDS-typed volatile (round 6): through a generic volatile pointer the spin read
// and the release store compiled to flat_load / flat_store sc0 sc1, and every flat access is followed by an
// s_waitcnt vmcnt(0) -- each poll of the self wave (and the contact wave after its release) waited for the wave's
// outstanding row stores to reach memory
// A workgroup-scope float add on an LDS-typed pointer (ds_add_f32): atomicAdd through the generic reference is an agent-
// scope atomic, and the memory legalizer put an s_waitcnt vmcnt(0) (the wave's outstanding row stores) ahead of each
// pass's first one
H12_DEV void lds_add(float& x, float v) {
  __hip_atomic_fetch_add((__attribute__((address_space(3))) float*)&x, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
H12_DEV volatile __attribute__((address_space(3))) int* self_done() {
  return (volatile __attribute__((address_space(3))) int*)&self_lds().done;
}

// Self-contacts, phase 1 (self_stage): broad phase and, when some env of the wave has a candidate pair, the LDS
// staging of the wave's capsules and body kinematics; returns the wave's candidate mask (0: nothing staged, no
// self-contact anywhere in the wave).  Phase 2 (self_finish): the pair jobs and each lane's wrenches.  Rk/pk, vk:
// knee pose (lane frame) and body velocity, Rf/pf, vf: the foot's.  Pair-uniform control flow at every DPP
// swap; wave-uniform at every wave_sync.
// self_broad: the broad phase alone (returns the wave's candidate mask; flags: the env's candidate bits, k01: this
// leg's knee segment, real frame).  step_kernel's self wave runs it before R1 and the staging (self_stage_geo, which
// needs the link velocities) after R1 in candidate waves only.
// The foot's collision points (the sole rods' ends, the bounding capsule's) lie in one foot-frame plane z = SOLE_Z:
// with c = pf + SOLE_Z Rf e_z (sole_plane), a point is c + x Rf e_x + y Rf e_y, real frame (two fma per component)
constexpr float SOLE_Z = h12m::ROD[0][0][2];
static_assert(h12m::ROD[1][0][2] == SOLE_Z && h12m::ROD[2][0][2] == SOLE_Z && h12m::ROD[3][0][2] == SOLE_Z &&
              h12m::ROD[0][1][2] == SOLE_Z && h12m::ROD[1][1][2] == SOLE_Z && h12m::ROD[2][1][2] == SOLE_Z &&
              h12m::ROD[3][1][2] == SOLE_Z && h12m::FB0[2] == SOLE_Z && h12m::FB1[2] == SOLE_Z,
              "sole rods and foot bound in one foot-frame plane");
static_assert(h12m::KNEE0[0] == 0.f && h12m::KNEE0[1] == 0.f && h12m::KNEE1[0] == 0.f && h12m::KNEE1[1] == 0.f,
              "knee segment along the knee link's z axis");
H12_DEV void sole_plane(const float (&Rf)[3][3], const float* pf, float* c) {
  for (int i = 0; i < 3; ++i) c[i] = pf[i] + Rf[i][2] * SOLE_Z;
}
H12_DEV void sole_point(const float (&Rf)[3][3], const float* c, const float* pl, float sg, float* o) {
  for (int i = 0; i < 3; ++i) o[i] = c[i] + Rf[i][0] * pl[0] + Rf[i][1] * pl[1];
  o[1] *= sg;
}
H12_DEV void knee_point(const float (&Rk)[3][3], const float* pk, float z, float sg, float* o) {
  for (int i = 0; i < 3; ++i) o[i] = pk[i] + Rk[i][2] * z;
  o[1] *= sg;
}
// the knee segment's ends (k01, real frame) and the sole plane's offset c (sole_plane), shared by the broad phase and
// the staging
H12_DEV void self_points(int leg, const float (&Rk)[3][3], const float* pk, const float (&Rf)[3][3], const float* pf,
                         float* k01, float* c) {
  const float sg = leg ? -1.f : 1.f;
  knee_point(Rk, pk, h12m::KNEE0[2], sg, k01);
  knee_point(Rk, pk, h12m::KNEE1[2], sg, k01 + 3);
  sole_plane(Rf, pf, c);
}
H12_DEV uint64_t self_broad(int leg, const float (&Rf)[3][3], const float* k01, const float* c, int& flags) {
  const float sg = leg ? -1.f : 1.f;
  // ---- broad phase: lane 0 tests (left knee | right knee, right foot), lane 1 (left foot | right knee, right foot)
  float k0[3] = {k01[0], k01[1], k01[2]}, k1[3] = {k01[3], k01[4], k01[5]};
  float b0[3], b1[3], ok0[3], ok1[3], ob0[3], ob1[3];
  sole_point(Rf, c, h12m::FB0, sg, b0);
  sole_point(Rf, c, h12m::FB1, sg, b1);
  swap3(k0, ok0); swap3(k1, ok1); swap3(b0, ob0); swap3(b1, ob1);
  // own left capsule (lane 0: its knee; lane 1: the partner's = left foot bound) vs the right leg's two
  // value selects (a select between register arrays by pointer would go through scratch)
  float La[3], Lb[3], Rk0[3], Rk1[3], Rb0[3], Rb1[3];
  for (int a = 0; a < 3; ++a) {
    La[a] = leg ? ob0[a] : k0[a]; Lb[a] = leg ? ob1[a] : k1[a];
    Rk0[a] = leg ? k0[a] : ok0[a]; Rk1[a] = leg ? k1[a] : ok1[a];
    Rb0[a] = leg ? b0[a] : ob0[a]; Rb1[a] = leg ? b1[a] : ob1[a];
  }
  const float rl = leg ? h12m::FB_R : h12m::KNEE_R;
  const int f0 = capsules_near(La, Lb, Rk0, Rk1, rl + h12m::KNEE_R) ? 1 : 0;
  const int f1 = capsules_near(La, Lb, Rb0, Rb1, rl + h12m::FB_R) ? 1 : 0;
  const int mine = (f0 | f1 << 1) << (2 * leg);   // bits: 0 kk, 1 kf, 2 fk, 3 ff (left capsule major)
  flags = mine | pair_swap_i(mine);
  return __ballot(flags != 0 && leg == 0);
}
// the staging: this leg's capsules and body kinematics (real frame)
H12_DEV void self_stage_geo(int leg, float mu, const float* k01, const float (&Rk)[3][3], const float* pk,
                            const float* vk, const float (&Rf)[3][3], const float* pf, const float* vf, bool zero_acc,
                            const float* c) {
  SelfLds& L = self_lds();
  const float sg = leg ? -1.f : 1.f;
  const int el = (threadIdx.x & (BLOCK - 1)) >> 1;
  auto g = [&](int f) -> float4& { return L.geo[f][el][leg]; };
  g(SG_KNEE) = make_float4(k01[0], k01[1], k01[2], mu);  // w: this leg's (sole) dynamic friction coefficient
  g(SG_KNEE + 1) = make_float4(k01[3], k01[4], k01[5], 0.f);
#pragma unroll
  for (int r = 0; r < 4; ++r) {  // the rods' ends from the sole plane's offset c (sole_point)
    float a0[3], a1[3];
    sole_point(Rf, c, h12m::ROD[r][0], sg, a0);
    sole_point(Rf, c, h12m::ROD[r][1], sg, a1);
    g(SG_ROD + 2 * r) = make_float4(a0[0], a0[1], a0[2], 0.f);
    g(SG_ROD + 2 * r + 1) = make_float4(a1[0], a1[1], a1[2], 0.f);
  }
  // world angular velocity (a pseudo-vector: w_real = det(M) M w_lane, det M = sg), origin velocity, origin
  float w[3], v[3];
  mv(Rk, vk, w); mv(Rk, vk + 3, v);
  g(SG_KKIN) = make_float4(sg * w[0], w[1], sg * w[2], 0.f);
  g(SG_KKIN + 1) = make_float4(v[0], sg * v[1], v[2], 0.f);
  g(SG_KKIN + 2) = make_float4(pk[0], sg * pk[1], pk[2], 0.f);
  mv(Rf, vf, w); mv(Rf, vf + 3, v);
  g(SG_FKIN) = make_float4(sg * w[0], w[1], sg * w[2], 0.f);
  g(SG_FKIN + 1) = make_float4(v[0], sg * v[1], v[2], 0.f);
  g(SG_FKIN + 2) = make_float4(pf[0], sg * pf[1], pf[2], 0.f);
  if (zero_acc)
    for (int b = 0; b < 2; ++b)
      for (int a = 0; a < 6; ++a) L.acc[0][b][a][el][leg] = 0.f;
}
// a candidate wave's (act != 0, wave-uniform) job list: each candidate env's slot and bits, ranked by the ballot
H12_DEV void self_stage_slots(int leg, uint64_t act, int flags) {
  SelfLds& L = self_lds();
  if (leg == 0 && flags) {
    const int el = (threadIdx.x & (BLOCK - 1)) >> 1;
    const int rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(act >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)act, 0u));
    L.slot[rank] = el;
    L.flags[rank] = flags;
  }
  wave_sync();
}
// zero_acc false (step_kernel): the helper wave has zeroed this lane's accumulators after the previous R2 (self_acc_zero)
// early (step_kernel): the staging's LDS writes are issued ahead of the broad phase's tests, which they then overlap
// (in a wave without candidates they go unread)
H12_DEV uint64_t self_stage(const KParams& P, int leg, float mu, const float (&Rk)[3][3], const float* pk,
                            const float* vk, const float (&Rf)[3][3], const float* pf, const float* vf,
                            bool zero_acc = true, bool early = false) {
  float k01[6], c[3];
  int flags;
  self_points(leg, Rk, pk, Rf, pf, k01, c);
  if (early) self_stage_geo(leg, mu, k01, Rk, pk, vk, Rf, pf, vf, zero_acc, c);
  const uint64_t act = self_broad(leg, Rf, k01, c, flags);
  if ((threadIdx.x & 63) == 0) self_lds().ncand = __popcll(act);
  if (act == 0) return 0;  // wave-uniform: no candidate pair anywhere in the wave
  if (!early) self_stage_geo(leg, mu, k01, Rk, pk, vk, Rf, pf, vf, zero_acc, c);
  self_stage_slots(leg, act, flags);
  return act;
}
// both accumulator sets (self and contact wave) of this lane's env and leg, zeroed for the next inner step's jobs:
// step_kernel's helper wave, before its first inner step and after each barrier R2 (the sums were read before it),
// in its idle wait for barrier S (on the physics wave before R1 they made it the last wave there, r6x_light.json)
H12_DEV void self_acc_zero() {
  SelfLds& L = self_lds();
  const int l = threadIdx.x & (BLOCK - 1);
  for (int set = 0; set < 2; ++set)
    for (int b = 0; b < 2; ++b)
      for (int a = 0; a < 6; ++a) L.acc[set][b][a][l >> 1][l & 1] = 0.f;
}

// The pair jobs of the staged candidate envs: job = (env rank, left capsule i, right capsule j), this lane's jobs
// g0, g0 + stride, ... (one wave: its live lanes; step_kernel's self + contact waves: 2 x the live lanes).  Each job
// adds its contact wrenches into both bodies' LDS accumulators (atomics).
// The job count of the staged candidates (wave-uniform).  Foot-foot fast path (round 5): when every candidate env of
// the wave has only its feet' bounds near (the common case), its 16 rod-rod jobs alone are enumerated -- 4 envs per
// pass of 64 lanes instead of 2 of 25 jobs; the blocks with several candidate envs set the step's tail (light stamps:
// without self-collision p95 / max of the physics loop 22.2 / 23.6 us against 24.2 / 26.7)
H12_DEV int self_njobs(int ncand, bool& ffonly) {
  const SelfLds& L = self_lds();
  const int lr = threadIdx.x & 63;
  const int lf = lr < ncand ? L.flags[lr] : 0;
  ffonly = __ballot(lr < ncand && (lf & 7) != 0) == 0;
  return (ffonly ? 16 : 25) * ncand;
}
H12_DEV void self_jobs(const KParams& P, int njobs, bool ffonly, int g0, int stride, int set) {
  SelfLds& L = self_lds();
  for (int jb = g0; jb < njobs; jb += stride) {
    int rank, i, j;
    if (ffonly) {
      rank = jb >> 4;
      i = 1 + ((jb >> 2) & 3);
      j = 1 + (jb & 3);
    } else {
      rank = jb / 25;
      const int k = jb - 25 * rank;
      i = k / 5;
      j = k - 5 * i;
    }
    const int e = L.slot[rank], fl = L.flags[rank];
    if (!((fl >> (2 * (i > 0) + (j > 0))) & 1)) continue;
    auto gl = [&](int f) -> const float4& { return L.geo[f][e][0]; };
    auto gr = [&](int f) -> const float4& { return L.geo[f][e][1]; };
    // Coulomb cap: material multiply combine (PhysX friction_combine_mode 'multiply').  With the startup material
    // randomisation (randomize_rigid_body_material, C12/rsl_env_cfg.py:213-223, T/.../cat_env_cfg.py:236) it is
    // the product of the two legs' randomised coefficients, otherwise the fixed 0.6 x 0.6 (self_mu)
    const float smu = P.env_mu ? gl(SG_KNEE).w * gr(SG_KNEE).w : P.smu;
    const float4 la = gl(i == 0 ? SG_KNEE : SG_ROD + 2 * (i - 1)), lb = gl(i == 0 ? SG_KNEE + 1 : SG_ROD + 2 * (i - 1) + 1);
    const float4 ra = gr(j == 0 ? SG_KNEE : SG_ROD + 2 * (j - 1)), rb = gr(j == 0 ? SG_KNEE + 1 : SG_ROD + 2 * (j - 1) + 1);
    const float pa[3] = {la.x, la.y, la.z}, pb[3] = {lb.x, lb.y, lb.z}, qa[3] = {ra.x, ra.y, ra.z}, qb[3] = {rb.x, rb.y, rb.z};
    const float rs = (i == 0 ? h12m::KNEE_R : h12m::FOOT_R) + (j == 0 ? h12m::KNEE_R : h12m::FOOT_R);
    SegPts sp;
    seg_points(pa, pb, qa, qb, sp);
    const int kl = i == 0 ? SG_KKIN : SG_FKIN, kr = j == 0 ? SG_KKIN : SG_FKIN;
    const float4 wl = gl(kl), vl = gl(kl + 1), ol = gl(kl + 2), wr = gr(kr), vr_ = gr(kr + 1), orr = gr(kr + 2);
    auto al = [&](int a) -> float& { return L.acc[set][i > 0][a][e][0]; };
    auto ar = [&](int a) -> float& { return L.acc[set][j > 0][a][e][1]; };
#pragma unroll
    for (int q = 0; q < 2; ++q) {  // unrolled: sp's arrays stay in registers
      if (q >= sp.n) break;
      float cA[3], cB[3];
      const float sq = q ? sp.s1 : sp.s0, tq = q ? sp.t1 : sp.t0;
      for (int a = 0; a < 3; ++a) { cA[a] = pa[a] + sp.d1[a] * sq; cB[a] = qa[a] + sp.d2[a] * tq; }
      const float dv[3] = {cA[0] - cB[0], cA[1] - cB[1], cA[2] - cB[2]};
      const float d2 = dot3(dv, dv);
      if (!(d2 < rs * rs) || !(d2 > 1e-18f)) continue;
      const float d = fsqrt(d2), depth = rs - d, id = frcp(d);
      const float sgn = dv[0] * sp.ncx + dv[1] * sp.ncy + dv[2] * sp.ncz < 0.f ? -1.f : 1.f;
      const float n[3] = {sp.has_nc ? sgn * sp.ncx : dv[0] * id, sp.has_nc ? sgn * sp.ncy : dv[1] * id,
                          sp.has_nc ? sgn * sp.ncz : dv[2] * id};
      const float x[3] = {0.5f * (cA[0] + cB[0]), 0.5f * (cA[1] + cB[1]), 0.5f * (cA[2] + cB[2])};
      const float rl_[3] = {x[0] - ol.x, x[1] - ol.y, x[2] - ol.z}, rr_[3] = {x[0] - orr.x, x[1] - orr.y, x[2] - orr.z};
      const float WL[3] = {wl.x, wl.y, wl.z}, WR[3] = {wr.x, wr.y, wr.z};
      float ul[3], ur[3];
      cross(WL, rl_, ul);
      cross(WR, rr_, ur);
      const float vrel[3] = {vl.x + ul[0] - vr_.x - ur[0], vl.y + ul[1] - vr_.y - ur[1], vl.z + ul[2] - vr_.z - ur[2]};
      const float vn = dot3(vrel, n), fn = sp.w * (P.sk * depth - P.sc * vn);
      if (!(fn > 0.f)) continue;
      float F[3];
      for (int a = 0; a < 3; ++a) F[a] = -sp.w * P.sct * (vrel[a] - vn * n[a]);
      const float ftn2 = dot3(F, F), cap = smu * fn;
      if (ftn2 > cap * cap) { const float sc = cap * __builtin_amdgcn_rsqf(ftn2); F[0] *= sc; F[1] *= sc; F[2] *= sc; }
      for (int a = 0; a < 3; ++a) F[a] += fn * n[a];
      float m[3];
      cross(x, F, m);
      for (int a = 0; a < 3; ++a) {
        lds_add(al(a), F[a]); lds_add(al(3 + a), m[a]);
        lds_add(ar(a), -F[a]); lds_add(ar(3 + a), -m[a]);
      }
    }
  }
}

// Self-contact wrenches on this lane's knee (wk) and foot (wf), body coords of the lane frame; their forces are
// added to the reported knee / foot contact forces (fr).  act: self_stage's result.  shared (step_kernel): the contact
// wave runs every other 64-job pass of the inner step it (self_jobs_shared) into its own accumulator set (zeroed with
// this wave's by the helper wave, self_acc_zero), and when there is such a pass (more jobs than live lanes) its
// release (L.done > it) is awaited.
H12_DEV void self_finish(const KParams& P, int leg, uint64_t act, const float (&Rk)[3][3], const float* pk,
                         const float (&Rf)[3][3], const float* pf, float* wk, float* wf, Forces& fr,
                         bool shared = false, int it = 0) {
  for (int i = 0; i < 6; ++i) { wk[i] = 0.f; wf[i] = 0.f; }
  if (act == 0) return;
  SelfLds& L = self_lds();
  const float sg = leg ? -1.f : 1.f;
  const int el = (threadIdx.x & (BLOCK - 1)) >> 1;
  // over the wave's live lanes (a ragged last block has fewer)
  const uint64_t live = __ballot(1);
  const int nlive = __popcll(live);
  const int me = __builtin_amdgcn_mbcnt_hi((uint32_t)(live >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)live, 0u));
  bool ffonly;
  const int njobs = self_njobs(__popcll(act), ffonly);
  self_jobs(P, njobs, ffonly, me, shared ? 2 * nlive : nlive, 0);
  const bool sj = shared && njobs > nlive;  // the contact wave has jobs (self_jobs_shared)
  if (sj) {  // the contact wave's jobs: its release store follows its atomics (an LDS spin, no barrier)
    // bounded (~2 ms) so that a broken release can never hang the GPU; a wait that ends at the bound unreleased is
    // raised in the device diagnostic word, which h12env_check reports (the wrenches of that inner step may be partial)
    for (int k = 0; k < (1 << 16) && *self_done() <= it; ++k) __builtin_amdgcn_s_sleep(1);
    asm volatile("" ::: "memory");
    if (*self_done() <= it && (threadIdx.x & 63) == 0) atomicOr(P.diag, 1);
  }
  wave_sync();
  // ---- own bodies: moment about the body origin, real -> lane frame (force M F; moment sg M T) -> body coords
  const float ms[3] = {1.f, sg, 1.f};
  auto own_body = [&](int b, const float* po, const float (&Rb)[3][3], float* w, float* rep) {
    float ac[6];
    for (int a = 0; a < 6; ++a) ac[a] = shared ? L.acc[0][b][a][el][leg] + L.acc[1][b][a][el][leg] : L.acc[0][b][a][el][leg];
    const float Fr[3] = {ac[0], ac[1], ac[2]};
    const float por[3] = {po[0], sg * po[1], po[2]};
    float pxF[3];
    cross(por, Fr, pxF);
    float Fl[3], Tl[3], fb[3], tb[3];
    for (int a = 0; a < 3; ++a) { Fl[a] = ms[a] * Fr[a]; Tl[a] = sg * ms[a] * (ac[3 + a] - pxF[a]); }
    mtv(Rb, Fl, fb);
    mtv(Rb, Tl, tb);
    for (int a = 0; a < 3; ++a) { w[a] = tb[a]; w[3 + a] = fb[a]; rep[a] += fb[a]; }
  };
  own_body(0, pk, Rk, wk, fr.knee);
  own_body(1, pf, Rf, wf, fr.foot);
  wave_sync();  // the staging area is rewritten by the next physics step
}

// step_kernel's contact wave after R1 (self-collision on): every other 64-job pass of the inner step's self-contact
// jobs, then its release L.done = it + 1 once its LDS atomics are done (self_finish(shared) spins on it).  The blocks
// with several candidate envs set the step's tail: the physics wave waited 1.65 us per launch at R2 in the slowest 5 %
// of the blocks against 0.13 in the median ones (light stamps, profiles/r5/r5t_*); the contact wave waits ~1.9 us
// per launch there anyway
// Only when the jobs outnumber the live lanes (the self wave's first pass): otherwise nothing, no release; the self wave
// makes the same test (self_finish).  This wave's accumulator set is zeroed by the helper wave (self_acc_zero).
H12_DEV void self_jobs_shared(const KParams& P, int it) {
  SelfLds& L = self_lds();
  const int ncand = L.ncand;
  if (!ncand) return;
  bool ffonly;
  const int njobs = self_njobs(ncand, ffonly);
  const uint64_t live = __ballot(1);
  const int nlive = __popcll(live);
  if (njobs <= nlive) return;
  const int me = __builtin_amdgcn_mbcnt_hi((uint32_t)(live >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)live, 0u));
  self_jobs(P, njobs, ffonly, nlive + me, 2 * nlive, 1);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if ((threadIdx.x & 63) == 0 && !P.dbg_norel) *self_done() = it + 1;
}

H12_DEV void self_contacts(const KParams& P, int leg, float mu, const float (&Rk)[3][3], const float* pk,
                           const float* vk, const float (&Rf)[3][3], const float* pf, const float* vf, float* wk,
                           float* wf, Forces& fr) {
  const uint64_t act = self_stage(P, leg, mu, Rk, pk, vk, Rf, pf, vf);
  self_finish(P, leg, act, Rk, pk, Rf, pf, wk, wf, fr);
}

// ---- the helper waves (step_kernel: two or three more waves per block, on other SIMDs of the CU).  The forces of an
// inner step that do not depend on the articulated-inertia chain are computed from the state at the start of the inner
// step by helper waves while the physics wave runs the joint torques and the articulated-inertia chain of pass 2.
// Round 5: the velocity-product accelerations move into the rigid-body bias forces (the AV form: link_av, link_ia<AV>),
// so the physics wave needs neither the link velocities nor the link poses -- only the joint sin / cos; the soles'
// ground contacts go to the helper wave and a fourth (CONTACT) wave takes the knee / torso contacts and the bias forces
// of the lower leg.  Per inner step (workgroup barriers S, R1, R2):
//   physics wave: joint sin / cos, delayed PD + joint terms | R1 | inertia chain (+ sole / knee contact inertias) | R2 |
//                 bias-force chain, base solve, pass 3, integration, next state to LDS | S
//   helper wave:  S | pass 1, heel sole contacts (force, added inertia, stiction anchors) | R1 | a^v and bias forces
//                 of links 0-2, base body bias force (flat: torso contact) | R2
//   contact wave: S | pass 1, toe sole contacts, knee contact (terrain: torso contact) | R1 | a^v of the leg, bias
//                 forces of links 3-5 with the sole / knee added inertias' M a^v | R2
//   self wave:    S | pass 1, self-contact broad phase + staging | R1 | pair jobs, wrenches | R2
// (the self wave is launched only with self-collision).
struct HelpLds {
  float4 st[8][BLOCK];    // state: base pos (3), quat (4), v (3), w (3); leg q (6), qd (6) (lane frame); env origin (3);
                          // added torso mass (1), sole mu_d (1), mu_s (1), spare (1)
  float4 jt[4][BLOCK];    // knee contact: wrench (6), reported force (3), ImplC (5), z (1); spare (1)
  float4 bias_h[6][BLOCK];  // helper: bias forces b_0..b_2 (18), base body bias force (6; lane 0, else 0)
  float4 bias_c[5][BLOCK];  // contact wave: bias forces b_3..b_5 (18; the knee / sole added inertias' M a^v in), spare
  float4 cw1[2][11][BLOCK];  // before R1, per half of the soles (spheres 0-1: helper; 2-3: contact wave): their added
                          // inertia (AInertia, 21), minus their wrench (6), their force (3, body coords), the implicit
                          // report (flat: sum beta, sum gamma, sum beta p, sum gamma p, u = 11; terrain: beta[2],
                          // gamma[2], u[2][3] = 10)
  float4 cw2[3][BLOCK];   // contact wave before R2: a^v of links 3 and 5 (12)
  float4 cst[3][BLOCK];   // sole contact state across the env step: anchors (8, lane frame), contact mask bits of
                          // spheres 0-1 (helper) and 2-3 (contact wave) as two ints
  float4 selfw[3][BLOCK]; // knee self wrench (6), foot self wrench (6)
  uint4 rnd[4][BLOCK];    // the env's reset / command-resample Philox blocks of this step (reset_draws)
  float4 torso[4][BLOCK]; // torso-box ground contact (lane 0 of the pair): wrench (6), reported force (3), ImplC
                          // beta, gamma, u (5), contact flag (1), spare (1)
  float logv[LOG_NSTEP][ENVS_PER_BLOCK];  // episode-log values of this step's resetting envs (0 for the others)
};
// value barrier: x is computed before this point (an empty volatile asm that reads and rewrites it)
H12_DEV void pin(float& x) { asm volatile("" : "+v"(x)); }
H12_DEV HelpLds& help_lds() {
  __shared__ HelpLds H;
  return H;
}
// Stores of the step's outputs use the streaming (nt) policy: nothing in the launch reads them back, and the lines
// go out while the physics runs instead of at the end-of-kernel release -- A/B on one box, 3 interleaved runs:
// step_kernel 34.1 -> 33.8 us, 124.6 -> 125.7 M env-steps/s (profiles/r4/r4o_store_policy_ab.txt)
constexpr int ST_POL = 2;  // buffer store aux bits: 2 = nt
// one float4 of an observation row (16-byte aligned rows) at float4 index j of dst
H12_DEV void st_row4(float* dst, int j, float4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, v),
                                         __builtin_amdgcn_make_buffer_rsrc(dst, 0, -1, 0x00020000), j * 16, 0,
                                         ST_POL);
}
// ---- Fused observation assembly (step path; the history layouts -- Flat, Rsl, CaT: StepArgs.fuse).  The rows
// obs_assemble_kernel would write are stored by step_kernel's helper waves instead, mostly while the physics wave
// integrates: a row is 90 % shifted history (obs[e, slot h] = obs_prev[e, slot h + 1]), which this step's physics
// does not change.  After the first physics step's R2 barrier the helper waves LDS-DMA the block's 32 rows of
// obs_prev (drained before the next R2); after each later R2 -- the physics wave's pass 2 / 3 and integration, where
// they would idle -- each lane stores its share of the shifted rows as float4s (fuse_early).  At the end of the step
// only the newest slot (45 floats per row, the noisy scaled frame the physics wave leaves in LDS), the rows of
// resetting envs (the frame in every slot) and frame_out are written (fuse_late, after barrier F).  Spreading the
// 57.6 KB per block over the physics loop matters: the same stores issued after the loop cost ~6.6 us per step
// (128 CUs at ~9 GB/s each), more than the separate kernel over all 256 CUs.  Bit-identical to the two-kernel path:
// the same copies and the same float operations.
constexpr int FUSE_ROWS = ENVS_PER_BLOCK;
constexpr int FUSE_F4_MAX = FUSE_ROWS * H12_OBS_FRAME * H12_NHIST / 4;  // float4s of a block's rows (history 10)
constexpr int FUSE_CODE_BYTES = (FUSE_F4_MAX + H12_OBS_FRAME * H12_NHIST + 1023) / 1024 * 1024;  // 1 KB DMA chunks
struct FuseLds {
  float hist[FUSE_ROWS * H12_OBS_FRAME * (H12_NHIST + 1)];  // the rows (45 hist floats each), then frames [row][45]
  uint8_t code[FUSE_CODE_BYTES];  // fuse_code_table: per float4 of the rows bit q = float q's shift is 12 (else 3);
                                  // from FUSE_F4_MAX on, per row column its frame component
  float noise[FUSE_ROWS][33];  // noise values of the row's 30 noisy components (padded row: conflict-free)
  int fill[FUSE_ROWS];         // the row restarts its history (terminated | truncated)
};
extern __shared__ float4 h12_dyn_lds[];
H12_DEV FuseLds& fuse_lds() { return *reinterpret_cast<FuseLds*>(h12_dyn_lds); }
struct FuseCtx {
  const float* src;  // the block's first row of obs_prev
  float* dst;        // ... of obs
  const uint8_t* code;  // fuse_code_table (device, FUSE_CODE_BYTES)
  int row;           // floats per row (45 x history)
  int on;            // whole block, 16-byte aligned, >= 2 physics steps: the spread path; else fuse_late alone
};
// One 1-KB LDS-DMA piece (global_load_lds_dwordx4: this lane's 16 B of src into LDS at lds + 16 x lane) written as inline
// asm (round 6): the compiler tracks a builtin LDS-DMA as a pending LDS write and, unable to tell it apart from the
// self-contact accumulators, put an s_waitcnt vmcnt(0) ahead of every inner step's first LDS atomic in the self / contact
// waves -- each job pass waited for the wave's outstanding row stores.  The issuing wave drains its pieces itself
// (fuse_drain's s_waitcnt before barrier R2 of inner step 1; the reads follow that barrier); a VMEM op the compiler does
// not count only makes its own vmcnt(k) waits stricter (the counter drains in issue order)
H12_DEV void lds_dma16(const void* src, const void* lds_chunk) {
  const uint32_t m0 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)lds_chunk;
  asm volatile("global_load_lds_dwordx4 %0, off" : : "v"(src), "{m0}"(m0) : "memory");
}
// helper-wave lane t of nt, after the R2 barrier of inner step it (n_steps in the env step)
// the rows -> LDS: 1 KB LDS-DMA chunks, issued by each helper wave after barrier R2 of the first inner step (fuse_early)
// and drained before R2 of inner step 1 (fuse_drain).  The helper waves wait ~0.7 us per launch at that drain (light
// stamps, profiles/r6/); issued before the first barrier S instead, the chunks delayed the physics wave's state loads:
// step_kernel +1.1 us (profiles/r6/not_kept/r6n_*)
H12_DEV void fuse_dma(const FuseCtx& f, int t, int nt) {
  if (!f.on) return;
  FuseLds& F = fuse_lds();
  const int f4 = FUSE_ROWS * f.row / 4;
  const int w = t >> 6, lane = t & 63, nw = nt >> 6, nch = (f4 + 63) / 64;
  for (int ch = w; ch < nch; ch += nw)
    if (ch * 64 + lane < f4)
      lds_dma16(reinterpret_cast<const float4*>(f.src) + ch * 64 + lane, F.hist + ch * 256);
  for (int ch = w; ch < FUSE_CODE_BYTES / 1024; ch += nw)
    lds_dma16(reinterpret_cast<const uint4*>(f.code) + ch * 64 + lane, F.code + ch * 1024);
}
H12_DEV void fuse_early(const FuseCtx& f, int it, int n_steps, int t, int nt) {
  if (!f.on) return;
  if (it == 0) {
    fuse_dma(f, t, nt);
    return;
  }
  FuseLds& F = fuse_lds();
  const int f4 = FUSE_ROWS * f.row / 4;
  // this lane's float4s j = t + k nt, k in its share of the remaining inner steps: every float gets the next-newer
  // slot (+3 in the 3-wide terms, +12 in the 12-wide ones, fuse_code_table); the newest slot's floats get a
  // placeholder that fuse_late overwrites, as it rewrites the rows of resetting envs (after barrier F, when every
  // early store has completed)
  const int kmax = (f4 + nt - 1) / nt;
  const int k0 = (it - 1) * kmax / (n_steps - 1), k1 = it * kmax / (n_steps - 1);
  for (int k = k0; k < k1; ++k) {
    const int j = t + k * nt;
    if (j >= f4) break;
    const uint32_t cd = F.code[j];
    const float* pb = F.hist + 4 * j;
    st_row4(f.dst, j, make_float4(pb[0 + ((cd & 1u) ? 12 : 3)], pb[1 + ((cd & 2u) ? 12 : 3)],
                                  pb[2 + ((cd & 4u) ? 12 : 3)], pb[3 + ((cd & 8u) ? 12 : 3)]));
  }
}
// step_kernel's helper threads (its launch: (self_coll ? 4 : 3) x BLOCK).  From the kernel parameters: blockDim.x is a
// load from the dispatch packet, and its s_waitcnt vmcnt(0) also waited for the episode sums' loads issued before it,
// ~0.5 us of HBM latency ahead of the first barrier S (light stamps: the helper wave was the block's last there)
H12_DEV int helper_threads(const KParams& P) { return (P.self_coll ? 3 : 2) * BLOCK; }
// before the R2 barrier of inner step 1: this wave's LDS-DMA has landed (the other waves' reads follow R2)
H12_DEV void fuse_drain(const FuseCtx& f, int it) {
  if (f.on && it == 1) __builtin_amdgcn_s_waitcnt(0);
}

// CaT, after the physics loop: the step's raw constraint values and the no_move flag [col][env], in the contact wave's
// R1 hand-off array (free once the last inner step's physics wave has read it)
constexpr int CAT_LDS_EXTRA = 13;
// rows of 33: the contact wave's hand-off reads a column per lane (lane col, row col) -- with rows of 32 floats every
// other lane hit the same bank (28-way conflicts per read)
typedef float CatLds[H12_NCSTR_COLS + CAT_LDS_EXTRA][ENVS_PER_BLOCK + 1];
// rows past the values: CAT_ROW_EPLEN; CAT_LROW_EPOCH (the fold epoch this block waits past, its bits in [0]);
// CAT_LROW_RINV, +1: the running maxima's reciprocals once folded; CAT_LROW_PRE .. +7: the blocks' still prefixes
// (cat_prob_inline)
constexpr int CAT_LROW_EPOCH = H12_NCSTR_COLS + 2, CAT_LROW_RINV = H12_NCSTR_COLS + 3, CAT_LROW_PRE = H12_NCSTR_COLS + 5;
// only the first half: cw1[1] holds the reward inputs (put_rin), written in the same window before barrier L
static_assert(sizeof(CatLds) <= sizeof(HelpLds::cw1[0]), "CaT values fit the first sole hand-off half");
H12_DEV CatLds& cat_lds() { return *reinterpret_cast<CatLds*>(&help_lds().cw1[0][0][0]); }
// Hand-off arrays between the waves of a block: declared as float4 [n4][BLOCK], used FIELD-MAJOR as float [4 n4][BLOCK]
// (value i of lane l at i * 256 + 4 l bytes): the writes / reads pair into ds_write2_b32 / ds_read2_b32 with two
// independent data registers, where float4-per-lane ds_write_b128 needs its 4 values moved into an aligned register
// quad first (round 5: ~100 v_mov per inner step)
H12_DEV void put4(float4 (*dst)[BLOCK], int l, const float* x, int n4) {
  float (*d)[BLOCK] = reinterpret_cast<float (*)[BLOCK]>(dst);
  for (int i = 0; i < 4 * n4; ++i) d[i][l] = x[i];
}
H12_DEV void get4(const float4 (*src)[BLOCK], int l, float* x, int n4) {
  const float (*d)[BLOCK] = reinterpret_cast<const float (*)[BLOCK]>(src);
  for (int i = 0; i < 4 * n4; ++i) x[i] = d[i][l];
}
H12_DEV void put_state(int l, const Base& b, const Leg& lg, const float* org) {
  float x[32] = {b.pos[0], b.pos[1], b.pos[2], b.quat[0], b.quat[1], b.quat[2], b.quat[3],
                 b.vlin[0], b.vlin[1], b.vlin[2], b.wang[0], b.wang[1], b.wang[2]};
  for (int k = 0; k < NL; ++k) { x[13 + k] = lg.q[k]; x[19 + k] = lg.qd[k]; }
  x[25] = org[0]; x[26] = org[1]; x[27] = org[2];
  x[28] = lg.dmass; x[29] = lg.mud; x[30] = lg.mus; x[31] = 0.f;
  put4(help_lds().st, l, x, 8);
}
// the sole contact state (stiction anchors, contact mask; lane frame) of the env step: the physics wave hands it to the
// contact wave before the first inner step and reads it back after the last (barrier L)
H12_DEV void put_cst(int l, const Leg& lg) {
  float x[12];
  for (int q = 0; q < H12_NFOOT_PTS; ++q) { x[2 * q] = lg.anc[q][0]; x[2 * q + 1] = lg.anc[q][1]; }
  x[8] = __int_as_float(lg.cmask);
  x[9] = __int_as_float(0);
  x[10] = x[11] = 0.f;
  put4(help_lds().cst, l, x, 3);
}
H12_DEV void get_cst(int l, Leg& lg) {
  float x[12];
  get4(help_lds().cst, l, x, 3);
  for (int q = 0; q < H12_NFOOT_PTS; ++q) { lg.anc[q][0] = x[2 * q]; lg.anc[q][1] = x[2 * q + 1]; }
  lg.cmask = __float_as_int(x[8]) | __float_as_int(x[9]);
}
// After the physics loop (round 5): the reward terms' inputs beyond the final state (put_state) for the helper wave,
// which computes the rewards while the physics wave resets and observes; in the second sole hand-off array (free
// once the last inner step's physics wave has read it)
struct RewIn {
  float act[NL], act1[NL], tau[NL], jacc[NL], cmd[3], air, con, fmax_foot, metric[2];
  int term, tout;
};
H12_DEV void put_rin(int l, const RewIn& r) {
  static_assert(sizeof(RewIn) <= 36 * sizeof(float), "reward inputs fit 9 float4");
  float x[36];
  const float* f = reinterpret_cast<const float*>(&r);
  for (int i = 0; i < 36; ++i) x[i] = i < (int)(sizeof(RewIn) / sizeof(float)) ? f[i] : 0.f;
  put4(help_lds().cw1[1], l, x, 9);
}
H12_DEV void get_rin(int l, RewIn& r) {
  float x[36];
  get4(help_lds().cw1[1], l, x, 9);
  float* f = reinterpret_cast<float*>(&r);
  for (int i = 0; i < (int)(sizeof(RewIn) / sizeof(float)); ++i) f[i] = x[i];
}
// the owner of sole spheres Q0, Q0 + 1 hands their final anchors and contact bits back (field-major rows: the two
// owners write disjoint floats)
template <int Q0>
H12_DEV void put_cst_half(int l, const Leg& lg) {
  float (*d)[BLOCK] = reinterpret_cast<float (*)[BLOCK]>(help_lds().cst);
  for (int q = Q0; q < Q0 + 2; ++q) { d[2 * q][l] = lg.anc[q][0]; d[2 * q + 1][l] = lg.anc[q][1]; }
  d[8 + Q0 / 2][l] = __int_as_float(lg.cmask & (3 << Q0));
}

H12_DEV void rng(const KParams& P, uint32_t g, uint32_t lo, uint32_t hi, int stream, int block, uint32_t out[4]);
H12_DEV void get_draws(int l, uint32_t* r) {
  for (int c = 0; c < 4; ++c) {
    const uint4 y = help_lds().rnd[c][l];
    r[4 * c] = y.x; r[4 * c + 1] = y.y; r[4 * c + 2] = y.z; r[4 * c + 3] = y.w;
  }
}

// DelayedPDActuator (IsaacLab mode; A/robots/h12.py:58-112): delayed target = CircularBuffer[lag] with the lag
// clamped to pushes - 1, held over physics step st; MuJoCo mode: PD towards the current action
struct PdIn {
  float act[NL], act1[NL], act2[NL];
  int lagpk, since_reset;  // the three delay groups' lags, 3 bits each (a runtime-indexed lag[] would live in scratch)
};
H12_DEV void pd_torque(const KParams& P, const PdIn& d, const Leg& lg, int st, float* tau) {
  const int dec = P.decimation;
  if (P.mode == H12_MODE_ISAACLAB) {
    const int npush = d.since_reset * dec + st + 1;
#pragma unroll
    for (int k = 0; k < NL; ++k) {
      const int L = min((d.lagpk >> (3 * P.dgroup[k])) & 7, npush - 1);
      // bit-mask selects: a ?: chain over the three arrays is folded into a load from a selected address (scratch)
      const uint32_t m0 = 0u - (uint32_t)(L <= st), m1 = 0u - (uint32_t)(L <= st + dec);
      const uint32_t a12 = (__float_as_uint(d.act1[k]) & m1) | (__float_as_uint(d.act2[k]) & ~m1);
      const float a = __uint_as_float((__float_as_uint(d.act[k]) & m0) | (a12 & ~m0));
      const float tgt = h12m::Q0[k] + P.action_scale * a;
      const float v = P.kp[k] * (tgt - lg.q[k]) + P.kd[k] * (0.f - lg.qd[k]);
      tau[k] = fminf(fmaxf(v, -P.elim[k]), P.elim[k]);
    }
  } else {
#pragma unroll
    for (int k = 0; k < NL; ++k) {
      const float tgt = h12m::Q0[k] + P.action_scale * d.act[k];
      const float v = P.kp[k] * (tgt - lg.q[k]) - P.kd[k] * lg.qd[k];
      tau[k] = fminf(fmaxf(v, -P.elim[k]), P.elim[k]);
    }
  }
}
// joint torques beyond the PD term (tq) and the implicit joint inertia of the active limits (dl), from q / qd
H12_DEV void joint_terms(const KParams& P, const Leg& lg, float h, float* tq, float* dl) {
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    const float q = lg.q[k], qd = lg.qd[k];
    // joint limit, branch-free (selects instead of divergent branches): with the implicit penalty active when the
    // predicted end-of-step position q + h qd is beyond the range; dl: h (lc + h lk) of an active limit (oracle
    // joint_limit_torque)
    const float dhi = q - h12m::QHI[k], dlo = q - h12m::QLO[k], hq = P.impl ? h * qd : 0.f;
    const float thi = fminf(0.f, -P.lk * dhi - P.lc * qd), tlo = fmaxf(0.f, -P.lk * dlo - P.lc * qd);
    const float tl = dhi + hq > 0.f ? thi : (dlo + hq < 0.f ? tlo : 0.f);
    float t = tl;
    dl[k] = tl != 0.f ? P.dl : 0.f;
    // PhysX max joint velocity: implicit stiff damper on the excess with a C1 ramp-in over H12_VLIM_RAMP
    // (h12env.h; oracle joint_limit_torque); zero below the limit
    const float ex = fmaxf(fabsf(qd) - P.vmax[k], 0.f);
    const float r = fminf(ex * (1.f / H12_VLIM_RAMP), 1.f);
    const float mag = ex < H12_VLIM_RAMP ? 0.5f * P.cv * ex * r : P.cv * (ex - 0.5f * H12_VLIM_RAMP);
    t -= copysignf(mag, qd);
    dl[k] += h * P.cv * r;
    t -= P.dimpl[k] * qd;
    if (P.use_fl) t -= h12m::FRICTIONLOSS[k] * tanhf(qd * 100.f);
    tq[k] = t;
  }
}

// pass 1 from the state: lane-frame base pose / velocity, then the 6 links' joint sin / cos, spatial velocities
// and world poses; Rk / pk: the knee's pose, R / p on exit: the foot's.
// rel: positions relative to the base origin (the self-contact geometry: only differences of body points enter it,
// and pelvis-relative fp32 points carry the ulp of ~1 m instead of the env's world position); HWTRIG: the joint sin /
// cos without the radial correction (fsincos_hw: the self-contact wave)
template <int K, bool HWTRIG = false>
H12_DEV void leg_pass1(int leg, const Base& b, const Leg& lg, const float* org, float (&R0)[3][3], float* vb,
                       float* pb0, float (&cs)[NL][2], float (&v)[NL][6], float (&Rk)[3][3], float* pk,
                       float (&R)[3][3], float* p, bool rel = false) {
  constexpr bool HW = HWTRIG;
  const float sg = leg ? -1.f : 1.f;
  quat_R(b.quat, R0);
  mtv(R0, b.vlin, vb);
  // base quantities in the lane frame: R' = M R M, v' = s6 * v, p' = M p
  const float mm[3] = {1.f, sg, 1.f};
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) R[i][j] = mm[i] * mm[j] * R0[i][j];
  float vl0[6] = {b.wang[0], b.wang[1], b.wang[2], vb[0], vb[1], vb[2]};
  for (int i = 0; i < 6; ++i) vl0[i] *= s6(i, sg);
  // base position: env-local on terrain (contact geometry relative to the env origin, ground_local)
  pb0[0] = b.pos[0]; pb0[1] = b.pos[1]; pb0[2] = b.pos[2];
  if constexpr (Feat<K>::terrain) { pb0[0] -= org[0]; pb0[1] -= org[1]; pb0[2] -= org[2]; }
  if (rel) { pb0[0] = 0.f; pb0[1] = 0.f; pb0[2] = 0.f; }
  p[0] = pb0[0]; p[1] = sg * pb0[1]; p[2] = pb0[2];
  // the links on pairs (link_pass1_pk)
  f32x2 C[3], V0[3], V[NL][3];
  float R2[3];
  for (int j = 0; j < 3; ++j) {
    C[j] = pk2(R[0][j], R[1][j]);
    R2[j] = R[2][j];
    V0[j] = pk2(vl0[j], vl0[3 + j]);
  }
  f32x2 p01 = pk2(p[0], p[1]);
  float p2 = p[2];
  link_pass1_pk<0, HW>(lg, cs, V0, V, C, R2, p01, p2);
  link_pass1_pk<1, HW>(lg, cs, V[0], V, C, R2, p01, p2);
  link_pass1_pk<2, HW>(lg, cs, V[1], V, C, R2, p01, p2);
  link_pass1_pk<3, HW>(lg, cs, V[2], V, C, R2, p01, p2);
  for (int j = 0; j < 3; ++j) {
    Rk[0][j] = C[j].x;
    Rk[1][j] = C[j].y;
    Rk[2][j] = R2[j];
  }
  pk[0] = p01.x; pk[1] = p01.y; pk[2] = p2;
  link_pass1_pk<4, HW>(lg, cs, V[3], V, C, R2, p01, p2);
  link_pass1_pk<5, HW>(lg, cs, V[4], V, C, R2, p01, p2);
  for (int j = 0; j < 3; ++j) {
    R[0][j] = C[j].x;
    R[1][j] = C[j].y;
    R[2][j] = R2[j];
  }
  p[0] = p01.x; p[1] = p01.y; p[2] = p2;
  for (int l = 0; l < NL; ++l)
    for (int k = 0; k < 3; ++k) {
      v[l][k] = V[l][k].x;
      v[l][3 + k] = V[l][k].y;
    }
}
// knee capsule contact with the ground: lower end point, evaluated at the knee link pose (Rk / pk / vk)
template <int K>
H12_DEV void knee_contact(const KParams& P, float sg, const float (&Rk)[3][3], const float* pk, const float* vk,
                          const float* org, float* fext_knee, float* rep, ImplC& ick, float& knee_pz) {
  float w0[3], w1[3];
  mv(Rk, h12m::KNEE0, w0);
  mv(Rk, h12m::KNEE1, w1);
  const bool lo0 = w0[2] <= w1[2];
  const float* pl = lo0 ? h12m::KNEE0 : h12m::KNEE1;
  knee_pz = lo0 ? h12m::KNEE0[2] : h12m::KNEE1[2];
  float dummy[2];
  contact_sphere<false, Feat<K>::terrain>(P, Rk, pk, vk, pl, h12m::KNEE_R, fext_knee, rep, dummy, false, sg, org, P.mus,
                                          P.mud, ick);
}
// where step_kernel evaluates the knee capsule's ground contact with self-collision on: the self-contact wave (true) or
// the contact wave (false; always without a self wave)
constexpr bool KNEE_ON_SELF = false;
// knee_contact into the physics wave's R1 hand-off (H.jt: the external wrench, the report, the linearisation)
template <int K>
H12_DEV void knee_handoff(const KParams& P, int l, int leg, const float (&Rk)[3][3], const float* pk, const float* vk,
                          const float* org, ImplC& ick, float& knee_pz) {
  float jt[16];
  for (int i = 0; i < 9; ++i) jt[i] = 0.f;
  knee_contact<K>(P, leg ? -1.f : 1.f, Rk, pk, vk, org, jt, jt + 6, ick, knee_pz);
  jt[9] = ick.beta; jt[10] = ick.gamma; jt[11] = ick.u[0]; jt[12] = ick.u[1]; jt[13] = ick.u[2];
  jt[14] = knee_pz; jt[15] = 0.f;
  put4(help_lds().jt, l, jt, 4);
}
// Torso box (URDF box collider h12_12dof.urdf:387, welded to the pelvis) on the ground: the lowest corner is the
// implicit contact (torso_corner, contact_sphere); the other three corners of the lowest face (on terrain only while
// the lowest corner touches: their heightfield lookups stay off a standing robot's helper wave) --
// the face whose normal is the box axis closest to the vertical -- add their explicit forces (torso_face), so a torso
// lying on a face or an edge is carried by that face's corners (oracle contacts(), the same corners in the same
// order).  Evaluated by helper_torso: the contact wave before R1 on terrain, the helper wave between R1 and R2 on flat
// ground.
H12_DEV void torso_corner(const float (&R0)[3][3], float* corner) {
  for (int a = 0; a < 3; ++a) corner[a] = h12m::TORSO_C[a] + (R0[2][a] > 0.f ? -h12m::TORSO_H[a] : h12m::TORSO_H[a]);
}
template <bool TERRAIN>
H12_DEV void torso_face(const KParams& P, const float (&R0)[3][3], const float* pb0, const float* v0, const float* org,
                        float* f, float* fw) {
  const float z0 = fabsf(R0[2][0]), z1 = fabsf(R0[2][1]), z2 = fabsf(R0[2][2]);
  const int an = (z0 >= z1 && z0 >= z2) ? 0 : (z1 >= z2 ? 1 : 2);
  const int ab = an == 0 ? 1 : 0, ac = an == 2 ? 1 : 2;  // the face's two in-plane axes
  auto corner_k = [&](int k) {
    float p[3];
    for (int a = 0; a < 3; ++a) {
      const bool flip = ((k & 1) && a == ab) || ((k & 2) && a == ac);
      const bool neg = (R0[2][a] > 0.f) != flip;
      p[a] = h12m::TORSO_C[a] + (neg ? -h12m::TORSO_H[a] : h12m::TORSO_H[a]);
    }
    ImplC dz;
    float dummy[2];
    contact_sphere<false, TERRAIN, true>(P, R0, pb0, v0, p, 0.f, f, fw, dummy, false, 1.f, org, P.mus, P.mud, dz);
  };
  if constexpr (TERRAIN) {  // one copy of the heightfield contact code in the helper wave's loop
#pragma unroll 1
    for (int k = 1; k < 4; ++k) corner_k(k);
  } else {
#pragma unroll
    for (int k = 1; k < 4; ++k) corner_k(k);
  }
}

// rigid body of the base (with the added torso mass): inertia Rg and bias force v x* (Rg v) (pelvis coords)
template <int K>
H12_DEV void base_body(const KParams& P, const Leg& lg, const float* v0, AInertia& Rg, float* pb) {
  ai_rigid(Rg, h12m::BASE_IBAR, h12m::BASE_MC, h12m::BASE_M);
  if (Feat<K>::ext && P.env_mass) ai_add_point_mass(Rg, lg.dmass, h12m::TORSO_COM);
  float hb[6];
  ai_mul(Rg, v0, hb);
  float x1[3], x2[3], x3[3];
  cross(v0, hb, x1);
  cross(v0 + 3, hb + 3, x2);
  cross(v0, hb + 3, x3);
  pb[0] = x1[0] + x2[0]; pb[1] = x1[1] + x2[1]; pb[2] = x1[2] + x2[2];
  pb[3] = x3[0]; pb[4] = x3[1]; pb[5] = x3[2];
}

// rigid-body bias forces of the 6 links (link coords, lane frame)
H12_DEV void leg_bias(const float (&v)[NL][6], float (&pbias)[NL][6]) {
  bias<0>(v[0], pbias[0]);
  bias<1>(v[1], pbias[1]);
  bias<2>(v[2], pbias[2]);
  bias<3>(v[3], pbias[3]);
  bias<4>(v[4], pbias[4]);
  bias<5>(v[5], pbias[5]);
}

H12_DEV void get_state(int l, Base& b, Leg& lg, float* org) {
  float x[32];
  get4(help_lds().st, l, x, 8);
  lg.dmass = x[28];
  lg.mud = x[29];
  lg.mus = x[30];
  for (int i = 0; i < 3; ++i) { b.pos[i] = x[i]; b.vlin[i] = x[7 + i]; b.wang[i] = x[10 + i]; org[i] = x[25 + i]; }
  for (int i = 0; i < 4; ++i) b.quat[i] = x[3 + i];
  for (int k = 0; k < NL; ++k) { lg.q[k] = x[13 + k]; lg.qd[k] = x[19 + k]; }
}

// step_kernel's env chunk of this block: XCD-aware (xcd_block), so the blocks one XCD runs cover one contiguous
// range of envs -- each XCD's state loads / stores are contiguous runs of every field instead of 128-B chunks
// 1 KB apart (the round-robin order put the tail of the waves on some XCDs 2 us behind the others)
H12_DEV int xcd_block(int b, int nb);
H12_DEV int step_block() { return xcd_block(blockIdx.x, gridDim.x); }

// The torso-box ground contact of the helper wave (flat, after R1) or the contact wave (terrain, before R1): the lowest
// corner's implicit contact and the face's other three corners' explicit ones (torso_face's rule: on terrain only while
// the lowest corner touches) -> H.torso for the physics wave's base combine after R2.  Round 6: the four corners split
// over the lane pair -- leg 0 the lowest corner (implicit) and face corner 1, leg 1 face corners 2 and 3 -- as ONE
// instruction stream (contact_sphere's implicit block switched off per lane): a fallen robot's torso put four full
// sphere contacts on one lane, and the waves of the blocks holding one were the step's slowest at barrier R2 in 24 of
// 40 launches (light stamps, profiles/r6/).  Lane 0's hand-off carries the pair's summed reported force and the
// implicit linearisation; lane 1's its corners' wrench (the physics wave sums the pair's wrenches anyway).  Flat ground
// only: on terrain the split left env-steps of the Rough / C5 parity tests off the oracle that the harness could not
// explain (profiles/r6/), so there lane 0 keeps all four corners.
// the largest distance of a torso-box corner from the base origin (helper_torso's skip test)
constexpr float TORSO_RMAX = 0.2200f;
static_assert((h12m::TORSO_C[0] + h12m::TORSO_H[0]) * (h12m::TORSO_C[0] + h12m::TORSO_H[0]) +
                      (h12m::TORSO_C[1] + h12m::TORSO_H[1]) * (h12m::TORSO_C[1] + h12m::TORSO_H[1]) +
                      (h12m::TORSO_C[2] + h12m::TORSO_H[2]) * (h12m::TORSO_C[2] + h12m::TORSO_H[2]) <=
                  TORSO_RMAX * TORSO_RMAX &&
              h12m::TORSO_C[0] == 0.f && h12m::TORSO_C[1] == 0.f && h12m::TORSO_C[2] >= 0.f,
              "torso corners within TORSO_RMAX of the base origin");
template <int K>
H12_DEV void helper_torso(const KParams& P, int l, int leg, const Base& b, const float* vb, const float (&R0)[3][3],
                          const float* pb0, const float* org) {
  constexpr bool T = Feat<K>::terrain;
  float t[16] = {};
  if constexpr (!T) {
    // flat ground: no corner of the box can activate when its lowest point is higher than a step's travel of any
    // corner (activation needs z_k < -h vn_k <= h (|v| + |w| r_k), r_k <= TORSO_RMAX): the wave skips the contact code
    // when that holds for all its envs (the upright robots of most blocks; exact, the skipped calls return no force)
    float zmin = pb0[2];
#pragma unroll
    for (int a = 0; a < 3; ++a) zmin += R0[2][a] * h12m::TORSO_C[a] - fabsf(R0[2][a]) * h12m::TORSO_H[a];
    const float v2 = b.vlin[0] * b.vlin[0] + b.vlin[1] * b.vlin[1] + b.vlin[2] * b.vlin[2];
    const float w2 = b.wang[0] * b.wang[0] + b.wang[1] * b.wang[1] + b.wang[2] * b.wang[2];
    // (|v| + |w| r)^2 <= 2 (|v|^2 + r^2 |w|^2); margin 1e-4 m for the rounding of zmin
    const float reach2 = 2.f * P.h * P.h * (v2 + TORSO_RMAX * TORSO_RMAX * w2);
    const bool clear = zmin > 1e-4f && zmin * zmin > reach2;
    if (__ballot(!clear) == 0) {
      put4(help_lds().torso, l, t, 4);
      return;
    }
  }
  const float v0[6] = {b.wang[0], b.wang[1], b.wang[2], vb[0], vb[1], vb[2]};
  // corner k of the lowest face (k = 0: the lowest corner, torso_corner; 1..3: torso_face's)
  const float z0 = fabsf(R0[2][0]), z1 = fabsf(R0[2][1]), z2 = fabsf(R0[2][2]);
  const int an = (z0 >= z1 && z0 >= z2) ? 0 : (z1 >= z2 ? 1 : 2);
  const int ab = an == 0 ? 1 : 0, ac = an == 2 ? 1 : 2;
  auto corner_k = [&](int k, float* p) {
    for (int a = 0; a < 3; ++a) {
      const bool flip = ((k & 1) && a == ab) || ((k & 2) && a == ac);
      const bool neg = (R0[2][a] > 0.f) != flip;
      p[a] = h12m::TORSO_C[a] + (neg ? -h12m::TORSO_H[a] : h12m::TORSO_H[a]);
    }
  };
  ImplC ict;
  float dummy[2], p[3];
  bool c = false;
  if constexpr (T) {  // terrain (the contact wave, before R1): lane 0 alone, the face's corners while the lowest touches
    if (leg == 0) {
      corner_k(0, p);
      c = contact_sphere<false, T>(P, R0, pb0, v0, p, 0.f, t, t + 6, dummy, false, 1.f, org, P.mus, P.mud, ict);
      if (c) torso_face<T>(P, R0, pb0, v0, org, t, t + 6);
    }
  } else {
    corner_k(leg ? 2 : 0, p);
    c = contact_sphere<false, T>(P, R0, pb0, v0, p, 0.f, t, t + 6, dummy, false, 1.f, org, P.mus, P.mud, ict, leg != 0);
    corner_k(leg ? 3 : 1, p);
    ImplC dz;
    contact_sphere<false, T, true>(P, R0, pb0, v0, p, 0.f, t, t + 6, dummy, false, 1.f, org, P.mus, P.mud, dz);
  }
  for (int a = 0; a < 3; ++a) {  // the reported force (|F| feeds the illegal-contact test): the pair's sum on lane 0
    const float o = pair_swap(t[6 + a]);
    t[6 + a] = leg ? 0.f : t[6 + a] + o;
  }
  if (leg == 0) {
    t[9] = ict.beta; t[10] = ict.gamma; t[11] = ict.u[0]; t[12] = ict.u[1]; t[13] = ict.u[2];
    t[14] = c ? 1.f : 0.f;
  }
  put4(help_lds().torso, l, t, 4);
}

// Half of the soles' ground contacts of the leg (spheres Q0, Q0 + 1: penalty force, stiction anchors, the implicit added
// inertia; step_kernel's helper / contact wave, before R1) into the cw1[Q0 / 2] hand-off: dI (foot coords), minus the
// wrench, the force, the implicit report
template <int K, int Q0>
H12_DEV void sole_handoff(const KParams& P, int l, float sg, Leg& lg, const float (&R)[3][3], const float* p,
                          const float* v5, const float* org) {
  AInertia dI;
  for (int i = 0; i < 6; ++i) { dI.A[i] = 0.f; dI.C[i] = 0.f; }
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) dI.B[i][j] = 0.f;
  float o[44];
  float* pc = o + 21;  // minus the sole wrench (foot coords)
  float* fw = o + 27;  // the soles' force (body coords; only its norm is used)
  for (int i = 21; i < 44; ++i) o[i] = 0.f;
  if constexpr (!Feat<K>::terrain) {
    SoleSums ss;
    sole_contacts_flat<Q0, Q0 + 2>(P, R, p, v5, lg, dI, pc, fw, ss);
    o[30] = ss.sb; o[31] = ss.sg;
    for (int a = 0; a < 3; ++a) { o[32 + a] = ss.pb[a]; o[35 + a] = ss.pg[a]; o[38 + a] = R[2][a]; }
  } else {
    float fext[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int nmask = 0;
#pragma unroll
    for (int q = Q0; q < Q0 + 2; ++q) {
      const bool was = (lg.cmask >> q) & 1;
      ImplC ic;
      if (contact_sphere<true, true>(P, R, p, v5, h12m::FOOT[q], h12m::FOOT_R, fext, fw, lg.anc[q], was, sg, org,
                                     lg.mus, lg.mud, ic)) {
        nmask |= 1 << q;
        if (P.impl) {
          ai_add_contact(dI, h12m::FOOT[q], ic.u, ic.beta, ic.gamma);
          const int j = q - Q0;
          o[30 + j] = ic.beta; o[32 + j] = ic.gamma;
          o[34 + 3 * j] = ic.u[0]; o[35 + 3 * j] = ic.u[1]; o[36 + 3 * j] = ic.u[2];
        }
      }
    }
    lg.cmask = (lg.cmask & ~(3 << Q0)) | nmask;
    for (int i = 0; i < 6; ++i) pc[i] = -fext[i];
  }
  const float* di = &dI.A[0];
  static_assert(sizeof(AInertia) == 21 * sizeof(float), "AInertia layout");
  for (int i = 0; i < 21; ++i) o[i] = di[i];
  put4(help_lds().cw1[Q0 / 2], l, o, 11);
}

// The helper wave: before R1 its own pass 1 and the heel spheres' ground contacts (sole_handoff; their anchors and
// contact bits stay in its registers through the env step, LDS cst hand-off with the physics wave before the first /
// after the last inner step); after R1 the bias forces of links 0-2 (AV form), the base body's and, on flat ground,
// the torso box's contact.
template <int K>
H12_DEV void helper_wave(const KParams& P, int n, int n_steps, uint32_t g, uint32_t lo, uint32_t hi, const FuseCtx& fc) {
  const int l = threadIdx.x - BLOCK;
  const int leg = l & 1;
  const float sg = leg ? -1.f : 1.f;
  const bool active = step_block() * ENVS_PER_BLOCK + (l >> 1) < n;
  HelpLds& H = help_lds();
  // the Philox blocks a reset (ST_RESET 0, 1) or a command resample (ST_CMD 0, 1) of this step would draw: they
  // depend only on the env id and the step counter, so they are drawn during the physics loop (a resetting wave
  // otherwise spends ~1.5 us on them after the loop, and the step time is the slowest wave's) -- block k after
  // barrier R2 of inner step k, where this wave waits for the physics wave's bias chain anyway.  Before the first
  // barrier S (rounds 3-5) their 80 quarter-rate integer multiplies per block made the whole block wait ~1 us for
  // this wave (light stamps, profiles/r5/)
  auto draw = [&](int k) {
    if (!active) return;
    uint32_t r[4];
    rng(P, g, lo, hi, k < 2 ? ST_RESET : ST_CMD, k & 1, r);
    H.rnd[k][l] = make_uint4(r[0], r[1], r[2], r[3]);
  };
  Leg lg;
  if (P.self_coll) self_acc_zero();
  H12_BW_DECL;
  for (int it = 0; it < n_steps; ++it) {
    SYNC_W(it ? 0 : 3);  // S: the state of this inner step
    Base b;
    float org[3];
    float R0[3][3], vb[3], pb0[3], cs[NL][2], v[NL][6];
    if (active) {
      get_state(l, b, lg, org);
      if (it == 0) get_cst(l, lg);
      float Rk[3][3], pk[3], R[3][3], p[3];
      leg_pass1<K>(leg, b, lg, org, R0, vb, pb0, cs, v, Rk, pk, R, p);
      sole_handoff<K, 0>(P, l, sg, lg, R, p, v[5], org);  // the heel spheres
    }
    SYNC_W(1);  // R1: sole contacts (helper, contact wave), knee contact (contact wave)
    if (active) {
      // bias forces b_i = I_i a^v_i + v_i x* I_i v_i of links 0-2 (the AV form; links 3-5: the contact wave) and the
      // base body's v x* I v (a^v of the base is 0)
      float o[24], av[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      bias<0>(v[0], o);
      link_av<0>(lg, cs, v, av);
      rigid_mul_add<0>(av, o);
      bias<1>(v[1], o + 6);
      link_av<1>(lg, cs, v, av);
      rigid_mul_add<1>(av, o + 6);
      bias<2>(v[2], o + 12);
      link_av<2>(lg, cs, v, av);
      rigid_mul_add<2>(av, o + 12);
      const float v0[6] = {b.wang[0], b.wang[1], b.wang[2], vb[0], vb[1], vb[2]};
      AInertia Rg;
      base_body<K>(P, lg, v0, Rg, o + 18);
      if (leg) for (int i = 18; i < 24; ++i) o[i] = 0.f;
      put4(H.bias_h, l, o, 6);
      if constexpr (!Feat<K>::terrain) helper_torso<K>(P, l, leg, b, vb, R0, pb0, org);
    }
    fuse_drain(fc, it);
    SYNC_W(2);  // R2: bias forces (flat: torso contact)
    fuse_early(fc, it, n_steps, l, helper_threads(P));
    if (it < 4) draw(it);
    if (P.self_coll) self_acc_zero();
  }
  for (int k = n_steps; k < 4; ++k) draw(k);
  H12_BW_STORE();
  if (active) put_cst_half<0>(l, lg);  // the env step's final heel anchors / contact bits (read after L)
}

// The contact wave (round 5): before R1 its own pass 1, the toe spheres' and the knee capsule's ground contacts
// (terrain: the torso box's too); after R1 the leg's velocity-product accelerations a^v and the bias forces of links
// 3-5, including the M a^v of the implicit knee and sole contacts (the AV form: a contact's added inertia M sees the
// link's acceleration a~ + a^v; the soles' added inertia from both halves' cw1 hand-offs).
template <int K>
H12_DEV void contact_wave(const KParams& P, int n, int n_steps, const FuseCtx& fc) {
  const int l = threadIdx.x - 2 * BLOCK;
  const int leg = l & 1;
  const bool active = step_block() * ENVS_PER_BLOCK + (l >> 1) < n;
  HelpLds& H = help_lds();
  Leg lg;
  H12_BW_DECL;
  for (int it = 0; it < n_steps; ++it) {
    SYNC_W(it ? 0 : 3);  // S: the state of this inner step
    float cs[NL][2], v[NL][6];
    Base b;
    float org[3], R0[3][3], vb[3], pb0[3];
    ImplC ick;
    float knee_pz = 0.f;
    if (active) {
      get_state(l, b, lg, org);
      if (it == 0) get_cst(l, lg);
      float Rk[3][3], pk[3], R[3][3], p[3];
      leg_pass1<K>(leg, b, lg, org, R0, vb, pb0, cs, v, Rk, pk, R, p);
      sole_handoff<K, 2>(P, l, leg ? -1.f : 1.f, lg, R, p, v[5], org);  // the toe spheres
      if (!(KNEE_ON_SELF && P.self_coll)) knee_handoff<K>(P, l, leg, Rk, pk, v[3], org, ick, knee_pz);
      // torso-box ground contact (the base body; lane 0 of the pair): data-dependent work (a fallen robot's) kept off
      // the physics wave's chain; on terrain before R1, on flat ground after R1
      if constexpr (Feat<K>::terrain) helper_torso<K>(P, l, leg, b, vb, R0, pb0, org);
    }
    SYNC_W(1);  // R1: the helper's sole contacts
    if (active) {
      if (P.self_coll) self_jobs_shared(P, it);  // first: the self-contact wave waits for its release
      if (KNEE_ON_SELF && P.self_coll) {  // the knee contact's linearisation, from the self wave's hand-off
        float jt[16];
        get4(H.jt, l, jt, 4);
        ick.beta = jt[9]; ick.gamma = jt[10]; ick.u[0] = jt[11]; ick.u[1] = jt[12]; ick.u[2] = jt[13];
        knee_pz = jt[14];
      }
      float o[20], av[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, av3[6];
      link_av<0>(lg, cs, v, av);
      link_av<1>(lg, cs, v, av);
      link_av<2>(lg, cs, v, av);
      link_av<3>(lg, cs, v, av);
      for (int i = 0; i < 6; ++i) { av3[i] = av[i]; o[i] = 0.f; }
      bias<3>(v[3], o);
      rigid_mul_add<3>(av, o);
      if (P.impl && ick.beta + ick.gamma > 0.f) {  // the knee contact's added point inertia sees a^v_3 too
        const float pkz[3] = {0.f, 0.f, knee_pz};
        point_inertia_mul_add(av, pkz, ick.u, ick.beta, ick.gamma, o);
      }
      link_av<4>(lg, cs, v, av);
      bias<4>(v[4], o + 6);
      rigid_mul_add<4>(av, o + 6);
      link_av<5>(lg, cs, v, av);
      bias<5>(v[5], o + 12);
      rigid_mul_add<5>(av, o + 12);
      {  // the soles' added inertia (both halves, cw1) times a^v_5
        float x[24], y[24];
        get4(H.cw1[0], l, x, 6);
        get4(H.cw1[1], l, y, 6);
        AInertia& dI = *reinterpret_cast<AInertia*>(x);
        ai_add(dI, *reinterpret_cast<const AInertia*>(y));
        float ma[6];
        ai_mul(dI, av, ma);
        for (int i = 0; i < 6; ++i) o[12 + i] += ma[i];
      }
      o[18] = o[19] = 0.f;
      put4(H.bias_c, l, o, 5);
      float w[12];
      for (int i = 0; i < 6; ++i) { w[i] = av3[i]; w[6 + i] = av[i]; }
      put4(H.cw2, l, w, 3);
    }
    fuse_drain(fc, it);
    SYNC_W(2);  // R2
    fuse_early(fc, it, n_steps, threadIdx.x - BLOCK, helper_threads(P));
  }
  H12_BW_STORE();
  if (active) put_cst_half<2>(l, lg);  // the env step's final toe anchors / contact bits (read after L)
}

template <int K>
H12_DEV void self_wave(const KParams& P, int n, int n_steps, const FuseCtx& fc) {
  const int l = threadIdx.x - 3 * BLOCK;
  const int leg = l & 1;
  const bool active = step_block() * ENVS_PER_BLOCK + (l >> 1) < n;
  HelpLds& H = help_lds();
  if ((threadIdx.x & 63) == 0) self_lds().done = 0;  // before the first barrier S: the contact wave's release count
  H12_BW_DECL;
  for (int it = 0; it < n_steps; ++it) {
    SYNC_W(it ? 0 : 3);  // S: the state of this inner step
    float Rk[3][3], pk[3], R[3][3], p[3];
    uint64_t act = 0;
    if (active) {
      Base b;
      Leg lg;
      float org[3];
      get_state(l, b, lg, org);
      float R0[3][3], vb[3], pb0[3], cs[NL][2], v[NL][6];
      leg_pass1<K, true>(leg, b, lg, org, R0, vb, pb0, cs, v, Rk, pk, R, p, true);  // pelvis-relative positions
      // broad phase and, in a candidate wave, the staging (after R1 instead, the staging made this wave the last at R2:
      // -3 %, profiles/r5/r5p_*)
      act = self_stage(P, leg, lg.mud, Rk, pk, v[3], R, p, v[5], false, true);
      if constexpr (KNEE_ON_SELF) {
        // the knee capsule's ground contact (the contact wave's without a self wave): the knee origin back at the base
        // position (env-local on terrain, lane frame)
        float pka[3] = {b.pos[0], b.pos[1], b.pos[2]};
        if constexpr (Feat<K>::terrain) { pka[0] -= org[0]; pka[1] -= org[1]; pka[2] -= org[2]; }
        pka[0] += pk[0]; pka[1] = (leg ? -pka[1] : pka[1]) + pk[1]; pka[2] += pk[2];
        ImplC ick;
        float knee_pz;
        knee_handoff<K>(P, l, leg, Rk, pka, v[3], org, ick, knee_pz);
      }
    }
    SYNC_W(1);  // R1
    if (active) {
      float w[12];
      Forces fr = {};
      self_finish(P, leg, act, Rk, pk, R, p, w, w + 6, fr, true, it);
      PHN(__popcll(act));
      put4(H.selfw, l, w, 3);
    }
    fuse_drain(fc, it);
    SYNC_W(2);  // R2: self-contact wrenches
    fuse_early(fc, it, n_steps, threadIdx.x - BLOCK, helper_threads(P));
  }
  H12_BW_STORE();
}

// One inner step of length h for the lane's leg and the shared base, the whole step in ONE wave (physics_kernel, the
// MuJoCo-mode parity hook; step_kernel's waves split it, inner_step_hw): tau_pd, the actuator torques of the lane's 6
// joints (lane frame).  Adds this lane's contact forces into fr.
template <int K>
H12_DEV void inner_step_1w(const KParams& P, int leg, Base& b, Leg& lg, const float* tau_pd, float h, Forces& fr,
                           const float* org) {
  const float sg = leg ? -1.f : 1.f;
  float R0[3][3], vb[3], pb0[3], cs[NL][2], v[NL][6], Rk[3][3], pk[3], R[3][3], p[3];
  leg_pass1<K>(leg, b, lg, org, R0, vb, pb0, cs, v, Rk, pk, R, p);
  const float v0[6] = {b.wang[0], b.wang[1], b.wang[2], vb[0], vb[1], vb[2]};
  float fext_knee[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  ImplC ick;      // knee contact linearisation (added to link 3 in pass 2)
  float knee_pz;  // z of the knee contact point (KNEE0 or KNEE1; x = y = 0)
  knee_contact<K>(P, sg, Rk, pk, v[3], org, fext_knee, fr.knee, ick, knee_pz);
  // ---- foot: 4 anchored sole spheres on the ankle-roll link; the inertia chain of pass 2 starts at link 5
  int smask = 0;                      // implicit: sole spheres whose stiction spring sticks
  float fu[H12_NFOOT_PTS][3];         // implicit: ground normal at each sole sphere, foot coords
  AInertia IA;
  ai_rigid(IA, h12m::IBAR[5], h12m::MC[5], h12m::M[5]);
  float pc[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // minus the sole contact wrench (foot coords)
  SoleSums ss;
  if constexpr (!Feat<K>::terrain) {
    sole_contacts_flat(P, R, p, v[5], lg, IA, pc, fr.foot, ss);
  } else {
    float fext[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int nmask = 0;
#pragma unroll
    for (int q = 0; q < H12_NFOOT_PTS; ++q) {
      bool was = (lg.cmask >> q) & 1;
      ImplC ic;
      if (contact_sphere<true, Feat<K>::terrain>(P, R, p, v[5], h12m::FOOT[q], h12m::FOOT_R, fext, fr.foot, lg.anc[q], was, sg, org, lg.mus,
                               lg.mud, ic)) {
        nmask |= 1 << q;
        if (P.impl) {
          ai_add_contact(IA, h12m::FOOT[q], ic.u, ic.beta, ic.gamma);
          smask |= (ic.beta > 0.f ? 1 : 0) << q;
          fu[q][0] = ic.u[0]; fu[q][1] = ic.u[1]; fu[q][2] = ic.u[2];
        }
      }
    }
    lg.cmask = nmask;
    for (int i = 0; i < 6; ++i) pc[i] = -fext[i];
  }
  // ---- joint torques beyond PD, implicit limit inertias
  float tau[NL], dl[NL];
  {
    float tq[NL];
    joint_terms(P, lg, h, tq, dl);
    for (int k = 0; k < NL; ++k) tau[k] = tau_pd[k] + tq[k];
  }
  // ---- pass 2, articulated-inertia chain (leaf -> root)
  float U[NL][6], Dinv[NL], u[NL], Ic[NL][6];
  link_ia<5>(P, lg, cs, v, ick, knee_pz, dl, IA, U, Dinv, Ic, h);
  link_ia<4>(P, lg, cs, v, ick, knee_pz, dl, IA, U, Dinv, Ic, h);
  link_ia<3>(P, lg, cs, v, ick, knee_pz, dl, IA, U, Dinv, Ic, h);
  link_ia<2>(P, lg, cs, v, ick, knee_pz, dl, IA, U, Dinv, Ic, h);
  link_ia<1>(P, lg, cs, v, ick, knee_pz, dl, IA, U, Dinv, Ic, h);
  link_ia<0>(P, lg, cs, v, ick, knee_pz, dl, IA, U, Dinv, Ic, h);
  float pbias[NL][6], wk[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, wf[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float pbase[6];  // base body bias force (lane 0; 0 on lane 1)
  AInertia Rg;     // base body inertia (lane 0)
  {
    leg_bias(v, pbias);
    base_body<K>(P, lg, v0, Rg, pbase);
    if (P.self_coll) {  // pelvis-relative geometry, as the self wave's (subtracted here: one pass 1 in this wave)
      Forces fs = {};
      const float pbl[3] = {pb0[0], sg * pb0[1], pb0[2]};
      const float pkr[3] = {pk[0] - pbl[0], pk[1] - pbl[1], pk[2] - pbl[2]}, pr[3] = {p[0] - pbl[0], p[1] - pbl[1], p[2] - pbl[2]};
      self_contacts(P, leg, lg.mud, Rk, pkr, v[3], R, pr, v[5], wk, wf, fs);
    }
  }
  for (int i = 0; i < 6; ++i) fext_knee[i] += wk[i];
  for (int a = 0; a < 3; ++a) { fr.knee[a] += wk[3 + a]; fr.foot[a] += wf[3 + a]; }
  // ---- pass 2, bias-force chain (leaf -> root)
  float pAcc[6];
  for (int i = 0; i < 6; ++i) pAcc[i] = pbias[5][i] + pc[i] - wf[i];
  link_p<5>(cs, U, Dinv, Ic, tau, pbias, fext_knee, pAcc, u);
  link_p<4>(cs, U, Dinv, Ic, tau, pbias, fext_knee, pAcc, u);
  link_p<3>(cs, U, Dinv, Ic, tau, pbias, fext_knee, pAcc, u);
  link_p<2>(cs, U, Dinv, Ic, tau, pbias, fext_knee, pAcc, u);
  link_p<1>(cs, U, Dinv, Ic, tau, pbias, fext_knee, pAcc, u);
  link_p<0>(cs, U, Dinv, Ic, tau, pbias, fext_knee, pAcc, u);
  // ---- un-mirror the leg's contribution to the base (I' = S I S, p' = S p)
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) IA.B[i][j] *= s6(i, sg) * s6(3 + j, sg);
  IA.A[3] *= sg; IA.A[5] *= sg;  // xy, yz of the angular block (s = (sg,1,sg))
  IA.C[3] *= sg; IA.C[5] *= sg;  // xy, yz of the linear block (s = (1,sg,1))
  for (int i = 0; i < 6; ++i) pAcc[i] *= s6(i, sg);
  // ---- lane 0 adds the base body: rigid inertia, bias force, torso-box contact
  float ag[6] = {0.f, 0.f, 0.f, -P.g * R0[2][0], -P.g * R0[2][1], -P.g * R0[2][2]};
  ImplC ict;  // torso contact linearisation (lane 0)
  float corner[3];
  ict.beta = ict.gamma = 0.f;
  if (leg == 0) {
    ai_add(IA, Rg);
    for (int i = 0; i < 6; ++i) pAcc[i] += pbase[i];
    torso_corner(R0, corner);
    float ft[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    bool c;
    {
      float dummy[2];
      c = contact_sphere<false, Feat<K>::terrain>(P, R0, pb0, v0, corner, 0.f, ft, fr.torso, dummy, false, 1.f, org,
                                                   P.mus, P.mud, ict);
      if (c || !Feat<K>::terrain) torso_face<Feat<K>::terrain>(P, R0, pb0, v0, org, ft, fr.torso);
    }
    if (c && P.impl) ai_add_contact(IA, corner, ict.u, ict.beta, ict.gamma);
    for (int i = 0; i < 6; ++i) pAcc[i] -= ft[i];
  }
  // ---- pair sum in fixed (left + right) order: both lanes hold bit-identical base quantities
  AInertia IB;
  float pB[6];
  {
    auto comb = [&](float x) {
      float y = pair_swap(x);
      return leg ? (y + x) : (x + y);
    };
    for (int i = 0; i < 6; ++i) { IB.A[i] = comb(IA.A[i]); IB.C[i] = comb(IA.C[i]); pB[i] = comb(pAcc[i]); }
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) IB.B[i][j] = comb(IA.B[i][j]);
  }
  float a0[6];
  if (P.fix_base) {
    for (int i = 0; i < 6; ++i) a0[i] = -ag[i];
  } else {
    float rhs[6] = {-pB[0], -pB[1], -pB[2], -pB[3], -pB[4], -pB[5]};
    solve6(IB, rhs, a0);
  }
  if (P.impl && leg == 0 && ict.gamma + ict.beta > 0.f) impl_force(a0, corner, ict.u, ict.beta, ict.gamma, fr.torso);
  // ---- pass 3 (root -> leaf) in the lane frame
  float a[6];
  for (int i = 0; i < 6; ++i) a[i] = s6(i, sg) * a0[i];
  float qdd[NL];
  link_pass3<0>(lg, cs, v, U, Dinv, u, a, qdd);
  link_pass3<1>(lg, cs, v, U, Dinv, u, a, qdd);
  link_pass3<2>(lg, cs, v, U, Dinv, u, a, qdd);
  link_pass3<3>(lg, cs, v, U, Dinv, u, a, qdd);
  if (P.impl && ick.gamma + ick.beta > 0.f) {  // implicit part of the knee contact force
    const float pk[3] = {0.f, 0.f, knee_pz};
    impl_force(a, pk, ick.u, ick.beta, ick.gamma, fr.knee);
  }
  link_pass3<4>(lg, cs, v, U, Dinv, u, a, qdd);
  link_pass3<5>(lg, cs, v, U, Dinv, u, a, qdd);
  if constexpr (!Feat<K>::terrain) {
    if (P.impl && lg.cmask) sole_impl_force_flat(a, R, ss, fr.foot);
  } else if (P.impl && lg.cmask) {  // implicit part of the sole forces (a = foot acceleration, shifted frame)
    const float hb = P.h * P.fc, ha = P.h * P.cc;
#pragma unroll
    for (int q = 0; q < H12_NFOOT_PTS; ++q) {
      const float beta = ((smask >> q) & 1) ? hb : 0.f;
      const float gamma = ((lg.cmask >> q) & 1) ? ha - beta : 0.f;
      if ((lg.cmask >> q) & 1) impl_force(a, h12m::FOOT[q], fu[q], beta, gamma, fr.foot);
    }
  }
  // ---- semi-implicit Euler (mj_Euler conventions), base in real coordinates
  if (!P.fix_base) {
    float nd[6];
    for (int i = 0; i < 6; ++i) nd[i] = a0[i] + ag[i];
    float wxv[3];
    cross(b.wang, vb, wxv);
    float al[3] = {nd[3] + wxv[0], nd[4] + wxv[1], nd[5] + wxv[2]}, aw[3];
    mv(R0, al, aw);
    for (int i = 0; i < 3; ++i) { b.vlin[i] += h * aw[i]; b.wang[i] += h * nd[i]; }
    for (int i = 0; i < 3; ++i) b.pos[i] += h * b.vlin[i];
    quat_integrate(b.quat, b.wang, h);
  }
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    lg.qd[k] += h * qdd[k];
    float q = lg.q[k] + h * lg.qd[k];
    // hard-limit residual (oracle limit_projection): beyond the range by more than lproj -> back to the tolerance,
    // outward velocity zeroed; branch-free
    const float hi = h12m::QHI[k] + P.lproj, lo = h12m::QLO[k] - P.lproj;
    const bool over = q > hi, under = q < lo;
    lg.qd[k] = over ? fminf(lg.qd[k], 0.f) : (under ? fmaxf(lg.qd[k], 0.f) : lg.qd[k]);
    lg.q[k] = fminf(fmaxf(q, lo), hi);
  }
}



// One inner step of step_kernel's PHYSICS wave (round 5): the critical chain only -- the joint sin / cos, the delayed PD
// and joint terms, the articulated-inertia chain and, after R2, the bias-force chain, the base solve, pass 3 and the
// integration.  The ABA runs in the AV form (link_ia<AV>): the velocity-product accelerations are in the rigid-body bias
// forces the helper / contact waves hand over, so this wave needs no link velocities or poses; the sole contacts are
// the helper wave's (their added inertia, wrench and force arrive at R1), the knee contact the contact wave's.  tau_pd: the
// delayed-PD torque of the current physics step (computed here at its first inner step from pd, held over it); with
// `more` the next inner step's state is put to LDS (barrier S).
template <int K>
H12_DEV void inner_step_hw(const KParams& P, int leg, Base& b, Leg& lg, const PdIn& pd, int it, float* tau_pd, float h,
                           Forces& fr, const float* org, bool more H12_BW_PARAM) {
  PHX_INIT();
  const float sg = leg ? -1.f : 1.f;
  HelpLds& H = help_lds();
  float cs[NL][2];
#pragma unroll
  for (int k = 0; k < NL; ++k) fsincos(lg.q[k], &cs[k][1], &cs[k][0]);
  // ---- joint torques: the delayed PD (held over the physics step), limit penalty, max-velocity damper, damping,
  // friction loss; implicit limit inertias
  if (it % P.inner == 0) pd_torque(P, pd, lg, it / P.inner, tau_pd);
  float tau[NL], dl[NL];
  {
    float tq[NL];
    joint_terms(P, lg, h, tq, dl);
    for (int k = 0; k < NL; ++k) tau[k] = tau_pd[k] + tq[k];
  }
  PHX(10);
  SYNC_W(1);  // R1: sole contacts (helper), knee contact (contact wave)
  PHX(8);
  float fext_knee[6];
  ImplC ick;
  float knee_pz;
  {
    float jt[16];
    get4(H.jt, threadIdx.x, jt, 4);
    for (int i = 0; i < 6; ++i) fext_knee[i] = jt[i];
    for (int a = 0; a < 3; ++a) fr.knee[a] += jt[6 + a];
    ick.beta = jt[9]; ick.gamma = jt[10]; ick.u[0] = jt[11]; ick.u[1] = jt[12]; ick.u[2] = jt[13];
    knee_pz = jt[14];
  }
  // ---- pass 2, articulated-inertia chain (leaf -> root), from the foot's rigid inertia + the soles' added inertia
  AInertia IA;
  {
    float x[32], y[32];
    get4(H.cw1[0], threadIdx.x, x, 8);
    get4(H.cw1[1], threadIdx.x, y, 8);
    ai_rigid(IA, h12m::IBAR[5], h12m::MC[5], h12m::M[5]);
    ai_add(IA, *reinterpret_cast<const AInertia*>(x));
    ai_add(IA, *reinterpret_cast<const AInertia*>(y));
    for (int a = 0; a < 3; ++a) fr.foot[a] += x[27 + a] + y[27 + a];
  }
  PHX(11);
  f32x2 U[NL][3];  // (angular, linear) pairs
  float Dinv[NL], u[NL], Ic[NL][6];
  float v[NL][6];  // unused in the AV form
  link_ia<5, true>(P, lg, cs, v, ick, knee_pz, dl, IA, U, Dinv, Ic, h);
  link_ia<4, true>(P, lg, cs, v, ick, knee_pz, dl, IA, U, Dinv, Ic, h);
  link_ia<3, true>(P, lg, cs, v, ick, knee_pz, dl, IA, U, Dinv, Ic, h);
  link_ia<2, true>(P, lg, cs, v, ick, knee_pz, dl, IA, U, Dinv, Ic, h);
  link_ia<1, true>(P, lg, cs, v, ick, knee_pz, dl, IA, U, Dinv, Ic, h);
  link_ia<0, true>(P, lg, cs, v, ick, knee_pz, dl, IA, U, Dinv, Ic, h);
  // the inertia chain stays ahead of R2 (else the compiler sinks most of it past the barrier)
  for (int i = 0; i < 6; ++i) { pin(IA.A[i]); pin(IA.C[i]); }
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) pin(IA.B[i][j]);
  PHX(12);
  SYNC_W(2);  // R2: bias forces (helper: links 0-2 + base; contact wave: links 3-5), torso contact, self wrenches
  PHX(9);
  float pbias[NL][6], wk[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, wf[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  f32x2 pb[NL][3];  // pbias as (angular, linear) pairs, the knee's external wrench subtracted from link 3's
  float pbase[6];  // base body bias force (lane 0; 0 on lane 1)
  {
    float o[24], c[20];
    get4(H.bias_h, threadIdx.x, o, 6);
    get4(H.bias_c, threadIdx.x, c, 5);
    for (int i = 0; i < 6; ++i) {
      pbias[0][i] = o[i]; pbias[1][i] = o[6 + i]; pbias[2][i] = o[12 + i]; pbase[i] = o[18 + i];
      pbias[3][i] = c[i]; pbias[4][i] = c[6 + i]; pbias[5][i] = c[12 + i];
    }
  }
  AInertia Rg;  // base body inertia (lane 0)
  ai_rigid(Rg, h12m::BASE_IBAR, h12m::BASE_MC, h12m::BASE_M);
  if (Feat<K>::ext && P.env_mass) ai_add_point_mass(Rg, lg.dmass, h12m::TORSO_COM);
  if (P.self_coll) {
    float w[12];
    get4(H.selfw, threadIdx.x, w, 3);
    for (int i = 0; i < 6; ++i) { wk[i] = w[i]; wf[i] = w[6 + i]; }
  }
  PHX(13);
  for (int i = 0; i < 6; ++i) fext_knee[i] += wk[i];
  for (int a = 0; a < 3; ++a) { fr.knee[a] += wk[3 + a]; fr.foot[a] += wf[3 + a]; }
  for (int j = 0; j < NL; ++j)
    for (int k = 0; k < 3; ++k)
      pb[j][k] = j == 3 ? pk2(pbias[j][k] - fext_knee[k], pbias[j][3 + k] - fext_knee[3 + k])
                        : pk2(pbias[j][k], pbias[j][3 + k]);
  // ---- pass 2, bias-force chain (leaf -> root), on (angular, linear) pairs
  float pAcc[6];
  {
    float pa[8], pc[8];
    get4(&H.cw1[0][5], threadIdx.x, pa, 2);  // floats 20..27 of each half's hand-off: the soles' -wrench at 21..26
    get4(&H.cw1[1][5], threadIdx.x, pc, 2);
    f32x2 p[3];
    for (int k = 0; k < 3; ++k)
      p[k] = pk2(pbias[5][k] + (pa[1 + k] + pc[1 + k]) - wf[k], pbias[5][3 + k] + (pa[4 + k] + pc[4 + k]) - wf[3 + k]);
    link_p_pk<5>(cs, U, Dinv, tau, pb, p, u);
    link_p_pk<4>(cs, U, Dinv, tau, pb, p, u);
    link_p_pk<3>(cs, U, Dinv, tau, pb, p, u);
    link_p_pk<2>(cs, U, Dinv, tau, pb, p, u);
    link_p_pk<1>(cs, U, Dinv, tau, pb, p, u);
    link_p_pk<0>(cs, U, Dinv, tau, pb, p, u);
    PHL(0);
    for (int k = 0; k < 3; ++k) { pAcc[k] = p[k].x; pAcc[3 + k] = p[k].y; }
  }
  // ---- un-mirror the leg's contribution to the base (I' = S I S, p' = S p)
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) IA.B[i][j] *= s6(i, sg) * s6(3 + j, sg);
  IA.A[3] *= sg; IA.A[5] *= sg;  // xy, yz of the angular block (s = (sg,1,sg))
  IA.C[3] *= sg; IA.C[5] *= sg;  // xy, yz of the linear block (s = (1,sg,1))
  for (int i = 0; i < 6; ++i) pAcc[i] *= s6(i, sg);
  // ---- lane 0 adds the base body: rigid inertia, bias force, torso-box contact (helper wave)
  float R0[3][3];
  quat_R_unit(b.quat, R0);  // (quat_R_unit: off the critical chain's reciprocal)
  float ag[6] = {0.f, 0.f, 0.f, -P.g * R0[2][0], -P.g * R0[2][1], -P.g * R0[2][2]};
  // (lane 1's hand-offs hold zeros here -- the helper wave writes the base body's bias force and the torso contact on
  // lane 0 only -- so both lanes run this without a branch; the base body's rigid inertia (dmass: an env-level value,
  // the same in both lanes) is added after the pair sum)
  ImplC ict;  // torso contact linearisation (lane 0)
  float corner[3];
  {
    for (int i = 0; i < 6; ++i) pAcc[i] += pbase[i];
    torso_corner(R0, corner);
    float t[16];
    get4(H.torso, threadIdx.x, t, 4);
    for (int a = 0; a < 3; ++a) fr.torso[a] += t[6 + a];
    ict.beta = t[9]; ict.gamma = t[10]; ict.u[0] = t[11]; ict.u[1] = t[12]; ict.u[2] = t[13];
    const bool c = t[14] != 0.f;
    if (c && P.impl) ai_add_contact(IA, corner, ict.u, ict.beta, ict.gamma);
    for (int i = 0; i < 6; ++i) pAcc[i] -= t[i];
  }
  // ---- pair sum in fixed (left + right) order: both lanes hold bit-identical base quantities
  AInertia IB;
  float pB[6];
  {
    auto comb = [&](float x) {
      float y = pair_swap(x);
      return leg ? (y + x) : (x + y);
    };
    for (int i = 0; i < 6; ++i) { IB.A[i] = comb(IA.A[i]); IB.C[i] = comb(IA.C[i]); pB[i] = comb(pAcc[i]); }
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) IB.B[i][j] = comb(IA.B[i][j]);
    ai_add(IB, Rg);
  }
  // branch-free (the fixed base selects afterwards): the pair sums stay in the solve's block, where each DPP swap folds
  // into its add
  float a0[6];
  {
    float rhs[6] = {-pB[0], -pB[1], -pB[2], -pB[3], -pB[4], -pB[5]};
    solve6(IB, rhs, a0);
    for (int i = 0; i < 6; ++i) a0[i] = P.fix_base ? -ag[i] : a0[i];
  }
  PHL(1);
  if (P.impl && leg == 0 && ict.gamma + ict.beta > 0.f) impl_force(a0, corner, ict.u, ict.beta, ict.gamma, fr.torso);
  // ---- pass 3 (root -> leaf) in the lane frame: a~ (the implicit contact reports use a~ + a^v)
  float avk[12];
  get4(H.cw2, threadIdx.x, avk, 3);
  f32x2 ap[3];  // (angular, linear) pairs
  for (int k = 0; k < 3; ++k) ap[k] = pk2(s6(k, sg) * a0[k], s6(3 + k, sg) * a0[3 + k]);
  float qdd[NL];
  link_pass3_pk<0>(cs, U, Dinv, u, ap, qdd);
  link_pass3_pk<1>(cs, U, Dinv, u, ap, qdd);
  link_pass3_pk<2>(cs, U, Dinv, u, ap, qdd);
  link_pass3_pk<3>(cs, U, Dinv, u, ap, qdd);
  if (P.impl && ick.gamma + ick.beta > 0.f) {  // implicit part of the knee contact force
    const float pk[3] = {0.f, 0.f, knee_pz};
    float ah[6];
    for (int k = 0; k < 3; ++k) { ah[k] = ap[k].x + avk[k]; ah[3 + k] = ap[k].y + avk[3 + k]; }
    impl_force(ah, pk, ick.u, ick.beta, ick.gamma, fr.knee);
  }
  link_pass3_pk<4>(cs, U, Dinv, u, ap, qdd);
  link_pass3_pk<5>(cs, U, Dinv, u, ap, qdd);
  PHL(2);
  if (P.impl) {  // implicit part of the sole forces (a~ + a^v = the foot's acceleration, shifted frame)
    float ah[6], r[2][16];
    for (int k = 0; k < 3; ++k) { ah[k] = ap[k].x + avk[6 + k]; ah[3 + k] = ap[k].y + avk[9 + k]; }
    get4(&H.cw1[0][7], threadIdx.x, r[0], 4);  // floats 28..43 of each half: the report at 30..
    get4(&H.cw1[1][7], threadIdx.x, r[1], 4);
    if constexpr (!Feat<K>::terrain) {
      // without a branch: a sole out of contact reports zero sums (sole_handoff)
      SoleSums ss;
      ss.sb = r[0][2] + r[1][2];
      ss.sg = r[0][3] + r[1][3];
      for (int i = 0; i < 3; ++i) { ss.pb[i] = r[0][4 + i] + r[1][4 + i]; ss.pg[i] = r[0][7 + i] + r[1][7 + i]; }
      const float Rf[3][3] = {{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}, {r[0][10], r[0][11], r[0][12]}};
      sole_impl_force_flat(ah, Rf, ss, fr.foot);
    } else {
#pragma unroll
      for (int q = 0; q < H12_NFOOT_PTS; ++q) {
        const float* rh = r[q / 2];
        const int j = q % 2;
        const float beta = rh[2 + j], gamma = rh[4 + j];
        const float uq[3] = {rh[6 + 3 * j], rh[7 + 3 * j], rh[8 + 3 * j]};
        if (beta + gamma > 0.f) impl_force(ah, h12m::FOOT[q], uq, beta, gamma, fr.foot);
      }
    }
  }
  // ---- semi-implicit Euler (mj_Euler conventions), base in real coordinates.  The step's start pose, velocities and
  // joint angles are read back from the helper waves' LDS copy (put_state, the same floats): their registers die
  // after the sin / cos instead of being parked through the ABA passes
  {
    float x[20];
    get4(H.st, threadIdx.x, x, 5);
    for (int i = 0; i < 3; ++i) { b.pos[i] = x[i]; b.vlin[i] = x[7 + i]; b.wang[i] = x[10 + i]; }
    for (int i = 0; i < 4; ++i) b.quat[i] = x[3 + i];
    for (int k = 0; k < NL; ++k) lg.q[k] = x[13 + k];
  }
  if (!P.fix_base) {
    float nd[6];
    for (int i = 0; i < 6; ++i) nd[i] = a0[i] + ag[i];
    float vb[3];
    mtv(R0, b.vlin, vb);
    float wxv[3];
    cross(b.wang, vb, wxv);
    float al[3] = {nd[3] + wxv[0], nd[4] + wxv[1], nd[5] + wxv[2]}, aw[3];
    mv(R0, al, aw);
    for (int i = 0; i < 3; ++i) { b.vlin[i] += h * aw[i]; b.wang[i] += h * nd[i]; }
    for (int i = 0; i < 3; ++i) b.pos[i] += h * b.vlin[i];
    quat_integrate(b.quat, b.wang, h);
  }
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    lg.qd[k] += h * qdd[k];
    float q = lg.q[k] + h * lg.qd[k];
    // hard-limit residual (oracle limit_projection): beyond the range by more than lproj -> back to the tolerance,
    // outward velocity zeroed; branch-free
    const float hi = h12m::QHI[k] + P.lproj, lo = h12m::QLO[k] - P.lproj;
    const bool over = q > hi, under = q < lo;
    lg.qd[k] = over ? fminf(lg.qd[k], 0.f) : (under ? fmaxf(lg.qd[k], 0.f) : lg.qd[k]);
    lg.q[k] = fminf(fmaxf(q, lo), hi);
  }
  if (more) {
    put_state(threadIdx.x, b, lg, org);
    SYNC_W(0);  // S: the next inner step's state
  }
  PHX(14);
}
// ------------------------------------------------------------------ state load / store
// Workspace access through buffer resources built from the kernargs (wave-uniform): the env's byte offset
// e*4 is the one per-lane VGPR (voffset), the field offset f*n*4 an SGPR (soffset).  Flat global accesses
// would keep a 64-bit address per field alive from the state loads to the stores (~200 registers).
// h12env_create bounds n so that every offset fits in 32 bits.
H12_DEV __amdgpu_buffer_rsrc_t ws_rsrc(void* base) { return __builtin_amdgcn_make_buffer_rsrc(base, 0, -1, 0x00020000); }
// f must be wave-uniform (soffset); a lane-dependent part of the field index (the leg) goes into lf
H12_DEV float ldf(const Workspace& W, int f, int e, int lf = 0) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ws_rsrc(W.F), (e + lf * W.n) * 4, f * W.n * 4, 0));
}
H12_DEV __amdgpu_buffer_rsrc_t st_F(const Workspace& W) { return ws_rsrc(W.F); }
H12_DEV __amdgpu_buffer_rsrc_t st_I(const Workspace& W) { return ws_rsrc(W.I); }
H12_DEV void stf(const Workspace& W, int f, int e, float x, int lf = 0) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, x), st_F(W), (e + lf * W.n) * 4, f * W.n * 4,
                                        ST_POL);
}
H12_DEV int ldi(const Workspace& W, int f, int e) {
  return (int)__builtin_amdgcn_raw_buffer_load_b32(ws_rsrc(W.I), e * 4, f * W.n * 4, 0);
}
H12_DEV void sti(const Workspace& W, int f, int e, int x, int lf = 0) {
  __builtin_amdgcn_raw_buffer_store_b32((uint32_t)x, st_I(W), (e + lf * W.n) * 4, f * W.n * 4, ST_POL);
}

struct EnvSt {
  Base b;
  Leg lg;                         // lane frame
  float act[NL], act1[NL];        // a_t, a_{t-1} of this leg (lane frame)
  float cmd[3], heading, cmd_time, push_t;
  float air, con, last_air, last_con;  // this lane's foot
  float epsum[H12_NREW];
  float metric[2];                // command metrics error_vel_xy, error_vel_yaw (episode accumulators)
  int eplen, lag[3], since_reset, is_heading, is_standing;
  float origin[3];                // env origin (terrain tasks)
  int tcell;                      // terrain level | type << 16
};

// physics part of the state (loaded before the physics loop)
template <int K>
H12_DEV void load_phys(const KParams& P, const Workspace& W, int e, int leg, EnvSt& s) {
  const float sg = leg ? -1.f : 1.f;
  for (int i = 0; i < 3; ++i) s.b.pos[i] = ldf(W, H12_F_POS + i, e);
  for (int i = 0; i < 4; ++i) s.b.quat[i] = ldf(W, H12_F_QUAT + i, e);
  for (int i = 0; i < 3; ++i) s.b.vlin[i] = ldf(W, H12_F_VLIN + i, e);
  for (int i = 0; i < 3; ++i) s.b.wang[i] = ldf(W, H12_F_WANG + i, e);
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    float js = jsign(k, sg);
    s.lg.q[k] = js * ldf(W, H12_F_Q + k, e, NL * leg);
    s.lg.qd[k] = js * ldf(W, H12_F_QD + k, e, NL * leg);
    s.act[k] = js * ldf(W, H12_F_ACT + k, e, NL * leg);
    s.act1[k] = js * ldf(W, H12_F_ACT_PREV + k, e, NL * leg);
  }
  int pk = ldi(W, H12_I_PACK, e);
  int cm = (pk >> (13 + 4 * leg)) & 0xF;
  s.lg.cmask = 0;
#pragma unroll
  for (int q = 0; q < H12_NFOOT_PTS; ++q) {
    int qr = leg ? (q ^ 1) : q;  // mirrored sole sphere q is real sphere q^1
    s.lg.anc[q][0] = ldf(W, H12_F_ANCHOR + 2 * q, e, 8 * leg + 2 * (qr - q));
    s.lg.anc[q][1] = sg * ldf(W, H12_F_ANCHOR + 2 * q + 1, e, 8 * leg + 2 * (qr - q));
    s.lg.cmask |= ((cm >> qr) & 1) << q;
  }
  for (int g = 0; g < 3; ++g) s.lag[g] = (pk >> (3 * g)) & 7;
  s.since_reset = (pk >> 9) & 3;
  s.is_heading = (pk >> 11) & 1;
  s.is_standing = (pk >> 12) & 1;
  const bool mu = Feat<K>::ext && P.env_mu;
  s.lg.mus = mu ? ldf(W, H12_F_MU, e, 2 * leg) : P.mus;
  s.lg.mud = mu ? ldf(W, H12_F_MU + 1, e, 2 * leg) : P.mud;
  s.lg.dmass = (Feat<K>::ext && P.env_mass) ? ldf(W, H12_F_DMASS, e) : 0.f;
}

// MDP part of the state (loaded after the physics loop)
// the episode reward sums of an env (step_kernel: the helper wave's, which computes the rewards)
template <int K>
H12_DEV void load_epsum(const KParams& P, const Workspace& W, int e, float* epsum) {
  for (int t = 0; t < H12_NREW_FLAT; ++t) epsum[t] = ldf(W, H12_F_EPSUM + t, e);
  for (int t = H12_NREW_FLAT; t < H12_NREW; ++t)
    epsum[t] = (Feat<K>::ext && P.rsl) ? ldf(W, H12_F_EPSUM2 + t - H12_NREW_FLAT, e) : 0.f;
}
// ... stored by the two lanes of the env (field t from the left lane, t + 6 from the right: one instruction per pair)
template <int K>
H12_DEV void store_epsum(const KParams& P, const Workspace& W0, int e, int leg, const float* epsum) {
  Workspace W = W0;
  asm volatile("" : "+s"(W.n));
  const uint32_t lm = 0u - (uint32_t)leg;
  auto lsel = [lm](float a, float b) {
    const uint32_t ua = __float_as_uint(a);
    return __uint_as_float(ua ^ ((ua ^ __float_as_uint(b)) & lm));
  };
#pragma unroll
  for (int t = 0; t < 6; ++t) stf(W, H12_F_EPSUM + t, e, lsel(epsum[t], epsum[t + 6]), 6 * leg);
  if (Feat<K>::ext && P.rsl) {
#pragma unroll
    for (int t = 0; t < 4; ++t)
      stf(W, H12_F_EPSUM2 + t, e, lsel(epsum[H12_NREW_FLAT + t], epsum[H12_NREW_FLAT + t + 4]), 4 * leg);
  }
}

// EPS: with the episode reward sums (step_kernel's physics wave leaves them to the helper wave)
template <int K, bool EPS = true>
H12_DEV void load_mdp(const KParams& P, const Workspace& W, int e, int leg, EnvSt& s) {
  for (int i = 0; i < 3; ++i) s.cmd[i] = ldf(W, H12_F_CMD + i, e);
  s.heading = ldf(W, H12_F_HEADING, e);
  s.cmd_time = ldf(W, H12_F_CMD_TIME, e);
  s.air = ldf(W, H12_F_AIR, e, leg);
  s.con = ldf(W, H12_F_CONTACT, e, leg);
  s.last_air = ldf(W, H12_F_LAST_AIR, e, leg);
  s.last_con = ldf(W, H12_F_LAST_CONTACT, e, leg);
  if (EPS) load_epsum<K>(P, W, e, s.epsum);
  else
    for (int t = 0; t < H12_NREW; ++t) s.epsum[t] = 0.f;
  s.push_t = (Feat<K>::ext && P.push) ? ldf(W, H12_F_PUSH_TIME, e) : 0.f;
  s.metric[0] = ldf(W, H12_F_METRIC, e);
  s.metric[1] = ldf(W, H12_F_METRIC + 1, e);
  s.eplen = ldi(W, H12_I_EPLEN, e);
  if (Feat<K>::terrain) {
    for (int i = 0; i < 3; ++i) s.origin[i] = ldf(W, H12_F_ORIGIN + i, e);
    s.tcell = ldi(W, H12_I_TERRAIN, e);
  } else {
    s.origin[0] = s.origin[1] = s.origin[2] = 0.f;
    s.tcell = 0;
  }
}

template <int K>
H12_DEV void load_env(const KParams& P, const Workspace& W, int e, int leg, EnvSt& s) {
  load_phys<K>(P, W, e, leg, s);
  load_mdp<K>(P, W, e, leg, s);
}

// PARTS: bit 0 the physics state (base pose / velocity, q, qd, stiction anchors), bit 1 everything else but the episode
// reward sums, bit 2 those (step_kernel: the helper wave stores them)
template <int K, int PARTS = 7>
H12_DEV void store_env(const KParams& P, const Workspace& W0, int e, int leg, const EnvSt& s) {
  constexpr bool PH_ = PARTS & 1, RE_ = PARTS & 2, EP_ = PARTS & 4;
  const float sg = leg ? -1.f : 1.f;
  // an opaque copy of n made here: the field offsets of the stores are then computed here, not shared with the
  // loads at the top of the kernel (68 SGPRs kept live across the physics loop spill to VGPR lanes)
  Workspace W = W0;
  asm volatile("" : "+s"(W.n));
  if (RE_ && Feat<K>::terrain && leg == 0) {
    for (int i = 0; i < 3; ++i) stf(W, H12_F_ORIGIN + i, e, s.origin[i]);
    sti(W, H12_I_TERRAIN, e, s.tcell);
  }
  // Env-level fields (base, command, episode sums) hold bit-identical copies in both legs' lanes: each store
  // instruction writes two of them, field f from the left lane and f + D from the right (lane offset leg * D).
  // The write-back is bound by the chip-wide rate of store instructions, so this halves
  // the 30 single-lane stores of this block.
  // the right lane's value selected by bit masking: a ?: chain over neighbouring fields of one struct is turned
  // into a dynamic index (scratch)
  const uint32_t lm = 0u - (uint32_t)leg;
  auto lsel = [lm](float a, float b) {
    const uint32_t ua = __float_as_uint(a);
    return __uint_as_float(ua ^ ((ua ^ __float_as_uint(b)) & lm));
  };
  {
    const float bb[13] = {s.b.pos[0],  s.b.pos[1],  s.b.pos[2],  s.b.quat[0], s.b.quat[1], s.b.quat[2], s.b.quat[3],
                          s.b.vlin[0], s.b.vlin[1], s.b.vlin[2], s.b.wang[0], s.b.wang[1], s.b.wang[2]};
    static_assert(H12_F_QUAT == H12_F_POS + 3 && H12_F_VLIN == H12_F_POS + 7 && H12_F_WANG == H12_F_POS + 10,
                  "base fields contiguous");
    if (PH_) {
#pragma unroll
      for (int i = 0; i < 6; ++i) stf(W, H12_F_POS + i, e, lsel(bb[i], bb[i + 7]), 7 * leg);
      if (leg == 0) stf(W, H12_F_POS + 6, e, bb[6]);
    }
    if (RE_) {
      static_assert(H12_F_HEADING == H12_F_CMD + 3 && H12_F_CMD_TIME == H12_F_CMD + 4, "command fields contiguous");
      stf(W, H12_F_CMD, e, lsel(s.cmd[0], s.heading), 3 * leg);
      stf(W, H12_F_CMD + 1, e, lsel(s.cmd[1], s.cmd_time), 3 * leg);
      if (EP_) {
#pragma unroll
        for (int t = 0; t < 6; ++t) stf(W, H12_F_EPSUM + t, e, lsel(s.epsum[t], s.epsum[t + 6]), 6 * leg);
        if (Feat<K>::ext && P.rsl) {
#pragma unroll
          for (int t = 0; t < 4; ++t)
            stf(W, H12_F_EPSUM2 + t, e, lsel(s.epsum[H12_NREW_FLAT + t], s.epsum[H12_NREW_FLAT + t + 4]), 4 * leg);
        }
      }
      if (leg == 0) {
        stf(W, H12_F_CMD + 2, e, s.cmd[2]);
        if (Feat<K>::ext && P.push) stf(W, H12_F_PUSH_TIME, e, s.push_t);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    float js = jsign(k, sg);
    if (PH_) {
      stf(W, H12_F_Q + k, e, js * s.lg.q[k], NL * leg);
      stf(W, H12_F_QD + k, e, js * s.lg.qd[k], NL * leg);
    }
    if (RE_) {
      stf(W, H12_F_ACT + k, e, js * s.act[k], NL * leg);
      stf(W, H12_F_ACT_PREV + k, e, js * s.act1[k], NL * leg);
    }
  }
  int cm_real = 0;
#pragma unroll
  for (int q = 0; q < H12_NFOOT_PTS; ++q) {
    int qr = leg ? (q ^ 1) : q;
    if (PH_) {
      stf(W, H12_F_ANCHOR + 2 * q, e, s.lg.anc[q][0], 8 * leg + 2 * (qr - q));
      stf(W, H12_F_ANCHOR + 2 * q + 1, e, sg * s.lg.anc[q][1], 8 * leg + 2 * (qr - q));
    }
    cm_real |= ((s.lg.cmask >> q) & 1) << qr;
  }
  if (!RE_) return;
  stf(W, H12_F_METRIC, e, lsel(s.metric[0], s.metric[1]), leg);
  stf(W, H12_F_AIR, e, s.air, leg);
  stf(W, H12_F_CONTACT, e, s.con, leg);
  stf(W, H12_F_LAST_AIR, e, s.last_air, leg);
  stf(W, H12_F_LAST_CONTACT, e, s.last_con, leg);
  int cm_other = pair_swap_i(cm_real);
  int pk = 0;
  for (int g = 0; g < 3; ++g) pk |= (s.lag[g] & 7) << (3 * g);
  pk |= (s.since_reset & 3) << 9;
  pk |= (s.is_heading & 1) << 11;
  pk |= (s.is_standing & 1) << 12;
  pk |= (cm_real & 0xF) << 13;  // the left lane's own masks are the left foot's: its pack is the one stored
  pk |= (cm_other & 0xF) << 17;
  // one instruction: the left lane stores the pack word, the right lane the (identical) episode length
  static_assert(H12_I_EPLEN == 0 && H12_I_PACK == 1, "int fields");
  sti(W, H12_I_EPLEN, e, (int)(((uint32_t)pk & ~lm) | ((uint32_t)s.eplen & lm)), 1 - leg);
}

// ------------------------------------------------------------------ MDP pieces
H12_DEV void rng(const KParams& P, uint32_t g, uint32_t lo, uint32_t hi, int stream, int block, uint32_t out[4]) {
  philox(P.seed_lo, P.seed_hi, g, lo, ((uint32_t)stream << 16) | (uint32_t)block, hi, out);
}

H12_DEV float wrap_pi(float x) {
  const float TWO_PI = 6.283185307179586f, PI_F = 3.141592653589793f;
  float r = fmodf(x, TWO_PI);
  if (r < 0.f) r += TWO_PI;
  return r > PI_F ? r - TWO_PI : r;
}

// CommandTerm._resample: UniformVelocityCommand._resample_command (upstream; in-repo twin
// utils/mdp/commands.py:19-59) + time_left ~ U(resampling_time_range).  blk: first of the two Philox blocks
// (0: reset / time-out resample, 3: the deadzone's re-activation resample of the same step)
H12_DEV void cmd_resample(const KParams& P, EnvSt& s, uint32_t g, uint32_t lo, uint32_t hi, int blk = 0,
                          const uint32_t* pre = nullptr) {
  uint32_t r0[4], r1[4];
  if (pre) {  // blk 0's two blocks drawn ahead by the helper wave (reset_draws)
    for (int i = 0; i < 4; ++i) { r0[i] = pre[i]; r1[i] = pre[4 + i]; }
  } else {
    rng(P, g, lo, hi, ST_CMD, blk, r0);
    rng(P, g, lo, hi, ST_CMD, blk + 1, r1);
  }
  s.cmd[0] = uab(r0[0], P.cmd_x0, P.cmd_x1);
  s.cmd[1] = uab(r0[1], P.cmd_y0, P.cmd_y1);
  s.cmd[2] = uab(r0[2], P.cmd_w0, P.cmd_w1);
  s.heading = uab(r0[3], P.cmd_h0, P.cmd_h1);
  s.is_heading = u01(r1[0]) <= P.rel_head;
  s.is_standing = u01(r1[1]) <= P.rel_stand;
  s.cmd_time = uab(r1[2], P.cmd_T, P.cmd_T1);
}

// UniformVelocityCommand._update_command (heading control, standing envs), or with P.dz the Rsl/CaT
// UniformVelocityCommandWithDeadzone._update_command (utils/mdp/commands.py:41-96): keep half of the envs
// in the deadzone |cmd_xy| < v_dz -- with too few, each active env is zeroed with probability
// (target - count) / (n - count); with too many, each deadzone env is resampled with probability
// (count - target) / count -- which is the per-env marginal of the reference's randperm selection.  The
// count is the previous step's (dz_prev; a grid-wide count of this step would need a second pass); for
// the shipped velocity_deadzone = 0 it is 0 and the rule is exact.  Then cmd_z flips sign with
// probability physics_dt / episode_length_s.  Standing envs are not zeroed in this class.
template <int K>
H12_DEV void cmd_update(const KParams& P, EnvSt& s, uint32_t g, uint32_t lo, uint32_t hi, int dz_prev, int n) {
  if (s.is_heading) {
    float R[3][3];
    quat_R(s.b.quat, R);
    float hw = atan2f(R[1][0], R[0][0]);
    float w = P.head_k * wrap_pi(s.heading - hw);
    s.cmd[2] = fminf(fmaxf(w, P.cmd_w0), P.cmd_w1);
  }
  if (Feat<K>::ext && P.dz) {
    uint32_t r[4];
    rng(P, g, lo, hi, ST_CMD, 2, r);
    const int target = n / 2;
    const bool in_dz = s.cmd[0] * s.cmd[0] + s.cmd[1] * s.cmd[1] < P.dz_v * P.dz_v;
    // Bernoulli(num / den) on the 24-bit uniform u: u * den < num * 2^24, exact in integers
    const uint64_t u24 = r[0] >> 8;
    if (dz_prev < target) {
      if (!in_dz && u24 * (uint64_t)(n - dz_prev) < ((uint64_t)(target - dz_prev) << 24)) s.cmd[0] = s.cmd[1] = 0.f;
    } else if (dz_prev > target) {
      if (in_dz && u24 * (uint64_t)dz_prev < ((uint64_t)(dz_prev - target) << 24)) cmd_resample(P, s, g, lo, hi, 3);
    }
    if (u01(r[1]) < P.flip_p) s.cmd[2] = -s.cmd[2];
    return;
  }
  if (s.is_standing) s.cmd[0] = s.cmd[1] = s.cmd[2] = 0.f;
}

// ---- CaT constraints (T/utils/cat/constraints.py) on the pre-reset state of the step, raw values into the
// scratch [col][n] (each lane its leg's joint columns and its foot's columns, lane 0 of the pair the base
// ones), the no_move activity flag and the pre-reset episode length for cat_prob_kernel.  foot_clearance
// keeps its swing state (max foot height since the last touchdown) in H12_F_SWING_H; WB = false (the term-evaluation
// hook) evaluates the constraint on the stored swing state and writes the updated one to rows CAT_ROWS + leg of
// the caller's buffer instead of the workspace.
template <int LINK>
H12_DEV void link_pos(const Leg& lg, float (&R)[3][3], float* p) {
  float sn, cs;
  fsincos(lg.q[LINK], &sn, &cs);
  float Rr[3];
  mv(R, h12m::R[LINK], Rr);
  p[0] += Rr[0]; p[1] += Rr[1]; p[2] += Rr[2];
  rmul_axis<AX[LINK]>(R, cs, sn);
}

// constraints.no_move applies while every command component is inside the deadzone
H12_DEV bool cat_still(const KParams& P, const EnvSt& s) {
  return fabsf(s.cmd[0]) < P.c_nm_dz && fabsf(s.cmd[1]) < P.c_nm_dz && fabsf(s.cmd[2]) < P.c_nm_dz;
}

template <bool LDS, bool WB = true>
H12_DEV void cat_constraints(const KParams& P, const Workspace& W, int e, int leg, const EnvSt& s, const float* tau,
                             float fmax_foot, int term, const float R[3][3], int eplen_pre) {
  const int n = W.n;
  float* S = P.cscr;
  // every value also goes to the block's LDS copy (step_kernel): the helper wave forms the block's column maxima
  auto put = [&](int row, float v) {
    S[(size_t)row * n + e] = v;
    if constexpr (LDS) {
      if (row <= CAT_ROW_EPLEN) cat_lds()[row][e & (ENVS_PER_BLOCK - 1)] = v;
    }
  };
  const float sg = leg ? -1.f : 1.f;
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    const int j = NL * leg + k;
    const float q = s.lg.q[k], qd = fabsf(s.lg.qd[k]);
    put((C_COL0[H12_C_JOINT_POS_LIMITS] + j), fmaxf(soft_lo(P, k) - q, q - soft_hi(P, k)));
    put((C_COL0[H12_C_JOINT_VEL_LIMITS] + j), qd - P.cvlim[k]);
    put((C_COL0[H12_C_JOINT_TORQUE_LIMITS] + j), fabsf(tau[k]) - P.celim[k]);
    put((C_COL0[H12_C_NO_MOVE] + j), qd - P.c_nm_v);
  }
  put((C_COL0[H12_C_FOOT_CONTACT_FORCE] + leg), fmax_foot - P.c_ff);
  // foot_clearance: touchdown = ContactSensor.compute_first_contact(step_dt); command active = any |cmd| > dz
  {
    const bool touchdown = s.con > 0.f && s.con < P.step_dt + 1e-8f;
    const bool active = fabsf(s.cmd[0]) > P.c_clr_dz || fabsf(s.cmd[1]) > P.c_clr_dz || fabsf(s.cmd[2]) > P.c_clr_dz;
    float Rf[3][3];
    const float mm[3] = {1.f, sg, 1.f};
    for (int i = 0; i < 3; ++i)
      for (int jj = 0; jj < 3; ++jj) Rf[i][jj] = mm[i] * mm[jj] * R[i][jj];
    float p[3] = {0.f, 0.f, 0.f};
    link_pos<0>(s.lg, Rf, p); link_pos<1>(s.lg, Rf, p); link_pos<2>(s.lg, Rf, p);
    link_pos<3>(s.lg, Rf, p); link_pos<4>(s.lg, Rf, p); link_pos<5>(s.lg, Rf, p);
    const float foot_z = s.b.pos[2] + p[2];  // body_link_pos_w z of the ankle-roll link
    float& sw = W.F[(size_t)(H12_F_SWING_H + leg) * n + e];
    const float sh = sw;
    put((C_COL0[H12_C_FOOT_CLEARANCE] + leg), (touchdown && active) ? (P.c_clr - sh) : 0.f);
    const float sw_new = touchdown ? 0.f : fmaxf(sh, foot_z);
    if constexpr (WB) sw = sw_new;
    else S[(size_t)(CAT_ROWS + leg) * n + e] = sw_new;  // the hook: to the caller's rows, workspace untouched
  }
  const int nfeet = (fmax_foot > 1.0f ? 1 : 0) + (pair_swap(fmax_foot) > 1.0f ? 1 : 0);
  if (leg == 0) {
    put(C_COL0[H12_C_CONTACT], term ? 1.f : 0.f);
    const float gx = R[2][0], gy = R[2][1];  // projected gravity xy (sign irrelevant under the norm)
    put(C_COL0[H12_C_BASE_ORIENTATION], fsqrt(gx * gx + gy * gy) - P.c_or);
    const float z = s.b.pos[2];
    put(C_COL0[H12_C_BASE_HEIGHT], (z < P.c_h - P.c_hstd || z > P.c_h + P.c_hstd) ? 1.f : 0.f);
    put(C_COL0[H12_C_FOOT_CONTACT], (nfeet < 1 || nfeet > 2) ? 1.f : 0.f);
    put(CAT_ROW_NOMOVE, cat_still(P, s) ? 1.f : 0.f);
    put(CAT_ROW_EPLEN, (float)eplen_pre);
  }
}

// push_by_setting_velocity as an interval event (EventManager.apply(mode="interval"), rsl_env_cfg.py:262-273):
// time_left -= step_dt; at < 1e-6 a new interval is drawn and U(range) is added to the root x / y velocity
template <int K>
H12_DEV void push_event(const KParams& P, EnvSt& s, uint32_t g, uint32_t lo, uint32_t hi) {
  if (!(Feat<K>::ext && P.push)) return;
  s.push_t -= P.step_dt;
  if (s.push_t < 1e-6f) {
    uint32_t r[4];
    rng(P, g, lo, hi, ST_PUSH, 0, r);
    s.push_t = uab(r[2], P.push_t0, P.push_t1);
    s.b.vlin[0] += uab(r[0], P.push_x0, P.push_x1);
    s.b.vlin[1] += uab(r[1], P.push_y0, P.push_y1);
  }
}

// _reset_idx: scene reset (delay lags, sensors), reset events, manager resets (cat_env.py:195-248)
template <int K>
H12_DEV void env_reset(const KParams& P, EnvSt& s, int leg, uint32_t g, uint32_t lo, uint32_t hi,
                       const uint32_t* pre = nullptr) {
  uint32_t r0[4], r1[4];
  if (pre) {  // drawn ahead by the helper wave (reset_draws): ST_RESET blocks 0, 1, then ST_CMD blocks 0, 1
    for (int i = 0; i < 4; ++i) { r0[i] = pre[i]; r1[i] = pre[4 + i]; }
  } else {
    rng(P, g, lo, hi, ST_RESET, 0, r0);
    rng(P, g, lo, hi, ST_RESET, 1, r1);
  }
  if (Feat<K>::terrain && P.curriculum) {
    // CurriculumManager.compute runs first in _reset_idx, on the pre-reset state:
    // terrain_levels_vel (velocity/mdp/curriculums.py:21-52) + TerrainImporter.update_env_origins
    float dx = s.b.pos[0] - s.origin[0], dy = s.b.pos[1] - s.origin[1];
    float dist = fsqrt(dx * dx + dy * dy);
    bool up = dist > 0.5f * P.terrain_size;
    bool down = !up && dist < fsqrt(s.cmd[0] * s.cmd[0] + s.cmd[1] * s.cmd[1]) * P.ep_len_s * 0.5f;
    int lvl = (s.tcell & 0xFFFF) + (up ? 1 : 0) - (down ? 1 : 0);
    const int typ = s.tcell >> 16;
    if (lvl >= P.t_rows) {
      uint32_t r2[4];
      rng(P, g, lo, hi, ST_RESET, 2, r2);
      lvl = (int)(r2[0] % (uint32_t)P.t_rows);
    }
    lvl = max(lvl, 0);
    s.tcell = lvl | (typ << 16);
    const float* o = P.t_origin + 3 * ((size_t)lvl * P.t_cols + typ);
    s.origin[0] = o[0]; s.origin[1] = o[1]; s.origin[2] = o[2];
  }
  // reset_root_state_uniform: default root state + env origin + uniform pose offsets
  s.b.pos[0] = s.origin[0] + uab(r0[0], P.rx0, P.rx1);
  s.b.pos[1] = s.origin[1] + uab(r0[1], P.ry0, P.ry1);
  s.b.pos[2] = s.origin[2] + P.root_z;
  float yaw = uab(r0[2], P.ryaw0, P.ryaw1);
  float sy, cy;
  sincosf(0.5f * yaw, &sy, &cy);
  s.b.quat[0] = cy; s.b.quat[1] = 0.f; s.b.quat[2] = 0.f; s.b.quat[3] = sy;
  for (int i = 0; i < 3; ++i) { s.b.vlin[i] = 0.f; s.b.wang[i] = 0.f; }
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    // reset_joints_by_scale (x1.0) clamped to the soft limits, in the lane frame
    s.lg.q[k] = fminf(fmaxf(h12m::Q0[k], soft_lo(P, k)), soft_hi(P, k));
    s.lg.qd[k] = 0.f;
    s.act[k] = 0.f;
    s.act1[k] = 0.f;
  }
  for (int q = 0; q < H12_NFOOT_PTS; ++q) { s.lg.anc[q][0] = 0.f; s.lg.anc[q][1] = 0.f; }
  s.lg.cmask = 0;
  uint32_t span = (uint32_t)(P.max_delay - P.min_delay + 1);
  s.lag[0] = P.min_delay + (int)(r0[3] % span);
  s.lag[1] = P.min_delay + (int)(r1[0] % span);
  s.lag[2] = P.min_delay + (int)(r1[1] % span);
  s.since_reset = 0;
  s.air = s.con = s.last_air = s.last_con = 0.f;
  for (int t = 0; t < H12_NREW; ++t) s.epsum[t] = 0.f;
  s.metric[0] = s.metric[1] = 0.f;  // CommandTerm.reset
  s.eplen = 0;
  if (Feat<K>::ext && P.push) {  // EventManager.reset: a new push interval for the reset envs
    uint32_t r3[4];
    rng(P, g, lo, hi, ST_RESET, 3, r3);
    s.push_t = uab(r3[0], P.push_t0, P.push_t1);
  }
  cmd_resample(P, s, g, lo, hi, 0, pre ? pre + 8 : nullptr);
}

// root (composite COM) linear velocity in world: v_origin + w x (R c); c moves with the added torso mass
template <int K>
H12_DEV void base_com_vel(const KParams& P, const EnvSt& s, const float R[3][3], float* vcom) {
  // the pelvis rigid body's own COM (the added torso mass sits on torso_link, another rigid body)
  const float c[3] = {h12m::ROOT_COM[0], h12m::ROOT_COM[1], h12m::ROOT_COM[2]};
  float ww[3], cw[3], wxc[3];
  mv(R, s.b.wang, ww);
  mv(R, c, cw);
  cross(ww, cw, wxc);
  for (int a = 0; a < 3; ++a) vcom[a] = s.b.vlin[a] + wxc[a];
}

// UniformVelocityCommand._update_metrics (IsaacLab 2.1): per step, |v*_xy - v_b,xy| and |w*_z - w_b,z| / (the
// resampling time range's upper end in steps), v_b = root_lin_vel_b (COM velocity in the base frame), w_b the
// base angular velocity; CommandTerm.reset logs their means over the reset envs and zeroes them (env_reset).
template <int K>
H12_DEV void cmd_metrics(const KParams& P, EnvSt& s) {
  float R[3][3], vcom[3], vb[3];
  quat_R(s.b.quat, R);
  base_com_vel<K>(P, s, R, vcom);
  mtv(R, vcom, vb);
  const float ex = s.cmd[0] - vb[0], ey = s.cmd[1] - vb[1];
  const float w = P.step_dt * frcp(P.cmd_T1);  // 1 / max_command_step
  s.metric[0] += fsqrt(ex * ex + ey * ey) * w;
  s.metric[1] += fabsf(s.cmd[2] - s.b.wang[2]) * w;
}

// this lane's part of the new (noise-free) observation frame, real coordinates, into the frame
// scratch laid out [rows][n] (coalesced across the wave).  Noise / history / height scan are added by
// the assembly kernels.  Flat: 45 rows (ang_vel, gravity, command, q-q0, qd, action).  Rough: base_lin_vel
// first (48 rows), then base position (3) and yaw cos / sin (2) for the height scan.
template <int K>
H12_DEV void obs_frame(const KParams& P, const EnvSt& s, int leg, int e, int n, float* frame) {
  const float sg = leg ? -1.f : 1.f;
  const int o = (Feat<K>::ext && P.task == H12_TASK_ROUGH) ? 3 : 0;
  if (leg == 0) {
    float R[3][3];
    quat_R(s.b.quat, R);
    if (o) {
      float vcom[3], vb[3];
      base_com_vel<K>(P, s, R, vcom);
      mtv(R, vcom, vb);
      for (int a = 0; a < 3; ++a) frame[(size_t)a * n + e] = vb[a];
      for (int a = 0; a < 3; ++a) frame[(size_t)(H12_ROUGH_FRAME + a) * n + e] = s.b.pos[a];
      float hx = R[0][0], hy = R[1][0], hn = __builtin_amdgcn_rsqf(hx * hx + hy * hy);
      frame[(size_t)(H12_ROUGH_FRAME + 3) * n + e] = hx * hn;
      frame[(size_t)(H12_ROUGH_FRAME + 4) * n + e] = hy * hn;
    }
    for (int a = 0; a < 3; ++a) frame[(size_t)(o + a) * n + e] = s.b.wang[a];
    for (int a = 0; a < 3; ++a) frame[(size_t)(o + 3 + a) * n + e] = -R[2][a];
    for (int a = 0; a < 3; ++a) frame[(size_t)(o + 6 + a) * n + e] = s.cmd[a];
  }
  // joint rows: values materialised first, then stored back to back through a buffer resource (see store_env)
  float jv[3 * NL];
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    float js = jsign(k, sg);
    jv[k] = js * (s.lg.q[k] - h12m::Q0[k]);
    jv[NL + k] = js * s.lg.qd[k];
    jv[2 * NL + k] = js * s.act[k];
  }
  for (auto& x : jv) asm volatile("" : "+v"(x));
  __builtin_amdgcn_sched_barrier(0);
  const auto rs = ws_rsrc(frame);
  const int vo = (e + NL * leg * n) * 4;
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, jv[k]), rs, vo, (o + 9 + k) * n * 4, 0);
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, jv[NL + k]), rs, vo, (o + 21 + k) * n * 4, 0);
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, jv[2 * NL + k]), rs, vo, (o + 33 + k) * n * 4, 0);
  }
}

// noise index of frame component c (ang_vel 0-2, gravity 3-5, joint_pos 6-17, joint_vel 18-29;
// command and last action are noise-free: -1)
H12_DEV int noise_index(int c) { return c < 6 ? c : (c < 9 ? -1 : (c < 33 ? c - 3 : -1)); }
// observation term of frame component c: ang_vel 0, gravity 1, command 2, q-q0 3, qd 4, action 5
H12_DEV int term_index(int c) { return c < 9 ? c / 3 : 3 + (c - 9) / 12; }

// additive uniform noise of noise index t (ObservationTermCfg noise=Unoise(-n, n)); 0 when off
H12_DEV float noise_of(const KParams& P, int t, uint32_t r) {
  float nmax = t < 3 ? P.n_w : (t < 6 ? P.n_g : (t < 18 ? P.n_q : P.n_qd));
  return P.corrupt ? (-nmax + 2.f * nmax * u01(r)) : 0.f;
}

// ObservationManager.compute + CircularBuffer.append for a batch of envs, full-chip.  One block owns
// ASM_ROWS whole rows (4 x 1800 B, 16-byte aligned): the rows are staged into LDS by LDS-DMA
// (global_load_lds_dwordx4), the frame's component-major rows are read alongside, each row's 8 Philox noise blocks
// are drawn once (one thread each) and added to the frame in LDS, and every output float4 is assembled
// from LDS through a column table -- the shifted history obs[e, slot h] = obs_prev[e, slot h + 1]
// (h < 9), or the noisy new frame in the newest slot and in every slot of a row being (re)filled -- and
// stored with one float4 store.  All global reads precede the first barrier, so obs may alias obs_prev.
// Reset mode: rows with sel[e] (all if sel is NULL) are filled, the others are rewritten unchanged
// from obs itself.  Otherwise fill[e] = fill_a[e] | fill_b[e].
// XCD-aware block order: the dispatcher deals blocks round-robin over the 8 XCDs (blocks b and b + 8 share one
// XCD and its L2; MI355X_MICROARCH.md, workgroup dispatch), so consecutive logical blocks -- which share cache
// lines of the [45][n] frame scratch (a 128-B line holds 32 envs' component = 8 blocks of 4 rows) and the row
// boundaries -- are mapped to one XCD: logical block = (b % 8) * q + min(b % 8, r) + b / 8 with nb = 8 q + r.
// Affinity only (placement is not a contract); a bijection on [0, nb).
H12_DEV int xcd_block(int b, int nb) {
  const int x = b & 7, k = b >> 3, q = nb >> 3, r = nb & 7;
  return x * q + min(x, r) + k;
}

struct AsmArgs {
  const float* obs_prev;
  float* obs;
  const float* frame;
  const uint8_t* fill_a;
  const uint8_t* fill_b;
  const uint8_t* sel;
  int reset_mode;
  int vec;  // obs and the source rows are 16-byte aligned
  const int16_t* tab;  // gather table (asm_gather_table) for the whole-block path of step / observe, or null
  int n;
  int64_t env_offset;
  uint32_t lo, hi;
  float* log_part;  // step_kernel's per-block episode-log partials ([LOG_NPART][log_nb]) ...
  float* log_acc;   // ... folded into the caller's accumulator by block 0 (null: nothing to fold)
  int log_nb;
  float* frame_out; // (n, 45) the new frames as they enter the history (h12env_step_out.frame_out), or null
};
constexpr int ASM_BLOCK = 256;

// Episode-log fold, in the assembly kernel: block pv < LOG_NPART (its first wave) sums step_kernel's partials of
// value pv over the step's blocks into log_acc[log_slot(pv)] and zeroes them for the next step (stream order:
// step_kernel wrote them, the next step_kernel starts after this kernel).  The loads are issued when the block
// starts (log_load) and consumed when it ends (log_fold), so their round trip hides behind the block's own work.
H12_DEV bool log_block(const AsmArgs& A) { return A.log_acc && blockIdx.x < LOG_NPART && threadIdx.x < 64; }
H12_DEV float log_load(const AsmArgs& A) {
  float acc = 0.f;
  if (log_block(A)) {
    const float* q = A.log_part + (size_t)blockIdx.x * A.log_nb;
    for (int b = threadIdx.x; b < A.log_nb; b += 64) acc += q[b];
  }
  return acc;
}
H12_DEV void log_fold_one(const AsmArgs& A, int pv, float acc) {
  float* q = A.log_part + (size_t)pv * A.log_nb;
  for (int b = threadIdx.x; b < A.log_nb; b += 64) q[b] = 0.f;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (threadIdx.x == 0 && acc != 0.f) A.log_acc[log_slot(pv)] += acc;
}
H12_DEV void log_fold(const AsmArgs& A, float acc) {
  if (!log_block(A)) return;
  log_fold_one(A, blockIdx.x, acc);
  // a grid smaller than LOG_NPART (a few envs): the remaining values, one round trip each
  for (int pv = blockIdx.x + gridDim.x; pv < LOG_NPART; pv += gridDim.x) {
    float a = 0.f;
    const float* q = A.log_part + (size_t)pv * A.log_nb;
    for (int b = threadIdx.x; b < A.log_nb; b += 64) a += q[b];
    log_fold_one(A, pv, a);
  }
}
constexpr int ASM_ROWS = 4;  // rows per block (the frame's [45][n] rows are read in 4*ROWS-byte segments)
static_assert((ASM_ROWS * H12_OBS_FRAME) % 4 == 0, "float4 rows for every history length");
static_assert(ASM_ROWS * 8 <= ASM_BLOCK, "one Philox block per thread");

H12_DEV bool asm_row_written(const AsmArgs& A, int e, bool& fill) {
  // no short-circuit on the byte loads: both are issued together (uniform pointer checks only)
  const int sel = A.sel ? (int)A.sel[e] : 1;
  const int fa = A.fill_a ? (int)A.fill_a[e] : 0;
  const int fb = A.fill_b ? (int)A.fill_b[e] : 0;
  if (A.reset_mode) {
    fill = true;
    return sel != 0;
  }
  fill = (fa | fb) != 0;
  return true;
}

// column table entry of row-local column col of a 45 x NH row (term-major blocks of 3NH, 3NH, 3NH, 12NH,
// 12NH, 12NH floats, oldest slot first): frame component c (bits 0-7), history shift d (bits 8-15),
// newest-slot flag (bit 16)
H12_DEV uint32_t hist_col_entry(int col, int nh) {
  int c, hh, d;
  if (col < 9 * nh) {
    int t = col / (3 * nh), r = col - 3 * nh * t;
    hh = r / 3;
    c = 3 * t + (r - 3 * hh);
    d = 3;
  } else {
    int k = col - 9 * nh, t = k / (12 * nh), r = k - 12 * nh * t;
    hh = r / 12;
    c = 9 + 12 * t + (r - 12 * hh);
    d = 12;
  }
  return (uint32_t)c | ((uint32_t)d << 8) | (hh == nh - 1 ? (1u << 16) : 0u);
}
template <int NH>
H12_DEV uint32_t asm_col_entry(int col) { return hist_col_entry(col, NH); }

// NH: history length (10 Flat, 6 Rsl); the row is 45 * NH floats
template <int NH>
H12_DEV void obs_assemble_body(const KParams& P, const AsmArgs& A) {
  constexpr int ROW = H12_OBS_FRAME * NH;
  constexpr int ASM_F4 = ASM_ROWS * ROW / 4;
  constexpr int ASM_CHUNKS = (ASM_F4 + 63) / 64;  // 1 KB LDS-DMA chunks (64 lanes x 16 B) per block
  // rows, then the noisy scaled frames right behind them (the gather table addresses both from s_hist)
  __shared__ __attribute__((aligned(16))) float s_hist[ASM_ROWS * (ROW + H12_OBS_FRAME)];
  float* s_frame = s_hist + ASM_ROWS * ROW;
  __shared__ float s_noise[ASM_ROWS * 32];
  __shared__ uint32_t s_col[ROW];
  __shared__ int s_write[ASM_ROWS], s_fill[ASM_ROWS];
  const int n = A.n;
  const int tid = threadIdx.x;
  const int r0 = xcd_block(blockIdx.x, gridDim.x) * ASM_ROWS;
  const int rows = min(ASM_ROWS, n - r0);
  const bool full = A.vec && rows == ASM_ROWS;
  const size_t base = (size_t)r0 * ROW;
  const float* src = (A.reset_mode ? A.obs : A.obs_prev) + base;
  // phase 1: all global reads (rows -> LDS, raw frames, flags), noise draws, column table
  // every global load is issued before the first LDS write (one memory round trip per wave; indices
  // are clamped instead of guarded so the loads stay unconditional and batched); the Philox draws run
  // while they are in flight
  bool fill_flag = false;
  const int fe = r0 + min(tid, rows - 1);
  const bool write_flag = asm_row_written(A, fe, fill_flag) && tid < rows;
  constexpr int NFR = (ASM_ROWS * H12_OBS_FRAME + ASM_BLOCK - 1) / ASM_BLOCK;
  float fv[NFR];
  if (full) {
    // rows -> LDS by LDS-DMA (global_load_lds_dwordx4): no register round trip, drained at the barrier
    // (the last chunk's surplus lanes are masked off: the frames live right behind the rows)
    const int wave = tid >> 6, lane = tid & 63;
    for (int ch = wave; ch < ASM_CHUNKS; ch += ASM_BLOCK / 64) {
      const float4* g = reinterpret_cast<const float4*>(src) + ch * 64 + lane;
      if (ch * 64 + lane < ASM_F4)
        __builtin_amdgcn_global_load_lds((const void*)g, (__attribute__((address_space(3))) void*)(s_hist + ch * 256),
                                         16, 0, 0);
    }
  }
  // gather path (step / observe, whole aligned blocks): each output float4 reads 4 int16 source offsets
  const bool gather = full && !A.reset_mode && A.tab;
  constexpr int NG = (ASM_F4 + ASM_BLOCK - 1) / ASM_BLOCK;
  uint2 gt[NG];
  if (gather) {
#pragma unroll
    for (int u = 0; u < NG; ++u) gt[u] = reinterpret_cast<const uint2*>(A.tab)[min(u * ASM_BLOCK + tid, ASM_F4 - 1)];
  }
#pragma unroll
  for (int u = 0; u < NFR; ++u) {
    int k = min(u * ASM_BLOCK + tid, ASM_ROWS * H12_OBS_FRAME - 1);
    int c = k / ASM_ROWS, row = min(k - c * ASM_ROWS, rows - 1);  // component-major: ROWS envs per component
    fv[u] = A.frame[(size_t)c * n + r0 + row];
  }
  for (int col = tid; col < ROW; col += ASM_BLOCK) s_col[col] = asm_col_entry<NH>(col);
  if (tid < ASM_ROWS) {
    s_write[tid] = write_flag ? 1 : 0;
    s_fill[tid] = fill_flag ? 1 : 0;
  }
  if (tid < 8 * rows) {
    int row = tid >> 3, blk = tid & 7;
    uint32_t r[4];
    philox(P.seed_lo, P.seed_hi, (uint32_t)(A.env_offset + r0 + row), A.lo, ((uint32_t)ST_OBS << 16) | (uint32_t)blk,
           A.hi, r);
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      int t = 4 * blk + a;
      s_noise[row * 32 + t] = t < 30 ? noise_of(P, t, r[a]) : 0.f;
    }
  }
  if (!full) {
    for (int j = tid; j < rows * ROW; j += ASM_BLOCK) s_hist[j] = src[j];
  }
#pragma unroll
  for (int u = 0; u < NFR; ++u) {
    int k = u * ASM_BLOCK + tid;
    int c = k / ASM_ROWS, row = k - c * ASM_ROWS;
    if (k < ASM_ROWS * H12_OBS_FRAME) s_frame[row * H12_OBS_FRAME + c] = fv[u];
  }
  __syncthreads();
  // phase 2: noisy frames, then the term scale (ObservationManager: noise, clip, scale)
  for (int k = tid; k < ASM_ROWS * H12_OBS_FRAME; k += ASM_BLOCK) {
    int row = k / H12_OBS_FRAME, c = k - row * H12_OBS_FRAME;
    int tn = noise_index(c);
    float v = s_frame[k];
    if (tn >= 0) v += s_noise[row * 32 + tn];
    v *= P.oscale[term_index(c)];
    s_frame[k] = v;
    // rollout record: the block's rows are consecutive, so its frames are one contiguous run of rows x 45 floats
    if (A.frame_out && row < rows) A.frame_out[(size_t)r0 * H12_OBS_FRAME + k] = v;
  }
  __syncthreads();
  // phase 3: assemble + store (obs may alias obs_prev: every read of these rows happened in phase 1)
  float* dst = A.obs + base;
  if (gather) {
    // a refilled row first gets its new frame in every slot of its LDS copy; then one branch-free gather
    // (history slot -> the next-newer slot, newest slot -> the frame behind the rows) serves every row
    int any_fill = 0;
#pragma unroll
    for (int r = 0; r < ASM_ROWS; ++r) any_fill |= s_fill[r];
    if (any_fill) {  // block-uniform
      for (int r = 0; r < ASM_ROWS; ++r)
        if (s_fill[r])
          for (int col = tid; col < ROW; col += ASM_BLOCK) s_hist[r * ROW + col] = s_frame[r * H12_OBS_FRAME + (s_col[col] & 0xFFu)];
      __syncthreads();
    }
#pragma unroll
    for (int u = 0; u < NG; ++u) {
      const int j = u * ASM_BLOCK + tid;
      if (j < ASM_F4) {
        const float* pb = s_hist + 4 * j;
        const uint2 t = gt[u];
        st_row4(dst, j, make_float4(pb[0 + (int)(int16_t)(t.x & 0xFFFFu)], pb[1 + ((int)t.x >> 16)],
                                    pb[2 + (int)(int16_t)(t.y & 0xFFFFu)], pb[3 + ((int)t.y >> 16)]));
      }
    }
    return;
  }
  auto value = [&](int row, int col) -> float {
    const uint32_t t = s_col[col];
    const int p = row * ROW + col;
    if (!s_write[row]) return s_hist[p];
    if (!s_fill[row] && !(t & (1u << 16))) return s_hist[p + (int)((t >> 8) & 0xFF)];
    return s_frame[row * H12_OBS_FRAME + (int)(t & 0xFF)];
  };
  if (full) {
    for (int j = tid; j < ASM_F4; j += ASM_BLOCK) {
      float v[4];
      const int p0 = 4 * j, row0 = p0 / ROW, col0 = p0 - row0 * ROW;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        int col = col0 + q, row = row0;
        if (col >= ROW) { col -= ROW; row += 1; }  // a float4 may straddle two rows (450 % 4 = 2)
        v[q] = value(row, col);
      }
      reinterpret_cast<float4*>(dst)[j] = make_float4(v[0], v[1], v[2], v[3]);
    }
  } else {
    for (int pp = tid; pp < rows * ROW; pp += ASM_BLOCK) {
      int row = pp / ROW, col = pp - row * ROW;
      if (s_write[row]) dst[pp] = value(row, col);
    }
  }
}
// Deferred episode-log folds (fused step path): block (v, k) folds value v of pending step k -- the same per-lane
// sums and shuffle tree as log_load / log_fold_one, so the accumulators are bit-identical to the immediate fold.
// One block per (value, step) and no two pending steps share an accumulator (h12env_step flushes first), so every
// accumulator word has one writer.
constexpr int LOG_RING = 64;  // partial sets (steps) the handle holds; a full ring is folded by the next step
struct FoldArgs {
  float* part;  // the handle's ring: [LOG_RING][LOG_NPART][nb]
  int nb;
  int slot[LOG_RING];
  float* acc[LOG_RING];
};
__global__ void __launch_bounds__(64) log_flush_kernel(FoldArgs F) {
  const int v = blockIdx.x, k = blockIdx.y;
  float* q = F.part + ((size_t)F.slot[k] * LOG_NPART + v) * F.nb;
  float acc = 0.f;
  for (int b = threadIdx.x; b < F.nb; b += 64) acc += q[b];
  for (int b = threadIdx.x; b < F.nb; b += 64) q[b] = 0.f;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (threadIdx.x == 0 && acc != 0.f) F.acc[k][log_slot(v)] += acc;
}
template <int NH>
__global__ void __launch_bounds__(ASM_BLOCK) obs_assemble_kernel(KParams P, AsmArgs A) {
  const float lacc = log_load(A);
  obs_assemble_body<NH>(P, A);
  log_fold(A, lacc);
}

// Rough task observation (no history): one thread per (env, element) of the 235-float row --
// base_lin_vel, base_ang_vel, projected_gravity, velocity_commands, joint_pos_rel, joint_vel_rel,
// last_action, height_scan (velocity_env_cfg.py:118-137; noise then clip, as ObservationManager does).
// Height scan: RayCasterCfg at the torso_link origin (= pelvis origin), attach_yaw_only, grid pattern
// 1.6 x 1.0 m at 0.1 m (17 x 11 rays, x fastest: meshgrid 'xy' order), rays straight down onto the
// heightfield; value = sensor z - hit z - 0.5 (isaaclab mdp.height_scan).
H12_DEV float rough_noise(const KParams& P, const AsmArgs& A, int e, int t) {
  uint32_t r[4];
  philox(P.seed_lo, P.seed_hi, (uint32_t)(A.env_offset + e), A.lo, ((uint32_t)ST_OBS << 16) | (uint32_t)(t >> 2), A.hi, r);
  uint32_t rv = (t & 3) == 0 ? r[0] : ((t & 3) == 1 ? r[1] : ((t & 3) == 2 ? r[2] : r[3]));
  float nmax = t < 3 ? P.n_lin : (t < 6 ? P.n_w : (t < 9 ? P.n_g : (t < 21 ? P.n_q : (t < 33 ? P.n_qd : P.n_scan))));
  return P.corrupt ? (-nmax + 2.f * nmax * u01(rv)) : 0.f;
}

__global__ void __launch_bounds__(ASM_BLOCK) rough_obs_kernel(KParams P, AsmArgs A) {
  log_fold(A, log_load(A));
  const int n = A.n;
  const int gid = blockIdx.x * ASM_BLOCK + threadIdx.x;
  if (gid >= n * H12_NOBS_ROUGH) return;
  const int e = gid / H12_NOBS_ROUGH;
  const int k = gid - e * H12_NOBS_ROUGH;
  if (A.reset_mode && A.sel && !A.sel[e]) return;
  float v;
  if (k < H12_ROUGH_FRAME) {
    v = A.frame[(size_t)k * n + e];
    int t = k < 9 ? k : ((k >= 12 && k < 36) ? k - 3 : -1);
    if (t >= 0) v += rough_noise(P, A, e, t);
  } else {
    const int r = k - H12_ROUGH_FRAME, iy = r / H12_SCAN_NX, ix = r - iy * H12_SCAN_NX;
    const float xl = P.scan_res * (float)(ix - (H12_SCAN_NX - 1) / 2), yl = P.scan_res * (float)(iy - (H12_SCAN_NY - 1) / 2);
    const float px = A.frame[(size_t)H12_ROUGH_FRAME * n + e], py = A.frame[(size_t)(H12_ROUGH_FRAME + 1) * n + e];
    const float pz = A.frame[(size_t)(H12_ROUGH_FRAME + 2) * n + e];
    const float cy = A.frame[(size_t)(H12_ROUGH_FRAME + 3) * n + e], sy = A.frame[(size_t)(H12_ROUGH_FRAME + 4) * n + e];
    float hz = 0.f;
    if (P.terrain) {
      float gx, gy;
      hz = ground(P, px + cy * xl - sy * yl, py + sy * xl + cy * yl, gx, gy);
    }
    v = pz - hz - P.scan_off + rough_noise(P, A, e, k - 15);
    v = fminf(fmaxf(v, -P.scan_clip), P.scan_clip);
  }
  A.obs[(size_t)e * H12_NOBS_ROUGH + k] = v;
}

// ------------------------------------------------------------------ kernels
// The reward terms of one env on its post-physics, pre-reset state (RewardManager.compute's term functions,
// unweighted; SURVEY.md a8.1-a8.12 + the Rsl extras), shared by step_kernel and the term-evaluation hook
// (terms_kernel).  The lane pair holds the two legs: leg sums are combined with one DPP swap (psum).
template <int K>
H12_DEV void mdp_terms(const KParams& P, const EnvSt& s, int leg, const float R[3][3], const float* tau,
                       const float* jacc, float fmax_foot, int term, float* terms) {
  const float sg = leg ? -1.f : 1.f;
  float ww[3];
  mv(R, s.b.wang, ww);
  float vcom[3];
  base_com_vel<K>(P, s, R, vcom);
  // yaw frame: heading direction of the body x axis in the world xy-plane
  float hx = R[0][0], hy = R[1][0];
  float hn = __builtin_amdgcn_rsqf(hx * hx + hy * hy);
  float cy = hx * hn, sy = hy * hn;
  float vy0 = cy * vcom[0] + sy * vcom[1], vy1 = -sy * vcom[0] + cy * vcom[1];
  float ex = s.cmd[0] - vy0, ey = s.cmd[1] - vy1, ew = s.cmd[2] - ww[2];
  terms[H12_R_TRACK_LIN_VEL_XY] = __expf(-(ex * ex + ey * ey) * P.std2_inv);
  terms[H12_R_TRACK_ANG_VEL_Z] = __expf(-(ew * ew) * P.std2_inv);
  terms[H12_R_ANG_VEL_XY_L2] = s.b.wang[0] * s.b.wang[0] + s.b.wang[1] * s.b.wang[1];
  float st_ = 0.f, sa_ = 0.f, sr_ = 0.f, sl_ = 0.f, sd_ = 0.f;
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    st_ += tau[k] * tau[k];
    sa_ += jacc[k] * jacc[k];
    float dr = s.act[k] - s.act1[k];
    sr_ += dr * dr;
  }
#pragma unroll
  for (int k = 4; k < 6; ++k) {  // ankle pitch / roll soft limits (symmetric under the mirror)
    float q = s.lg.q[k], lo_s = soft_lo(P, k), hi_s = soft_hi(P, k);
    sl_ += (q < lo_s ? lo_s - q : 0.f) + (q > hi_s ? q - hi_s : 0.f);
  }
  sd_ = fabsf(s.lg.q[0] - h12m::Q0[0]) + fabsf(s.lg.q[2] - h12m::Q0[2]);  // hip yaw, hip roll
  auto psum = [&](float x) {
    float y = pair_swap(x);
    return leg ? (y + x) : (x + y);
  };
  terms[H12_R_DOF_TORQUES_L2] = psum(st_);
  terms[H12_R_DOF_ACC_L2] = psum(sa_);
  terms[H12_R_ACTION_RATE_L2] = psum(sr_);
  {
    float con_o = pair_swap(s.con), air_o = pair_swap(s.air);
    float conL = leg ? con_o : s.con, conR = leg ? s.con : con_o;
    float airL = leg ? air_o : s.air, airR = leg ? s.air : air_o;
    int incL = conL > 0.f, incR = conR > 0.f;
    float mL = incL ? conL : airL, mR = incR ? conR : airR;
    float r = ((incL + incR) == 1) ? fminf(mL, mR) : 0.f;
    r = fminf(r, P.air_thr);
    float cn2 = s.cmd[0] * s.cmd[0] + s.cmd[1] * s.cmd[1];
    terms[H12_R_FEET_AIR_TIME] = cn2 > 0.01f ? r : 0.f;
  }
  terms[H12_R_FLAT_ORIENTATION_L2] = R[2][0] * R[2][0] + R[2][1] * R[2][1];
  terms[H12_R_DOF_POS_LIMITS] = psum(sl_);
  terms[H12_R_TERMINATION] = term ? 1.f : 0.f;
  {
    // feet_slide: |v_xy| of the foot COM (lane frame; the norm is mirror-invariant) where max_h |F| > 1
    float fs = 0.f;
    if (fmax_foot > 1.0f) {
      const float mm[3] = {1.f, sg, 1.f};
      float Rf[3][3];
      for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) Rf[i][j] = mm[i] * mm[j] * R[i][j];
      float vb[3];
      mtv(R, s.b.vlin, vb);
      float v0[6] = {s.b.wang[0], s.b.wang[1], s.b.wang[2], vb[0], vb[1], vb[2]};
      for (int i = 0; i < 6; ++i) v0[i] *= s6(i, sg);
      float csd[NL][2], vd[NL][6], pd[3] = {0.f, 0.f, 0.f};
      link_pass1<0>(s.lg, csd, v0, vd, Rf, pd);
      link_pass1<1>(s.lg, csd, vd[0], vd, Rf, pd);
      link_pass1<2>(s.lg, csd, vd[1], vd, Rf, pd);
      link_pass1<3>(s.lg, csd, vd[2], vd, Rf, pd);
      link_pass1<4>(s.lg, csd, vd[3], vd, Rf, pd);
      link_pass1<5>(s.lg, csd, vd[4], vd, Rf, pd);
      float vc[3], vw[3];
      cross(vd[5], h12m::COM[5], vc);
      vc[0] += vd[5][3]; vc[1] += vd[5][4]; vc[2] += vd[5][5];
      mv(Rf, vc, vw);
      fs = fsqrt(vw[0] * vw[0] + vw[1] * vw[1]);
    }
    terms[H12_R_FEET_SLIDE] = psum(fs);
  }
  terms[H12_R_JOINT_DEV_HIP] = psum(sd_);
  // terms of the Rsl table (rsl_env_cfg.py:279-407), base-frame tracking and the extra penalties
  if (Feat<K>::ext) {
    for (int t = H12_NREW_FLAT; t < H12_NREW; ++t) terms[t] = 0.f;
    if (P.rsl) {
      float vb[3];
      mtv(R, vcom, vb);  // root_lin_vel_b (composite COM velocity in the base frame)
      float bx = s.cmd[0] - vb[0], by = s.cmd[1] - vb[1], bw = s.cmd[2] - s.b.wang[2];
      terms[H12_R_TRACK_LIN_VEL_XY_BASE] = __expf(-(bx * bx + by * by) * P.std2_inv);
      terms[H12_R_TRACK_ANG_VEL_Z_BASE] = __expf(-(bw * bw) * P.std2_inv);
      float dh = s.b.pos[2] - P.h_target;
      terms[H12_R_BASE_HEIGHT_L2] = dh * dh;
      float sv_ = 0.f, sh_ = 0.f;
#pragma unroll
      for (int k = 0; k < NL; ++k) sv_ += s.lg.qd[k] * s.lg.qd[k];
#pragma unroll
      for (int k = 0; k < 3; k += 2) {  // hip yaw (0), hip roll (2) soft limits
        float q = s.lg.q[k], lo_s = soft_lo(P, k), hi_s = soft_hi(P, k);
        sh_ += (q < lo_s ? lo_s - q : 0.f) + (q > hi_s ? q - hi_s : 0.f);
      }
      terms[H12_R_JOINT_VEL_L2] = psum(sv_);
      terms[H12_R_JOINT_DEV_ANKLE] = psum(fabsf(s.lg.q[4] - h12m::Q0[4]) + fabsf(s.lg.q[5] - h12m::Q0[5]));
      terms[H12_R_DOF_POS_LIMITS_HIP] = psum(sh_);
      terms[H12_R_CONTACT_FORCES] = psum(fmaxf(fmax_foot - P.cf_thr, 0.f));
      terms[H12_R_LIN_VEL_Z_L2] = vb[2] * vb[2];
    }
  }
}

struct StepArgs {
  const float* actions;
  const float* obs_prev;
  float* obs;
  float* rew;
  uint8_t* term;
  uint8_t* trunc;
  float* log_part;  // [LOG_NPART][gridDim.x] per-block episode-log partials (handle-owned), or null: no log
  float* applied_torque;
  float* foot_force;
  const uint8_t* reset_mask;
  union {
    const float* q_ref;  // physics_kernel: the physics-only hook's joint targets
    float* cstr_prob;    // step_kernel with cat_inline: CaT's termination probabilities (h12env_outputs.cstr_prob), or null
  };
  float* frame;        // [45][n] noise-free observation frame scratch (handle-owned)
  int64_t env_offset;
  uint32_t lo, hi;
  int n_substeps;
  int dz_slot;  // deadzone counter read this step (P.dz_cnt[dz_slot]); +1 is counted into, +2 zeroed
  int fuse;     // the observation rows are assembled inside step_kernel (FuseCtx; dynamic LDS)
  int cat_inline;  // CaT: step_kernel also applies the probabilities (cat_prob_inline; the grid is resident)
  const uint8_t* fuse_code;  // fuse_code_table of the handle's history length
  float* frame_out;         // (n, 45) noisy scaled frames as they enter the history (fused path), or null
};

// helper waves (lane t of nt), before barrier L: the rows' noise blocks (and, off the spread path, the rows -> LDS)
H12_DEV void fuse_stage(const KParams& P, const StepArgs& A, const FuseCtx& fc, int n, int t, int nt) {
  FuseLds& F = fuse_lds();
  const int e0 = step_block() * FUSE_ROWS, ne = min(FUSE_ROWS, n - e0);
  if (!fc.on)
    for (int j = t; j < ne * fc.row; j += nt) F.hist[j] = fc.src[j];  // plain copies (ragged block / 1 physics step)
  for (int w = t; w < 8 * ne; w += nt) {
    const int r = w >> 3, blk = w & 7;
    uint32_t q[4];
    philox(P.seed_lo, P.seed_hi, (uint32_t)(A.env_offset + e0 + r), A.lo, ((uint32_t)ST_OBS << 16) | (uint32_t)blk,
           A.hi, q);
#pragma unroll
    for (int a = 0; a < 4; ++a)
      if (4 * blk + a < 30) F.noise[r][4 * blk + a] = noise_of(P, 4 * blk + a, q[a]);
  }
}

// column of frame component c's newest slot in a row of history nh (term-major blocks, oldest slot first)
H12_DEV int newest_col(int c, int nh) {
  if (c < 9) return (c / 3) * 3 * nh + 3 * (nh - 1) + c % 3;
  const int k = c - 9;
  return 9 * nh + (k / 12) * 12 * nh + 12 * (nh - 1) + k % 12;
}

// helper waves, after barrier F: the newest slots, the refilled rows and frame_out (spread path), or whole rows
H12_DEV void fuse_late(const KParams& P, const StepArgs& A, const FuseCtx& fc, int n, int t, int nt) {
  const FuseLds& F = fuse_lds();
  const int e0 = step_block() * FUSE_ROWS, ne = min(FUSE_ROWS, n - e0);
  const int row = fc.row, nh = P.hist;
  const float* fr = F.hist + FUSE_ROWS * row;
  if (A.frame_out) {  // the block's frames are one contiguous run of ne x 45 floats
    float* fo = A.frame_out + (size_t)e0 * H12_OBS_FRAME;
    if (ne == FUSE_ROWS && ((uintptr_t)fo & 15u) == 0) {  // 360 float4s, reads before stores
      constexpr int NF4 = FUSE_ROWS * H12_OBS_FRAME / 4, FMAX = (NF4 + 63) / 64;
      float4 fv[FMAX];
#pragma unroll
      for (int k = 0; k < FMAX; ++k) fv[k] = reinterpret_cast<const float4*>(fr)[min(t + k * nt, NF4 - 1)];
#pragma unroll
      for (int k = 0; k < FMAX; ++k)
        if (t + k * nt < NF4) reinterpret_cast<float4*>(fo)[t + k * nt] = fv[k];
    } else {
      for (int k = t; k < ne * H12_OBS_FRAME; k += nt) fo[k] = fr[k];
    }
  }
  if (fc.on) {
    // lane u < 90: frame component c = u % 45 of rows u / 45, + 2, + 4, ... -- its newest column computed once, the
    // 16 LDS reads before the 16 stores.  Decoding (row, component, column) per element instead left these waves
    // ending 0.96 us after the physics wave (light stamps); now 0.12 us, +2.2 % env-steps/s (profiles/r4/)
    constexpr int NRI = FUSE_ROWS / 2;
    for (int u = t; u < 2 * H12_OBS_FRAME; u += nt) {
      const int r0 = u >= H12_OBS_FRAME ? 1 : 0, c = u - r0 * H12_OBS_FRAME;
      const int col = newest_col(c, nh);
      float v[NRI];
#pragma unroll
      for (int i = 0; i < NRI; ++i) v[i] = fr[H12_OBS_FRAME * (r0 + 2 * i) + c];
      float* d = fc.dst + r0 * row + col;
#pragma unroll
      for (int i = 0; i < NRI; ++i) d[(size_t)(2 * i) * row] = v[i];
    }
    // a resetting env's row restarts its history: the frame in every slot
    constexpr uint32_t ROWS_MASK = FUSE_ROWS >= 32 ? ~0u : (1u << FUSE_ROWS) - 1u;  // a lane per row, no repeats
    uint32_t fm = (uint32_t)__ballot(F.fill[threadIdx.x & (FUSE_ROWS - 1)] != 0) & ROWS_MASK;  // wave-uniform
    while (fm) {
      const int r = __builtin_ctz(fm);
      fm &= fm - 1u;
      for (int col = t; col < row; col += nt) fc.dst[r * row + col] = fr[H12_OBS_FRAME * r + F.code[FUSE_F4_MAX + col]];
    }
    return;
  }
  for (int p = t; p < ne * row; p += nt) {
    const int r = p / row, col = p - r * row;
    const uint32_t te = hist_col_entry(col, nh);
    fc.dst[p] = (F.fill[r] || (te >> 16)) ? fr[H12_OBS_FRAME * r + (int)(te & 0xFFu)] : F.hist[p + (int)((te >> 8) & 0xFFu)];
  }
}

// physics wave, fused path: obs_frame's values (Flat layout) with the noise (drawn by fuse_stage) and the term
// scale applied as obs_assemble_body does, into the block's LDS frame row r; and the row's refill flag
H12_DEV void obs_frame_fused(const KParams& P, const EnvSt& s, int leg, int r, bool fill) {
  FuseLds& F = fuse_lds();
  float* fr = F.hist + FUSE_ROWS * H12_OBS_FRAME * P.hist + H12_OBS_FRAME * r;
  const float* nz = F.noise[r];
  const float sg = leg ? -1.f : 1.f;
  if (leg == 0) {
    float R[3][3];
    quat_R(s.b.quat, R);
    for (int a = 0; a < 3; ++a) fr[a] = (s.b.wang[a] + nz[a]) * P.oscale[0];
    for (int a = 0; a < 3; ++a) {
      // the projected gravity rounded on its own, as the two-kernel path stores it (quat_R's products are no longer
      // exact doublings; contracted into the noise addition they would round differently)
      float gr = -R[2][a];
      pin(gr);
      fr[3 + a] = (gr + nz[3 + a]) * P.oscale[1];
    }
    for (int a = 0; a < 3; ++a) fr[6 + a] = s.cmd[a] * P.oscale[2];
    F.fill[r] = fill ? 1 : 0;
  }
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    const int j = NL * leg + k;
    const float js = jsign(k, sg);
    fr[9 + j] = (js * (s.lg.q[k] - h12m::Q0[k]) + nz[6 + j]) * P.oscale[3];
    fr[21 + j] = (js * s.lg.qd[k] + nz[18 + j]) * P.oscale[4];
    fr[33 + j] = js * s.act[k] * P.oscale[5];
  }
}

// Every 64-B line of the kernel arguments into the scalar cache at once, at the start of every wave: the compiler sinks
// each kernel-argument load to its first use, so the helper waves' way to their first barrier held 3-4 dependent
// rounds of scalar loads and waits (light stamps: they started their roles 0.8-1.0 us after the physics wave, which
// waited ~0.5 us for them at the first barrier S).  The loads' values are dropped; the wait is in the same statement.
static_assert(sizeof(KParams) + sizeof(Workspace) + sizeof(StepArgs) <= 1024, "kernel arguments within 16 lines");
H12_DEV void kernarg_warm() {
  const auto ka = __builtin_amdgcn_kernarg_segment_ptr();
  uint32_t d0, d1, d2, d3;
  asm volatile(
      "s_load_dword %0, %4, 0x0\n\ts_load_dword %1, %4, 0x40\n\ts_load_dword %2, %4, 0x80\n\t"
      "s_load_dword %3, %4, 0xc0\n\ts_load_dword %0, %4, 0x100\n\ts_load_dword %1, %4, 0x140\n\t"
      "s_load_dword %2, %4, 0x180\n\ts_load_dword %3, %4, 0x1c0\n\ts_load_dword %0, %4, 0x200\n\t"
      "s_load_dword %1, %4, 0x240\n\ts_load_dword %2, %4, 0x280\n\ts_load_dword %3, %4, 0x2c0\n\t"
      "s_load_dword %0, %4, 0x300\n\ts_load_dword %1, %4, 0x340\n\ts_load_dword %2, %4, 0x380\n\t"
      "s_load_dword %3, %4, 0x3c0\n\ts_waitcnt lgkmcnt(0)"
      : "=&s"(d0), "=&s"(d1), "=&s"(d2), "=&s"(d3)
      : "s"(ka)
      : "memory");
}

// CaT fold (round 6): the contact wave of the last step_kernel block to arrive, once every block's hand-off is out (the
// agent-scope counter, cat_arrive): the running maxima (CaT.add, constraint_manager.py:42-78) from the column maxima
// every block maxed in, and the still envs in ascending order (constraints.no_move hands env i the row of the
// (i mod m)-th still env, constraints.py:202-238) from the blocks' masks -- what the one-block cat_reduce_kernel launch
// did (7.1 us per step).  Every load of the hand-off is an sc1 (agent-scope relaxed) load, as the hand-off's rule asks;
// with cat_inline the fold's outputs also go out as epoch-tagged words (cpub).
constexpr int CAT_META_INTS = 64 + 8 * H12_NCSTR_COLS;  // meta, then the eight column-maxima sets (cat_cmax)
H12_DEV int* cat_ccount(const KParams& P) { return P.cmeta + 2; }
H12_DEV uint32_t* cat_cstill(const KParams& P) { return reinterpret_cast<uint32_t*>(P.cmeta + CAT_META_INTS); }
template <typename T>
H12_DEV T ld_sc1(const T* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
template <typename T>
H12_DEV void st_sc1(T* p, T v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
// the published fold (cat_inline): every value the blocks read after the fold is an 8-B word tagged with the fold's
// epoch (epoch << 32 | value; +1 per fold), so a word is its own "ready" flag -- no store-completion wait and no
// separate flag store in the fold, and the waiters poll the very words they need.  A block reads the epoch (the m
// word's tag) before its own arrival, so it cannot see the next one early: the fold needs every arrival.
// cat_cpub: every word (epoch << 32 | value): [0, 56) the reciprocals, [56] m, [64 + b] the still envs in blocks
// before block b (the exclusive prefix of the blocks' still counts); then, as floats, the blocks' still envs' no_move
// rows compacted by the hand-off, [block][12][32] (cat_rows: env i's remapped row -- the (i mod m)-th still env's --
// is found from the prefixes, one load round trip shorter than a still list)
constexpr int CPUB_M = 56, CPUB_LIST = 64;
constexpr int CAT_NMC = C_COL0[H12_C_NO_MOVE + 1] - C_COL0[H12_C_NO_MOVE];
H12_DEV int cat_nbpad(int n) { return ((n + ENVS_PER_BLOCK - 1) / ENVS_PER_BLOCK + 31) / 32 * 32; }
constexpr size_t CPUB_OFF = 512;  // after crun (2 x 56 floats, its section 256-B aligned: h12env_create)
static_assert(2 * H12_NCSTR_COLS * sizeof(float) <= CPUB_OFF, "crun fits ahead of the published fold");
H12_DEV unsigned long long* cat_cpub(const float* crun) {
  return reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(const_cast<float*>(crun)) + CPUB_OFF);
}
H12_DEV float* cat_rows(const float* crun, int n) {
  return reinterpret_cast<float*>(cat_cpub(crun) + CPUB_LIST + cat_nbpad(n));
}
H12_DEV unsigned long long cat_tag(unsigned epoch, unsigned v) { return (unsigned long long)epoch << 32 | v; }
// the column maxima: float -> unsigned with the same order (sign bit flipped for >= 0, all bits for < 0), so every
// block's maxima go in with one unsigned atomic max per column (exact, order-free); 0 (below every encoding) = none
// eight sets of them, one per XCD slot of the block (blockIdx.x mod 8): 16 blocks per address instead of 128, the
// fold takes the max of the eight
constexpr int CAT_CMAX_SETS = 8;
H12_DEV unsigned* cat_cmax(const KParams& P, int set) {
  return reinterpret_cast<unsigned*>(P.cmeta + 64) + set * H12_NCSTR_COLS;
}
H12_DEV unsigned cat_enc(float f) {
  const unsigned b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
H12_DEV float cat_dec(unsigned u) { return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u); }
H12_DEV void cat_fold(const KParams& P, int n, bool inl) {
  const int lane = threadIdx.x & 63;
  const unsigned e1 = inl ? __float_as_uint(cat_lds()[CAT_LROW_EPOCH][0]) + 1u : 0u;  // this fold's epoch
  const int nb = (n + ENVS_PER_BLOCK - 1) / ENVS_PER_BLOCK;
  // the column maxima (lane col), read and reset for the next step (the blocks' atomic maxima, cat_handoff)
  float cmx = CAT_NEG;
  if (lane < H12_NCSTR_COLS) {
    unsigned u[CAT_CMAX_SETS];
#pragma unroll
    for (int x = 0; x < CAT_CMAX_SETS; ++x) u[x] = ld_sc1(cat_cmax(P, x) + lane);
    unsigned um = 0u;
#pragma unroll
    for (int x = 0; x < CAT_CMAX_SETS; ++x) {
      um = max(um, u[x]);
      st_sc1(cat_cmax(P, x) + lane, 0u);
    }
    cmx = cat_dec(um);
  }
  // the still envs: lane l owns the env chunks [l q, l q + q), an exclusive prefix of the counts over the lanes
  // (the masks loaded once: at most 4 chunks per lane -- cat_inline grids have <= 256 blocks, the fallback's larger
  // ones loop)
  const int q = (nb + 63) / 64, c0 = min(nb, lane * q), c1 = min(nb, c0 + q);
  uint32_t mk[4] = {};
  int cnt = 0;
  for (int c = c0; c < c1; ++c) {
    const uint32_t b = ld_sc1(&cat_cstill(P)[c]);
    if (c - c0 < 4) mk[c - c0] = b;
    cnt += __popc(b);
  }
  int incl = cnt;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(incl, d, 64);
    if (lane >= d) incl += y;
  }
  const int m = __shfl(incl, 63, 64);
  int off = incl - cnt;
  if (inl) {  // the blocks' prefixes
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (c0 + i < c1) {
        st_sc1(&cat_cpub(P.crun)[CPUB_LIST + c0 + i], cat_tag(e1, (unsigned)off));
        off += __popc(mk[i]);
      }
    }
  } else {  // the still list (cat_prob_kernel)
    for (int c = c0; c < c1; ++c)
      for (uint32_t b = ld_sc1(&cat_cstill(P)[c]); b; b &= b - 1u) st_sc1(&P.clist[off++], c * ENVS_PER_BLOCK + __builtin_ctz(b));
  }
  if (lane < H12_NCSTR_COLS) {
    float cm = cmx;
    const bool nm = lane >= C_COL0[H12_C_NO_MOVE] && lane < C_COL0[H12_C_NO_MOVE + 1];
    if (nm && m == 0) cm = 0.f;  // constraints.no_move returns zeros when no env is still
    cm = fmaxf(cm, 1e-6f);       // constraint.max(dim=0).clamp(min=1e-6)
    const float old = P.crun[lane];
    const float run = P.cmeta[1] ? P.ctau * old + (1.f - P.ctau) * cm : cm;
    st_sc1(&P.crun[lane], run);
    st_sc1(&P.crun[H12_NCSTR_COLS + lane], 1.f / run);
    if (inl) st_sc1(&cat_cpub(P.crun)[lane], cat_tag(e1, __float_as_uint(1.f / run)));
  }
  if (lane == 0) {
    st_sc1(&P.cmeta[0], m);
    st_sc1(&P.cmeta[1], 1);
    st_sc1(cat_ccount(P), 0);  // the next launch's count
    if (inl) st_sc1(&cat_cpub(P.crun)[CPUB_M], cat_tag(e1, (unsigned)m));
  }
}

// CaT hand-off (round 6): step_kernel's contact wave, after barrier L (it idles there until barrier F): this block's
// column maxima (CaT.add's constraint.max(dim=0); no_move columns over the still envs only) into the step's maxima with
// one agent-scope atomic max per column (a [block][56] row for the fold to read took 2-3 more memory round trips on its
// critical path), its still envs as an sc1-stored mask, all waited for, then one agent-scope add per block (cat_arrive);
// the block whose add came last folds (cat_fold) -- the cross-workgroup hand-off of MI355X_MICROARCH.md (stores, atomics
// and loads all agent scope, one arrival atomic per workgroup, the last adder loads after its add returned).  The
// one-block cat_reduce_kernel launch it replaces took 7.1 us per step (rocprofv3, profiles/r6/)
H12_DEV unsigned cat_handoff(const KParams& P, int n, bool inl) {
  const int col = threadIdx.x & 63;
  const int ne = min(ENVS_PER_BLOCK, n - step_block() * ENVS_PER_BLOCK);
  const CatLds& cv = cat_lds();
  // cat_inline: the fold epoch before this block's arrival (in flight until the arrival's vmcnt(0)), and the still
  // envs' no_move rows again as sc1 stores (cat_prob_inline reads them across blocks: constraints.no_move's remap)
  const unsigned e0 = inl && col == 0 ? (unsigned)(ld_sc1(&cat_cpub(P.crun)[CPUB_M]) >> 32) : 0u;
  if (inl) {  // compacted: the block's r-th still env at [block][k][r]
    constexpr int NM0 = C_COL0[H12_C_NO_MOVE];
    const int j = col & (ENVS_PER_BLOCK - 1);
    const uint32_t sm = (uint32_t)__ballot(col < ENVS_PER_BLOCK && col < ne && cv[CAT_ROW_NOMOVE][col] != 0.f);
    if ((sm >> j) & 1u) {
      const int r = __popc(sm & ((1u << j) - 1u));
      float* rows = cat_rows(P.crun, n) + (size_t)step_block() * CAT_NMC * ENVS_PER_BLOCK + r;
      for (int k = col / ENVS_PER_BLOCK; k < CAT_NMC; k += 64 / ENVS_PER_BLOCK)
        st_sc1(&rows[k * ENVS_PER_BLOCK], cv[NM0 + k][j]);
    }
  }
  if (col < H12_NCSTR_COLS) {
    const bool nm = col >= C_COL0[H12_C_NO_MOVE] && col < C_COL0[H12_C_NO_MOVE + 1];
    float m = CAT_NEG;
#pragma unroll
    for (int j = 0; j < ENVS_PER_BLOCK; ++j) {  // unrolled: the LDS reads issue back to back
      const float x = cv[col][j];
      const bool ok = j < ne && (!nm || cv[CAT_ROW_NOMOVE][j] != 0.f);
      m = ok ? fmaxf(m, x) : m;
    }
    __hip_atomic_fetch_max(cat_cmax(P, blockIdx.x % CAT_CMAX_SETS) + col, cat_enc(m), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
  }
  const uint32_t still = (uint32_t)__ballot(col < ENVS_PER_BLOCK && col < ne && cv[CAT_ROW_NOMOVE][col] != 0.f);
  if (col == 0) __hip_atomic_store(&cat_cstill(P)[step_block()], still, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return e0;
}
// ... after the wave's s_waitcnt vmcnt(0) (the stores above have completed): the block's add.  The returned count is
// only looked at after barrier F and the rows (cat_is_last), so its round trip overlaps them
H12_DEV int cat_arrive(const KParams& P) {
  int old = -1;
  if ((threadIdx.x & 63) == 0) old = __hip_atomic_fetch_add(cat_ccount(P), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return old;
}
H12_DEV bool cat_is_last(int old) { return __shfl(old, 0, 64) == (int)gridDim.x - 1; }

// CaT's episode statistics of the resetting envs (cat_prob_inline, cat_prob_kernel): L[k][j] holds env j's
// value k of one step_kernel block (k < NCSTR: the violation sum over the episode length, then the probability sum;
// zero for envs that do not reset), summed in env order by lane k and added to the block's partial slot -- the same
// order on both paths (float atomics from one instruction, the round-5 form, summed in an order the two paths did not
// share).  `any`: some env of the block resets (else nothing to add).
template <int S>
H12_DEV void cat_log_block(uint32_t cmask, const float (*L)[S], int k, bool any, float* log_part,
                           int log_nb, int slot) {
  if (!any || !log_part || k >= 2 * H12_NCSTR || !((cmask >> (k % H12_NCSTR)) & 1u)) return;
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < ENVS_PER_BLOCK; ++j) sum += L[k][j];
  float& d = log_part[(size_t)(LOG_NSTEP + k) * log_nb + slot];
  d = d + sum;
}
constexpr int CAT_WAIT_POLLS = 1 << 18;
// step_kernel's KParams read through the kernarg segment pointer (its first argument, offset 0) instead of the by-value
// parameter: code that indexes the parameter in a way the compiler cannot resolve (here the new CaT functions' loads,
// merged into selects of addresses) makes it copy all 856 B of KParams to scratch first
H12_DEV const __attribute__((address_space(4))) KParams& kparams4() {
  return *(const __attribute__((address_space(4))) KParams*)__builtin_amdgcn_kernarg_segment_ptr();
}
constexpr int cat_col_term(int col) {
  int t = 0;
  while (C_COL0[t + 1] <= col) ++t;
  return t;
}
// one env's probabilities (the leg-0 lane of a pair): the reward factor 1 - p_max, the dones' probability, the
// constraint sums, and its episode statistics into lg (zero unless it resets)
H12_DEV float cat_prob_env(const Workspace& W, const StepArgs& A, int he, int j, bool reset, const float* vs,
                           const float* vp, const float* srow, const float* rinv, float* lg) {
  const auto& P = kparams4();
  const CatLds& cv = cat_lds();
  constexpr int NM0 = C_COL0[H12_C_NO_MOVE], NM1 = C_COL0[H12_C_NO_MOVE + 1];
  float nmv[NM1 - NM0];
#pragma unroll
  for (int k = 0; k < NM1 - NM0; ++k) nmv[k] = srow ? ld_sc1(&srow[k * ENVS_PER_BLOCK]) : 0.f;
  // one flat loop over the columns (constant trip count: fully unrolled, every index static -- the nested form left
  // a dynamic KParams index that made the compiler copy KParams to scratch); max is exact, so the order is free
  float pt[H12_NCSTR];
#pragma unroll
  for (int t = 0; t < H12_NCSTR; ++t) pt[t] = 0.f;
#pragma unroll
  for (int col = 0; col < H12_NCSTR_COLS; ++col) {
    const int t = cat_col_term(col);
    const bool on_t = (P.cmask >> t) & 1u;
    const float c = (col >= NM0 && col < NM1) ? nmv[col - NM0] : cv[col][j];
    const float p = P.cminp + fminf(fmaxf(c * rinv[col], 0.f), 1.f) * (P.cmaxp[t] - P.cminp);
    pt[t] = fmaxf(pt[t], (on_t && c > 0.f) ? p : 0.f);
  }
  float pmax = 0.f;
#pragma unroll
  for (int t = 0; t < H12_NCSTR; ++t) pmax = fmaxf(pmax, pt[t]);
  if (A.cstr_prob) A.cstr_prob[he] = reset ? 1.f : pmax;
  const float inv_len = 1.f / cv[CAT_ROW_EPLEN][j];
  const int n = W.n;
#pragma unroll
  for (int t = 0; t < H12_NCSTR; ++t) {
    lg[t] = lg[H12_NCSTR + t] = 0.f;
    if (!((P.cmask >> t) & 1u)) continue;  // (the sums of an inactive term stay as they are)
    float a = vs[t] + (pt[t] > 0.f ? 1.f : 0.f), b = vp[t] + pt[t];
    if (reset) {
      lg[t] = a * inv_len;
      lg[H12_NCSTR + t] = b * inv_len;
      a = b = 0.f;
    }
    W.F[(size_t)(H12_F_CSTR_SUM + t) * n + he] = a;
    W.F[(size_t)(H12_F_CSTR_P + t) * n + he] = b;
  }
  float keep = 1.f - pmax;  // pinned as in cat_prob_kernel (the same rounding on both paths)
  pin(keep);
  return keep;
}
// CaT probabilities inside step_kernel (round 6, A.cat_inline: the whole grid is resident, h12env_create checks it):
// cat_prob_kernel's per-env step (below) by the helper wave after barrier F, once the last block's fold is published --
// the running maxima's reciprocals, the still list and the still envs' no_move rows (all sc1) -- for env he (the leg-0
// lane of each pair, `on`); the env's own constraint values and episode length come from the block's LDS copy.
// Returns the reward factor 1 - p_max.  The wait is bounded (~20 ms): at the bound it raises bit 1 of the device
// diagnostic word (h12env_check) and goes on with what it has.
H12_DEV float cat_prob_inline(const Workspace& W, const StepArgs& A, int he, int j, bool on, bool reset,
                              const float* vs, const float* vp) {
  const auto& P = kparams4();
  const int lane = threadIdx.x & 63;
  CatLds& cv = cat_lds();
  // the wave polls the words it needs -- lanes 0-55 their reciprocal's, lane 56 m's, every lane up to four block
  // prefixes -- until each carries this step's epoch (sc1 loads, a short sleep between rounds; bounded, ~20 ms)
  const unsigned e1 = __float_as_uint(cv[CAT_LROW_EPOCH][0]) + 1u;
  const int nb = (W.n + ENVS_PER_BLOCK - 1) / ENVS_PER_BLOCK;
  static_assert(CAT_LROW_PRE + 8 <= H12_NCSTR_COLS + CAT_LDS_EXTRA, "256 block prefixes in the CaT rows");
  const unsigned long long* pub = cat_cpub(P.crun);
  unsigned long long w[5] = {};
  uint32_t need = 0;
  if (lane <= CPUB_M) need |= 1u;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (lane + 64 * i < nb) need |= 2u << i;
  int k = 0;
  for (; k < CAT_WAIT_POLLS; ++k) {
#pragma unroll
    for (int i = 0; i < 5; ++i)
      if ((need >> i) & 1u) {
        w[i] = ld_sc1(i == 0 ? &pub[lane] : &pub[CPUB_LIST + lane + 64 * (i - 1)]);
        if ((unsigned)(w[i] >> 32) == e1) need &= ~(1u << i);
      }
    if (__ballot(need != 0) == 0) break;
    __builtin_amdgcn_s_sleep(2);
  }
  if (k == CAT_WAIT_POLLS && lane == 0) atomicOr(P.diag, 2);
  const int m = __shfl((int)(unsigned)w[0], CPUB_M, 64);
  float* rinv = &cv[CAT_LROW_RINV][0];  // two rows: 64 floats
  if (lane < H12_NCSTR_COLS) rinv[lane] = __uint_as_float((unsigned)w[0]);
  int* pre = reinterpret_cast<int*>(&cv[CAT_LROW_PRE][0]);  // the blocks' prefixes, 8 rows: 256 ints
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (lane + 64 * i < nb) pre[lane + 64 * i] = (int)(unsigned)w[1 + i];
  wave_sync();
  float keep = 1.f;
  float lg[2 * H12_NCSTR] = {};
  // env he's remapped row: the (he mod m)-th still env, in the last block whose prefix is <= he mod m
  const float* srow = nullptr;
  if (on && m > 0) {
    const int kk = he % m;
    int lo = 0, hi = nb - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (pre[mid] <= kk) lo = mid;
      else hi = mid - 1;
    }
    srow = cat_rows(P.crun, W.n) + (size_t)lo * CAT_NMC * ENVS_PER_BLOCK + (kk - pre[lo]);
  }
  if (on) keep = cat_prob_env(W, A, he, j, reset, vs, vp, srow, rinv, lg);
  // the block's episode statistics: the value rows reused (every lane has read its values)
  const bool any = __ballot(on && reset) != 0;
  wave_sync();
  if (any && (lane & 1) == 0)
#pragma unroll
    for (int k = 0; k < 2 * H12_NCSTR; ++k) cv[k][j] = lg[k];
  wave_sync();
  cat_log_block(P.cmask, cv, lane, any, A.log_part, gridDim.x, step_block());  // the envs' block: cat_prob_kernel's slot
  return keep;
}

// LDS budget of step_kernel (round 6): the static hand-offs (HelpLds, SelfLds; the same for every feature level K) plus
// the fused path's dynamic FuseLds must fit the CU's 160 KiB.  A dispatch over the limit is not a HIP error code: the
// queue aborts (HSA_STATUS_ERROR_INVALID_ALLOCATION) and the next call reports an illegal address (round 5's r7e
// variant, group_seg_size 166416).  Checked here at compile time and at h12env_create against the compiled kernel's
// static size and the device's limit (check_step_lds), which refuses the handle with H12_E_STATE instead.
constexpr size_t LDS_CU_BYTES = 160 * 1024;
constexpr size_t STEP_LDS_STATIC = sizeof(HelpLds) + sizeof(SelfLds);
static_assert(STEP_LDS_STATIC + sizeof(FuseLds) <= LDS_CU_BYTES, "step_kernel's static + fused dynamic LDS exceed 160 KiB");

template <int K>
__global__ void __launch_bounds__(4 * BLOCK) step_kernel(KParams P, Workspace W, StepArgs A) {
  H12_BW_KSTART();
  kernarg_warm();
  if (threadIdx.x >= BLOCK) {  // the helper waves (inner_step_hw, helper_wave, contact_wave, self_wave)
    const int nsteps = P.decimation * P.inner;
    FuseCtx fc = {};
    if (A.fuse) {
      const int e0 = step_block() * ENVS_PER_BLOCK, row = H12_OBS_FRAME * P.hist;
      fc = {A.obs_prev + (size_t)e0 * row, A.obs + (size_t)e0 * row, A.fuse_code, row,
            e0 + ENVS_PER_BLOCK <= W.n && nsteps >= 2};
    }
    const int ft = threadIdx.x - BLOCK, fnt = helper_threads(P);  // lane among the helper waves
    if (threadIdx.x < 2 * BLOCK) {
      const int hl = threadIdx.x - BLOCK, hleg = hl & 1;
      const int he = step_block() * ENVS_PER_BLOCK + (hl >> 1);
      // the episode reward sums: this wave computes the rewards after the physics loop (round 5); loaded here, their
      // memory round trip overlaps the loop
      float ep[H12_NREW];
      if (he < W.n) load_epsum<K>(P, W, he, ep);
      helper_wave<K>(P, W.n, nsteps, (uint32_t)(A.env_offset + he), A.lo, A.hi, fc);
      if (A.fuse) fuse_stage(P, A, fc, W.n, ft, fnt);
      {
        __syncthreads();  // L: the final state and the reward inputs (and CaT constraint values)
      }
      // ---- rewards on the pre-reset state (mdp_terms: the 12 Flat / 20 extended terms), the episode sums, the reward
      // output and the episode-log values of the resetting envs -- the physics wave's until round 4: it resets and
      // observes meanwhile (light stamps: sensor + rewards were ~1.0 us of its post-loop 3.7 us)
      constexpr int NT = Feat<K>::ext ? H12_NREW : H12_NREW_FLAT;
      float r = 0.f;
      bool hreset = false;
      // cat_inline: the env's constraint sums, loaded now (their round trip overlaps the rewards and barrier F)
      const bool cat_on = Feat<K>::ext && A.cat_inline && he < W.n && hleg == 0;
      float cvs[H12_NCSTR], cvp[H12_NCSTR];
      if (cat_on)
#pragma unroll
        for (int t = 0; t < H12_NCSTR; ++t) {
          cvs[t] = W.F[(size_t)(H12_F_CSTR_SUM + t) * W.n + he];
          cvp[t] = W.F[(size_t)(H12_F_CSTR_P + t) * W.n + he];
        }
      if (he < W.n) {
        EnvSt rs;
        float org[3];
        RewIn ri;
        get_state(hl, rs.b, rs.lg, org);
        get_rin(hl, ri);
        for (int k = 0; k < NL; ++k) { rs.act[k] = ri.act[k]; rs.act1[k] = ri.act1[k]; }
        for (int a = 0; a < 3; ++a) rs.cmd[a] = ri.cmd[a];
        rs.air = ri.air;
        rs.con = ri.con;
        float R[3][3];
        quat_R(rs.b.quat, R);
        float terms[H12_NREW];
        mdp_terms<K>(P, rs, hleg, R, ri.tau, ri.jacc, ri.fmax_foot, ri.term, terms);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const float v = terms[t] * P.rew_w[t] * P.step_dt;
          r += v;
          ep[t] += v;
        }
        const bool reset = ri.term || ri.tout;
        hreset = reset;
        // episode log: the resetting envs' sums go to LDS and lane v below adds value v over the block into this block's
        // own partial slot (value-major [LOG_NPART][blocks]; one shared accumulator made every wave's atomics queue on
        // the same L2 lines: +4.2 us per step).  The assembly kernel that follows folds the partials into log_acc
        // (log_load / log_fold).
        if (A.log_part && hleg == 0) {
          float(&L)[LOG_NSTEP][ENVS_PER_BLOCK] = help_lds().logv;
          const int j = hl >> 1;
          for (int t = 0; t < NT; ++t) L[t][j] = reset ? ep[t] : 0.f;
          L[H12_NREW][j] = reset ? 1.f : 0.f;
          L[H12_NREW + 1][j] = (reset && ri.tout) ? 1.f : 0.f;
          L[H12_NREW + 2][j] = (reset && ri.term) ? 1.f : 0.f;
          L[H12_NREW + 3][j] = reset ? ri.metric[0] : 0.f;  // CommandTerm.reset: metrics of the ended episode
          L[H12_NREW + 4][j] = reset ? ri.metric[1] : 0.f;
        }
        if (reset)
          for (int t = 0; t < H12_NREW; ++t) ep[t] = 0.f;  // _reset_idx: the episode sums restart
      }
      wave_sync();  // the episode-log values of this wave's lanes
      // lane v: value v summed over the block's envs, stored into this block's partial slot (value-major
      // [LOG_NPART][blocks]: each block owns its slots, so a plain store of every used value, zeros included); on
      // the fused path after the rows, off barrier F's path
      float lacc = 0.f;
      const int v = threadIdx.x - BLOCK;
      const bool lv = A.log_part && v < LOG_NSTEP && (v < NT || v >= H12_NREW);
      if (lv) {
        const int ne = min(ENVS_PER_BLOCK, W.n - step_block() * ENVS_PER_BLOCK);
        const HelpLds& H = help_lds();
        for (int j = 0; j < ne; ++j) lacc += H.logv[v][j];
      }
      if (A.fuse) {
        __builtin_amdgcn_s_waitcnt(0);  // this wave's shifted-row stores have completed (fuse_late rewrites some)
        H12_BW_F_ARRIVAL();
        __syncthreads();                // F: the physics wave's noisy frames and refill flags
        fuse_late(P, A, fc, W.n, ft, fnt);
      }
      if (Feat<K>::ext && A.cat_inline) r *= cat_prob_inline(W, A, he, hl >> 1, cat_on, hreset, cvs, cvp);
      // the reward and the episode sums last: their stores issued before barrier F held the vmcnt(0) ahead of it
      if (he < W.n) {
        if (hleg == 0) A.rew[he] = r;
        store_epsum<K>(P, W, he, hleg, ep);
      }
      if (lv) A.log_part[(size_t)v * gridDim.x + blockIdx.x] = lacc;
    } else {
      if (threadIdx.x < 3 * BLOCK) contact_wave<K>(P, W.n, nsteps, fc);
      else self_wave<K>(P, W.n, nsteps, fc);
      if (A.fuse) fuse_stage(P, A, fc, W.n, ft, fnt);
      __syncthreads();  // L (the helper's final sole contact state is in LDS)
      const bool cat_w = Feat<K>::ext && P.cat && threadIdx.x < 3 * BLOCK;  // the contact wave: the CaT hand-off
      const bool cat_inl = Feat<K>::ext && A.cat_inline;  // (only with A.fuse: barrier F orders the epoch's LDS copy)
      unsigned cat_e0 = 0;
      if (cat_w) cat_e0 = cat_handoff(P, W.n, cat_inl);
      int cat_old = -1;
      if (A.fuse) {
        __builtin_amdgcn_s_waitcnt(0);
        if (cat_w) {
          cat_old = cat_arrive(P);
          // cat_inline: every block's helper wave waits for the fold, so the last block folds at once, while its
          // physics wave resets and observes (off that wave's way to barrier F)
          if (cat_inl) {
            if ((threadIdx.x & 63) == 0) cat_lds()[CAT_LROW_EPOCH][0] = __uint_as_float(cat_e0);
            if (cat_is_last(cat_old)) cat_fold(P, W.n, true);
          }
        }
        H12_BW_F_ARRIVAL();
        __syncthreads();  // F
        fuse_late(P, A, fc, W.n, ft, fnt);
      } else if (cat_w) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        cat_old = cat_arrive(P);
      }
      if (cat_w && !cat_inl && cat_is_last(cat_old)) cat_fold(P, W.n, false);
    }
    PH_HELPER_END();
    return;
  }
  const int lane_pair = threadIdx.x >> 1;
  const int leg = threadIdx.x & 1;
  const float sg = leg ? -1.f : 1.f;
  const int e0 = step_block() * ENVS_PER_BLOCK;
  const int e = e0 + lane_pair;
  const bool active = e < W.n;
  const uint32_t g = (uint32_t)(A.env_offset + e);
  PH_INIT();
  H12_BW_ENTRY();
  if (Feat<K>::ext && P.dz && blockIdx.x == 0 && threadIdx.x == 0) P.dz_cnt[(A.dz_slot + 2) % 3] = 0;
  if (active) {
    EnvSt s;
    load_phys<K>(P, W, e, leg, s);
    // the MDP part of the state is loaded here too: its memory round trip overlaps the physics loop (the episode sums:
    // the helper wave's)
    load_mdp<K, false>(P, W, e, leg, s);
    PH(0);
    // ActionManager.process_action: prev <- action, action <- a ; a_{t-2} kept for the delay ring
    float a_t2[NL];
#pragma unroll
    for (int k = 0; k < NL; ++k) {
      a_t2[k] = s.act1[k];
      s.act1[k] = s.act[k];
      s.act[k] = jsign(k, sg) * A.actions[(size_t)e * NJ + NL * leg + k];
    }
    const int dec = P.decimation;
    float tau[NL], jacc[NL];
    float fmax_knee = 0.f, fmax_torso = 0.f, fmax_foot = 0.f, flast_foot = 0.f;
    uint32_t cflags = 0;  // foot contact flag of every physics step (ContactSensor replay)
    const float wgt = frcp((float)P.inner);
    PdIn pd;  // the delayed PD's inputs (pd_torque, once per physics step in inner_step_hw)
    for (int k = 0; k < NL; ++k) { pd.act[k] = s.act[k]; pd.act1[k] = s.act1[k]; pd.act2[k] = a_t2[k]; }
    pd.lagpk = (s.lag[0] & 7) | (s.lag[1] & 7) << 3 | (s.lag[2] & 7) << 6;
    pd.since_reset = s.since_reset;
    put_state(threadIdx.x, s.b, s.lg, s.origin);
    put_cst(threadIdx.x, s.lg);
    H12_BW_DECL;
    H12_BW_SET_ENTRY();
    SYNC_W(3);  // S: the first inner step's state (and the sole contact state) for the other waves
    for (int st = 0; st < dec; ++st) {
      const bool last = st == dec - 1;
      if (last)
        for (int k = 0; k < NL; ++k) jacc[k] = s.lg.qd[k];
      Forces fr = {};
      for (int it = 0; it < P.inner; ++it)
        inner_step_hw<K>(P, leg, s.b, s.lg, pd, st * P.inner + it, tau, P.h, fr, s.origin,
                         !last || it < P.inner - 1 H12_BW_ARG);
      if (last)
        for (int k = 0; k < NL; ++k) jacc[k] = (s.lg.qd[k] - jacc[k]) * frcp(P.dt);
      // ContactSensor: net force = mean over the inner steps of the physics step
      float fn = fsqrt(fr.foot[0] * fr.foot[0] + fr.foot[1] * fr.foot[1] + fr.foot[2] * fr.foot[2]) * wgt;
      cflags |= (fn > P.cthr ? 1u : 0u) << st;
      flast_foot = fn;
      if (st >= dec - 3) {  // net_forces_w_history (history_length 3)
        fmax_foot = fmaxf(fmax_foot, fn);
        fmax_knee = fmaxf(fmax_knee, wgt * fsqrt(fr.knee[0] * fr.knee[0] + fr.knee[1] * fr.knee[1] + fr.knee[2] * fr.knee[2]));
        fmax_torso = fmaxf(fmax_torso, wgt * fsqrt(fr.torso[0] * fr.torso[0] + fr.torso[1] * fr.torso[1] + fr.torso[2] * fr.torso[2]));
      }
    }
    PH(1);
    H12_BW_STORE();
    // ContactSensor._update_buffers_impl replayed per physics step (threshold 1 N, elapsed = dt)
    for (int st = 0; st < dec; ++st) {
      bool is_c = (cflags >> st) & 1u;
      bool first_c = (s.air > 0.f) && is_c;
      bool first_d = (s.con > 0.f) && !is_c;
      if (first_c) s.last_air = s.air + P.dt;
      s.air = is_c ? 0.f : s.air + P.dt;
      if (first_d) s.last_con = s.con + P.dt;
      s.con = is_c ? s.con + P.dt : 0.f;
    }
    s.eplen += 1;
    // ---- terminations: time_out, illegal_contact (pair-combined)
    PH(2);
    const bool tout = s.eplen >= P.max_len;
    int ill = (P.ill_knees && fmax_knee > P.cthr) || (P.ill_torso && fmax_torso > P.cthr) || base_diverged(s.b);
    const int term = ill | pair_swap_i(ill);
    // ---- rewards on the pre-reset state: the helper wave's (round 5), while this wave resets and observes -- the final
    // state and the terms' other inputs to LDS
    put_state(threadIdx.x, s.b, s.lg, s.origin);
    {
      RewIn ri;
      for (int k = 0; k < NL; ++k) { ri.act[k] = s.act[k]; ri.act1[k] = s.act1[k]; ri.tau[k] = tau[k]; ri.jacc[k] = jacc[k]; }
      for (int a = 0; a < 3; ++a) ri.cmd[a] = s.cmd[a];
      ri.air = s.air; ri.con = s.con; ri.fmax_foot = fmax_foot;
      ri.metric[0] = s.metric[0]; ri.metric[1] = s.metric[1];
      ri.term = term; ri.tout = tout ? 1 : 0;
      put_rin(threadIdx.x, ri);
    }
    if (Feat<K>::ext && P.cat) {
      float R[3][3];
      quat_R(s.b.quat, R);
      cat_constraints<true>(P, W, e, leg, s, tau, fmax_foot, term, R, s.eplen);
    }
    PH(3);
    const bool reset = term || tout;
    if (leg == 0) {
      A.term[e] = (uint8_t)term;
      A.trunc[e] = (uint8_t)tout;
    }
    if (A.applied_torque)
      for (int k = 0; k < NL; ++k) A.applied_torque[(size_t)e * NJ + NL * leg + k] = jsign(k, sg) * tau[k];
    if (A.foot_force) A.foot_force[2 * e + leg] = flast_foot;
    __syncthreads();  // L: the helper wave computes the rewards, the episode sums and the episode-log values
    get_cst(threadIdx.x, s.lg);  // the helper / contact waves' final stiction anchors and sole contact masks
    PH(4);
    if (reset) {
      uint32_t pre[16];
      get_draws(threadIdx.x, pre);
      env_reset<K>(P, s, leg, g, A.lo, A.hi, pre);
    }
    else s.since_reset = min(s.since_reset + 1, 2);
    // ---- CommandTerm.compute(step_dt): UniformVelocityCommand._update_metrics on the post-reset state, then
    // the resampling clock
    cmd_metrics<K>(P, s);
    s.cmd_time -= P.step_dt;
    if (s.cmd_time <= 0.f) {
      uint32_t pre[16];
      get_draws(threadIdx.x, pre);
      cmd_resample(P, s, g, A.lo, A.hi, 0, pre + 8);
    }
    if (Feat<K>::ext && P.dz) {
      cmd_update<K>(P, s, g, A.lo, A.hi, P.dz_cnt[A.dz_slot], W.n);
      if (leg == 0 && s.cmd[0] * s.cmd[0] + s.cmd[1] * s.cmd[1] < P.dz_v * P.dz_v)
        atomicAdd(&P.dz_cnt[(A.dz_slot + 1) % 3], 1);
    } else {
      cmd_update<K>(P, s, g, A.lo, A.hi, 0, W.n);
    }
    // ---- interval events
    push_event<K>(P, s, g, A.lo, A.hi);
    // ---- observation frame (after reset: ObservationManager.compute, cat_env.py:190)
    PH(5);
    if (A.fuse) {
      obs_frame_fused(P, s, leg, lane_pair, term || tout);
      H12_BW_F_ARRIVAL();
      __syncthreads();  // F: the helper waves assemble and store the block's rows
    } else {
      obs_frame<K>(P, s, leg, e, W.n, A.frame);
    }
    PH(6);
    store_env<K, 3>(P, W, e, leg, s);  // the episode sums are the helper wave's
    PH(7);
    PH_WAVE_END();
  }
}

// Self-contact hook (h12env_eval_self_contacts, parity tests only): the self-contact wrenches step_kernel's
// physics applies on the workspace state as it stands, per env [leg][knee, foot][moment xyz, force xyz] in
// REAL body coordinates (the oracle's fext layout).
template <int K>
__global__ void __launch_bounds__(BLOCK) selfc_kernel(KParams P, Workspace W, float* out) {
  const int leg = threadIdx.x & 1;
  const float sg = leg ? -1.f : 1.f;
  const int e = blockIdx.x * ENVS_PER_BLOCK + (threadIdx.x >> 1);
  if (e >= W.n) return;
  EnvSt s;
  load_phys<K>(P, W, e, leg, s);
  float R0[3][3];
  quat_R(s.b.quat, R0);
  float vb[3];
  mtv(R0, s.b.vlin, vb);
  const float mm[3] = {1.f, sg, 1.f};
  float R[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) R[i][j] = mm[i] * mm[j] * R0[i][j];
  float v0[6] = {s.b.wang[0], s.b.wang[1], s.b.wang[2], vb[0], vb[1], vb[2]};
  for (int i = 0; i < 6; ++i) v0[i] *= s6(i, sg);
  float p[3] = {0.f, 0.f, 0.f};  // pelvis-relative positions, as step_kernel's self-contact wave
  float cs[NL][2], v[NL][6];
  link_pass1<0>(s.lg, cs, v0, v, R, p);
  link_pass1<1>(s.lg, cs, v[0], v, R, p);
  link_pass1<2>(s.lg, cs, v[1], v, R, p);
  link_pass1<3>(s.lg, cs, v[2], v, R, p);
  float Rk[3][3], pk[3];
  for (int i = 0; i < 3; ++i) {
    pk[i] = p[i];
    for (int j = 0; j < 3; ++j) Rk[i][j] = R[i][j];
  }
  link_pass1<4>(s.lg, cs, v[3], v, R, p);
  link_pass1<5>(s.lg, cs, v[4], v, R, p);
  float wk[6], wf[6];
  Forces fr = {};
  self_contacts(P, leg, s.lg.mud, Rk, pk, v[3], R, p, v[5], wk, wf, fr);
  float* o = out + ((size_t)e * 2 + leg) * 12;
  for (int a = 0; a < 3; ++a) {  // lane body frame -> real body frame (force M f, moment sg M m)
    o[a] = sg * mm[a] * wk[a]; o[3 + a] = mm[a] * wk[3 + a];
    o[6 + a] = sg * mm[a] * wf[a]; o[9 + a] = mm[a] * wf[3 + a];
  }
}

// Term-evaluation hook (h12env_eval_terms, parity tests only): the reward terms, terminations and CaT constraint
// values of step_kernel's code on a state written into the workspace (post-physics, pre-reset; EPLEN already
// counted) plus injected per-step quantities: applied torques, joint accelerations, and the per-body maxima over
// the contact history (left / right foot, left / right knee, torso).
struct TermArgs {
  const float* tau;   // (n, 12) real joint frame
  const float* jacc;  // (n, 12)
  const float* fmax;  // (n, 5)
  float* terms;       // [H12_NREW][n]
  uint8_t* term;      // (n,)
  uint8_t* trunc;     // (n,)
};
template <int K>
__global__ void __launch_bounds__(BLOCK) terms_kernel(KParams P, Workspace W, TermArgs T) {
  const int leg = threadIdx.x & 1;
  const float sg = leg ? -1.f : 1.f;
  const int e = blockIdx.x * ENVS_PER_BLOCK + (threadIdx.x >> 1);
  if (e >= W.n) return;
  EnvSt s;
  load_phys<K>(P, W, e, leg, s);
  load_mdp<K>(P, W, e, leg, s);
  float tau[NL], jacc[NL];
  for (int k = 0; k < NL; ++k) {
    tau[k] = jsign(k, sg) * T.tau[(size_t)e * NJ + NL * leg + k];
    jacc[k] = jsign(k, sg) * T.jacc[(size_t)e * NJ + NL * leg + k];
  }
  const float fmax_foot = T.fmax[5 * (size_t)e + leg], fmax_knee = T.fmax[5 * (size_t)e + 2 + leg];
  const float fmax_torso = T.fmax[5 * (size_t)e + 4];
  int ill = (P.ill_knees && fmax_knee > P.cthr) || (P.ill_torso && fmax_torso > P.cthr) || base_diverged(s.b);
  const int term = ill | pair_swap_i(ill);
  float R[3][3];
  quat_R(s.b.quat, R);
  float terms[H12_NREW];
  for (int t = 0; t < H12_NREW; ++t) terms[t] = 0.f;
  mdp_terms<K>(P, s, leg, R, tau, jacc, fmax_foot, term, terms);
  if (leg == 0) {
    for (int t = 0; t < H12_NREW; ++t) T.terms[(size_t)t * W.n + e] = terms[t];
    T.term[e] = (uint8_t)term;
    T.trunc[e] = (uint8_t)(s.eplen >= P.max_len);
  }
  // no swing-state write-back: the hook leaves the workspace as it found it
  if (Feat<K>::ext && P.cat) cat_constraints<false, false>(P, W, e, leg, s, tau, fmax_foot, term, R, s.eplen);
}


// CaT, last: per env, p = min_p + clamp(c / running_max, 0, 1) (max_p - min_p) on violated columns, the max over
// all columns scales the reward (CaTEnv.step, cat_env.py:148-153) and is returned as dones (1 where the env
// was reset); ConstraintManager's episode statistics, logged and cleared for the envs reset this step.
struct CatArgs {
  float* rew;
  const uint8_t* term;
  const uint8_t* trunc;
  float* cstr_prob;
  float* log_part;  // the handle's per-block log partials ([LOG_NPART][log_nb]), or null: no log
  int log_nb;
};
constexpr int CAT_PBLOCK = 64;
__global__ void __launch_bounds__(CAT_PBLOCK) cat_prob_kernel(KParams P, Workspace W, CatArgs A) {
  static_assert(CAT_PBLOCK == 2 * ENVS_PER_BLOCK, "one wave: two step_kernel blocks' envs");
  __shared__ float Lg[2][2 * H12_NCSTR][ENVS_PER_BLOCK];  // the episode statistics of both step blocks (cat_log_block)
  const int n = W.n;
  const int i = blockIdx.x * CAT_PBLOCK + threadIdx.x;
  const bool valid = i < n;
  const int ii = valid ? i : n - 1;  // (the tail lanes compute on a real env and write nothing)
  const float* S = P.cscr;
  // every load is issued up front (one memory round trip for the env's own rows and statistics, one more
  // for the no_move rows of the remapped env), then branch-free arithmetic
  float cv[H12_NCSTR_COLS], vs[H12_NCSTR], vp[H12_NCSTR];
  constexpr int NM0 = C_COL0[H12_C_NO_MOVE], NM1 = C_COL0[H12_C_NO_MOVE + 1];
#pragma unroll
  for (int col = 0; col < H12_NCSTR_COLS; ++col)
    if (col < NM0 || col >= NM1) cv[col] = S[(size_t)col * n + ii];
#pragma unroll
  for (int t = 0; t < H12_NCSTR; ++t) {
    vs[t] = W.F[(size_t)(H12_F_CSTR_SUM + t) * n + ii];
    vp[t] = W.F[(size_t)(H12_F_CSTR_P + t) * n + ii];
  }
  const float len = S[(size_t)CAT_ROW_EPLEN * n + ii];
  const int m = P.cmeta[0];
  const int src = m > 0 ? P.clist[ii % m] : -1;
  const int srow = src >= 0 ? src : ii;
#pragma unroll
  for (int col = NM0; col < NM1; ++col) cv[col] = src >= 0 ? S[(size_t)col * n + srow] : 0.f;
  float pmax = 0.f;
  float pt[H12_NCSTR];
#pragma unroll
  for (int t = 0; t < H12_NCSTR; ++t) {
    pt[t] = 0.f;
    const bool on = (P.cmask >> t) & 1u;
#pragma unroll
    for (int col = C_COL0[t]; col < C_COL0[t + 1]; ++col) {
      const float c = cv[col];
      // c / running_max as c * (1 / running_max): within 1 ulp of the division
      const float p = P.cminp + fminf(fmaxf(c * P.crun[H12_NCSTR_COLS + col], 0.f), 1.f) * (P.cmaxp[t] - P.cminp);
      pt[t] = fmaxf(pt[t], (on && c > 0.f) ? p : 0.f);
    }
    pmax = fmaxf(pmax, pt[t]);
  }
  // the factor pinned: r * (1 - p) left to the compiler became fma(-p, r, r) in one kernel and not the other
  float keep = 1.f - pmax;
  pin(keep);
  const bool reset = valid && (A.term[ii] || A.trunc[ii]);
  if (valid) {
    A.rew[i] *= keep;
    if (A.cstr_prob) A.cstr_prob[i] = reset ? 1.f : pmax;
  }
  const float inv_len = 1.f / len;
  const int g = threadIdx.x / ENVS_PER_BLOCK, j = threadIdx.x % ENVS_PER_BLOCK;
#pragma unroll
  for (int t = 0; t < H12_NCSTR; ++t) {
    Lg[g][t][j] = Lg[g][H12_NCSTR + t][j] = 0.f;
    if (!((P.cmask >> t) & 1u)) continue;
    float a = vs[t] + (pt[t] > 0.f ? 1.f : 0.f), b = vp[t] + pt[t];
    if (reset) {
      Lg[g][t][j] = a * inv_len;
      Lg[g][H12_NCSTR + t][j] = b * inv_len;
      a = b = 0.f;
    }
    if (valid) {
      W.F[(size_t)(H12_F_CSTR_SUM + t) * n + i] = a;
      W.F[(size_t)(H12_F_CSTR_P + t) * n + i] = b;
    }
  }
  // the episode statistics per step_kernel block, summed in env order (the order cat_prob_inline sums in)
  const uint64_t rs = __ballot(reset);
  wave_sync();
  const int slot = blockIdx.x * 2 + g;
  if (slot < A.log_nb)
    cat_log_block(P.cmask, Lg[g], j, ((rs >> (g * ENVS_PER_BLOCK)) & 0xffffffffull) != 0, A.log_part, A.log_nb, slot);
}

template <int K>
__global__ void __launch_bounds__(BLOCK) reset_kernel(KParams P, Workspace W, StepArgs A) {
  const int lane_pair = threadIdx.x >> 1;
  const int leg = threadIdx.x & 1;
  const int e0 = blockIdx.x * ENVS_PER_BLOCK;
  const int e = e0 + lane_pair;
  const bool sel = e < W.n && (!A.reset_mask || A.reset_mask[e]);
  if (sel) {
    const uint32_t g = (uint32_t)(A.env_offset + e);
    EnvSt s;
    load_env<K>(P, W, e, leg, s);
    env_reset<K>(P, s, leg, g, A.lo, A.hi);
    obs_frame<K>(P, s, leg, e, W.n, A.frame);
    store_env<K>(P, W, e, leg, s);
  }
}

// ObservationManager.compute() outside step(): new frame from the current state, history shifted
// (or filled where fill_mask[e]); RNG counter domain (observe call, 0xFFFFFFFE)
template <int K>
__global__ void __launch_bounds__(BLOCK) observe_kernel(KParams P, Workspace W, StepArgs A) {
  const int lane_pair = threadIdx.x >> 1;
  const int leg = threadIdx.x & 1;
  const int e0 = blockIdx.x * ENVS_PER_BLOCK;
  const int e = e0 + lane_pair;
  if (e < W.n) {
    EnvSt s;
    load_env<K>(P, W, e, leg, s);
    obs_frame<K>(P, s, leg, e, W.n, A.frame);
  }
}

// parity hook (h12env_step_physics): n_substeps physics steps, PD to held q_ref every physics step
template <int K>
__global__ void __launch_bounds__(BLOCK) physics_kernel(KParams P, Workspace W, StepArgs A) {
  const int lane_pair = threadIdx.x >> 1;
  const int leg = threadIdx.x & 1;
  const float sg = leg ? -1.f : 1.f;
  const int e = blockIdx.x * ENVS_PER_BLOCK + lane_pair;
  if (e >= W.n) return;
  EnvSt s;
  load_env<K>(P, W, e, leg, s);
  float qr[NL];
  for (int k = 0; k < NL; ++k) qr[k] = jsign(k, sg) * A.q_ref[(size_t)e * NJ + NL * leg + k];
  for (int st = 0; st < A.n_substeps; ++st) {
    float tau[NL];
    for (int k = 0; k < NL; ++k) {
      float v = P.kp[k] * (qr[k] - s.lg.q[k]) - P.kd[k] * s.lg.qd[k];
      tau[k] = fminf(fmaxf(v, -P.elim[k]), P.elim[k]);
    }
    Forces fr = {};
    for (int it = 0; it < P.inner; ++it) inner_step_1w<K>(P, leg, s.b, s.lg, tau, P.h, fr, s.origin);
  }
  store_env<K>(P, W, e, leg, s);
}

// ------------------------------------------------------------------ rollout records (C4: all-gathered rollouts)
// Step record of one shard (h12env_rollout_layout): frames f32 [n][45], actions f32 [n][12], rewards f32 [n],
// terminated u8 [n], truncated u8 [n], each section 256-B aligned; gathered in chunks of G steps (see the header).
inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }
void rollout_offsets(int n, size_t* off, size_t* step) {
  const size_t nn = (size_t)n;
  off[0] = 0;
  off[1] = align256(off[0] + nn * H12_OBS_FRAME * 4);
  off[2] = align256(off[1] + nn * H12_NJ * 4);
  off[3] = align256(off[2] + nn * 4);
  off[4] = align256(off[3] + nn);
  *step = align256(off[4] + nn);
}

// Observation rows from rollout records (h12env_rollout_decode).  One block per DEC_ENVS consecutive envs of one
// shard, all rows of [t0, t1) in windows of DEC_WT rows: the block stages its envs' tail rows once and, per window,
// the frames the window's rows can reach (steps [w0 - (H - 1), w1)) and each env's last done step per row, then
// writes the rows -- for a fixed t the block's ne rows are one contiguous run of ne * 45H floats (float4 stores
// when 16-B aligned).  HBM-bound on the row stores; each frame is read once per window.
constexpr int DEC_ENVS = 8, DEC_BLOCK = 256, DEC_WT = 16, DEC_FR = DEC_WT + H12_NHIST - 1, DEC_MAX_BLOCKS = 96;
struct DecArgs {
  const uint8_t* rec;  // gathered records
  size_t step_bytes, off[5];
  int n_shards, n, T, G, t0, t1;
  const float* tail;
  float* out;
};
// step s of shard r in the gathered buffer (chunk-major, then shard, then step)
__device__ __forceinline__ const uint8_t* dec_step(const DecArgs& D, int r, int s) {
  const int c = s / D.G, gc = min(D.G, D.T - c * D.G);
  return D.rec + ((size_t)c * D.G * D.n_shards + (size_t)r * gc + (size_t)(s - c * D.G)) * D.step_bytes;
}
// float copy global -> LDS, float4 when both ends are 16-B aligned (all loads issued before any use)
__device__ __forceinline__ void dec_stage(float* dst, const float* src, int cnt, int tid) {
  if ((((uintptr_t)src | (uintptr_t)dst) & 15u) == 0) {
    const float4* s4 = reinterpret_cast<const float4*>(src);
    float4* d4 = reinterpret_cast<float4*>(dst);
    for (int j = tid; j < cnt / 4; j += DEC_BLOCK) d4[j] = s4[j];
    for (int k = (cnt / 4) * 4 + tid; k < cnt; k += DEC_BLOCK) dst[k] = src[k];
  } else {
    for (int k = tid; k < cnt; k += DEC_BLOCK) dst[k] = src[k];
  }
}

template <int NH>
__global__ void __launch_bounds__(DEC_BLOCK) rollout_decode_kernel(DecArgs D) {
  constexpr int ROW = H12_OBS_FRAME * NH;
  __shared__ __attribute__((aligned(16))) float s_tail[DEC_ENVS * ROW];
  __shared__ __attribute__((aligned(16))) float s_fr[DEC_FR][DEC_ENVS * H12_OBS_FRAME];
  __shared__ uint8_t s_dn[DEC_FR][DEC_ENVS];
  __shared__ int s_last[DEC_ENVS][DEC_WT];
  __shared__ uint32_t s_col[ROW];
  const int tid = threadIdx.x;
  const int bps = (D.n + DEC_ENVS - 1) / DEC_ENVS;
  const size_t NG = (size_t)D.n_shards * D.n;
  for (int col = tid; col < ROW; col += DEC_BLOCK) {  // frame component, term width, slot (0 oldest)
    const uint32_t ce = asm_col_entry<NH>(col);
    const int c = (int)(ce & 0xFFu);
    const int h = c < 9 ? (col % (3 * NH)) / 3 : ((col - 9 * NH) % (12 * NH)) / 12;
    s_col[col] = (ce & 0xFFFFu) | ((uint32_t)h << 16);
  }
  // a capped grid strides over the env groups (DEC_MAX_BLOCKS: a caller may launch the decode on a stream of its own
  // beside the env kernels, which then keep CUs; h12env.rollout's RolloutGather launches it on the env's stream)
  for (int grp = blockIdx.x; grp < D.n_shards * bps; grp += gridDim.x) {
  const int shard = grp / bps, e0 = (grp - shard * bps) * DEC_ENVS;
  const int ne = min(DEC_ENVS, D.n - e0);
  const size_t g0 = (size_t)shard * D.n + e0;
  __syncthreads();  // the previous group's stores read s_tail
  // the envs' rows before step 0 (every read of them precedes the first row store: tail may alias the output)
  dec_stage(s_tail, D.tail + g0 * ROW, ne * ROW, tid);
  for (int w0 = D.t0; w0 < D.t1; w0 += DEC_WT) {
    const int w1 = min(w0 + DEC_WT, D.t1);
    // steps a row of the window can reach: [w0 - (H - 1), w1).  A done step before f0 cannot matter (every slot's
    // step is >= t - (H - 1) >= f0), so the last done step is looked for inside the window only
    const int f0 = max(0, w0 - (NH - 1)), nf = w1 - f0;
    __syncthreads();  // the previous window's stores read s_fr / s_last
    for (int ts = 0; ts < nf; ++ts)
      dec_stage(s_fr[ts], reinterpret_cast<const float*>(dec_step(D, shard, f0 + ts) + D.off[0]) + (size_t)e0 * H12_OBS_FRAME,
                ne * H12_OBS_FRAME, tid);
    if (tid < nf * ne) {
      const int ts = tid / ne, e = tid - ts * ne;
      const uint8_t* st = dec_step(D, shard, f0 + ts);
      s_dn[ts][e] = st[D.off[3] + e0 + e] | st[D.off[4] + e0 + e];
    }
    __syncthreads();
    if (tid < ne) {
      int last = -1;
      for (int ts = 0; ts < nf; ++ts) {
        if (s_dn[ts][tid]) last = f0 + ts;
        if (f0 + ts >= w0) s_last[tid][f0 + ts - w0] = last;
      }
    }
    __syncthreads();
    for (int t = w0; t < w1; ++t) {
      float* dst = D.out + ((size_t)t * NG + g0) * ROW;
      auto value = [&](int k) -> float {
        const int e = k / ROW, col = k - e * ROW;
        const uint32_t ce = s_col[col];
        const int c = (int)(ce & 0xFFu), d = (int)((ce >> 8) & 0xFFu), h = (int)(ce >> 16);
        int src = t - (NH - 1 - h);
        const int last = s_last[e][t - w0];
        if (src < last) src = last;
        return src >= 0 ? s_fr[src - f0][e * H12_OBS_FRAME + c] : s_tail[e * ROW + col + (t + 1) * d];
      };
      const int cnt = ne * ROW;
      if (((uintptr_t)dst & 15u) == 0) {
        float4* d4 = reinterpret_cast<float4*>(dst);
        for (int j = tid; j < cnt / 4; j += DEC_BLOCK)
          d4[j] = make_float4(value(4 * j), value(4 * j + 1), value(4 * j + 2), value(4 * j + 3));
        for (int k = (cnt / 4) * 4 + tid; k < cnt; k += DEC_BLOCK) dst[k] = value(k);
      } else {
        for (int k = tid; k < cnt; k += DEC_BLOCK) dst[k] = value(k);
      }
    }
  }
  }
}

// ------------------------------------------------------------------ host side
struct Handle {
  KParams P;
  Workspace W;
  bool own;
  int device;
  int64_t env_offset;
  uint64_t reset_calls, observe_calls;
  double flops_per_env;
  float* frame;  // [45][n] observation frame scratch between the env kernels and obs_assemble_kernel
  int* dz_cnt = nullptr;  // 3 rotating deadzone counters (UniformVelocityCommandWithDeadzone), then the diagnostic word
  size_t lds_static = 0;  // step_kernel's static LDS as compiled (hipFuncGetAttributes) and the device's LDS per CU
  int lds_limit = 0;
  bool cat_inline = false;  // CaT's probabilities inside step_kernel (cat_prob_inline; check_cat_inline)
  uint64_t dz_step = 0;
  void* cat_mem = nullptr;  // CaT buffers (scratch, column keys, running maxima, no_move list, meta)
  bool timing = false;
  int16_t* asm_tab = nullptr;  // obs_assemble_kernel gather table for P.hist (Flat / Rsl layouts)
  bool fuse = false;           // step_kernel assembles the observation rows itself (FuseCtx; else obs_assemble_kernel)
  uint8_t* fuse_code = nullptr;  // fuse_code_table(P.hist) on the device
  float* log_part = nullptr;   // ring of LOG_RING [LOG_NPART][step blocks] episode-log partial sets (step_kernel ->
                               // the assembly kernel's immediate fold, or log_flush_kernel for fused steps)
  int log_pos = 0;             // ring slot of the next step with a log
  int n_pend = 0;              // fused steps whose partials await log_flush_kernel (ring slots log_pos - n_pend ..)
  float* pend_acc[LOG_RING] = {};
  // kernel timing: 4 events per timed step bound to the launches themselves (hipExtLaunchKernelGGL:
  // the events take the dispatch packet's begin / end timestamps, as rocprofv3's kernel trace does) --
  // step_kernel begin / end, observation kernel begin / end
  std::vector<hipEvent_t> ev;
  std::vector<uint8_t> ev_k1;  // per timed step: its pair 1 was recorded (a fused step without a flush has none)
  size_t n_timed = 0;
};

constexpr size_t MAX_TIMED_STEPS = 4096;

// the event pair of kernel k (0 = env kernel, 1 = the step's second kernel: assembly or log fold) of the current
// timed step, or nulls; timing_next moves on to the next step
bool timing_events(Handle* h, int k, hipEvent_t* e0, hipEvent_t* e1) {
  *e0 = *e1 = nullptr;
  if (!h->timing || h->n_timed >= MAX_TIMED_STEPS) return false;
  const size_t i = 4 * h->n_timed + 2 * k;
  while (h->ev.size() <= i + 1) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) { h->timing = false; return false; }
    h->ev.push_back(e);
  }
  *e0 = h->ev[i];
  *e1 = h->ev[i + 1];
  if (h->ev_k1.size() <= h->n_timed) h->ev_k1.resize(h->n_timed + 1, 0);
  if (k == 1) h->ev_k1[h->n_timed] = 1;
  return true;
}
// the current timed step's pair 1 is already in use (a log fold flushed ahead of it)
bool pair1_taken(const Handle* h) { return h->n_timed < h->ev_k1.size() && h->ev_k1[h->n_timed]; }
void timing_next(Handle* h) {
  if (!h->timing || h->n_timed >= MAX_TIMED_STEPS) return;
  h->n_timed++;
  if (h->ev_k1.size() > h->n_timed) h->ev_k1[h->n_timed] = 0;
}

bool close(float a, float b) { return fabsf(a - b) <= 1e-6f * (1.f + fabsf(a) + fabsf(b)); }

// the kernel compiles the H1-2 model in (h12_model_gen.h); refuse any other model
int check_model(const h12env_model* m) {
  for (int leg = 0; leg < 2; ++leg)
    for (int k = 0; k < NL; ++k) {
      int j = NL * leg + k;
      int want_parent = k == 0 ? -1 : j - 1;
      if (m->parent[j] != want_parent || m->axis[j] != AX[k])
        return set_err(H12_E_ARG, "model joint %d: tree/axis differ from the compiled H1-2 model", j);
      float my = leg ? -1.f : 1.f;
      float js = AX[k] == 1 ? 1.f : my;
      bool ok = close(m->joint_pos[j][0], h12m::R[k][0]) && close(m->joint_pos[j][1], my * h12m::R[k][1]) &&
                close(m->joint_pos[j][2], h12m::R[k][2]) && close(m->link_mass[j], h12m::M[k]) &&
                close(m->link_com[j][0], h12m::COM[k][0]) && close(m->link_com[j][1], my * h12m::COM[k][1]) &&
                close(m->link_com[j][2], h12m::COM[k][2]) && close(m->armature[j], h12m::ARM[k]) &&
                close(m->damping[j], h12m::DAMP[k]) && close(m->q_default[j], js * h12m::Q0[k]) &&
                close(fminf(js * m->q_lower[j], js * m->q_upper[j]), h12m::QLO[k]) &&
                close(fmaxf(js * m->q_lower[j], js * m->q_upper[j]), h12m::QHI[k]);
      if (!ok) return set_err(H12_E_ARG, "model joint %d differs from the compiled H1-2 model (regenerate h12_model_gen.h)", j);
    }
  if (!close(m->base_mass, h12m::BASE_M) || !close(m->base_com[0], h12m::BASE_COM[0]) ||
      !close(m->base_com[2], h12m::BASE_COM[2]) || !close(m->foot_radius, h12m::FOOT_R) ||
      !close(m->knee_radius, h12m::KNEE_R) || !close(m->torso_com[0], h12m::TORSO_COM[0]) ||
      !close(m->torso_com[1], h12m::TORSO_COM[1]) || !close(m->torso_com[2], h12m::TORSO_COM[2]) ||
      !close(m->root_com[0], h12m::ROOT_COM[0]) || !close(m->root_com[1], h12m::ROOT_COM[1]) ||
      !close(m->root_com[2], h12m::ROOT_COM[2]))
    return set_err(H12_E_ARG, "base / contact geometry differs from the compiled H1-2 model");
  for (int r = 0; r < 4; ++r)
    for (int e = 0; e < 2; ++e)
      for (int a = 0; a < 3; ++a)
        if (!close(m->foot_rods[r][e][a], h12m::ROD[r][e][a]))
          return set_err(H12_E_ARG, "sole rod geometry differs from the compiled H1-2 model");
  return 0;
}

int build_params(const h12env_model* m, const h12env_config* c, KParams& P) {
  memset(&P, 0, sizeof P);
  if (int rc = check_model(m)) return rc;
  if (c->decimation < 1 || c->decimation > MAX_DEC || c->inner_steps < 1 || !(c->physics_dt > 0))
    return set_err(H12_E_ARG, "bad decimation (1..%d) / inner_steps / dt", MAX_DEC);
  if (c->mode != H12_MODE_ISAACLAB && c->mode != H12_MODE_MUJOCO) return set_err(H12_E_ARG, "bad mode %d", c->mode);
  if (c->min_delay < 0 || c->max_delay < c->min_delay || c->max_delay > 7 || c->max_delay > 2 * c->decimation)
    return set_err(H12_E_ARG, "delay range [%d,%d] unsupported", c->min_delay, c->max_delay);
  for (int k = 0; k < NL; ++k) {
    if (c->delay_group[k] != c->delay_group[NL + k] || c->delay_group[k] < 0 || c->delay_group[k] > 2)
      return set_err(H12_E_ARG, "delay groups must be leg-symmetric and in 0..2");
    if (c->kp[k] != c->kp[NL + k] || c->kd[k] != c->kd[NL + k] || c->effort_limit[k] != c->effort_limit[NL + k] ||
        c->max_joint_vel[k] != c->max_joint_vel[NL + k] || c->max_joint_vel[k] < 0)
      return set_err(H12_E_ARG, "gains / velocity limits must be leg-symmetric (and >= 0)");
  }
  if (!(c->friction_k > 0)) return set_err(H12_E_ARG, "friction_k must be > 0");
  const bool mj = c->mode == H12_MODE_MUJOCO;
  for (int k = 0; k < NL; ++k) {
    P.kp[k] = c->kp[k];
    P.kd[k] = c->kd[k];
    P.elim[k] = mj ? m->mj_frc_limit[k] : c->effort_limit[k];
    P.dimpl[k] = mj ? m->damping[k] : 0.f;
    P.dgroup[k] = c->delay_group[k];
    P.vmax[k] = (c->max_joint_vel[k] > 0.f && c->max_joint_vel_damping > 0.f) ? c->max_joint_vel[k] : 3.0e38f;
  }
  P.cv = c->max_joint_vel_damping;
  P.g = m->gravity;
  P.mode = c->mode;
  P.fix_base = c->fix_base;
  P.decimation = c->decimation;
  P.inner = c->inner_steps;
  P.max_len = c->max_episode_length;
  P.min_delay = c->min_delay;
  P.max_delay = c->max_delay;
  P.use_fl = c->use_frictionloss;
  P.corrupt = c->enable_corruption;
  P.ill_knees = c->illegal_contact_knees;
  P.ill_torso = c->illegal_contact_torso;
  P.dt = c->physics_dt;
  P.h = c->physics_dt / (float)c->inner_steps;
  P.step_dt = c->physics_dt * (float)c->decimation;
  P.action_scale = c->action_scale;
  P.soft_f = c->soft_limit_factor;
  P.ck = c->contact_k; P.cc = c->contact_c; P.fk = c->friction_k; P.fc = c->friction_c;
  P.mus = c->mu_static; P.mud = c->mu_dynamic; P.lk = c->limit_k; P.lc = c->limit_c;
  P.fc_v = c->friction_c;
  P.impl = c->implicit_penalty != 0;
  P.self_coll = c->self_collision != 0;
  P.sk = c->self_k; P.sc = c->self_c; P.sct = c->self_ct; P.smu = c->self_mu;
  if (!(c->limit_projection >= 0.f)) return set_err(H12_E_ARG, "limit_projection must be >= 0");
  P.lproj = c->limit_projection > 0.f ? c->limit_projection : 3.0e38f;
  if (!(c->max_depenetration_velocity >= 0.f)) return set_err(H12_E_ARG, "max_depenetration_velocity must be >= 0");
  P.dl = 0.f;
  if (P.impl) {  // the springs act at the end of the substep: extra damping h k (oracle contact_point)
    P.cc = c->contact_c + P.h * c->contact_k;
    P.fc = c->friction_c + P.h * c->friction_k;
    P.lc = c->limit_c + P.h * c->limit_k;
    P.dl = P.h * P.lc;
  }
  P.dcap = (P.impl && c->max_depenetration_velocity > 0.f) ? P.h * c->max_depenetration_velocity : 3.0e38f;
  P.cthr = c->contact_threshold;
  P.cmd_T = c->cmd_resample_time;
  P.cmd_x0 = c->cmd_lin_x[0]; P.cmd_x1 = c->cmd_lin_x[1];
  P.cmd_y0 = c->cmd_lin_y[0]; P.cmd_y1 = c->cmd_lin_y[1];
  P.cmd_w0 = c->cmd_ang_z[0]; P.cmd_w1 = c->cmd_ang_z[1];
  P.cmd_h0 = c->cmd_heading[0]; P.cmd_h1 = c->cmd_heading[1];
  P.rel_stand = c->rel_standing_envs; P.rel_head = c->rel_heading_envs; P.head_k = c->heading_stiffness;
  P.rx0 = c->reset_x[0]; P.rx1 = c->reset_x[1]; P.ry0 = c->reset_y[0]; P.ry1 = c->reset_y[1];
  P.ryaw0 = c->reset_yaw[0]; P.ryaw1 = c->reset_yaw[1];
  P.root_z = m->root_height;
  P.n_w = c->noise_ang_vel; P.n_g = c->noise_gravity; P.n_q = c->noise_joint_pos; P.n_qd = c->noise_joint_vel;
  for (int t = 0; t < H12_NREW; ++t) P.rew_w[t] = c->rew_w[t];
  P.std2_inv = 1.f / (c->track_std * c->track_std);
  P.air_thr = c->air_time_threshold;
  P.seed_lo = (uint32_t)c->seed;
  P.seed_hi = (uint32_t)(c->seed >> 32);
  if (c->task != H12_TASK_FLAT && c->task != H12_TASK_ROUGH) return set_err(H12_E_ARG, "bad task %d", c->task);
  if (c->terrain_curriculum && !c->terrain) return set_err(H12_E_ARG, "terrain_curriculum needs terrain = 1");
  if (c->task == H12_TASK_ROUGH && !(c->scan_resolution > 0)) return set_err(H12_E_ARG, "scan_resolution must be > 0");
  P.task = c->task;
  P.terrain = c->terrain;
  P.curriculum = c->terrain_curriculum;
  P.env_mu = c->per_env_friction;
  P.env_mass = c->per_env_mass;
  P.n_lin = c->noise_lin_vel;
  P.n_scan = c->noise_height_scan;
  P.scan_off = c->scan_offset;
  P.scan_clip = c->scan_clip;
  P.scan_res = c->scan_resolution;
  P.terrain_size = c->terrain_size;
  P.ep_len_s = (float)c->max_episode_length * P.step_dt;
  // Rsl task
  if (!(c->cmd_resample_time_max >= c->cmd_resample_time))
    return set_err(H12_E_ARG, "cmd_resample_time_max must be >= cmd_resample_time");
  P.cmd_T1 = c->cmd_resample_time_max;
  P.rsl = 0;
  for (int t = H12_NREW_FLAT; t < H12_NREW; ++t) P.rsl |= c->rew_w[t] != 0.f;
  P.dz = c->cmd_deadzone;
  P.dz_v = c->velocity_deadzone;
  P.flip_p = c->ang_flip_prob;
  P.push = c->push_enable;
  if (P.push && !(c->push_interval[1] >= c->push_interval[0] && c->push_interval[0] > 0))
    return set_err(H12_E_ARG, "push_interval must be 0 < lo <= hi");
  P.push_t0 = c->push_interval[0]; P.push_t1 = c->push_interval[1];
  P.push_x0 = c->push_vel_x[0]; P.push_x1 = c->push_vel_x[1];
  P.push_y0 = c->push_vel_y[0]; P.push_y1 = c->push_vel_y[1];
  if (c->task == H12_TASK_FLAT && (c->history_length < 1 || c->history_length > H12_NHIST))
    return set_err(H12_E_ARG, "history_length %d out of 1..%d", c->history_length, H12_NHIST);
  P.hist = c->task == H12_TASK_FLAT ? c->history_length : 1;
  for (int t = 0; t < 6; ++t) P.oscale[t] = c->obs_scale[t];
  if (c->task == H12_TASK_ROUGH)
    for (int t = 0; t < 6; ++t)
      if (c->obs_scale[t] != 1.f) return set_err(H12_E_ARG, "observation scales need the flat layout");
  P.h_target = c->base_height_target;
  P.cf_thr = c->contact_force_threshold;
  // CaT
  P.cat = c->cat_enable;
  P.cmask = c->cstr_mask;
  for (int t = 0; t < H12_NCSTR; ++t) P.cmaxp[t] = c->cstr_max_p[t];
  P.ctau = c->cat_tau;
  P.cminp = c->cat_min_p;
  for (int k = 0; k < NL; ++k) {
    if (c->cstr_joint_vel_limit[k] != c->cstr_joint_vel_limit[NL + k] ||
        c->cstr_joint_effort_limit[k] != c->cstr_joint_effort_limit[NL + k])
      return set_err(H12_E_ARG, "constraint joint limits must be leg-symmetric");
    P.cvlim[k] = c->cstr_joint_vel_limit[k];
    P.celim[k] = c->cstr_joint_effort_limit[k];
  }
  P.c_ff = c->cstr_foot_force_limit;
  P.c_nm_dz = c->cstr_nomove_deadzone;
  P.c_nm_v = c->cstr_nomove_vel;
  P.c_or = c->cstr_orient_limit;
  P.c_h = c->cstr_height;
  P.c_hstd = c->cstr_height_std;
  P.c_clr = c->cstr_clearance_min;
  P.c_clr_dz = c->cstr_clearance_deadzone;
  return 0;
}

int n_blocks(const Handle* h) { return (h->W.n + ENVS_PER_BLOCK - 1) / ENVS_PER_BLOCK; }

// obs_assemble_kernel gather table for history length nh: for every float of an ASM_ROWS-row block (row r,
// column col), the offset from its own position in the block's LDS copy to its source -- the next-newer
// history slot (+3 / +12), or, for the newest slot, frame component c stored behind the rows
// (asm_col_entry's mapping); 4 int16 per output float4
std::vector<int16_t> asm_gather_table(int nh) {
  const int row = H12_OBS_FRAME * nh, nf = ASM_ROWS * row;
  std::vector<int16_t> t((size_t)nf, 0);
  for (int p = 0; p < nf; ++p) {
    const int r = p / row, col = p - r * row;
    int hh, c, d;
    if (col < 9 * nh) {
      const int k = col / (3 * nh), q = col - 3 * nh * k;
      hh = q / 3;
      c = 3 * k + (q - 3 * hh);
      d = 3;
    } else {
      const int k = (col - 9 * nh) / (12 * nh), q = col - 9 * nh - 12 * nh * k;
      hh = q / 12;
      c = 9 + 12 * k + (q - 12 * hh);
      d = 12;
    }
    t[(size_t)p] = (int16_t)(hh == nh - 1 ? nf + H12_OBS_FRAME * r + c - p : d);
  }
  return t;
}

// fused assembly: one code byte per float4 of a block's 32 rows of history nh (the same for every block) -- bit q:
// float q's next-newer slot is 12 floats on (the 12-wide terms; else 3) -- then, from byte FUSE_F4_MAX, one byte per
// row column: its frame component (a refilled row holds the frame in every slot)
std::vector<uint8_t> fuse_code_table(int nh) {
  const int row = H12_OBS_FRAME * nh, f4 = ENVS_PER_BLOCK * row / 4;
  std::vector<uint8_t> t((size_t)FUSE_CODE_BYTES, 0);
  for (int j = 0; j < f4; ++j) {
    uint8_t c = 0;
    for (int q = 0; q < 4; ++q) {
      const int col = (4 * j + q) % row;
      if (col >= 9 * nh) c |= (uint8_t)(1u << q);
    }
    t[(size_t)j] = c;
  }
  for (int col = 0; col < row; ++col) {
    const int k = col < 9 * nh ? col : col - 9 * nh, w = col < 9 * nh ? 3 : 12;
    t[(size_t)FUSE_F4_MAX + col] = (uint8_t)((col < 9 * nh ? 0 : 9) + w * (k / (w * nh)) + k % w);
  }
  return t;
}

// feature level of the env kernels (Feat<K>)
int feature_level(const KParams& P) {
  if (P.terrain) return 2;
  return (P.task != H12_TASK_FLAT || P.env_mu || P.env_mass || P.curriculum || P.rsl || P.dz || P.push || P.cat) ? 1
                                                                                                             : 0;
}
#define LAUNCH_K(KERNEL, ...)                                                   \
  do {                                                                          \
    switch (feature_level(h->P)) {                                              \
      case 0: hipLaunchKernelGGL(KERNEL<0>, __VA_ARGS__); break;                \
      case 1: hipLaunchKernelGGL(KERNEL<1>, __VA_ARGS__); break;                \
      default: hipLaunchKernelGGL(KERNEL<2>, __VA_ARGS__); break;               \
    }                                                                           \
  } while (0)
// launch with an optional event pair bound to the dispatch (kernel timing)
#define LAUNCH_KT(KERNEL, E0, E1, GRID, BLK, SHM, STREAM, ...)                                              \
  do {                                                                                                      \
    switch (feature_level(h->P)) {                                                                          \
      case 0: hipExtLaunchKernelGGL(KERNEL<0>, GRID, BLK, SHM, STREAM, E0, E1, 0, __VA_ARGS__); break;      \
      case 1: hipExtLaunchKernelGGL(KERNEL<1>, GRID, BLK, SHM, STREAM, E0, E1, 0, __VA_ARGS__); break;      \
      default: hipExtLaunchKernelGGL(KERNEL<2>, GRID, BLK, SHM, STREAM, E0, E1, 0, __VA_ARGS__); break;     \
    }                                                                                                       \
  } while (0)

// step_kernel's LDS against the device (see LDS_CU_BYTES): the compiled kernel's static size plus the fused path's
// dynamic FuseLds; H12_E_STATE when they exceed the device's LDS per CU
int check_step_lds(Handle* h) {
  hipFuncAttributes fa = {};
  hipError_t e;
  switch (feature_level(h->P)) {
    case 0: e = hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&step_kernel<0>)); break;
    case 1: e = hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&step_kernel<1>)); break;
    default: e = hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&step_kernel<2>)); break;
  }
  if (e != hipSuccess) return set_err(H12_E_HIP, "hipFuncGetAttributes(step_kernel): %s", hipGetErrorString(e));
  int lim = 0;
  if (hipDeviceGetAttribute(&lim, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, h->device) != hipSuccess ||
      lim <= 0)
    lim = (int)LDS_CU_BYTES;
  h->lds_static = fa.sharedSizeBytes;
  h->lds_limit = lim;
  const size_t dyn = h->fuse ? sizeof(FuseLds) : 0;
  if (fa.sharedSizeBytes + dyn > (size_t)lim)
    return set_err(H12_E_STATE, "step_kernel needs %zu B of LDS (%zu static + %zu dynamic), the device has %d per CU",
                   fa.sharedSizeBytes + dyn, fa.sharedSizeBytes, dyn, lim);
  return 0;
}

// CaT with the fused rows: step_kernel applies the probabilities itself (cat_prob_inline) when its whole grid is
// resident -- every block's helper wave waits for the last block's fold, so a block that could not start until another
// ended would wait for ever (bounded, and reported by h12env_check, but wrong) -- else cat_prob_kernel follows as before.
// H12_CAT_INLINE=0 at h12env_create asks for the two-kernel path.
void check_cat_inline(Handle* h) {
  h->cat_inline = false;
  if (!h->P.cat || !h->fuse) return;
  const char* ci = getenv("H12_CAT_INLINE");
  if (ci && ci[0] == '0') return;
  int per_cu = 0, cus = 0;
  const int threads = (h->P.self_coll ? 4 : 3) * BLOCK;
  hipError_t e;
  switch (feature_level(h->P)) {
    case 0: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, step_kernel<0>, threads, sizeof(FuseLds)); break;
    case 1: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, step_kernel<1>, threads, sizeof(FuseLds)); break;
    default: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, step_kernel<2>, threads, sizeof(FuseLds)); break;
  }
  if (e != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, h->device) != hipSuccess)
    return;
  // (and at most 256 blocks: the waiting wave reads four block prefixes per lane, cat_prob_inline)
  h->cat_inline = (long long)per_cu * cus >= (long long)n_blocks(h) && n_blocks(h) <= 256;
}

// obs_assemble_kernel after an env kernel on the same stream (history blocks + frame blocks)
int launch_assemble(const Handle* h, const float* obs_prev, float* obs, const uint8_t* fill_a, const uint8_t* fill_b,
                    const uint8_t* sel, int reset_mode, uint32_t lo, uint32_t hi, hipStream_t stream,
                    hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr, float* log_acc = nullptr,
                    float* frame_out = nullptr, float* log_part = nullptr) {
  AsmArgs A = {};
  A.frame_out = frame_out;
  A.log_part = log_part;
  A.log_acc = log_acc;
  A.log_nb = n_blocks(h);
  A.obs_prev = obs_prev;
  A.obs = obs;
  A.frame = h->frame;
  A.fill_a = fill_a;
  A.fill_b = fill_b;
  A.sel = sel;
  A.reset_mode = reset_mode;
  A.tab = h->asm_tab;
  A.n = h->W.n;
  A.env_offset = h->env_offset;
  A.lo = lo;
  A.hi = hi;
  if (h->P.task == H12_TASK_ROUGH) {
    if (frame_out) return set_err(H12_E_ARG, "frame_out needs the flat observation layout (history)");
    const int nb = (int)(((size_t)h->W.n * H12_NOBS_ROUGH + ASM_BLOCK - 1) / ASM_BLOCK);
    hipExtLaunchKernelGGL(rough_obs_kernel, dim3(nb), dim3(ASM_BLOCK), 0, stream, e0, e1, 0, h->P, A);
    HIP_TRY(hipGetLastError());
    return 0;
  }
  const float* src = reset_mode ? obs : obs_prev;
  A.vec = (((uintptr_t)obs | (uintptr_t)src) & 15u) == 0;
  const int nb = (h->W.n + ASM_ROWS - 1) / ASM_ROWS;
#define H12_ASM_CASE(NH) \
  case NH: hipExtLaunchKernelGGL(obs_assemble_kernel<NH>, dim3(nb), dim3(ASM_BLOCK), 0, stream, e0, e1, 0, h->P, A); break;
  switch (h->P.hist) {
    H12_ASM_CASE(1) H12_ASM_CASE(2) H12_ASM_CASE(3) H12_ASM_CASE(4) H12_ASM_CASE(5)
    H12_ASM_CASE(6) H12_ASM_CASE(7) H12_ASM_CASE(8) H12_ASM_CASE(9) H12_ASM_CASE(10)
    default: return set_err(H12_E_ARG, "history_length %d out of 1..%d", h->P.hist, H12_NHIST);
  }
#undef H12_ASM_CASE
  HIP_TRY(hipGetLastError());
  return 0;
}

}  // namespace

// ================================================================== C-ABI
extern "C" {

int h12env_abi_version(void) { return H12ENV_ABI_VERSION; }

size_t h12env_sizeof_struct(int which) {
  switch (which) {
    case 0: return sizeof(h12env_model);
    case 1: return sizeof(h12env_config);
    case 2: return sizeof(h12env_step_out);
    default: return 0;
  }
}

const char* h12env_last_error(void) { return g_err; }

int h12env_config_default(h12env_config* c) {
  if (!c) return set_err(H12_E_ARG, "null config");
  memset(c, 0, sizeof *c);
  c->abi_version = H12ENV_ABI_VERSION;
  c->mode = H12_MODE_ISAACLAB;
  c->physics_dt = 0.005f;
  c->decimation = 4;
  c->inner_steps = 1;
  c->implicit_penalty = 1;
  c->max_episode_length = 1000;
  c->action_scale = 0.5f;
  const float kp[6] = {200, 200, 200, 300, 40, 40}, kd[6] = {2.5f, 2.5f, 2.5f, 4, 2, 2};
  const float E[6] = {220, 220, 220, 360, 45, 45};
  const int grp[6] = {0, 0, 0, 1, 2, 2};
  for (int j = 0; j < H12_NJ; ++j) {
    c->kp[j] = kp[j % 6]; c->kd[j] = kd[j % 6]; c->effort_limit[j] = E[j % 6]; c->delay_group[j] = grp[j % 6];
  }
  c->min_delay = 0; c->max_delay = 5;
  const float vmax[6] = {23, 23, 23, 14, 9, 9};  // URDF velocity limits as the USD / PhysX hold them
  for (int j = 0; j < H12_NJ; ++j) c->max_joint_vel[j] = vmax[j % 6];
  c->max_joint_vel_damping = 1.0e3f;
  c->self_collision = 1; c->self_k = 3e4f; c->self_c = 50.f; c->self_ct = 50.f; c->self_mu = 0.36f;
  c->contact_k = 1e5f; c->contact_c = 100.f; c->friction_k = 3e4f; c->friction_c = 100.f;
  c->limit_projection = 0.01f;
  c->max_depenetration_velocity = 1.f;
  c->mu_static = 0.8f; c->mu_dynamic = 0.6f; c->limit_k = 1.0e6f; c->limit_c = 2.f; c->contact_threshold = 1.f;
  c->cmd_resample_time = 10.f;
  c->cmd_lin_x[0] = 0.f; c->cmd_lin_x[1] = 1.f; c->cmd_lin_y[0] = -0.5f; c->cmd_lin_y[1] = 0.5f;
  c->cmd_ang_z[0] = -1.f; c->cmd_ang_z[1] = 1.f;
  c->cmd_heading[0] = -3.14159265f; c->cmd_heading[1] = 3.14159265f;
  c->rel_standing_envs = 0.02f; c->rel_heading_envs = 1.f; c->heading_stiffness = 0.5f;
  c->reset_x[0] = -0.5f; c->reset_x[1] = 0.5f; c->reset_y[0] = -0.5f; c->reset_y[1] = 0.5f;
  c->reset_yaw[0] = -3.14f; c->reset_yaw[1] = 3.14f;
  c->enable_corruption = 1;
  c->noise_ang_vel = 0.2f; c->noise_gravity = 0.05f; c->noise_joint_pos = 0.01f; c->noise_joint_vel = 1.5f;
  const float w[H12_NREW_FLAT] = {1.0f, 1.0f, -0.05f, -2e-6f, -1e-7f, -0.005f, 0.75f, -1.0f, -1.0f, -200.f, -0.25f, -0.2f};
  for (int t = 0; t < H12_NREW; ++t) c->rew_w[t] = t < H12_NREW_FLAT ? w[t] : 0.f;
  c->track_std = 0.5f; c->air_time_threshold = 0.4f; c->soft_limit_factor = 0.9f;
  c->illegal_contact_knees = 1; c->illegal_contact_torso = 1;
  c->seed = 42;
  c->task = H12_TASK_FLAT;
  c->noise_lin_vel = 0.1f; c->noise_height_scan = 0.1f;
  c->scan_offset = 0.5f; c->scan_clip = 1.f; c->scan_resolution = 0.1f; c->terrain_size = 8.f;
  c->cmd_resample_time_max = c->cmd_resample_time;
  c->cmd_deadzone = 0; c->velocity_deadzone = 0.f; c->ang_flip_prob = 0.f;
  c->push_enable = 0;
  c->push_interval[0] = 5.f; c->push_interval[1] = 8.f;
  c->push_vel_x[0] = -1.f; c->push_vel_x[1] = 1.f; c->push_vel_y[0] = -1.f; c->push_vel_y[1] = 1.f;
  c->history_length = H12_NHIST;
  for (int t = 0; t < 6; ++t) c->obs_scale[t] = 1.f;
  c->base_height_target = 1.f;
  c->contact_force_threshold = 800.f;
  c->cat_enable = 0;
  c->cstr_mask = (1u << H12_NCSTR) - 1u;
  for (int t = 0; t < H12_NCSTR; ++t) c->cstr_max_p[t] = t == H12_C_CONTACT ? 1.f : 0.25f;
  c->cat_tau = 0.95f;
  c->cat_min_p = 0.f;
  const float vlim[NL] = {23.f, 23.f, 23.f, 14.f, 9.f, 9.f};  // h12_12dof.urdf joint velocity limits
  for (int j = 0; j < H12_NJ; ++j) {
    c->cstr_joint_vel_limit[j] = vlim[j % NL];
    c->cstr_joint_effort_limit[j] = 1e9f;
  }
  c->cstr_foot_force_limit = 750.f;
  c->cstr_nomove_deadzone = 0.2f;
  c->cstr_nomove_vel = 6.f;
  c->cstr_orient_limit = 0.1f;
  c->cstr_height = 1.f;
  c->cstr_height_std = 0.05f;
  c->cstr_clearance_min = 0.1f;
  c->cstr_clearance_deadzone = 0.2f;
  return 0;
}

int h12env_set_terrain(h12env* hh, const float* heights, int nx, int ny, float hscale, float x0, float y0,
                       const float* origins, int rows, int cols) {
  Handle* h = (Handle*)hh;
  if (!h) return set_err(H12_E_ARG, "null handle");
  if (!heights || nx < 2 || ny < 2 || !(hscale > 0)) return set_err(H12_E_ARG, "heights (nx, ny >= 2, hscale > 0) required");
  if ((origins == nullptr) != (rows <= 0 || cols <= 0) || rows > 0xFFFF || cols > 0x7FFF)
    return set_err(H12_E_ARG, "origins need rows, cols in 1..32767");
  if (h->P.curriculum && !origins) return set_err(H12_E_ARG, "the terrain curriculum needs the origins table");
  h->P.t_h = heights;
  h->P.t_nx = nx;
  h->P.t_ny = ny;
  h->P.t_inv_hs = 1.f / hscale;
  h->P.t_x0 = x0;
  h->P.t_y0 = y0;
  h->P.t_origin = origins;
  h->P.t_rows = rows;
  h->P.t_cols = cols;
  return 0;
}

size_t h12env_state_bytes(int n_envs) {
  if (n_envs <= 0) return 0;
  return (size_t)(H12_NF_FLOAT + H12_NF_INT) * sizeof(float) * (size_t)n_envs;
}

int h12env_create(const h12env_model* model, const h12env_config* cfg, int n_envs, int64_t env_offset, int device,
                  void* state_dev, h12env** out) {
  if (!model || !cfg || !out) return set_err(H12_E_ARG, "null argument");
  *out = nullptr;
  if (n_envs <= 0) return set_err(H12_E_ARG, "n_envs must be > 0 (got %d)", n_envs);
  if ((int64_t)n_envs * H12_NF_FLOAT * 4 >= (int64_t)0x7FFFFFFF)  // buffer offsets of the workspace (ldf / stf)
    return set_err(H12_E_ARG, "n_envs %d too large for one handle (max %d)", n_envs, 0x7FFFFFFF / (H12_NF_FLOAT * 4));
  if (env_offset < 0 || env_offset + (int64_t)n_envs > (int64_t)0xFFFFFFFFll)
    return set_err(H12_E_ARG, "global env ids must fit in 32 bits");
  if (cfg->abi_version != H12ENV_ABI_VERSION)
    return set_err(H12_E_ARG, "config abi %d != %d", cfg->abi_version, H12ENV_ABI_VERSION);
  Handle* h = new (std::nothrow) Handle();
  if (!h) return set_err(H12_E_ALLOC, "host allocation failed");
  if (int rc = build_params(model, cfg, h->P)) { delete h; return rc; }
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) { delete h; return set_err(H12_E_HIP, "hipSetDevice(%d): %s", device, hipGetErrorString(e)); }
  size_t bytes = h12env_state_bytes(n_envs);
  h->own = state_dev == nullptr;
  if (h->own) {
    e = hipMalloc(&state_dev, bytes);
    if (e != hipSuccess) { delete h; return set_err(H12_E_ALLOC, "hipMalloc(%zu): %s", bytes, hipGetErrorString(e)); }
    e = hipMemset(state_dev, 0, bytes);
    if (e != hipSuccess) { (void)hipFree(state_dev); delete h; return set_err(H12_E_HIP, "hipMemset: %s", hipGetErrorString(e)); }
  }
  h->W.F = (float*)state_dev;
  h->W.I = (int32_t*)((float*)state_dev + (size_t)H12_NF_FLOAT * n_envs);
  h->W.n = n_envs;
  e = hipMalloc(&h->frame, sizeof(float) * FRAME_ROWS * (size_t)n_envs);
  if (e != hipSuccess) {
    if (h->own) (void)hipFree(state_dev);
    delete h;
    return set_err(H12_E_ALLOC, "hipMalloc(frame): %s", hipGetErrorString(e));
  }
  e = hipMalloc(&h->dz_cnt, 4 * sizeof(int));
  if (e == hipSuccess) e = hipMemset(h->dz_cnt, 0, 4 * sizeof(int));
  const size_t log_bytes = sizeof(float) * LOG_RING * LOG_NPART * (size_t)((n_envs + ENVS_PER_BLOCK - 1) / ENVS_PER_BLOCK);
  if (e == hipSuccess) e = hipMalloc(&h->log_part, log_bytes);
  if (e == hipSuccess) e = hipMemset(h->log_part, 0, log_bytes);
  if (e != hipSuccess) {
    if (h->own) (void)hipFree(state_dev);
    (void)hipFree(h->frame);
    delete h;
    return set_err(H12_E_ALLOC, "hipMalloc(dz_cnt): %s", hipGetErrorString(e));
  }
  h->P.dz_cnt = h->dz_cnt;
  h->P.diag = h->dz_cnt + 3;
  {
    const char* nr = getenv("H12_TEST_SKIP_SELF_RELEASE");
    h->P.dbg_norel = nr && nr[0] == '1';
  }
  if (h->P.cat) {
    const size_t nn = (size_t)n_envs;
    const size_t nbk = (nn + ENVS_PER_BLOCK - 1) / ENVS_PER_BLOCK;
    auto al = [](size_t x) { return (x + 255) / 256 * 256; };  // every section 256-B aligned (cat_fold's 8-B loads)
    const size_t bytes_cat = al(sizeof(float) * CAT_ROWS * nn) + al(sizeof(float) * 2 * H12_NCSTR_COLS) +
                             al(sizeof(unsigned long long) * (CPUB_LIST + (nbk + 31) / 32 * 32) +
                                sizeof(float) * CAT_NMC * ENVS_PER_BLOCK * nbk) + al(sizeof(int) * nn) + al(sizeof(int) * CAT_META_INTS) +
                             al(sizeof(uint32_t) * nbk);
    e = hipMalloc(&h->cat_mem, bytes_cat);
    if (e == hipSuccess) e = hipMemset(h->cat_mem, 0, bytes_cat);
    if (e != hipSuccess) {
      if (h->own) (void)hipFree(state_dev);
      (void)hipFree(h->frame);
      (void)hipFree(h->dz_cnt);
      delete h;
      return set_err(H12_E_ALLOC, "hipMalloc(CaT buffers): %s", hipGetErrorString(e));
    }
    char* q = (char*)h->cat_mem;
    h->P.cscr = (float*)q; q += al(sizeof(float) * CAT_ROWS * nn);
    h->P.crun = (float*)q; q += al(sizeof(float) * 2 * H12_NCSTR_COLS);
    static_assert((sizeof(float) * 2 * H12_NCSTR_COLS + 255) / 256 * 256 == CPUB_OFF, "cat_cpub follows crun's section");
    q += al(sizeof(unsigned long long) * (CPUB_LIST + (nbk + 31) / 32 * 32) +
            sizeof(float) * CAT_NMC * ENVS_PER_BLOCK * nbk);
    h->P.clist = (int*)q; q += al(sizeof(int) * nn);
    h->P.cmeta = (int*)q;  // CAT_META_INTS ints of meta and column maxima, then the still masks (cat_ccount, cat_cstill)
  }
  h->device = device;
  if (h->P.task == H12_TASK_FLAT) {
    const std::vector<int16_t> t = asm_gather_table(h->P.hist);
    e = hipMalloc(&h->asm_tab, t.size() * sizeof(int16_t));
    if (e == hipSuccess) e = hipMemcpy(h->asm_tab, t.data(), t.size() * sizeof(int16_t), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      h12env_destroy((h12env*)h);
      return set_err(H12_E_ALLOC, "gather table: %s", hipGetErrorString(e));
    }
    // the step path assembles the rows inside step_kernel (FuseCtx) unless H12_FUSE_OBS=0 asks for the two-kernel
    // path (CaT's kernels after step_kernel read the done flags and rescale the reward, they leave the rows alone)
    const char* fz = getenv("H12_FUSE_OBS");
    h->fuse = !(fz && fz[0] == '0');
    if (h->fuse) {
      const std::vector<uint8_t> c = fuse_code_table(h->P.hist);
      e = hipMalloc(&h->fuse_code, c.size());
      if (e == hipSuccess) e = hipMemcpy(h->fuse_code, c.data(), c.size(), hipMemcpyHostToDevice);
      if (e != hipSuccess) {
        h12env_destroy((h12env*)h);
        return set_err(H12_E_ALLOC, "fused-assembly code table: %s", hipGetErrorString(e));
      }
    }
  }
  if (int rc = check_step_lds(h)) {
    h12env_destroy((h12env*)h);
    return rc;
  }
  check_cat_inline(h);
  h->env_offset = env_offset;
  h->reset_calls = 0;
  h->observe_calls = 0;
  // counted algorithmic FLOPs per env step (DESIGN.md "Roofline"): per inner step and leg lane
  // ~2.9k (pass 1 0.6k, contacts 0.35k, pass 2 1.5k, pass 3 0.25k, integration 0.1k), base combine +
  // 6x6 solve ~0.3k per lane, implicit penalty terms (contact inertias and their force report, limit
  // dampers) ~0.6k per lane; MDP (rewards, resets, commands, obs, RNG) ~3k per env
  h->flops_per_env = (double)cfg->decimation * cfg->inner_steps * 2.0 *
                         (2900.0 + 300.0 + (cfg->implicit_penalty ? 600.0 : 0.0)) + 3000.0;
  *out = (h12env*)h;
  return 0;
}

void h12env_destroy(h12env* hh) {
  Handle* h = (Handle*)hh;
  if (!h) return;
  if (h->own && h->W.F) (void)hipFree(h->W.F);
  if (h->frame) (void)hipFree(h->frame);
  if (h->dz_cnt) (void)hipFree(h->dz_cnt);
  if (h->log_part) (void)hipFree(h->log_part);
  if (h->cat_mem) (void)hipFree(h->cat_mem);
  if (h->asm_tab) (void)hipFree(h->asm_tab);
  if (h->fuse_code) (void)hipFree(h->fuse_code);
  for (hipEvent_t e : h->ev) (void)hipEventDestroy(e);
  delete h;
}

int h12env_reset(h12env* hh, const uint8_t* mask, float* obs, void* stream) {
  Handle* h = (Handle*)hh;
  if (!h) return set_err(H12_E_ARG, "null handle");
  if (!obs) return set_err(H12_E_ARG, "obs is required");
  if (h->P.terrain && !h->P.t_h) return set_err(H12_E_STATE, "terrain = 1 but h12env_set_terrain was not called");
  StepArgs A = {};
  A.obs = obs;
  A.reset_mask = mask;
  A.env_offset = h->env_offset;
  A.lo = (uint32_t)h->reset_calls;
  A.hi = 0xFFFFFFFFu;
  A.frame = h->frame;
  h->reset_calls++;
  LAUNCH_K(reset_kernel, dim3(n_blocks(h)), dim3(BLOCK), 0, (hipStream_t)stream, h->P, h->W, A);
  HIP_TRY(hipGetLastError());
  return launch_assemble(h, nullptr, obs, nullptr, nullptr, mask, 1, A.lo, A.hi, (hipStream_t)stream);
}

// the pending fused steps' log folds, in one launch (log_flush_kernel), on the stream the steps ran on
int flush_logs(Handle* h, hipStream_t stream, hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr) {
  if (!h->n_pend) return 0;
  FoldArgs F = {};
  F.part = h->log_part;
  F.nb = n_blocks(h);
  for (int k = 0; k < h->n_pend; ++k) {
    F.slot[k] = (h->log_pos - h->n_pend + k + LOG_RING) % LOG_RING;
    F.acc[k] = h->pend_acc[k];
  }
  hipExtLaunchKernelGGL(log_flush_kernel, dim3(LOG_NPART, h->n_pend), dim3(64), 0, stream, e0, e1, 0, F);
  h->n_pend = 0;
  HIP_TRY(hipGetLastError());
  return 0;
}

int h12env_step(h12env* hh, const float* actions, const float* obs_prev, const h12env_step_out* out,
                int64_t step_index, void* stream) {
  Handle* h = (Handle*)hh;
  if (!h) return set_err(H12_E_ARG, "null handle");
  if (!actions || !out || !out->obs || !out->rew || !out->terminated || !out->truncated)
    return set_err(H12_E_ARG, "actions, obs, rew, terminated, truncated are required");
  if (!obs_prev && h->P.task == H12_TASK_FLAT) return set_err(H12_E_ARG, "obs_prev is required (history source)");
  if (h->P.terrain && !h->P.t_h) return set_err(H12_E_STATE, "terrain = 1 but h12env_set_terrain was not called");
  if (step_index < 1) return set_err(H12_E_ARG, "step_index must be >= 1 (got %lld)", (long long)step_index);
  StepArgs A = {};
  A.actions = actions;
  A.obs_prev = obs_prev;
  A.obs = out->obs;
  A.rew = out->rew;
  A.term = out->terminated;
  A.trunc = out->truncated;
  // this step's partial set in the ring; a pending fold into the same accumulator, or a full ring, is folded first
  // (stream order keeps every accumulator's additions in step order)
  hipStream_t st = (hipStream_t)stream;
  hipEvent_t t0, t1;
  bool flushed = false;
  if (out->log_acc && h->n_pend) {
    bool dup = h->n_pend == LOG_RING;
    for (int k = 0; k < h->n_pend && !dup; ++k) dup = h->pend_acc[k] == out->log_acc;
    if (dup) {
      t0 = t1 = nullptr;
      if (!pair1_taken(h)) timing_events(h, 1, &t0, &t1);  // this step's second kernel
      if (int rc = flush_logs(h, st, t0, t1)) return rc;
      flushed = true;
    }
  }
  float* part = out->log_acc ? h->log_part + (size_t)h->log_pos * LOG_NPART * n_blocks(h) : nullptr;
  A.log_part = part;
  A.applied_torque = out->applied_torque;
  A.foot_force = out->foot_force;
  A.env_offset = h->env_offset;
  A.lo = (uint32_t)step_index;
  A.hi = (uint32_t)((uint64_t)step_index >> 32);
  A.frame = h->frame;
  A.dz_slot = (int)(h->dz_step++ % 3);
  // fused assembly: whole 16-byte aligned rows (the LDS-DMA); otherwise obs_assemble_kernel follows
  A.fuse = h->fuse && ((((uintptr_t)obs_prev | (uintptr_t)out->obs) & 15u) == 0);
  A.frame_out = out->frame_out;
  A.fuse_code = h->fuse_code;
  A.cat_inline = h->cat_inline && A.fuse;
  if (A.cat_inline) A.cstr_prob = out->cstr_prob;
  // timing: pair 0 = step_kernel, pair 1 = the second kernel (a flushed fold above, the assembly kernel below, or
  // an empty pair)
  hipEvent_t k0, k1;
  timing_events(h, 0, &k0, &k1);
  // every block carries a helper wave and, with self-collision, a self-contact wave (helper_wave, self_wave)
  LAUNCH_KT(step_kernel, k0, k1, dim3(n_blocks(h)), dim3((h->P.self_coll ? 4 : 3) * BLOCK),
            A.fuse ? sizeof(FuseLds) : 0, st, h->P, h->W, A);
  HIP_TRY(hipGetLastError());
  if (out->log_acc) h->log_pos = (h->log_pos + 1) % LOG_RING;
  if (h->P.cat && !A.cat_inline) {
    // (the running maxima and the still list were folded by step_kernel's last block, cat_fold)
    static_assert(CAT_PBLOCK >= ENVS_PER_BLOCK, "cat_prob_kernel's blocks fit the partial slots of step_kernel's");
    CatArgs C = {out->rew, out->terminated, out->truncated, out->cstr_prob, part, n_blocks(h)};
    hipLaunchKernelGGL(cat_prob_kernel, dim3((h->W.n + CAT_PBLOCK - 1) / CAT_PBLOCK), dim3(CAT_PBLOCK), 0, st, h->P,
                       h->W, C);
    HIP_TRY(hipGetLastError());
  }
  if (A.fuse) {
    // the rows are stored; the log partials are folded later (log_flush_kernel: a full ring, a reused accumulator,
    // h12env_flush_log)
    if (out->log_acc) h->pend_acc[h->n_pend++] = out->log_acc;
    timing_next(h);  // no second kernel unless a fold was flushed above
    return 0;
  }
  t0 = t1 = nullptr;
  if (!flushed && !pair1_taken(h)) timing_events(h, 1, &t0, &t1);
  timing_next(h);
  // fill = terminated | truncated: the envs reset inside the step restart their history
  return launch_assemble(h, obs_prev, out->obs, out->terminated, out->truncated, nullptr, 0, A.lo, A.hi, st, t0, t1,
                         out->log_acc, out->frame_out, part);
}

int h12env_observe(h12env* hh, const float* obs_prev, float* obs, const uint8_t* fill_mask, void* stream) {
  Handle* h = (Handle*)hh;
  if (!h) return set_err(H12_E_ARG, "null handle");
  if (!obs || (!obs_prev && h->P.task == H12_TASK_FLAT)) return set_err(H12_E_ARG, "obs_prev and obs are required");
  if (h->P.terrain && !h->P.t_h) return set_err(H12_E_STATE, "terrain = 1 but h12env_set_terrain was not called");
  StepArgs A = {};
  A.obs_prev = obs_prev;
  A.obs = obs;
  A.reset_mask = fill_mask;
  A.env_offset = h->env_offset;
  A.lo = (uint32_t)h->observe_calls;
  A.hi = 0xFFFFFFFEu;
  h->observe_calls++;
  A.frame = h->frame;
  LAUNCH_K(observe_kernel, dim3(n_blocks(h)), dim3(BLOCK), 0, (hipStream_t)stream, h->P, h->W, A);
  HIP_TRY(hipGetLastError());
  return launch_assemble(h, obs_prev, obs, fill_mask, nullptr, nullptr, 0, A.lo, A.hi, (hipStream_t)stream);
}

int h12env_step_physics(h12env* hh, const float* q_ref, int n_substeps, void* stream) {
  Handle* h = (Handle*)hh;
  if (!h) return set_err(H12_E_ARG, "null handle");
  if (!q_ref || n_substeps < 0) return set_err(H12_E_ARG, "q_ref required, n_substeps >= 0");
  StepArgs A = {};
  A.q_ref = q_ref;
  A.n_substeps = n_substeps;
  LAUNCH_K(physics_kernel, dim3(n_blocks(h)), dim3(BLOCK), 0, (hipStream_t)stream, h->P, h->W, A);
  HIP_TRY(hipGetLastError());
  return 0;
}

int h12env_eval_terms(h12env* hh, const float* tau, const float* jacc, const float* fmax, float* terms,
                      uint8_t* terminated, uint8_t* truncated, float* cstr, void* stream) {
  Handle* h = (Handle*)hh;
  if (!h) return set_err(H12_E_ARG, "null handle");
  if (!tau || !jacc || !fmax || !terms || !terminated || !truncated)
    return set_err(H12_E_ARG, "tau, jacc, fmax, terms, terminated, truncated are required");
  if (h->P.cat && !cstr) return set_err(H12_E_ARG, "cstr is required on a CaT env");
  KParams P = h->P;
  if (P.cat) P.cscr = cstr;  // the constraint rows go to the caller's buffer, not the step's scratch
  TermArgs T = {tau, jacc, fmax, terms, terminated, truncated};
  LAUNCH_K(terms_kernel, dim3(n_blocks(h)), dim3(BLOCK), 0, (hipStream_t)stream, P, h->W, T);
  HIP_TRY(hipGetLastError());
  return 0;
}

int h12env_eval_self_contacts(h12env* hh, float* out, void* stream) {
  Handle* h = (Handle*)hh;
  if (!h) return set_err(H12_E_ARG, "null handle");
  if (!out) return set_err(H12_E_ARG, "out is required");
  if (!h->P.self_coll) return set_err(H12_E_STATE, "self_collision is off in this env's config");
  LAUNCH_K(selfc_kernel, dim3(n_blocks(h)), dim3(BLOCK), 0, (hipStream_t)stream, h->P, h->W, out);
  HIP_TRY(hipGetLastError());
  return 0;
}

int h12env_rollout_layout(int n, size_t offsets[5], size_t* step_bytes) {
  if (n < 1 || !offsets || !step_bytes) return set_err(H12_E_ARG, "n >= 1 and output pointers required");
  rollout_offsets(n, offsets, step_bytes);
  return 0;
}

int h12env_rollout_decode(const void* records, int n_shards, int n, int T, int G, int history, int t0, int t1,
                          const float* tail, float* obs_out, void* stream) {
  if (!records || !tail || !obs_out) return set_err(H12_E_ARG, "records, tail and obs_out are required");
  if (n_shards < 1 || n < 1 || T < 1 || G < 1) return set_err(H12_E_ARG, "n_shards, n, T, G must be >= 1");
  if (history < 1 || history > H12_NHIST) return set_err(H12_E_ARG, "history %d out of 1..%d", history, H12_NHIST);
  if (t0 < 0 || t1 > T || t0 > t1) return set_err(H12_E_ARG, "rows [%d, %d) outside [0, %d]", t0, t1, T);
  if (t0 == t1) return 0;
  DecArgs D = {};
  D.rec = (const uint8_t*)records;
  rollout_offsets(n, D.off, &D.step_bytes);
  D.n_shards = n_shards;
  D.n = n;
  D.T = T;
  D.G = min(G, T);
  D.t0 = t0;
  D.t1 = t1;
  D.tail = tail;
  D.out = obs_out;
  const int nb = min(n_shards * ((n + DEC_ENVS - 1) / DEC_ENVS), DEC_MAX_BLOCKS);
  hipStream_t st = (hipStream_t)stream;
#define H12_DEC_CASE(NH) case NH: hipLaunchKernelGGL(rollout_decode_kernel<NH>, dim3(nb), dim3(DEC_BLOCK), 0, st, D); break;
  switch (history) {
    H12_DEC_CASE(1) H12_DEC_CASE(2) H12_DEC_CASE(3) H12_DEC_CASE(4) H12_DEC_CASE(5)
    H12_DEC_CASE(6) H12_DEC_CASE(7) H12_DEC_CASE(8) H12_DEC_CASE(9) H12_DEC_CASE(10)
  }
#undef H12_DEC_CASE
  HIP_TRY(hipGetLastError());
  return 0;
}

struct h12env_fence {
  std::vector<uint64_t*> ctr;  // one HSA signal (8 bytes, hipMallocSignalMemory) per slot
  int device;
};

void h12env_fence_destroy(h12env_fence* f) {
  if (!f) return;
  for (uint64_t* c : f->ctr)
    if (c) (void)hipFree(c);
  delete f;
}

int h12env_fence_create(int device, int n_slots, h12env_fence** out) {
  if (!out || n_slots < 1) return set_err(H12_E_ARG, "n_slots >= 1 and out required");
  *out = nullptr;
  HIP_TRY(hipSetDevice(device));
  int ok = 0;
  HIP_TRY(hipDeviceGetAttribute(&ok, hipDeviceAttributeCanUseStreamWaitValue, device));
  if (!ok) return set_err(H12_E_STATE, "device %d does not support hipStreamWaitValue64", device);
  h12env_fence* f = new (std::nothrow) h12env_fence();
  if (!f) return set_err(H12_E_ALLOC, "host allocation failed");
  f->device = device;
  for (int i = 0; i < n_slots; ++i) {
    uint64_t* c = nullptr;
    hipError_t e = hipExtMallocWithFlags((void**)&c, sizeof(uint64_t), hipMallocSignalMemory);
    if (e == hipSuccess) {
      f->ctr.push_back(c);
      e = hipStreamWriteValue64(nullptr, c, 0, 0);  // counters start at 0
    }
    if (e != hipSuccess) {
      (void)hipGetLastError();  // leave no sticky error behind for the caller's next HIP call
      h12env_fence_destroy(f);
      return set_err(H12_E_ALLOC, "signal memory: %s", hipGetErrorString(e));
    }
  }
  hipError_t e = hipStreamSynchronize(nullptr);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    h12env_fence_destroy(f);
    return set_err(H12_E_HIP, "fence init: %s", hipGetErrorString(e));
  }
  *out = f;
  return 0;
}

int h12env_fence_signal(h12env_fence* f, int slot, uint64_t value, void* stream) {
  if (!f || slot < 0 || slot >= (int)f->ctr.size()) return set_err(H12_E_ARG, "bad fence or slot");
  HIP_TRY(hipStreamWriteValue64((hipStream_t)stream, f->ctr[slot], value, 0));
  return 0;
}

int h12env_fence_wait(h12env_fence* f, int slot, uint64_t value, void* stream) {
  if (!f || slot < 0 || slot >= (int)f->ctr.size()) return set_err(H12_E_ARG, "bad fence or slot");
  HIP_TRY(hipStreamWaitValue64((hipStream_t)stream, f->ctr[slot], value, hipStreamWaitValueGte, ~0ull));
  return 0;
}

void* h12env_field_ptr(h12env* hh, int is_int, int field) {
  Handle* h = (Handle*)hh;
  if (!h) { set_err(H12_E_ARG, "null handle"); return nullptr; }
  if (is_int) {
    if (field < 0 || field >= H12_NF_INT) { set_err(H12_E_ARG, "int field %d out of range", field); return nullptr; }
    return h->W.I + (size_t)field * h->W.n;
  }
  if (field < 0 || field >= H12_NF_FLOAT) { set_err(H12_E_ARG, "float field %d out of range", field); return nullptr; }
  return h->W.F + (size_t)field * h->W.n;
}

#ifdef H12_PHASE_PROFILE
int h12env_phase_profile(unsigned long long* out16, int clear) {
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_phase), sizeof(unsigned long long) * 16));
  if (clear) {
    unsigned long long z[16] = {};
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_phase), z, sizeof z));
  }
  return 0;
}
#ifdef H12_PHASE_LIGHT
int h12env_barrier_waits(unsigned long long* out, int nblocks) {
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bw), sizeof(unsigned long long) * 64 * (size_t)nblocks));
  return 0;
}
int h12env_kernel_starts(unsigned long long* out, int nblocks) {
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_kstart), sizeof(unsigned long long) * 4 * (size_t)nblocks));
  return 0;
}
#endif
int h12env_wave_times(unsigned long long* out, int nwaves) {
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wave), sizeof(unsigned long long) * 11 * (size_t)nwaves));
  return 0;
}
#endif

int h12env_num_envs(const h12env* hh) { return hh ? ((const Handle*)hh)->W.n : -1; }

int h12env_obs_dim(const h12env* hh) {
  if (!hh) return set_err(H12_E_ARG, "null handle");
  const KParams& P = ((const Handle*)hh)->P;
  return P.task == H12_TASK_ROUGH ? H12_NOBS_ROUGH : H12_OBS_FRAME * P.hist;
}

int h12env_set_constraint_max_p(h12env* hh, const float* max_p, int n) {
  Handle* h = (Handle*)hh;
  if (!h || !max_p) return set_err(H12_E_ARG, "null argument");
  if (n < 0 || n > H12_NCSTR) return set_err(H12_E_ARG, "n must be in 0..%d (got %d)", H12_NCSTR, n);
  for (int t = 0; t < n; ++t) h->P.cmaxp[t] = max_p[t];
  return 0;
}

int h12env_set_reward_weights(h12env* hh, const float* w, int n) {
  Handle* h = (Handle*)hh;
  if (!h || !w) return set_err(H12_E_ARG, "null argument");
  if (n < 0 || n > H12_NREW) return set_err(H12_E_ARG, "n must be in 0..%d (got %d)", H12_NREW, n);
  int rsl = 0;
  for (int t = 0; t < H12_NREW; ++t) rsl |= (t < n ? w[t] : h->P.rew_w[t]) != 0.f && t >= H12_NREW_FLAT;
  // terms 12-19 are computed by the extended kernel only, and their episode sums live in fields that
  // kernel keeps: switching them on mid-run is a different kernel configuration (recreate the handle)
  if (rsl && !h->P.rsl) return set_err(H12_E_STATE, "reward terms 12-19 were off at creation; recreate the env");
  for (int t = 0; t < n; ++t) h->P.rew_w[t] = w[t];
  return 0;
}

int h12env_kernel_cost(const h12env* hh, int kernel, double* bytes_per_env, double* flops_per_env) {
  const Handle* h = (const Handle*)hh;
  if (!h) return set_err(H12_E_ARG, "null handle");
  const KParams& P = h->P;
  const bool rough = P.task == H12_TASK_ROUGH;
  double bytes, flops;
  if (kernel == 0) {
    // state fields the kernel reads and writes (106 on the plane: ABI 7 added the two command metrics), actions,
    // reward / terminated / truncated, applied torque and foot force (the ArticulationData / ContactSensor views),
    // the noise-free frame
    double fields = 106.0 + (P.terrain ? 4.0 : 0.0) + (P.env_mu ? 4.0 : 0.0) + (P.env_mass ? 1.0 : 0.0) +
                    (P.rsl ? 8.0 : 0.0) + (P.push ? 1.0 : 0.0) + (P.cat ? 22.0 : 0.0);
    // CaT: the constraint scratch written and read back, the no_move list entry, reward and dones rewritten
    const double cat_bytes = P.cat ? (double)CAT_ROWS * 4.0 * 2.0 + 4.0 + 4.0 * 2.0 + 4.0 : 0.0;
    bytes = fields * 4.0 * 2.0 + (double)H12_NJ * 4.0 + 4.0 + 2.0 + (double)H12_NJ * 4.0 + 2.0 * 4.0 + cat_bytes;
    if (h->fuse) {  // the observation row: H-1 old frames read, H frames written (H = 10 Flat, 6 Rsl)
      const double row = (double)H12_OBS_FRAME * P.hist;
      bytes += (row - H12_OBS_FRAME) * 4.0 + row * 4.0;
    } else {
      bytes += (rough ? (double)FRAME_ROWS : (double)H12_OBS_FRAME) * 4.0;  // the frame scratch
    }
    flops = h->flops_per_env + (h->fuse ? 30.0 * 3.0 + 45.0 + 8.0 * 10.0 * 6.0 : 0.0);
  } else if (kernel == 1) {
    if (h->fuse) {
      // log_flush_kernel, per step and env: the block's partial slots read and zeroed
      bytes = (double)LOG_NPART * 4.0 * 2.0 / ENVS_PER_BLOCK;
      flops = (double)LOG_NPART / ENVS_PER_BLOCK;
    } else if (rough) {
      // frame read, one height sample per ray, the 235-float row written
      bytes = (double)FRAME_ROWS * 4.0 + (double)H12_NSCAN * 4.0 + (double)H12_NOBS_ROUGH * 4.0;
      flops = 55.0 * 10.0 * 6.0 + (double)H12_NSCAN * 20.0;
    } else {
      // H-1 old frames + the new frame + the two reset flags read, H frames written (H = 10 Flat, 6 Rsl)
      const double row = (double)H12_OBS_FRAME * P.hist;
      bytes = (row - H12_OBS_FRAME) * 4.0 + (double)H12_OBS_FRAME * 4.0 + 2.0 + row * 4.0;
      flops = 30.0 * 3.0 + 45.0 + 8.0 * 10.0 * 6.0;  // noise affine + scale + Philox rounds
    }
  } else {
    return set_err(H12_E_ARG, "kernel must be 0 or 1 (got %d)", kernel);
  }
  if (bytes_per_env) *bytes_per_env = bytes;
  if (flops_per_env) *flops_per_env = flops;
  return 0;
}

int h12env_step_cost(const h12env* hh, double* bytes_per_env, double* flops_per_env) {
  double b0, f0, b1, f1;
  if (int rc = h12env_kernel_cost(hh, 0, &b0, &f0)) return rc;
  if (int rc = h12env_kernel_cost(hh, 1, &b1, &f1)) return rc;
  // the frame round trip between the kernels is not compulsory traffic of the step (none on the fused path)
  const Handle* h = (const Handle*)hh;
  const double fr = h->fuse ? 0.0 : (h->P.task == H12_TASK_ROUGH ? (double)FRAME_ROWS : (double)H12_OBS_FRAME) * 4.0;
  if (bytes_per_env) *bytes_per_env = b0 + b1 - 2.0 * fr;
  if (flops_per_env) *flops_per_env = f0 + f1;
  return 0;
}

int h12env_step_lds(const h12env* hh, size_t* static_bytes, size_t* dynamic_bytes, size_t* limit_bytes) {
  const Handle* h = (const Handle*)hh;
  if (static_bytes) *static_bytes = h ? h->lds_static : STEP_LDS_STATIC;
  if (dynamic_bytes) *dynamic_bytes = (!h || h->fuse) ? sizeof(FuseLds) : 0;
  if (limit_bytes) *limit_bytes = h ? (size_t)h->lds_limit : LDS_CU_BYTES;
  return 0;
}

int h12env_check(h12env* hh, void* stream) {
  Handle* h = (Handle*)hh;
  if (!h) return set_err(H12_E_ARG, "null handle");
  HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
  int d = 0;
  HIP_TRY(hipMemcpy(&d, h->P.diag, sizeof(int), hipMemcpyDeviceToHost));
  if (!d) return 0;
  HIP_TRY(hipMemset(h->P.diag, 0, sizeof(int)));
  if (d & 1)
    return set_err(H12_E_STATE,
                   "self-contact: a wait for the contact wave's release ended at its bound (diagnostic 0x%x) since the "
                   "last check; the self-contact wrenches of that inner step may be partial", (unsigned)d);
  return set_err(H12_E_STATE,
                 "CaT: a block's wait for the last block's fold ended at its bound (diagnostic 0x%x) since the last "
                 "check; that step's constraint probabilities may be stale", (unsigned)d);
}

int h12env_cat_inline(const h12env* hh) {
  const Handle* h = (const Handle*)hh;
  return h && h->cat_inline ? 1 : 0;
}

int h12env_obs_fused(const h12env* hh) {
  const Handle* h = (const Handle*)hh;
  return h && h->fuse ? 1 : 0;
}

int h12env_flush_log(h12env* hh, void* stream) {
  Handle* h = (Handle*)hh;
  if (!h) return set_err(H12_E_ARG, "null handle");
  // kernel timing: the fold is counted as the second kernel of the next step
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (h->n_pend && !pair1_taken(h)) timing_events(h, 1, &e0, &e1);
  return flush_logs(h, (hipStream_t)stream, e0, e1);
}

int h12env_set_kernel_timing(h12env* hh, int enable) {
  Handle* h = (Handle*)hh;
  if (!h) return set_err(H12_E_ARG, "null handle");
  h->timing = enable != 0;
  h->n_timed = 0;
  std::fill(h->ev_k1.begin(), h->ev_k1.end(), 0);
  return 0;
}

int h12env_kernel_times(h12env* hh, double* env_ms, double* obs_ms, int* n_steps) {
  Handle* h = (Handle*)hh;
  if (!h) return set_err(H12_E_ARG, "null handle");
  double a = 0.0, b = 0.0;
  if (h->n_timed > 0) {  // the last step's kernels (its pair 1 exists only if that step had a second kernel)
    const size_t l = h->n_timed - 1;
    HIP_TRY(hipEventSynchronize(h->ev[4 * l + 1]));
    if (l < h->ev_k1.size() && h->ev_k1[l]) HIP_TRY(hipEventSynchronize(h->ev[4 * l + 3]));
  }
  for (size_t i = 0; i < h->n_timed; ++i) {
    float t0 = 0.f, t1 = 0.f;
    HIP_TRY(hipEventElapsedTime(&t0, h->ev[4 * i], h->ev[4 * i + 1]));
    if (i < h->ev_k1.size() && h->ev_k1[i]) HIP_TRY(hipEventElapsedTime(&t1, h->ev[4 * i + 2], h->ev[4 * i + 3]));
    a += t0;
    b += t1;
  }
  if (env_ms) *env_ms = a;
  if (obs_ms) *obs_ms = b;
  if (n_steps) *n_steps = (int)h->n_timed;
  h->n_timed = 0;
  std::fill(h->ev_k1.begin(), h->ev_k1.end(), 0);
  return 0;
}

}  // extern "C"
