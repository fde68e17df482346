/*
 * h12_oracle.c — CPU restatement of the H1-2 Flat velocity env (TEST INFRASTRUCTURE ONLY).
 * See h12_oracle.h for scope and parity status.  Double precision, generic 6x6 spatial
 * algebra (Featherstone, "Rigid Body Dynamics Algorithms", 2008): written for clarity, not speed,
 * and independent of the fp32 structured kernel in h1v2-isaac_amd/csrc/h12env.hip.
 */
#include "h12_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define NJ H12_NJ
#define NB (NJ + 1)
#define PI_D 3.14159265358979323846

/* ------------------------------------------------------------------ RNG (Philox4x32-10) */
void orc_philox(uint64_t seed, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t out[4]) {
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  uint32_t x0 = c0, x1 = c1, x2 = c2, x3 = c3;
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)0xD2511F53u * x0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * x2;
    uint32_t y0 = (uint32_t)(p1 >> 32) ^ x1 ^ k0;
    uint32_t y2 = (uint32_t)(p0 >> 32) ^ x3 ^ k1;
    x1 = (uint32_t)p1;
    x3 = (uint32_t)p0;
    x0 = y0;
    x2 = y2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  out[0] = x0; out[1] = x1; out[2] = x2; out[3] = x3;
}
/* streams (counter word c2 = stream << 16 | block) */
enum { ST_RESET = 1, ST_CMD = 2, ST_OBS = 3, ST_PUSH = 4 };
static double u01(uint32_t x) { return (double)(x >> 8) * (1.0 / 16777216.0); }
static double uab(uint32_t x, double a, double b) { return a + (b - a) * (double)(float)u01(x); }

static void rng_block(uint64_t seed, int64_t env, uint32_t ctr_lo, uint32_t ctr_hi, int stream, int block,
                      uint32_t out[4]) {
  orc_philox(seed, (uint32_t)env, ctr_lo, ((uint32_t)stream << 16) | (uint32_t)block, ctr_hi, out);
}

/* ------------------------------------------------------------------ terrain */
static struct {
  const float* h;
  int nx, ny, rows, cols;
  double hs, x0, y0;
  const float* origins;
} g_terrain;

void orc_set_terrain(const float* heights, int nx, int ny, double hscale, double x0, double y0,
                     const float* origins, int rows, int cols) {
  g_terrain.h = heights; g_terrain.nx = nx; g_terrain.ny = ny; g_terrain.hs = hscale;
  g_terrain.x0 = x0; g_terrain.y0 = y0; g_terrain.origins = origins; g_terrain.rows = rows; g_terrain.cols = cols;
}

/* triangle mesh of isaaclab.terrains.utils.convert_height_field_to_mesh: cell (ix, iy) split along
 * its (ix, iy)-(ix+1, iy+1) diagonal; barycentric height on the containing triangle */
double orc_ground(const h12env_config* c, double x, double y, double* gx, double* gy) {
  if (!c->terrain || !g_terrain.h) { *gx = *gy = 0; return 0; }
  double u = (x - g_terrain.x0) / g_terrain.hs, v = (y - g_terrain.y0) / g_terrain.hs;
  double umax = g_terrain.nx - 1 - 1e-3, vmax = g_terrain.ny - 1 - 1e-3;
  u = u < 0 ? 0 : (u > umax ? umax : u);
  v = v < 0 ? 0 : (v > vmax ? vmax : v);
  int ix = (int)u, iy = (int)v;
  double fu = u - ix, fv = v - iy;
  const float* hp = g_terrain.h + (size_t)ix * g_terrain.ny + iy;
  double h00 = hp[0], h01 = hp[1], h10 = hp[g_terrain.ny], h11 = hp[g_terrain.ny + 1], a, b;
  if (fv >= fu) { a = h11 - h01; b = h01 - h00; }
  else { a = h10 - h00; b = h11 - h10; }
  *gx = a / g_terrain.hs;
  *gy = b / g_terrain.hs;
  return h00 + fu * a + fv * b;
}

int orc_obs_dim(const h12env_config* c) {
  return c->task == H12_TASK_ROUGH ? H12_NOBS_ROUGH : H12_OBS_FRAME * c->history_length;
}

/* deadzone command count carried between steps (UniformVelocityCommandWithDeadzone; see cmd_update) */
static int g_dz_count = 0;
void orc_set_dz_count(int v) { g_dz_count = v; }
int orc_dz_count(void) { return g_dz_count; }

/* ------------------------------------------------------------------ small linear algebra */
typedef double m3[3][3];
static double dot3(const double a[3], const double b[3]) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static double clampd(double x, double lo, double hi) { return x < lo ? lo : (x > hi ? hi : x); }
static void cross3(const double a[3], const double b[3], double o[3]) {
  double t0 = a[1] * b[2] - a[2] * b[1], t1 = a[2] * b[0] - a[0] * b[2], t2 = a[0] * b[1] - a[1] * b[0];
  o[0] = t0; o[1] = t1; o[2] = t2;
}
static void m3v(const m3 A, const double v[3], double o[3]) {
  double t[3];
  for (int i = 0; i < 3; ++i) t[i] = A[i][0] * v[0] + A[i][1] * v[1] + A[i][2] * v[2];
  memcpy(o, t, sizeof t);
}
static void m3tv(const m3 A, const double v[3], double o[3]) {
  double t[3];
  for (int i = 0; i < 3; ++i) t[i] = A[0][i] * v[0] + A[1][i] * v[1] + A[2][i] * v[2];
  memcpy(o, t, sizeof t);
}
static void m3mul(const m3 A, const m3 B, m3 C) {
  m3 T;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) T[i][j] = A[i][0] * B[0][j] + A[i][1] * B[1][j] + A[i][2] * B[2][j];
  memcpy(C, T, sizeof T);
}
static void rot_axis(int axis, double q, m3 R) { /* child frame rotated by q about parent axis */
  double c = cos(q), s = sin(q);
  memset(R, 0, sizeof(m3));
  if (axis == 0) { R[0][0] = 1; R[1][1] = c; R[1][2] = -s; R[2][1] = s; R[2][2] = c; }
  else if (axis == 1) { R[1][1] = 1; R[0][0] = c; R[0][2] = s; R[2][0] = -s; R[2][2] = c; }
  else { R[2][2] = 1; R[0][0] = c; R[0][1] = -s; R[1][0] = s; R[1][1] = c; }
}
static void quat_to_R(const double q[4], m3 R) {
  double w = q[0], x = q[1], y = q[2], z = q[3];
  double n = sqrt(w * w + x * x + y * y + z * z);
  w /= n; x /= n; y /= n; z /= n;
  R[0][0] = 1 - 2 * (y * y + z * z); R[0][1] = 2 * (x * y - w * z); R[0][2] = 2 * (x * z + w * y);
  R[1][0] = 2 * (x * y + w * z); R[1][1] = 1 - 2 * (x * x + z * z); R[1][2] = 2 * (y * z - w * x);
  R[2][0] = 2 * (x * z - w * y); R[2][1] = 2 * (y * z + w * x); R[2][2] = 1 - 2 * (x * x + y * y);
}

/* 6x6 spatial matrices (row major, blocks [ang; lin]) */
typedef double m6[6][6];
static void m6v(const m6 A, const double v[6], double o[6]) {
  double t[6];
  for (int i = 0; i < 6; ++i) { t[i] = 0; for (int j = 0; j < 6; ++j) t[i] += A[i][j] * v[j]; }
  memcpy(o, t, sizeof t);
}
static void m6tv(const m6 A, const double v[6], double o[6]) {
  double t[6];
  for (int i = 0; i < 6; ++i) { t[i] = 0; for (int j = 0; j < 6; ++j) t[i] += A[j][i] * v[j]; }
  memcpy(o, t, sizeof t);
}
/* C = X^T I X */
static void congruence(const m6 X, const m6 I, m6 C) {
  m6 T;
  for (int i = 0; i < 6; ++i)
    for (int j = 0; j < 6; ++j) { double s = 0; for (int k = 0; k < 6; ++k) s += I[i][k] * X[k][j]; T[i][j] = s; }
  for (int i = 0; i < 6; ++i)
    for (int j = 0; j < 6; ++j) { double s = 0; for (int k = 0; k < 6; ++k) s += X[k][i] * T[k][j]; C[i][j] = s; }
}
/* motion transform parent->child from (E, r): [E 0; -E rx E] */
static void xform(const m3 E, const double r[3], m6 X) {
  memset(X, 0, sizeof(m6));
  m3 rx = {{0, -r[2], r[1]}, {r[2], 0, -r[0]}, {-r[1], r[0], 0}};
  m3 Erx;
  m3mul(E, rx, Erx);
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) { X[i][j] = E[i][j]; X[3 + i][3 + j] = E[i][j]; X[3 + i][j] = -Erx[i][j]; }
}
static void crm(const double v[6], const double m[6], double o[6]) { /* v x m */
  double a[3], b[3];
  cross3(v, m, a);
  cross3(v, m + 3, o + 3);
  cross3(v + 3, m, b);
  o[0] = a[0]; o[1] = a[1]; o[2] = a[2];
  o[3] += b[0]; o[4] += b[1]; o[5] += b[2];
}
static void crf(const double v[6], const double f[6], double o[6]) { /* v x* f */
  double a[3], b[3];
  cross3(v, f, a);
  cross3(v + 3, f + 3, b);
  cross3(v, f + 3, o + 3);
  o[0] = a[0] + b[0]; o[1] = a[1] + b[1]; o[2] = a[2] + b[2];
}
/* rigid-body spatial inertia at body origin from mass, COM, COM inertia (xx yy zz xy xz yz) */
static void rb_inertia(double mass, const float com[3], const float Ic[6], m6 I) {
  double c[3] = {com[0], com[1], com[2]};
  double cc = c[0] * c[0] + c[1] * c[1] + c[2] * c[2];
  double Icm[3][3] = {{Ic[0], Ic[3], Ic[4]}, {Ic[3], Ic[1], Ic[5]}, {Ic[4], Ic[5], Ic[2]}};
  m3 cx = {{0, -c[2], c[1]}, {c[2], 0, -c[0]}, {-c[1], c[0], 0}};
  memset(I, 0, sizeof(m6));
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      I[i][j] = Icm[i][j] + mass * ((i == j ? cc : 0.0) - c[i] * c[j]);
      I[i][3 + j] = mass * cx[i][j];
      I[3 + i][j] = -mass * cx[i][j]; /* (m cx)^T = -m cx */
      I[3 + i][3 + j] = (i == j) ? mass : 0.0;
    }
}
/* in-place Cholesky solve of SPD A (n x n) x = b */
static int chol_solve(double* A, int n, double* b) {
  for (int j = 0; j < n; ++j) {
    double s = A[j * n + j];
    for (int k = 0; k < j; ++k) s -= A[j * n + k] * A[j * n + k];
    if (!(s > 0)) return -1;
    double d = sqrt(s);
    A[j * n + j] = d;
    for (int i = j + 1; i < n; ++i) {
      double t = A[i * n + j];
      for (int k = 0; k < j; ++k) t -= A[i * n + k] * A[j * n + k];
      A[i * n + j] = t / d;
    }
  }
  for (int i = 0; i < n; ++i) { double t = b[i]; for (int k = 0; k < i; ++k) t -= A[i * n + k] * b[k]; b[i] = t / A[i * n + i]; }
  for (int i = n - 1; i >= 0; --i) { double t = b[i]; for (int k = i + 1; k < n; ++k) t -= A[k * n + i] * b[k]; b[i] = t / A[i * n + i]; }
  return 0;
}

/* ------------------------------------------------------------------ kinematics */
typedef struct kin_t {
  m6 X[NB];        /* parent -> body motion transforms (X[0] unused) */
  m6 I[NB];        /* rigid spatial inertias at body origins */
  double v[NB][6]; /* body spatial velocities (body coords) */
  m3 R[NB];        /* world rotation of body frames */
  double p[NB][3]; /* world position of body origins */
  double ag[6];    /* gravity spatial acceleration in base coords */
} kin_t;

static void kinematics(const h12env_model* m, const orc_phys* s, kin_t* k) {
  quat_to_R(s->quat, k->R[0]);
  memcpy(k->p[0], s->pos, sizeof(double) * 3);
  rb_inertia(m->base_mass, m->base_com, m->base_inertia, k->I[0]);
  if (s->env_params && s->dmass != 0.0) { /* point mass at the torso COM (randomize_rigid_body_mass) */
    m6 Ip;
    const float zero6[6] = {0, 0, 0, 0, 0, 0};
    rb_inertia(s->dmass, m->torso_com, zero6, Ip);
    for (int a = 0; a < 6; ++a)
      for (int b2 = 0; b2 < 6; ++b2) k->I[0][a][b2] += Ip[a][b2];
  }
  double vb[3];
  m3tv(k->R[0], s->vlin, vb);
  k->v[0][0] = s->wang[0]; k->v[0][1] = s->wang[1]; k->v[0][2] = s->wang[2];
  k->v[0][3] = vb[0]; k->v[0][4] = vb[1]; k->v[0][5] = vb[2];
  double gw[3] = {0, 0, -m->gravity}, gb[3];
  m3tv(k->R[0], gw, gb);
  k->ag[0] = k->ag[1] = k->ag[2] = 0;
  k->ag[3] = gb[0]; k->ag[4] = gb[1]; k->ag[5] = gb[2];
  for (int j = 0; j < NJ; ++j) {
    int b = j + 1, par = m->parent[j] + 1;
    m3 Rj, E;
    rot_axis(m->axis[j], s->q[j], Rj);
    for (int a = 0; a < 3; ++a)
      for (int c = 0; c < 3; ++c) E[a][c] = Rj[c][a];
    double r[3] = {m->joint_pos[j][0], m->joint_pos[j][1], m->joint_pos[j][2]};
    xform(E, r, k->X[b]);
    rb_inertia(m->link_mass[j], m->link_com[j], m->link_inertia[j], k->I[b]);
    m6v(k->X[b], k->v[par], k->v[b]);
    k->v[b][m->axis[j]] += s->qd[j];
    m3mul(k->R[par], Rj, k->R[b]);
    double t[3];
    m3v(k->R[par], r, t);
    for (int a = 0; a < 3; ++a) k->p[b][a] = k->p[par][a] + t[a];
  }
}

/* ------------------------------------------------------------------ test hooks: fp32-rounding jitters
 * (tests/helpers/forced.py only; single-env re-runs, the draw sequences are global and not thread-safe; eps = 0, the
 * default, is the exact model).
 * Self contacts: every capsule end point of the self-contacts gets an independent uniform +-eps (m) per
 * coordinate -- the GPU rounds each rod end it computes independently (fp32, ~1e-7 m at ~1 m), a perturbation that
 * no perturbation of the joint state reproduces.
 * Switching thresholds: the joint-limit activation (predicted end-of-step position against the range, and the
 * one-sided torque test) and the ground-contact activation (predicted end-of-step depth, and the one-sided normal
 * force test) are DECIDED with the limit / the depth shifted by a fresh uniform +-eps (rad / m) per evaluation; the
 * forces themselves use the exact values.  A joint pressed against its limit is pinned by the stiff implicit spring
 * onto the activation surface itself (q + h qd = q_upper to ~1e-9 rad), where the kernel's fp32 evaluation decides
 * either way and a perturbation of the step's initial state is contracted away by that same spring. */
static double g_sj_eps = 0.0, g_tj_lim = 0.0, g_tj_ct = 0.0;
static uint64_t g_sj_state = 0, g_tj_state = 0;
void orc_set_self_jitter(double eps, uint64_t seed) {
  g_sj_eps = eps;
  g_sj_state = seed;
}
void orc_set_threshold_jitter(double lim_eps, double contact_eps, uint64_t seed) {
  g_tj_lim = lim_eps;
  g_tj_ct = contact_eps;
  g_tj_state = seed;
}
static double splitmix_u(uint64_t* st) { /* splitmix64 -> uniform [-1, 1) */
  uint64_t z = (*st += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (double)(z >> 11) * (2.0 / 9007199254740992.0) - 1.0;
}
static double sj_draw(void) { return splitmix_u(&g_sj_state); }
static double tj_draw(double eps) { return eps > 0.0 ? eps * splitmix_u(&g_tj_state) : 0.0; }

/* ------------------------------------------------------------------ penalty contact */
/* Penalty force on a sphere (centre pl in body b coords, radius rad).  Normal: spring-damper,
 * clipped at 0.  Tangential: for sole spheres (anc != NULL) an anchored stiction spring-damper
 * capped by the Coulomb cone (mu_static to stick, mu_dynamic while slipping, anchor dragged
 * along when slipping); for knee / torso a viscous term capped at mu_dynamic.  Accumulates the
 * spatial force (body coords) into fext[b] and the world force into fw.  Returns 1 in contact. */
/* implicit-penalty contacts of one solve: after the accelerations are known, the reported contact force
 * gets the implicit part -Mw a_p (the force the linearised spring-damper applied over the substep) */
typedef struct impl_rec {
  int b;
  double pl[3], Mw[3][3];
  double* fw;
} impl_rec;
typedef struct impl_set {
  int n;
  impl_rec r[16];
} impl_set;

static int contact_point(const h12env_config* c, const kin_t* k, int b, const double pl[3], double rad,
                         double fext[NB][6], double fw[3], const double* anc_in, int was_in, double* anc_out,
                         double mus, double mud, double hi, m6 Madd[NB], double g, impl_set* rec) {
  double xw[3];
  m3v(k->R[b], pl, xw);
  for (int a = 0; a < 3; ++a) xw[a] += k->p[b][a];
  double gx, gy, hg = orc_ground(c, xw[0], xw[1], &gx, &gy);
  double in = 1.0 / sqrt(1.0 + gx * gx + gy * gy), nrm[3] = {-gx * in, -gy * in, in};
  double depth = rad - (xw[2] - hg) * in;
  double vl[3];
  cross3(k->v[b], pl, vl);
  for (int a = 0; a < 3; ++a) vl[a] += k->v[b][3 + a];
  double vw[3];
  m3v(k->R[b], vl, vw);
  double vn = nrm[0] * vw[0] + nrm[1] * vw[1] + nrm[2] * vw[2];
  /* active when the point is predicted below the ground at the end of the substep (implicit: depth - hi vn), so a
   * point arriving at speed is caught within the substep instead of one substep deep */
  const double dj = tj_draw(g_tj_ct); /* 0 unless the threshold-jitter test hook is on */
  if (depth + dj - hi * vn <= 0) return 0;
  /* implicit contact (hi > 0): the spring-damper force at the END of the substep, k (d - hi vn') - c vn'
   * with vn' = vn + hi an, is the explicit force with damping c + hi k plus the term -hi (c + hi k) an,
   * linear in the contact point's acceleration: an added point inertia (alpha along the normal, beta
   * tangentially while the stiction spring sticks / the viscous drag is below its cap) */
  double cn = c->contact_c + hi * c->contact_k;
  /* PhysX max_depenetration_velocity (A/robots/h12.py:29): a sole contact that OPENS with a penetration is pushed
   * out at most this fast (elastic term capped at hi v_max); a persistent contact carries any load */
  double dcap = (hi > 0 && c->max_depenetration_velocity > 0 && anc_out && !was_in) ? hi * c->max_depenetration_velocity
                                                                                     : 1e300;
  double fn = c->contact_k * (depth < dcap ? depth : dcap) - cn * vn;
  /* Madd == NULL: the force only, without its implicit part (the torso face's secondary corners) */
  if (dj != 0.0) {
    if (c->contact_k * (depth + dj < dcap ? depth + dj : dcap) - cn * vn <= 0) return 0;
    if (fn < 0) fn = 0;
  } else if (fn <= 0) return 0;
  double ft0, ft1, beta = 0;
  if (anc_out) {
    double ax = was_in ? anc_in[0] : xw[0], ay = was_in ? anc_in[1] : xw[1];
    double ct = c->friction_c + hi * c->friction_k;
    ft0 = -c->friction_k * (xw[0] - ax) - ct * vw[0];
    ft1 = -c->friction_k * (xw[1] - ay) - ct * vw[1];
    double ftn = sqrt(ft0 * ft0 + ft1 * ft1);
    if (ftn > mus * fn) {
      double sc = mud * fn / ftn;
      ft0 *= sc;
      ft1 *= sc;
      ax = xw[0] + ft0 / c->friction_k;
      ay = xw[1] + ft1 / c->friction_k;
    } else {
      beta = hi * ct;
    }
    anc_out[0] = ax;
    anc_out[1] = ay;
  } else {
    ft0 = -c->friction_c * vw[0];
    ft1 = -c->friction_c * vw[1];
    double ftn = sqrt(ft0 * ft0 + ft1 * ft1), cap = mud * fn;
    if (ftn > cap) { ft0 *= cap / ftn; ft1 *= cap / ftn; }
    else beta = hi * c->friction_c;
  }
  /* normal force along the ground normal, tangential (stiction / drag) force in world xy */
  double F[3] = {ft0 + fn * nrm[0], ft1 + fn * nrm[1], fn * nrm[2]}, fl[3], nl[3];
  if (hi > 0 && Madd) {
    /* world mass tensor Mw = alpha n n^T + beta (I - n n^T) -> body coords Mb = R^T Mw R; point inertia at
     * pl: [[-px Mb px, px Mb], [-Mb px, Mb]].  The dynamics run with gravity as a base acceleration, which
     * would weigh the added inertia: cancel with the force g Mw e_z at the point. */
    double alpha = hi * cn, Mw[3][3], Mb[3][3], T[3][3];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) Mw[i][j] = (alpha - beta) * nrm[i] * nrm[j] + (i == j ? beta : 0.0);
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        double t = 0;
        for (int a = 0; a < 3; ++a) t += Mw[i][a] * k->R[b][a][j];
        T[i][j] = t;
      }
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        double t = 0;
        for (int a = 0; a < 3; ++a) t += k->R[b][a][i] * T[a][j];
        Mb[i][j] = t;
      }
    m3 px = {{0, -pl[2], pl[1]}, {pl[2], 0, -pl[0]}, {-pl[1], pl[0], 0}}, PM, MP, PMP;
    m3mul(px, Mb, PM);
    m3mul(Mb, px, MP);
    m3mul(PM, px, PMP);
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        Madd[b][i][j] -= PMP[i][j];
        Madd[b][i][3 + j] += PM[i][j];
        Madd[b][3 + i][j] -= MP[i][j];
        Madd[b][3 + i][3 + j] += Mb[i][j];
      }
    for (int a = 0; a < 3; ++a) F[a] += g * Mw[a][2];
    if (rec && rec->n < 16) {
      impl_rec* ir = &rec->r[rec->n++];
      ir->b = b;
      memcpy(ir->pl, pl, sizeof ir->pl);
      memcpy(ir->Mw, Mw, sizeof ir->Mw);
      ir->fw = fw;
    }
  }
  /* reported force: the applied one (with the implicit part -Mw a added after the solve, implicit_report) */
  for (int a = 0; a < 3; ++a) fw[a] += F[a];
  m3tv(k->R[b], F, fl);
  cross3(pl, fl, nl);
  for (int a = 0; a < 3; ++a) { fext[b][a] += nl[a]; fext[b][3 + a] += fl[a]; }
  return 1;
}

/* ---- self-collision between the legs (ArticulationCfg enabled_self_collisions=True, A/robots/h12.py:32).
 * Colliders of the URDF the IsaacLab USD was converted from: the knee cylinders (h12_12dof.urdf:116,286) and
 * the four sole rods of each foot (:168-191, :338-361), as capsules (segment + radius).  PhysX filters
 * jointed parent/child pairs; within one leg no knee/foot pair can touch (shank 0.4 m), so every left/right
 * pair is tested.  Generic restatement (world frame, every pair, fp64); the kernel mirrors it per lane pair. */

/* Contact points of two capsule axes p1-q1 and p2-q2 (the self-contact model; the kernel's seg_points restates it):
 * * general (sin^2 of the angle between the axes >= 1e-3): the closest points (the standard clamped-parameter
 *   construction), one point.  When both parameters are interior the closest-point difference is along d1 x d2, and
 *   the contact normal is taken from that cross product (sign: the difference's side): the same direction, but
 *   well-conditioned where the axes nearly intersect (rods pressed through each other to their axes), where the
 *   difference itself is a few fp32 ulps long and its direction is noise;
 * * nearly parallel (sin^2 < 1e-3, 1.8 deg): a LINE contact -- two points, at the two ends of the overlap of the
 *   segments along the first one, each with half the pair's stiffness and damping (a uniformly pressed parallel pair
 *   gets the one-point law; a tilted one is pressed at its closer end).  Without overlap: the nearest ends, one point.
 * Returns the number of points; w: the per-point weight; nc: the cross-product normal (unit, from segment 2 towards
 * segment 1) when has_nc. */
typedef struct seg_pts {
  int n, has_nc;
  double w, c1[2][3], c2[2][3], nc[3];
} seg_pts;
static double seg_t(double B, double F, double E, double s) { return clampd((B * s + F) / E, 0.0, 1.0); }
static void seg_points(const double p1[3], const double q1[3], const double p2[3], const double q2[3], seg_pts* o) {
  double d1[3], d2[3], r[3];
  for (int a = 0; a < 3; ++a) { d1[a] = q1[a] - p1[a]; d2[a] = q2[a] - p2[a]; r[a] = p1[a] - p2[a]; }
  const double A = dot3(d1, d1), E = dot3(d2, d2), F = dot3(d2, r), C = dot3(d1, r), B = dot3(d1, d2);
  const double den = A * E - B * B;
  double sp[2], tp[2];
  o->n = 1;
  o->w = 1.0;
  o->has_nc = 0;
  o->nc[0] = o->nc[1] = o->nc[2] = 0.0;
  if (den > 1e-3 * A * E) {
    double s = clampd((B * F - C * E) / den, 0.0, 1.0), t = (B * s + F) / E;
    if (t < 0.0) { t = 0.0; s = clampd(-C / A, 0.0, 1.0); }
    else if (t > 1.0) { t = 1.0; s = clampd((B - C) / A, 0.0, 1.0); }
    else if (s > 0.0 && s < 1.0) {
      double c[3];
      cross3(d1, d2, c);
      const double cn = 1.0 / sqrt(dot3(c, c));
      for (int a = 0; a < 3; ++a) o->nc[a] = c[a] * cn;
      o->has_nc = 1;
    }
    sp[0] = s;
    tp[0] = t;
  } else {
    const double t0 = -C / A, t1 = (B - C) / A; /* segment 2's ends projected onto segment 1 */
    const double lo = fmax(0.0, fmin(t0, t1)), hi = fmin(1.0, fmax(t0, t1));
    if (hi > lo) {
      o->n = 2;
      o->w = 0.5;
      sp[0] = lo;
      sp[1] = hi;
      tp[0] = seg_t(B, F, E, lo);
      tp[1] = seg_t(B, F, E, hi);
    } else { /* end to end: the nearest ends */
      double s = clampd(0.5 * (lo + hi), 0.0, 1.0), t = (B * s + F) / E;
      if (t < 0.0) { t = 0.0; s = clampd(-C / A, 0.0, 1.0); }
      else if (t > 1.0) { t = 1.0; s = clampd((B - C) / A, 0.0, 1.0); }
      sp[0] = s;
      tp[0] = t;
    }
  }
  for (int k = 0; k < o->n; ++k)
    for (int a = 0; a < 3; ++a) { o->c1[k][a] = p1[a] + d1[a] * sp[k]; o->c2[k][a] = p2[a] + d2[a] * tp[k]; }
}

typedef struct capsule_w {
  int b;               /* body */
  double p0[3], p1[3]; /* world segment */
  double r;
} capsule_w;

/* The self-contact geometry runs in PELVIS-RELATIVE world axes (positions minus the base origin, |x| < 1.2 m): only
 * differences of body points enter it, and the kernel does the same so that its fp32 points carry the ulp of ~1 m,
 * not of the env's world position.  po(k, b): body b's origin relative to the base origin. */
static void po(const kin_t* k, int b, double out[3]) {
  for (int a = 0; a < 3; ++a) out[a] = k->p[b][a] - k->p[0][a];
}

static void capsule_world(const kin_t* k, int b, const float* p0, const float* p1, double r, capsule_w* out) {
  double a0[3] = {p0[0], p0[1], p0[2]}, a1[3] = {p1[0], p1[1], p1[2]}, ob[3];
  out->b = b;
  out->r = r;
  m3v(k->R[b], a0, out->p0);
  m3v(k->R[b], a1, out->p1);
  po(k, b, ob);
  for (int a = 0; a < 3; ++a) { out->p0[a] += ob[a]; out->p1[a] += ob[a]; }
  if (g_sj_eps > 0.0)
    for (int a = 0; a < 3; ++a) { out->p0[a] += g_sj_eps * sj_draw(); out->p1[a] += g_sj_eps * sj_draw(); }
}

/* world velocity of the body-b material point at x (pelvis-relative, see po) */
static void point_vel(const kin_t* k, int b, const double x[3], double v[3]) {
  double w[3], vo[3], rx[3], wr[3], ob[3];
  m3v(k->R[b], k->v[b], w);
  m3v(k->R[b], k->v[b] + 3, vo);
  po(k, b, ob);
  for (int a = 0; a < 3; ++a) rx[a] = x[a] - ob[a];
  cross3(w, rx, wr);
  for (int a = 0; a < 3; ++a) v[a] = vo[a] + wr[a];
}

/* world force F at point x (pelvis-relative, see po) on body b -> body-coordinate spatial force */
static void apply_world_force(const kin_t* k, int b, const double x[3], const double F[3], double fext[NB][6]) {
  double rx[3], xb[3], fb[3], nb[3], ob[3];
  po(k, b, ob);
  for (int a = 0; a < 3; ++a) rx[a] = x[a] - ob[a];
  m3tv(k->R[b], rx, xb);
  m3tv(k->R[b], F, fb);
  cross3(xb, fb, nb);
  for (int a = 0; a < 3; ++a) { fext[b][a] += nb[a]; fext[b][3 + a] += fb[a]; }
}

static void self_contacts(const h12env_model* m, const h12env_config* c, const kin_t* k, const orc_phys* s,
                          double fext[NB][6], orc_contact_report* rr) {
  /* Coulomb cap of the leg-leg pairs: PhysX multiply combine of the two bodies' materials -- with the startup
   * material randomisation (randomize_rigid_body_material, C12/rsl_env_cfg.py:213-223) the product of the two
   * legs' randomised dynamic coefficients, otherwise the fixed 0.6 x 0.6 (self_mu) */
  const double smu = (c->per_env_friction && s->env_params) ? s->mu[0][1] * s->mu[1][1] : c->self_mu;
  capsule_w cap[2][5]; /* per leg: knee, then the four sole rods */
  for (int f = 0; f < 2; ++f) {
    capsule_world(k, 6 * f + 4, m->knee_p0, m->knee_p1, m->knee_radius, &cap[f][0]);
    for (int r = 0; r < 4; ++r) {
      float p0[3], p1[3];
      for (int a = 0; a < 3; ++a) {
        /* the right foot's rods are the mirror images (y -> -y) of the left foot's */
        const double sy = (f == 1 && a == 1) ? -1.0 : 1.0;
        p0[a] = (float)(sy * m->foot_rods[r][0][a]);
        p1[a] = (float)(sy * m->foot_rods[r][1][a]);
      }
      capsule_world(k, 6 * f + 6, p0, p1, m->foot_radius, &cap[f][1 + r]);
    }
  }
  for (int i = 0; i < 5; ++i)
    for (int j = 0; j < 5; ++j) {
      const capsule_w *A = &cap[0][i], *Bc = &cap[1][j];
      seg_pts sp;
      seg_points(A->p0, A->p1, Bc->p0, Bc->p1, &sp);
      for (int q = 0; q < sp.n; ++q) {
        const double *cA = sp.c1[q], *cB = sp.c2[q];
        double dv[3] = {cA[0] - cB[0], cA[1] - cB[1], cA[2] - cB[2]};
        const double d = sqrt(dot3(dv, dv)), depth = A->r + Bc->r - d;
        if (!(depth > 0.0) || d < 1e-9) continue;
        double n[3], x[3], va[3], vb[3], vr[3];
        const double sgn = dot3(dv, sp.nc) < 0.0 ? -1.0 : 1.0;
        for (int a = 0; a < 3; ++a) { n[a] = sp.has_nc ? sgn * sp.nc[a] : dv[a] / d; x[a] = 0.5 * (cA[a] + cB[a]); }
        point_vel(k, A->b, x, va);
        point_vel(k, Bc->b, x, vb);
        for (int a = 0; a < 3; ++a) vr[a] = va[a] - vb[a];
        const double vn = dot3(vr, n), fn = sp.w * (c->self_k * depth - c->self_c * vn);
        if (!(fn > 0.0)) continue;
        double ft[3];
        for (int a = 0; a < 3; ++a) ft[a] = -sp.w * c->self_ct * (vr[a] - vn * n[a]);
        const double ftn = sqrt(dot3(ft, ft)), cap_t = smu * fn;
        if (ftn > cap_t) for (int a = 0; a < 3; ++a) ft[a] *= cap_t / ftn;
        double F[3], Fm[3];
        for (int a = 0; a < 3; ++a) { F[a] = fn * n[a] + ft[a]; Fm[a] = -F[a]; }
        apply_world_force(k, A->b, x, F, fext);
        apply_world_force(k, Bc->b, x, Fm, fext);
        double* ra = i == 0 ? rr->knee_force[0] : rr->foot_force[0];
        double* rb = j == 0 ? rr->knee_force[1] : rr->foot_force[1];
        for (int a = 0; a < 3; ++a) { ra[a] += F[a]; rb[a] -= F[a]; }
      }
    }
}

/* evaluates every contact primitive; s->anchor/cmask are read, next_anchor/next_mask written */
static void contacts(const h12env_model* m, const h12env_config* c, const kin_t* k, const orc_phys* s,
                     double fext[NB][6], orc_contact_report* rep, double next_anchor[2][H12_NFOOT_PTS][2],
                     int32_t* next_mask, double hi, m6 Madd[NB], impl_set* rec) {
  orc_contact_report local, *rr = rep ? rep : &local; /* written in place: implicit corrections follow */
  memset(rr, 0, sizeof *rr);
  if (!rep) rec = NULL;
  int32_t mask = 0;
  for (int f = 0; f < 2; ++f) {
    int b = 6 * f + 6; /* ankle roll link of leg f */
    for (int p = 0; p < H12_NFOOT_PTS; ++p) {
      double pl[3] = {m->foot_pts[p][0], m->foot_pts[p][1], m->foot_pts[p][2]};
      int bit = 4 * f + p;
      double tmp[2];
      double* out = next_anchor ? next_anchor[f][p] : tmp;
      double mus = s->env_params ? s->mu[f][0] : c->mu_static, mud = s->env_params ? s->mu[f][1] : c->mu_dynamic;
      if (contact_point(c, k, b, pl, m->foot_radius, fext, rr->foot_force[f], s->anchor[f][p], (s->cmask >> bit) & 1, out,
                        mus, mud, hi, Madd, m->gravity, rec))
        mask |= 1 << bit;
    }
    /* knee capsule: lower end point of the segment in world z */
    int bk = 6 * f + 4;
    double a0[3] = {m->knee_p0[0], m->knee_p0[1], m->knee_p0[2]}, a1[3] = {m->knee_p1[0], m->knee_p1[1], m->knee_p1[2]};
    double w0[3], w1[3];
    m3v(k->R[bk], a0, w0);
    m3v(k->R[bk], a1, w1);
    contact_point(c, k, bk, (w0[2] <= w1[2]) ? a0 : a1, m->knee_radius, fext, rr->knee_force[f], 0, 0, 0,
                  c->mu_static, c->mu_dynamic, hi, Madd, m->gravity, rec);
  }
  /* torso box (welded to the base): lowest corner */
  double corner[3];
  for (int a = 0; a < 3; ++a) {
    double sg = k->R[0][2][a] > 0 ? -1.0 : 1.0;
    corner[a] = m->torso_center[a] + sg * m->torso_half[a];
  }
  /* the other three corners of the lowest face (normal: the box axis closest to the vertical), explicit forces
   * only -- a torso lying on a face or an edge rests on that face's corners (kernel torso_face, same order); on
   * terrain only while the lowest corner touches (the kernel keeps the heightfield lookups off a standing robot) */
  const int lowest = contact_point(c, k, 0, corner, 0.0, fext, rr->torso_force, 0, 0, 0, c->mu_static, c->mu_dynamic,
                                   hi, Madd, m->gravity, rec);
  if (lowest || !c->terrain) {
    const double z0 = fabs(k->R[0][2][0]), z1 = fabs(k->R[0][2][1]), z2 = fabs(k->R[0][2][2]);
    const int an = (z0 >= z1 && z0 >= z2) ? 0 : (z1 >= z2 ? 1 : 2);
    const int ab = an == 0 ? 1 : 0, ac = an == 2 ? 1 : 2;
    for (int q = 1; q < 4; ++q) {
      double pc[3];
      for (int a = 0; a < 3; ++a) {
        const int flip = ((q & 1) && a == ab) || ((q & 2) && a == ac);
        const int neg = (k->R[0][2][a] > 0) != flip;
        pc[a] = m->torso_center[a] + (neg ? -1.0 : 1.0) * m->torso_half[a];
      }
      contact_point(c, k, 0, pc, 0.0, fext, rr->torso_force, 0, 0, 0, c->mu_static, c->mu_dynamic, hi, NULL,
                    m->gravity, NULL);
    }
  }
  if (c->self_collision) self_contacts(m, c, k, s, fext, rr);
  if (next_mask) *next_mask = mask;
}

/* ------------------------------------------------------------------ dynamics */
/* RNEA: generalised force for accelerations nudot (base spatial accel + qdd), with external forces */
static void rnea(const h12env_model* m, const kin_t* k, const orc_phys* s, const double nudot[18],
                 double fext[NB][6], m6 Madd[NB], double out[18]) {
  double a[NB][6], f[NB][6];
  for (int i = 0; i < 6; ++i) a[0][i] = nudot[i] - k->ag[i];
  for (int j = 0; j < NJ; ++j) {
    int b = j + 1, par = m->parent[j] + 1;
    double sq[6] = {0, 0, 0, 0, 0, 0}, t[6];
    sq[m->axis[j]] = s->qd[j];
    m6v(k->X[b], a[par], a[b]);
    a[b][m->axis[j]] += nudot[6 + j];
    crm(k->v[b], sq, t);
    for (int i = 0; i < 6; ++i) a[b][i] += t[i];
  }
  for (int b = 0; b < NB; ++b) {
    double Iv[6], Ia[6], t[6];
    m6v(k->I[b], k->v[b], Iv);
    m6v(k->I[b], a[b], Ia);
    crf(k->v[b], Iv, t);
    for (int i = 0; i < 6; ++i) f[b][i] = Ia[i] + t[i] - fext[b][i];
    if (Madd) {
      double Ma[6];
      m6v(Madd[b], a[b], Ma);
      for (int i = 0; i < 6; ++i) f[b][i] += Ma[i];
    }
  }
  for (int j = NJ - 1; j >= 0; --j) {
    int b = j + 1, par = m->parent[j] + 1;
    out[6 + j] = f[b][m->axis[j]];
    double t[6];
    m6tv(k->X[b], f[b], t);
    for (int i = 0; i < 6; ++i) f[par][i] += t[i];
  }
  for (int i = 0; i < 6; ++i) out[i] = f[0][i];
}

static void crba(const h12env_model* m, const kin_t* k, m6 Madd[NB], double H[18 * 18]) {
  m6 Ic[NB];
  memcpy(Ic, k->I, sizeof Ic);
  if (Madd)
    for (int b = 0; b < NB; ++b)
      for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) Ic[b][i][j] += Madd[b][i][j];
  for (int j = NJ - 1; j >= 0; --j) {
    int b = j + 1, par = m->parent[j] + 1;
    m6 T;
    congruence(k->X[b], Ic[b], T);
    for (int a = 0; a < 6; ++a)
      for (int c = 0; c < 6; ++c) Ic[par][a][c] += T[a][c];
  }
  memset(H, 0, sizeof(double) * 18 * 18);
  for (int a = 0; a < 6; ++a)
    for (int c = 0; c < 6; ++c) H[a * 18 + c] = Ic[0][a][c];
  for (int j = 0; j < NJ; ++j) {
    int b = j + 1;
    double F[6];
    for (int i = 0; i < 6; ++i) F[i] = Ic[b][i][m->axis[j]];
    H[(6 + j) * 18 + 6 + j] = F[m->axis[j]];
    int jj = j;
    while (m->parent[jj] >= 0) {
      double t[6];
      m6tv(k->X[jj + 1], F, t);
      memcpy(F, t, sizeof t);
      jj = m->parent[jj];
      H[(6 + j) * 18 + 6 + jj] = H[(6 + jj) * 18 + 6 + j] = F[m->axis[jj]];
    }
    double t[6];
    m6tv(k->X[jj + 1], F, t);
    for (int i = 0; i < 6; ++i) H[(6 + j) * 18 + i] = H[i * 18 + 6 + j] = t[i];
  }
}

static int aba(const h12env_model* m, const h12env_config* c, const kin_t* k, const orc_phys* s,
               const double tau[NJ], const double dimpl[NJ], double fext[NB][6], m6 Madd[NB], double nudot[18]) {
  m6 IA[NB];
  double pA[NB][6], cb[NB][6], U[NB][6], D[NB], u[NB];
  for (int b = 0; b < NB; ++b) {
    double Iv[6];
    for (int i = 0; i < 6; ++i)
      for (int j = 0; j < 6; ++j) IA[b][i][j] = k->I[b][i][j] + Madd[b][i][j];
    m6v(k->I[b], k->v[b], Iv);
    crf(k->v[b], Iv, pA[b]);
    for (int i = 0; i < 6; ++i) pA[b][i] -= fext[b][i];
  }
  for (int j = 0; j < NJ; ++j) {
    int b = j + 1;
    double sq[6] = {0, 0, 0, 0, 0, 0};
    sq[m->axis[j]] = s->qd[j];
    crm(k->v[b], sq, cb[b]);
  }
  for (int j = NJ - 1; j >= 0; --j) {
    int b = j + 1, par = m->parent[j] + 1, ax = m->axis[j];
    for (int i = 0; i < 6; ++i) U[b][i] = IA[b][i][ax];
    D[b] = U[b][ax] + m->armature[j] + dimpl[j];
    u[b] = tau[j] - pA[b][ax];
    m6 Ia;
    for (int a = 0; a < 6; ++a)
      for (int cc = 0; cc < 6; ++cc) Ia[a][cc] = IA[b][a][cc] - U[b][a] * U[b][cc] / D[b];
    double pa[6], t[6];
    m6v(Ia, cb[b], t);
    for (int i = 0; i < 6; ++i) pa[i] = pA[b][i] + t[i] + U[b][i] * u[b] / D[b];
    m6 T;
    congruence(k->X[b], Ia, T);
    for (int a = 0; a < 6; ++a)
      for (int cc = 0; cc < 6; ++cc) IA[par][a][cc] += T[a][cc];
    m6tv(k->X[b], pa, t);
    for (int i = 0; i < 6; ++i) pA[par][i] += t[i];
  }
  double a[NB][6];
  if (c->fix_base) {
    for (int i = 0; i < 6; ++i) a[0][i] = -k->ag[i];
  } else {
    double A[36], rhs[6];
    for (int i = 0; i < 6; ++i) { rhs[i] = -pA[0][i]; for (int j = 0; j < 6; ++j) A[i * 6 + j] = IA[0][i][j]; }
    if (chol_solve(A, 6, rhs)) return -1;
    memcpy(a[0], rhs, sizeof rhs);
  }
  for (int j = 0; j < NJ; ++j) {
    int b = j + 1, par = m->parent[j] + 1, ax = m->axis[j];
    double ap[6];
    m6v(k->X[b], a[par], ap);
    for (int i = 0; i < 6; ++i) ap[i] += cb[b][i];
    double ua = 0;
    for (int i = 0; i < 6; ++i) ua += U[b][i] * ap[i];
    double qdd = (u[b] - ua) / D[b];
    ap[ax] += qdd;
    memcpy(a[b], ap, sizeof ap);
    nudot[6 + j] = qdd;
  }
  if (c->fix_base) for (int i = 0; i < 6; ++i) nudot[i] = 0;
  else for (int i = 0; i < 6; ++i) nudot[i] = a[0][i] + k->ag[i];
  return 0;
}

int orc_mass_matrix(const h12env_model* m, const orc_phys* s, double M[18 * 18]) {
  kin_t k;
  kinematics(m, s, &k);
  crba(m, &k, NULL, M);
  for (int j = 0; j < NJ; ++j) M[(6 + j) * 18 + 6 + j] += m->armature[j];
  return 0;
}

/* joint limits (PhysX holds the URDF ranges as hard limits, A/robots/h12.py:18-35, h12_12dof.urdf:53-198): a stiff
 * one-sided spring-damper outside the MJCF range.  With the implicit penalty (hi > 0) it acts on the joint's
 * position at the END of the substep, q + hi qd': active when the predicted end position q + hi qd is beyond the
 * range (a joint arriving at speed is stopped at the limit within the step instead of one step past it), torque
 * -lk (q + hi qd' - limit) - lc qd' linearised in the acceleration: explicit part -lk (q - limit) - (lc + hi lk) qd
 * (repulsive only) and the added joint inertia dl[j] = hi (lc + hi lk) -- implicit Euler on the limit spring,
 * stable at any stiffness.  Explicit integration (hi = 0): active past the range. */
static void joint_limit_torque(const h12env_model* m, const h12env_config* c, const orc_phys* s, double hi,
                               double hdyn, double tau[NJ], double dl[NJ]) {
  double cl = c->limit_c + hi * c->limit_k;
  for (int j = 0; j < NJ; ++j) {
    double q = s->q[j], qd = s->qd[j], t = 0, qe = q + hi * qd;
    const double uh = m->q_upper[j] + tj_draw(g_tj_lim), ul = m->q_lower[j] + tj_draw(g_tj_lim); /* decisions */
    dl[j] = 0;
    if (qe > uh) {
      t = -c->limit_k * (q - m->q_upper[j]) - cl * qd;
      if (-c->limit_k * (q - uh) - cl * qd > 0) t = 0; else { dl[j] = hi * cl; if (t > 0) t = 0; }
    } else if (qe < ul) {
      t = -c->limit_k * (q - m->q_lower[j]) - cl * qd;
      if (-c->limit_k * (q - ul) - cl * qd < 0) t = 0; else { dl[j] = hi * cl; if (t < 0) t = 0; }
    }
    /* PhysX max joint velocity: stiff damper on the excess, implicit over the substep (always: the solve
     * must carry the reaction; h = 0 would make it explicit and unstable) */
    double vm = c->max_joint_vel[j], cv = c->max_joint_vel_damping, ex = fabs(qd) - vm, rp = H12_VLIM_RAMP;
    if (vm > 0 && cv > 0 && ex > 0) {
      double mag = ex < rp ? cv * ex * ex / (2 * rp) : cv * (ex - 0.5 * rp);
      t += qd > 0 ? -mag : mag;
      dl[j] += hdyn * cv * (ex < rp ? ex / rp : 1.0);
    }
    tau[j] += t;
  }
}

/* add the implicit part of every implicit-penalty contact to its reported force.  The linearised force is
 * F_e - Mw a_p (a_p: the point's true acceleration); the solve runs in the gravity-shifted frame
 * (accelerations a' = a - ag) where -Mw a_p = g Mw e_z - Mw a'_p: contact_point already added g Mw e_z
 * (the weight-cancelling force), this adds -Mw a'_p */
static void implicit_report(const h12env_model* m, const kin_t* k, const orc_phys* s, int fix_base,
                            const double nudot[18], impl_set* rec) {
  if (!rec->n) return;
  double a[NB][6];
  for (int i = 0; i < 6; ++i) a[0][i] = (fix_base ? 0.0 : nudot[i]) - k->ag[i];
  for (int j = 0; j < NJ; ++j) {
    int b = j + 1, par = m->parent[j] + 1;
    double sq[6] = {0, 0, 0, 0, 0, 0}, t[6];
    sq[m->axis[j]] = s->qd[j];
    m6v(k->X[b], a[par], a[b]);
    a[b][m->axis[j]] += nudot[6 + j];
    crm(k->v[b], sq, t);
    for (int i = 0; i < 6; ++i) a[b][i] += t[i];
  }
  for (int i = 0; i < rec->n; ++i) {
    const impl_rec* r = &rec->r[i];
    double ap[3], aw[3];
    cross3(a[r->b], r->pl, ap);
    for (int q = 0; q < 3; ++q) ap[q] += a[r->b][3 + q];
    m3v(k->R[r->b], ap, aw);
    for (int q = 0; q < 3; ++q) r->fw[q] -= r->Mw[q][0] * aw[0] + r->Mw[q][1] * aw[1] + r->Mw[q][2] * aw[2];
  }
}

static int forward_dynamics(const h12env_model* m, const h12env_config* c, const orc_phys* s, const double tau[NJ],
                            int algo, double dt_impl, const double* dl, int with_contact, double nudot[18],
                            orc_contact_report* rep, double next_anchor[2][H12_NFOOT_PTS][2], int32_t* next_mask) {
  kin_t k;
  kinematics(m, s, &k);
  double fext[NB][6];
  m6 Madd[NB];
  memset(fext, 0, sizeof fext);
  memset(Madd, 0, sizeof Madd);
  impl_set rec;
  rec.n = 0;
  if (with_contact)
    contacts(m, c, &k, s, fext, rep, next_anchor, next_mask, c->implicit_penalty ? dt_impl : 0.0, Madd, &rec);
  else {
    if (rep) memset(rep, 0, sizeof *rep);
    if (next_mask) *next_mask = 0;
  }
  double dimpl[NJ], tq[NJ];
  int mj = (c->mode == H12_MODE_MUJOCO);
  for (int j = 0; j < NJ; ++j) {
    double d = mj ? m->damping[j] : 0.0;
    dimpl[j] = dt_impl * d + (dl ? dl[j] : 0.0);
    tq[j] = tau[j] - d * s->qd[j];
    if (c->use_frictionloss) tq[j] -= m->frictionloss[j] * tanh(s->qd[j] / 0.01);
  }
  if (algo == 1) {
    if (aba(m, c, &k, s, tq, dimpl, fext, Madd, nudot)) return -1;
    implicit_report(m, &k, s, c->fix_base, nudot, &rec);
    return 0;
  }
  double H[18 * 18], C[18], zero[18] = {0};
  crba(m, &k, Madd, H);
  rnea(m, &k, s, zero, fext, Madd, C);
  for (int j = 0; j < NJ; ++j) H[(6 + j) * 18 + 6 + j] += m->armature[j] + dimpl[j];
  double b[18];
  for (int i = 0; i < 6; ++i) b[i] = -C[i];
  for (int j = 0; j < NJ; ++j) b[6 + j] = tq[j] - C[6 + j];
  if (c->fix_base) {
    /* base rows removed: solve the 12 x 12 joint block with the base held (nudot_base = 0) */
    double Hj[NJ * NJ];
    for (int a = 0; a < NJ; ++a)
      for (int cc = 0; cc < NJ; ++cc) Hj[a * NJ + cc] = H[(6 + a) * 18 + 6 + cc];
    double bj[NJ];
    memcpy(bj, b + 6, sizeof bj);
    if (chol_solve(Hj, NJ, bj)) return -1;
    for (int i = 0; i < 6; ++i) nudot[i] = 0;
    memcpy(nudot + 6, bj, sizeof bj);
    return 0;
  }
  if (chol_solve(H, 18, b)) return -1;
  memcpy(nudot, b, sizeof b);
  implicit_report(m, &k, s, 0, nudot, &rec);
  return 0;
}

int orc_forward_dynamics(const h12env_model* m, const h12env_config* c, const orc_phys* s, const double tau[NJ],
                         int algo, double dt_impl, int with_contact, double nudot[18], orc_contact_report* rep) {
  return forward_dynamics(m, c, s, tau, algo, dt_impl, NULL, with_contact, nudot, rep, 0, 0);
}

/* the self-contact wrenches alone (body-coordinate spatial forces, NB x 6) and their report, for tests */
int orc_self_contacts(const h12env_model* m, const h12env_config* c, const orc_phys* s, double* fext,
                      orc_contact_report* rep) {
  kin_t k;
  kinematics(m, s, &k);
  memset(fext, 0, sizeof(double) * NB * 6);
  memset(rep, 0, sizeof *rep);
  self_contacts(m, c, &k, s, (double(*)[6])fext, rep);
  return 0;
}

/* world pose (R row-major, p) of every body, for tests */
int orc_body_poses(const h12env_model* m, const orc_phys* s, double* R, double* p) {
  kin_t k;
  kinematics(m, s, &k);
  for (int b = 0; b < NB; ++b) {
    for (int i = 0; i < 3; ++i) {
      p[3 * b + i] = k.p[b][i];
      for (int j = 0; j < 3; ++j) R[9 * b + 3 * i + j] = k.R[b][i][j];
    }
  }
  return 0;
}

int orc_energy_momentum(const h12env_model* m, const orc_phys* s, double* energy, double lin[3], double ang[3]) {
  kin_t k;
  kinematics(m, s, &k);
  double ke = 0, pe = 0;
  for (int a = 0; a < 3; ++a) lin[a] = ang[a] = 0;
  for (int b = 0; b < NB; ++b) {
    double h[6];
    m6v(k.I[b], k.v[b], h);
    for (int i = 0; i < 6; ++i) ke += 0.5 * k.v[b][i] * h[i];
    double hl[3], ha[3], t[3];
    m3v(k.R[b], h + 3, hl);
    m3v(k.R[b], h, ha);
    cross3(k.p[b], hl, t);
    for (int a = 0; a < 3; ++a) { lin[a] += hl[a]; ang[a] += ha[a] + t[a]; }
    double mass = b == 0 ? m->base_mass : m->link_mass[b - 1];
    const float* com = b == 0 ? m->base_com : m->link_com[b - 1];
    double cl[3] = {com[0], com[1], com[2]}, cw[3];
    m3v(k.R[b], cl, cw);
    pe += mass * m->gravity * (k.p[b][2] + cw[2]);
  }
  if (s->env_params && s->dmass != 0.0) { /* added torso point mass: kinetic part is in k.I[0] */
    double ct[3] = {m->torso_com[0], m->torso_com[1], m->torso_com[2]}, cw[3];
    m3v(k.R[0], ct, cw);
    pe += s->dmass * m->gravity * (k.p[0][2] + cw[2]);
  }
  for (int j = 0; j < NJ; ++j) ke += 0.5 * m->armature[j] * s->qd[j] * s->qd[j];
  *energy = ke + pe;
  return 0;
}

/* semi-implicit Euler in MuJoCo coordinates (mj_Euler + mju_quatIntegrate) */
static void integrate(orc_phys* s, const double nd[18], double dt, int fix_base) {
  if (!fix_base) {
    m3 R;
    quat_to_R(s->quat, R);
    double vb[3], wxv[3], al[3], aw[3];
    m3tv(R, s->vlin, vb);
    cross3(s->wang, vb, wxv);
    for (int a = 0; a < 3; ++a) al[a] = nd[3 + a] + wxv[a];
    m3v(R, al, aw);
    for (int a = 0; a < 3; ++a) { s->vlin[a] += dt * aw[a]; s->wang[a] += dt * nd[a]; }
    for (int a = 0; a < 3; ++a) s->pos[a] += dt * s->vlin[a];
    double w2 = s->wang[0] * s->wang[0] + s->wang[1] * s->wang[1] + s->wang[2] * s->wang[2];
    double wn = sqrt(w2);
    if (wn > 0) {
      double ang = wn * dt, sh = sin(0.5 * ang) / wn, ch = cos(0.5 * ang);
      double r[4] = {ch, s->wang[0] * sh, s->wang[1] * sh, s->wang[2] * sh};
      double* q = s->quat;
      double o[4] = {q[0] * r[0] - q[1] * r[1] - q[2] * r[2] - q[3] * r[3],
                     q[0] * r[1] + q[1] * r[0] + q[2] * r[3] - q[3] * r[2],
                     q[0] * r[2] - q[1] * r[3] + q[2] * r[0] + q[3] * r[1],
                     q[0] * r[3] + q[1] * r[2] - q[2] * r[1] + q[3] * r[0]};
      double n = sqrt(o[0] * o[0] + o[1] * o[1] + o[2] * o[2] + o[3] * o[3]);
      for (int a = 0; a < 4; ++a) q[a] = o[a] / n;
    }
  }
  for (int j = 0; j < NJ; ++j) { s->qd[j] += dt * nd[6 + j]; s->q[j] += dt * s->qd[j]; }
}

/* hard-limit residual: a joint that the other forces carried further than limit_projection past its range within
 * the step (the limit spring acts only where the step started or was predicted beyond the range) is projected back
 * to that tolerance and its outward velocity zeroed -- the position-level limit correction of a hard-limit solver.
 * Off (0) in MuJoCo mode, whose limits are soft. */
static void limit_projection(const h12env_model* m, const h12env_config* c, orc_phys* s) {
  if (!(c->limit_projection > 0)) return;
  for (int j = 0; j < NJ; ++j) {
    double hi = m->q_upper[j] + c->limit_projection, lo = m->q_lower[j] - c->limit_projection;
    if (s->q[j] > hi) { s->q[j] = hi; if (s->qd[j] > 0) s->qd[j] = 0; }
    else if (s->q[j] < lo) { s->q[j] = lo; if (s->qd[j] < 0) s->qd[j] = 0; }
  }
}

int orc_physics_step(const h12env_model* m, const h12env_config* c, orc_phys* s, const double tau_pd[NJ],
                     int with_contact, int algo, orc_contact_report* rep) {
  int n = c->inner_steps < 1 ? 1 : c->inner_steps;
  double h = c->physics_dt / n;
  orc_contact_report acc;
  memset(&acc, 0, sizeof acc);
  for (int it = 0; it < n; ++it) {
    double tau[NJ], nd[18];
    memcpy(tau, tau_pd, sizeof tau);
    double dl[NJ];
    joint_limit_torque(m, c, s, c->implicit_penalty ? h : 0.0, h, tau, dl);
    orc_contact_report r;
    double nanc[2][H12_NFOOT_PTS][2];
    int32_t nmask = 0;
    memcpy(nanc, s->anchor, sizeof nanc);
    if (forward_dynamics(m, c, s, tau, algo, h, dl, with_contact, nd, &r, nanc, &nmask)) return -1;
    double* pa = (double*)&acc;
    const double* pr = (const double*)&r;
    for (size_t i = 0; i < sizeof acc / sizeof(double); ++i) pa[i] += pr[i] / n;
    integrate(s, nd, h, c->fix_base);
    limit_projection(m, c, s);
    memcpy(s->anchor, nanc, sizeof nanc);
    s->cmask = nmask;
  }
  if (rep) *rep = acc;
  return 0;
}

int orc_mujoco_rollout(const h12env_model* m, const h12env_config* c, orc_phys* s, const double* q_ref, int n_steps,
                       int with_contact, int algo, double* traj_q) {
  for (int t = 0; t < n_steps; ++t) {
    double tau[NJ];
    for (int j = 0; j < NJ; ++j) {
      double v = c->kp[j] * (q_ref[j] - s->q[j]) - c->kd[j] * s->qd[j];
      double lim = m->mj_frc_limit[j];
      tau[j] = v > lim ? lim : (v < -lim ? -lim : v);
    }
    if (orc_physics_step(m, c, s, tau, with_contact, algo, 0)) return -1;
    if (traj_q) memcpy(traj_q + (size_t)t * NJ, s->q, sizeof(double) * NJ);
  }
  return 0;
}

/* ------------------------------------------------------------------ MDP (IsaacLab semantics) */
typedef struct orc_env {
  orc_phys p;
  double act[NJ], act_prev[NJ], cmd[3], heading, cmd_time, air[2], con[2], last_air[2], last_con[2], epsum[H12_NREW];
  double push_t;
  double metric[2]; /* UniformVelocityCommand metrics error_vel_xy, error_vel_yaw */
  int eplen, lag[3], since_reset, is_heading, is_standing;
  double origin[3];
  int32_t tcell; /* terrain level | type << 16 */
} orc_env;

/* per-env startup parameters and terrain cell (fields used by the configured features only) */
static void env_load_extra(const h12env_config* c, const float* F, const int32_t* I, int n, int i, orc_env* e) {
  e->p.env_params = c->per_env_friction || c->per_env_mass;
  for (int f = 0; f < 2; ++f) {
    e->p.mu[f][0] = c->per_env_friction ? F[(size_t)(H12_F_MU + 2 * f) * n + i] : c->mu_static;
    e->p.mu[f][1] = c->per_env_friction ? F[(size_t)(H12_F_MU + 2 * f + 1) * n + i] : c->mu_dynamic;
  }
  e->p.dmass = c->per_env_mass ? F[(size_t)H12_F_DMASS * n + i] : 0.0;
  for (int a = 0; a < 3; ++a) e->origin[a] = c->terrain ? F[(size_t)(H12_F_ORIGIN + a) * n + i] : 0.0;
  e->tcell = (c->terrain && I) ? I[(size_t)H12_I_TERRAIN * n + i] : 0;
  /* stiction anchors are stored relative to the env origin (the kernel's env-local contact geometry) */
  for (int f = 0; f < 2; ++f)
    for (int q = 0; q < H12_NFOOT_PTS; ++q)
      for (int a = 0; a < 2; ++a) e->p.anchor[f][q][a] += e->origin[a];
}
static void env_store_extra(const h12env_config* c, float* F, int32_t* I, int n, int i, const orc_env* e) {
  if (!c->terrain) return;
  for (int f = 0; f < 2; ++f)
    for (int q = 0; q < H12_NFOOT_PTS; ++q)
      for (int a = 0; a < 2; ++a)
        F[(size_t)(H12_F_ANCHOR + 2 * H12_NFOOT_PTS * f + 2 * q + a) * n + i] = (float)(e->p.anchor[f][q][a] - e->origin[a]);
  for (int a = 0; a < 3; ++a) F[(size_t)(H12_F_ORIGIN + a) * n + i] = (float)e->origin[a];
  I[(size_t)H12_I_TERRAIN * n + i] = e->tcell;
}

static void env_load(const float* F, const int32_t* I, int n, int i, orc_env* e) {
#define LD(dst, fld, cnt) for (int a = 0; a < (cnt); ++a) (dst)[a] = F[(size_t)((fld) + a) * n + i]
  LD(e->p.pos, H12_F_POS, 3); LD(e->p.quat, H12_F_QUAT, 4); LD(e->p.vlin, H12_F_VLIN, 3);
  LD(e->p.wang, H12_F_WANG, 3); LD(e->p.q, H12_F_Q, NJ); LD(e->p.qd, H12_F_QD, NJ);
  LD(e->act, H12_F_ACT, NJ); LD(e->act_prev, H12_F_ACT_PREV, NJ); LD(e->cmd, H12_F_CMD, 3);
  LD(&e->heading, H12_F_HEADING, 1); LD(&e->cmd_time, H12_F_CMD_TIME, 1); LD(e->air, H12_F_AIR, 2);
  LD(e->con, H12_F_CONTACT, 2); LD(e->last_air, H12_F_LAST_AIR, 2); LD(e->last_con, H12_F_LAST_CONTACT, 2);
  LD(e->epsum, H12_F_EPSUM, H12_NREW_FLAT);
  LD(e->epsum + H12_NREW_FLAT, H12_F_EPSUM2, H12_NREW - H12_NREW_FLAT);
  LD(&e->push_t, H12_F_PUSH_TIME, 1);
  LD(e->metric, H12_F_METRIC, 2);
  LD(&e->p.anchor[0][0][0], H12_F_ANCHOR, 2 * H12_NFOOT_PTS * 2);
#undef LD
  e->eplen = I[(size_t)H12_I_EPLEN * n + i];
  int32_t pk = I[(size_t)H12_I_PACK * n + i];
  for (int g = 0; g < 3; ++g) e->lag[g] = (pk >> (3 * g)) & 7;
  e->since_reset = (pk >> 9) & 3;
  e->is_heading = (pk >> 11) & 1;
  e->is_standing = (pk >> 12) & 1;
  e->p.cmask = (pk >> 13) & 0xFF;
}
static void env_store(float* F, int32_t* I, int n, int i, const orc_env* e) {
#define ST(src, fld, cnt) for (int a = 0; a < (cnt); ++a) F[(size_t)((fld) + a) * n + i] = (float)(src)[a]
  ST(e->p.pos, H12_F_POS, 3); ST(e->p.quat, H12_F_QUAT, 4); ST(e->p.vlin, H12_F_VLIN, 3);
  ST(e->p.wang, H12_F_WANG, 3); ST(e->p.q, H12_F_Q, NJ); ST(e->p.qd, H12_F_QD, NJ);
  ST(e->act, H12_F_ACT, NJ); ST(e->act_prev, H12_F_ACT_PREV, NJ); ST(e->cmd, H12_F_CMD, 3);
  ST(&e->heading, H12_F_HEADING, 1); ST(&e->cmd_time, H12_F_CMD_TIME, 1); ST(e->air, H12_F_AIR, 2);
  ST(e->con, H12_F_CONTACT, 2); ST(e->last_air, H12_F_LAST_AIR, 2); ST(e->last_con, H12_F_LAST_CONTACT, 2);
  ST(e->epsum, H12_F_EPSUM, H12_NREW_FLAT);
  ST(e->epsum + H12_NREW_FLAT, H12_F_EPSUM2, H12_NREW - H12_NREW_FLAT);
  ST(&e->push_t, H12_F_PUSH_TIME, 1);
  ST(e->metric, H12_F_METRIC, 2);
  ST(&e->p.anchor[0][0][0], H12_F_ANCHOR, 2 * H12_NFOOT_PTS * 2);
#undef ST
  I[(size_t)H12_I_EPLEN * n + i] = e->eplen;
  int32_t pk = 0;
  for (int g = 0; g < 3; ++g) pk |= (e->lag[g] & 7) << (3 * g);
  pk |= (e->since_reset & 3) << 9;
  pk |= (e->is_heading & 1) << 11;
  pk |= (e->is_standing & 1) << 12;
  pk |= (e->p.cmask & 0xFF) << 13;
  I[(size_t)H12_I_PACK * n + i] = pk;
}

static double wrap_to_pi(double x) {
  double r = fmod(x, 2 * PI_D);
  if (r < 0) r += 2 * PI_D;
  return r > PI_D ? r - 2 * PI_D : r;
}
static double heading_w(const orc_phys* p) { /* atan2 of the body x axis in world */
  m3 R;
  quat_to_R(p->quat, R);
  return atan2(R[1][0], R[0][0]);
}

/* CommandTerm._resample: UniformVelocityCommand._resample_command (upstream; in-repo twin
 * utils/mdp/commands.py:19-59) and time_left ~ U(resampling_time_range).  blk: first Philox block. */
static void cmd_resample(const h12env_config* c, orc_env* e, int64_t g, uint32_t lo, uint32_t hi, int blk) {
  uint32_t r0[4], r1[4];
  rng_block(c->seed, g, lo, hi, ST_CMD, blk, r0);
  rng_block(c->seed, g, lo, hi, ST_CMD, blk + 1, r1);
  e->cmd[0] = uab(r0[0], c->cmd_lin_x[0], c->cmd_lin_x[1]);
  e->cmd[1] = uab(r0[1], c->cmd_lin_y[0], c->cmd_lin_y[1]);
  e->cmd[2] = uab(r0[2], c->cmd_ang_z[0], c->cmd_ang_z[1]);
  e->heading = uab(r0[3], c->cmd_heading[0], c->cmd_heading[1]);
  e->is_heading = (float)u01(r1[0]) <= c->rel_heading_envs;
  e->is_standing = (float)u01(r1[1]) <= c->rel_standing_envs;
  e->cmd_time = uab(r1[2], c->cmd_resample_time, c->cmd_resample_time_max);
}
/* UniformVelocityCommand._update_command given its decisions (utils/mdp/commands.py:83-138, the heading part
 * :89-101 being the twin of the Flat task's IsaacLab command): heading envs get
 * cmd_z = clip(stiffness * wrap_to_pi(heading - heading_w), ang_vel_z range); then, for the deadzone subclass,
 * deactivate -> cmd_xy = 0, flip -> cmd_z *= -1; the plain command zeroes standing envs.  Returns 1 when the
 * deadzone subclass asks for a resample of this env (activate). */
int orc_cmd_update_decided(const h12env_config* c, double cmd[3], double heading_target, const double quat[4],
                           int is_heading, int is_standing, int deactivate, int activate, int flip) {
  if (is_heading) {
    orc_phys p;
    memcpy(p.quat, quat, sizeof p.quat);
    double err = wrap_to_pi(heading_target - heading_w(&p));
    double w = c->heading_stiffness * err;
    cmd[2] = w < c->cmd_ang_z[0] ? c->cmd_ang_z[0] : (w > c->cmd_ang_z[1] ? c->cmd_ang_z[1] : w);
  }
  if (c->cmd_deadzone) {
    if (deactivate) cmd[0] = cmd[1] = 0;
    if (flip) cmd[2] = -cmd[2];
    return activate;
  }
  if (is_standing) cmd[0] = cmd[1] = cmd[2] = 0;
  return 0;
}

/* UniformVelocityCommand._update_command; with cmd_deadzone the Rsl/CaT subclass
 * (utils/mdp/commands.py:41-96): the reference picks exactly (target - count) of the active envs
 * (or (count - target) of the deadzone ones) by randperm; here each env draws the per-env marginal
 * of that choice, Bernoulli((target - count) / (n - count)) resp. Bernoulli((count - target) / count),
 * with the count of the previous step (dz_prev; exact for the shipped velocity_deadzone = 0, where the
 * count is always 0).  Then cmd_z *= -1 with probability ang_flip_prob.  No standing-env zeroing. */
static void cmd_update(const h12env_config* c, orc_env* e, int64_t g, uint32_t lo, uint32_t hi, int dz_prev, int n) {
  int deact = 0, act = 0, flip = 0;
  if (c->cmd_deadzone) {
    uint32_t r[4];
    rng_block(c->seed, g, lo, hi, ST_CMD, 2, r);
    int target = n / 2;
    double v = (double)c->velocity_deadzone;
    /* membership uses cmd_xy, which the heading law (run first in the reference) does not change */
    int in_dz = (float)e->cmd[0] * (float)e->cmd[0] + (float)e->cmd[1] * (float)e->cmd[1] < (float)(v * v);
    uint64_t u24 = r[0] >> 8;
    if (dz_prev < target) deact = !in_dz && u24 * (uint64_t)(n - dz_prev) < ((uint64_t)(target - dz_prev) << 24);
    else if (dz_prev > target) act = in_dz && u24 * (uint64_t)dz_prev < ((uint64_t)(dz_prev - target) << 24);
    flip = u01(r[1]) < (double)c->ang_flip_prob;
  }
  if (orc_cmd_update_decided(c, e->cmd, e->heading, e->p.quat, e->is_heading, e->is_standing, deact, act, 0)) {
    cmd_resample(c, e, g, lo, hi, 3);
  }
  if (flip) e->cmd[2] = -e->cmd[2];
}

/* push_by_setting_velocity interval event (EventManager.apply(mode="interval"), rsl_env_cfg.py:262-273) */
static void push_event(const h12env_config* c, orc_env* e, int64_t g, uint32_t lo, uint32_t hi, double step_dt) {
  if (!c->push_enable) return;
  e->push_t = (float)(e->push_t - step_dt);
  if (e->push_t < 1e-6) {
    uint32_t r[4];
    rng_block(c->seed, g, lo, hi, ST_PUSH, 0, r);
    e->push_t = uab(r[2], c->push_interval[0], c->push_interval[1]);
    e->p.vlin[0] += uab(r[0], c->push_vel_x[0], c->push_vel_x[1]);
    e->p.vlin[1] += uab(r[1], c->push_vel_y[0], c->push_vel_y[1]);
  }
}

/* terrain_levels_vel (velocity/mdp/curriculums.py:27-58): move up when the distance walked from the env origin
 * exceeds half the sub-terrain size, down when it is below half the commanded distance of an episode (and
 * not up) */
void orc_terrain_move(const h12env_config* c, const double pos[3], const double origin[3], const double cmd[3], int* up,
                      int* down) {
  double dx = pos[0] - origin[0], dy = pos[1] - origin[1];
  double dist = sqrt(dx * dx + dy * dy);
  double ep_s = c->max_episode_length * c->physics_dt * c->decimation;
  *up = dist > 0.5 * c->terrain_size;
  *down = !*up && dist < sqrt(cmd[0] * cmd[0] + cmd[1] * cmd[1]) * ep_s * 0.5;
}

/* _reset_idx: scene reset (delay lags, sensor), reset events, manager resets (cat_env.py:195-248) */
static void env_reset_one(const h12env_model* m, const h12env_config* c, orc_env* e, int64_t g, uint32_t lo,
                          uint32_t hi) {
  uint32_t r0[4], r1[4];
  rng_block(c->seed, g, lo, hi, ST_RESET, 0, r0);
  rng_block(c->seed, g, lo, hi, ST_RESET, 1, r1);
  if (c->terrain_curriculum && g_terrain.origins) {
    /* terrain_levels_vel (velocity/mdp/curriculums.py:21-52) on the pre-reset state, then
     * TerrainImporter.update_env_origins (solvers of the last level go to a random one) */
    int up, down;
    orc_terrain_move(c, e->p.pos, e->origin, e->cmd, &up, &down);
    int lvl = (e->tcell & 0xFFFF) + up - down, typ = e->tcell >> 16;
    if (lvl >= g_terrain.rows) {
      uint32_t r2[4];
      rng_block(c->seed, g, lo, hi, ST_RESET, 2, r2);
      lvl = (int)(r2[0] % (uint32_t)g_terrain.rows);
    }
    if (lvl < 0) lvl = 0;
    e->tcell = lvl | (typ << 16);
    const float* o = g_terrain.origins + 3 * ((size_t)lvl * g_terrain.cols + typ);
    for (int a = 0; a < 3; ++a) e->origin[a] = o[a];
  }
  /* keep the per-env startup parameters across the state reset */
  int32_t ep = e->p.env_params;
  double mu[2][2], dm = e->p.dmass;
  memcpy(mu, e->p.mu, sizeof mu);
  memset(&e->p, 0, sizeof e->p);
  e->p.env_params = ep;
  memcpy(e->p.mu, mu, sizeof mu);
  e->p.dmass = dm;
  /* cleared stiction anchors: 0 in the stored (origin-relative) frame */
  for (int f = 0; f < 2; ++f)
    for (int q = 0; q < H12_NFOOT_PTS; ++q)
      for (int a = 0; a < 2; ++a) e->p.anchor[f][q][a] = e->origin[a];
  e->p.pos[0] = e->origin[0] + (double)(float)uab(r0[0], c->reset_x[0], c->reset_x[1]);
  e->p.pos[1] = e->origin[1] + (double)(float)uab(r0[1], c->reset_y[0], c->reset_y[1]);
  e->p.pos[2] = e->origin[2] + m->root_height;
  double yaw = uab(r0[2], c->reset_yaw[0], c->reset_yaw[1]);
  e->p.quat[0] = cos(0.5 * (float)yaw);
  e->p.quat[3] = sin(0.5 * (float)yaw);
  for (int j = 0; j < NJ; ++j) {
    double q = m->q_default[j];
    double mid = 0.5 * (m->q_lower[j] + m->q_upper[j]), half = 0.5 * (m->q_upper[j] - m->q_lower[j]) * c->soft_limit_factor;
    if (q < mid - half) q = mid - half;
    if (q > mid + half) q = mid + half;
    e->p.q[j] = q;
  }
  int span = c->max_delay - c->min_delay + 1;
  e->lag[0] = c->min_delay + (int)(r0[3] % (uint32_t)span);
  e->lag[1] = c->min_delay + (int)(r1[0] % (uint32_t)span);
  e->lag[2] = c->min_delay + (int)(r1[1] % (uint32_t)span);
  e->since_reset = 0;
  memset(e->act, 0, sizeof e->act);
  memset(e->act_prev, 0, sizeof e->act_prev);
  memset(e->air, 0, sizeof e->air);
  memset(e->con, 0, sizeof e->con);
  memset(e->last_air, 0, sizeof e->last_air);
  memset(e->last_con, 0, sizeof e->last_con);
  memset(e->epsum, 0, sizeof e->epsum);
  memset(e->metric, 0, sizeof e->metric); /* CommandTerm.reset */
  e->eplen = 0;
  if (c->push_enable) { /* EventManager.reset: new interval for the reset envs */
    uint32_t r3[4];
    rng_block(c->seed, g, lo, hi, ST_RESET, 3, r3);
    e->push_t = uab(r3[0], c->push_interval[0], c->push_interval[1]);
  }
  cmd_resample(c, e, g, lo, hi, 0);
}

/* ObservationManager.compute_group per term (observation_manager.py:318-337): noise (Unoise: value + n_min +
 * (n_max - n_min) u, u the term's uniform draw), then scale.  raw: the 45 noise-free frame components (base_ang_vel,
 * projected_gravity, velocity_commands, joint_pos_rel, joint_vel_rel, last_action); u: the 30 draws of the noisy
 * components in order (commands and actions carry no noise). */
void orc_obs_frame_from(const h12env_config* c, const double raw[H12_OBS_FRAME], const double u[30],
                        double fr[H12_OBS_FRAME]) {
  for (int k = 0; k < H12_OBS_FRAME; ++k) fr[k] = raw[k];
  if (c->enable_corruption) {
    const int idx[30] = {0, 1, 2, 3, 4, 5, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20,
                         21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32};
    for (int t = 0; t < 30; ++t) {
      double nmax = t < 3 ? c->noise_ang_vel : t < 6 ? c->noise_gravity : t < 18 ? c->noise_joint_pos : c->noise_joint_vel;
      fr[idx[t]] += (double)(float)(-nmax + 2.0 * nmax * (double)(float)u[t]);
    }
  }
  /* ObsTerm scale, after noise (observation_manager.py:327-336) */
  for (int k2 = 0; k2 < H12_OBS_FRAME; ++k2) {
    int t = k2 < 9 ? k2 / 3 : 3 + (k2 - 9) / NJ;
    fr[k2] *= (double)c->obs_scale[t];
  }
}

/* observation frame (ObservationManager.compute_group, observation_manager.py:318-351) */
static void obs_frame(const h12env_model* m, const h12env_config* c, const orc_env* e, int64_t g, uint32_t lo,
                      uint32_t hi, double fr[H12_OBS_FRAME]) {
  m3 R;
  quat_to_R(e->p.quat, R);
  double gw[3] = {0, 0, -1}, gb[3];
  m3tv(R, gw, gb);
  double noise[32];
  for (int b = 0; b < 8; ++b) {
    uint32_t r[4];
    rng_block(c->seed, g, lo, hi, ST_OBS, b, r);
    for (int a = 0; a < 4; ++a) noise[4 * b + a] = u01(r[a]);
  }
  double raw[H12_OBS_FRAME];
  int k = 0;
  for (int a = 0; a < 3; ++a) raw[k++] = e->p.wang[a];
  for (int a = 0; a < 3; ++a) raw[k++] = gb[a];
  for (int a = 0; a < 3; ++a) raw[k++] = e->cmd[a];
  for (int j = 0; j < NJ; ++j) raw[k++] = e->p.q[j] - m->q_default[j];
  for (int j = 0; j < NJ; ++j) raw[k++] = e->p.qd[j];
  for (int j = 0; j < NJ; ++j) raw[k++] = e->act[j];
  orc_obs_frame_from(c, raw, noise, fr);
}
static const int TERM_DIM[6] = {3, 3, 3, NJ, NJ, NJ};
/* CircularBuffer append + buffer() flattening of a term-major row, nh frames per term (oldest first) */
static void obs_write(const double fr[H12_OBS_FRAME], const float* prev, float* out, int fill, int nh) {
  int off = 0, fo = 0;
  for (int t = 0; t < 6; ++t) {
    int d = TERM_DIM[t];
    for (int h = 0; h < nh; ++h)
      for (int a = 0; a < d; ++a) {
        double v;
        if (fill || h == nh - 1) v = fr[fo + a];
        else v = prev[off + (h + 1) * d + a];
        out[off + h * d + a] = (float)v;
      }
    off += d * nh;
    fo += d;
  }
}

/* root_lin_vel_w: the linear velocity of the root rigid body's COM (the pelvis body alone, model root_com;
 * IsaacLab ArticulationData.root_com_vel_w) in world axes */
static void base_com_vel(const h12env_model* m, const orc_phys* p, const m3 R, double vcom[3]) {
  (void)p->dmass;  /* the added torso mass sits on torso_link, another rigid body */
  const double c[3] = {m->root_com[0], m->root_com[1], m->root_com[2]};
  double wb[3] = {p->wang[0], p->wang[1], p->wang[2]}, ww[3], cw[3], wxc[3];
  m3v(R, wb, ww);
  m3v(R, c, cw);
  cross3(ww, cw, wxc);
  for (int a = 0; a < 3; ++a) vcom[a] = p->vlin[a] + wxc[a];
}

/* ObservationManager.compute_group of the rough policy group (observation_manager.py:318-337): per noisy
 * component t (all but velocity_commands and actions: 220) value + n_min + (n_max - n_min) u[t], then the
 * height scan's clip (velocity_env_cfg.py:133-137); no scales, no history. */
void orc_rough_row_from(const h12env_config* c, const double raw[H12_NOBS_ROUGH], const double u[H12_NOBS_ROUGH - 15],
                        float* out) {
  for (int kk = 0; kk < H12_NOBS_ROUGH; ++kk) {
    double v = raw[kk];
    int t = kk < 9 ? kk : ((kk >= 12 && kk < 36) ? kk - 3 : (kk >= H12_ROUGH_FRAME ? kk - 15 : -1));
    if (t >= 0 && c->enable_corruption) {
      double nmax = t < 3 ? c->noise_lin_vel : t < 6 ? c->noise_ang_vel : t < 9 ? c->noise_gravity
                  : t < 21 ? c->noise_joint_pos : t < 33 ? c->noise_joint_vel : c->noise_height_scan;
      v += (double)(float)(-nmax + 2.0 * nmax * (double)(float)u[t]);
    }
    if (kk >= H12_ROUGH_FRAME) v = v < -c->scan_clip ? -c->scan_clip : (v > c->scan_clip ? c->scan_clip : v);
    out[kk] = (float)v;
  }
}

/* Rough task observation row (velocity_env_cfg.py:118-137): base_lin_vel, base_ang_vel, projected_gravity,
 * velocity_commands, joint_pos_rel, joint_vel_rel, last_action, height_scan; noise then clip.  Height scan:
 * 17 x 11 rays at 0.1 m around the torso_link origin (= pelvis origin), yaw-aligned, x fastest;
 * value = sensor z - ground z - 0.5 (isaaclab mdp.height_scan). */
static void obs_row_rough(const h12env_model* m, const h12env_config* c, const orc_env* e, int64_t g, uint32_t lo,
                          uint32_t hi, float* out) {
  m3 R;
  quat_to_R(e->p.quat, R);
  double v[H12_NOBS_ROUGH];
  double vcom[3], vb[3], gw[3] = {0, 0, -1}, gb[3];
  base_com_vel(m, &e->p, R, vcom);
  m3tv(R, vcom, vb);
  m3tv(R, gw, gb);
  int k = 0;
  for (int a = 0; a < 3; ++a) v[k++] = vb[a];
  for (int a = 0; a < 3; ++a) v[k++] = e->p.wang[a];
  for (int a = 0; a < 3; ++a) v[k++] = gb[a];
  for (int a = 0; a < 3; ++a) v[k++] = e->cmd[a];
  for (int j = 0; j < NJ; ++j) v[k++] = e->p.q[j] - m->q_default[j];
  for (int j = 0; j < NJ; ++j) v[k++] = e->p.qd[j];
  for (int j = 0; j < NJ; ++j) v[k++] = e->act[j];
  double hx = R[0][0], hy = R[1][0], hn = sqrt(hx * hx + hy * hy), cy = hx / hn, sy = hy / hn;
  for (int iy = 0; iy < H12_SCAN_NY; ++iy)
    for (int ix = 0; ix < H12_SCAN_NX; ++ix) {
      double xl = c->scan_resolution * (ix - (H12_SCAN_NX - 1) / 2), yl = c->scan_resolution * (iy - (H12_SCAN_NY - 1) / 2);
      double gx, gy;
      double hz = orc_ground(c, e->p.pos[0] + cy * xl - sy * yl, e->p.pos[1] + sy * xl + cy * yl, &gx, &gy);
      v[k++] = e->p.pos[2] - hz - c->scan_offset;
    }
  double u[H12_NOBS_ROUGH - 15];
  for (int t = 0; t < H12_NOBS_ROUGH - 15; ++t) {
    uint32_t r[4];
    rng_block(c->seed, g, lo, hi, ST_OBS, t >> 2, r);
    u[t] = u01(r[t & 3]);
  }
  orc_rough_row_from(c, v, u, out);
}

/* DelayBuffer = CircularBuffer(max_delay + 1)[lag] (circular_buffer.py:139-170) with one push per
 * physics step and a constant target within an env step: the delayed target of substep s is the
 * target of env step t - src.  The first push after a reset fills the ring (:131-135), which the
 * clamp lag <= pushes - 1 reproduces. */
int orc_delay_source(int lag, int since_reset, int substep, int decimation) {
  int npush = since_reset * decimation + substep + 1;
  int L = lag > npush - 1 ? npush - 1 : lag;
  return L <= substep ? 0 : (L <= substep + decimation ? 1 : 2);
}

void orc_history_write(const double frame[H12_OBS_FRAME], const float* prev_row, float* out_row, int fill) {
  obs_write(frame, prev_row, out_row, fill, H12_NHIST);
}
void orc_history_write_n(const double frame[H12_OBS_FRAME], const float* prev_row, float* out_row, int fill, int nh) {
  obs_write(frame, prev_row, out_row, fill, nh);
}

/* ObservationManager.compute() outside step(): one new frame per env, history shifted (or filled
 * where fill_mask[i]); noise stream keyed by (env, counter, 0xFFFFFFFE). */
int orc_env_observe(const h12env_model* m, const h12env_config* c, int n, int64_t env_offset, float* F, int32_t* I,
                    const float* obs_prev, float* obs, const uint8_t* fill_mask, uint64_t counter) {
  uint32_t lo = (uint32_t)counter, hi = 0xFFFFFFFEu;
  for (int i = 0; i < n; ++i) {
    orc_env e;
    env_load(F, I, n, i, &e);
    env_load_extra(c, F, I, n, i, &e);
    if (c->task == H12_TASK_ROUGH) {
      obs_row_rough(m, c, &e, env_offset + i, lo, hi, obs + (size_t)i * H12_NOBS_ROUGH);
      continue;
    }
    double fr[H12_OBS_FRAME];
    const size_t row = (size_t)orc_obs_dim(c);
    obs_frame(m, c, &e, env_offset + i, lo, hi, fr);
    obs_write(fr, obs_prev + (size_t)i * row, obs + (size_t)i * row, fill_mask ? fill_mask[i] : 0, c->history_length);
  }
  return 0;
}

int orc_env_reset(const h12env_model* m, const h12env_config* c, int n, int64_t env_offset, float* F, int32_t* I,
                  const uint8_t* mask, float* obs, uint64_t reset_counter) {
  uint32_t lo = (uint32_t)reset_counter, hi = 0xFFFFFFFFu;
  for (int i = 0; i < n; ++i) {
    if (mask && !mask[i]) continue;
    orc_env e;
    env_load(F, I, n, i, &e); /* the pre-reset state feeds the terrain curriculum */
    env_load_extra(c, F, I, n, i, &e);
    int64_t g = env_offset + i;
    env_reset_one(m, c, &e, g, lo, hi);
    if (c->task == H12_TASK_ROUGH) {
      obs_row_rough(m, c, &e, g, lo, hi, obs + (size_t)i * H12_NOBS_ROUGH);
    } else {
      double fr[H12_OBS_FRAME];
      obs_frame(m, c, &e, g, lo, hi, fr);
      obs_write(fr, 0, obs + (size_t)i * orc_obs_dim(c), 1, c->history_length);
    }
    env_store(F, I, n, i, &e);
    env_store_extra(c, F, I, n, i, &e);
  }
  return 0;
}

static double sq(double x) { return x * x; }

/* The MDP terms of one env on its post-physics, pre-reset state (the code orc_env_step runs): the
 * time_out / illegal_contact terminations (velocity_env_cfg.py:264-268; bodies rough_env_cfg.py:95-109,
 * threshold 1 N on max_h |F| over net_forces_w_history) and the 20 reward terms of the kernel table (unweighted;
 * the Flat 12 of SURVEY.md a8.1-a8.12 + the Rsl extras).  Reference code among them:
 * feet_air_time_positive_biped (velocity/mdp/rewards.py:38-62), action_rate_l2 (utils/mdp/rewards.py:23-30). */
int orc_mdp_terms(const h12env_model* m, const h12env_config* c, const orc_term_in* in, double terms[H12_NREW],
                  int* terminated, int* time_out) {
  int tout = in->eplen >= c->max_episode_length;
  int term = 0;
  if (c->illegal_contact_knees && (in->fmax_knee[0] > c->contact_threshold || in->fmax_knee[1] > c->contact_threshold)) term = 1;
  if (c->illegal_contact_torso && in->fmax_torso > c->contact_threshold) term = 1;
  /* a diverged floating base terminates as well (round 6; the kernel's base_diverged: a component of the base's angular
   * velocity above 200 rad/s or of its linear velocity above 50 m/s, or not finite) -- no reference counterpart: PhysX
   * does not blow up where the penalty contacts can */
  for (int a = 0; a < 3; ++a)
    if (!(fabs((double)in->p.wang[a]) <= 200.0) || !(fabs((double)in->p.vlin[a]) <= 50.0)) term = 1;
  /* rewards (pre-reset state) */
  m3 R;
  quat_to_R(in->p.quat, R);
  double wb[3] = {in->p.wang[0], in->p.wang[1], in->p.wang[2]}, ww[3];
  m3v(R, wb, ww);
  double gw[3] = {0, 0, -1}, gb[3];
  m3tv(R, gw, gb);
  double vcom[3];
  base_com_vel(m, &in->p, R, vcom);
  double yaw = atan2(R[1][0], R[0][0]);
  double cy = cos(yaw), sy = sin(yaw);
  double vy0 = cy * vcom[0] + sy * vcom[1], vy1 = -sy * vcom[0] + cy * vcom[1];
  double std2 = c->track_std * c->track_std;
  terms[H12_R_TRACK_LIN_VEL_XY] = exp(-(sq(in->cmd[0] - vy0) + sq(in->cmd[1] - vy1)) / std2);
  terms[H12_R_TRACK_ANG_VEL_Z] = exp(-sq(in->cmd[2] - ww[2]) / std2);
  terms[H12_R_ANG_VEL_XY_L2] = sq(wb[0]) + sq(wb[1]);
  double s_t = 0, s_a = 0, s_r = 0, s_lim = 0, s_dev = 0;
  for (int j = 0; j < NJ; ++j) {
    s_t += sq(in->tau[j]);
    s_a += sq(in->jacc[j]);
    s_r += sq(in->act[j] - in->act_prev[j]);
  }
  terms[H12_R_DOF_TORQUES_L2] = s_t;
  terms[H12_R_DOF_ACC_L2] = s_a;
  terms[H12_R_ACTION_RATE_L2] = s_r;
  /* feet_air_time_positive_biped (mdp/rewards.py:38-62) */
  {
    int inc[2] = {in->con[0] > 0, in->con[1] > 0};
    double mode_t[2] = {inc[0] ? in->con[0] : in->air[0], inc[1] ? in->con[1] : in->air[1]};
    int single = (inc[0] + inc[1]) == 1;
    double r = single ? (mode_t[0] < mode_t[1] ? mode_t[0] : mode_t[1]) : 0.0;
    if (r > c->air_time_threshold) r = c->air_time_threshold;
    double cn = sqrt(sq(in->cmd[0]) + sq(in->cmd[1]));
    terms[H12_R_FEET_AIR_TIME] = cn > 0.1 ? r : 0.0;
  }
  terms[H12_R_FLAT_ORIENTATION_L2] = sq(gb[0]) + sq(gb[1]);
  for (int f = 0; f < 2; ++f)
    for (int k = 4; k < 6; ++k) { /* ankle pitch, ankle roll */
      int j = 6 * f + k;
      double mid = 0.5 * (m->q_lower[j] + m->q_upper[j]), half = 0.5 * (m->q_upper[j] - m->q_lower[j]) * c->soft_limit_factor;
      double lo_s = mid - half, hi_s = mid + half, q = in->p.q[j];
      s_lim += (q < lo_s ? lo_s - q : 0.0) + (q > hi_s ? q - hi_s : 0.0);
    }
  terms[H12_R_DOF_POS_LIMITS] = s_lim;
  terms[H12_R_TERMINATION] = term ? 1.0 : 0.0;
  {
    /* feet_slide: |v_xy| of the ankle-roll link COM where max_h |F| > 1 */
    kin_t k;
    kinematics(m, &in->p, &k);
    double fs = 0;
    for (int f = 0; f < 2; ++f) {
      int b = 6 * f + 6;
      if (!(in->fmax_foot[f] > 1.0)) continue;
      double cl[3] = {m->link_com[b - 1][0], m->link_com[b - 1][1], m->link_com[b - 1][2]}, vl[3], vw[3];
      cross3(k.v[b], cl, vl);
      for (int a = 0; a < 3; ++a) vl[a] += k.v[b][3 + a];
      m3v(k.R[b], vl, vw);
      fs += sqrt(sq(vw[0]) + sq(vw[1]));
    }
    terms[H12_R_FEET_SLIDE] = fs;
  }
  for (int f = 0; f < 2; ++f) {
    int j0 = 6 * f + 0, j2 = 6 * f + 2; /* hip yaw, hip roll */
    s_dev += fabs(in->p.q[j0] - m->q_default[j0]) + fabs(in->p.q[j2] - m->q_default[j2]);
  }
  terms[H12_R_JOINT_DEV_HIP] = s_dev;
  /* Rsl table (rsl_env_cfg.py:279-407) */
  {
    double vb[3];
    m3tv(R, vcom, vb); /* root_lin_vel_b */
    terms[H12_R_TRACK_LIN_VEL_XY_BASE] = exp(-(sq(in->cmd[0] - vb[0]) + sq(in->cmd[1] - vb[1])) / std2);
    terms[H12_R_TRACK_ANG_VEL_Z_BASE] = exp(-sq(in->cmd[2] - wb[2]) / std2);
    terms[H12_R_BASE_HEIGHT_L2] = sq(in->p.pos[2] - c->base_height_target);
    double s_v = 0, s_da = 0, s_lh = 0, s_cf = 0;
    for (int j = 0; j < NJ; ++j) s_v += sq(in->p.qd[j]);
    for (int f = 0; f < 2; ++f) {
      for (int k = 4; k < 6; ++k) s_da += fabs(in->p.q[6 * f + k] - m->q_default[6 * f + k]);
      for (int k = 0; k < 3; k += 2) { /* hip yaw, hip roll soft limits */
        int j = 6 * f + k;
        double mid = 0.5 * (m->q_lower[j] + m->q_upper[j]), half = 0.5 * (m->q_upper[j] - m->q_lower[j]) * c->soft_limit_factor;
        double lo_s = mid - half, hi_s = mid + half, q = in->p.q[j];
        s_lh += (q < lo_s ? lo_s - q : 0.0) + (q > hi_s ? q - hi_s : 0.0);
      }
      double viol = in->fmax_foot[f] - c->contact_force_threshold;
      s_cf += viol > 0 ? viol : 0.0;
    }
    terms[H12_R_JOINT_VEL_L2] = s_v;
    terms[H12_R_JOINT_DEV_ANKLE] = s_da;
    terms[H12_R_DOF_POS_LIMITS_HIP] = s_lh;
    terms[H12_R_CONTACT_FORCES] = s_cf;
    terms[H12_R_LIN_VEL_Z_L2] = sq(vb[2]);
  }
  if (terminated) *terminated = term;
  if (time_out) *time_out = tout;
  return 0;
}

/* ---------------------------------------------------------------- CaT (T/utils/cat, cat_env_cfg.py) */
enum { CAT_ROW_NOMOVE = H12_NCSTR_COLS, CAT_ROW_EPLEN = H12_NCSTR_COLS + 1, CAT_ROWS = H12_NCSTR_COLS + 2 };
static const int C_COL0[H12_NCSTR + 1] = {0, 1, 13, 25, 37, 39, 51, 52, 53, 54, 56};
/* CaT.running_maxes, carried from one orc_env_step to the next (process-global, like the kernel's buffer) */
static double g_crun[H12_NCSTR_COLS];
static int g_crun_init = 0;
static double* g_cs_last = NULL;  /* the last step's raw constraints [CAT_ROWS][n] (tests) */
static int g_cs_n = 0;
void orc_cat_reset(void) { g_crun_init = 0; }
int orc_cat_last_constraints(double* out, int n) {
  if (!g_cs_last || n != g_cs_n) return -1;
  memcpy(out, g_cs_last, sizeof(double) * (size_t)CAT_ROWS * (size_t)n);
  return 0;
}
void orc_cat_running_max(double out[H12_NCSTR_COLS]) { memcpy(out, g_crun, sizeof g_crun); }

/* constraints.py:24-308 for one env on its pre-reset state (the ten terms of cat_env_cfg.py:336-425):
 * joint_position_limits :24-33, joint_velocity_limits :36-44, joint_torque_limits :47-55, contact :86-99
 * (= the illegal-contact termination: same bodies, same 1 N test), base_orientation :102-108, no_move :196-228
 * (raw |qd| - limit of THIS env; the repeat-remap over still envs is orc_cat_probs'), base_height :251-266,
 * foot_contact :171-193, foot_clearance :269-308 (swing_h = swing_max_height in/out), foot_contact_force
 * :161-168; plus the still flag of no_move (all |cmd| < deadzone) and the episode length.
 * out[col * stride], col in 0 .. H12_NCSTR_COLS + 1. */
int orc_cat_row(const h12env_model* m, const h12env_config* c, const orc_term_in* in, int terminated,
                double swing_h[2], double* out, size_t stride) {
#define CS(col) out[(size_t)(col) * stride]
  const double step_dt = c->physics_dt * c->decimation;
  for (int j = 0; j < NJ; ++j) {
    double mid = 0.5 * (m->q_lower[j] + m->q_upper[j]), half = 0.5 * (m->q_upper[j] - m->q_lower[j]) * c->soft_limit_factor;
    double q = in->p.q[j], qd = fabs(in->p.qd[j]);
    double lo_v = (mid - half) - q, hi_v = q - (mid + half);
    CS(C_COL0[H12_C_JOINT_POS_LIMITS] + j) = lo_v > hi_v ? lo_v : hi_v;
    CS(C_COL0[H12_C_JOINT_VEL_LIMITS] + j) = qd - c->cstr_joint_vel_limit[j];
    CS(C_COL0[H12_C_JOINT_TORQUE_LIMITS] + j) = fabs(in->tau[j]) - c->cstr_joint_effort_limit[j];
    CS(C_COL0[H12_C_NO_MOVE] + j) = qd - c->cstr_nomove_vel;
  }
  kin_t k;
  kinematics(m, &in->p, &k);
  m3 R;
  quat_to_R(in->p.quat, R);
  double gw[3] = {0, 0, -1}, gb[3];
  m3tv(R, gw, gb);
  int active = fabs(in->cmd[0]) > c->cstr_clearance_deadzone || fabs(in->cmd[1]) > c->cstr_clearance_deadzone ||
               fabs(in->cmd[2]) > c->cstr_clearance_deadzone;
  int nfeet = 0;
  for (int f = 0; f < 2; ++f) {
    CS(C_COL0[H12_C_FOOT_CONTACT_FORCE] + f) = in->fmax_foot[f] - c->cstr_foot_force_limit;
    nfeet += in->fmax_foot[f] > 1.0;
    /* foot_clearance: touchdown = compute_first_contact(step_dt); swing max height of the ankle-roll link */
    int touchdown = in->con[f] > 0 && in->con[f] < step_dt + 1e-8;
    double sh = swing_h[f], foot_z = k.p[6 * f + 6][2];
    CS(C_COL0[H12_C_FOOT_CLEARANCE] + f) = (touchdown && active) ? c->cstr_clearance_min - sh : 0.0;
    swing_h[f] = touchdown ? 0.0 : (foot_z > sh ? foot_z : sh);
  }
  CS(C_COL0[H12_C_CONTACT]) = terminated ? 1.0 : 0.0;
  CS(C_COL0[H12_C_BASE_ORIENTATION]) = sqrt(sq(gb[0]) + sq(gb[1])) - c->cstr_orient_limit;
  double z = in->p.pos[2];
  CS(C_COL0[H12_C_BASE_HEIGHT]) = (z < c->cstr_height - c->cstr_height_std || z > c->cstr_height + c->cstr_height_std) ? 1.0 : 0.0;
  CS(C_COL0[H12_C_FOOT_CONTACT]) = (nfeet < 1 || nfeet > 2) ? 1.0 : 0.0;
  double dz = c->cstr_nomove_deadzone;
  CS(CAT_ROW_NOMOVE) = (fabs(in->cmd[0]) < dz && fabs(in->cmd[1]) < dz && fabs(in->cmd[2]) < dz) ? 1.0 : 0.0;
  CS(CAT_ROW_EPLEN) = in->eplen;
#undef CS
  return 0;
}

/* CaT.add / get_probs over the batch (constraint_manager.py:40-82) with no_move's row remap
 * (constraints.py:214-228: env i takes the row of the (i mod m)-th still env, zeros when none):
 * column maxima clamped at 1e-6, running maxima (Polyak tau; the first call sets them), per-term
 * probabilities min_p + clamp(c / running_max, 0, 1) (max_p - min_p) where c > 0, their max over terms.
 * cs is [CAT_ROWS][n]; pterm [H12_NCSTR][n] and ceff [H12_NCSTR_COLS][n] (the values CaT.add saw) may be NULL. */
int orc_cat_probs(const h12env_config* c, int n, const double* cs, double run_max[H12_NCSTR_COLS], int* run_init,
                  double* pmax, double* pterm, double* ceff) {
  int* list = (int*)malloc(sizeof(int) * (size_t)(n > 0 ? n : 1));
  if (!list) return -1;
  int mcount = 0;
  for (int i = 0; i < n; ++i)
    if (cs[(size_t)CAT_ROW_NOMOVE * n + i] != 0) list[mcount++] = i;
  for (int col = 0; col < H12_NCSTR_COLS; ++col) {
    int nm = col >= C_COL0[H12_C_NO_MOVE] && col < C_COL0[H12_C_NO_MOVE + 1];
    double cm = -1e300;
    if (nm) {
      if (mcount == 0) cm = 0.0;
      for (int a = 0; a < mcount; ++a) { double v = cs[(size_t)col * n + list[a]]; if (v > cm) cm = v; }
    } else {
      for (int i = 0; i < n; ++i) { double v = cs[(size_t)col * n + i]; if (v > cm) cm = v; }
    }
    if (cm < 1e-6) cm = 1e-6;
    run_max[col] = *run_init ? c->cat_tau * run_max[col] + (1.0 - (double)c->cat_tau) * cm : cm;
  }
  *run_init = 1;
  for (int i = 0; i < n; ++i) {
    int src = mcount > 0 ? list[i % mcount] : -1;
    double pm = 0;
    for (int t = 0; t < H12_NCSTR; ++t) {
      double pt = 0;
      for (int col = C_COL0[t]; col < C_COL0[t + 1]; ++col) {
        double v = t == H12_C_NO_MOVE ? (src >= 0 ? cs[(size_t)col * n + src] : 0.0) : cs[(size_t)col * n + i];
        if (ceff) ceff[(size_t)col * n + i] = v;
        if (!((c->cstr_mask >> t) & 1u)) continue;
        double p = 0;
        if (v > 0) {
          double r = v / run_max[col];
          r = r < 0 ? 0 : (r > 1 ? 1 : r);
          p = c->cat_min_p + r * (c->cstr_max_p[t] - c->cat_min_p);
        }
        if (p > pt) pt = p;
      }
      if (pterm) pterm[(size_t)t * n + i] = pt;
      if (pt > pm) pm = pt;
    }
    pmax[i] = pm;
  }
  free(list);
  return 0;
}

/* ConstraintManager.compute + CaTEnv.step's use of it (constraint_manager.py:42-78, 222-237; cat_env.py:148-153,
 * 164-166) over the whole batch: column maxima (no_move: env i takes the row of the (i mod m)-th still env),
 * running maxima, probabilities, reward scaling, dones, episode statistics. */
/* ConstraintManager statistics (constraint_manager.py:221-227) and their reset (:195-210): per term the episode
 * sums of [p_term > 0] and of p_term; at a reset the env adds sum / episode_length to the log accumulator
 * (log_acc[H12_NREW + 4 + t]: violations, [H12_NREW + 4 + H12_NCSTR + t]: probabilities; the host divides by
 * the number of reset envs, x 100 for violations) and its sums restart.  sum_v / sum_p are [H12_NCSTR][n]. */
void orc_cat_stats(const h12env_config* c, int n, const double* pterm, const double* eplen, const uint8_t* reset,
                   float* sum_v, float* sum_p, float* log_acc) {
  for (int i = 0; i < n; ++i)
    for (int t = 0; t < H12_NCSTR; ++t) {
      if (!((c->cstr_mask >> t) & 1u)) continue;
      double pt = pterm[(size_t)t * n + i];
      float* fs = &sum_v[(size_t)t * n + i];
      float* fp = &sum_p[(size_t)t * n + i];
      double vs = *fs + (pt > 0 ? 1.0 : 0.0), vp = *fp + pt;
      if (reset[i]) {
        if (log_acc) {
          log_acc[H12_NREW + 4 + t] += (float)(vs / eplen[i]);
          log_acc[H12_NREW + 4 + H12_NCSTR + t] += (float)(vp / eplen[i]);
        }
        vs = vp = 0;
      }
      *fs = (float)vs;
      *fp = (float)vp;
    }
}

static void cat_pass(const h12env_config* c, int n, float* F, const double* cs, float* rew, const uint8_t* terminated,
                     const uint8_t* truncated, float* cstr_prob, float* log_acc) {
  const size_t nn = (size_t)(n > 0 ? n : 1);
  double* pmax = (double*)malloc(sizeof(double) * nn);
  double* pterm = (double*)malloc(sizeof(double) * (size_t)H12_NCSTR * nn);
  uint8_t* reset = (uint8_t*)malloc(nn);
  orc_cat_probs(c, n, cs, g_crun, &g_crun_init, pmax, pterm, NULL);
  for (int i = 0; i < n; ++i) {
    rew[i] = (float)(rew[i] * (1.0 - pmax[i]));
    reset[i] = terminated[i] || truncated[i];
    if (cstr_prob) cstr_prob[i] = reset[i] ? 1.0f : (float)pmax[i];
  }
  /* the workspace keeps the sums field-major: [H12_NCSTR][n] from H12_F_CSTR_SUM / H12_F_CSTR_P */
  orc_cat_stats(c, n, pterm, cs + (size_t)CAT_ROW_EPLEN * n, reset, F + (size_t)H12_F_CSTR_SUM * n,
                F + (size_t)H12_F_CSTR_P * n, log_acc);
  free(pmax);
  free(pterm);
  free(reset);
}

int orc_env_step(const h12env_model* m, const h12env_config* c, int n, int64_t env_offset, float* F, int32_t* I,
                 const float* actions, const float* obs_prev, float* obs, float* rew, uint8_t* terminated,
                 uint8_t* truncated, float* log_acc, float* applied_torque, float* foot_force, float* cstr_prob,
                 int64_t step_index, int n_threads) {
  const uint32_t lo = (uint32_t)step_index, hi = (uint32_t)((uint64_t)step_index >> 32);
  const int dec = c->decimation;
  const double dt = c->physics_dt, step_dt = c->physics_dt * dec;
  const int dz_prev = g_dz_count;
  int dz_next = 0;
  int err = 0;
  double* cs = c->cat_enable ? (double*)calloc((size_t)CAT_ROWS * (size_t)n, sizeof(double)) : NULL;
#ifdef _OPENMP
  if (n_threads < 1) n_threads = 1;
#pragma omp parallel for num_threads(n_threads) schedule(static)
#endif
  for (int i = 0; i < n; ++i) {
    orc_env e;
    env_load(F, I, n, i, &e);
    env_load_extra(c, F, I, n, i, &e);
    const int64_t g = env_offset + i;
    double a_t[NJ], a_t1[NJ], a_t2[NJ];
    for (int j = 0; j < NJ; ++j) {
      a_t[j] = actions[(size_t)i * NJ + j];
      a_t1[j] = e.act[j];
      a_t2[j] = e.act_prev[j];
    }
    /* ActionManager.process_action: prev_action <- action; action <- a */
    memcpy(e.act_prev, e.act, sizeof e.act);
    memcpy(e.act, a_t, sizeof a_t);
    double tau_applied[NJ] = {0}, jacc[NJ] = {0};
    double fmax_knee[2] = {0, 0}, fmax_torso = 0, fmax_foot[2] = {0, 0}, flast_foot[2] = {0, 0};
    for (int s = 0; s < dec; ++s) {
      double tau[NJ];
      if (c->mode == H12_MODE_ISAACLAB) {
        /* DelayedPDActuator.compute: delay buffer read at lag (clamped to pushes-1) */
        for (int j = 0; j < NJ; ++j) {
          int src = orc_delay_source(e.lag[c->delay_group[j]], e.since_reset, s, dec);
          double a = src == 0 ? a_t[j] : (src == 1 ? a_t1[j] : a_t2[j]);
          double tgt = m->q_default[j] + c->action_scale * (double)(float)a;
          double v = c->kp[j] * (tgt - e.p.q[j]) + c->kd[j] * (0.0 - e.p.qd[j]);
          double E = c->effort_limit[j];
          tau[j] = v > E ? E : (v < -E ? -E : v);
        }
      } else {
        for (int j = 0; j < NJ; ++j) {
          double tgt = m->q_default[j] + c->action_scale * a_t[j];
          double v = c->kp[j] * (tgt - e.p.q[j]) - c->kd[j] * e.p.qd[j];
          double E = m->mj_frc_limit[j];
          tau[j] = v > E ? E : (v < -E ? -E : v);
        }
      }
      double qd0[NJ];
      memcpy(qd0, e.p.qd, sizeof qd0);
      orc_contact_report rep;
      if (orc_physics_step(m, c, &e.p, tau, 1, 1, &rep)) err = -1;
      memcpy(tau_applied, tau, sizeof tau);
      for (int j = 0; j < NJ; ++j) jacc[j] = (e.p.qd[j] - qd0[j]) / dt;
      /* ContactSensor._update_buffers_impl: air / contact time (history 3, threshold 1 N) */
      for (int f = 0; f < 2; ++f) {
        double fn = sqrt(sq(rep.foot_force[f][0]) + sq(rep.foot_force[f][1]) + sq(rep.foot_force[f][2]));
        int is_c = fn > c->contact_threshold;
        int first_c = (e.air[f] > 0) && is_c;
        int first_d = (e.con[f] > 0) && !is_c;
        if (first_c) e.last_air[f] = e.air[f] + dt;
        e.air[f] = is_c ? 0.0 : e.air[f] + dt;
        if (first_d) e.last_con[f] = e.con[f] + dt;
        e.con[f] = is_c ? e.con[f] + dt : 0.0;
        flast_foot[f] = fn;
        if (s >= dec - 3 && fn > fmax_foot[f]) fmax_foot[f] = fn;
      }
      if (s >= dec - 3) {
        for (int f = 0; f < 2; ++f) {
          double fk = sqrt(sq(rep.knee_force[f][0]) + sq(rep.knee_force[f][1]) + sq(rep.knee_force[f][2]));
          if (fk > fmax_knee[f]) fmax_knee[f] = fk;
        }
        double ft = sqrt(sq(rep.torso_force[0]) + sq(rep.torso_force[1]) + sq(rep.torso_force[2]));
        if (ft > fmax_torso) fmax_torso = ft;
      }
    }
    e.eplen += 1;
    orc_term_in ti;
    ti.p = e.p;
    memcpy(ti.act, e.act, sizeof ti.act);
    memcpy(ti.act_prev, e.act_prev, sizeof ti.act_prev);
    memcpy(ti.cmd, e.cmd, sizeof ti.cmd);
    memcpy(ti.air, e.air, sizeof ti.air);
    memcpy(ti.con, e.con, sizeof ti.con);
    memcpy(ti.tau, tau_applied, sizeof ti.tau);
    memcpy(ti.jacc, jacc, sizeof ti.jacc);
    memcpy(ti.fmax_foot, fmax_foot, sizeof ti.fmax_foot);
    memcpy(ti.fmax_knee, fmax_knee, sizeof ti.fmax_knee);
    ti.fmax_torso = fmax_torso;
    ti.eplen = e.eplen;
    double terms[H12_NREW];
    int term, tout;
    orc_mdp_terms(m, c, &ti, terms, &term, &tout);
    double r = 0;
    for (int t = 0; t < H12_NREW; ++t) {
      double v = terms[t] * c->rew_w[t] * step_dt;
      r += v;
      e.epsum[t] += v;
    }
    rew[i] = (float)r;
    if (cs) {
      double sw[2] = {F[(size_t)H12_F_SWING_H * n + i], F[(size_t)(H12_F_SWING_H + 1) * n + i]};
      orc_cat_row(m, c, &ti, term, sw, cs + i, (size_t)n);
      F[(size_t)H12_F_SWING_H * n + i] = (float)sw[0];
      F[(size_t)(H12_F_SWING_H + 1) * n + i] = (float)sw[1];
    }
    terminated[i] = (uint8_t)term;
    truncated[i] = (uint8_t)tout;
    if (applied_torque) for (int j = 0; j < NJ; ++j) applied_torque[(size_t)i * NJ + j] = (float)tau_applied[j];
    if (foot_force) { foot_force[2 * i] = (float)flast_foot[0]; foot_force[2 * i + 1] = (float)flast_foot[1]; }
    int reset = term || tout;
    if (reset) {
      if (log_acc) {
#ifdef _OPENMP
#pragma omp critical
#endif
        {
          for (int t = 0; t < H12_NREW; ++t) log_acc[t] += (float)e.epsum[t];
          log_acc[H12_NREW] += 1.0f;
          log_acc[H12_NREW + 1] += (float)tout;
          log_acc[H12_NREW + 2] += (float)term;
          /* CommandTerm.reset: the ended episode's command metrics (mean over the reset envs on the host) */
          log_acc[H12_LOG_METRIC] += (float)e.metric[0];
          log_acc[H12_LOG_METRIC + 1] += (float)e.metric[1];
        }
      }
      env_reset_one(m, c, &e, g, lo, hi);
    } else {
      e.since_reset = e.since_reset < 2 ? e.since_reset + 1 : 2;
    }
    /* CommandTerm.compute(dt): UniformVelocityCommand._update_metrics on the post-reset state (IsaacLab 2.1:
     * |v*_xy - root_lin_vel_b,xy| and |w*_z - root_ang_vel_b,z| over max_command_step =
     * resampling_time_range[1] / step_dt), then the resampling clock */
    {
      m3 R;
      quat_to_R(e.p.quat, R);
      double vcom[3], vb[3];
      base_com_vel(m, &e.p, R, vcom);
      m3tv(R, vcom, vb);
      const double mcs = c->cmd_resample_time_max / step_dt;
      e.metric[0] += sqrt(sq(e.cmd[0] - vb[0]) + sq(e.cmd[1] - vb[1])) / mcs;
      e.metric[1] += fabs(e.cmd[2] - e.p.wang[2]) / mcs;
    }
    e.cmd_time = (float)(e.cmd_time - step_dt);
    if (e.cmd_time <= 0) cmd_resample(c, &e, g, lo, hi, 0);
    cmd_update(c, &e, g, lo, hi, dz_prev, n);
    if (c->cmd_deadzone && (float)e.cmd[0] * (float)e.cmd[0] + (float)e.cmd[1] * (float)e.cmd[1] <
                               (float)((double)c->velocity_deadzone * c->velocity_deadzone)) {
#ifdef _OPENMP
#pragma omp atomic
#endif
      dz_next++;
    }
    /* interval events */
    push_event(c, &e, g, lo, hi, step_dt);
    if (c->task == H12_TASK_ROUGH) {
      obs_row_rough(m, c, &e, g, lo, hi, obs + (size_t)i * H12_NOBS_ROUGH);
    } else {
      double fr[H12_OBS_FRAME];
      const size_t row = (size_t)orc_obs_dim(c);
      obs_frame(m, c, &e, g, lo, hi, fr);
      obs_write(fr, obs_prev + (size_t)i * row, obs + (size_t)i * row, reset, c->history_length);
    }
    env_store(F, I, n, i, &e);
    env_store_extra(c, F, I, n, i, &e);
  }
  if (c->cmd_deadzone) g_dz_count = dz_next;
  if (cs) {
    cat_pass(c, n, F, cs, rew, terminated, truncated, cstr_prob, log_acc);
    free(g_cs_last);
    g_cs_last = cs;
    g_cs_n = n;
  }
  return err;
}

int orc_env_step_physics(const h12env_model* m, const h12env_config* c, int n, float* F, int32_t* I,
                         const float* q_ref, int n_substeps) {
  for (int i = 0; i < n; ++i) {
    orc_env e;
    memset(&e, 0, sizeof e);
    int32_t pk = I ? I[(size_t)H12_I_PACK * n + i] : 0;
    int32_t cm = (pk >> 13) & 0xFF;
    int32_t* cmask = &cm;
    /* only physics fields are used */
    for (int a = 0; a < 3; ++a) e.p.pos[a] = F[(size_t)(H12_F_POS + a) * n + i];
    for (int a = 0; a < 4; ++a) e.p.quat[a] = F[(size_t)(H12_F_QUAT + a) * n + i];
    for (int a = 0; a < 3; ++a) e.p.vlin[a] = F[(size_t)(H12_F_VLIN + a) * n + i];
    for (int a = 0; a < 3; ++a) e.p.wang[a] = F[(size_t)(H12_F_WANG + a) * n + i];
    for (int j = 0; j < NJ; ++j) { e.p.q[j] = F[(size_t)(H12_F_Q + j) * n + i]; e.p.qd[j] = F[(size_t)(H12_F_QD + j) * n + i]; }
    for (int a = 0; a < 16; ++a) (&e.p.anchor[0][0][0])[a] = F[(size_t)(H12_F_ANCHOR + a) * n + i];
    e.p.cmask = *cmask;
    env_load_extra(c, F, I, n, i, &e);
    for (int t = 0; t < n_substeps; ++t) {
      double tau[NJ];
      for (int j = 0; j < NJ; ++j) {
        double v = c->kp[j] * (q_ref[(size_t)i * NJ + j] - e.p.q[j]) - c->kd[j] * e.p.qd[j];
        double E = c->mode == H12_MODE_MUJOCO ? m->mj_frc_limit[j] : c->effort_limit[j];
        tau[j] = v > E ? E : (v < -E ? -E : v);
      }
      if (orc_physics_step(m, c, &e.p, tau, 1, 1, 0)) return -1;
    }
    for (int a = 0; a < 3; ++a) F[(size_t)(H12_F_POS + a) * n + i] = (float)e.p.pos[a];
    for (int a = 0; a < 4; ++a) F[(size_t)(H12_F_QUAT + a) * n + i] = (float)e.p.quat[a];
    for (int a = 0; a < 3; ++a) F[(size_t)(H12_F_VLIN + a) * n + i] = (float)e.p.vlin[a];
    for (int a = 0; a < 3; ++a) F[(size_t)(H12_F_WANG + a) * n + i] = (float)e.p.wang[a];
    for (int j = 0; j < NJ; ++j) { F[(size_t)(H12_F_Q + j) * n + i] = (float)e.p.q[j]; F[(size_t)(H12_F_QD + j) * n + i] = (float)e.p.qd[j]; }
    for (int f = 0; f < 2; ++f)
      for (int q = 0; q < H12_NFOOT_PTS; ++q)
        for (int a = 0; a < 2; ++a)
          F[(size_t)(H12_F_ANCHOR + 2 * H12_NFOOT_PTS * f + 2 * q + a) * n + i] = (float)(e.p.anchor[f][q][a] - e.origin[a]);
    if (I) I[(size_t)H12_I_PACK * n + i] = (pk & ~(0xFF << 13)) | ((e.p.cmask & 0xFF) << 13);
  }
  return 0;
}
