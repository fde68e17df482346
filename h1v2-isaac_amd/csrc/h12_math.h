// h12_math.h — fp32 device helpers for the H1-2 env kernels (CDNA4 / gfx950).
//
// Spatial-vector conventions (Featherstone): motion m = (w; v), force f = (n; f), 6-vectors with the
// angular part first.  Every H1-2 leg joint turns about a coordinate axis of its parent frame and
// carries no fixed rotation (MJCF h12_12dof.xml:71-134), so every per-link transform is "rotate about
// axis A by q, then shift by r" and all rotations below are templated on the axis.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define H12_DEV __device__ __forceinline__

namespace h12 {

// out = R_A(q) * in   (child coords -> parent axes); c = cos q, s = sin q
template <int A>
H12_DEV void rot(float c, float s, const float* in, float* out) {
  float x = in[0], y = in[1], z = in[2];
  if constexpr (A == 0) { out[0] = x; out[1] = c * y - s * z; out[2] = s * y + c * z; }
  else if constexpr (A == 1) { out[0] = c * x + s * z; out[1] = y; out[2] = -s * x + c * z; }
  else { out[0] = c * x - s * y; out[1] = s * x + c * y; out[2] = z; }
}
// out = R_A(q)^T * in (parent axes -> child coords)
template <int A>
H12_DEV void rotT(float c, float s, const float* in, float* out) { rot<A>(c, -s, in, out); }

H12_DEV void cross(const float* a, const float* b, float* o) {
  float t0 = a[1] * b[2] - a[2] * b[1];
  float t1 = a[2] * b[0] - a[0] * b[2];
  float t2 = a[0] * b[1] - a[1] * b[0];
  o[0] = t0; o[1] = t1; o[2] = t2;
}
H12_DEV float dot3(const float* a, const float* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

// 3x3 rotation from unit quaternion (w x y z); R maps body -> world
// the rotation of q / |q| (round 6): a stored fp32 quaternion is unit only to its rounding, and the one the kernel's own
// normalisation (rsq) leaves is short by ~2e-8 on average; the unit-quaternion formula then scales the rotation's off-
// diagonal part by |q|^2 and showed up as a signed bias of lying robots (VLIN2 -3.5e-7, z = -69; the oracle normalises
// first, quat_to_R).  Writing 2 / |q|^2 for the formula's 2 makes it exact for any |q| (+5 VALU)
// (every product-sum is an explicit fma: the call sites of the fused and the two-kernel observation paths must round
// alike, and the compiler's contraction choice may differ between them).  quat_R_unit: the unit-quaternion formula
// (step_kernel's physics wave after barrier R2, where the reciprocal sat on the step's critical chain: -0.9 % in an
// interleaved A/B; its R0 only turns gravity and the base velocities, which a |q|^2 - 1 of ~1e-7 moves by as much)
H12_DEV void quat_R_unit(const float* q, float R[3][3]) {
  float w = q[0], x = q[1], y = q[2], z = q[3];
  R[0][0] = 1.f - 2.f * (y * y + z * z); R[0][1] = 2.f * (x * y - w * z); R[0][2] = 2.f * (x * z + w * y);
  R[1][0] = 2.f * (x * y + w * z); R[1][1] = 1.f - 2.f * (x * x + z * z); R[1][2] = 2.f * (y * z - w * x);
  R[2][0] = 2.f * (x * z - w * y); R[2][1] = 2.f * (y * z + w * x); R[2][2] = 1.f - 2.f * (x * x + y * y);
}
H12_DEV void quat_R(const float* q, float R[3][3]) {
  const float w = q[0], x = q[1], y = q[2], z = q[3];
  const float F = __builtin_fmaf(w, w, __builtin_fmaf(x, x, __builtin_fmaf(y, y, z * z)));
  const float t = 2.f * __builtin_amdgcn_rcpf(F);
  const float xx = x * x, yy = y * y, zz = z * z;
  R[0][0] = __builtin_fmaf(-t, yy + zz, 1.f);
  R[0][1] = t * __builtin_fmaf(x, y, -(w * z));
  R[0][2] = t * __builtin_fmaf(x, z, w * y);
  R[1][0] = t * __builtin_fmaf(x, y, w * z);
  R[1][1] = __builtin_fmaf(-t, xx + zz, 1.f);
  R[1][2] = t * __builtin_fmaf(y, z, -(w * x));
  R[2][0] = t * __builtin_fmaf(x, z, -(w * y));
  R[2][1] = t * __builtin_fmaf(y, z, w * x);
  R[2][2] = __builtin_fmaf(-t, xx + yy, 1.f);
}
H12_DEV void mv(const float R[3][3], const float* v, float* o) {
  float t0 = R[0][0] * v[0] + R[0][1] * v[1] + R[0][2] * v[2];
  float t1 = R[1][0] * v[0] + R[1][1] * v[1] + R[1][2] * v[2];
  float t2 = R[2][0] * v[0] + R[2][1] * v[1] + R[2][2] * v[2];
  o[0] = t0; o[1] = t1; o[2] = t2;
}
H12_DEV void mtv(const float R[3][3], const float* v, float* o) {
  float t0 = R[0][0] * v[0] + R[1][0] * v[1] + R[2][0] * v[2];
  float t1 = R[0][1] * v[0] + R[1][1] * v[1] + R[2][1] * v[2];
  float t2 = R[0][2] * v[0] + R[1][2] * v[1] + R[2][2] * v[2];
  o[0] = t0; o[1] = t1; o[2] = t2;
}
// R <- R * R_A(q)  (world rotation of a child frame)
template <int A>
H12_DEV void rmul_axis(float R[3][3], float c, float s) {
  for (int i = 0; i < 3; ++i) {
    float row[3] = {R[i][0], R[i][1], R[i][2]}, o[3];
    // row * R_A = (R_A^T row^T)^T
    rotT<A>(c, s, row, o);
    R[i][0] = o[0]; R[i][1] = o[1]; R[i][2] = o[2];
  }
}

// Articulated-body inertia I = [[A, B], [B^T, C]] with A, C symmetric (xx yy zz xy xz yz).
struct AInertia {
  float A[6];
  float B[3][3];
  float C[6];
};
H12_DEV float sget(const float* S, int i, int j) {
  // symmetric accessor, indices resolved at compile time after unrolling
  if (i == j) return S[i];
  int a = i < j ? i : j, b = i < j ? j : i;
  return (a == 0) ? (b == 1 ? S[3] : S[4]) : S[5];
}
H12_DEV void sym_full(const float* S, float M[3][3]) {
  M[0][0] = S[0]; M[1][1] = S[1]; M[2][2] = S[2];
  M[0][1] = M[1][0] = S[3]; M[0][2] = M[2][0] = S[4]; M[1][2] = M[2][1] = S[5];
}
H12_DEV void full_sym(const float M[3][3], float* S) {
  S[0] = M[0][0]; S[1] = M[1][1]; S[2] = M[2][2]; S[3] = M[0][1]; S[4] = M[0][2]; S[5] = M[1][2];
}
// I * m for a 6-vector m = (w; v):  (A w + B v ; B^T w + C v)
H12_DEV void ai_mul(const AInertia& I, const float* m, float* o) {
  const float* w = m;
  const float* v = m + 3;
  for (int i = 0; i < 3; ++i) {
    o[i] = sget(I.A, i, 0) * w[0] + sget(I.A, i, 1) * w[1] + sget(I.A, i, 2) * w[2] +
           I.B[i][0] * v[0] + I.B[i][1] * v[1] + I.B[i][2] * v[2];
    o[3 + i] = I.B[0][i] * w[0] + I.B[1][i] * w[1] + I.B[2][i] * w[2] +
               sget(I.C, i, 0) * v[0] + sget(I.C, i, 1) * v[1] + sget(I.C, i, 2) * v[2];
  }
}
// rigid-body inertia at the body origin from (Ibar = I_origin (sym), mc = m*c, m)
H12_DEV void ai_rigid(AInertia& I, const float* Ibar, const float* mc, float m) {
  for (int i = 0; i < 6; ++i) I.A[i] = Ibar[i];
  // B = m [c]x
  I.B[0][0] = 0.f; I.B[0][1] = -mc[2]; I.B[0][2] = mc[1];
  I.B[1][0] = mc[2]; I.B[1][1] = 0.f; I.B[1][2] = -mc[0];
  I.B[2][0] = -mc[1]; I.B[2][1] = mc[0]; I.B[2][2] = 0.f;
  I.C[0] = I.C[1] = I.C[2] = m;
  I.C[3] = I.C[4] = I.C[5] = 0.f;
}
// add a point mass dm at c (rigidly attached, inertia about the body origin): randomize_rigid_body_mass
// with recompute_inertia=False adds mass without changing the body's inertia about its COM
H12_DEV void ai_add_point_mass(AInertia& I, float dm, const float* c) {
  const float c2 = c[0] * c[0] + c[1] * c[1] + c[2] * c[2];
  I.A[0] += dm * (c2 - c[0] * c[0]); I.A[1] += dm * (c2 - c[1] * c[1]); I.A[2] += dm * (c2 - c[2] * c[2]);
  I.A[3] -= dm * c[0] * c[1]; I.A[4] -= dm * c[0] * c[2]; I.A[5] -= dm * c[1] * c[2];
  // B = m [c]x with m c -> dm c
  I.B[0][1] -= dm * c[2]; I.B[0][2] += dm * c[1];
  I.B[1][0] += dm * c[2]; I.B[1][2] -= dm * c[0];
  I.B[2][0] -= dm * c[1]; I.B[2][1] += dm * c[0];
  I.C[0] += dm; I.C[1] += dm; I.C[2] += dm;
}
H12_DEV void ai_add(AInertia& I, const AInertia& J) {
  for (int i = 0; i < 6; ++i) { I.A[i] += J.A[i]; I.C[i] += J.C[i]; }
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) I.B[i][j] += J.B[i][j];
}
// symmetric-index helper: position of (i,j) in the (xx yy zz xy xz yz) packing
H12_DEV constexpr int sidx(int i, int j) {
  return i == j ? i : ((i + j == 1) ? 3 : ((i + j == 2) ? 4 : 5));
}
// S <- R_A S R_A^T for symmetric S: only the (i, j) plane orthogonal to the axis k = A rotates,
// v_i' = c v_i - s v_j, v_j' = s v_i + c v_j with (i, j) = (y, z), (z, x), (x, y) for A = x, y, z
template <int A>
H12_DEV void sym_rotate(float* S, float c, float s) {
  constexpr int i = (A + 1) % 3, j = (A + 2) % 3, k = A;
  const float cc = c * c, ss = s * s, cs = c * s;
  float sii = S[sidx(i, i)], sjj = S[sidx(j, j)], sij = S[sidx(i, j)];
  float sik = S[sidx(i, k)], sjk = S[sidx(j, k)];
  S[sidx(i, i)] = cc * sii - 2.f * cs * sij + ss * sjj;
  S[sidx(j, j)] = ss * sii + 2.f * cs * sij + cc * sjj;
  S[sidx(i, j)] = cs * (sii - sjj) + (cc - ss) * sij;
  S[sidx(i, k)] = c * sik - s * sjk;
  S[sidx(j, k)] = s * sik + c * sjk;
}
// two floats in one 64-bit register pair: v_pk_{fma,mul,add}_f32 do both lanes of the pair in one VALU op
typedef float f32x2 __attribute__((ext_vector_type(2)));
// a pair from two scalars.  The empty asm hands lane 0 over as a value: otherwise the optimiser turns "element k
// of S into lane 0" into a 2-wide load at &S[k] (then replaces lane 1), and that overlapping access keeps the
// whole array on the stack (scratch)
H12_DEV f32x2 pk2(float a, float b) {
  asm("" : "+v"(a));
  f32x2 v;
  v.x = a;
  v.y = b;
  return v;
}
// sym_rotate of the A and C blocks together (the same rotation, elementwise the same operations): one packed op
// per pair of scalar ones
template <int A>
H12_DEV void sym_rotate_ac(float* SA, float* SC, float c, float s) {
  constexpr int i = (A + 1) % 3, j = (A + 2) % 3, k = A;
  const float cc = c * c, ss = s * s, cs = c * s;
  const f32x2 sii = pk2(SA[sidx(i, i)], SC[sidx(i, i)]), sjj = pk2(SA[sidx(j, j)], SC[sidx(j, j)]);
  const f32x2 sij = pk2(SA[sidx(i, j)], SC[sidx(i, j)]);
  const f32x2 sik = pk2(SA[sidx(i, k)], SC[sidx(i, k)]), sjk = pk2(SA[sidx(j, k)], SC[sidx(j, k)]);
  const f32x2 nii = cc * sii - 2.f * cs * sij + ss * sjj;
  const f32x2 njj = ss * sii + 2.f * cs * sij + cc * sjj;
  const f32x2 nij = cs * (sii - sjj) + (cc - ss) * sij;
  const f32x2 nik = c * sik - s * sjk;
  const f32x2 njk = s * sik + c * sjk;
  SA[sidx(i, i)] = nii.x; SC[sidx(i, i)] = nii.y;
  SA[sidx(j, j)] = njj.x; SC[sidx(j, j)] = njj.y;
  SA[sidx(i, j)] = nij.x; SC[sidx(i, j)] = nij.y;
  SA[sidx(i, k)] = nik.x; SC[sidx(i, k)] = nik.y;
  SA[sidx(j, k)] = njk.x; SC[sidx(j, k)] = njk.y;
}
// rotate every block into parent axes: X_rot^T I X_rot with E^T = R_A(q)
template <int A>
H12_DEV void ai_rotate(AInertia& I, float c, float s) {
  float T[3][3];
  sym_rotate_ac<A>(I.A, I.C, c, s);
  // B block: R B R^T (columns 0 / 1, then rows 0 / 1, as packed pairs)
  {
    const f32x2 x = pk2(I.B[0][0], I.B[0][1]), y = pk2(I.B[1][0], I.B[1][1]), z = pk2(I.B[2][0], I.B[2][1]);
    f32x2 o0, o1, o2;
    if constexpr (A == 0) { o0 = x; o1 = c * y - s * z; o2 = s * y + c * z; }
    else if constexpr (A == 1) { o0 = c * x + s * z; o1 = y; o2 = -s * x + c * z; }
    else { o0 = c * x - s * y; o1 = s * x + c * y; o2 = z; }
    T[0][0] = o0.x; T[0][1] = o0.y; T[1][0] = o1.x; T[1][1] = o1.y; T[2][0] = o2.x; T[2][1] = o2.y;
    float col[3] = {I.B[0][2], I.B[1][2], I.B[2][2]}, o[3];
    rot<A>(c, s, col, o);
    T[0][2] = o[0]; T[1][2] = o[1]; T[2][2] = o[2];
  }
  {
    const f32x2 x = pk2(T[0][0], T[1][0]), y = pk2(T[0][1], T[1][1]), z = pk2(T[0][2], T[1][2]);
    f32x2 o0, o1, o2;
    if constexpr (A == 0) { o0 = x; o1 = c * y - s * z; o2 = s * y + c * z; }
    else if constexpr (A == 1) { o0 = c * x + s * z; o1 = y; o2 = -s * x + c * z; }
    else { o0 = c * x - s * y; o1 = s * x + c * y; o2 = z; }
    I.B[0][0] = o0.x; I.B[1][0] = o0.y; I.B[0][1] = o1.x; I.B[1][1] = o1.y; I.B[0][2] = o2.x; I.B[1][2] = o2.y;
    float row[3] = {T[2][0], T[2][1], T[2][2]}, o[3];
    rot<A>(c, s, row, o);
    I.B[2][0] = o[0]; I.B[2][1] = o[1]; I.B[2][2] = o[2];
  }
}
// shift the reference point from the child origin to the parent origin (child origin at r in
// parent coords, parent axes): A += S + S^T - T rx, B += T, with T = rx C, S = rx B^T.
H12_DEV void ai_shift(AInertia& I, const float* r) {
  float Cf[3][3], T[3][3], S[3][3];
  sym_full(I.C, Cf);
  for (int j = 0; j < 3; ++j) { float col[3] = {Cf[0][j], Cf[1][j], Cf[2][j]}, o[3]; cross(r, col, o); T[0][j] = o[0]; T[1][j] = o[1]; T[2][j] = o[2]; }
  // S = rx B^T : column j of B^T is row j of B
  for (int j = 0; j < 3; ++j) { float col[3] = {I.B[j][0], I.B[j][1], I.B[j][2]}, o[3]; cross(r, col, o); S[0][j] = o[0]; S[1][j] = o[1]; S[2][j] = o[2]; }
  // (T rx)_ij = T_i . rx_col_j ; rx = [[0,-rz,ry],[rz,0,-rx],[-ry,rx,0]]
  auto trx = [&](int i, int j) {
    float rxc0 = (j == 0) ? 0.f : (j == 1 ? -r[2] : r[1]);
    float rxc1 = (j == 0) ? r[2] : (j == 1 ? 0.f : -r[0]);
    float rxc2 = (j == 0) ? -r[1] : (j == 1 ? r[0] : 0.f);
    return T[i][0] * rxc0 + T[i][1] * rxc1 + T[i][2] * rxc2;
  };
  I.A[0] += 2.f * S[0][0] - trx(0, 0);
  I.A[1] += 2.f * S[1][1] - trx(1, 1);
  I.A[2] += 2.f * S[2][2] - trx(2, 2);
  I.A[3] += S[0][1] + S[1][0] - trx(0, 1);
  I.A[4] += S[0][2] + S[2][0] - trx(0, 2);
  I.A[5] += S[1][2] + S[2][1] - trx(1, 2);
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) I.B[i][j] += T[i][j];
}

// Philox4x32-10 (same streams as oracle/h12_oracle.c)
H12_DEV void philox(uint32_t k0, uint32_t k1, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t out[4]) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
    uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
    uint32_t y0 = hi1 ^ c1 ^ k0;
    uint32_t y2 = hi0 ^ c3 ^ k1;
    c1 = lo1;
    c3 = lo0;
    c0 = y0;
    c2 = y2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}
// single-instruction transcendental / reciprocal / sqrt (v_sin, v_cos, v_rcp, v_sqrt: ~1 ulp, no
// range-reduction or Newton sequences; arguments here are joint angles and positive magnitudes)
//
// fsincos (round 6): the hardware sine / cosine with their radial bias removed.  __sinf / __cosf (v_mul by fp32(1/2pi),
// v_sin_f32 / v_cos_f32) carry two systematic errors on MI355X (tools/probe/hw_trig_table.hip, profiles/r6/r6e_*):
// the constant fp32(1/2pi) is 4.03e-8 (relative) low, so every angle comes out 4.03e-8 x smaller; and the results lie
// 3.2e-8 inside the unit circle at every angle (a round-down of ~0.3-0.5 ulp).  The second one shortens every rotated
// link offset by 3.2e-8 per joint: it is what the fp32 oracle with that error table reproduces as the kernel's signed
// bias in the sole scenarios (the feet a few 1e-8 m high, weaker support: stance VLIN2 -1.75e-6, z = -144; DESIGN.md
// section 4, tools/bias_attrib.py); the angle error alone moves nothing measurable there.  So each (sin, cos) pair is
// put back on the unit circle to first order: d = s^2 + c^2 - 1 from two fma (their one rounding is zero-mean), then
// (s, c)(1 - d / 2): +5 VALU per call.  fsincos_hw: the uncorrected pair (the self-contact wave's pass 1, where the
// step's most critical wave before barrier R1 would pay for it and a 3e-8 shift of a leg-leg contact point moves
// nothing a gate sees).
H12_DEV void fsincos_hw(float x, float* s, float* c) { *s = __sinf(x); *c = __cosf(x); }
H12_DEV void fsincos(float x, float* s, float* c) {
  float sv, cv;
  fsincos_hw(x, &sv, &cv);
  const float d = __builtin_fmaf(cv, cv, __builtin_fmaf(sv, sv, -1.f));
  const float k = -0.5f * d;  // the one rounding (of s^2 - 1) is zero-mean; (1 + d)^(-1/2) = 1 - d / 2 to 1e-15
  *s = __builtin_fmaf(sv, k, sv);
  *c = __builtin_fmaf(cv, k, cv);
}
H12_DEV float frcp(float x) { return __builtin_amdgcn_rcpf(x); }
H12_DEV float fsqrt(float x) { return __builtin_amdgcn_sqrtf(x); }

H12_DEV float u01(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }
H12_DEV float uab(uint32_t x, float a, float b) { return a + (b - a) * u01(x); }

// lane-pair exchange (lanes 2e and 2e+1 hold the two legs of env e): one DPP quad_perm(1,0,3,2)
// move (a VALU op) instead of __shfl_xor's ds_bpermute round trip through the LDS crossbar.  bound_ctrl set: the
// compiler then folds the move into a consuming VALU op (x + pair_swap(x) -> one v_add_f32_dpp); a quad_perm source
// is never out of bounds, and the callers keep both lanes of a pair active at every swap
H12_DEV int pair_swap_i(int x) { return __builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, true); }
H12_DEV float pair_swap(float x) { return __int_as_float(pair_swap_i(__float_as_int(x))); }

}  // namespace h12
