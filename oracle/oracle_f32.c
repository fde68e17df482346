/*
 * oracle_f32.c -- the oracle's source compiled with single-precision arithmetic (TEST INFRASTRUCTURE ONLY): every
 * `double` of h12_oracle.c becomes `float` and every floating literal single precision (-fsingle-precision-constant);
 * the libm calls still round through double.  Used as a second, independent fp32 evaluation of the same algorithm
 * (tools/bias_attrib.py, tests/test_forced_harness.py): the signed bias an fp32 evaluation of the sole-contact
 * scenarios carries against the fp64 oracle, which the kernel's bias gate is then measured against
 * (DESIGN.md section 4).  Only the env-level entry points (orc_env_reset / orc_env_step, float / int arguments)
 * keep the fp64 build's ABI; the single-env ones take float where the header says double.
 */
#include <math.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "../include/h12env.h"
#if defined(H12_F32_HWTRIG) && !defined(H12_F32_HWTRIG_TABLE)
/* the kernel's __sinf / __cosf: v_mul_f32 by fp32(1 / 2 pi), then the hardware's sin / cos of that many revolutions
 * (evaluated here exactly, in double, and rounded: the prescale's rounding is the only fp32 error kept) */
static float hw_sin(float x) { return (float)sin(6.283185307179586 * (double)(x * 0.15915494f)); }
static float hw_cos(float x) { return (float)cos(6.283185307179586 * (double)(x * 0.15915494f)); }
#endif
#ifdef H12_F32_HWTRIG_TABLE
/* the kernel's __sinf / __cosf as measured: the exact value plus the hardware's mean signed error of the argument's
 * bin, linearly interpolated between bin centres (hw_trig_err.h, tools/probe/hw_trig_table.hip) */
#include "hw_trig_err.h"
static float trig_err(const float* t, float x) {
  const double u = ((double)x + 3.14159265358979323846) / (2 * 3.14159265358979323846) * H12_TRIG_NB - 0.5;
  int i = (int)floor(u);
  const double f = u - i;
  const int i0 = i < 0 ? 0 : (i > H12_TRIG_NB - 1 ? H12_TRIG_NB - 1 : i);
  const int i1 = i + 1 < 0 ? 0 : (i + 1 > H12_TRIG_NB - 1 ? H12_TRIG_NB - 1 : i + 1);
  return (float)((1 - f) * t[i0] + f * t[i1]);
}
static float hw_sin(float x) { return (float)(sin((double)x) + trig_err(h12_sin_err, x)); }
static float hw_cos(float x) { return (float)(cos((double)x) + trig_err(h12_cos_err, x)); }
#define H12_F32_HWTRIG
#endif
#define double float
#ifdef H12_F32_HWTRIG
#define sin(x) hw_sin(x)
#define cos(x) hw_cos(x)
#endif
#include "h12_oracle.c"
