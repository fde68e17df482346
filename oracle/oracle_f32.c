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
#ifdef H12_F32_HWTRIG
/* the kernel's __sinf / __cosf: v_mul_f32 by fp32(1 / 2 pi), then the hardware's sin / cos of that many revolutions
 * (evaluated here exactly, in double, and rounded: the prescale's rounding is the only fp32 error kept) */
static float hw_sin(float x) { return (float)sin(6.283185307179586 * (double)(x * 0.15915494f)); }
static float hw_cos(float x) { return (float)cos(6.283185307179586 * (double)(x * 0.15915494f)); }
#endif
#define double float
#ifdef H12_F32_HWTRIG
#define sin(x) hw_sin(x)
#define cos(x) hw_cos(x)
#endif
#include "h12_oracle.c"
