// Bias probe (tools only, not shipped; round 6): the SIGNED mean error of the kernel's single-
// instruction math -- __sinf / __cosf (v_mul by fp32(1/2pi), v_sin_f32 / v_cos_f32), __builtin_amdgcn_rsqf (v_rsq_f32),
// __builtin_amdgcn_rcpf (v_rcp_f32), __builtin_amdgcn_sqrtf (v_sqrt_f32), __expf -- against the host's double
// libm, in units of the result's fp32 ulp, over the argument ranges the kernel feeds them.  A zero-mean error
// averages out over env-steps; a signed one shifts every env the same way (the sole-contact scenarios' signed
// bias gate, tests/test_gpu_sensitivity.py).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <vector>

#include "../../h1v2-isaac_amd/csrc/h12_math.h"

__global__ void k(const float* x, float* o, int n, int op) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float v = x[i];
  float r;
  switch (op) {
    case 0: r = __sinf(v); break;
    case 1: r = __cosf(v); break;
    case 2: r = __builtin_amdgcn_rsqf(v); break;
    case 3: r = __builtin_amdgcn_rcpf(v); break;
    case 4: r = __builtin_amdgcn_sqrtf(v); break;
    case 5: r = __expf(v); break;
    case 6: { float c_; h12::fsincos(v, &r, &c_); break; }  // the product's fsincos (round 6)
    default: { float s_; h12::fsincos(v, &s_, &r); break; }
  }
  o[i] = r;
}

static double ref(int op, double v) {
  switch (op) {
    case 0: case 6: return std::sin(v);
    case 1: case 7: return std::cos(v);
    case 2: return 1.0 / std::sqrt(v);
    case 3: return 1.0 / v;
    case 4: return std::sqrt(v);
    default: return std::exp(v);
  }
}

int main() {
  const int n = 1 << 22;
  std::vector<float> x(n), o(n);
  float *dx, *dout;
  if (hipMalloc(&dx, n * 4) != hipSuccess || hipMalloc(&dout, n * 4) != hipSuccess) return 1;
  struct C { int op; double lo, hi; const char* name; } cases[] = {
      {0, -1.6, 1.6, "sin   [-1.6, 1.6] (joint angles)"},   {1, -1.6, 1.6, "cos   [-1.6, 1.6] (joint angles)"},
      {0, 1e-5, 0.05, "sin   [1e-5, 0.05] (quat half-angle)"}, {1, 1e-5, 0.05, "cos   [1e-5, 0.05] (quat half-angle)"},
      {2, 0.5, 2.0, "rsq   [0.5, 2] (normalisations)"},     {2, 1e-4, 1e4, "rsq   [1e-4, 1e4]"},
      {3, 0.5, 2.0, "rcp   [0.5, 2]"},                      {3, 1e-3, 1e3, "rcp   [1e-3, 1e3] (1/D of the ABA)"},
      {4, 1e-4, 1e4, "sqrt  [1e-4, 1e4]"},                   {5, -10.0, 0.0, "exp   [-10, 0] (tracking rewards)"},
      {6, -1.6, 1.6, "fsincos sin [-1.6, 1.6] (product)"},  {7, -1.6, 1.6, "fsincos cos [-1.6, 1.6] (product)"},
      {6, -3.2, 3.2, "fsincos sin [-3.2, 3.2] (product)"},  {7, -3.2, 3.2, "fsincos cos [-3.2, 3.2] (product)"},
      {6, 0.3, 1.2, "fsincos sin [0.3, 1.2] (product)"},    {7, 0.3, 1.2, "fsincos cos [0.3, 1.2] (product)"},
      {0, 0.3, 1.2, "sin   [0.3, 1.2]"},                    {1, 0.3, 1.2, "cos   [0.3, 1.2]"}};
  for (auto& c : cases) {
    for (int i = 0; i < n; ++i) {
      const double t = (i + 0.5) / n;
      x[i] = (float)((c.op >= 2 && c.op <= 4 && c.lo > 0) ? c.lo * std::pow(c.hi / c.lo, t) : c.lo + (c.hi - c.lo) * t);
    }
    hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice);
    k<<<n / 256, 256>>>(dx, dout, n, c.op);
    hipMemcpy(o.data(), dout, n * 4, hipMemcpyDeviceToHost);
    double su = 0, sa = 0, mx = 0, sr = 0, sabs = 0;
    for (int i = 0; i < n; ++i) {
      const double r = ref(c.op, (double)x[i]);
      const float rf = (float)r;
      const double ulp = std::fabs((double)std::nextafter(rf, INFINITY) - (double)rf);
      const double e = (double)o[i] - r;
      su += e / ulp;
      sa += std::fabs(e / ulp);
      sr += r != 0.0 ? e / std::fabs(r) : 0.0;
      sabs += e;
      mx = std::fmax(mx, std::fabs(e / ulp));
    }
    std::printf("%-38s mean signed %+.4f ulp  mean |err| %.4f ulp  max %.3f ulp  mean signed rel %+.3e  abs %+.3e\n",
                c.name, su / n, sa / n, mx, sr / n, sabs / n);
  }
  return 0;
}
