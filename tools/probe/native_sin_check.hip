// Accuracy probe (tools only, not shipped): the hardware sine / cosine (__sinf / __cosf -> v_sin_f32 / v_cos_f32)
// against the host's double-precision sin / cos, over the argument ranges the kernel feeds them: half rotation
// angles of the base quaternion increment (|w| h / 2, ~1e-6 .. 0.1 rad) and joint angles (-3 .. 3 rad).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>

__global__ void k(const float* x, float* s, float* c, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) { s[i] = __sinf(x[i]); c[i] = __cosf(x[i]); }
}

int main() {
  const int n = 1 << 20;
  std::vector<float> x(n), s(n), c(n);
  float *dx, *ds, *dc;
  hipMalloc(&dx, n * 4); hipMalloc(&ds, n * 4); hipMalloc(&dc, n * 4);
  struct R { double lo, hi; const char* name; } ranges[] = {
      {1e-6, 1e-4, "tiny [1e-6,1e-4]"}, {1e-4, 1e-2, "small [1e-4,1e-2]"}, {1e-2, 0.5, "mid [1e-2,0.5]"},
      {0.5, 3.0, "joint [0.5,3]"}};
  for (auto& r : ranges) {
    for (int i = 0; i < n; ++i) x[i] = (float)(r.lo * std::pow(r.hi / r.lo, (i + 0.5) / n));
    hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice);
    k<<<n / 256, 256>>>(dx, ds, dc, n);
    hipMemcpy(s.data(), ds, n * 4, hipMemcpyDeviceToHost);
    hipMemcpy(c.data(), dc, n * 4, hipMemcpyDeviceToHost);
    double sa = 0, sr = 0, ca = 0, sbias = 0;
    for (int i = 0; i < n; ++i) {
      double xs = std::sin((double)x[i]), xc = std::cos((double)x[i]);
      double es = s[i] - xs;
      sa = std::fmax(sa, std::fabs(es));
      sr = std::fmax(sr, std::fabs(es) / std::fabs(xs));
      sbias += es / std::fabs(xs);
      ca = std::fmax(ca, std::fabs(c[i] - xc));
    }
    printf("%-20s sin: max abs %.3g max rel %.3g mean rel %.3g | cos: max abs %.3g\n", r.name, sa, sr, sbias / n, ca);
  }
  return 0;
}
