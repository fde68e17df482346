// Error table of the kernel's __sinf / __cosf (v_mul by fp32(1/2pi), then v_sin_f32 / v_cos_f32) against the host's
// double sin / cos (tools only, not shipped; round 6): the mean SIGNED absolute error in 512 bins over
// [-pi, pi] (every 64th fp32 value of each bin's range is evaluated), printed as "bin lo hi mean_sin_err mean_cos_err
// count" lines for tools/bias_attrib.py (oracle/oracle_f32.c -DH12_F32_HWTRIG_TABLE emulates the table).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

__global__ void k(const float* x, float* s, float* c, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) { s[i] = __sinf(x[i]); c[i] = __cosf(x[i]); }
}

int main() {
  const int NB = 512;
  const double PI = 3.14159265358979323846;
  std::vector<float> x;
  std::vector<int> bin;
  for (int b = 0; b < NB; ++b) {
    const float lo = (float)(-PI + 2 * PI * b / NB), hi = (float)(-PI + 2 * PI * (b + 1) / NB);
    for (float v = lo; v < hi; ) {
      x.push_back(v);
      bin.push_back(b);
      uint32_t u;
      std::memcpy(&u, &v, 4);
      // step 64 fp32 values (toward +inf for positive, toward 0 for negative numbers)
      for (int s = 0; s < 64 && v < hi; ++s) v = std::nextafter(v, INFINITY);
    }
  }
  const int n = (int)x.size();
  std::vector<float> s(n), c(n);
  float *dx, *ds, *dc;
  if (hipMalloc(&dx, n * 4) != hipSuccess || hipMalloc(&ds, n * 4) != hipSuccess || hipMalloc(&dc, n * 4) != hipSuccess) return 1;
  hipMemcpy(dx, x.data(), (size_t)n * 4, hipMemcpyHostToDevice);
  k<<<(n + 255) / 256, 256>>>(dx, ds, dc, n);
  hipMemcpy(s.data(), ds, (size_t)n * 4, hipMemcpyDeviceToHost);
  hipMemcpy(c.data(), dc, (size_t)n * 4, hipMemcpyDeviceToHost);
  std::vector<double> es(NB, 0.0), ec(NB, 0.0), cnt(NB, 0.0);
  for (int i = 0; i < n; ++i) {
    es[bin[i]] += (double)s[i] - std::sin((double)x[i]);
    ec[bin[i]] += (double)c[i] - std::cos((double)x[i]);
    cnt[bin[i]] += 1.0;
  }
  std::printf("# points %d\n", n);
  for (int b = 0; b < NB; ++b)
    std::printf("%d %.9f %.9f %.6e %.6e %.0f\n", b, -PI + 2 * PI * b / NB, -PI + 2 * PI * (b + 1) / NB,
                es[b] / cnt[b], ec[b] / cnt[b], cnt[b]);
  return 0;
}
