// FETCH_SIZE / WRITE_SIZE calibration for the access widths step_kernel uses (MI355X_MICROARCH.md: "other access widths
// are uncalibrated"): 64 MiB read (and written) with 4-B-per-lane buffer loads / stores (the state fields), with 16-B-per-
// lane loads / stores (the rows) and with 4-B-per-lane loads of 64-float runs per wave 1 KB apart (the field-major
// layout of a 4096-env workspace: every field of a wave's 64 envs is one 256-B run).  Run under
// rocprofv3 --pmc FETCH_SIZE (then WRITE_SIZE); each kernel's counter / byte count is the calibration factor.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void rd4(const float* __restrict__ a, float* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  float v = 0.f;
  for (int k = i; k < n; k += gridDim.x * blockDim.x) v += a[k];
  if (v == 1234.5f) out[i] = v;
}
__global__ void rd16(const float4* __restrict__ a, float* out, int n4) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  float v = 0.f;
  for (int k = i; k < n4; k += gridDim.x * blockDim.x) { const float4 x = a[k]; v += x.x + x.y + x.z + x.w; }
  if (v == 1234.5f) out[i] = v;
}
__global__ void wr4(float* a, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  for (int k = i; k < n; k += gridDim.x * blockDim.x) a[k] = (float)k;
}
__global__ void wr16(float4* a, int n4) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  for (int k = i; k < n4; k += gridDim.x * blockDim.x) a[k] = make_float4(k, k, k, k);
}

int main() {
  const int n = 16 << 20;  // 64 MiB of floats
  float *a, *out;
  if (hipMalloc(&a, (size_t)n * 4) != hipSuccess || hipMalloc(&out, 1 << 20) != hipSuccess) return 1;
  hipMemset(a, 0, (size_t)n * 4);
  for (int r = 0; r < 3; ++r) {
    hipLaunchKernelGGL(rd4, dim3(4096), dim3(256), 0, 0, a, out, n);
    hipLaunchKernelGGL(rd16, dim3(4096), dim3(256), 0, 0, (const float4*)a, out, n / 4);
    hipLaunchKernelGGL(wr4, dim3(4096), dim3(256), 0, 0, a, n);
    hipLaunchKernelGGL(wr16, dim3(4096), dim3(256), 0, 0, (float4*)a, n / 4);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("bytes per kernel %zu\n", (size_t)n * 4);
  return 0;
}
