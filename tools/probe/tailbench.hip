// Store-tail probe (tools only, not shipped; round 4).  A skeleton of step_kernel's fused launch at 4096 envs
// with the physics replaced by a dependent FMA chain, to find why the frame + state-store tail of the physics waves
// takes 2-3 us on four XCDs and 6-10 us on the other four:
//   128 blocks x 3 waves (192 threads), block b -> env chunk xcd_block(b) (one contiguous env range per XCD);
//   wave 0 ("physics"): 4 x (spin, barrier R) ; frame -> LDS ; barrier F ; 88 dword state stores (field-major
//     [f][4096], lane pair = env, one field per leg lane) ;
//   waves 1-2 ("helpers"): in the windows after R of steps 1..3 one third each of the block's 32 history rows
//     (32 x 450 floats = 57.6 KB) copied obs_prev -> obs as float4s ; s_waitcnt(0) ; barrier F ; the newest-slot
//     floats (45 per row, 4-byte stores at col*10 + 9).
// Per wave: s_memrealtime at start, after the spin, after barrier F, after the last store issued, after
// s_waitcnt vmcnt(0); XCC id.  Variants by flag bits (run-time, one binary):
//   1 no row copies, 2 no waitcnt before F, 4 no state stores, 8 no newest-slot stores, 16 rows stored nt,
//   32 plain block -> chunk map, 64 rows copied after barrier F instead of in the windows,
//   128 obs_prev / obs NOT swapped between launches (the same buffer written every launch),
//   256 the helper waves store the block's 17 episode-log partials after the newest slot, value-major
//     [17][blocks] indexed by blockIdx.x (step_kernel's log_part layout: a 128-B line holds 32 blocks' values,
//     blocks round-robin over the XCDs), 512 the same indexed by the env chunk (a line's blocks on one XCD),
//   1024 block-major [blocks][64] (each block its own two lines)
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int N = 4096, EPB = 32, NB = N / EPB, ROW = 450, NF = 88;
struct Stamp { unsigned long long t[6]; };

// flag 2048: instead of the two-FMA spin, each wave role runs a LARGE unrolled chain of distinct instructions (its
// own template instance: physics ~24 KB, helpers ~16 KB of machine code), like step_kernel's loops (physics 23.7 KB,
// helper 15.9 KB, self-contact 10.3 KB of a 71.6 KB kernel) -- does the code footprint reproduce the XCD split?
template <int SEED, int LEN>
__device__ __attribute__((noinline)) float chain(float x, float y) {
#pragma unroll
  for (int i = 0; i < LEN; ++i) {
    x = __builtin_fmaf(x, y + (float)(i * 7 + SEED) * 1e-7f, (float)(i ^ SEED) * 1e-9f);
    y = __builtin_fmaf(y, 0.9999f, x * (float)(i + SEED) * 1e-12f);
  }
  return x + y;
}

__device__ int xcd_block(int b, int nb) {
  const int x = b & 7, k = b >> 3, q = nb >> 3, r = nb & 7;
  return x * q + std::min(x, r) + k;
}

__global__ void __launch_bounds__(192) tail_kernel(const float* obs_prev, float* obs, float* F, Stamp* st, int flags,
                                                   int spin, float* logp) {
  __shared__ float frame[EPB * 45];
  const int blk = (flags & 32) ? blockIdx.x : xcd_block(blockIdx.x, gridDim.x);
  const int e0 = blk * EPB;
  const int w = threadIdx.x >> 6;
  unsigned long long s0 = __builtin_amdgcn_s_memrealtime(), s1 = 0, s2 = 0, s3 = 0, s4 = 0;
  const float4* src = reinterpret_cast<const float4*>(obs_prev + (size_t)e0 * ROW);
  float4* dst = reinterpret_cast<float4*>(obs + (size_t)e0 * ROW);
  constexpr int F4 = EPB * ROW / 4;  // 3600 float4 per block
  const int aux = (flags & 16) ? 2 : 0;
  if (w == 0) {
    float x = threadIdx.x * 1e-3f, y = 1.0001f;
    for (int step = 0; step < 4; ++step) {
      if (flags & 2048) {
        for (int i = 0; i < spin; ++i) x = chain<1, 700>(x, y);
      } else {
        for (int i = 0; i < spin; ++i) {
          x = __builtin_fmaf(x, y, 1e-7f);
          y = __builtin_fmaf(y, 0.99999f, x * 1e-9f);
        }
      }
      __syncthreads();  // R
    }
    s1 = __builtin_amdgcn_s_memrealtime();
    for (int c = threadIdx.x; c < EPB * 45; c += 64) frame[c] = x + c;
    __syncthreads();  // F
    s2 = __builtin_amdgcn_s_memrealtime();
    if (!(flags & 4)) {
      const int e = e0 + (threadIdx.x >> 1), leg = threadIdx.x & 1;
      auto rs = __builtin_amdgcn_make_buffer_rsrc(F, 0, -1, 0x00020000);
#pragma unroll 8
      for (int f = 0; f < NF / 2; ++f)
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, x + f), rs, (e + leg * (NF / 2) * N) * 4,
                                              f * N * 4, 0);
    }
    s3 = __builtin_amdgcn_s_memrealtime();
  } else {
    const int t = threadIdx.x - 64, nt = 128;
    auto rd = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, -1, 0x00020000);
    auto wr = __builtin_amdgcn_make_buffer_rsrc((void*)dst, 0, -1, 0x00020000);
    float hx = t * 1e-3f;
    for (int step = 0; step < 4; ++step) {
      if (flags & 2048) {
        if (w == 1) hx = chain<2, 450>(hx, 1.0001f);
        else hx = chain<3, 300>(hx, 1.0001f);
      }
      __syncthreads();  // R
      if (!(flags & 1) && !(flags & 64) && step < 3) {
        const int k0 = step * F4 / 3, k1 = (step + 1) * F4 / 3;
        for (int j = k0 + t; j < k1; j += nt) {
          auto v = __builtin_amdgcn_raw_buffer_load_b128(rd, j * 16, 0, 0);
          if (aux) __builtin_amdgcn_raw_buffer_store_b128(v, wr, j * 16, 0, 2); else __builtin_amdgcn_raw_buffer_store_b128(v, wr, j * 16, 0, 0);
        }
      }
    }
    s1 = __builtin_amdgcn_s_memrealtime();
    if (!(flags & 2)) __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();  // F
    s2 = __builtin_amdgcn_s_memrealtime();
    if (!(flags & 1) && (flags & 64)) {
      for (int j = t; j < F4; j += nt) {
        auto v = __builtin_amdgcn_raw_buffer_load_b128(rd, j * 16, 0, 0);
        if (aux) __builtin_amdgcn_raw_buffer_store_b128(v, wr, j * 16, 0, 2); else __builtin_amdgcn_raw_buffer_store_b128(v, wr, j * 16, 0, 0);
      }
    }
    if (!(flags & 8)) {
      float* d = obs + (size_t)e0 * ROW;
      for (int wv = t; wv < EPB * 45; wv += nt) {
        const int r = wv / 45, c = wv - r * 45;
        d[r * ROW + c * 10 + 9] = frame[wv] + hx * 1e-30f;
      }
    }
    if ((flags & (256 | 512 | 1024)) && t < 17) {
      const float v = frame[t] + 1.f;
      if (flags & 256) logp[t * gridDim.x + blockIdx.x] = v;
      else if (flags & 512) logp[t * gridDim.x + blk] = v;
      else logp[blk * 64 + t] = v;
    }
    s3 = __builtin_amdgcn_s_memrealtime();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  s4 = __builtin_amdgcn_s_memrealtime();
  unsigned xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  if ((threadIdx.x & 63) == 0) {
    Stamp& o = st[blockIdx.x * 3 + w];
    o.t[0] = s0; o.t[1] = s1; o.t[2] = s2; o.t[3] = s3; o.t[4] = s4; o.t[5] = xcc & 15u;
  }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

int main(int argc, char** argv) {
  const int spin = argc > 1 ? atoi(argv[1]) : 700;
  const int launches = 40;
  float *obsA, *obsB, *F, *logp;
  Stamp* st;
  CK(hipMalloc(&obsA, sizeof(float) * N * ROW));
  CK(hipMalloc(&obsB, sizeof(float) * N * ROW));
  CK(hipMalloc(&F, sizeof(float) * N * NF));
  CK(hipMalloc(&st, sizeof(Stamp) * NB * 3));
  CK(hipMalloc(&logp, sizeof(float) * NB * 64));
  CK(hipMemset(obsA, 0, sizeof(float) * N * ROW));
  CK(hipMemset(obsB, 0, sizeof(float) * N * ROW));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  std::vector<Stamp> h(NB * 3);
  const int variants[] = {2048, 2048 | 1, 2048 | 4, 0};
  for (int flags : variants) {
    double sum_ms = 0;
    std::vector<std::vector<double>> phys(8), tailv(8), fwait(8), hack(8);
    for (int it = 0; it < 10 + launches; ++it) {
      const bool swap = !(flags & 128) && (it & 1);
      CK(hipEventRecord(a, 0));
      hipLaunchKernelGGL(tail_kernel, dim3(NB), dim3(192), 0, 0, swap ? obsB : obsA, swap ? obsA : obsB, F, st, flags,
                         spin, logp);
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      if (it < 10) continue;
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      sum_ms += ms;
      CK(hipMemcpy(h.data(), st, sizeof(Stamp) * NB * 3, hipMemcpyDeviceToHost));
      unsigned long long t0 = ~0ull;
      for (auto& s : h) t0 = std::min(t0, s.t[0]);
      for (int blk = 0; blk < NB; ++blk) {
        const Stamp& p = h[blk * 3];
        const int x = (int)p.t[5] & 7;
        phys[x].push_back((p.t[1] - p.t[0]) / 100.0);
        fwait[x].push_back((p.t[2] - p.t[1]) / 100.0);
        tailv[x].push_back((p.t[4] - p.t[1]) / 100.0);
        hack[x].push_back((h[blk * 3 + 1].t[2] - h[blk * 3 + 1].t[1]) / 100.0);
      }
    }
    auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v.empty() ? 0.0 : v[v.size() / 2]; };
    printf("flags %3d  kernel %.2f us | per XCC: spin / F-wait / tail after spin (physics wave) / helper wait before F\n",
           flags, 1e3 * sum_ms / launches);
    for (int x = 0; x < 8; ++x)
      printf("   xcc %d  %6.2f  %6.2f  %6.2f  %6.2f\n", x, med(phys[x]), med(fwait[x]), med(tailv[x]), med(hack[x]));
    fflush(stdout);
  }
  return 0;
}
