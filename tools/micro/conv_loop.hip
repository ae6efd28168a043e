// Micro-benchmark of the register-weight 7x7 conv loop (pt_device.h
// conv_run_nobar, the MFMA phase of k_fused_fa / k_fused_fb / k_conv_bwd_band2)
// in isolation: the tile already in LDS, the weight fragments in global memory
// (L2-resident, as in the cell), nothing else running.  Per wave: 4 output
// rows x 49 taps x 2 k-steps = 392 v_mfma_f32_32x32x16_bf16 (32 cycles each
// at the issue bound).  Reports shader cycles per MFMA per SIMD (s_memtime
// around the loop, wave 0 of every workgroup) for 4 waves per workgroup (one
// per SIMD, the band-1 conv's situation) and 8 (two per SIMD).
// -DRANDOM_DATA (r06): the tile and the weights hold pseudo-random bf16 values
// in [-1, 1) instead of constants (MFMA power depends on the operand bits),
// and each configuration also runs 200 launches back to back (sustained
// clock).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize
//        -I include -I pathtracker-models_amd/csrc tools/micro/conv_loop.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <algorithm>
#include <vector>

#include "pt_device.h"

using namespace ptc;

struct WregHook {
  __device__ __forceinline__ void operator()(int, const f32x16&) const {}
  __device__ __forceinline__ void prefetch() const {}
  static constexpr bool active = false;
  static constexpr bool prefetch_active = false;
  static constexpr bool wreg = true;
};

template <int NW>
__global__ __launch_bounds__(NW * 64, 1) void k_loop(const Tr<bf16_t>::frag* __restrict__ wf, float* out,
                                                     unsigned long long* cyc) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* tile = (bf16_t*)smem;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
#ifdef RANDOM_DATA
  for (int i = tid; i < 22 * TILE * C / 2; i += NW * 64) {   // 2 bf16 per word, [-1, 1)
    unsigned x = (unsigned)(i * 2654435761u) ^ (blockIdx.x * 40503u);
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    const unsigned lo = 0x3f80u | (x & 0x807fu), hi = 0x3f80u | ((x >> 16) & 0x807fu);
    ((unsigned*)tile)[i] = (lo & 0xbfffu) | ((hi & 0xbfffu) << 16);
  }
#else
  for (int i = tid; i < 22 * TILE * C / 8; i += NW * 64) ((uint4*)tile)[i] = make_uint4(0x3f803f80u, 0, 0x3f80u, 0);
#endif
  __syncthreads();
  f32x16 acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = zero16();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  conv_run_nobar<bf16_t, 4, NW * 64>(acc, wf, tile, 7, (wave & 3) * 4, lane, tid, 0, WregHook{});
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) s += acc[i][r];
  out[blockIdx.x * NW * 64 + tid] = s;
  if (lane == 0) cyc[blockIdx.x * NW + wave] = t1 - t0;
}

template <int NW>
void run(const Tr<bf16_t>::frag* wf, float* out, unsigned long long* cyc, int grid, int lds) {
  hipFuncSetAttribute((const void*)k_loop<NW>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  hipLaunchKernelGGL(k_loop<NW>, dim3(grid), dim3(NW * 64), lds, 0, wf, out, cyc);
  hipDeviceSynchronize();
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
#ifndef REPS
#ifdef RANDOM_DATA
#define REPS 200
#else
#define REPS 20
#endif
#endif
  const int R = REPS;
  hipEventRecord(a, 0);
  for (int r = 0; r < R; ++r) hipLaunchKernelGGL(k_loop<NW>, dim3(grid), dim3(NW * 64), lds, 0, wf, out, cyc);
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  std::vector<unsigned long long> c(grid * NW);
  hipMemcpy(c.data(), cyc, c.size() * 8, hipMemcpyDeviceToHost);
  std::vector<unsigned long long> s(c);
  std::sort(s.begin(), s.end());
  const double wps = NW / 4.0 * (grid > 256 ? 2 : 1);   // waves per SIMD
  printf("waves/WG %d grid %d LDS %d KB: launch %.2f us; loop cycles per wave median %llu max %llu -> "
         "%.1f cycles per MFMA per wave, %.1f per SIMD (32 = issue bound)\n",
         NW, grid, lds / 1024, 1e3 * ms / R, s[s.size() / 2], s.back(), s[s.size() / 2] / 392.0,
         s[s.size() / 2] / (392.0 * wps));
}

int main() {
  Tr<bf16_t>::frag* wf;
  const size_t nfr = 49 * 2 * 64;
  hipMalloc(&wf, nfr * sizeof(Tr<bf16_t>::frag));
  hipMemset(wf, 0, nfr * sizeof(Tr<bf16_t>::frag));
#ifdef RANDOM_DATA
  {
    std::vector<unsigned short> hw(nfr * sizeof(Tr<bf16_t>::frag) / 2);
    unsigned x = 12345u;
    for (auto& v : hw) {
      x = x * 1664525u + 1013904223u;
      v = (unsigned short)(0x3c00u | ((x >> 9) & 0x80ffu));   // |w| in [2^-7, 2^-6), either sign
    }
    hipMemcpy(wf, hw.data(), hw.size() * 2, hipMemcpyHostToDevice);
  }
#endif
  float* out;
  hipMalloc(&out, 256 * 512 * 4);
  unsigned long long* cyc;
  hipMalloc(&cyc, 256 * 8 * 8);
  run<4>(wf, out, cyc, 256, 100 * 1024);     // one workgroup per CU, one wave per SIMD
  run<8>(wf, out, cyc, 256, 100 * 1024);     // two waves per SIMD (the same 4 rows twice)
  run<4>(wf, out, cyc, 512, 64 * 1024);      // two 4-wave workgroups per CU
  return 0;
}
