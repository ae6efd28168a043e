// pt_pr.h — the half-row "PR" (channel pair) register layout of the r04
// backward point-wise kernels (k_pw_bb2), gfx950.
//
// One wave = 16 pixels x 32 channels of an image row (half a row):
//   lane l -> channel pair n = l & 15 (channels 2n, 2n + 1), pixel group g = l >> 4
//   element e = 4 k + i (i < 4, k < 2) -> pixel 4 g + i of the half row, channel 2 n + k
//   (k-major: the two 16x16 MFMA C/D tiles are elements 0-3 and 4-7)
// 8 values per lane (f32x8) instead of the CL layout's 16, so a row tile costs
// half the VGPRs and the kernels run 4 waves per SIMD instead of 2.
//   * HBM: a pixel's channel pair is one dword (bf16) / two (f32): 4 loads or
//     stores per tile and lane, no lane-select permutes.
//   * Per-channel parameters and sums: 2 registers per quantity; a sum over the
//     half row is lane-local over i, then two cross-lane steps (xor 16, 32).
//   * 1x1 gates Y = X G^T: the 16x16 MFMA's C/D tile is exactly this layout
//     (lane -> column n, registers -> rows 4 g + i) when rows are pixels and the
//     columns of output tile k are the channels 2n + k; the A operand (8
//     channels of one pixel per lane) is the tile transposed through a per-wave
//     LDS scratch.
//   * 1x1 weight gradients dW = D^T X: the operand tiles are staged
//     channel-major in LDS ([ch][px], 8 contiguous pixels per 16 B), so the
//     contraction's A and B fragments are plain 16-B reads.
// MFMA flavours: bf16 v_mfma_f32_16x16x32_bf16 (one K step of 32 channels);
// f32 v_mfma_f32_16x16x4_f32 (8 steps; the exact parity path).
#pragma once
#include "pt_device.h"

namespace ptc {

typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

constexpr int HR = 16;                 // pixels per half row

template <class S> struct T16;
template <> struct T16<bf16_t> {
  using frag = bf16x8;
  static constexpr int KS = 1;         // K steps per 32-channel contraction
  __device__ static inline f32x4 mma(frag a, frag b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct T16<float> {
  using frag = float;
  static constexpr int KS = 8;
  __device__ static inline f32x4 mma(frag a, frag b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
};

__device__ __forceinline__ f32x8 zero8() {
  f32x8 v;
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = 0.f;
  return v;
}

// A packed tile as stored: bf16 -> 4 dwords (dword i: elements i and 4 + i,
// the channel pair of pixel i), f32 -> f32x8.
template <class S> struct PrPkT;
template <> struct PrPkT<bf16_t> { using type = u32x4; };
template <> struct PrPkT<float> { using type = f32x8; };
template <class S> using PrPk = typename PrPkT<S>::type;

// seg: channel 0 of pixel 0 of the half row in a channels-last [px][32] row
template <class S>
__device__ __forceinline__ PrPk<S> pr_load_pk(const S* __restrict__ seg, int lane) {
  const int n = lane & 15, g = lane >> 4;
  if constexpr (sizeof(S) == 2) {
    const uint32_t* w = (const uint32_t*)seg + (4 * g) * (C / 2) + n;
    u32x4 v;
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = w[i * (C / 2)];
    return v;
  } else {
    const f32x2* w = (const f32x2*)seg + (4 * g) * (C / 2) + n;
    f32x8 v;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const f32x2 p = w[i * (C / 2)];
      v[i] = p[0];
      v[4 + i] = p[1];
    }
    return v;
  }
}
__device__ __forceinline__ f32x8 pr_widen(const u32x4& p) {
  f32x8 v;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[i] = __uint_as_float(p[i] << 16);
    v[4 + i] = __uint_as_float(p[i] & 0xffff0000u);
  }
  return v;
}
__device__ __forceinline__ f32x8 pr_widen(const f32x8& p) { return p; }
template <class S>
__device__ __forceinline__ f32x8 pr_load(const S* __restrict__ seg, int lane) {
  return pr_widen(pr_load_pk<S>(seg, lane));
}
__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
  const bf16x2 v = {(bf16_t)a, (bf16_t)b};
  return __builtin_bit_cast(uint32_t, v);
}
template <class S>
__device__ __forceinline__ void pr_store(S* __restrict__ seg, int lane, const f32x8& v) {
  const int n = lane & 15, g = lane >> 4;
  if constexpr (sizeof(S) == 2) {
    uint32_t* w = (uint32_t*)seg + (4 * g) * (C / 2) + n;
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i * (C / 2)] = pk_bf16(v[i], v[4 + i]);
  } else {
    f32x2* w = (f32x2*)seg + (4 * g) * (C / 2) + n;
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i * (C / 2)] = f32x2{v[i], v[4 + i]};
  }
}
// this lane's two channels of a per-channel parameter vector
__device__ __forceinline__ f32x2 pr_par(const float* __restrict__ p, int lane) {
  return *((const f32x2*)p + (lane & 15));
}

// ------------------------------------------------------------- 1x1 gates
// Per-wave transpose scratch: the half-row tile as [16 px][32 ch] in S with a
// padded row (bf16: 80 B, f32: 136 B), so that the pair writes (lane (n, g),
// pixel 4g + i) and the A-fragment reads (lane: pixel l & 15, channels
// 8 (l >> 4) ..) are bank-conflict free.
template <class S> constexpr int prs_stride() { return sizeof(S) == 2 ? 40 : 34; }   // elements
template <class S> constexpr int prs_bytes() { return HR * prs_stride<S>() * (int)sizeof(S); }

template <class S> struct PrA { typename T16<S>::frag f[T16<S>::KS]; };

// The A operand (pixel rows, channel K) of a PR tile.  All waves call this
// for their own scratch; the reads follow the writes in the same wave.
template <class S, class V>
__device__ __forceinline__ PrA<S> pr_to_a(S* __restrict__ scr, const V& v, int lane) {
  const int n = lane & 15, g = lane >> 4, p = lane & 15, kg = lane >> 4;
  PrA<S> a;
  if constexpr (sizeof(S) == 2) {
    uint32_t* w = (uint32_t*)scr;
#pragma unroll
    for (int i = 0; i < 4; ++i) w[(4 * g + i) * (prs_stride<S>() / 2) + n] = pk_bf16(v[i], v[4 + i]);
    wave_sync();
    a.f[0] = *(const bf16x8*)(scr + p * prs_stride<S>() + 8 * kg);
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      *(f32x2*)(scr + (4 * g + i) * prs_stride<S>() + 2 * n) = f32x2{(float)v[i], (float)v[4 + i]};
    wave_sync();
#pragma unroll
    for (int s = 0; s < 8; ++s) a.f[s] = scr[p * prs_stride<S>() + 4 * s + kg];
  }
  wave_sync();
  return a;
}
// acc += A G'^T for a prepared gate (fragments [k 2][KS][64 lanes], see k_prep:
// column n of output tile k is channel 2n + k).
template <class S>
__device__ __forceinline__ f32x8 pr_mm(const PrA<S>& a, const typename T16<S>::frag* __restrict__ g16,
                                       f32x8 acc, int lane) {
  asm volatile("" : "+s"(g16));       // the fragment loads stay at their use
  f32x4 d0 = __builtin_shufflevector(acc, acc, 0, 1, 2, 3);
  f32x4 d1 = __builtin_shufflevector(acc, acc, 4, 5, 6, 7);
#pragma unroll
  for (int s = 0; s < T16<S>::KS; ++s) {
    d0 = T16<S>::mma(a.f[s], g16[(0 * T16<S>::KS + s) * 64 + lane], d0);
    d1 = T16<S>::mma(a.f[s], g16[(1 * T16<S>::KS + s) * 64 + lane], d1);
  }
  return __builtin_shufflevector(d0, d1, 0, 1, 2, 3, 4, 5, 6, 7);
}

// --------------------------------------------------- 1x1 weight gradients
// Operand tiles staged channel-major: [32 ch][NPX + 8 pad] in S for the NPX
// pixels of a workgroup; a wave writes its half row (16 pixels at column
// offset px0) as 2 x 8-B (bf16) / 2 x 16-B (f32) stores per channel pair.
template <class S, int NPX> constexpr int stg_stride() { return NPX + (sizeof(S) == 2 ? 8 : 4); }
template <class S, int NPX> constexpr int stg_bytes() { return C * stg_stride<S, NPX>() * (int)sizeof(S); }

template <class S, int NPX, class V>
__device__ __forceinline__ void pr_stage(S* __restrict__ stg, const V& v, int px0, int lane) {
  const int n = lane & 15, g = lane >> 4;
  constexpr int SS = stg_stride<S, NPX>();
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    S* row = stg + (2 * n + k) * SS + px0 + 4 * g;
    if constexpr (sizeof(S) == 2) {
      *(u32x2*)row = u32x2{pk_bf16(v[4 * k], v[4 * k + 1]), pk_bf16(v[4 * k + 2], v[4 * k + 3])};
    } else {
      *(f32x4*)row = f32x4{(float)v[4 * k], (float)v[4 * k + 1], (float)v[4 * k + 2], (float)v[4 * k + 3]};
    }
  }
}
// One wave: dW[16 mt + r][16 nt + c] += sum over the NPX staged pixels of
// D[p][.] X[p][.] for output tiles (mt, nt), nt = 0, 1 (two f32x4: lane l reg
// i -> row 16 mt + 4 (l >> 4) + i, column 16 nt + (l & 15)).
template <class S, int NPX>
__device__ __forceinline__ void pr_wgrad_acc(const S* __restrict__ dst, const S* __restrict__ xst, int mt,
                                             f32x4 (&acc)[2], int lane) {
  constexpr int SS = stg_stride<S, NPX>();
  const int r = lane & 15, kg = lane >> 4;
  if constexpr (sizeof(S) == 2) {
    const S* da = dst + (16 * mt + r) * SS + 8 * kg;
    const S* x0 = xst + r * SS + 8 * kg;
    const S* x1 = xst + (16 + r) * SS + 8 * kg;
#pragma unroll
    for (int kb = 0; kb < NPX / 32; ++kb) {
      const bf16x8 a = *(const bf16x8*)(da + 32 * kb);
      const bf16x8 b0 = *(const bf16x8*)(x0 + 32 * kb), b1 = *(const bf16x8*)(x1 + 32 * kb);
      acc[0] = T16<S>::mma(a, b0, acc[0]);
      acc[1] = T16<S>::mma(a, b1, acc[1]);
    }
  } else {
    const S* da = dst + (16 * mt + r) * SS + kg;
    const S* x0 = xst + r * SS + kg;
    const S* x1 = xst + (16 + r) * SS + kg;
#pragma unroll 4
    for (int kb = 0; kb < NPX / 4; ++kb) {
      const float a = da[4 * kb];
      acc[0] = T16<S>::mma(a, x0[4 * kb], acc[0]);
      acc[1] = T16<S>::mma(a, x1[4 * kb], acc[1]);
    }
  }
}

// Sum over the 16 pixels of the half row (lane-local over i, then over the
// 4 pixel groups): every lane ends with the totals of its channel pair.
__device__ __forceinline__ f32x2 pr_hsum(const f32x8& v) {
  f32x2 s = {v[0] + v[1] + v[2] + v[3], v[4] + v[5] + v[6] + v[7]};
  s[0] += __shfl_xor(s[0], 16);
  s[1] += __shfl_xor(s[1], 16);
  s[0] += __shfl_xor(s[0], 32);
  s[1] += __shfl_xor(s[1], 32);
  return s;
}

}  // namespace ptc
