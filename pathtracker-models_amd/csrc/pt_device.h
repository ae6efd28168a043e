// pt_device.h — gfx950 device building blocks for the recurrent-cell kernels.
//
// Register layouts used throughout (one wave = one 32-pixel image row):
//
//  CL ("channel on lane")  the C/D layout of a 32x32 MFMA tile whose rows are
//      the 32 pixels of a row and whose columns are the 32 channels:
//        lane l -> channel c = l & 31, half h = l >> 5
//        reg  r -> pixel   x = (r & 3) + 8 (r >> 2) + 4 h
//      Every per-pixel tensor lives in this layout (f32x16 per lane), so
//      per-channel parameters are ONE register per lane and BatchNorm sums are
//      lane-local.
//
//  PA ("pixel on A")  the A-operand layout of the same tile: lane l holds
//      pixel p = l & 31 and, at k-step s, the channels frag_chan<S>(s, h, j).
//      Needed where a 1x1 conv contracts over channels; produced from CL by a
//      per-wave LDS transpose (cl_to_pa).
//
// MFMA flavours (storage type S):
//   S = float  : v_mfma_f32_32x32x2_f32   (exact f32, parity path; 16 k-steps / 32 ch)
//   S = __bf16 : v_mfma_f32_32x32x16_bf16 (f32 accumulate; 2 k-steps / 32 ch)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ptc {

constexpr int C = 32;          // channels (MFMA tile width)
constexpr int IMG = 32;        // H = W = 32
constexpr int NPIX = IMG * IMG;
constexpr int PADMAX = 3;      // halo for k <= 7
constexpr int TILE = IMG + 2 * PADMAX;   // 38
constexpr int NT = 256;        // threads per block
constexpr int NWAVE = NT / 64;
constexpr int RPW = IMG / NWAVE;         // image rows per wave (8)
constexpr int MAXTAP = 49;

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16_t;

template <class S> struct Tr;
template <> struct Tr<float> {
  using frag = float;
  static constexpr int KS = 16;     // k-steps per 32-channel contraction
  static constexpr int EPL = 1;     // fragment elements per lane
  static constexpr int CP = 16;     // channels per conv pass held in LDS
  static constexpr int NPASS = 2;
  __device__ static inline f32x16 mma(frag a, frag b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
  }
};
template <> struct Tr<bf16_t> {
  using frag = bf16x8;
  static constexpr int KS = 2;
  static constexpr int EPL = 8;
  static constexpr int CP = 32;
  static constexpr int NPASS = 1;
  __device__ static inline f32x16 mma(frag a, frag b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
};

// Channel carried by element j of a lane in half h at k-step s.
template <class S> __host__ __device__ constexpr int frag_chan(int s, int h, int j);
template <> __host__ __device__ constexpr int frag_chan<float>(int s, int h, int) { return 2 * s + h; }
template <> __host__ __device__ constexpr int frag_chan<bf16_t>(int s, int h, int j) {
  return 16 * s + 8 * h + j;
}

__device__ __forceinline__ int cl_x(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

__device__ __forceinline__ float ldf(const float* p) { return *p; }
__device__ __forceinline__ float ldf(const bf16_t* p) { return (float)*p; }
__device__ __forceinline__ void stf(float* p, float v) { *p = v; }
__device__ __forceinline__ void stf(bf16_t* p, float v) { *p = (bf16_t)v; }

// Load / store one CL row tile from a channels-last [32 px][32 ch] row.
template <class S>
__device__ __forceinline__ f32x16 load_cl(const S* __restrict__ row, int c, int h) {
  f32x16 v;
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = ldf(row + cl_x(r, h) * C + c);
  return v;
}
template <class S>
__device__ __forceinline__ void store_cl(S* __restrict__ row, int c, int h, const f32x16& v) {
#pragma unroll
  for (int r = 0; r < 16; ++r) stf(row + cl_x(r, h) * C + c, v[r]);
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 v;
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = 0.f;
  return v;
}

// Consume per-row accumulators in a non-unrolled row loop without dynamic
// register indexing (which LLVM would lower to scratch): use a[0], then shift.
template <int N>
__device__ __forceinline__ void shift_rows(f32x16 (&a)[N]) {
#pragma unroll
  for (int k = 0; k + 1 < N; ++k) a[k] = a[k + 1];
}

__device__ __forceinline__ float hsum16(const f32x16& v) {
  float s = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) s += v[r];
  return s;
}

// ---------------------------------------------------------------- activations
// nl = softplus(beta=1, threshold=20) or tanh (models/InT.py:184, engine.py:145).
// Hardware exp/log/rcp (v_exp_f32 / v_log_f32 / v_rcp_f32, ~1 ulp): absolute
// deviations from libm are O(1e-7), far inside the 1e-3 parity bound.
__device__ __forceinline__ float fexp(float x) { return __expf(x); }
__device__ __forceinline__ float frcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float sigm(float x) { return frcp(1.f + fexp(-x)); }
__device__ __forceinline__ float ftanh(float x) {
  const float t = 1.f - 2.f * frcp(fexp(2.f * fabsf(x)) + 1.f);
  return copysignf(t, x);
}
__device__ __forceinline__ float act_f(float x, int act) {
  if (act == 0) return x > 20.f ? x : __logf(1.f + fexp(x));
  return ftanh(x);
}
__device__ __forceinline__ float act_d(float x, int act) {   // d nl / d x
  if (act == 0) return x > 20.f ? 1.f : sigm(x);
  const float t = ftanh(x);
  return 1.f - t * t;
}

// --------------------------------------------------------- per-wave transpose
// 32x32 f32 scratch with a padded row stride: the CL write (fixed pixel per
// half-wave, 32 consecutive channels) and the PA read (32 pixels, same
// channels) are both bank-conflict free, and every address is a per-lane base
// plus a compile-time offset (no per-register address VGPRs to hoist/spill).
//   f32 reads  (ds_read_b32,  lane = pixel): stride 33 -> banks (p + k) % 32
//   bf16 reads (ds_read_b128, 8 channels)  : stride 36 -> 16-B aligned rows,
//            slot (9p + q) % 16 distinct within every 16-lane group
template <class S> constexpr int scr_stride() { return sizeof(S) == 4 ? 33 : 36; }
constexpr int SCR_FLOATS = 32 * 36;     // per wave
template <class S> __device__ __forceinline__ int scr_idx(int p, int c) {
  return p * scr_stride<S>() + c;
}

__device__ __forceinline__ void wave_sync() {
  // DS instructions of one wave execute in order; this only pins the compiler.
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

template <class S>
__device__ __forceinline__ void cl_to_pa(float* __restrict__ scr, const f32x16& v, int lane,
                                         typename Tr<S>::frag (&pa)[Tr<S>::KS]) {
  const int c = lane & 31, h = lane >> 5, p = lane & 31;
#pragma unroll
  for (int r = 0; r < 16; ++r) scr[scr_idx<S>(cl_x(r, h), c)] = v[r];
  wave_sync();
  if constexpr (sizeof(S) == 4) {
#pragma unroll
    for (int s = 0; s < Tr<S>::KS; ++s) pa[s] = scr[scr_idx<float>(p, 2 * s + h)];
  } else {
#pragma unroll
    for (int s = 0; s < Tr<S>::KS; ++s) {
      const f32x4 lo = *(const f32x4*)(scr + scr_idx<S>(p, 16 * s + 8 * h));
      const f32x4 hi = *(const f32x4*)(scr + scr_idx<S>(p, 16 * s + 8 * h + 4));
      bf16x8 f;
#pragma unroll
      for (int j = 0; j < 4; ++j) { f[j] = (bf16_t)lo[j]; f[4 + j] = (bf16_t)hi[j]; }
      pa[s] = f;
    }
  }
  wave_sync();
}

// Y[p][n] += sum_c X[p][c] G[n][c]; X in PA, G as prepared B fragments [KS][64].
template <class S>
__device__ __forceinline__ f32x16 gemm_pa(const typename Tr<S>::frag (&pa)[Tr<S>::KS],
                                          const typename Tr<S>::frag* __restrict__ g, f32x16 acc,
                                          int lane) {
#pragma unroll
  for (int s = 0; s < Tr<S>::KS; ++s) acc = Tr<S>::mma(pa[s], g[s * 64 + lane], acc);
  return acc;
}

// dW[n][ci] += sum_p D[p][n] X[p][ci] with D, X both in CL registers: the
// accumulator tiles are used directly as A (= D^T) and B operands; the k
// (pixel) order is the same permutation on both sides.
template <class S>
__device__ __forceinline__ f32x16 wgrad_cl(const f32x16& d, const f32x16& x, f32x16 acc) {
  if constexpr (sizeof(S) == 4) {
#pragma unroll
    for (int s = 0; s < 16; ++s) acc = Tr<float>::mma(d[s], x[s], acc);
  } else {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 fa, fb;
#pragma unroll
      for (int j = 0; j < 8; ++j) { fa[j] = (bf16_t)d[8 * s + j]; fb[j] = (bf16_t)x[8 * s + j]; }
      acc = Tr<bf16_t>::mma(fa, fb, acc);
    }
  }
  return acc;
}

// -------------------------------------------------------------- conv LDS tile
// [TILE rows][TILE cols][CP channels] of S, zero halo.  bf16: 16-B chunks of
// 8 channels XOR-swizzled by (col >> 2) & 3 so the 32 lanes of an A-fragment
// read (consecutive columns, same chunk) hit distinct bank groups.
template <class S> __device__ __forceinline__ int tile_off(int trow, int tcol, int ch);
template <> __device__ __forceinline__ int tile_off<float>(int trow, int tcol, int ch) {
  return (trow * TILE + tcol) * Tr<float>::CP + ch;
}
template <> __device__ __forceinline__ int tile_off<bf16_t>(int trow, int tcol, int ch) {
  return (trow * TILE + tcol) * 32 + ((((ch >> 3) ^ ((tcol >> 2) & 3))) << 3) + (ch & 7);
}
template <class S>
__host__ __device__ constexpr int tile_bytes() {
  return TILE * TILE * Tr<S>::CP * (int)sizeof(S);
}

template <class S>
__device__ void tile_zero(S* tile, int tid) {
  uint4* p = (uint4*)tile;
  const int n = tile_bytes<S>() / 16;
  for (int i = tid; i < n; i += NT) p[i] = make_uint4(0, 0, 0, 0);
}

// Fill the tile interior with channels [pass*CP, pass*CP+CP) of a
// channels-last clip image (global, [32][32][32] of S).  All 16 loads of a
// thread are issued before any LDS store so one memory round trip covers the
// whole 64 KB image (one wave per SIMD has nothing else to hide latency with).
template <class S>
__device__ __forceinline__ void tile_fill(S* __restrict__ tile, const S* __restrict__ src,
                                          int pass, int tid) {
  constexpr int CPB = 16 / (int)sizeof(S);          // channels per 16-B chunk
  constexpr int NCH = Tr<S>::CP / CPB;               // chunks per pixel
  constexpr int PER = NPIX * NCH / NT;               // chunks per thread (16)
  uint4 v[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int idx = tid + k * NT;
    const int pix = idx / NCH, q = idx % NCH;
    v[k] = *(const uint4*)(src + pix * C + pass * Tr<S>::CP + q * CPB);
  }
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int idx = tid + k * NT;
    const int pix = idx / NCH, q = idx % NCH;
    const int y = pix >> 5, x = pix & 31;
    *(uint4*)(tile + tile_off<S>(y + PADMAX, x + PADMAX, q * CPB)) = v[k];
  }
}

// Implicit-GEMM k x k conv over the LDS tile for this wave's RPW rows:
//   acc[i][x][n] += sum_{tap,ci} in[row0+i+kh-pad][x+kw-pad][ci] * W[n][ci][tap]
// wf: B fragments [K*K][KS][64] (prepared by k_prep), streamed from L2 with a
// two-tap-deep register prefetch so each tap's 16 (bf16) MFMAs never wait on
// a global load.  `fill(pass)` writes the tile interior (channels of that
// pass); the caller has zeroed the halo.
template <class S, int K, class Fill>
__device__ __forceinline__ void conv_run_k(f32x16 (&acc)[RPW], Fill& fill,
                                           const typename Tr<S>::frag* __restrict__ wf, S* tile,
                                           int row0, int lane, int ablate) {
  using TT = Tr<S>;
  using F = typename TT::frag;
  constexpr int KSP = TT::KS / TT::NPASS;   // k-steps per pass per tap
  constexpr int KK = K * K;
  constexpr int off = PADMAX - K / 2;
  const int h = lane >> 5, px = lane & 31;
  for (int pass = 0; pass < TT::NPASS; ++pass) {
    __syncthreads();
    if (!(ablate & 2)) fill(pass);
    __syncthreads();
    if (ablate & 1) continue;
    const F* w = wf + pass * KSP * 64 + lane;
    F b0[KSP], b1[KSP], b2[KSP];
#pragma unroll
    for (int s = 0; s < KSP; ++s) {
      b0[s] = w[(0 * TT::KS + s) * 64];
      b1[s] = w[((KK > 1 ? 1 : 0) * TT::KS + s) * 64];
    }
    for (int tap = 0; tap < KK; ++tap) {
      const int tn = tap + 2 < KK ? tap + 2 : KK - 1;
#pragma unroll
      for (int s = 0; s < KSP; ++s) b2[s] = w[(tn * TT::KS + s) * 64];
      const int kh = tap / K, kw = tap - kh * K;
      const int tcol = px + kw + off;
#pragma unroll
      for (int s = 0; s < KSP; ++s) {
#pragma unroll
        for (int i = 0; i < RPW; ++i) {
          const int trow = row0 + i + kh + off;
          F a;
          if constexpr (sizeof(S) == 4) {
            a = tile[tile_off<S>(trow, tcol, 2 * s + h)];
          } else {
            a = *(const bf16x8*)(tile + tile_off<S>(trow, tcol, 16 * s + 8 * h));
          }
          acc[i] = TT::mma(a, b0[s], acc[i]);
        }
      }
#pragma unroll
      for (int s = 0; s < KSP; ++s) { b0[s] = b1[s]; b1[s] = b2[s]; }
    }
  }
}

template <class S, class Fill>
__device__ __forceinline__ void conv_run(f32x16 (&acc)[RPW], Fill& fill,
                                         const typename Tr<S>::frag* __restrict__ wf, S* tile,
                                         int K, int row0, int lane, int ablate) {
  switch (K) {
    case 7: conv_run_k<S, 7>(acc, fill, wf, tile, row0, lane, ablate); break;
    case 5: conv_run_k<S, 5>(acc, fill, wf, tile, row0, lane, ablate); break;
    case 3: conv_run_k<S, 3>(acc, fill, wf, tile, row0, lane, ablate); break;
    default: conv_run_k<S, 1>(acc, fill, wf, tile, row0, lane, ablate); break;
  }
}

}  // namespace ptc
