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

#include <type_traits>

// Diagnostic builds (-DPT_DIAG=1, tools/ only: ptamd/build.py builds them as
// libptcell_diag.so) honour the PT_CELL_ABLATE phase / precision switches,
// PT_CELL_DEBUG_STOP and pt_cell_trace.  In the release library every switch
// test below is a compile-time 0: the environment cannot alter a result.
#ifndef PT_DIAG
#define PT_DIAG 0
#endif
#define PT_ABL(x) (PT_DIAG ? (x) : 0)

// Kernel-variant switches (the A/B experiments of DESIGN.md §9: PT_CELL_FUSED,
// PT_PWB2, PT_WG16, PT_LCONV_FAST, ...): PT_SW(name, default) reads the
// environment variable `name` (its first digit) in the diagnostic builds only.
// The release libraries compile every switch to its default -- the name is not
// even in the binary -- so the environment cannot change which kernels run.
#if PT_DIAG
#include <stdlib.h>
inline int pt_sw_env(const char* name, int dflt) {
  const char* e = getenv(name);
  return e && e[0] >= '0' && e[0] <= '9' ? e[0] - '0' : dflt;
}
#define PT_SW(name, dflt) pt_sw_env(name, dflt)
#else
#define PT_SW(name, dflt) (dflt)
#endif

namespace ptc {

constexpr int C = 32;          // channels (MFMA tile width)
constexpr int IMG = 32;        // H = W = 32
constexpr int NPIX = IMG * IMG;
constexpr int PADMAX = 3;      // halo for k <= 7 (the engine's k = 7: the fast path)
constexpr int TILE = IMG + 2 * PADMAX;   // 38
constexpr int PADBIG = 7;      // halo for 9 <= k <= 15 (the reference constructors' default k = 15)
template <int PAD> constexpr int tile_w() { return IMG + 2 * PAD; }   // 38 / 46
constexpr int pad_for(int K) { return K <= 2 * PADMAX + 1 ? PADMAX : PADBIG; }
constexpr int NT = 256;        // threads per block
constexpr int NWAVE = NT / 64;
constexpr int RPW = IMG / NWAVE;         // image rows per wave (8)
constexpr int MAXTAP = 49;     // taps at PAD = PADMAX (k <= 7)

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16_t;
typedef __bf16 bf16x16 __attribute__((ext_vector_type(16)));
// native 16-B vector (HIP's uint4 is a struct whose copies lower to memcpy,
// which can pin arrays of it in scratch)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

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

// bf16 from global memory by 4-B loads of the channel pair, the lane's half
// picked by one v_perm_b32 (PT_LD32, default): the 2-B loads
// (global_load_ushort) returned zeros in one 16-lane quarter of a load now and
// then on some boxes (tools/det_locate.py: dcE = 0 at one pixel, channels
// 16-31), which the dword loads of the f32 path never did.  Same instruction
// count; the perm replaces the shift that widened the 2-B load.
#ifndef PT_LD32
#define PT_LD32 1
#endif
__device__ __forceinline__ uint32_t bf16_sel(int c) { return (c & 1) ? 0x03020c0cu : 0x01000c0cu; }
__device__ __forceinline__ float ldg(const float* p) { return *p; }
__device__ __forceinline__ float ldg(const bf16_t* p) {
#if PT_LD32
  const uintptr_t a = (uintptr_t)p;
  const uint32_t w = *(const uint32_t*)(a & ~(uintptr_t)3);
  return __uint_as_float((a & 2) ? (w & 0xffff0000u) : (w << 16));
#else
  return (float)*p;
#endif
}

// Load / store one CL row tile from a channels-last [32 px][32 ch] row.
template <class S>
__device__ __forceinline__ f32x16 load_cl(const S* __restrict__ row, int c, int h) {
  f32x16 v;
#if PT_LD32
  if constexpr (sizeof(S) == 2) {
    const uint32_t* w = (const uint32_t*)(row + (c & ~1));      // 64-B aligned rows
    const uint32_t sel = bf16_sel(c);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const uint32_t x = w[cl_x(r, h) * (C / 2)];
      v[r] = __uint_as_float(__builtin_amdgcn_perm(x, x, sel));
    }
    return v;
  }
#endif
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = ldf(row + cl_x(r, h) * C + c);
  return v;
}
template <class S>
__device__ __forceinline__ void store_cl(S* __restrict__ row, int c, int h, const f32x16& v) {
#pragma unroll
  for (int r = 0; r < 16; ++r) stf(row + cl_x(r, h) * C + c, v[r]);
}

// Packed CL row tile in the storage type (bf16: 8 VGPRs instead of 16):
// loaded tensors that stay live across a kernel's long middle part are kept
// packed and widened at each use.
template <class S> struct PkT;
template <> struct PkT<float> { using type = f32x16; };
template <> struct PkT<bf16_t> { using type = bf16x16; };
template <class S> using Pk = typename PkT<S>::type;
template <class S>
__device__ __forceinline__ Pk<S> load_pk(const S* __restrict__ row, int c, int h) {
  Pk<S> v;
#if PT_LD32
  if constexpr (sizeof(S) == 2) {
    const uint32_t* w = (const uint32_t*)(row + (c & ~1));
    // elements r (low half) and r + 1 (high half) of one packed register
    const uint32_t sel = (c & 1) ? 0x07060302u : 0x05040100u;
    typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));
    u32x8 pk;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint32_t lo = w[cl_x(2 * k, h) * (C / 2)], hi = w[cl_x(2 * k + 1, h) * (C / 2)];
      pk[k] = __builtin_amdgcn_perm(hi, lo, sel);
    }
    return __builtin_bit_cast(Pk<S>, pk);
  }
#endif
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = row[cl_x(r, h) * C + c];
  return v;
}
template <class S> __device__ __forceinline__ Pk<S> to_pk(const f32x16& v) {
  Pk<S> o;
#pragma unroll
  for (int r = 0; r < 16; ++r) o[r] = (S)v[r];
  return o;
}
template <class S> __device__ __forceinline__ Pk<S> zero_pk() {
  Pk<S> v;
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = (S)0.f;
  return v;
}

// PL ("pixel on lane"): the C/D layout of the transposed product D^T[n][p]
// (conv kernels put the weights on the A side): lane l -> pixel p = l & 31,
// half h = l >> 5; reg r -> channel pl_ch(r, h) = (r & 3) + 8 (r >> 2) + 4 h.
// A lane's 16 channels are 4 runs of 4 contiguous channels, so a row tile
// moves with 4 x 16 B (f32) / 4 x 8 B (bf16) accesses per lane.
__device__ __forceinline__ int pl_ch(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// px: pointer to channel 0 of this lane's pixel in a channels-last image.
__device__ __forceinline__ void store_pl(float* __restrict__ px, int h, const f32x16& v) {
#pragma unroll
  for (int g = 0; g < 4; ++g)
    *(f32x4*)(px + 8 * g + 4 * h) = f32x4{v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]};
}
__device__ __forceinline__ void store_pl(bf16_t* __restrict__ px, int h, const f32x16& v) {
#pragma unroll
  for (int g = 0; g < 4; ++g)
    *(bf16x4*)(px + 8 * g + 4 * h) = bf16x4{(bf16_t)v[4 * g], (bf16_t)v[4 * g + 1],
                                            (bf16_t)v[4 * g + 2], (bf16_t)v[4 * g + 3]};
}
// Streaming (nontemporal) form of store_pl for outputs written once per launch.
__device__ __forceinline__ void store_pl_nt(float* __restrict__ px, int h, const f32x16& v) {
#pragma unroll
  for (int g = 0; g < 4; ++g)
    __builtin_nontemporal_store(f32x4{v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]},
                                (f32x4*)(px + 8 * g + 4 * h));
}
__device__ __forceinline__ void store_pl_nt(bf16_t* __restrict__ px, int h, const f32x16& v) {
#pragma unroll
  for (int g = 0; g < 4; ++g)
    __builtin_nontemporal_store(bf16x4{(bf16_t)v[4 * g], (bf16_t)v[4 * g + 1], (bf16_t)v[4 * g + 2],
                                       (bf16_t)v[4 * g + 3]},
                                (bf16x4*)(px + 8 * g + 4 * h));
}
__device__ __forceinline__ void add_pl(const float* __restrict__ px, int h, f32x16& v) {
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const f32x4 a = *(const f32x4*)(px + 8 * g + 4 * h);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[4 * g + j] += a[j];
  }
}
__device__ __forceinline__ void add_pl(const bf16_t* __restrict__ px, int h, f32x16& v) {
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const bf16x4 a = *(const bf16x4*)(px + 8 * g + 4 * h);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[4 * g + j] += (float)a[j];
  }
}

// Sum a PL tile's 16 registers over the 32 pixel lanes of each half by
// recursive halving (16 cross-lane moves instead of 5 x 16): on return lane l
// holds the total of register pl_sum_reg(l) (channel pl_ch(pl_sum_reg(l), h));
// lanes l and l ^ 16 hold the same value.
__device__ __forceinline__ int pl_sum_reg(int lane) {
  const int q = lane & 15;
  return 8 * (q & 1) + 4 * ((q >> 1) & 1) + 2 * ((q >> 2) & 1) + ((q >> 3) & 1);
}
// Each halving step selects between two NAMED values: written as
// (b ? v[j + 8] : v[j]) LLVM folds the pair into one dynamic element index and
// lowers it as a 16-way compare/select chain (~1200 VALU per wave in the conv
// epilogue, ~4.6 us per launch); pin() keeps both extracts static.
__device__ __forceinline__ void pin(float& x, float& y) { asm volatile("" : "+v"(x), "+v"(y)); }
__device__ __forceinline__ float pl_lane_sum(const f32x16& v, int lane) {
  float a[8], b[4], c[2];
  const bool b0 = lane & 1, b1 = lane & 2, b2 = lane & 4, b3 = lane & 8;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float lo = v[j], hi = v[j + 8];
    pin(lo, hi);
    a[j] = (b0 ? hi : lo) + __shfl_xor(b0 ? lo : hi, 1);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float lo = a[j], hi = a[j + 4];
    pin(lo, hi);
    b[j] = (b1 ? hi : lo) + __shfl_xor(b1 ? lo : hi, 2);
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    float lo = b[j], hi = b[j + 2];
    pin(lo, hi);
    c[j] = (b2 ? hi : lo) + __shfl_xor(b2 ? lo : hi, 4);
  }
  float lo = c[0], hi = c[1];
  pin(lo, hi);
  const float d = (b3 ? hi : lo) + __shfl_xor(b3 ? lo : hi, 8);
  return d + __shfl_xor(d, 16);
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
// Raw v_exp_f32 / v_log_f32 (2^x, log2 x): __expf/__logf add a denormal
// range fix-up (cmp + cndmask + ldexp) around every call; no argument here
// needs it (results that would be denormal flush to 0, which is harmless for
// 1 + e^x, sigmoid and tanh).
// (r04: each transcendental as inline asm with a wait state on either side
// was tried against the run-to-run divergence and did not remove it; the cause
// was the packed-FP32 pair reads, DESIGN.md §4 / ptamd/build.py.)
__device__ __forceinline__ float hw_exp2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ float hw_log2(float x) { return __builtin_amdgcn_logf(x); }
__device__ __forceinline__ float hw_rcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float fexp(float x) { return hw_exp2(x * 1.4426950408889634f); }
__device__ __forceinline__ float flog(float x) { return hw_log2(x) * 0.6931471805599453f; }
__device__ __forceinline__ float frcp(float x) { return hw_rcp(x); }
__device__ __forceinline__ float sigm(float x) { return frcp(1.f + fexp(-x)); }
// sigmoid(x + b) with nb = sig_nb(b) precomputed: the bias add and the 2^x
// scaling fold into one FMA
constexpr float L2E = 1.4426950408889634f;
__device__ __forceinline__ float sig_nb(float b) { return -b * L2E; }
__device__ __forceinline__ float sigm_b(float x, float nb) {
  return frcp(1.f + hw_exp2(fmaf(x, -L2E, nb)));
}
__device__ __forceinline__ float ftanh(float x) {
  const float t = 1.f - 2.f * frcp(fexp(2.f * fabsf(x)) + 1.f);
  return copysignf(t, x);
}
// Compile-time activation (a runtime switch made the compiler branch around
// every transcendental).  Branch-free: both sides are computed and selected.
//   softplus: f = x > 20 ? x : log(1 + e^x);  f' = x > 20 ? 1 : e^x / (1 + e^x)
//             (as max(log(1 + e^min(x, 20)), x) and e / (1 + e) at e = e^min(x, 20):
//             the selects folded, r04; equal to within an ulp)
//   tanh    : f = tanh x;                     f' = 1 - tanh^2 x
template <int ACT> struct Act;
template <> struct Act<0> {
  __device__ static __forceinline__ float f(float x) {
    // log(1 + e^x) > x for every x, and at the clamp (x > 20) it is 20.0: the
    // threshold select is a max
    return fmaxf(flog(1.f + fexp(fminf(x, 20.f))), x);
  }
  __device__ static __forceinline__ float d(float x) {
    // e / (1 + e) at the clamp (x > 20) is 1 to within an ulp: no select
    const float e = fexp(fminf(x, 20.f));
    return e * frcp(1.f + e);
  }
  // f and f' from one exponential
  __device__ static __forceinline__ void fd(float x, float& f, float& d) {
    const float e = fexp(fminf(x, 20.f));
    const float s = 1.f + e;
    const float lf = flog(s), ld = e * frcp(s);
    f = fmaxf(lf, x);
    d = ld;
  }
};
template <> struct Act<1> {
  __device__ static __forceinline__ float f(float x) { return ftanh(x); }
  __device__ static __forceinline__ float d(float x) {
    const float t = ftanh(x);
    return 1.f - t * t;
  }
  __device__ static __forceinline__ void fd(float x, float& f, float& d) {
    f = ftanh(x);
    d = 1.f - f * f;
  }
};

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

// Diagnostic rounding (PT_DIAG builds, f32 path): v as the bf16 path stores it.
__device__ __forceinline__ float rbf(bool on, float v) { return on ? (float)(bf16_t)v : v; }

template <class S, class V>
__device__ __forceinline__ void cl_to_pa(float* __restrict__ scr, const V& v, int lane,
                                         typename Tr<S>::frag (&pa)[Tr<S>::KS], bool rnd = false) {
  const int c = lane & 31, h = lane >> 5, p = lane & 31;
#pragma unroll
  for (int r = 0; r < 16; ++r) scr[scr_idx<S>(cl_x(r, h), c)] = rbf(rnd, (float)v[r]);
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
  // the fragment loads stay at their use (laundered base): hoisted out of a
  // row loop as invariants they pinned 8 VGPRs per gate for the whole loop
  asm volatile("" : "+s"(g));
#pragma unroll
  for (int s = 0; s < Tr<S>::KS; ++s) acc = Tr<S>::mma(pa[s], g[s * 64 + lane], acc);
  return acc;
}

// dW[n][ci] += sum_p D[p][n] X[p][ci] with D, X both in CL registers: the
// accumulator tiles are used directly as A (= D^T) and B operands; the k
// (pixel) order is the same permutation on both sides.
template <class S, class V>
__device__ __forceinline__ f32x16 wgrad_cl(const f32x16& d, const V& x, f32x16 acc) {
  if constexpr (sizeof(S) == 4) {
#pragma unroll
    for (int s = 0; s < 16; ++s) acc = Tr<float>::mma(d[s], (float)x[s], acc);
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
// PAD = halo width: PADMAX (38 x 38 tile) for k <= 7, PADBIG (46 x 46) above.
template <class S, int PAD = PADMAX>
__device__ __forceinline__ int tile_off(int trow, int tcol, int ch) {
  constexpr int TW = tile_w<PAD>();
  if constexpr (sizeof(S) == 4) return (trow * TW + tcol) * Tr<float>::CP + ch;
  else return (trow * TW + tcol) * 32 + ((((ch >> 3) ^ ((tcol >> 2) & 3))) << 3) + (ch & 7);
}
template <class S, int PAD = PADMAX>
__host__ __device__ constexpr int tile_bytes() {
  return tile_w<PAD>() * tile_w<PAD>() * Tr<S>::CP * (int)sizeof(S);
}

template <class S, int PAD = PADMAX, int NTH = NT>
__device__ void tile_zero(S* tile, int tid) {
  uint4* p = (uint4*)tile;
  const int n = tile_bytes<S, PAD>() / 16;
  for (int i = tid; i < n; i += NTH) p[i] = make_uint4(0, 0, 0, 0);
}

// Zero only the halo ring of the tile (the fused forward writes every interior
// pixel before its conv reads the tile): 420 of 1444 pixels at PAD 3.
template <class S, int PAD = PADMAX, int NTH = NT>
__device__ void tile_zero_halo(S* tile, int tid) {
  constexpr int TW = tile_w<PAD>(), PXB = Tr<S>::CP * (int)sizeof(S), CPP = PXB / 16;  // 16-B chunks per pixel
  constexpr int NH = 2 * PAD * TW + 2 * PAD * IMG;
  for (int i = tid; i < NH * CPP; i += NTH) {
    const int hp = i / CPP, q = i - hp * CPP;
    int r, c;
    if (hp < 2 * PAD * TW) { const int j = hp / TW; r = j < PAD ? j : IMG + j; c = hp - j * TW; }
    else { const int k = hp - 2 * PAD * TW, j = k / (2 * PAD); r = PAD + j; const int m = k - j * 2 * PAD; c = m < PAD ? m : IMG + m; }
    *(uint4*)((char*)tile + (r * TW + c) * PXB + q * 16) = make_uint4(0, 0, 0, 0);
  }
}

// Fill the tile interior with channels [pass*CP, pass*CP+CP) of a
// channels-last clip image (global, [32][32][32] of S).  All 16 loads of a
// thread are issued before any LDS store so one memory round trip covers the
// whole 64 KB image (one wave per SIMD has nothing else to hide latency with).
template <class S, int PAD = PADMAX, int NTH = NT>
__device__ __forceinline__ void tile_fill(S* __restrict__ tile, const S* __restrict__ src,
                                          int pass, int tid) {
  constexpr int CPB = 16 / (int)sizeof(S);          // channels per 16-B chunk
  constexpr int NCH = Tr<S>::CP / CPB;               // chunks per pixel
  constexpr int PER = NPIX * NCH / NTH;              // chunks per thread (16 at 256 threads)
  uint4 v[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int idx = tid + k * NTH;
    const int pix = idx / NCH, q = idx % NCH;
    v[k] = *(const uint4*)(src + pix * C + pass * Tr<S>::CP + q * CPB);
  }
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int idx = tid + k * NTH;
    const int pix = idx / NCH, q = idx % NCH;
    const int y = pix >> 5, x = pix & 31;
    *(uint4*)(tile + tile_off<S, PAD>(y + PAD, x + PAD, q * CPB)) = v[k];
  }
}

// Implicit-GEMM k x k conv over the LDS tile for this wave's RPW rows, computed
// transposed so the result lands in the PL layout (lane = pixel):
//   acc[i][n][x] += sum_{tap,ci} W[n][ci][tap] * in[row0+i+kh-pad][x+kw-pad][ci]
// Column-tap-major with row reuse: for one kernel column kw the wave walks the
// RPW+K-1 tile rows it touches; each A fragment (tile row, kw, k-step) is read
// from LDS ONCE and feeds the K MFMAs (kh = 0..K-1) of the output rows
// i = tr - kh it contributes to (K x fewer A reads than tap-major order).
// B fragments: wf is [K*K][KS][64] (prepared by k_prep).  The K taps of one
// column (one "slice", 14 KB) are staged in LDS, double-buffered: the slice of
// column kw+1 is fetched from L2 into registers at the top of column kw and
// written to LDS after its MFMAs, so no MFMA ever waits on an L2 round trip
// and each workgroup reads the weights once instead of once per wave.
#ifndef CONV_PF
#define CONV_PF 3                    // A-fragment prefetch depth (tile rows)
#endif
#ifndef CONV_PF_W
#define CONV_PF_W 5                  // the same for the register-weight (WREG) flat pipeline
#endif
// 1 (default): one software pipeline over all (kernel column, tile row) steps
// of a bf16 conv, the A fragments CONV_PF(_W) steps ahead across column
// boundaries too; 0: a pipeline per column, drained at every column's end.
// Same MFMA order per accumulator (bitwise equal).  Measured (interleaved,
// B=256 T=64): fused fa / fb 73.8 / 51.9 -> 72.7 / 51.4 us, conv_ba / conv_bb
// 34.0 / 38.6 -> 33.3 / 37.9 us; A depth 5 on the register-weight path
// another -0.6 / -0.4 us on fa / fb (6 lost on conv_ba).
#ifndef PT_CONV_FLAT
#define PT_CONV_FLAT 1
#endif
#ifndef PT_CONV_NOWRELOAD
#define PT_CONV_NOWRELOAD 0          // timing experiments only (wrong results): column 0's weights for every column
#endif
#ifndef PT_BAND_LEAD
#define PT_BAND_LEAD 5               // banded backward conv: addend loads, tile-row steps ahead (r05: 0 / 3 / 5 = conv_bb 38.9 / 35.8 / 35.5 us)
#endif
#ifndef PT_BAND_XNOADD
#define PT_BAND_XNOADD 0
#endif
#ifndef PT_BAND_XNOFILL
#define PT_BAND_XNOFILL 0
#endif
#ifndef PT_CONV_ROT
#define PT_CONV_ROT 1                // register-weight pipeline: one rotating fragment set (below)
#endif
constexpr int WSLICE_CHUNKS = 896;   // 16-B chunks per slice: 7 taps x 2 x 64 x 16 B (bf16)
                                     //                       = 7 taps x 8 x 64 x 4 B (f32, per pass)
constexpr int WSLICE_BYTES = WSLICE_CHUNKS * 16;
template <int NTH> constexpr int wslice_per() { return (WSLICE_CHUNKS + NTH - 1) / NTH; }  // 4 / 2

// A slice in flight: four named chunks (an array here ends up in scratch).
struct WSlice { u32x4 v0, v1, v2, v3; };
template <int J> __device__ __forceinline__ u32x4& wsl(WSlice& w) {
  if constexpr (J == 0) return w.v0;
  else if constexpr (J == 1) return w.v1;
  else if constexpr (J == 2) return w.v2;
  else return w.v3;
}
static_assert(wslice_per<NT>() == 4, "WSlice holds 4 chunks per thread");

template <class S, int K, int J, int NTH>
__device__ __forceinline__ void wslice_load1(WSlice& r, const typename Tr<S>::frag* __restrict__ wf,
                                             int pass, int kw, int tid) {
  using TT = Tr<S>;
  constexpr int KSP = TT::KS / TT::NPASS;
  constexpr int RC = 64 * (int)sizeof(typename TT::frag) / 16;   // chunks per (tap, k-step) row
  constexpr int N = K * KSP * RC;
  // unconditional (clamped) loads: predicated ones get parked in scratch
  const int e = tid + J * NTH < N ? tid + J * NTH : N - 1;
  const int kh = e / (KSP * RC), rem = e - kh * (KSP * RC);
  const int s = rem / RC, q = rem - s * RC;
  wsl<J>(r) = ((const u32x4*)(wf + ((kh * K + kw) * TT::KS + pass * KSP + s) * 64))[q];
}
template <class S, int K, int NTH = NT>
__device__ __forceinline__ void wslice_load(WSlice& r, const typename Tr<S>::frag* __restrict__ wf,
                                            int pass, int kw, int tid) {
  constexpr int PER = wslice_per<NTH>();
  wslice_load1<S, K, 0, NTH>(r, wf, pass, kw, tid);
  if constexpr (PER > 1) wslice_load1<S, K, 1, NTH>(r, wf, pass, kw, tid);
  if constexpr (PER > 2) wslice_load1<S, K, 2, NTH>(r, wf, pass, kw, tid);
  if constexpr (PER > 3) wslice_load1<S, K, 3, NTH>(r, wf, pass, kw, tid);
}
template <int K, int NTH = NT>
__device__ __forceinline__ void wslice_store(WSlice& r, char* buf, int tid) {
  constexpr int PER = wslice_per<NTH>();
  static_assert(PER <= 4, "WSlice holds at most 4 chunks per thread");
  u32x4* b = (u32x4*)buf;
  if (PER > 1 || tid < WSLICE_CHUNKS) b[tid] = r.v0;
  if constexpr (PER > 1) { if (PER > 2 || tid + NTH < WSLICE_CHUNKS) b[tid + NTH] = r.v1; }
  if constexpr (PER > 2) { if (PER > 3 || tid + 2 * NTH < WSLICE_CHUNKS) b[tid + 2 * NTH] = r.v2; }
  if constexpr (PER > 3) { if (tid + 3 * NTH < WSLICE_CHUNKS) b[tid + 3 * NTH] = r.v3; }
}

// Row-final hook: called as done(i, acc[i]) the moment output row i has
// received its last MFMA (last pass, last kernel column, tile row i + K - 1),
// so an epilogue can store row i while the later rows' MFMAs still run.
// A hook may also prefetch (prefetch_active): called once, at the first kernel
// column right after the next weight slice's loads are issued, so the loads
// it issues overlap the MFMA loop and never delay the fill or the slices.
struct NoRowHook {
  __device__ __forceinline__ void operator()(int, const f32x16&) const {}
  __device__ __forceinline__ void prefetch() const {}
  static constexpr bool active = false;
  static constexpr bool prefetch_active = false;
  static constexpr bool wreg = false;
};

// Row-final hooks with a per-row pre-load (row_pre_lead = L > 0): pre(i) is
// called L tile-row steps before done(i), in the last kernel column.
template <class D, class = void> struct RowPreLead { static constexpr int v = 0; };
template <class D> struct RowPreLead<D, std::void_t<decltype(D::row_pre_lead)>> {
  static constexpr int v = D::row_pre_lead;
};
template <class D> __device__ __forceinline__ void row_pre(const D& d, int i) {
  if constexpr (RowPreLead<D>::v > 0) d.pre(i);
}

// Compile-time loop: fn(std::integral_constant<int, I>) for I in [I0, N), so
// every register-array index derived from I is a constant (a #pragma unroll
// the compiler declines would leave dynamic indices, i.e. scratch).
template <int I, int N, class Fn>
__device__ __forceinline__ void static_for(Fn&& fn) {
  if constexpr (I < N) {
    fn(std::integral_constant<int, I>{});
    static_for<I + 1, N>(fn);
  }
}

// k > 7 (PAD = PADBIG): the 46 x 46 tile leaves no LDS for weight slices;
// every wave reads its column's K x KSP B fragments straight from L2 at the
// top of the column (the ~K * RPW * KSP MFMAs of the column cover the fetch).
template <class S, int K, int PAD, int RW, int NTH, class Fill, class Done = NoRowHook, bool BAR = true>
__device__ __forceinline__ void conv_run_k(f32x16 (&acc)[RW], Fill& fill,
                                           const typename Tr<S>::frag* __restrict__ wf, S* tile,
                                           char* wbuf, int row0, int lane, int tid, int ablate,
                                           const Done& done = Done()) {
  using TT = Tr<S>;
  using F = typename TT::frag;
  // Done::wreg (k <= 7): each wave reads its B fragments from L2 into
  // registers one column ahead instead of the LDS slice ring -- no
  // workgroup barrier per column
  constexpr bool WREG = Done::wreg && K <= 2 * PADMAX + 1;
  constexpr bool LDSW = K <= 2 * PADMAX + 1 && !WREG;  // weight slices staged in LDS
  constexpr int KSP = TT::KS / TT::NPASS;   // k-steps per pass per tap
  constexpr int off = PAD - K / 2;
  constexpr int NTR = RW + K - 1;           // tile rows touched by this wave
  const int h = lane >> 5, px = lane & 31;
#if PT_CONV_FLAT
  // One software pipeline over all (column, tile row) steps: the A fragments
  // run CONV_PF steps ahead ACROSS column boundaries too (the per-column
  // loop below drains its prefetch at the end of every column), and the
  // column fragments alternate between two register sets (no copies).
  if constexpr (WREG && TT::NPASS == 1) {
    // PT_CONV_ROT (r05): ONE register set of column fragments, kernel row kd
    // of column kw + 1 reloaded into bw[kd] right after output row RW - 1 has
    // taken column kw's (step (kw, tr = kd + RW - 1)); its first use, step
    // (kw + 1, kd), is NTR - RW + 1 steps later.  The two-set form (column
    // kw + 1 loaded whole at the top of column kw) spilled.
    constexpr int NSET = PT_CONV_ROT ? 1 : 2;
    F bw[NSET][K][KSP];
    auto load_colw = [&](int kw, F (&dst)[K][KSP]) {
#pragma unroll
      for (int kh = 0; kh < K; ++kh)
#pragma unroll
        for (int s = 0; s < KSP; ++s) dst[kh][s] = wf[((kh * K + kw) * TT::KS + s) * 64 + lane];
    };
    load_colw(0, bw[0]);
    if constexpr (BAR) {      // (!BAR: the caller filled the tile and synchronised)
      __syncthreads();
      if (!(PT_ABL(ablate) & 2)) fill(0);
      __syncthreads();
    }
    if (PT_ABL(ablate) & 1) return;
    constexpr int NST = K * NTR;
    constexpr int PF = CONV_PF_W < NST ? CONV_PF_W : NST;
    F av[PF + 1][KSP];
    auto load_step = [&](int st) {
      const int kw = st / NTR, tr = st - kw * NTR;
      const int trow = row0 + tr + off, tcol = px + kw + off;
#pragma unroll
      for (int s = 0; s < KSP; ++s)
        av[st % (PF + 1)][s] = *(const F*)(tile + tile_off<S, PAD>(trow, tcol, 16 * s + 8 * h));
    };
    static_for<0, PF>([&](auto c) { load_step(decltype(c)::value); });
    static_for<0, NST>([&](auto c) {
      constexpr int st = decltype(c)::value;
      constexpr int kw = st / NTR, tr = st - kw * NTR;
      if constexpr (tr == 0) {
        if constexpr (NSET == 2 && kw + 1 < K) load_colw(kw + 1, bw[(kw + 1) % NSET]);
        if constexpr (Done::prefetch_active && kw == 0) done.prefetch();
      }
      if constexpr (st + PF < NST) load_step(st + PF);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int s = 0; s < KSP; ++s)
#pragma unroll
        for (int kh = 0; kh < K; ++kh) {
          const int i = tr - kh;
          if (i >= 0 && i < RW) acc[i] = TT::mma(bw[kw % NSET][kh][s], av[st % (PF + 1)][s], acc[i]);
        }
      if constexpr (NSET == 1 && kw + 1 < K && tr >= RW - 1 && tr - (RW - 1) < K && !PT_CONV_NOWRELOAD) {
        constexpr int kd = tr - (RW - 1);
#pragma unroll
        for (int s = 0; s < KSP; ++s) bw[0][kd][s] = wf[((kd * K + kw + 1) * TT::KS + s) * 64 + lane];
      }
      if constexpr (Done::active && RowPreLead<Done>::v > 0 && kw == K - 1) {
        // row i's pre-load at step tr = i + K - 1 - lead of the last column,
        // or at its first step when that is earlier (k < lead + 2: without
        // the clamp rows 0 .. lead - k + 1 never had their addends loaded)
        constexpr int L = RowPreLead<Done>::v;
        if constexpr (tr == 0) {
          static_for<0, RW>([&](auto c) {
            constexpr int i = decltype(c)::value;
            if constexpr (i + K - 1 - L <= 0) row_pre(done, i);
          });
        } else {
          constexpr int ip = tr - (K - 1) + L;
          if constexpr (ip >= 0 && ip < RW) row_pre(done, ip);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (Done::active && kw == K - 1 && tr >= K - 1 && tr - (K - 1) < RW)
        done(tr - (K - 1), acc[tr - (K - 1)]);
    });
    return;
  }
  // the LDS slice ring (k <= 7 without register weights: the backward convs),
  // same single pipeline: the A fragments of the next column are in flight
  // across the column's slice hand-off barrier
  if constexpr (LDSW && TT::NPASS == 1) {
    WSlice pre;
    wslice_load<S, K, NTH>(pre, wf, 0, 0, tid);
    __syncthreads();
    if (!(PT_ABL(ablate) & 2)) fill(0);
    wslice_store<K, NTH>(pre, wbuf, tid);
    __syncthreads();
    if (PT_ABL(ablate) & 1) return;
    constexpr int NST = K * NTR;
    constexpr int PF = CONV_PF < NST ? CONV_PF : NST;
    F av[PF + 1][KSP];
    F bc[K][KSP];
    auto load_step = [&](int st) {
      const int kw = st / NTR, tr = st - kw * NTR;
      const int trow = row0 + tr + off, tcol = px + kw + off;
#pragma unroll
      for (int s = 0; s < KSP; ++s)
        av[st % (PF + 1)][s] = *(const F*)(tile + tile_off<S, PAD>(trow, tcol, 16 * s + 8 * h));
    };
    static_for<0, PF>([&](auto c) { load_step(decltype(c)::value); });
    static_for<0, NST>([&](auto c) {
      constexpr int st = decltype(c)::value;
      constexpr int kw = st / NTR, tr = st - kw * NTR;
      if constexpr (tr == 0) {
        if constexpr (kw > 0) {                 // publish column kw's slice
          wslice_store<K, NTH>(pre, wbuf + (kw & 1) * WSLICE_BYTES, tid);
          __syncthreads();
        }
        const F* wl = (const F*)(wbuf + (kw & 1) * WSLICE_BYTES) + lane;
#pragma unroll
        for (int kh = 0; kh < K; ++kh)
#pragma unroll
          for (int s = 0; s < KSP; ++s) bc[kh][s] = wl[(kh * KSP + s) * 64];
        if constexpr (kw + 1 < K) wslice_load<S, K, NTH>(pre, wf, 0, kw + 1, tid);
        if constexpr (Done::prefetch_active && kw == 0) done.prefetch();
      }
      if constexpr (st + PF < NST) load_step(st + PF);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int s = 0; s < KSP; ++s)
#pragma unroll
        for (int kh = 0; kh < K; ++kh) {
          const int i = tr - kh;
          if (i >= 0 && i < RW) acc[i] = TT::mma(bc[kh][s], av[st % (PF + 1)][s], acc[i]);
        }
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (Done::active && kw == K - 1 && tr >= K - 1 && tr - (K - 1) < RW)
        done(tr - (K - 1), acc[tr - (K - 1)]);
    });
    return;
  }
#endif
  F bn[K][KSP];                             // WREG: the next column's fragments
  auto load_col = [&](int pass, int kw) {
#pragma unroll
    for (int kh = 0; kh < K; ++kh)
#pragma unroll
      for (int s = 0; s < KSP; ++s) bn[kh][s] = wf[((kh * K + kw) * TT::KS + pass * KSP + s) * 64 + lane];
  };
  if constexpr (WREG) load_col(0, 0);
  for (int pass = 0; pass < TT::NPASS; ++pass) {
    WSlice pre;
    if constexpr (LDSW) wslice_load<S, K, NTH>(pre, wf, pass, 0, tid);
    __syncthreads();
    if (!(PT_ABL(ablate) & 2)) fill(pass);
    if constexpr (LDSW) wslice_store<K, NTH>(pre, wbuf, tid);
    __syncthreads();
    if (PT_ABL(ablate) & 1) continue;
    for (int kw = 0; kw < K; ++kw) {
      F bc[K][KSP];
      if constexpr (LDSW) {
        const F* wl = (const F*)(wbuf + (kw & 1) * WSLICE_BYTES) + lane;
        if (kw + 1 < K && !(PT_ABL(ablate) & 16384)) wslice_load<S, K, NTH>(pre, wf, pass, kw + 1, tid);
        if constexpr (Done::prefetch_active)
          if (kw == 0 && pass == TT::NPASS - 1) done.prefetch();
#pragma unroll
        for (int kh = 0; kh < K; ++kh)
#pragma unroll
          for (int s = 0; s < KSP; ++s) bc[kh][s] = wl[(kh * KSP + s) * 64];
      } else if constexpr (WREG) {
#pragma unroll
        for (int kh = 0; kh < K; ++kh)
#pragma unroll
          for (int s = 0; s < KSP; ++s) bc[kh][s] = bn[kh][s];
        if (kw + 1 < K) load_col(pass, kw + 1);
        else if (pass + 1 < TT::NPASS) load_col(pass + 1, 0);
        if constexpr (Done::prefetch_active)
          if (kw == 0 && pass == TT::NPASS - 1) done.prefetch();
      } else {
#pragma unroll
        for (int kh = 0; kh < K; ++kh)
#pragma unroll
          for (int s = 0; s < KSP; ++s)
            bc[kh][s] = wf[((kh * K + kw) * TT::KS + pass * KSP + s) * 64 + lane];
        if constexpr (Done::prefetch_active)
          if (kw == 0 && pass == TT::NPASS - 1) done.prefetch();
      }
      const int tcol = px + kw + off;
      // A fragments of tile row tr, software-pipelined CONV_PF rows ahead of
      // their MFMAs (one wave per SIMD: nothing else hides LDS latency)
      F av[NTR][KSP];
      auto load_a = [&](int tr) {
        const int trow = row0 + tr + off;
#pragma unroll
        for (int s = 0; s < KSP; ++s) {
          if constexpr (sizeof(S) == 4) {
            av[tr][s] = tile[tile_off<S, PAD>(trow, tcol, 2 * s + h)];
          } else {
            av[tr][s] = *(const bf16x8*)(tile + tile_off<S, PAD>(trow, tcol, 16 * s + 8 * h));
          }
        }
      };
      constexpr int PF = CONV_PF < NTR ? CONV_PF : NTR;
#pragma unroll
      for (int tr = 0; tr < PF; ++tr) load_a(tr);
#pragma unroll
      for (int tr = 0; tr < NTR; ++tr) {
        if (tr + PF < NTR) load_a(tr + PF);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s = 0; s < KSP; ++s) {
          // D^T[n][p] += W[n][k] X^T[k][p]: weights on A, pixels on B -> PL output
#pragma unroll
          for (int kh = 0; kh < K; ++kh) {
            const int i = tr - kh;
            if (i >= 0 && i < RW) acc[i] = TT::mma(bc[kh][s], av[tr][s], acc[i]);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (Done::active) {
          const int i = tr - (K - 1);
          if (i >= 0 && i < RW && kw == K - 1 && pass == TT::NPASS - 1) done(i, acc[i < 0 ? 0 : i]);
        }
      }
      if constexpr (LDSW) {
        if (kw + 1 < K && !(PT_ABL(ablate) & 16384)) {
          wslice_store<K, NTH>(pre, wbuf + ((kw + 1) & 1) * WSLICE_BYTES, tid);
          __syncthreads();
        }
      }
    }
  }
}

template <class S, int PAD, int RW = RPW, int NTH = NT, class Fill, class Done = NoRowHook>
__device__ __forceinline__ void conv_run(f32x16 (&acc)[RW], Fill& fill,
                                         const typename Tr<S>::frag* __restrict__ wf, S* tile,
                                         char* wbuf, int K, int row0, int lane, int tid,
                                         int ablate, const Done& done = Done()) {
  if constexpr (PAD == PADMAX) {
    switch (K) {
      case 7: conv_run_k<S, 7, PAD, RW, NTH>(acc, fill, wf, tile, wbuf, row0, lane, tid, ablate, done); break;
      case 5: conv_run_k<S, 5, PAD, RW, NTH>(acc, fill, wf, tile, wbuf, row0, lane, tid, ablate, done); break;
      case 3: conv_run_k<S, 3, PAD, RW, NTH>(acc, fill, wf, tile, wbuf, row0, lane, tid, ablate, done); break;
      default: conv_run_k<S, 1, PAD, RW, NTH>(acc, fill, wf, tile, wbuf, row0, lane, tid, ablate, done); break;
    }
  } else {
    switch (K) {
      case 15: conv_run_k<S, 15, PAD, RW, NTH>(acc, fill, wf, tile, wbuf, row0, lane, tid, ablate, done); break;
      case 13: conv_run_k<S, 13, PAD, RW, NTH>(acc, fill, wf, tile, wbuf, row0, lane, tid, ablate, done); break;
      case 11: conv_run_k<S, 11, PAD, RW, NTH>(acc, fill, wf, tile, wbuf, row0, lane, tid, ablate, done); break;
      default: conv_run_k<S, 9, PAD, RW, NTH>(acc, fill, wf, tile, wbuf, row0, lane, tid, ablate, done); break;
    }
  }
}

// The register-weight pipeline without its workgroup barriers (the caller has
// filled the tile and synchronised the waves that read it): k <= 7, bf16.
template <class S, int RW, int NTH, class Done>
__device__ __forceinline__ void conv_run_nobar(f32x16 (&acc)[RW], const typename Tr<S>::frag* __restrict__ wf,
                                               S* tile, int K, int row0, int lane, int tid, int ablate,
                                               const Done& done) {
  static_assert(Done::wreg, "the barrier-free form is the register-weight pipeline");
  auto nofill = [](int) {};
  switch (K) {
    case 7: conv_run_k<S, 7, PADMAX, RW, NTH, decltype(nofill), Done, false>(acc, nofill, wf, tile, nullptr, row0, lane, tid, ablate, done); break;
    case 5: conv_run_k<S, 5, PADMAX, RW, NTH, decltype(nofill), Done, false>(acc, nofill, wf, tile, nullptr, row0, lane, tid, ablate, done); break;
    case 3: conv_run_k<S, 3, PADMAX, RW, NTH, decltype(nofill), Done, false>(acc, nofill, wf, tile, nullptr, row0, lane, tid, ablate, done); break;
    default: conv_run_k<S, 1, PADMAX, RW, NTH, decltype(nofill), Done, false>(acc, nofill, wf, tile, nullptr, row0, lane, tid, ablate, done); break;
  }
}

// Zero-fill as a kernel node.  The captured launch sequences used
// hipMemsetAsync; replayed as part of a hipGraph, the 54 MB slab clear was
// not reliably ordered before the kernels that accumulate into the slab
// (tools/nan_hunt.py: non-finite slab-derived gradients on some replays of
// a cached graph, never with direct launches).
__global__ void k_zero(uint32_t* __restrict__ p, size_t n_words) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t n16 = n_words / 4;
  for (size_t j = i; j < n16; j += stride) ((u32x4*)p)[j] = u32x4{0u, 0u, 0u, 0u};
  for (size_t j = n16 * 4 + i; j < n_words; j += stride) p[j] = 0u;
}
inline hipError_t zero_async(void* p, size_t bytes, hipStream_t st) {
  // every cleared region is a multiple of 4 bytes and 16-byte aligned (256-B plan offsets)
  const size_t words = bytes / 4;
  size_t blocks = (words / 4 + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(k_zero, dim3((unsigned)blocks), dim3(256), 0, st, (uint32_t*)p, words);
  return hipGetLastError();
}

}  // namespace ptc
