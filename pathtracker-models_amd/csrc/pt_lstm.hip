// pt_lstm.hip — ConvLSTM cell (models/convlstm.py) forward + BPTT for MI355X (gfx950).
//
// Reference path replaced (paths relative to the reference repo):
//   ConvLSTMCell.forward  models/convlstm.py:84-90     one step: 8 k x k convs + gates
//   ConvLSTM bptt loop    models/convlstm.py:137-143   `timesteps` steps on a static x
//   autograd BPTT         (loss.backward through that loop)
//   Jacobian penalty      models/convlstm.py:150-161   two one-step VJPs
//
// x is static over the steps, so its four gate convolutions are computed ONCE
// (xg = Wx * x + b, N = 4 gates x 32 padded channels = 128) and every step adds
// the h convolution P_t = xg + Wh * h_{t-1} from one implicit-GEMM kernel whose
// four waves each own one gate tile (k_lconv<.., NI=1, NO=4>).  The gate
// non-linearities and the c / h update are a point-wise kernel (k_lpw_fwd).
// BPTT runs the same conv kernel transposed (Wh^T, 4 gates in, 32 out,
// k_lconv<.., NI=4, NO=1>), a point-wise backward (k_lpw_bwd), and one
// weight-gradient kernel per conv family over all (step, image) pairs
// (k_lwgrad).  Because x is static, dWx and dx need only sum_t dP_t.
//
// Layouts (channels-last, channels padded to 32 per gate; padded channels stay
// exactly zero: zero weights / bias give P = 0 -> c stays 0, h = 0.5 tanh 0 = 0):
//   x_cl  [B][1024][32] S         xg, P_t [B][1024][128] f32 (gate g at 32 g)
//   h_t   [T][B][1024][32] S      c_t     [T][B][1024][32] f32
//   dP_t  [T][B][1024][128] S     dPsum   [B][1024][128] f32 (+ an S copy)
// The forward conv tiles the 32x32 image in 4 bands of 8 output rows; the band
// plus its (k-1)-row / (k-1)-column zero halo is one LDS tile (22 x 46 x 32
// bf16 = 63 KB at k = 15).  The transposed conv takes the whole image per
// workgroup (46 x 46 x 32 bf16 = 132 KB at k = 15).
#include "pt_device.h"
#include "pt_graph.h"
#include "../../include/pt_lstm.h"

#include <algorithm>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

namespace ptl {
using namespace ptc;

constexpr int HC = 32;             // padded hidden / input channels
constexpr int NG = 4;              // gates i, f, c, o
constexpr int GC = NG * HC;        // 128
constexpr int KMAX = 15;
// output rows per conv workgroup: 4 for the 4-gate forward (one gate tile per
// wave, 4 rows each: 132 VGPRs, two workgroups per CU hide each other's
// column-start waits; 8 rows at one wave per SIMD ran 120 us per launch), the
// whole image for the 4-gates-in transposed conv (one output tile: each wave
// takes 8 rows, reusing every LDS fragment across 8 output rows)
#ifndef PT_LCONV_RB
#define PT_LCONV_RB 4       // 4-gate rows per workgroup for f32 and k > 7 (plain column loop)
#endif
#ifndef PT_LCONV_ROT
#define PT_LCONV_ROT 1      // the column loop's weight fragments rotate in one register set
#endif
#ifndef PT_LCONVT_RB
#define PT_LCONVT_RB 32     // (experiments: 16-row bands of the transposed conv, two per CU)
#endif
#ifndef PT_LCONV_RB_FAST
#define PT_LCONV_RB_FAST 8  // bf16 k <= 7 (the rotating-weight column loop): 8 rows, one wave per gate tile
#endif
// r05: with one rotating weight set the 8-row 4-gate workgroup fits two waves
// per SIMD (224 VGPRs, no spills): each weight fragment feeds 8 output rows
// instead of 4, half the L2 weight reads per MFMA (cfg3 -0.63 ms per step,
// profiles/r05_lstmab_rb8.txt); the other shapes keep 4 rows
template <class S, int K, int NO> constexpr int conv_rb() {
  return NO == 4 ? (sizeof(S) == 2 && K <= 7 ? PT_LCONV_RB_FAST : PT_LCONV_RB) : PT_LCONVT_RB;
}
// The two-source conv (DUAL) runs the step's point-wise update in its epilogue
// only for the shapes whose epilogue exchange is written for: four gate tiles
// on four waves and a multiple of 4 output rows per wave.  The host passes the
// c / h outputs only to those instantiations (conv_dual), and skips the
// separate k_lpw_fwd launch only when it did.
template <class S, int K, int NTH> constexpr bool dual_fuses() {
  return NTH / 64 == 4 && (conv_rb<S, K, 4>() * 4 / (NTH / 64)) % 4 == 0;
}
// workgroups per CU the register budget allows (NO = 4: 4 rows per wave, two
// waves per SIMD; NO = 1: 8 rows per wave over 4 input groups, one)
#ifndef PT_LCONVT8_DEF
#define PT_LCONVT8_DEF 0    // the transposed conv on 8 waves x 4 rows (PT_LCONVT8 in diag builds)
#endif
#ifndef PT_LCONV_OCC
#define PT_LCONV_OCC 2      // 4-row 4-gate workgroups per CU (r05 experiments: 3, 161 VGPRs)
#endif
template <class S, int K, int NO> constexpr int conv_occ() {
  return NO == 4 ? PT_LCONV_OCC : (PT_LCONVT_RB == 16 ? 2 : 1);
}

// ------------------------------------------------------------------ conv tile
template <class S, int K, int RB> struct LTile {
  static constexpr int P = K / 2;
  static constexpr int TR = RB + K - 1;      // tile rows
  static constexpr int TC = IMG + K - 1;     // tile columns
  static constexpr int CP = Tr<S>::CP;       // channels per pass in LDS
  static constexpr int BYTES = TR * TC * CP * (int)sizeof(S);
  // bf16: 16-B chunks of 8 channels XOR-swizzled by (col >> 2) & 3 so the 32
  // lanes of a B-fragment read (consecutive columns) spread over bank groups
  __device__ static __forceinline__ int off(int trow, int tcol, int ch) {
    if constexpr (sizeof(S) == 4) {
      return (trow * TC + tcol) * CP + ch;
    } else {
      return (trow * TC + tcol) * 32 + ((((ch >> 3) ^ ((tcol >> 2) & 3))) << 3) + (ch & 7);
    }
  }
};

// The ConvLSTM point-wise forward of one (pixel, 4-channel quad) -- shared by
// k_lpw_fwd and the two-source conv's fused epilogue, so both run the same
// instructions.  Gates (models/convlstm.py:85-89):
//   i = sig(P_i)  f = sig(P_f)  g = tanh(P_c)  o = sig(P_o)
//   c' = f c + i g            h' = o tanh(c')
__device__ __forceinline__ void lpw_fwd_quad(const f32x4& pi, const f32x4& pf, const f32x4& pg,
                                             const f32x4& po, f32x4& c, f32x4& hn, int q, int ch) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const bool live = 4 * q + j < ch;
    const float cn = sigm(pf[j]) * c[j] + sigm(pi[j]) * ftanh(pg[j]);
    c[j] = live ? cn : 0.f;
    hn[j] = live ? sigm(po[j]) * ftanh(cn) : 0.f;
  }
}
__device__ __forceinline__ f32x4 ld4(const float* p) { return *(const f32x4*)p; }
__device__ __forceinline__ void st4(float* p, const f32x4& v) { *(f32x4*)p = v; }
__device__ __forceinline__ void st4(bf16_t* p, const f32x4& v) {
  *(bf16x4*)p = bf16x4{(bf16_t)v[0], (bf16_t)v[1], (bf16_t)v[2], (bf16_t)v[3]};
}

struct LConvArgs {
  const void* src;      // S [nimg][NPIX][32*NI]  (DUAL: input group 0, [nimg][NPIX][32])
  const void* wf;       // fragments [NO][NI][K*K][KS][64]  (DUAL: group 0's, [NO][1][K*K][KS][64])
  const void* src2;     // DUAL: input group 1, S [nimg][NPIX][32]
  const void* wf2;      // DUAL: group 1's fragments
  float* out;           // f32 [nimg][NPIX][32*NO]
  const float* add;     // f32, same layout as out, or null
  const float* bias;    // f32 [32*NO] or null
  int nimg;
  int fast;             // bf16, k <= 7: the prefetching column loop (PT_LCONV_FAST=0: the plain one)
  // DUAL with cout != null (r05): the step's point-wise update in the epilogue
  // (k_lpw_fwd's arithmetic): c_t = f c_{t-1} + i g -> cout, h_t = o tanh c_t -> hout
  const float* cprev;   // f32 [nimg][NPIX][32] or null (c_{t-1} = 0)
  float* cout;
  void* hout;           // S [nimg][NPIX][32]
  int ch;               // live channels
};

// out[img][p][32 o + n] = sum_{ig, ci, tap} W[o, ig][n][ci][tap] src[img][p + tap][32 ig + ci]
//                          (+ add) (+ bias)
// Weights on the MFMA A side, pixels on B: the result is in the PL layout
// (lane = pixel) and leaves with 16-B vector stores.  Column-tap-major loop
// with row reuse as in pt_device.h conv_run_k: each B fragment (tile row,
// kw, k-step) is read from LDS once and feeds the K MFMAs of the output rows
// it contributes to.  Wave w: output tile o = w % NO, rows (w / NO) * RW ...
// DUAL (NI = 2, r05): the two input groups come from separate tensors with
// their own fragment sets -- the per-step x-conv and h-conv of the clip
// ConvLSTM in ONE launch, P_t = Wx x_t + Wh h_{t-1} + b, instead of an
// all-steps x-conv whose P_t the h-conv then read back and rewrote.
// Issue priority by progress (r06, PT_LPRIO; the cell library's PT_PRIO 4):
// two workgroups share a CU and at equal priority the SIMD arbiter prefers the
// older wave, so the first one runs ahead and the second finishes alone; a
// workgroup lowers its priority as it progresses (3 at the start, 0 in the
// last quarter).  bit 0: k_lconv (kernel columns), bit 1: k_lwgrad (units).
#ifndef PT_LPRIO
#define PT_LPRIO 0
#endif
__device__ __forceinline__ void lprio(int done, int total) {
  const int q = total > 0 ? 3 - (4 * done) / total : 0;
  switch (q < 0 ? 0 : q) {
    case 3: __builtin_amdgcn_s_setprio(3); break;
    case 2: __builtin_amdgcn_s_setprio(2); break;
    case 1: __builtin_amdgcn_s_setprio(1); break;
    default: __builtin_amdgcn_s_setprio(0); break;
  }
}

template <class S, int K, int NI, int NO, int NTH = NT, bool DUAL = false>
__global__ __launch_bounds__(NTH, (conv_occ<S, K, NO>())) void k_lconv(LConvArgs a) {
  static_assert(!DUAL || NI == 2, "DUAL: two input groups");
  constexpr int NT = NTH, NWAVE = NTH / 64;   // (8 waves: the transposed conv at two waves per SIMD)
  using TT = Tr<S>;
  using F = typename TT::frag;
  constexpr int RB = conv_rb<S, K, NO>(), NBAND = IMG / RB;
  using L = LTile<S, K, RB>;
  constexpr int KK = K * K;
  constexpr int KSP = TT::KS / TT::NPASS;
  constexpr int RW = RB * NO / NWAVE;        // 8
  constexpr int NTR = RW + K - 1;
  constexpr int CPB = 16 / (int)sizeof(S);   // channels per 16-B chunk
  constexpr int NCH = L::CP / CPB;           // chunks per pixel per pass (4)
  constexpr int NCHUNK = L::TR * IMG * NCH;
  constexpr int PER = (NCHUNK + NT - 1) / NT;
  constexpr int SRCC = DUAL ? 32 : 32 * NI;     // channels per pixel of one source tensor
  extern __shared__ __attribute__((aligned(16))) char smem[];
  S* tile = (S*)smem;
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, px = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int img = blockIdx.x / NBAND, band = blockIdx.x % NBAND, y0 = band * RB;
  const int o = wave % NO, r0 = (wave / NO) * RW;
  const S* src = (const S*)a.src + (size_t)img * NPIX * SRCC;
  const S* src2 = DUAL ? (const S*)a.src2 + (size_t)img * NPIX * SRCC : nullptr;
  const F* wf = (const F*)a.wf;
  const F* wf2 = (const F*)a.wf2;
  // input group ig: its source pixel row base and channel offset, its fragments
  auto gsrc = [&](int ig) { return DUAL ? (ig == 0 ? src : src2) : src + ig * 32; };
  auto gwf = [&](int ig) {
    return DUAL ? (ig == 0 ? wf : wf2) + (size_t)o * KK * TT::KS * 64
                : wf + (size_t)(o * NI + ig) * KK * TT::KS * 64;
  };

  // DUAL: both groups' tiles are staged at the start, side by side (no
  // mid-kernel fill: its registers, live beside two weight columns, spilled)
  constexpr int NBUF = DUAL ? 2 : 1;
  for (int i = tid; i < NBUF * L::BYTES / 16; i += NT) ((u32x4*)tile)[i] = u32x4{0u, 0u, 0u, 0u};

  f32x16 acc[RW];
#pragma unroll
  for (int i = 0; i < RW; ++i) acc[i] = zero16();

  // bf16, k <= 7 (r04): the next kernel column's weight fragments are loaded
  // under the current column's MFMAs (ping-pong registers; loading them at the
  // column start exposed an L2 round trip per column), and the transposed
  // conv's next input group is loaded into registers under the current group's
  // columns and stored to the tile between two barriers afterwards.  Same MFMA
  // order per accumulator as the loop below (bitwise equal).
  constexpr bool FAST = sizeof(S) == 2 && K <= 7;
  bool done = false;
  if constexpr (FAST) if (a.fast) {
    done = true;
    u32x4 v[PER], v2[DUAL ? PER : 1];
    auto ld_tile = [&](int ig, u32x4 (&v)[PER]) {
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int idx0 = tid + k * NT;
        const int idx = idx0 < NCHUNK ? idx0 : NCHUNK - 1;
        const int q = idx % NCH, pc = idx / NCH, col = pc % IMG, row = pc / IMG;
        const int iy = y0 + row - L::P;
        const int cy = iy < 0 ? 0 : (iy >= IMG ? IMG - 1 : iy);
        v[k] = *(const u32x4*)(gsrc(ig) + (size_t)(cy * IMG + col) * SRCC + q * CPB);
        if (iy != cy) v[k] = u32x4{0u, 0u, 0u, 0u};
      }
    };
    auto st_tile = [&](S* tl, const u32x4 (&v)[PER]) {
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int idx = tid + k * NT;
        if (PER * NT == NCHUNK || idx < NCHUNK) {
          const int q = idx % NCH, pc = idx / NCH, col = pc % IMG, row = pc / IMG;
          *(u32x4*)(tl + L::off(row, col + L::P, q * CPB)) = v[k];
        }
      }
    };
    F wa[K][KSP], wb[K][KSP];
    auto ld_w = [&](int c, F (&w)[K][KSP]) {
      const int ig = c / K, kw = c - ig * K;
      const F* wk = gwf(ig) + (size_t)kw * TT::KS * 64 + lane;
#pragma unroll
      for (int kh = 0; kh < K; ++kh)
#pragma unroll
        for (int s2 = 0; s2 < KSP; ++s2) w[kh][s2] = wk[((size_t)kh * K * TT::KS + s2) * 64];
    };
#if PT_LCONV_ROT
    ld_w(0, wa);                           // (before the tile: both latencies at once, and the
#endif                                     // column loop starts with no weight load in flight)
    ld_tile(0, v);
    if constexpr (DUAL) ld_tile(1, v2);
    __syncthreads();                       // the clear is done
    st_tile(tile, v);
    if constexpr (DUAL) st_tile(tile + L::BYTES / sizeof(S), v2);
    __syncthreads();
    constexpr int NC = NI * K;             // (input group, kernel column) steps
    auto step = [&](int c, const F (&bc)[K][KSP], F (&nx)[K][KSP]) {
      const int ig = c / K, kw = c - ig * K;
      if (c + 1 < NC) ld_w(c + 1, nx);
      // (two workgroups per CU: the registers are not there, the other one covers the fill)
      constexpr bool TPF = conv_occ<S, K, NO>() == 1 && NTH == 256;
      if (!DUAL && TPF && NI > 1 && kw == 0 && ig + 1 < NI) ld_tile(ig + 1, v);
      const S* tl = DUAL && ig ? tile + L::BYTES / sizeof(S) : tile;
      __builtin_amdgcn_sched_barrier(0);   // the loads go out before this column's MFMAs
      const int tcol = px + kw;
      F av[NTR][KSP];
      auto load_a = [&](int tr) {
        const int trow = r0 + tr;
#pragma unroll
        for (int s2 = 0; s2 < KSP; ++s2) av[tr][s2] = *(const bf16x8*)(tl + L::off(trow, tcol, 16 * s2 + 8 * h));
      };
      constexpr int PF = 3 < NTR ? 3 : NTR;
#pragma unroll
      for (int tr = 0; tr < PF; ++tr) load_a(tr);
#pragma unroll
      for (int tr = 0; tr < NTR; ++tr) {
        if (tr + PF < NTR) load_a(tr + PF);
#pragma unroll
        for (int s2 = 0; s2 < KSP; ++s2) {
#pragma unroll
          for (int kh = 0; kh < K; ++kh) {
            const int i = tr - kh;
            if (i >= 0 && i < RW) acc[i] = TT::mma(bc[kh][s2], av[tr][s2], acc[i]);
          }
        }
      }
      if (!DUAL && NI > 1 && kw == K - 1 && ig + 1 < NI) {
        if (!TPF) ld_tile(ig + 1, v);
        __syncthreads();                   // every wave is done with this group's tile
        st_tile(tile, v);
        __syncthreads();
      }
    };
#if PT_LCONV_ROT
    // r05: ONE weight set, rotated in place -- kernel row kh's fragments are
    // dead once output row RW - 1 has taken them (tile row kh + RW - 1), and
    // the next column's kh fragments are loaded into the same registers there;
    // the first use of them is tile row kh of the next column, 6 tile rows of
    // MFMAs later.  Two sets (ping-pong) spilled the two-source conv and the
    // 8-wave transposed conv.  Same MFMA order per accumulator.
    (void)wb;
    constexpr bool TPF = conv_occ<S, K, NO>() == 1 && NTH == 256;
#pragma unroll
    for (int ig = 0; ig < NI; ++ig) {
    if (!DUAL && TPF && ig + 1 < NI) ld_tile(ig + 1, v);
#pragma unroll 1
    for (int kw = 0; kw < K; ++kw) {
      if constexpr ((PT_LPRIO & 1) != 0) lprio(ig * K + kw, NI * K);
      const S* tl = DUAL && ig ? tile + L::BYTES / sizeof(S) : tile;
      // (after the last column: a harmless reload of group 0's first column)
      const F* wkn = kw + 1 < K ? gwf(ig) + (size_t)(kw + 1) * TT::KS * 64 + lane
                                : gwf(ig + 1 < NI ? ig + 1 : 0) + lane;
      const int tcol = px + kw;
      F av[NTR][KSP];
      auto load_a = [&](int tr) {
        const int trow = r0 + tr;
#pragma unroll
        for (int s2 = 0; s2 < KSP; ++s2) av[tr][s2] = *(const bf16x8*)(tl + L::off(trow, tcol, 16 * s2 + 8 * h));
      };
      constexpr int PF = 3 < NTR ? 3 : NTR;
#pragma unroll
      for (int tr = 0; tr < PF; ++tr) load_a(tr);
#pragma unroll
      for (int tr = 0; tr < NTR; ++tr) {
        if (tr + PF < NTR) load_a(tr + PF);
#pragma unroll
        for (int s2 = 0; s2 < KSP; ++s2) {
#pragma unroll
          for (int kh = 0; kh < K; ++kh) {
            const int i = tr - kh;
            if (i >= 0 && i < RW) acc[i] = TT::mma(wa[kh][s2], av[tr][s2], acc[i]);
          }
        }
        constexpr int RWm = RW - 1;
        const int kd = tr - RWm;
        if (kd >= 0 && kd < K) {
#pragma unroll
          for (int s2 = 0; s2 < KSP; ++s2) wa[kd][s2] = wkn[((size_t)kd * K * TT::KS + s2) * 64];
        }
        __builtin_amdgcn_sched_barrier(0);   // each kernel row's reload stays where it is freed
      }
    }
    // the next input group's tile (outside the column loop: its waits then
    // stay out of the loop head)
    if (!DUAL && ig + 1 < NI) {
      if (!TPF) ld_tile(ig + 1, v);
      __syncthreads();                     // every wave is done with this group's tile
      st_tile(tile, v);
      __syncthreads();
    }
    }
#else
    ld_w(0, wa);
    for (int c = 0; c < NC; c += 2) {
      step(c, wa, wb);
      if (c + 1 < NC) step(c + 1, wb, wa);
    }
#endif
  }
  // (the release libraries run the column loop above for bf16 k <= 7: the
  // plain loop is compiled in there only for the shapes that need it, so that
  // its registers do not count against the fast one)
  if (!FAST || PT_DIAG)
  if (!done)
  for (int ig = 0; ig < NI; ++ig) {
    for (int pass = 0; pass < TT::NPASS; ++pass) {
      // ---- fill the band tile (rows outside the image are written as zeros;
      // the halo columns stay zero from the initial clear)
      u32x4 v[PER];
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int idx0 = tid + k * NT;
        const int idx = idx0 < NCHUNK ? idx0 : NCHUNK - 1;
        const int q = idx % NCH, pc = idx / NCH, col = pc % IMG, row = pc / IMG;
        const int iy = y0 + row - L::P;
        const int cy = iy < 0 ? 0 : (iy >= IMG ? IMG - 1 : iy);
        v[k] = *(const u32x4*)(gsrc(ig) + (size_t)(cy * IMG + col) * SRCC + pass * L::CP + q * CPB);
        if (iy != cy) v[k] = u32x4{0u, 0u, 0u, 0u};
      }
      __syncthreads();   // the previous pass's fragment reads are done
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int idx = tid + k * NT;
        if (PER * NT == NCHUNK || idx < NCHUNK) {
          const int q = idx % NCH, pc = idx / NCH, col = pc % IMG, row = pc / IMG;
          *(u32x4*)(tile + L::off(row, col + L::P, q * CPB)) = v[k];
        }
      }
      __syncthreads();

      for (int kw = 0; kw < K; ++kw) {
        F bc[K][KSP];
        const F* wk = gwf(ig) + ((size_t)kw * TT::KS + pass * KSP) * 64 + lane;
#pragma unroll
        for (int kh = 0; kh < K; ++kh)
#pragma unroll
          for (int s = 0; s < KSP; ++s) bc[kh][s] = wk[((size_t)kh * K * TT::KS + s) * 64];
        const int tcol = px + kw;
        F av[NTR][KSP];
        auto load_a = [&](int tr) {
          const int trow = r0 + tr;
#pragma unroll
          for (int s = 0; s < KSP; ++s) {
            if constexpr (sizeof(S) == 4) {
              av[tr][s] = tile[L::off(trow, tcol, 2 * s + h)];
            } else {
              av[tr][s] = *(const bf16x8*)(tile + L::off(trow, tcol, 16 * s + 8 * h));
            }
          }
        };
        constexpr int PF = 3 < NTR ? 3 : NTR;
#pragma unroll
        for (int tr = 0; tr < PF; ++tr) load_a(tr);
#pragma unroll
        for (int tr = 0; tr < NTR; ++tr) {
          if (tr + PF < NTR) load_a(tr + PF);
#pragma unroll
          for (int s = 0; s < KSP; ++s) {
#pragma unroll
            for (int kh = 0; kh < K; ++kh) {
              const int i = tr - kh;
              if (i >= 0 && i < RW) acc[i] = TT::mma(bc[kh][s], av[tr][s], acc[i]);
            }
          }
        }
      }
    }
  }

  // ---- epilogue: PL layout, lane = pixel, register r = channel pl_ch(r, h)
  if constexpr (DUAL && dual_fuses<S, K, NTH>()) {
    static_assert(NO == 4 && RW % 4 == 0 && NWAVE == NO && (4 * 32 * 8) % NT == 0, "fused epilogue shape");
    if (a.cout) {
      // P_t rows stored (the backward reads them), then exchanged through LDS
      // 4 rows at a time ([row][gate][px][36]: 16-B stores conflict-free) and
      // the point-wise step run on them: one thread per (row, pixel, quad)
      float* xg = (float*)smem;
      constexpr int XS = 36;
      __syncthreads();                     // every wave is done with the tiles
#pragma unroll
      for (int g2 = 0; g2 < RW / 4; ++g2) {
#pragma unroll
        for (int i4 = 0; i4 < 4; ++i4) {
          const int i = g2 * 4 + i4;
          const int y = y0 + r0 + i;
          const size_t po = ((size_t)img * NPIX + y * IMG + px) * (32 * NO) + o * 32;
          f32x16 v = acc[i];
          if (a.bias) {
#pragma unroll
            for (int r = 0; r < 16; ++r) v[r] += a.bias[o * 32 + pl_ch(r, h)];
          }
          store_pl(a.out + po, h, v);
          store_pl(xg + ((i4 * 4 + o) * 32 + px) * XS, h, v);
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 4 * 32 * 8 / NT; ++k) {
          const int it = tid + k * NT, i4 = it >> 8, xq = it & 255, xp = xq >> 3, q = xq & 7;
          const float* pr = xg + (i4 * 4 * 32 + xp) * XS + 4 * q;
          const f32x4 pi = *(const f32x4*)pr, pf = *(const f32x4*)(pr + 32 * XS),
                      pg = *(const f32x4*)(pr + 64 * XS), pq = *(const f32x4*)(pr + 96 * XS);
          const size_t pix = (size_t)img * NPIX + (y0 + r0 + g2 * 4 + i4) * IMG + xp;
          f32x4 c = a.cprev ? ld4(a.cprev + pix * HC + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};
          f32x4 hn;
          lpw_fwd_quad(pi, pf, pg, pq, c, hn, q, a.ch);
          st4(a.cout + pix * HC + 4 * q, c);
          st4((S*)a.hout + pix * HC + 4 * q, hn);
        }
        __syncthreads();
      }
      return;
    }
  }
  if constexpr (DUAL && !dual_fuses<S, K, NTH>())
    if (a.cout) __builtin_trap();          // the host never passes c / h outputs here
#pragma unroll
  for (int i = 0; i < RW; ++i) {
    const int y = y0 + r0 + i;
    const size_t po = ((size_t)img * NPIX + y * IMG + px) * (32 * NO) + o * 32;
    f32x16 v = acc[i];
    if (a.add) add_pl(a.add + po, h, v);
    if (a.bias) {
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] += a.bias[o * 32 + pl_ch(r, h)];
    }
    store_pl(a.out + po, h, v);
  }
}

// ------------------------------------------------------------- point-wise
// One thread per (pixel, 4-channel quad).  Gates (models/convlstm.py:85-89):
//   i = sig(P_i)  f = sig(P_f)  g = tanh(P_c)  o = sig(P_o)
//   c' = f c + i g            h' = o tanh(c')
template <class S>
__global__ void k_lpw_fwd(const float* __restrict__ P, const float* __restrict__ cprev,
                          float* __restrict__ cout, S* __restrict__ hout, int npix, int ch) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= npix * 8) return;
  const int pix = e >> 3, q = e & 7;
  const float* pp = P + (size_t)pix * GC + 4 * q;
  const f32x4 pi = ld4(pp), pf = ld4(pp + 32), pg = ld4(pp + 64), po = ld4(pp + 96);
  f32x4 c = cprev ? ld4(cprev + (size_t)pix * HC + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 hn;
  lpw_fwd_quad(pi, pf, pg, po, c, hn, q, ch);
  st4(cout + (size_t)pix * HC + 4 * q, c);
  st4(hout + (size_t)pix * HC + 4 * q, hn);
}

// BPTT through one step.  dh: dL/dh_t (f32, CL), dc: dL/dc_t in, dL/dc_{t-1} out.
//   tc = tanh c_t;  dc += dh o (1 - tc^2)
//   dP_i = dc g i(1-i)   dP_f = dc c_{t-1} f(1-f)   dP_c = dc i (1-g^2)   dP_o = dh tc o(1-o)
//   dc_{t-1} = dc f
// dP -> dP_t (S) and dPsum (+=, f32; `first` initialises); `sum_s` gets an S
// copy of the final dPsum (the last step of the sweep).
template <class S>
__global__ void k_lpw_bwd(const float* __restrict__ dh, float* __restrict__ dc,
                          const float* __restrict__ P, const float* __restrict__ cc,
                          const float* __restrict__ cprev, S* __restrict__ dP,
                          float* __restrict__ dPsum, S* __restrict__ sum_s, int first, int npix,
                          int ch) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= npix * 8) return;
  const int pix = e >> 3, q = e & 7;
  const size_t pg0 = (size_t)pix * GC + 4 * q, pc0 = (size_t)pix * HC + 4 * q;
  const f32x4 pi = ld4(P + pg0), pf = ld4(P + pg0 + 32), pg = ld4(P + pg0 + 64),
              po = ld4(P + pg0 + 96);
  const f32x4 c = ld4(cc + pc0);
  const f32x4 cp = cprev ? ld4(cprev + pc0) : f32x4{0.f, 0.f, 0.f, 0.f};
  const f32x4 g_h = ld4(dh + pc0);
  f32x4 g_c = ld4(dc + pc0);
  f32x4 di, df, dg, dq, dcp;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const bool live = 4 * q + j < ch;
    const float i = sigm(pi[j]), f = sigm(pf[j]), g = ftanh(pg[j]), o = sigm(po[j]);
    const float tc = ftanh(c[j]);
    const float dct = g_c[j] + g_h[j] * o * (1.f - tc * tc);
    di[j] = live ? dct * g * i * (1.f - i) : 0.f;
    df[j] = live ? dct * cp[j] * f * (1.f - f) : 0.f;
    dg[j] = live ? dct * i * (1.f - g * g) : 0.f;
    dq[j] = live ? g_h[j] * tc * o * (1.f - o) : 0.f;
    dcp[j] = live ? dct * f : 0.f;
  }
  st4(dc + pc0, dcp);
  st4(dP + pg0, di); st4(dP + pg0 + 32, df); st4(dP + pg0 + 64, dg); st4(dP + pg0 + 96, dq);
  if (!dPsum) return;      // per-step input: the sums over steps are formed from dP itself
  f32x4 s0 = di, s1 = df, s2 = dg, s3 = dq;
  if (!first) {
    s0 += ld4(dPsum + pg0); s1 += ld4(dPsum + pg0 + 32);
    s2 += ld4(dPsum + pg0 + 64); s3 += ld4(dPsum + pg0 + 96);
  }
  st4(dPsum + pg0, s0); st4(dPsum + pg0 + 32, s1); st4(dPsum + pg0 + 64, s2); st4(dPsum + pg0 + 96, s3);
  if (sum_s) {
    st4(sum_s + pg0, s0); st4(sum_s + pg0 + 32, s1); st4(sum_s + pg0 + 64, s2); st4(sum_s + pg0 + 96, s3);
  }
}

// Jacobian-penalty seeds at the last step (t = T-1), two VJPs per image:
//   image b      : dh_t = 1, dc_t = 0   (J_h^T 1, through P_t only)
//   image B + b  : dh_t = 0, dc_t = 1   (J_c^T 1, its h_{t-1} part)
template <class S>
__global__ void k_ljv_seed(const float* __restrict__ P, const float* __restrict__ cc,
                           const float* __restrict__ cprev, S* __restrict__ dP, int npix, int ch) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= npix * 8) return;
  const int pix = e >> 3, q = e & 7;
  const size_t pg0 = (size_t)pix * GC + 4 * q, pc0 = (size_t)pix * HC + 4 * q;
  const f32x4 pi = ld4(P + pg0), pf = ld4(P + pg0 + 32), pg = ld4(P + pg0 + 64),
              po = ld4(P + pg0 + 96);
  const f32x4 c = ld4(cc + pc0), cp = ld4(cprev + pc0);
  f32x4 a0, a1, a2, a3, b0, b1, b2, b3;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const bool live = 4 * q + j < ch;
    const float i = sigm(pi[j]), f = sigm(pf[j]), g = ftanh(pg[j]), o = sigm(po[j]);
    const float tc = ftanh(c[j]);
    const float dct = o * (1.f - tc * tc);            // seed dh = 1
    a0[j] = live ? dct * g * i * (1.f - i) : 0.f;
    a1[j] = live ? dct * cp[j] * f * (1.f - f) : 0.f;
    a2[j] = live ? dct * i * (1.f - g * g) : 0.f;
    a3[j] = live ? tc * o * (1.f - o) : 0.f;
    b0[j] = live ? g * i * (1.f - i) : 0.f;           // seed dc = 1
    b1[j] = live ? cp[j] * f * (1.f - f) : 0.f;
    b2[j] = live ? i * (1.f - g * g) : 0.f;
    b3[j] = 0.f;
  }
  S* d0 = dP + pg0;
  S* d1 = dP + (size_t)npix * GC + pg0;
  st4(d0, a0); st4(d0 + 32, a1); st4(d0 + 64, a2); st4(d0 + 96, a3);
  st4(d1, b0); st4(d1 + 32, b1); st4(d1 + 64, b2); st4(d1 + 96, b3);
}

// jv = clamp(jh - mu)^2 + clamp(jc - mu)^2 with jh = conv^T part of seed 1 and
// jc = f_{T-1} + dh'_{T-2} o_{T-2} (1 - tanh^2 c_{T-2})  -> NCHW fp32 [B][ch][NPIX]
__global__ void k_ljv_final(const float* __restrict__ jdh, const float* __restrict__ Pl,
                            const float* __restrict__ Pp, const float* __restrict__ cp, float mu,
                            float* __restrict__ out, int B, int ch) {
  const int n = B * NPIX * ch;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
    const int pix = e % NPIX, c = (e / NPIX) % ch, b = e / (NPIX * ch);
    const size_t p = (size_t)b * NPIX + pix;
    const float jh = jdh[p * HC + c];
    const float f = sigm(Pl[p * GC + 32 + c]);
    const float o = sigm(Pp[p * GC + 96 + c]);
    const float tc = ftanh(cp[p * HC + c]);
    const float jc = f + jdh[((size_t)B * NPIX + p) * HC + c] * o * (1.f - tc * tc);
    const float a = fmaxf(jh - mu, 0.f), bb = fmaxf(jc - mu, 0.f);
    out[e] = a * a + bb * bb;
  }
}

// ----------------------------------------------------------- weight grads
// dW[g][co][ci][kh K + kw] = sum_{img, p} D_img[p][32 g + co] X_img[p + tap][ci]
// over the image list (two segments, e.g. (h_{t-1}, dP_t) pairs).  Workgroup
// (kh, slice): wave g owns gate g and the K taps of kernel row kh (K
// accumulator tiles); D / X row bands are staged in LDS (double-buffered,
// register prefetch), fragments come from ds_read_b64_tr_b16 transposed reads.
#ifndef PT_LW_DSWZ
#define PT_LW_DSWZ 1        // bf16 D band: chunk swizzle against 4-way bank conflicts (LWBand::dswz)
#endif
#ifndef PT_LW_RB
#define PT_LW_RB 2          // bf16 D rows per weight-gradient band (r04: 2, two workgroups per CU)
#endif
template <class S> constexpr int lw_rb() { return sizeof(S) == 2 ? PT_LW_RB : 2; }   // D rows per band
template <class S, int K> struct LWBand {
  static constexpr int P = K / 2;
  static constexpr int TC = IMG + K - 1;
  static constexpr int RBW = lw_rb<S>();
  static constexpr int CPB = 16 / (int)sizeof(S);
  static constexpr int XE = RBW * TC * HC;              // X band elements (with halo cols)
  static constexpr int DE = RBW * IMG * GC;             // D band elements
  static constexpr int BE = XE + DE;
  static constexpr int XPER = RBW * IMG * (HC / CPB) / NT;   // 2
  static constexpr int DPER = RBW * IMG * (GC / CPB) / NT;   // 8
  static constexpr int BYTES = 2 * BE * (int)sizeof(S);
  u32x4 x[XPER], d[DPER];
  int xvalid;
  __device__ __forceinline__ void load(const S* __restrict__ X, const S* __restrict__ D, int y0,
                                       int kh, int tid) {
    xvalid = 0;
#pragma unroll
    for (int j = 0; j < XPER; ++j) {
      const int idx = tid + j * NT;
      const int q = idx % (HC / CPB), pc = idx / (HC / CPB), col = pc % IMG, row = pc / IMG;
      const int iy = y0 + row + kh - P;
      const bool ok = iy >= 0 && iy < IMG;
      x[j] = *(const u32x4*)(X + (size_t)((ok ? iy : 0) * IMG + col) * HC + q * CPB);
      xvalid |= (int)ok << j;
    }
#pragma unroll
    for (int j = 0; j < DPER; ++j) {
      const int idx = tid + j * NT;
      const int q = idx % (GC / CPB), pc = idx / (GC / CPB);
      d[j] = *(const u32x4*)(D + (size_t)(y0 * IMG + pc) * GC + q * CPB);
    }
  }
  __device__ __forceinline__ void store(S* xt, S* dt, int tid) const {
#pragma unroll
    for (int j = 0; j < XPER; ++j) {
      const int idx = tid + j * NT;
      const int q = idx % (HC / CPB), pc = idx / (HC / CPB), col = pc % IMG, row = pc / IMG;
      *(u32x4*)(xt + (row * TC + col + P) * HC + q * CPB) =
          (xvalid >> j) & 1 ? x[j] : u32x4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int j = 0; j < DPER; ++j) {
      const int idx = tid + j * NT;
      *(u32x4*)(dt + dswz(idx)) = d[j];
    }
  }
  // bf16 (PT_LW_DSWZ, r05): the 16 16-B chunks of a D pixel XOR-swizzled by
  // 4 * (pixel & 3), so that the four pixels of a transposed fragment read
  // (256 B apart: one bank set) land on four bank sets -- 4-way conflicted before
  __device__ static __forceinline__ int dswz(int idx) {     // element offset of 16-B chunk idx
    if constexpr (sizeof(S) == 2 && PT_LW_DSWZ) {
      const int pc = idx >> 4, q = idx & 15;
      return pc * GC + ((q ^ ((pc & 3) << 2)) << 3);
    } else {
      return idx * CPB;
    }
  }
};

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
__device__ __forceinline__ bf16x4 tr_read(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(p));
}
template <int STRIDE>   // elements between pixel x and pixel x + 1
__device__ __forceinline__ bf16x8 tr_read8(const bf16_t* p) {
  return __builtin_shufflevector(tr_read(p), tr_read(p + 4 * STRIDE), 0, 1, 2, 3, 4, 5, 6, 7);
}

struct LWgradArgs {
  const void *X0, *D0, *X1, *D1;   // segment images: X [n][NPIX][32], D [n][NPIX][128] (S)
  int n0, n1, nsl;
  float* wslab;                     // [nsl][NG][K*K][32 co][32 ci]
};

template <class S, int K>
__global__ __launch_bounds__(NT, 1) void k_lwgrad(LWgradArgs a) {
  using Bd = LWBand<S, K>;
  constexpr int KK = K * K, RBW = Bd::RBW, NBW = IMG / RBW, TC = Bd::TC;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  S* buf = (S*)smem;
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5;
  const int g = __builtin_amdgcn_readfirstlane(tid >> 6);     // gate of this wave
  // XCD-aware (kh, slice) of this workgroup: blocks b and b + 8 share an XCD
  // (MI355X_MICROARCH.md), so the K kernel-row workgroups of one slice, which
  // stream the same D / X bands, are dealt to the same XCD's L2
  const int xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
  const int kh = j % K, sl = xcd + 8 * (j / K);
  if (sl >= a.nsl) return;
  const int nimg = a.n0 + a.n1;
  const int nmine = nimg > sl ? (nimg - sl + a.nsl - 1) / a.nsl : 0;
  const int nunits = nmine * NBW;

  f32x16 acc[K];
#pragma unroll
  for (int m = 0; m < K; ++m) acc[m] = zero16();
  for (int i = tid; i < Bd::BYTES / 16; i += NT) ((u32x4*)buf)[i] = u32x4{0u, 0u, 0u, 0u};
  __syncthreads();

  auto unit_src = [&](int u, const S*& X, const S*& D, int& y0) {
    const int j = sl + (u / NBW) * a.nsl;
    y0 = (u % NBW) * RBW;
    if (j < a.n0) {
      X = (const S*)a.X0 + (size_t)j * NPIX * HC;
      D = (const S*)a.D0 + (size_t)j * NPIX * GC;
    } else {
      X = (const S*)a.X1 + (size_t)(j - a.n0) * NPIX * HC;
      D = (const S*)a.D1 + (size_t)(j - a.n0) * NPIX * GC;
    }
  };
  Bd band;
  if (nunits > 0) {
    const S *X, *D;
    int y0;
    unit_src(0, X, D, y0);
    band.load(X, D, y0, kh, tid);
    band.store(buf, buf + Bd::XE, tid);
  }
  __syncthreads();
  for (int u = 0; u < nunits; ++u) {
    if constexpr ((PT_LPRIO & 2) != 0) lprio(u, nunits);
    const S* xt = buf + (u & 1) * Bd::BE;
    const S* dt = xt + Bd::XE;
    const bool more = u + 1 < nunits;
    if (more) {
      const S *X, *D;
      int y0;
      unit_src(u + 1, X, D, y0);
      band.load(X, D, y0, kh, tid);
    }
    if constexpr (sizeof(S) == 4) {
      // k-step = 2 pixels (x0 + h); lane & 31 is ci for A (X), co for B (D)
      const int c = lane & 31;
      for (int yd = 0; yd < RBW; ++yd) {
        const float* xb = (const float*)xt + (yd * TC + h) * HC + c;
        const float* db = (const float*)dt + (yd * IMG + h) * GC + g * 32 + c;
        for (int x0 = 0; x0 < IMG; x0 += 2) {
          const float bv = db[x0 * GC];
#pragma unroll
          for (int m = 0; m < K; ++m) acc[m] = Tr<float>::mma(xb[(x0 + m) * HC], bv, acc[m]);
        }
      }
    } else {
      // k-step = 16 pixels; lane 4q+p' of each 16-lane group addresses pixel
      // x0 + 8 hh + q (+4) and channels 16 (grp & 1) + 4 p' .. +3
      const int grp = lane >> 4, m16 = lane & 15, q = m16 >> 2, pp = m16 & 3;
      const int chb = 16 * (grp & 1) + 4 * pp, hh = grp >> 1;
      constexpr int NSTEP = RBW * 2;
      auto xaddr = [&](int st) {
        const int yd = st >> 1, c0 = (st & 1) * 16 + 8 * hh + q;
        return (const bf16_t*)xt + (yd * TC + c0) * HC + chb;
      };
      auto daddr = [&](int st) {
        const int yd = st >> 1, c0 = (st & 1) * 16 + 8 * hh + q;
        // (pixel & 3) = q here and for the +4 pixel of tr_read8: one swizzle
        const int ch = PT_LW_DSWZ ? (g * 32 + chb) ^ (q << 5) : g * 32 + chb;
        return (const bf16_t*)dt + (yd * IMG + c0) * GC + ch;
      };
      bf16x8 av[2][K], bv[2];
      bv[0] = tr_read8<GC>(daddr(0));
#pragma unroll
      for (int m = 0; m < K; ++m) av[0][m] = tr_read8<HC>(xaddr(0) + m * HC);
#pragma unroll
      for (int st = 0; st < NSTEP; ++st) {
        const int cur = st & 1, nxt = cur ^ 1;
        if (st + 1 < NSTEP) {
          bv[nxt] = tr_read8<GC>(daddr(st + 1));
#pragma unroll
          for (int m = 0; m < K; ++m) av[nxt][m] = tr_read8<HC>(xaddr(st + 1) + m * HC);
        }
#pragma unroll
        for (int m = 0; m < K; ++m) acc[m] = Tr<bf16_t>::mma(av[cur][m], bv[cur], acc[m]);
      }
    }
    if (more) {
      S* xn = buf + ((u + 1) & 1) * Bd::BE;
      band.store(xn, xn + Bd::XE, tid);
      __syncthreads();
    }
  }
  // acc[m]: rows ci = cl_x(r, h), cols co = lane & 31
  float* dst = a.wslab + (((size_t)sl * NG + g) * KK + kh * K) * 1024;
  const int co = lane & 31;
#pragma unroll
  for (int m = 0; m < K; ++m) {
#pragma unroll
    for (int r = 0; r < 16; ++r) dst[m * 1024 + co * 32 + cl_x(r, h)] = acc[m][r];
  }
}

// bf16, k <= 7 (r04): the same sums with workgroup (kw, slice) owning kernel
// COLUMN kw (wave g: gate g, accumulator tiles kh = 0 .. K-1).  k_lwgrad reads
// one shifted X fragment per tap and MFMA (7 X + 1 D transposed reads per 7
// MFMAs: bound by the LDS reads); here the band's D fragments stay in
// registers and each X-row fragment (shift kw) feeds the MFMAs of all K kernel
// rows, as InT's k_wgrad does: (RB + K - 1) * 2 X reads + RB * 2 D reads per
// RB * 2 * K MFMAs.  The X band carries the K - 1 halo rows.  Same MFMA order
// per tile as k_lwgrad (D row, then pixel block): bitwise equal.
template <int K> struct LWBand2 {
  using S = bf16_t;
  static constexpr int P = K / 2;
  static constexpr int TC = IMG + K - 1;
  static constexpr int RBW = lw_rb<S>();
  static constexpr int XR = RBW + K - 1;                // X rows (with the vertical halo)
  static constexpr int CPB = 8;
  static constexpr int XE = XR * TC * HC;
  static constexpr int DE = RBW * IMG * GC;
  static constexpr int BE = XE + DE;
  static constexpr int XPER = XR * IMG * (HC / CPB) / NT;
  static constexpr int DPER = RBW * IMG * (GC / CPB) / NT;
  static constexpr int BYTES = 2 * BE * 2;
  static_assert(XR * IMG * (HC / CPB) % NT == 0, "X band split");
  u32x4 x[XPER], d[DPER];
  int xvalid;
  __device__ __forceinline__ void load(const S* __restrict__ X, const S* __restrict__ D, int y0, int tid) {
    xvalid = 0;
#pragma unroll
    for (int j = 0; j < XPER; ++j) {
      const int idx = tid + j * NT;
      const int q = idx % (HC / CPB), pc = idx / (HC / CPB), col = pc % IMG, row = pc / IMG;
      const int iy = y0 + row - P;
      const bool ok = iy >= 0 && iy < IMG;
      x[j] = *(const u32x4*)(X + (size_t)((ok ? iy : 0) * IMG + col) * HC + q * CPB);
      xvalid |= (int)ok << j;
    }
#pragma unroll
    for (int j = 0; j < DPER; ++j) {
      const int idx = tid + j * NT;
      const int q = idx % (GC / CPB), pc = idx / (GC / CPB);
      d[j] = *(const u32x4*)(D + (size_t)(y0 * IMG + pc) * GC + q * CPB);
    }
  }
  __device__ __forceinline__ void store(S* xt, S* dt, int tid) const {
#pragma unroll
    for (int j = 0; j < XPER; ++j) {
      const int idx = tid + j * NT;
      const int q = idx % (HC / CPB), pc = idx / (HC / CPB), col = pc % IMG, row = pc / IMG;
      *(u32x4*)(xt + (row * TC + col + P) * HC + q * CPB) = (xvalid >> j) & 1 ? x[j] : u32x4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int j = 0; j < DPER; ++j) *(u32x4*)(dt + (tid + j * NT) * CPB) = d[j];
  }
};

template <int K>
__global__ __launch_bounds__(NT, 1) void k_lwgrad2(LWgradArgs a) {
  using S = bf16_t;
  using Bd = LWBand2<K>;
  constexpr int KK = K * K, RBW = Bd::RBW, NBW = IMG / RBW, TC = Bd::TC, XR = Bd::XR;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  S* buf = (S*)smem;
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5;
  const int g = __builtin_amdgcn_readfirstlane(tid >> 6);     // gate of this wave
  const int xcd = blockIdx.x & 7, j = blockIdx.x >> 3;         // XCD-aware, as k_lwgrad
  const int kw = j % K, sl = xcd + 8 * (j / K);
  if (sl >= a.nsl) return;
  const int nimg = a.n0 + a.n1;
  const int nmine = nimg > sl ? (nimg - sl + a.nsl - 1) / a.nsl : 0;
  const int nunits = nmine * NBW;

  f32x16 acc[K];
#pragma unroll
  for (int m = 0; m < K; ++m) acc[m] = zero16();
  for (int i = tid; i < Bd::BYTES / 16; i += NT) ((u32x4*)buf)[i] = u32x4{0u, 0u, 0u, 0u};
  __syncthreads();
  auto unit_src = [&](int u, const S*& X, const S*& D, int& y0) {
    const int jj = sl + (u / NBW) * a.nsl;
    y0 = (u % NBW) * RBW;
    if (jj < a.n0) {
      X = (const S*)a.X0 + (size_t)jj * NPIX * HC;
      D = (const S*)a.D0 + (size_t)jj * NPIX * GC;
    } else {
      X = (const S*)a.X1 + (size_t)(jj - a.n0) * NPIX * HC;
      D = (const S*)a.D1 + (size_t)(jj - a.n0) * NPIX * GC;
    }
  };
  Bd band;
  if (nunits > 0) {
    const S *X, *D;
    int y0;
    unit_src(0, X, D, y0);
    band.load(X, D, y0, tid);
    band.store(buf, buf + Bd::XE, tid);
  }
  __syncthreads();
  const int grp = lane >> 4, m16 = lane & 15, q = m16 >> 2, pp = m16 & 3;
  const int chb = 16 * (grp & 1) + 4 * pp, hh = grp >> 1;
  for (int u = 0; u < nunits; ++u) {
    int bo = (u & 1) * Bd::BE;
    asm volatile("" : "+s"(bo));              // opaque: no per-buffer address sets hoisted
    const S* xt = buf + bo;
    const S* dt = xt + Bd::XE;
    const bool more = u + 1 < nunits;
    if (more) {
      const S *X, *D;
      int y0;
      unit_src(u + 1, X, D, y0);
      band.load(X, D, y0, tid);
    }
    // steps (X row r, pixel block blk), r outer: per tile (kh) the D rows
    // yd = r - kh then the blocks, k_lwgrad's order
    bf16x8 dv[RBW][2], av[2];
    auto xaddr = [&](int st) {
      return xt + ((st >> 1) * TC + (st & 1) * 16 + 8 * hh + q + kw) * HC + chb;
    };
#pragma unroll
    for (int yd = 0; yd < RBW; ++yd)
#pragma unroll
      for (int blk = 0; blk < 2; ++blk)
        dv[yd][blk] = tr_read8<GC>(dt + (yd * IMG + blk * 16 + 8 * hh + q) * GC + g * 32 + chb);
    av[0] = tr_read8<HC>(xaddr(0));
#pragma unroll
    for (int st = 0; st < 2 * XR; ++st) {
      const int r = st >> 1, blk = st & 1, cur = st & 1;
      if (st + 1 < 2 * XR) av[cur ^ 1] = tr_read8<HC>(xaddr(st + 1));
#pragma unroll
      for (int kh = 0; kh < K; ++kh) {
        const int yd = r - kh;
        if (yd >= 0 && yd < RBW) acc[kh] = Tr<S>::mma(av[cur], dv[yd][blk], acc[kh]);
      }
    }
    if (more) {
      S* xn = buf + ((u + 1) & 1) * Bd::BE;
      band.store(xn, xn + Bd::XE, tid);
      __syncthreads();
    }
  }
  // acc[kh]: rows ci = cl_x(r, h), cols co = lane & 31 (k_lwgrad's slab layout)
  float* dst = a.wslab + ((size_t)sl * NG + g) * KK * 1024;
  const int co = lane & 31;
#pragma unroll
  for (int kh = 0; kh < K; ++kh) {
#pragma unroll
    for (int r = 0; r < 16; ++r) dst[(kh * K + kw) * 1024 + co * 32 + cl_x(r, h)] = acc[kh][r];
  }
}

// ------------------------------------------------------------- reductions
// Column sums of [npix][GC] rows (the bias gradients): dPsum (static x) or, per-step
// input, the rows of every step's dP_t (npix = T * B * NPIX), read in S.
template <class S>
__global__ void k_lcolsum(const S* __restrict__ src, float* __restrict__ part, int npix) {
  // 16 threads per [GC] row, 8 channels (16 B bf16 / 32 B f32) each: 16 rows
  // per pass of the 256 threads (2-B loads of one channel per thread ran at
  // ~1.4 TB/s: 3 ms per call for the clip ConvLSTM's 4.3 GB dP)
  const int q = threadIdx.x & 15, r0 = threadIdx.x >> 4;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int step = gridDim.x * 16;
  auto add_row = [&](int r) {
    const S* p = src + (size_t)r * GC + 8 * q;
    if constexpr (sizeof(S) == 2) {
      const u32x4 v = *(const u32x4*)p;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        s[2 * j] += __uint_as_float(v[j] << 16);
        s[2 * j + 1] += __uint_as_float(v[j] & 0xffff0000u);
      }
    } else {
      const f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) { s[j] += a[j]; s[4 + j] += b[j]; }
    }
  };
  int r = blockIdx.x * 16 + r0;
  for (; r + 3 * step < npix; r += 4 * step) {
    add_row(r); add_row(r + step); add_row(r + 2 * step); add_row(r + 3 * step);
  }
  for (; r < npix; r += step) add_row(r);
  __shared__ float red[16][GC];
#pragma unroll
  for (int j = 0; j < 8; ++j) red[r0][8 * q + j] = s[j];
  __syncthreads();
  if (threadIdx.x < GC) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += red[k][threadIdx.x];
    part[(size_t)blockIdx.x * GC + threadIdx.x] = t;
  }
}

struct LReduceArgs {
  int K, nsl_h, nsl_x, ch, cin, nb;
  const float* wslab_h;   // [nsl_h][NG][KK][1024]
  const float* wslab_x;   // [nsl_x][NG][KK][1024]
  const float* colpart;   // [nb][128]
  float* wh[4];
  float* wx[4];
  float* bx[4];
};

__device__ __forceinline__ float lsum(const float* __restrict__ p, size_t stride, int n) {
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int i = 0;
  for (; i + 8 <= n; i += 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += p[(size_t)(i + j) * stride];
  }
  for (; i < n; ++i) acc[0] += p[(size_t)i * stride];
  return ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
}

__global__ void k_lreduce(LReduceArgs r) {
  const int KK = r.K * r.K;
  const int nw = NG * KK * 1024;
  const int total = 2 * nw + GC;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    if (e < 2 * nw) {
      const int fam = e / nw, rem = e % nw;            // 0: Wh, 1: Wx
      const int g = rem / (KK * 1024), tap = (rem / 1024) % KK, co = (rem % 1024) / 32,
                ci = rem % 32;
      const int cin = fam == 0 ? r.ch : r.cin;
      float* W = fam == 0 ? r.wh[g] : r.wx[g];
      if (!W || co >= r.ch || ci >= cin) continue;
      const float* src = fam == 0 ? r.wslab_h : r.wslab_x;
      const int nsl = fam == 0 ? r.nsl_h : r.nsl_x;
      W[((size_t)co * cin + ci) * KK + tap] = lsum(src + rem, (size_t)NG * KK * 1024, nsl);
    } else {
      const int c = e - 2 * nw, g = c / 32, co = c % 32;
      if (r.bx[g] && co < r.ch) r.bx[g][co] = lsum(r.colpart + c, GC, r.nb);
    }
  }
}

// ------------------------------------------------------------ conversions
// NCHW fp32 [B][nc][NPIX] -> channels-last [B][NPIX][32] (zero padded).
// tn > 1: frame t of [B][nc][tn][NPIX] (x_seq inputs / their gradients).
// lo (optional): the residual v - (S)v as a second plane (the split x-conv)
template <class S>
__global__ void k_to_cl(const float* __restrict__ src, S* __restrict__ dst, int B, int nc,
                        int tn = 1, int t = 0, S* __restrict__ lo = nullptr) {
  const int n = B * NPIX * HC;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
    const int c = e % HC, pix = (e / HC) % NPIX, b = e / (HC * NPIX);
    const float v = c < nc ? src[(((size_t)b * nc + c) * tn + t) * NPIX + pix] : 0.f;
    dst[e] = (S)v;
    if (lo) lo[e] = (S)(v - (float)(S)v);
  }
}
// All steps at once: [B][nc][T][NPIX] fp32 <-> [T][B][NPIX][32] channels-last
// (per-step inputs and their gradients; the per-step hidden states).  One
// workgroup per (image, 256-pixel chunk) through an LDS tile [32][256], so
// both the channel-plane side (1 KB rows) and the channels-last side (one
// 64 / 128-B pixel row per thread) are coalesced (element-per-thread forms
// read / wrote with a 4 KB stride: ~1.3 TB/s).
constexpr int SEQ_CH = 256;                 // pixels per workgroup
template <class S>
__global__ __launch_bounds__(256) void k_to_cl_seq(const float* __restrict__ src, S* __restrict__ dst,
                                                   int B, int nc, int T) {
  __shared__ float tile[HC][SEQ_CH];
  const int img = blockIdx.x / (NPIX / SEQ_CH), pix0 = (blockIdx.x % (NPIX / SEQ_CH)) * SEQ_CH;
  const int b = img % B, t = img / B, tid = threadIdx.x;
  for (int c = 0; c < HC; ++c)
    tile[c][tid] = c < nc ? src[(((size_t)b * nc + c) * T + t) * NPIX + pix0 + tid] : 0.f;
  __syncthreads();
  S* d = dst + ((size_t)img * NPIX + pix0 + tid) * HC;
  constexpr int CPB = 16 / (int)sizeof(S);
#pragma unroll
  for (int q = 0; q < HC / CPB; ++q) {
    if constexpr (sizeof(S) == 2) {
      u32x4 v;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
        const bf2 pr = {(S)tile[q * CPB + 2 * j][tid], (S)tile[q * CPB + 2 * j + 1][tid]};
        v[j] = __builtin_bit_cast(uint32_t, pr);
      }
      *(u32x4*)(d + q * CPB) = v;
    } else {
      *(f32x4*)(d + q * CPB) = f32x4{tile[q * CPB][tid], tile[q * CPB + 1][tid], tile[q * CPB + 2][tid],
                                     tile[q * CPB + 3][tid]};
    }
  }
}
template <class S>
__global__ __launch_bounds__(256) void k_from_cl_seq(const S* __restrict__ src, float* __restrict__ dst,
                                                     int B, int nc, int T) {
  __shared__ float tile[HC][SEQ_CH];
  const int img = blockIdx.x / (NPIX / SEQ_CH), pix0 = (blockIdx.x % (NPIX / SEQ_CH)) * SEQ_CH;
  const int b = img % B, t = img / B, tid = threadIdx.x;
  const S* sp = src + ((size_t)img * NPIX + pix0 + tid) * HC;
  constexpr int CPB = 16 / (int)sizeof(S);
#pragma unroll
  for (int q = 0; q < HC / CPB; ++q) {
    if constexpr (sizeof(S) == 2) {
      const u32x4 v = *(const u32x4*)(sp + q * CPB);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        tile[q * CPB + 2 * j][tid] = __uint_as_float(v[j] << 16);
        tile[q * CPB + 2 * j + 1][tid] = __uint_as_float(v[j] & 0xffff0000u);
      }
    } else {
      const f32x4 v = *(const f32x4*)(sp + q * CPB);
#pragma unroll
      for (int j = 0; j < 4; ++j) tile[q * CPB + j][tid] = v[j];
    }
  }
  __syncthreads();
  for (int c = 0; c < nc; ++c) dst[(((size_t)b * nc + c) * T + t) * NPIX + pix0 + tid] = tile[c][tid];
}
template <class S>
__global__ void k_from_cl(const S* __restrict__ src, float* __restrict__ dst, int B, int nc,
                          int tn = 1, int t = 0) {
  const int n = B * nc * NPIX;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
    const int pix = e % NPIX, c = (e / NPIX) % nc, b = e / (NPIX * nc);
    dst[(((size_t)b * nc + c) * tn + t) * NPIX + pix] = ldg(src + ((size_t)b * NPIX + pix) * HC + c);
  }
}

// ---------------------------------------------------------- parameter prep
// fp32 torch weights -> MFMA A-operand fragments (weights on the A side):
//   fwd  (NI = 1, NO = 4): F[o][0][tap][ks][lane][j]  = W_o[n = l&31][frag_chan(ks,h,j)][tap]
//   conv^T (NI = 4, NO = 1): F[0][ig][tap][ks][lane][j] = W_ig[frag_chan][n = l&31][KK-1-tap]
// (out-of-range channels are zero).  Families: 0 Wx fwd, 1 Wh fwd, 2 Wh^T, 3 Wx^T.
struct LPrepArgs {
  int K, ch, cin;
  const float* wx[4];
  const float* wh[4];
  const float* bx[4];
  void* fr[4];
  float* bias;     // [128]
  void* frlo;      // or null: family 4, Wx fwd's residual W - (S)W (the split x-conv)
};
template <class S>
__global__ void k_lprep(LPrepArgs p) {
  using TT = Tr<S>;
  const int KK = p.K * p.K;
  const int per = NG * KK * TT::KS * 64 * TT::EPL;     // elements per family
  const int nfam = p.frlo ? 5 : 4;
  const int total = nfam * per + GC;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    if (e >= nfam * per) {
      const int c = e - nfam * per, g = c / 32, co = c % 32;
      p.bias[c] = (p.bx[g] && co < p.ch) ? p.bx[g][co] : 0.f;
      continue;
    }
    const int fam = e / per, r = e % per;
    const int j = r % TT::EPL, l = (r / TT::EPL) % 64, ks = (r / (TT::EPL * 64)) % TT::KS;
    const int tap = (r / (TT::EPL * 64 * TT::KS)) % KK, blk = r / (TT::EPL * 64 * TT::KS * KK);
    const int n = l & 31, hh = l >> 5, kc = frag_chan<S>(ks, hh, j);
    float v = 0.f;
    if (fam < 2 || fam == 4) {          // blk = output gate o
      const float* W = fam != 1 ? p.wx[blk] : p.wh[blk];
      const int cin = fam != 1 ? p.cin : p.ch;
      if (n < p.ch && kc < cin) v = W[((size_t)n * cin + kc) * KK + tap];
      if (fam == 4) v -= (float)(S)v;
    } else {                            // blk = input gate ig; out channel n = fwd input channel
      const float* W = fam == 2 ? p.wh[blk] : p.wx[blk];
      const int cin = fam == 2 ? p.ch : p.cin;
      if (kc < p.ch && n < cin) v = W[((size_t)kc * cin + n) * KK + (KK - 1 - tap)];
    }
    ((S*)(fam == 4 ? p.frlo : p.fr[fam]))[r] = (S)v;
  }
}

// ------------------------------------------------------------- frame stem
// Clip ConvLSTM stem: y = softplus(W x + b) per voxel, a 1x1x1
// channel mix of x [B][CIN][n] into y [B][cout][n]; softplus as torch's
// (beta 1, threshold 20).  One thread per 4 voxels: 16-byte loads / stores,
// each output plane written contiguously; HBM-bound (CIN + cout floats/voxel).
__device__ __forceinline__ float softplus20(float z) { return z > 20.f ? z : log1pf(expf(z)); }
__device__ __forceinline__ float dsoftplus20(float z, float g) {
  if (z > 20.f) return g;
  const float e = expf(z);
  return g * e / (e + 1.f);
}

// The stem input: the f32 model input [B][CIN][n] (planar), or the raw clip
// bytes u8 [B][n][CIN] as the TFRecords hold them (voxel-interleaved),
// converted exactly as engine.prepare_data does (utils/engine.py:220-255: the
// float64 quotient u / 255 rounded to f32), so the f32 clip tensor never exists.
template <int CIN>
__device__ __forceinline__ void stem_load(const void* __restrict__ xv, int xu8, long bi, long v,
                                          long n4, float4 (&xi)[CIN]) {
  if (xu8) {
    // 4 voxels x CIN bytes, 4-byte aligned (v counts groups of 4 voxels)
    const uint32_t* q = (const uint32_t*)((const uint8_t*)xv + (bi * n4 + v) * 4 * CIN);
    uint32_t wd[CIN];
#pragma unroll
    for (int j = 0; j < CIN; ++j) wd[j] = q[j];
#pragma unroll
    for (int j = 0; j < 4 * CIN; ++j) {
      const float f = (float)((double)((wd[j >> 2] >> (8 * (j & 3))) & 0xffu) / 255.0);
      const int vox = j / CIN, k = j % CIN;
      if (vox == 0) xi[k].x = f; else if (vox == 1) xi[k].y = f; else if (vox == 2) xi[k].z = f; else xi[k].w = f;
    }
  } else {
    const float4* x = (const float4*)xv;
#pragma unroll
    for (int k = 0; k < CIN; ++k) xi[k] = x[(bi * CIN + k) * n4 + v];
  }
}

template <int CIN>
__global__ __launch_bounds__(256) void k_stem_fwd(const void* __restrict__ x, int xu8, const float* __restrict__ w,
                                                  const float* __restrict__ b, float4* __restrict__ y,
                                                  int cout, long n4, long total4) {
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total4; e += (long)gridDim.x * blockDim.x) {
    const long bi = e / n4, v = e - bi * n4;
    float4 xi[CIN];
    stem_load<CIN>(x, xu8, bi, v, n4, xi);
    for (int o = 0; o < cout; ++o) {
      float4 z = make_float4(b[o], b[o], b[o], b[o]);
#pragma unroll
      for (int k = 0; k < CIN; ++k) {
        const float wk = w[o * CIN + k];
        z.x += wk * xi[k].x; z.y += wk * xi[k].y; z.z += wk * xi[k].z; z.w += wk * xi[k].w;
      }
      y[(bi * cout + o) * n4 + v] =
          make_float4(softplus20(z.x), softplus20(z.y), softplus20(z.z), softplus20(z.w));
    }
  }
}

// dW [cout][CIN], db [cout] of the stem from dy, z recomputed from x: per-block
// partial sums part[block][32 * (CIN + 1)] (wave shuffles, then LDS across the
// 4 waves), summed in fixed order by k_stem_reduce (deterministic).
template <int CIN>
__global__ __launch_bounds__(256) void k_stem_bwd(const void* __restrict__ x, int xu8, const float* __restrict__ w,
                                                  const float* __restrict__ b, const float4* __restrict__ dy,
                                                  float* __restrict__ part, int cout, long n4, long total4) {
  constexpr int NA = 32 * (CIN + 1);
  float acc[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) acc[i] = 0.f;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total4; e += (long)gridDim.x * blockDim.x) {
    const long bi = e / n4, v = e - bi * n4;
    float4 xi[CIN];
    stem_load<CIN>(x, xu8, bi, v, n4, xi);
#pragma unroll
    for (int o = 0; o < 32; ++o) {
      if (o < cout) {
        float4 z = make_float4(b[o], b[o], b[o], b[o]);
#pragma unroll
        for (int k = 0; k < CIN; ++k) {
          const float wk = w[o * CIN + k];
          z.x += wk * xi[k].x; z.y += wk * xi[k].y; z.z += wk * xi[k].z; z.w += wk * xi[k].w;
        }
        const float4 d = dy[(bi * cout + o) * n4 + v];
        const float gx = dsoftplus20(z.x, d.x), gy = dsoftplus20(z.y, d.y), gz = dsoftplus20(z.z, d.z),
                    gw = dsoftplus20(z.w, d.w);
#pragma unroll
        for (int k = 0; k < CIN; ++k)
          acc[o * (CIN + 1) + k] += (gx * xi[k].x + gy * xi[k].y) + (gz * xi[k].z + gw * xi[k].w);
        acc[o * (CIN + 1) + CIN] += (gx + gy) + (gz + gw);
      }
    }
  }
  __shared__ float red[4][NA];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    float t = acc[i];
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) t += __shfl_xor(t, m);
    if (lane == 0) red[wv][i] = t;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < NA; i += blockDim.x)
    part[(size_t)blockIdx.x * NA + i] = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
}

// The clip ConvLSTM's stem fused into the recurrence (pt_lstm_forward_stem):
// y = softplus(W x + b) of 4 voxels per thread, computed exactly as k_stem_fwd
// does, stored straight into the recurrence's per-step input, channels-last
// [T][B][NPIX][32] in S with the channels >= cout zero -- bit for bit what
// k_to_cl_seq makes of k_stem_fwd's f32 [B][cout][T][NPIX], which therefore
// never exists.  One workgroup per (frame t, clip b) image, [T][B] order.
template <int CIN, class S>
__global__ __launch_bounds__(256) void k_stem_cl_fwd(const void* __restrict__ x, int xu8, const float* __restrict__ w,
                                                     const float* __restrict__ b, S* __restrict__ dst, int cout,
                                                     int B, int T) {
  const int img = blockIdx.x, t = img / B, bi = img - t * B, tid = threadIdx.x;
  const long n4 = (long)T * (NPIX / 4), v = (long)t * (NPIX / 4) + tid;   // pixels 4 tid .. 4 tid + 3
  float4 xi[CIN];
  stem_load<CIN>(x, xu8, bi, v, n4, xi);
  S* d = dst + ((size_t)img * NPIX + 4 * tid) * HC;
  constexpr int CPB = 16 / (int)sizeof(S);
#pragma unroll
  for (int q = 0; q < HC / CPB; ++q) {
    float yv[4][CPB];
#pragma unroll
    for (int j = 0; j < CPB; ++j) {
      const int o = q * CPB + j;
      float4 y = make_float4(0.f, 0.f, 0.f, 0.f);
      if (o < cout) {
        float4 z = make_float4(b[o], b[o], b[o], b[o]);
#pragma unroll
        for (int k = 0; k < CIN; ++k) {
          const float wk = w[o * CIN + k];
          z.x += wk * xi[k].x; z.y += wk * xi[k].y; z.z += wk * xi[k].z; z.w += wk * xi[k].w;
        }
        y = make_float4(softplus20(z.x), softplus20(z.y), softplus20(z.z), softplus20(z.w));
      }
      yv[0][j] = y.x; yv[1][j] = y.y; yv[2][j] = y.z; yv[3][j] = y.w;
    }
#pragma unroll
    for (int vx = 0; vx < 4; ++vx) {
      if constexpr (sizeof(S) == 2) {
        u32x4 o4;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
          const bf2 pr = {(S)yv[vx][2 * j], (S)yv[vx][2 * j + 1]};
          o4[j] = __builtin_bit_cast(uint32_t, pr);
        }
        *(u32x4*)(d + vx * HC + q * CPB) = o4;
      } else {
        *(f32x4*)(d + vx * HC + q * CPB) = f32x4{yv[vx][0], yv[vx][1], yv[vx][2], yv[vx][3]};
      }
    }
  }
}

// dW [cout][CIN], db [cout] of the fused stem from the recurrence's d x_t of
// all steps, channels-last f32 [T][B][NPIX][32] (the all-steps transposed
// conv's output), so the f32 [B][cout][T][NPIX] gradient tensor never exists
// either.  One thread per voxel: its 32 channels of d x_t are 128 contiguous
// bytes (8 x 16-B loads, a wave reads 8 KB in one run); z recomputed from x
// as k_stem_bwd does; per-block partials summed by k_stem_reduce.
template <int CIN>
__global__ __launch_bounds__(256) void k_stem_cl_bwd(const void* __restrict__ x, int xu8, const float* __restrict__ w,
                                                     const float* __restrict__ b, const float* __restrict__ dxs,
                                                     float* __restrict__ part, int cout, int B, int T) {
  constexpr int NA = 32 * (CIN + 1);
  float acc[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) acc[i] = 0.f;
  const long n = (long)T * NPIX, total = (long)B * n;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    // voxel e in [T][B][NPIX] order (the d x_t layout): frame t, clip bi, pixel p
    const long t = e / ((long)B * NPIX), r = e - t * B * NPIX, bi = r / NPIX, p = r - bi * NPIX;
    const long vox = t * NPIX + p;                     // within clip bi
    float xi[CIN];
    if (xu8) {
      const uint8_t* q = (const uint8_t*)x + (bi * n + vox) * CIN;
#pragma unroll
      for (int k = 0; k < CIN; ++k) xi[k] = (float)((double)q[k] / 255.0);
    } else {
#pragma unroll
      for (int k = 0; k < CIN; ++k) xi[k] = ((const float*)x)[(bi * CIN + k) * n + vox];
    }
    const f32x4* dp = (const f32x4*)(dxs + (size_t)e * HC);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const f32x4 d4 = dp[q];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int o = 4 * q + j;
        if (o < cout) {
          float z = b[o];
#pragma unroll
          for (int k = 0; k < CIN; ++k) z += w[o * CIN + k] * xi[k];
          const float gz = dsoftplus20(z, d4[j]);
#pragma unroll
          for (int k = 0; k < CIN; ++k) acc[o * (CIN + 1) + k] += gz * xi[k];
          acc[o * (CIN + 1) + CIN] += gz;
        }
      }
    }
  }
  __shared__ float red[4][NA];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    float t = acc[i];
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) t += __shfl_xor(t, m);
    if (lane == 0) red[wv][i] = t;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < NA; i += blockDim.x)
    part[(size_t)blockIdx.x * NA + i] = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
}

// One workgroup per accumulator: 256 threads stride the partials, then a
// fixed-order tree in LDS (deterministic), fp64 throughout.
__global__ __launch_bounds__(256) void k_stem_reduce(const float* __restrict__ part, int nblk, int cin,
                                                     int cout, float* __restrict__ dw, float* __restrict__ db) {
  const int na = 32 * (cin + 1), i = blockIdx.x;
  const int o = i / (cin + 1), k = i % (cin + 1);
  if (o >= cout) return;                       // uniform per workgroup
  double s = 0.0;
  for (int j = threadIdx.x; j < nblk; j += blockDim.x) s += part[(size_t)j * na + i];
  __shared__ double red[256];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int m = 128; m >= 1; m >>= 1) {
    if (threadIdx.x < m) red[threadIdx.x] += red[threadIdx.x + m];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (k < cin) { if (dw) dw[o * cin + k] = (float)red[0]; }
    else if (db) db[o] = (float)red[0];
  }
}

}  // namespace ptl

// =========================================================================
//                                  host side
// =========================================================================
using namespace ptl;

static thread_local char g_err[512];
static int fail(int code, const char* fmt, long v = 0) {
  snprintf(g_err, sizeof(g_err), fmt, v);
  return code;
}

namespace {

constexpr size_t ALIGN = 256;
inline size_t al(size_t x) { return (x + ALIGN - 1) / ALIGN * ALIGN; }

constexpr int STEM_BLOCKS = 1024;     // stem weight-gradient partials (k_stem_bwd / k_stem_cl_bwd)
// pt_lstm_forward_stem / pt_lstm_backward_stem: the raw clip batch and the
// stem's parameters (the recurrence's input channels = the stem's outputs)
struct StemIn { const void* x; int xu8, cin; const float *w, *b; };

struct LPlan {
  int B, T, K, ch, cin, nsl_h, nsl_x, nb;
  int xseq;           // one input image per step (desc.x_seq)
  size_t es, npix;
  // saved
  size_t o_fr[4], o_bias, o_x, o_xg, o_h0, o_c0, o_P, o_h, o_c, saved;
  size_t o_frlo, o_xlo;   // bf16 static x: the split x-conv's residual fragments / x plane
  int xsplit;
  // workspace
  size_t o_dh, o_dc, o_dP, o_dPsum, o_dPsumS, o_jvP, o_wsh, o_wsx, o_col, o_dx, o_stem, ws;
};

int check(const pt_lstm_desc* d) {
  if (!d) return fail(PT_LSTM_ERR_ARG, "null descriptor");
  if (d->channels < 1 || d->channels > 32)
    return fail(PT_LSTM_ERR_UNSUPPORTED, "hidden channels must be 1..32 (got %ld)", d->channels);
  if (d->in_channels < 1 || d->in_channels > 32)
    return fail(PT_LSTM_ERR_UNSUPPORTED, "input channels must be 1..32 (got %ld)", d->in_channels);
  if (d->height != 32 || d->width != 32)
    return fail(PT_LSTM_ERR_UNSUPPORTED, "only 32x32 images are supported (H=%ld)", d->height);
  if (d->ksize < 1 || d->ksize > KMAX || (d->ksize & 1) == 0)
    return fail(PT_LSTM_ERR_UNSUPPORTED, "ksize must be odd and <= 15 (got %ld)", d->ksize);
  if (d->batch < 1 || d->steps < 1) return fail(PT_LSTM_ERR_ARG, "batch and steps must be >= 1%ld");
  if (d->dtype != PT_LSTM_F32 && d->dtype != PT_LSTM_BF16) return fail(PT_LSTM_ERR_ARG, "bad dtype%ld");
  if (d->x_seq != 0 && d->x_seq != 1) return fail(PT_LSTM_ERR_ARG, "bad x_seq (%ld)", d->x_seq);
  return 0;
}

int slices(int nimg, int K) {
  int n = (512 + K - 1) / K;           // ~512 workgroups over the K tap rows
  if (n >= 8) n = n / 8 * 8;           // whole XCD groups (k_lwgrad's block mapping)
  if (n > nimg) n = nimg;
  return n < 1 ? 1 : n;
}

LPlan plan(const pt_lstm_desc* d) {
  LPlan p{};
  p.B = d->batch; p.T = d->steps; p.K = d->ksize; p.ch = d->channels; p.cin = d->in_channels;
  p.es = d->dtype == PT_LSTM_BF16 ? 2 : 4;
  p.npix = (size_t)p.B * NPIX;
  const size_t KK = (size_t)p.K * p.K;
  size_t o = 0;
  for (int i = 0; i < 4; ++i) { p.o_fr[i] = o; o += al(NG * KK * 1024 * p.es); }
  p.o_bias = o; o += al(GC * 4);
  p.xseq = d->x_seq != 0;
  p.o_x = o; o += al(p.npix * HC * p.es * (p.xseq ? p.T : 1));   // [steps][B][NPIX][32]
  // static x with a given h0: xg = Wx*x + b kept apart from P_0 (per-step
  // input: P_t = Wx*x_t + b is written into P directly, no xg)
  p.o_xg = o; o += p.xseq ? 0 : al(p.npix * GC * 4);
  // bf16 static x (r06): xg in three bf16 passes, x_hi W_hi + x_lo W_hi +
  // x_hi W_lo (~2^-16 relative, f32 accumulation): with bf16 x and Wx the
  // Gabor-squared input's x-conv pushed tanh(P_c) into saturation with a
  // bf16-sized error and the c-gate gradients to cosine 0.96
  // (tools/lstm_bf16_attrib.py, profiles/r06_lstm_bf16_attrib.json)
  p.xsplit = p.es == 2 && !p.xseq;
  p.o_frlo = o; o += p.xsplit ? al(NG * KK * 1024 * p.es) : 0;
  p.o_xlo = o; o += p.xsplit ? al(p.npix * HC * p.es) : 0;
  p.o_h0 = o; o += al(p.npix * HC * p.es);
  p.o_c0 = o; o += al(p.npix * HC * 4);
  p.o_P = o; o += al(p.npix * GC * 4 * p.T);
  p.o_h = o; o += al(p.npix * HC * p.es * p.T);
  p.o_c = o; o += al(p.npix * HC * 4 * p.T);
  p.saved = o;
  p.nsl_h = slices(p.B * p.T, p.K);
  p.nsl_x = slices(p.xseq ? p.B * p.T : p.B, p.K);
  p.nb = 256;
  o = 0;
  p.o_dh = o; o += al(2 * p.npix * HC * 4);
  p.o_dc = o; o += al(p.npix * HC * 4);
  p.o_dP = o; o += al(p.npix * GC * p.es * p.T);
  // sum over steps of dP (static x: its bias / weight / input gradients need
  // only that sum); per-step input: the bias sums come from dP itself
  p.o_dPsum = o; o += p.xseq ? 0 : al(p.npix * GC * 4);
  p.o_dPsumS = o; o += p.xseq ? 0 : al(p.npix * GC * p.es);
  p.o_jvP = o; o += al(2 * p.npix * GC * p.es);
  p.o_wsh = o; o += al((size_t)p.nsl_h * NG * KK * 1024 * 4);
  p.o_wsx = o; o += al((size_t)p.nsl_x * NG * KK * 1024 * 4);
  p.o_col = o; o += al((size_t)p.nb * GC * 4);
  // per-step input: d x_t of all steps from ONE transposed conv over B*T images
  p.o_dx = o; o += p.xseq ? al(p.npix * HC * 4 * p.T) : 0;
  // the fused stem's per-block partials (pt_lstm_backward_stem, up to 4 input channels)
  p.o_stem = o; o += p.xseq ? al((size_t)STEM_BLOCKS * 32 * 5 * 4) : 0;
  p.ws = o;
  return p;
}

#define HIPCHK(expr)                                                                     \
  do {                                                                                   \
    hipError_t e_ = (expr);                                                              \
    if (e_ != hipSuccess) {                                                              \
      snprintf(g_err, sizeof(g_err), "HIP error %s at line %d", hipGetErrorString(e_), __LINE__); \
      return PT_LSTM_ERR_HIP;                                                            \
    }                                                                                    \
  } while (0)

#define SETLDS(kern, bytes) \
  HIPCHK(hipFuncSetAttribute((const void*)(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (bytes)))

// K dispatch (odd kernel sizes 1..15)
#define K_SWITCH(K, CALL)                                  \
  switch (K) {                                             \
    case 1: { constexpr int KC = 1; CALL; } break;         \
    case 3: { constexpr int KC = 3; CALL; } break;         \
    case 5: { constexpr int KC = 5; CALL; } break;         \
    case 7: { constexpr int KC = 7; CALL; } break;         \
    case 9: { constexpr int KC = 9; CALL; } break;         \
    case 11: { constexpr int KC = 11; CALL; } break;       \
    case 13: { constexpr int KC = 13; CALL; } break;       \
    default: { constexpr int KC = 15; CALL; } break;       \
  }

// PT_LCONV_FAST=0 (diagnostic builds only, read per call) selects k_lconv's plain column loop (A/B test)
int lconv_fast_env() { return PT_SW("PT_LCONV_FAST", 1) != 0; }
// the transposed conv on 8 waves of 4 rows (two per SIMD) instead of 4 of 8:
// opt-in (PT_LCONVT8=1, diagnostic builds only, read per call).  Measured r04 (cfg3,
// profiles/r04_lconvt8_ab.txt): 45.83 vs 45.64 ms per step -- the 256-VGPR
// budget spills 42 registers and the 8 waves load the same weights twice as
// often as 4.
// PT_LPW_FUSE=0 (diag builds): the per-step point-wise update as its own
// launch (k_lpw_fwd) instead of in the two-source conv's epilogue (r05)
int lpw_fuse_env() { return PT_SW("PT_LPW_FUSE", 1) != 0; }
int lconvt8_env() { return PT_SW("PT_LCONVT8", PT_LCONVT8_DEF) == 1; }
template <class S, int K, int NI, int NO>
int conv(const void* src, const void* wf, float* out, const float* add, const float* bias, int nimg,
         hipStream_t st) {
  using L = LTile<S, K, conv_rb<S, K, NO>()>;
  LConvArgs a{src, wf, nullptr, nullptr, out, add, bias, nimg, lconv_fast_env()};
  if constexpr (sizeof(S) == 2 && K <= 7 && NO == 1) {
    if (lconvt8_env()) {
      hipLaunchKernelGGL((k_lconv<S, K, NI, NO, 2 * NT>), dim3(nimg * (IMG / conv_rb<S, K, NO>())), dim3(2 * NT),
                         L::BYTES, st, a);
      HIPCHK(hipGetLastError());
      return 0;
    }
  }
  hipLaunchKernelGGL((k_lconv<S, K, NI, NO>), dim3(nimg * (IMG / conv_rb<S, K, NO>())), dim3(NT),
                     L::BYTES, st, a);
  HIPCHK(hipGetLastError());
  return 0;
}

template <class S, int NI, int NO>
int conv_k(int K, const void* src, const void* wf, float* out, const float* add, const float* bias,
           int nimg, hipStream_t st) {
  int rc = 0;
  K_SWITCH(K, (rc = conv<S, KC, NI, NO>(src, wf, out, add, bias, nimg, st)));
  return rc;
}
// out = W0 * src0 + W1 * src1 + bias, the 4-gate forward with two input
// tensors in one launch (k_lconv DUAL): the clip ConvLSTM's per-step
// P_t = Wx x_t + Wh h_{t-1} + b
template <class S, int K>
constexpr int dual_lds_bytes() {           // both tiles, or the fused epilogue's gate exchange
  constexpr int T2 = 2 * LTile<S, K, conv_rb<S, K, 4>()>::BYTES, XG = 4 * 4 * 32 * 36 * 4;
  return T2 > XG ? T2 : XG;
}
template <class S, int K>
int conv_dual(const void* s0, const void* w0, const void* s1, const void* w1, float* out, const float* bias,
              int nimg, hipStream_t st, const float* cprev = nullptr, float* cout = nullptr,
              void* hout = nullptr, int ch = 0, bool* fused = nullptr) {
  const bool f = cout && dual_fuses<S, K, NT>();
  if (fused) *fused = f;
  LConvArgs a{s0, w0, s1, w1, out, nullptr, bias, nimg, lconv_fast_env(), f ? cprev : nullptr,
              f ? cout : nullptr, f ? hout : nullptr, ch};
  hipLaunchKernelGGL((k_lconv<S, K, 2, 4, NT, true>), dim3(nimg * (IMG / conv_rb<S, K, 4>())), dim3(NT),
                     (dual_lds_bytes<S, K>()), st, a);
  HIPCHK(hipGetLastError());
  return 0;
}
template <class S>
int conv_dual_k(int K, const void* s0, const void* w0, const void* s1, const void* w1, float* out,
                const float* bias, int nimg, hipStream_t st, const float* cprev = nullptr,
                float* cout = nullptr, void* hout = nullptr, int ch = 0, bool* fused = nullptr) {
  int rc = 0;
  K_SWITCH(K, (rc = conv_dual<S, KC>(s0, w0, s1, w1, out, bias, nimg, st, cprev, cout, hout, ch, fused)));
  return rc;
}

// k_lwgrad2 for bf16 k <= 7: opt-in (PT_LWGRAD2=1, diagnostic builds only, read per call).  Measured
// r04 (cfg3, profiles/r04_lwgrad2_ab.txt): 47.56 vs 46.96 ms per step for
// k_lwgrad -- its 2.3x fewer LDS reads did not pay for the 2.5x taller X band
// (the K - 1 halo rows) and the D fragments read at every band start.
int lwgrad2_env() { return PT_SW("PT_LWGRAD2", 0) == 1; }
template <class S, int K>
int wgrad(const LWgradArgs& a, hipStream_t st) {
  using Bd = LWBand<S, K>;
  if constexpr (sizeof(S) == 2 && K <= 7) {
    if (lwgrad2_env()) {
      hipLaunchKernelGGL((k_lwgrad2<K>), dim3(K * ((a.nsl + 7) / 8) * 8), dim3(NT), LWBand2<K>::BYTES, st, a);
      HIPCHK(hipGetLastError());
      return 0;
    }
  }
  hipLaunchKernelGGL((k_lwgrad<S, K>), dim3(K * ((a.nsl + 7) / 8) * 8), dim3(NT), Bd::BYTES, st, a);
  HIPCHK(hipGetLastError());
  return 0;
}

template <class S>
int wgrad_k(int K, const LWgradArgs& a, hipStream_t st) {
  int rc = 0;
  K_SWITCH(K, (rc = wgrad<S, KC>(a, st)));
  return rc;
}

// dynamic-LDS limits of the K-specific kernels, set once per (S, K) outside
// any stream capture
template <class S, int K>
int prime_k() {
  static bool done = false;     // idempotent; a race only repeats the calls
  if (done) return 0;
  SETLDS((k_lconv<S, K, 1, 4>), (LTile<S, K, conv_rb<S, K, 4>()>::BYTES));
  SETLDS((k_lconv<S, K, 2, 4, NT, true>), (dual_lds_bytes<S, K>()));
  SETLDS((k_lconv<S, K, 4, 1>), (LTile<S, K, conv_rb<S, K, 1>()>::BYTES));
  if constexpr (sizeof(S) == 2 && K <= 7) SETLDS((k_lconv<S, K, 4, 1, 2 * NT>), (LTile<S, K, conv_rb<S, K, 1>()>::BYTES));
  SETLDS((k_lwgrad<S, K>), (LWBand<S, K>::BYTES));
  if constexpr (sizeof(S) == 2 && K <= 7) SETLDS((k_lwgrad2<K>), (LWBand2<K>::BYTES));
  done = true;
  return 0;
}
template <class S>
int prime(int K) {
  int rc = 0;
  K_SWITCH(K, (rc = prime_k<S, KC>()));
  return rc;
}

ptg::GraphCache g_graphs;

inline dim3 grid_for(size_t n, int bs = 256) {
  size_t g = (n + bs - 1) / bs;
  return dim3((unsigned)(g > 8192 ? 8192 : (g < 1 ? 1 : g)));
}

template <class S>
int run_forward(const pt_lstm_desc* d, const float* x, const pt_lstm_params* pr, const float* h0,
                const float* c0, char* sv, float* h_out, float* c_out, hipStream_t st,
                const StemIn* sm = nullptr) {
  const LPlan p = plan(d);
  const int npix = (int)p.npix;
  LPrepArgs pa{};
  pa.K = p.K; pa.ch = p.ch; pa.cin = p.cin;
  for (int g = 0; g < 4; ++g) {
    if (!pr->wx[g] || !pr->wh[g]) return fail(PT_LSTM_ERR_ARG, "missing gate weight %ld", g);
    pa.wx[g] = pr->wx[g]; pa.wh[g] = pr->wh[g]; pa.bx[g] = pr->bx[g];
  }
  for (int i = 0; i < 4; ++i) pa.fr[i] = sv + p.o_fr[i];
  pa.bias = (float*)(sv + p.o_bias);
  pa.frlo = p.xsplit ? sv + p.o_frlo : nullptr;
  hipLaunchKernelGGL(k_lprep<S>, dim3(1024), dim3(256), 0, st, pa);
  HIPCHK(hipGetLastError());

  S* xcl = (S*)(sv + p.o_x);
  if (sm) {                  // the stem straight into the per-step input (k_stem_cl_fwd)
    switch (sm->cin) {
#define STEM_CF(CI) case CI: hipLaunchKernelGGL((k_stem_cl_fwd<CI, S>), dim3(p.B * p.T), dim3(256), 0, st, sm->x, sm->xu8, sm->w, sm->b, xcl, p.cin, p.B, p.T); break;
      STEM_CF(1) STEM_CF(2) STEM_CF(3) STEM_CF(4)
#undef STEM_CF
    }
  } else if (p.xseq)
    hipLaunchKernelGGL(k_to_cl_seq<S>, dim3(p.B * p.T * (NPIX / SEQ_CH)), dim3(256), 0, st, x, xcl,
                       p.B, p.cin, p.T);
  else
    hipLaunchKernelGGL(k_to_cl<S>, grid_for(p.npix * HC), dim3(256), 0, st, x, xcl, p.B, p.cin, 1, 0,
                       p.xsplit ? (S*)(sv + p.o_xlo) : nullptr);
  S* hinit = h0 ? (S*)(sv + p.o_h0) : nullptr;
  float* cinit = c0 ? (float*)(sv + p.o_c0) : nullptr;
  if (h0) hipLaunchKernelGGL(k_to_cl<S>, grid_for(p.npix * HC), dim3(256), 0, st, h0, hinit, p.B, p.ch);
  if (c0) hipLaunchKernelGGL(k_to_cl<float>, grid_for(p.npix * HC), dim3(256), 0, st, c0, cinit, p.B, p.ch);
  HIPCHK(hipGetLastError());

  float* P = (float*)(sv + p.o_P);
  S* H = (S*)(sv + p.o_h);
  float* Cc = (float*)(sv + p.o_c);
  const size_t pstep = p.npix * GC, hstep = p.npix * HC;
  // static x: xg = Wx*x + b once, P_t = xg + Wh*h_{t-1}; per-step x:
  // P_t = Wx*x_t + b, then += Wh*h_{t-1} in place
  // static x: xg = Wx*x + b (without h0, P_0 = xg); per-step x: the
  // x-convolutions of all steps do not depend on h, so ONE launch over the
  // B*T images writes every P_t = Wx*x_t + b ([T][B] image order in xcl and P)
  // per-step x without h0 (r05, the clip ConvLSTM): step 0's x-conv alone,
  // then ONE launch per step for both convs (conv_dual)
  // (bf16 k > 7: the plain column loop's two-source form spills at two waves
  // per SIMD; those shapes keep the all-steps x-conv + per-step h-conv)
  const bool dual = p.xseq && !hinit && !(sizeof(S) == 2 && p.K > 7);
  float* xg = p.xseq ? nullptr : (h0 ? (float*)(sv + p.o_xg) : P);
  if (int rc = conv_k<S, 1, 4>(p.K, xcl, sv + p.o_fr[0], p.xseq ? P : xg, nullptr, pa.bias,
                               dual ? p.B : p.xseq ? p.B * p.T : p.B, st))
    return rc;
  if (p.xsplit) {        // xg += Wx_hi x_lo + Wx_lo x_hi (in place: out = acc + add, per thread)
    if (int rc = conv_k<S, 1, 4>(p.K, sv + p.o_xlo, sv + p.o_fr[0], xg, xg, nullptr, p.B, st)) return rc;
    if (int rc = conv_k<S, 1, 4>(p.K, xcl, sv + p.o_frlo, xg, xg, nullptr, p.B, st)) return rc;
  }
  for (int t = 0; t < p.T; ++t) {
    const S* hin = t == 0 ? hinit : H + (t - 1) * hstep;
    if (dual && t > 0) {     // (r05) + the step's point-wise update in the conv's epilogue
      const bool fuse = lpw_fuse_env();
      bool fused = false;      // the instantiation ran the update (dual_fuses)
      if (int rc = conv_dual_k<S>(p.K, xcl + t * hstep, sv + p.o_fr[0], hin, sv + p.o_fr[1], P + t * pstep,
                                  pa.bias, p.B, st, fuse ? Cc + (t - 1) * hstep : nullptr,
                                  fuse ? Cc + t * hstep : nullptr, fuse ? H + t * hstep : nullptr, p.ch,
                                  &fused))
        return rc;
      if (fused) continue;
    } else if (hin) {
      if (int rc = conv_k<S, 1, 4>(p.K, hin, sv + p.o_fr[1], P + t * pstep,
                                   p.xseq ? P + t * pstep : xg, nullptr, p.B, st))
        return rc;
    }
    const float* cprev = t == 0 ? cinit : Cc + (t - 1) * hstep;
    hipLaunchKernelGGL(k_lpw_fwd<S>, grid_for((size_t)npix * 8), dim3(256), 0, st,
                       (const float*)(P + t * pstep), cprev, Cc + t * hstep, H + t * hstep, npix, p.ch);
    HIPCHK(hipGetLastError());
  }
  if (h_out)
    hipLaunchKernelGGL(k_from_cl<S>, grid_for(p.npix * p.ch), dim3(256), 0, st,
                       (const S*)(H + (p.T - 1) * hstep), h_out, p.B, p.ch);
  if (c_out)
    hipLaunchKernelGGL(k_from_cl<float>, grid_for(p.npix * p.ch), dim3(256), 0, st,
                       (const float*)(Cc + (p.T - 1) * hstep), c_out, p.B, p.ch);
  HIPCHK(hipGetLastError());
  return 0;
}

template <class S>
int run_backward(const pt_lstm_desc* d, const char* sv, char* ws,
                 const float* d_h, const float* d_c, const pt_lstm_grads* g, int has_h0,
                 int has_c0, hipStream_t st, const StemIn* sm = nullptr, float* dws = nullptr,
                 float* dbs = nullptr) {
  const LPlan p = plan(d);
  const int npix = (int)p.npix;
  const size_t pstep = p.npix * GC, hstep = p.npix * HC;
  const float* P = (const float*)(sv + p.o_P);
  const S* H = (const S*)(sv + p.o_h);
  const float* Cc = (const float*)(sv + p.o_c);
  const float* cinit = has_c0 ? (const float*)(sv + p.o_c0) : nullptr;
  float* dh = (float*)(ws + p.o_dh);
  float* dc = (float*)(ws + p.o_dc);
  S* dP = (S*)(ws + p.o_dP);
  float* dPsum = p.xseq ? nullptr : (float*)(ws + p.o_dPsum);
  S* dPsumS = p.xseq ? nullptr : (S*)(ws + p.o_dPsumS);

  hipLaunchKernelGGL(k_to_cl<float>, grid_for(p.npix * HC), dim3(256), 0, st, d_h, dh, p.B, p.ch);
  if (d_c)
    hipLaunchKernelGGL(k_to_cl<float>, grid_for(p.npix * HC), dim3(256), 0, st, d_c, dc, p.B, p.ch);
  else
    HIPCHK(zero_async(dc, p.npix * HC * 4, st));
  HIPCHK(hipGetLastError());
  const bool want_dh0 = has_h0 && g->d_h0;
  for (int t = p.T - 1; t >= 0; --t) {
    const float* cprev = t == 0 ? cinit : Cc + (t - 1) * hstep;
    hipLaunchKernelGGL(k_lpw_bwd<S>, grid_for((size_t)npix * 8), dim3(256), 0, st, (const float*)dh,
                       dc, P + t * pstep, Cc + t * hstep, cprev, dP + t * pstep, dPsum,
                       t == 0 ? dPsumS : (S*)nullptr, (int)(t == p.T - 1), npix, p.ch);
    HIPCHK(hipGetLastError());
    if (t > 0 || want_dh0)
      if (int rc = conv_k<S, 4, 1>(p.K, dP + t * pstep, sv + p.o_fr[2], dh, nullptr, nullptr, p.B, st))
        return rc;
  }
  if (want_dh0)
    hipLaunchKernelGGL(k_from_cl<float>, grid_for(p.npix * p.ch), dim3(256), 0, st,
                       (const float*)dh, g->d_h0, p.B, p.ch);
  if (has_c0 && g->d_c0)
    hipLaunchKernelGGL(k_from_cl<float>, grid_for(p.npix * p.ch), dim3(256), 0, st,
                       (const float*)dc, g->d_c0, p.B, p.ch);
  HIPCHK(hipGetLastError());

  // weight gradients: Wh over (h_{t-1}, dP_t), t >= 1 (+ (h0, dP_0)); Wx over (x, sum_t dP_t)
  LWgradArgs wa{};
  wa.X0 = H; wa.D0 = dP + pstep; wa.n0 = p.B * (p.T - 1);
  wa.X1 = sv + p.o_h0; wa.D1 = dP; wa.n1 = has_h0 ? p.B : 0;
  wa.nsl = p.nsl_h;
  wa.wslab = (float*)(ws + p.o_wsh);
  if (int rc = wgrad_k<S>(p.K, wa, st)) return rc;
  LWgradArgs wx{};
  // static x: one image against sum_t dP_t; per-step x: every (x_t, dP_t)
  wx.X0 = sv + p.o_x; wx.D0 = p.xseq ? (const void*)dP : (const void*)dPsumS;
  wx.n0 = p.xseq ? p.B * p.T : p.B;
  wx.X1 = nullptr; wx.D1 = nullptr; wx.n1 = 0;
  wx.nsl = p.nsl_x;
  wx.wslab = (float*)(ws + p.o_wsx);
  if (int rc = wgrad_k<S>(p.K, wx, st)) return rc;
  float* colp = (float*)(ws + p.o_col);
  if (p.xseq)
    hipLaunchKernelGGL(k_lcolsum<S>, dim3(p.nb), dim3(256), 0, st, (const S*)dP, colp, npix * p.T);
  else
    hipLaunchKernelGGL(k_lcolsum<float>, dim3(p.nb), dim3(256), 0, st, (const float*)dPsum, colp, npix);
  LReduceArgs ra{};
  ra.K = p.K; ra.nsl_h = p.nsl_h; ra.nsl_x = p.nsl_x; ra.ch = p.ch; ra.cin = p.cin; ra.nb = p.nb;
  ra.wslab_h = wa.wslab; ra.wslab_x = wx.wslab; ra.colpart = colp;
  for (int i = 0; i < 4; ++i) { ra.wh[i] = g->wh[i]; ra.wx[i] = g->wx[i]; ra.bx[i] = g->bx[i]; }
  hipLaunchKernelGGL(k_lreduce, dim3(1024), dim3(256), 0, st, ra);
  HIPCHK(hipGetLastError());
  const bool stem_g = sm && (dws || dbs);
  if (g->d_x || stem_g) {
    if (p.xseq) {        // all steps' d x_t from one transposed conv over the B*T images
      float* dxs = (float*)(ws + p.o_dx);
      if (int rc = conv_k<S, 4, 1>(p.K, dP, sv + p.o_fr[3], dxs, nullptr, nullptr, p.B * p.T, st))
        return rc;
      if (stem_g) {      // the fused stem's dW / db straight from d x_t (k_stem_cl_bwd)
        float* part = (float*)(ws + p.o_stem);
        switch (sm->cin) {
#define STEM_CB(CI) case CI: hipLaunchKernelGGL(k_stem_cl_bwd<CI>, dim3(STEM_BLOCKS), dim3(256), 0, st, sm->x, sm->xu8, sm->w, sm->b, (const float*)dxs, part, p.cin, p.B, p.T); break;
          STEM_CB(1) STEM_CB(2) STEM_CB(3) STEM_CB(4)
#undef STEM_CB
        }
        HIPCHK(hipGetLastError());
        hipLaunchKernelGGL(k_stem_reduce, dim3(32 * (sm->cin + 1)), dim3(256), 0, st, (const float*)part,
                           STEM_BLOCKS, sm->cin, p.cin, dws, dbs);
      }
      if (g->d_x)
        hipLaunchKernelGGL(k_from_cl_seq<float>, dim3(p.B * p.T * (NPIX / SEQ_CH)), dim3(256), 0, st,
                           (const float*)dxs, g->d_x, p.B, p.cin, p.T);
    } else {
      if (int rc = conv_k<S, 4, 1>(p.K, dPsumS, sv + p.o_fr[3], dh, nullptr, nullptr, p.B, st))
        return rc;
      hipLaunchKernelGGL(k_from_cl<float>, grid_for(p.npix * p.cin), dim3(256), 0, st,
                         (const float*)dh, g->d_x, p.B, p.cin);
    }
    HIPCHK(hipGetLastError());
  }
  return 0;
}

template <class S>
int run_jv(const pt_lstm_desc* d, const char* sv, char* ws, float mu, float* jv, hipStream_t st) {
  const LPlan p = plan(d);
  const int npix = (int)p.npix;
  const size_t pstep = p.npix * GC, hstep = p.npix * HC;
  const float* P = (const float*)(sv + p.o_P);
  const float* Cc = (const float*)(sv + p.o_c);
  S* jP = (S*)(ws + p.o_jvP);
  float* jdh = (float*)(ws + p.o_dh);
  const int t = p.T - 1;
  hipLaunchKernelGGL(k_ljv_seed<S>, grid_for((size_t)npix * 8), dim3(256), 0, st, P + t * pstep,
                     Cc + t * hstep, Cc + (t - 1) * hstep, jP, npix, p.ch);
  HIPCHK(hipGetLastError());
  if (int rc = conv_k<S, 4, 1>(p.K, jP, sv + p.o_fr[2], jdh, nullptr, nullptr, 2 * p.B, st)) return rc;
  hipLaunchKernelGGL(k_ljv_final, grid_for(p.npix * p.ch), dim3(256), 0, st, (const float*)jdh,
                     P + t * pstep, P + (t - 1) * pstep, Cc + (t - 1) * hstep, mu, jv, p.B, p.ch);
  HIPCHK(hipGetLastError());
  return 0;
}


int stem_check(const void* x, const float* w, int B, int cin, int cout, long long n) {
  if (!x || !w) return fail(PT_LSTM_ERR_ARG, "null x / w%ld");
  if (B < 1 || cin < 1 || cin > 4 || cout < 1 || cout > 32)
    return fail(PT_LSTM_ERR_UNSUPPORTED, "stem needs B >= 1, cin 1..4, cout 1..32 (cin=%ld)", cin);
  if (n < 4 || n % 4) return fail(PT_LSTM_ERR_UNSUPPORTED, "stem voxel count must be a multiple of 4 (%ld)", (long)n);
  return 0;
}

}  // namespace

extern "C" {

size_t pt_lstm_saved_bytes(const pt_lstm_desc* d) {
  if (check(d)) return 0;
  return plan(d).saved;
}
size_t pt_lstm_workspace_bytes(const pt_lstm_desc* d) {
  if (check(d)) return 0;
  return plan(d).ws;
}

int pt_lstm_forward(const pt_lstm_desc* d, const float* x, const pt_lstm_params* p,
                    const float* h0, const float* c0, void* saved, float* h_out, float* c_out,
                    pt_lstm_stream_t stream) {
  if (int rc = check(d)) return rc;
  if (!x || !p || !saved) return fail(PT_LSTM_ERR_ARG, "null x / params / saved%ld");
  if (!!h0 != !!(d->init_state & PT_LSTM_H0) || !!c0 != !!(d->init_state & PT_LSTM_C0))
    return fail(PT_LSTM_ERR_ARG, "h0 / c0 do not match desc.init_state (%ld)", d->init_state);
  const bool bf = d->dtype == PT_LSTM_BF16;
  if (int rc = bf ? prime<bf16_t>(d->ksize) : prime<float>(d->ksize)) return rc;
  auto body = [&](hipStream_t s) {
    return bf ? run_forward<bf16_t>(d, x, p, h0, c0, (char*)saved, h_out, c_out, s)
              : run_forward<float>(d, x, p, h0, c0, (char*)saved, h_out, c_out, s);
  };
  hipStream_t st = (hipStream_t)stream;
  if (!ptg::graphs_enabled()) return body(st);
  ptg::Key k;
  k.add(1).add(*d).add(x).add(*p).add(h0).add(c0).add(saved).add(h_out).add(c_out).add(lconv_fast_env()).add(lwgrad2_env()).add(lconvt8_env()).add(lpw_fuse_env());
  return g_graphs.run(k.b.data(), k.b.size(), st, PT_LSTM_ERR_HIP, body);
}

int pt_lstm_backward(const pt_lstm_desc* d, const void* saved, void* workspace, const float* d_h,
                     const float* d_c, const pt_lstm_grads* g, pt_lstm_stream_t stream) {
  if (int rc = check(d)) return rc;
  if (!saved || !workspace || !d_h || !g) return fail(PT_LSTM_ERR_ARG, "null saved / workspace / d_h / grads%ld");
  const int hh = (d->init_state & PT_LSTM_H0) != 0, hc = (d->init_state & PT_LSTM_C0) != 0;
  const bool bf = d->dtype == PT_LSTM_BF16;
  if (int rc = bf ? prime<bf16_t>(d->ksize) : prime<float>(d->ksize)) return rc;
  auto body = [&](hipStream_t s) {
    return bf ? run_backward<bf16_t>(d, (const char*)saved, (char*)workspace, d_h, d_c, g, hh, hc, s)
              : run_backward<float>(d, (const char*)saved, (char*)workspace, d_h, d_c, g, hh, hc, s);
  };
  hipStream_t st = (hipStream_t)stream;
  if (!ptg::graphs_enabled()) return body(st);
  ptg::Key k;
  k.add(2).add(*d).add(saved).add(workspace).add(d_h).add(d_c).add(*g).add(lconv_fast_env()).add(lwgrad2_env()).add(lconvt8_env()).add(lpw_fuse_env());
  return g_graphs.run(k.b.data(), k.b.size(), st, PT_LSTM_ERR_HIP, body);
}

int pt_lstm_forward_stem(const pt_lstm_desc* d, const void* x, int x_u8, int cin_s, const float* ws,
                         const float* bs, const pt_lstm_params* p, void* saved, float* h_out,
                         float* c_out, pt_lstm_stream_t stream) {
  if (int rc = check(d)) return rc;
  if (!d->x_seq) return fail(PT_LSTM_ERR_UNSUPPORTED, "the fused stem needs x_seq = 1%ld");
  if (d->init_state) return fail(PT_LSTM_ERR_UNSUPPORTED, "the fused stem starts from h0 = c0 = 0 (init_state %ld)", d->init_state);
  if (int rc = stem_check(x, ws, d->batch, cin_s, d->in_channels, 4)) return rc;
  if (x_u8 != 0 && x_u8 != 1) return fail(PT_LSTM_ERR_ARG, "bad x_u8 (%ld)", x_u8);
  if (!bs || !p || !saved) return fail(PT_LSTM_ERR_ARG, "null bs / params / saved%ld");
  const bool bf = d->dtype == PT_LSTM_BF16;
  if (int rc = bf ? prime<bf16_t>(d->ksize) : prime<float>(d->ksize)) return rc;
  const StemIn sm{x, x_u8, cin_s, ws, bs};
  auto body = [&](hipStream_t s) {
    return bf ? run_forward<bf16_t>(d, nullptr, p, nullptr, nullptr, (char*)saved, h_out, c_out, s, &sm)
              : run_forward<float>(d, nullptr, p, nullptr, nullptr, (char*)saved, h_out, c_out, s, &sm);
  };
  hipStream_t st = (hipStream_t)stream;
  if (!ptg::graphs_enabled()) return body(st);
  ptg::Key k;
  k.add(3).add(*d).add(x).add(x_u8).add(cin_s).add(ws).add(bs).add(*p).add(saved).add(h_out).add(c_out)
      .add(lconv_fast_env()).add(lwgrad2_env()).add(lconvt8_env()).add(lpw_fuse_env());
  return g_graphs.run(k.b.data(), k.b.size(), st, PT_LSTM_ERR_HIP, body);
}

int pt_lstm_backward_stem(const pt_lstm_desc* d, const void* x, int x_u8, int cin_s, const float* ws,
                          const float* bs, const void* saved, void* workspace, const float* d_h,
                          const float* d_c, const pt_lstm_grads* g, float* dws, float* dbs,
                          pt_lstm_stream_t stream) {
  if (int rc = check(d)) return rc;
  if (!d->x_seq || d->init_state)
    return fail(PT_LSTM_ERR_UNSUPPORTED, "the fused stem needs x_seq = 1 and h0 = c0 = 0 (init_state %ld)", d->init_state);
  if (int rc = stem_check(x, ws, d->batch, cin_s, d->in_channels, 4)) return rc;
  if (x_u8 != 0 && x_u8 != 1) return fail(PT_LSTM_ERR_ARG, "bad x_u8 (%ld)", x_u8);
  if (!bs || !saved || !workspace || !d_h || !g)
    return fail(PT_LSTM_ERR_ARG, "null bs / saved / workspace / d_h / grads%ld");
  const bool bf = d->dtype == PT_LSTM_BF16;
  if (int rc = bf ? prime<bf16_t>(d->ksize) : prime<float>(d->ksize)) return rc;
  const StemIn sm{x, x_u8, cin_s, ws, bs};
  auto body = [&](hipStream_t s) {
    return bf ? run_backward<bf16_t>(d, (const char*)saved, (char*)workspace, d_h, d_c, g, 0, 0, s, &sm, dws, dbs)
              : run_backward<float>(d, (const char*)saved, (char*)workspace, d_h, d_c, g, 0, 0, s, &sm, dws, dbs);
  };
  hipStream_t st = (hipStream_t)stream;
  if (!ptg::graphs_enabled()) return body(st);
  ptg::Key k;
  k.add(4).add(*d).add(x).add(x_u8).add(cin_s).add(ws).add(bs).add(saved).add(workspace).add(d_h).add(d_c)
      .add(*g).add(dws).add(dbs).add(lconv_fast_env()).add(lwgrad2_env()).add(lconvt8_env()).add(lpw_fuse_env());
  return g_graphs.run(k.b.data(), k.b.size(), st, PT_LSTM_ERR_HIP, body);
}

int pt_lstm_jv_penalty(const pt_lstm_desc* d, const void* saved, void* workspace, float mu,
                       float* jv, pt_lstm_stream_t stream) {
  if (int rc = check(d)) return rc;
  if (d->steps < 2)
    return fail(PT_LSTM_ERR_ARG, "the Jacobian penalty needs steps >= 2 (got %ld)", d->steps);
  if (!saved || !workspace || !jv) return fail(PT_LSTM_ERR_ARG, "null saved / workspace / jv%ld");
  const bool bf = d->dtype == PT_LSTM_BF16;
  if (int rc = bf ? prime<bf16_t>(d->ksize) : prime<float>(d->ksize)) return rc;
  hipStream_t st = (hipStream_t)stream;
  return bf ? run_jv<bf16_t>(d, (const char*)saved, (char*)workspace, mu, jv, st)
            : run_jv<float>(d, (const char*)saved, (char*)workspace, mu, jv, st);
}

int pt_lstm_export_h(const pt_lstm_desc* d, const void* saved, float* h_seq,
                     pt_lstm_stream_t stream) {
  if (int rc = check(d)) return rc;
  if (!saved || !h_seq) return fail(PT_LSTM_ERR_ARG, "null saved / h_seq%ld");
  const LPlan p = plan(d);
  hipStream_t st = (hipStream_t)stream;
  const char* H = (const char*)saved + p.o_h;
  if (d->dtype == PT_LSTM_BF16)
    hipLaunchKernelGGL(k_from_cl_seq<bf16_t>, dim3(p.B * p.T * (NPIX / SEQ_CH)), dim3(256), 0, st,
                       (const bf16_t*)H, h_seq, p.B, p.ch, p.T);
  else
    hipLaunchKernelGGL(k_from_cl_seq<float>, dim3(p.B * p.T * (NPIX / SEQ_CH)), dim3(256), 0, st,
                       (const float*)H, h_seq, p.B, p.ch, p.T);
  HIPCHK(hipGetLastError());
  return 0;
}

size_t pt_lstm_stem_workspace_bytes(int cin) {
  return cin < 1 || cin > 4 ? 0 : (size_t)STEM_BLOCKS * 32 * (cin + 1) * sizeof(float);
}

int pt_lstm_stem_forward(const void* x, int x_u8, const float* w, const float* b, int B, int cin,
                         int cout, long long n, float* y, pt_lstm_stream_t stream) {
  if (int rc = stem_check(x, w, B, cin, cout, n)) return rc;
  if (x_u8 != 0 && x_u8 != 1) return fail(PT_LSTM_ERR_ARG, "bad x_u8 (%ld)", x_u8);
  if (!b || !y) return fail(PT_LSTM_ERR_ARG, "null b / y%ld");
  const long n4 = (long)(n / 4), total4 = (long)B * n4;
  const int grid = (int)std::min<long>((total4 + 255) / 256, 8192);
  hipStream_t st = (hipStream_t)stream;
  switch (cin) {
#define STEM_F(C) case C: hipLaunchKernelGGL(k_stem_fwd<C>, dim3(grid), dim3(256), 0, st, x, x_u8, w, b, (float4*)y, cout, n4, total4); break;
    STEM_F(1) STEM_F(2) STEM_F(3) STEM_F(4)
#undef STEM_F
  }
  HIPCHK(hipGetLastError());
  return 0;
}

int pt_lstm_stem_backward(const void* x, int x_u8, const float* w, const float* b, const float* dy,
                          int B, int cin, int cout, long long n, void* workspace, float* dw,
                          float* db, pt_lstm_stream_t stream) {
  if (int rc = stem_check(x, w, B, cin, cout, n)) return rc;
  if (x_u8 != 0 && x_u8 != 1) return fail(PT_LSTM_ERR_ARG, "bad x_u8 (%ld)", x_u8);
  if (!b || !dy || !workspace) return fail(PT_LSTM_ERR_ARG, "null b / dy / workspace%ld");
  const long n4 = (long)(n / 4), total4 = (long)B * n4;
  hipStream_t st = (hipStream_t)stream;
  float* part = (float*)workspace;
  switch (cin) {
#define STEM_B(C) case C: hipLaunchKernelGGL(k_stem_bwd<C>, dim3(STEM_BLOCKS), dim3(256), 0, st, x, x_u8, w, b, (const float4*)dy, part, cout, n4, total4); break;
    STEM_B(1) STEM_B(2) STEM_B(3) STEM_B(4)
#undef STEM_B
  }
  HIPCHK(hipGetLastError());
  hipLaunchKernelGGL(k_stem_reduce, dim3(32 * (cin + 1)), dim3(256), 0, st, (const float*)part, STEM_BLOCKS, cin, cout, dw, db);
  HIPCHK(hipGetLastError());
  return 0;
}

const char* pt_lstm_last_error(void) { return g_err; }
#ifndef PT_SRC_HASH
#define PT_SRC_HASH "unstamped"
#endif
#if PT_DIAG
const char* pt_lstm_version(void) { return "pt_lstm 0.2 gfx950 diag src " PT_SRC_HASH; }
#else
const char* pt_lstm_version(void) { return "pt_lstm 0.2 gfx950 src " PT_SRC_HASH; }
#endif

}  // extern "C"
