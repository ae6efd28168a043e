// pt_cell.hip — InT recurrent cell, forward + BPTT backward, for MI355X (gfx950).
//
// Reference path replaced (paths relative to the reference repo):
//   frame loop      models/InT.py:223-235          -> k_fwd_a / k_fwd_b per frame
//   rCell.forward   models/InT.py:145-179          -> split at the two BatchNorms
//   autograd BPTT   mainclean.py:204 (loss.backward) -> k_bwd_a / k_bwd_b per frame,
//                                                     k_wgrad (7x7 weight grads), k_reduce
//
// One workgroup (4 waves) owns one clip for a whole frame step: the 32x32
// image is exactly one 38x38 zero-halo LDS tile, so the k x k convolutions need
// no halo exchange.  The only cross-clip coupling is BatchNorm's batch
// statistics (track_running_stats=False, models/InT.py:102): each kernel ends
// by publishing per-clip partial statistics, and the next kernel reduces them
// (kernel boundary = grid-wide sync).  Per frame:
//   FA(t): [E_{t-1} update (needs BN1(t-1))] att, gE, eg; conv(gE, w_inh) -> ci, BN0 partials
//   FB(t): [BN0(t)] Ihat, inh gate, I_t;              conv(I_t, w_exc) -> ce, BN1 partials
// and FA(T) closes the last frame.  Backward mirrors this (see k_bwd_a/b).
#include "pt_device.h"
#include "../../include/pt_cell.h"

#include <stdio.h>
#include <string.h>
#include <mutex>
#include <vector>

namespace ptc {

// ----------------------------------------------------------------- small slab
// Per-clip gradient accumulator ("slab"), RMW'd by the backward kernels of its
// own clip only (no atomics), reduced over clips at the end.
enum SmallSlot {
  SM_ALPHA = 0, SM_MU, SM_GAMMA, SM_KAPPA, SM_BN0W, SM_BN0B, SM_BN1W, SM_BN1B,
  SM_GBA, SM_GBI, SM_GBE, SM_PW0, SM_PW1, SM_PW2, SM_PB, NSMALL
};
constexpr int SLAB_G = 6 * 1024;                 // 6 gate weights [n][ci]
constexpr int SLAB = SLAB_G + NSMALL * 32;

constexpr int MISC_FLOATS = 2560;
template <class S>
constexpr int cell_lds_bytes() {
  return tile_bytes<S>() + NPIX * 16 /*xs*/ + NWAVE * 1024 * 4 /*scr*/ + MISC_FLOATS * 4;
}

struct Lds {
  char* tile;
  f32x4* xs;
  float* scr;     // [NWAVE][1024]
  float* stat;    // [4][32]
  float* red;     // [512]
  float* small;   // [NWAVE][NSMALL][32]
};
template <class S>
__device__ __forceinline__ Lds carve(char* smem) {
  Lds l;
  l.tile = smem;
  l.xs = (f32x4*)(smem + tile_bytes<S>());
  l.scr = (float*)(smem + tile_bytes<S>() + NPIX * 16);
  l.stat = l.scr + NWAVE * 1024;
  l.red = l.stat + 128;
  l.small = l.red + 512;
  return l;
}

// ----------------------------------------------------------------- arguments
template <class S>
struct CellArgs {
  using F = typename Tr<S>::frag;
  int B, T, K, act, no_inh;
  float eps;
  int t;
  const float* x;                       // [B][3][T][32][32]
  const float *wpre, *bpre;             // [32][3], [32]
  const float *alpha, *mu, *gamma, *kappa;
  const float *bnw0, *bnb0, *bnw1, *bnb1;
  const float* gb[6];                   // gate biases
  const F *wf_inh, *wf_exc, *wt_inh, *wt_exc;   // conv fragments (fwd, transposed)
  const F* gf[6];                       // 1x1 fragments, forward
  const F* gt[6];                       // 1x1 fragments, transposed (backward)
  S *E, *I, *gE, *ci, *ce, *eg;         // saved per frame [T][B][32][32][32]
  float* bnstat;                        // [T][4][32] mean0, rstd0, mean1, rstd1
  double* bnacc;                        // fwd BN sums [T][2][3][32]: sum mean_b, sum mean_b^2, sum M2_b
  float* gates;                         // [B][T][C][32][32] or null
  // backward
  float *dEn, *dcE, *dIl, *dEp, *dcI, *GI, *dgEp, *dxp;   // f32 [B][32][32][32]
  const float* GEfin;                   // f32 channels-last dE of the last frame
  S *dci_s, *dce_s;                     // [T][B][32][32][32] conv-output grads (for k_wgrad)
  double* bnbacc;                       // bwd BN sums [T][2][2][32]: sum dy, sum dy*xhat
  float* slab;                          // [B][SLAB]
};

__device__ __forceinline__ size_t fr_off(int t, int B) { return (size_t)t * B * NPIX * C; }
__device__ __forceinline__ size_t clip_off(int b) { return (size_t)b * NPIX * C; }

// Stage x[b, 0:3, t] as float4 per pixel.
__device__ void stage_x(const float* __restrict__ x, f32x4* xs, int b, int t, int T, int tid) {
  const float* x0 = x + ((size_t)(b * 3 + 0) * T + t) * NPIX;
  const float* x1 = x + ((size_t)(b * 3 + 1) * T + t) * NPIX;
  const float* x2 = x + ((size_t)(b * 3 + 2) * T + t) * NPIX;
  for (int p = tid; p < NPIX; p += NT) {
    f32x4 v;
    v[0] = x0[p]; v[1] = x1[p]; v[2] = x2[p]; v[3] = 0.f;
    xs[p] = v;
  }
}

// Stem (models/InT.py:212-213): z = W_pre x + b; xbn = nl(z); CL layout.
struct Stem { float w0, w1, w2, b; };
__device__ __forceinline__ void stem_cl(const f32x4* xs, int y, int h, const Stem& st, int act,
                                        f32x16& z, f32x16& xv) {
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const f32x4 v = xs[y * IMG + cl_x(r, h)];
    z[r] = st.w0 * v[0] + st.w1 * v[1] + st.w2 * v[2] + st.b;
    xv[r] = act_f(z[r], act);
  }
}

// Forward BN: batch mean / rstd per channel from the fp64 sums of per-clip
// (mean_b, mean_b^2, M2_b) (Chan et al.: M2 = sum M2_b + n (sum mean_b^2 -
// (sum mean_b)^2 / B)); all threads end with them in stat[0..63].
__device__ void bn_fwd_finalize(const double* __restrict__ acc, int B, float eps, float* stat,
                                float* gstat, int tid) {
  if (tid < 32) {
    const double s1 = acc[tid], s2 = acc[32 + tid], s3 = acc[64 + tid];
    const double mean = s1 / B;
    double m2 = s3 + (double)NPIX * (s2 - s1 * s1 / B);
    m2 = m2 > 0.0 ? m2 : 0.0;
    const float var = (float)(m2 / ((double)B * NPIX));
    const float rstd = 1.0f / sqrtf(var + eps);
    stat[tid] = (float)mean;
    stat[32 + tid] = rstd;
    if (gstat) { gstat[tid] = (float)mean; gstat[32 + tid] = rstd; }
  }
  __syncthreads();
}

// Backward BN: means of dy and dy*xhat from the fp64 sums, in stat[0..63].
__device__ void bn_bwd_finalize(const double* __restrict__ acc, int B, float* stat, int tid) {
  if (tid < 32) {
    const double inv = 1.0 / ((double)B * NPIX);
    stat[tid] = (float)(acc[tid] * inv);
    stat[32 + tid] = (float)(acc[32 + tid] * inv);
  }
  __syncthreads();
}

// Per-clip (mean, M2) of the conv outputs held in acc (two-pass, robust).
__device__ void bn_fwd_partial(const f32x16 (&acc)[RPW], float* red, double* out, int lane,
                               int wave, int tid) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < RPW; ++i) s += hsum16(acc[i]);
  s += __shfl_xor(s, 32);
  if (lane < 32) red[wave * 32 + lane] = s;
  __syncthreads();
  const int c = lane & 31;
  float mean = 0.f;
#pragma unroll
  for (int w = 0; w < NWAVE; ++w) mean += red[w * 32 + c];
  mean *= (1.f / NPIX);
  float m2 = 0.f;
#pragma unroll
  for (int i = 0; i < RPW; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) { const float d = acc[i][r] - mean; m2 += d * d; }
  m2 += __shfl_xor(m2, 32);
  __syncthreads();
  if (lane < 32) red[wave * 32 + lane] = m2;
  __syncthreads();
  if (tid < 32) {
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NWAVE; ++w) v += red[w * 32 + tid];
    unsafeAtomicAdd(out + tid, (double)mean);
    unsafeAtomicAdd(out + 32 + tid, (double)mean * (double)mean);
    unsafeAtomicAdd(out + 64 + tid, (double)v);
  }
}

// Workgroup sum of per-lane values for the lane's channel (halves combined):
// small[] gets every wave's contribution; thread tid<32*n reads totals.
template <int N>
__device__ void flush_small(float (&v)[N], const int (&slot)[N], float* small, float* slab_b,
                            int lane, int wave, int tid) {
#pragma unroll
  for (int k = 0; k < N; ++k) {
    const float s = v[k] + __shfl_xor(v[k], 32);
    if (lane < 32) small[(wave * N + k) * 32 + lane] = s;
  }
  __syncthreads();
  for (int e = tid; e < N * 32; e += NT) {
    const int k = e >> 5, c = e & 31;
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < NWAVE; ++w) s += small[(w * N + k) * 32 + c];
    slab_b[SLAB_G + slot[k] * 32 + c] += s;
  }
  __syncthreads();
}

// Sum a per-wave 1x1 weight-gradient tile (rows n, cols ci) over the waves
// and add it into the clip's slab.
__device__ void flush_gate(const f32x16& acc, float* scr, float* dst, int lane, int wave, int tid) {
  const int ci = lane & 31, h = lane >> 5;
#pragma unroll
  for (int r = 0; r < 16; ++r) scr[wave * 1024 + cl_x(r, h) * 32 + ci] = acc[r];
  __syncthreads();
  for (int e = tid; e < 1024; e += NT) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < NWAVE; ++w) s += scr[w * 1024 + e];
    dst[e] += s;
  }
  __syncthreads();
}

// Workgroup totals of two per-lane channel sums -> out[b][c] (BN bwd partials)
__device__ void bn_bwd_partial(float s0, float s1, float* red, double* out, int lane, int wave,
                               int tid) {
  s0 += __shfl_xor(s0, 32);
  s1 += __shfl_xor(s1, 32);
  if (lane < 32) { red[wave * 32 + lane] = s0; red[128 + wave * 32 + lane] = s1; }
  __syncthreads();
  if (tid < 32) {
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int w = 0; w < NWAVE; ++w) { a += red[w * 32 + tid]; b += red[128 + w * 32 + tid]; }
    unsafeAtomicAdd(out + tid, (double)a);
    unsafeAtomicAdd(out + 32 + tid, (double)b);
  }
  __syncthreads();
}

// =========================================================================
// Forward A (frame t, 0 <= t <= T):
//   t > 0 : close frame t-1: E_{t-1} = (1-eg) E_{t-2} + eg nl(BN1(ce) (kappa I_{t-1} + gamma))
//           (models/InT.py:172-175)
//   t < T : att = sig(a_w x_t + a_u E_{t-1}) (:148), gE = att*E_{t-1} (:153),
//           eg = sig(e_w I_{t-1} + e_u gE) (:171, uses the OLD inhibition),
//           ci = conv(gE, w_inh) (:161) -> BN0 partials
// =========================================================================
template <class S>
__global__ __launch_bounds__(NT, 1) void k_fwd_a(CellArgs<S> a) {
  using F = typename Tr<S>::frag;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const Lds L = carve<S>(smem);
  S* tile = (S*)L.tile;
  const int tid = threadIdx.x, lane = tid & 63, c = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int b = blockIdx.x, t = a.t, T = a.T, B = a.B;
  float* wscr = L.scr + wave * 1024;
  const size_t fs = fr_off(1, B), cb = clip_off(b);

  if (t < T) stage_x(a.x, L.xs, b, t, T, tid);
  if (t > 0)
    bn_fwd_finalize(a.bnacc + ((size_t)(t - 1) * 2 + 1) * 96, B, a.eps, L.stat + 64,
                    b == 0 ? a.bnstat + (size_t)(t - 1) * 128 + 64 : nullptr, tid);
  if (t < T && !a.no_inh) tile_zero<S>(tile, tid);
  __syncthreads();

  const Stem st{a.wpre[c * 3 + 0], a.wpre[c * 3 + 1], a.wpre[c * 3 + 2], a.bpre[c]};
  const float kap = a.kappa[c], gam = a.gamma[c], bw1 = a.bnw1[c], bb1 = a.bnb1[c];
  const float m1 = L.stat[64 + c], rs1 = L.stat[96 + c];
  const float ba = a.gb[0][c] + a.gb[1][c], be = a.gb[4][c] + a.gb[5][c];

  for (int i = 0; i < RPW; ++i) {
    const int y = wave * RPW + i;
    const size_t ro = cb + (size_t)y * IMG * C;
    f32x16 Ep = zero16(), Iv = zero16();
    if (t > 0) {
      Iv = load_cl(a.I + (t - 1) * fs + ro, c, h);
      const f32x16 Eo = t >= 2 ? load_cl(a.E + (t - 2) * fs + ro, c, h) : zero16();
      const f32x16 egv = load_cl(a.eg + (t - 1) * fs + ro, c, h);
      const f32x16 cev = load_cl(a.ce + (t - 1) * fs + ro, c, h);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float cn = bw1 * ((cev[r] - m1) * rs1) + bb1;
        const float eh = act_f(cn * (kap * Iv[r] + gam), a.act);
        Ep[r] = (1.f - egv[r]) * Eo[r] + egv[r] * eh;
      }
      store_cl(a.E + (t - 1) * fs + ro, c, h, Ep);
    }
    if (t == T) continue;
    f32x16 z, xv;
    stem_cl(L.xs, y, h, st, a.act, z, xv);
    F pax[Tr<S>::KS], pae[Tr<S>::KS];
    cl_to_pa<S>(wscr, xv, lane, pax);
    cl_to_pa<S>(wscr, Ep, lane, pae);
    f32x16 acc = zero16();
    acc = gemm_pa<S>(pax, a.gf[0], acc, lane);
    acc = gemm_pa<S>(pae, a.gf[1], acc, lane);
    f32x16 att, gEv;
#pragma unroll
    for (int r = 0; r < 16; ++r) { att[r] = sigm(acc[r] + ba); gEv[r] = att[r] * Ep[r]; }
    store_cl(a.gE + t * fs + ro, c, h, gEv);
    if (a.gates) {
      float* gp = a.gates + (((size_t)b * T + t) * C + c) * NPIX + y * IMG;
#pragma unroll
      for (int r = 0; r < 16; ++r) gp[cl_x(r, h)] = att[r];
    }
    // exc gate input: gated inhibition = old I (InT) or E (no_inh, :168)
    const f32x16 ginh = a.no_inh ? Ep : Iv;
    F pag[Tr<S>::KS], pai[Tr<S>::KS];
    cl_to_pa<S>(wscr, gEv, lane, pag);
    cl_to_pa<S>(wscr, ginh, lane, pai);
    acc = zero16();
    acc = gemm_pa<S>(pai, a.gf[4], acc, lane);
    acc = gemm_pa<S>(pag, a.gf[5], acc, lane);
    f32x16 egn;
#pragma unroll
    for (int r = 0; r < 16; ++r) egn[r] = sigm(acc[r] + be);
    store_cl(a.eg + t * fs + ro, c, h, egn);
  }
  if (t == T || a.no_inh) return;

  f32x16 acc[RPW];
#pragma unroll
  for (int i = 0; i < RPW; ++i) acc[i] = zero16();
  conv_run<S>(acc, a.gE + t * fs + cb, a.wf_inh, tile, a.K, wave * RPW, tid, lane);
#pragma unroll
  for (int i = 0; i < RPW; ++i)
    store_cl(a.ci + t * fs + cb + (size_t)(wave * RPW + i) * IMG * C, c, h, acc[i]);
  bn_fwd_partial(acc, L.red, a.bnacc + ((size_t)t * 2 + 0) * 96, lane, wave, tid);
}

// =========================================================================
// Forward B (frame t):  BN0 -> Ihat = nl(x - nl(c_i (alpha I + mu))) (:162),
//   ig = sig(i_w x + i_u I) (:165), I_t = (1-ig) I + ig Ihat (:166)
//   [no_inh: I_t = gE (:168)];  ce = conv(I_t, w_exc) (:172) -> BN1 partials
// =========================================================================
template <class S>
__global__ __launch_bounds__(NT, 1) void k_fwd_b(CellArgs<S> a) {
  using F = typename Tr<S>::frag;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const Lds L = carve<S>(smem);
  S* tile = (S*)L.tile;
  const int tid = threadIdx.x, lane = tid & 63, c = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int b = blockIdx.x, t = a.t, T = a.T, B = a.B;
  float* wscr = L.scr + wave * 1024;
  const size_t fs = fr_off(1, B), cb = clip_off(b);

  if (!a.no_inh) {
    stage_x(a.x, L.xs, b, t, T, tid);
    bn_fwd_finalize(a.bnacc + ((size_t)t * 2 + 0) * 96, B, a.eps, L.stat,
                    b == 0 ? a.bnstat + (size_t)t * 128 : nullptr, tid);
  }
  tile_zero<S>(tile, tid);
  __syncthreads();

  const Stem st{a.wpre[c * 3 + 0], a.wpre[c * 3 + 1], a.wpre[c * 3 + 2], a.bpre[c]};
  const float al = a.alpha[c], mu = a.mu[c], bw0 = a.bnw0[c], bb0 = a.bnb0[c];
  const float m0 = L.stat[c], rs0 = L.stat[32 + c];
  const float bi = a.gb[2][c] + a.gb[3][c];

  for (int i = 0; i < RPW; ++i) {
    const int y = wave * RPW + i;
    const size_t ro = cb + (size_t)y * IMG * C;
    f32x16 In;
    if (!a.no_inh) {
      const f32x16 civ = load_cl(a.ci + t * fs + ro, c, h);
      const f32x16 Iv = t > 0 ? load_cl(a.I + (t - 1) * fs + ro, c, h) : zero16();
      f32x16 z, xv, ih;
      stem_cl(L.xs, y, h, st, a.act, z, xv);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float cn = bw0 * ((civ[r] - m0) * rs0) + bb0;
        ih[r] = act_f(xv[r] - act_f(cn * (al * Iv[r] + mu), a.act), a.act);
      }
      F pax[Tr<S>::KS], pai[Tr<S>::KS];
      cl_to_pa<S>(wscr, xv, lane, pax);
      cl_to_pa<S>(wscr, Iv, lane, pai);
      f32x16 acc = zero16();
      acc = gemm_pa<S>(pax, a.gf[2], acc, lane);
      acc = gemm_pa<S>(pai, a.gf[3], acc, lane);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float ig = sigm(acc[r] + bi);
        In[r] = (1.f - ig) * Iv[r] + ig * ih[r];
      }
    } else {
      In = load_cl(a.gE + t * fs + ro, c, h);
    }
    store_cl(a.I + t * fs + ro, c, h, In);
  }

  f32x16 acc[RPW];
#pragma unroll
  for (int i = 0; i < RPW; ++i) acc[i] = zero16();
  conv_run<S>(acc, a.I + t * fs + cb, a.wf_exc, tile, a.K, wave * RPW, tid, lane);
#pragma unroll
  for (int i = 0; i < RPW; ++i)
    store_cl(a.ce + t * fs + cb + (size_t)(wave * RPW + i) * IMG * C, c, h, acc[i]);
  bn_fwd_partial(acc, L.red, a.bnacc + ((size_t)t * 2 + 1) * 96, lane, wave, tid);
}

// =========================================================================
// Backward A (t from T-1 down to -1).  Two halves:
//  tail (frame tt = t+1, if tt <= T-1): BN0 backward -> dci (saved for the
//     w_inh gradient), dgE = conv^T(dci, w_inh) + e_u^T d_e_pre (from k_bwd_b),
//     attention gate backward (a_w, a_u grads), dE_t complete, dx_{tt} complete
//     -> stem gradients.
//  head (frame t, if t >= 0): with dE_t: excitation update backward
//     (:175, :173) -> d_eg, dc_e (-> BN1 bwd partials), kappa/gamma grads,
//     dI_t (local), dE_{t-1} partial = (1-eg) dE_t.
// =========================================================================
template <class S>
__global__ __launch_bounds__(NT, 1) void k_bwd_a(CellArgs<S> a) {
  using F = typename Tr<S>::frag;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const Lds L = carve<S>(smem);
  S* tile = (S*)L.tile;
  const int tid = threadIdx.x, lane = tid & 63, c = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int b = blockIdx.x, t = a.t, T = a.T, B = a.B;
  float* wscr = L.scr + wave * 1024;
  const size_t fs = fr_off(1, B), cb = clip_off(b);
  const int tt = t + 1;
  const bool tail = tt <= T - 1, head = t >= 0;
  const bool conv = tail && head && !a.no_inh;   // E_{-1} = 0 makes the frame-0 conv^T dead
  float* slab_b = a.slab + (size_t)b * SLAB;

  if (tail) {
    stage_x(a.x, L.xs, b, tt, T, tid);
    if (!a.no_inh) bn_bwd_finalize(a.bnbacc + ((size_t)tt * 2 + 0) * 64, B, L.stat, tid);
  }
  if (conv) tile_zero<S>(tile, tid);
  __syncthreads();

  const Stem st{a.wpre[c * 3 + 0], a.wpre[c * 3 + 1], a.wpre[c * 3 + 2], a.bpre[c]};
  float sm[9] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int slots[9] = {SM_GBA, SM_KAPPA, SM_GAMMA, SM_BN1W, SM_BN1B, SM_PW0, SM_PW1, SM_PW2, SM_PB};
  f32x16 gaw = zero16(), gau = zero16();
  float bs0 = 0.f, bs1 = 0.f;   // BN1 bwd partial sums

  f32x16 acc[RPW];
#pragma unroll
  for (int i = 0; i < RPW; ++i) acc[i] = zero16();

  if (tail && !a.no_inh) {
    const float* bs = a.bnstat + (size_t)tt * 128;
    const float m0 = bs[c], rs0 = bs[32 + c], bw0 = a.bnw0[c];
    const float md = L.stat[c], mdx = L.stat[32 + c];
    for (int i = 0; i < RPW; ++i) {
      const int y = wave * RPW + i;
      const size_t ro = cb + (size_t)y * IMG * C;
      const f32x16 dcv = load_cl(a.dcI + ro, c, h);
      const f32x16 civ = load_cl(a.ci + tt * fs + ro, c, h);
      f32x16 v;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float xh = (civ[r] - m0) * rs0;
        v[r] = rs0 * bw0 * (dcv[r] - md - xh * mdx);
      }
      store_cl(a.dci_s + tt * fs + ro, c, h, v);
    }
    if (conv) conv_run<S>(acc, a.dci_s + tt * fs + cb, a.wt_inh, tile, a.K, wave * RPW, tid, lane);
  }

  const float ba = a.gb[0][c] + a.gb[1][c];
  const float kap = a.kappa[c], gam = a.gamma[c], bw1 = a.bnw1[c], bb1 = a.bnb1[c];
  float m1 = 0.f, rs1 = 0.f;
  if (head) { m1 = a.bnstat[(size_t)t * 128 + 64 + c]; rs1 = a.bnstat[(size_t)t * 128 + 96 + c]; }

  for (int i = 0; i < RPW; ++i) {
    const int y = wave * RPW + i;
    const size_t ro = cb + (size_t)y * IMG * C;
    f32x16 GE;
    if (tail) {
      f32x16 z, xv;
      stem_cl(L.xs, y, h, st, a.act, z, xv);
      f32x16 dx = load_cl(a.dxp + ro, c, h);
      if (head) {
        f32x16 dgE = load_cl(a.dgEp + ro, c, h);
        if (conv) dgE += acc[0];
        const f32x16 Et = load_cl(a.E + t * fs + ro, c, h);
        F pax[Tr<S>::KS], pae[Tr<S>::KS];
        cl_to_pa<S>(wscr, xv, lane, pax);
        cl_to_pa<S>(wscr, Et, lane, pae);
        f32x16 g = zero16();
        g = gemm_pa<S>(pax, a.gf[0], g, lane);
        g = gemm_pa<S>(pae, a.gf[1], g, lane);
        f32x16 att, dap;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          att[r] = sigm(g[r] + ba);
          dap[r] = dgE[r] * Et[r] * att[r] * (1.f - att[r]);
          sm[0] += dap[r];
        }
        gaw = wgrad_cl<S>(dap, xv, gaw);
        gau = wgrad_cl<S>(dap, Et, gau);
        F pad[Tr<S>::KS];
        cl_to_pa<S>(wscr, dap, lane, pad);
        GE = load_cl(a.dEn + ro, c, h);
#pragma unroll
        for (int r = 0; r < 16; ++r) GE[r] += dgE[r] * att[r];
        GE = gemm_pa<S>(pad, a.gt[1], GE, lane);
        dx = gemm_pa<S>(pad, a.gt[0], dx, lane);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const f32x4 xin = L.xs[y * IMG + cl_x(r, h)];
        const float dz = dx[r] * act_d(z[r], a.act);
        sm[5] += dz * xin[0]; sm[6] += dz * xin[1]; sm[7] += dz * xin[2]; sm[8] += dz;
      }
    } else {
      GE = load_cl(a.GEfin + ro, c, h);
    }
    if (head) {
      const f32x16 Iv = load_cl(a.I + t * fs + ro, c, h);
      const f32x16 cev = load_cl(a.ce + t * fs + ro, c, h);
      const f32x16 egv = load_cl(a.eg + t * fs + ro, c, h);
      const f32x16 Eo = t > 0 ? load_cl(a.E + (t - 1) * fs + ro, c, h) : zero16();
      f32x16 dIl, dEn, dEp, dcE;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float xe = (cev[r] - m1) * rs1;
        const float cn = bw1 * xe + bb1;
        const float w = kap * Iv[r] + gam;
        const float pe = cn * w;
        const float eh = act_f(pe, a.act);
        const float deg = GE[r] * (eh - Eo[r]);
        const float dpe = GE[r] * egv[r] * act_d(pe, a.act);
        const float dce = dpe * w;
        const float dw = dpe * cn;
        sm[1] += dw * Iv[r];
        sm[2] += dw;
        dIl[r] = dw * kap;
        dEn[r] = (1.f - egv[r]) * GE[r];
        dEp[r] = deg * egv[r] * (1.f - egv[r]);
        dcE[r] = dce;
        bs0 += dce;
        bs1 += dce * xe;
      }
      store_cl(a.dIl + ro, c, h, dIl);
      store_cl(a.dEn + ro, c, h, dEn);
      store_cl(a.dEp + ro, c, h, dEp);
      store_cl(a.dcE + ro, c, h, dcE);
    }
    shift_rows(acc);
  }
  sm[3] = bs1;   // d bn1.weight = sum dy * xhat
  sm[4] = bs0;   // d bn1.bias   = sum dy
  if (head) bn_bwd_partial(bs0, bs1, L.red, a.bnbacc + ((size_t)t * 2 + 1) * 64, lane, wave, tid);
  flush_small<9>(sm, slots, L.small, slab_b, lane, wave, tid);
  if (tail && head) {
    flush_gate(gaw, L.scr, slab_b + 0 * 1024, lane, wave, tid);
    flush_gate(gau, L.scr, slab_b + 1 * 1024, lane, wave, tid);
  }
}

// =========================================================================
// Backward B (frame t): BN1 backward -> dce (saved for the w_exc gradient),
//   dI_t = conv^T(dce, w_exc) + local + from frame t+1;
//   inhibition update backward (:166, :165, :162) -> i_w/i_u, alpha, mu,
//   dc_i (-> BN0 bwd partials), dx_t partial, dI_{t-1};
//   exc gate backward (:171) -> e_w/e_u grads, dI_{t-1}, dgE partial.
// =========================================================================
template <class S>
__global__ __launch_bounds__(NT, 1) void k_bwd_b(CellArgs<S> a) {
  using F = typename Tr<S>::frag;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const Lds L = carve<S>(smem);
  S* tile = (S*)L.tile;
  const int tid = threadIdx.x, lane = tid & 63, c = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int b = blockIdx.x, t = a.t, T = a.T, B = a.B;
  float* wscr = L.scr + wave * 1024;
  const size_t fs = fr_off(1, B), cb = clip_off(b);
  float* slab_b = a.slab + (size_t)b * SLAB;

  stage_x(a.x, L.xs, b, t, T, tid);
  bn_bwd_finalize(a.bnbacc + ((size_t)t * 2 + 1) * 64, B, L.stat, tid);
  tile_zero<S>(tile, tid);
  __syncthreads();

  const float* bs = a.bnstat + (size_t)t * 128;
  {
    const float m1 = bs[64 + c], rs1 = bs[96 + c], bw1 = a.bnw1[c];
    const float md = L.stat[c], mdx = L.stat[32 + c];
    for (int i = 0; i < RPW; ++i) {
      const int y = wave * RPW + i;
      const size_t ro = cb + (size_t)y * IMG * C;
      const f32x16 dcv = load_cl(a.dcE + ro, c, h);
      const f32x16 cev = load_cl(a.ce + t * fs + ro, c, h);
      f32x16 v;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float xh = (cev[r] - m1) * rs1;
        v[r] = rs1 * bw1 * (dcv[r] - md - xh * mdx);
      }
      store_cl(a.dce_s + t * fs + ro, c, h, v);
    }
  }
  f32x16 acc[RPW];
#pragma unroll
  for (int i = 0; i < RPW; ++i) acc[i] = zero16();
  conv_run<S>(acc, a.dce_s + t * fs + cb, a.wt_exc, tile, a.K, wave * RPW, tid, lane);

  const Stem st{a.wpre[c * 3 + 0], a.wpre[c * 3 + 1], a.wpre[c * 3 + 2], a.bpre[c]};
  const float al = a.alpha[c], mu = a.mu[c], bw0 = a.bnw0[c], bb0 = a.bnb0[c];
  const float m0 = bs[c], rs0 = bs[32 + c];
  const float bi = a.gb[2][c] + a.gb[3][c];
  float sm[7] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int slots[7] = {SM_ALPHA, SM_MU, SM_GBI, SM_GBE, SM_BN0W, SM_BN0B, SM_GBA};
  f32x16 giw = zero16(), giu = zero16(), gew = zero16(), geu = zero16();
  float bs0 = 0.f, bs1 = 0.f;

  for (int i = 0; i < RPW; ++i) {
    const int y = wave * RPW + i;
    const size_t ro = cb + (size_t)y * IMG * C;
    f32x16 dIt = acc[0] + load_cl(a.dIl + ro, c, h);
    if (t < T - 1 && !a.no_inh) dIt += load_cl(a.GI + ro, c, h);
    const f32x16 dep = load_cl(a.dEp + ro, c, h);
    const f32x16 gEv = load_cl(a.gE + t * fs + ro, c, h);
    if (!a.no_inh) {
      const f32x16 Iv = t > 0 ? load_cl(a.I + (t - 1) * fs + ro, c, h) : zero16();
      const f32x16 civ = load_cl(a.ci + t * fs + ro, c, h);
      f32x16 z, xv;
      stem_cl(L.xs, y, h, st, a.act, z, xv);
      F pax[Tr<S>::KS], pai[Tr<S>::KS];
      cl_to_pa<S>(wscr, xv, lane, pax);
      cl_to_pa<S>(wscr, Iv, lane, pai);
      f32x16 g = zero16();
      g = gemm_pa<S>(pax, a.gf[2], g, lane);
      g = gemm_pa<S>(pai, a.gf[3], g, lane);
      f32x16 dIp, dip, dx, dci;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float xi = (civ[r] - m0) * rs0;
        const float cn = bw0 * xi + bb0;
        const float u = al * Iv[r] + mu;
        const float p = cn * u;
        const float q = xv[r] - act_f(p, a.act);
        const float ih = act_f(q, a.act);
        const float ig = sigm(g[r] + bi);
        const float dih = dIt[r] * ig;
        dip[r] = dIt[r] * (ih - Iv[r]) * ig * (1.f - ig);
        const float dq = dih * act_d(q, a.act);
        const float dp = -dq * act_d(p, a.act);
        const float du = dp * cn;
        dci[r] = dp * u;
        dx[r] = dq;
        dIp[r] = dIt[r] * (1.f - ig) + du * al;
        sm[0] += du * Iv[r];
        sm[1] += du;
        sm[2] += dip[r];
        bs0 += dci[r];
        bs1 += dci[r] * xi;
      }
      giw = wgrad_cl<S>(dip, xv, giw);
      giu = wgrad_cl<S>(dip, Iv, giu);
      F pd[Tr<S>::KS];
      cl_to_pa<S>(wscr, dip, lane, pd);
      dx = gemm_pa<S>(pd, a.gt[2], dx, lane);
      dIp = gemm_pa<S>(pd, a.gt[3], dIp, lane);
      // exc gate: eg = sig(e_w I_{t-1} + e_u gE)
      gew = wgrad_cl<S>(dep, Iv, gew);
      geu = wgrad_cl<S>(dep, gEv, geu);
      F pe[Tr<S>::KS];
      cl_to_pa<S>(wscr, dep, lane, pe);
      dIp = gemm_pa<S>(pe, a.gt[4], dIp, lane);
      const f32x16 dg = gemm_pa<S>(pe, a.gt[5], zero16(), lane);
#pragma unroll
      for (int r = 0; r < 16; ++r) sm[3] += dep[r];
      store_cl(a.dcI + ro, c, h, dci);
      store_cl(a.GI + ro, c, h, dIp);
      store_cl(a.dxp + ro, c, h, dx);
      store_cl(a.dgEp + ro, c, h, dg);
    } else {
      // no_inh (:168): I_t = gE_t, eg = sig(e_w E_{t-1} + e_u gE_t)
      const f32x16 Ep = t > 0 ? load_cl(a.E + (t - 1) * fs + ro, c, h) : zero16();
      gew = wgrad_cl<S>(dep, Ep, gew);
      geu = wgrad_cl<S>(dep, gEv, geu);
      F pe[Tr<S>::KS];
      cl_to_pa<S>(wscr, dep, lane, pe);
      f32x16 dEn = load_cl(a.dEn + ro, c, h);
      dEn = gemm_pa<S>(pe, a.gt[4], dEn, lane);
      const f32x16 dg = gemm_pa<S>(pe, a.gt[5], dIt, lane);
#pragma unroll
      for (int r = 0; r < 16; ++r) sm[3] += dep[r];
      store_cl(a.dEn + ro, c, h, dEn);
      store_cl(a.dgEp + ro, c, h, dg);
      store_cl(a.dxp + ro, c, h, zero16());
    }
    shift_rows(acc);
  }
  sm[4] = bs1;
  sm[5] = bs0;
  if (!a.no_inh) bn_bwd_partial(bs0, bs1, L.red, a.bnbacc + ((size_t)t * 2 + 0) * 64, lane, wave, tid);
  flush_small<7>(sm, slots, L.small, slab_b, lane, wave, tid);
  if (!a.no_inh) {
    flush_gate(giw, L.scr, slab_b + 2 * 1024, lane, wave, tid);
    flush_gate(giu, L.scr, slab_b + 3 * 1024, lane, wave, tid);
  }
  flush_gate(gew, L.scr, slab_b + 4 * 1024, lane, wave, tid);
  flush_gate(geu, L.scr, slab_b + 5 * 1024, lane, wave, tid);
}

// =========================================================================
// k x k weight gradients over all (frame, clip) pairs:
//   dW[n][ci][tap] = sum_{t,b,p} D_t[b][p][n] X_t[b][p + tap][ci]
//   conv 0: (D, X) = (d ci_raw, gE)  -> w_inh;  conv 1: (d ce_raw, I_t) -> w_exc
// Each wave owns taps {w, w+4, ...} (<= 13 32x32 accumulator tiles); the
// D / X row bands are staged in LDS; per-workgroup partials go to wslab.
// =========================================================================
constexpr int WG_RB = 8;               // D rows per band
constexpr int WG_XR = WG_RB + 2 * PADMAX;
constexpr int WG_NACC = 13;
template <class S>
constexpr int wgrad_lds_bytes() {
  return (WG_XR * TILE * C + WG_RB * IMG * C) * (int)sizeof(S);
}

template <class S>
__device__ __forceinline__ int wx_off(int row, int col, int ch) {   // X band image
  if constexpr (sizeof(S) == 4) return (row * TILE + col) * C + ch;
  else return (row * TILE + col) * C + ((((ch >> 3) ^ ((col >> 2) & 3))) << 3) + (ch & 7);
}
template <class S>
__device__ __forceinline__ int wd_off(int row, int col, int ch) {   // D band image
  if constexpr (sizeof(S) == 4) return (row * IMG + col) * C + ch;
  else return (row * IMG + col) * C + ((((ch >> 3) ^ ((col >> 2) & 3))) << 3) + (ch & 7);
}

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
__device__ __forceinline__ bf16x4 tr_read(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(p));
}

template <class S>
__global__ __launch_bounds__(NT, 1) void k_wgrad(CellArgs<S> a, float* wslab, int nwg) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  S* xt = (S*)smem;
  S* dt = xt + WG_XR * TILE * C;
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = blockIdx.x, conv = blockIdx.y;
  const int K = a.K, KK = K * K, off = PADMAX - K / 2;
  const int B = a.B, T = a.T;
  const S* Xs = conv == 0 ? a.gE : a.I;
  const S* Ds = conv == 0 ? a.dci_s : a.dce_s;
  constexpr int CPB = 16 / (int)sizeof(S);
  constexpr int NCH = C / CPB;

  f32x16 acc[WG_NACC];
#pragma unroll
  for (int m = 0; m < WG_NACC; ++m) acc[m] = zero16();

  for (int f = g; f < B * T; f += nwg) {
    const int t = f / B, b = f % B;
    const S* xsrc = Xs + ((size_t)t * B + b) * NPIX * C;
    const S* dsrc = Ds + ((size_t)t * B + b) * NPIX * C;
    for (int y0 = 0; y0 < IMG; y0 += WG_RB) {
      __syncthreads();
      // X band: image rows y0-3 .. y0+RB+2, padded columns, zero outside
      for (int idx = tid; idx < WG_XR * TILE * NCH; idx += NT) {
        const int q = idx % NCH, pc = idx / NCH;
        const int col = pc % TILE, row = pc / TILE;
        const int iy = y0 + row - PADMAX, ix = col - PADMAX;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (iy >= 0 && iy < IMG && ix >= 0 && ix < IMG)
          v = *(const uint4*)(xsrc + (iy * IMG + ix) * C + q * CPB);
        *(uint4*)(xt + wx_off<S>(row, col, q * CPB)) = v;
      }
      for (int idx = tid; idx < WG_RB * IMG * NCH; idx += NT) {
        const int q = idx % NCH, pc = idx / NCH;
        const int col = pc % IMG, row = pc / IMG;
        *(uint4*)(dt + wd_off<S>(row, col, q * CPB)) =
            *(const uint4*)(dsrc + ((y0 + row) * IMG + col) * C + q * CPB);
      }
      __syncthreads();
      if constexpr (sizeof(S) == 4) {
        // f32: k-step = 2 pixels (x0 + h), lane (col = l&31) is ci for A, n for B
        const int ch = lane & 31;
        for (int yd = 0; yd < WG_RB; ++yd) {
          for (int x0 = 0; x0 < IMG; x0 += 2) {
            const float bv = dt[wd_off<S>(yd, x0 + h, ch)];
#pragma unroll
            for (int m = 0; m < WG_NACC; ++m) {
              const int tap = wave + 4 * m;
              if (tap < KK) {
                const int kh = tap / K, kw = tap - kh * K;
                const float av = xt[wx_off<S>(yd + kh + off, x0 + h + kw + off, ch)];
                acc[m] = Tr<float>::mma(av, bv, acc[m]);
              }
            }
          }
        }
      } else {
        // bf16: k-step = 16 pixels; fragments by ds_read_b64_tr_b16 from the
        // channels-last images (lane 4q+p' addresses pixel q, channels 4p'..4p'+3
        // of its 16-lane group's channel half).
        const int grp = lane >> 4, m16 = lane & 15, q = m16 >> 2, pp = m16 & 3;
        const int chb = 16 * (grp & 1) + 4 * pp;
        const int hh = grp >> 1;
        for (int yd = 0; yd < WG_RB; ++yd) {
          for (int x0 = 0; x0 < IMG; x0 += 16) {
            const int dc0 = x0 + 8 * hh + q;
            const bf16x4 b0 = tr_read((const bf16_t*)dt + wd_off<S>(yd, dc0, chb));
            const bf16x4 b1 = tr_read((const bf16_t*)dt + wd_off<S>(yd, dc0 + 4, chb));
            bf16x8 bv;
#pragma unroll
            for (int j = 0; j < 4; ++j) { bv[j] = b0[j]; bv[4 + j] = b1[j]; }
#pragma unroll
            for (int m = 0; m < WG_NACC; ++m) {
              const int tap = wave + 4 * m;
              if (tap < KK) {
                const int kh = tap / K, kw = tap - kh * K;
                const int tr = yd + kh + off, tc = dc0 + kw + off;
                const bf16x4 a0 = tr_read((const bf16_t*)xt + wx_off<S>(tr, tc, chb));
                const bf16x4 a1 = tr_read((const bf16_t*)xt + wx_off<S>(tr, tc + 4, chb));
                bf16x8 av;
#pragma unroll
                for (int j = 0; j < 4; ++j) { av[j] = a0[j]; av[4 + j] = a1[j]; }
                acc[m] = Tr<bf16_t>::mma(av, bv, acc[m]);
              }
            }
          }
        }
      }
    }
  }
  // acc[m]: rows ci = cl_x(r,h), cols n = lane&31
  float* dst = wslab + ((size_t)conv * nwg + g) * MAXTAP * 1024;
  const int n = lane & 31;
#pragma unroll
  for (int m = 0; m < WG_NACC; ++m) {
    const int tap = wave + 4 * m;
    if (tap < KK) {
#pragma unroll
      for (int r = 0; r < 16; ++r) dst[tap * 1024 + n * 32 + cl_x(r, h)] = acc[m][r];
    }
  }
}

// =========================================================================
// Parameter preparation: fp32 torch weights -> MFMA B-operand fragments.
//   conv fwd  wf[tap][ks][lane][j] = W[n=l&31][frag_chan(ks,h,j)][tap]
//   conv^T    wt[tap][ks][lane][j] = W[frag_chan(ks,h,j)][n=l&31][K*K-1-tap]
//   1x1 fwd   gf[ks][lane][j] = G[l&31][frag_chan]; bwd gt = G[frag_chan][l&31]
// =========================================================================
template <class S>
struct PrepArgs {
  int K;
  const float *w_inh, *w_exc;
  const float* g[6];
  S *wf_inh, *wf_exc, *wt_inh, *wt_exc;
  S* gf[6];
  S* gt[6];
};

template <class S>
__global__ void k_prep(PrepArgs<S> p) {
  using TT = Tr<S>;
  const int K = p.K, KK = K * K;
  const int nconv = KK * TT::KS * 64 * TT::EPL;   // == C*C*K*K
  const int ngate = TT::KS * 64 * TT::EPL;        // == C*C
  const int total = 4 * nconv + 12 * ngate;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    if (e < 4 * nconv) {
      const int which = e / nconv, r = e % nconv;
      const int j = r % TT::EPL, l = (r / TT::EPL) % 64, ks = (r / (TT::EPL * 64)) % TT::KS;
      const int tap = r / (TT::EPL * 64 * TT::KS);
      const int n = l & 31, h = l >> 5, kc = frag_chan<S>(ks, h, j);
      const float* W = (which == 0 || which == 2) ? p.w_inh : p.w_exc;
      S* dst = which == 0 ? p.wf_inh : which == 1 ? p.wf_exc : which == 2 ? p.wt_inh : p.wt_exc;
      if (W) {
        const float v = which < 2 ? W[(n * C + kc) * KK + tap] : W[(kc * C + n) * KK + (KK - 1 - tap)];
        dst[r] = (S)v;
      }
    } else {
      const int e2 = e - 4 * nconv;
      const int gi = e2 / ngate, r = e2 % ngate;
      const int gate = gi % 6, tr = gi / 6;
      const int j = r % TT::EPL, l = (r / TT::EPL) % 64, ks = r / (TT::EPL * 64);
      const int n = l & 31, h = l >> 5, kc = frag_chan<S>(ks, h, j);
      const float* G = p.g[gate];
      const float v = tr == 0 ? G[n * C + kc] : G[kc * C + n];
      (tr == 0 ? p.gf[gate] : p.gt[gate])[r] = (S)v;
    }
  }
}

// ---------------------------------------------------------------- reductions
struct ReduceArgs {
  int B, K, nwg;
  const float* slab;    // [B][SLAB]
  const float* wslab;   // [2][nwg][49][1024]
  pt_cell_grads g;
};

__global__ void k_reduce(ReduceArgs r) {
  const int KK = r.K * r.K;
  const int n_small = SLAB;                  // slab entries
  const int n_w = 2 * KK * 1024;             // conv weights
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < n_small + n_w;
       e += gridDim.x * blockDim.x) {
    if (e < n_small) {
      float s = 0.f;
      for (int b = 0; b < r.B; ++b) s += r.slab[(size_t)b * SLAB + e];
      if (e < SLAB_G) {
        const int gate = e / 1024;
        if (r.g.gate_w[gate]) r.g.gate_w[gate][e % 1024] = s;
      } else {
        const int slot = (e - SLAB_G) / 32, c = (e - SLAB_G) % 32;
        switch (slot) {
          case SM_ALPHA: if (r.g.alpha) r.g.alpha[c] = s; break;
          case SM_MU: if (r.g.mu) r.g.mu[c] = s; break;
          case SM_GAMMA: if (r.g.gamma) r.g.gamma[c] = s; break;
          case SM_KAPPA: if (r.g.kappa) r.g.kappa[c] = s; break;
          case SM_BN0W: if (r.g.bn_w[0]) r.g.bn_w[0][c] = s; break;
          case SM_BN0B: if (r.g.bn_b[0]) r.g.bn_b[0][c] = s; break;
          case SM_BN1W: if (r.g.bn_w[1]) r.g.bn_w[1][c] = s; break;
          case SM_BN1B: if (r.g.bn_b[1]) r.g.bn_b[1][c] = s; break;
          case SM_GBA:
            if (r.g.gate_b[0]) r.g.gate_b[0][c] = s;
            if (r.g.gate_b[1]) r.g.gate_b[1][c] = s;
            break;
          case SM_GBI:
            if (r.g.gate_b[2]) r.g.gate_b[2][c] = s;
            if (r.g.gate_b[3]) r.g.gate_b[3][c] = s;
            break;
          case SM_GBE:
            if (r.g.gate_b[4]) r.g.gate_b[4][c] = s;
            if (r.g.gate_b[5]) r.g.gate_b[5][c] = s;
            break;
          case SM_PW0: if (r.g.preproc_w) r.g.preproc_w[c * 3 + 0] = s; break;
          case SM_PW1: if (r.g.preproc_w) r.g.preproc_w[c * 3 + 1] = s; break;
          case SM_PW2: if (r.g.preproc_w) r.g.preproc_w[c * 3 + 2] = s; break;
          case SM_PB: if (r.g.preproc_b) r.g.preproc_b[c] = s; break;
          default: break;
        }
      }
    } else {
      const int e2 = e - n_small;
      const int conv = e2 / (KK * 1024), rem = e2 % (KK * 1024);
      const int tap = rem / 1024, nc = rem % 1024, n = nc / 32, ci = nc % 32;
      float s = 0.f;
      for (int gw = 0; gw < r.nwg; ++gw) s += r.wslab[(((size_t)conv * r.nwg + gw) * MAXTAP + tap) * 1024 + nc];
      float* W = conv == 0 ? r.g.w_inh : r.g.w_exc;
      if (W) W[(n * C + ci) * KK + tap] = s;
    }
  }
}

// channels-last [B][32][32][C] (S)  <->  NCHW fp32
template <class S>
__global__ void k_to_nchw(const S* __restrict__ src, float* __restrict__ dst, int B, int T, int t) {
  // dst [B][T][C][NPIX] (T=1,t=0 for a single frame)
  const int n = B * NPIX * C;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
    const int c = e % C, pix = (e / C) % NPIX, b = e / (C * NPIX);
    dst[(((size_t)b * T + t) * C + c) * NPIX + pix] = ldf(src + e);
  }
}
__global__ void k_from_nchw(const float* __restrict__ src, float* __restrict__ dst, int B) {
  const int n = B * NPIX * C;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
    const int c = e % C, pix = (e / C) % NPIX, b = e / (C * NPIX);
    dst[e] = src[((size_t)b * C + c) * NPIX + pix];
  }
}

}  // namespace ptc

// =========================================================================
//                                  host side
// =========================================================================
using namespace ptc;

static thread_local char g_err[512];
static int fail(int code, const char* fmt, const char* a = "", long v = 0) {
  snprintf(g_err, sizeof(g_err), fmt, a, v);
  return code;
}

namespace {

// ---- optional per-kind kernel timing (process-wide, mutex-guarded; autograd
// launches the backward from its own device thread, so this cannot be
// thread-local; see pt_cell.h) ----
struct Timing {
  std::mutex mu;
  uint32_t mask = 0;
  std::vector<hipEvent_t> pool;        // reusable events
  size_t used = 0;
  std::vector<int> kind;               // per recorded pair
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;
};
Timing g_tm;

hipEvent_t tm_event() {
  if (g_tm.used == g_tm.pool.size()) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    g_tm.pool.push_back(e);
  }
  return g_tm.pool[g_tm.used++];
}

// Launch wrapper: brackets the launch with events when its kind is enabled.
template <typename F>
void timed(int kind, hipStream_t st, F&& launch) {
  if (!(__atomic_load_n(&g_tm.mask, __ATOMIC_RELAXED) & (1u << kind))) { launch(); return; }
  std::lock_guard<std::mutex> lk(g_tm.mu);
  hipEvent_t a = tm_event(), b = tm_event();
  if (!a || !b) { launch(); return; }
  (void)hipEventRecord(a, st);
  launch();
  (void)hipEventRecord(b, st);
  g_tm.kind.push_back(kind);
  g_tm.ev.emplace_back(a, b);
}

constexpr size_t ALIGN = 256;
inline size_t al(size_t x) { return (x + ALIGN - 1) / ALIGN * ALIGN; }

struct Plan {
  int B, T, K, dt;
  size_t es;          // element size of S
  size_t frame;       // elements per frame tensor (B*NPIX*C)
  // saved offsets
  size_t o_E, o_I, o_gE, o_ci, o_ce, o_eg, o_bnstat, o_wf[4], o_g[12], saved;
  // workspace offsets
  size_t o_bnacc, o_bnbacc, o_tr[9], o_dci, o_dce, o_slab, o_wslab, ws;
  int nwg;
};

int check(const pt_cell_desc* d) {
  if (!d) return fail(PT_ERR_ARG, "null descriptor%s%ld");
  if (d->channels != 32) return fail(PT_ERR_UNSUPPORTED, "channels must be 32 (got %s%ld)", "", d->channels);
  if (d->height != 32 || d->width != 32)
    return fail(PT_ERR_UNSUPPORTED, "only 32x32 frames are supported%s (H=%ld)", "", d->height);
  if (d->ksize < 1 || d->ksize > 7 || (d->ksize & 1) == 0)
    return fail(PT_ERR_UNSUPPORTED, "ksize must be odd and <= 7%s (got %ld)", "", d->ksize);
  if (d->batch < 1 || d->frames < 1) return fail(PT_ERR_ARG, "batch and frames must be >= 1%s%ld");
  if (d->act != PT_ACT_SOFTPLUS && d->act != PT_ACT_TANH) return fail(PT_ERR_ARG, "bad act%s%ld");
  if (d->dtype != PT_DTYPE_F32 && d->dtype != PT_DTYPE_BF16) return fail(PT_ERR_ARG, "bad dtype%s%ld");
  if (d->cell != PT_CELL_INT) return fail(PT_ERR_UNSUPPORTED, "only the InT cell is built in this version%s%ld");
  return 0;
}

Plan plan(const pt_cell_desc* d) {
  Plan p{};
  p.B = d->batch; p.T = d->frames; p.K = d->ksize; p.dt = d->dtype;
  p.es = d->dtype == PT_DTYPE_BF16 ? 2 : 4;
  p.frame = (size_t)p.B * NPIX * C;
  const size_t fbytes = al(p.frame * p.T * p.es);
  size_t o = 0;
  p.o_E = o; o += fbytes;
  p.o_I = o; o += fbytes;
  p.o_gE = o; o += fbytes;
  p.o_ci = o; o += fbytes;
  p.o_ce = o; o += fbytes;
  p.o_eg = o; o += fbytes;
  p.o_bnstat = o; o += al((size_t)p.T * 128 * 4);
  for (int i = 0; i < 4; ++i) { p.o_wf[i] = o; o += al((size_t)C * C * MAXTAP * p.es); }
  for (int i = 0; i < 12; ++i) { p.o_g[i] = o; o += al((size_t)C * C * p.es); }
  p.saved = o;
  o = 0;
  p.o_bnacc = o; o += al((size_t)p.T * 2 * 96 * 8);
  p.o_bnbacc = o; o += al((size_t)p.T * 2 * 64 * 8);
  for (int i = 0; i < 9; ++i) { p.o_tr[i] = o; o += al(p.frame * 4); }
  p.o_dci = o; o += fbytes;
  p.o_dce = o; o += fbytes;
  p.o_slab = o; o += al((size_t)p.B * SLAB * 4);
  p.nwg = p.B * p.T < 256 ? p.B * p.T : 256;
  p.o_wslab = o; o += al((size_t)2 * p.nwg * MAXTAP * 1024 * 4);
  p.ws = o;
  return p;
}

template <class S>
void fill_args(CellArgs<S>& a, const pt_cell_desc* d, const Plan& p, const float* x,
               const pt_cell_params* pr, char* saved, char* ws) {
  using F = typename Tr<S>::frag;
  memset(&a, 0, sizeof(a));
  a.B = p.B; a.T = p.T; a.K = p.K; a.act = d->act; a.no_inh = d->no_inh; a.eps = d->eps;
  a.x = x;
  a.wpre = pr->preproc_w; a.bpre = pr->preproc_b;
  a.alpha = pr->alpha; a.mu = pr->mu; a.gamma = pr->gamma; a.kappa = pr->kappa;
  a.bnw0 = pr->bn_w[0]; a.bnb0 = pr->bn_b[0]; a.bnw1 = pr->bn_w[1]; a.bnb1 = pr->bn_b[1];
  for (int i = 0; i < 6; ++i) a.gb[i] = pr->gate_b[i];
  a.wf_inh = (const F*)(saved + p.o_wf[0]); a.wf_exc = (const F*)(saved + p.o_wf[1]);
  a.wt_inh = (const F*)(saved + p.o_wf[2]); a.wt_exc = (const F*)(saved + p.o_wf[3]);
  for (int i = 0; i < 6; ++i) {
    a.gf[i] = (const F*)(saved + p.o_g[i]);
    a.gt[i] = (const F*)(saved + p.o_g[6 + i]);
  }
  a.E = (S*)(saved + p.o_E); a.I = (S*)(saved + p.o_I); a.gE = (S*)(saved + p.o_gE);
  a.ci = (S*)(saved + p.o_ci); a.ce = (S*)(saved + p.o_ce); a.eg = (S*)(saved + p.o_eg);
  a.bnstat = (float*)(saved + p.o_bnstat);
  if (ws) {
    a.bnacc = (double*)(ws + p.o_bnacc);
    a.bnbacc = (double*)(ws + p.o_bnbacc);
    float** tr[9] = {&a.dEn, &a.dcE, &a.dIl, &a.dEp, &a.dcI, &a.GI, &a.dgEp, &a.dxp, nullptr};
    for (int i = 0; i < 8; ++i) *tr[i] = (float*)(ws + p.o_tr[i]);
    a.GEfin = (const float*)(ws + p.o_tr[8]);
    a.dci_s = (S*)(ws + p.o_dci); a.dce_s = (S*)(ws + p.o_dce);
    a.slab = (float*)(ws + p.o_slab);
  }
}

#define HIPCHK(expr)                                                              \
  do {                                                                            \
    hipError_t e_ = (expr);                                                       \
    if (e_ != hipSuccess) return fail(PT_ERR_HIP, "HIP error %s at line %ld", hipGetErrorString(e_), __LINE__); \
  } while (0)

template <class S>
int set_lds_attrs() {
  static thread_local bool done = false;   // per host thread; cheap either way
  if (done) return 0;
  HIPCHK(hipFuncSetAttribute((const void*)k_fwd_a<S>, hipFuncAttributeMaxDynamicSharedMemorySize, cell_lds_bytes<S>()));
  HIPCHK(hipFuncSetAttribute((const void*)k_fwd_b<S>, hipFuncAttributeMaxDynamicSharedMemorySize, cell_lds_bytes<S>()));
  HIPCHK(hipFuncSetAttribute((const void*)k_bwd_a<S>, hipFuncAttributeMaxDynamicSharedMemorySize, cell_lds_bytes<S>()));
  HIPCHK(hipFuncSetAttribute((const void*)k_bwd_b<S>, hipFuncAttributeMaxDynamicSharedMemorySize, cell_lds_bytes<S>()));
  HIPCHK(hipFuncSetAttribute((const void*)k_wgrad<S>, hipFuncAttributeMaxDynamicSharedMemorySize, wgrad_lds_bytes<S>()));
  done = true;
  return 0;
}

template <class S>
int run_forward(const pt_cell_desc* d, const float* x, const pt_cell_params* pr, void* saved,
                void* ws, float* e_last, float* gates, hipStream_t st) {
  const Plan p = plan(d);
  if (int rc = set_lds_attrs<S>()) return rc;
  CellArgs<S> a;
  fill_args<S>(a, d, p, x, pr, (char*)saved, (char*)ws);
  a.gates = gates;
  PrepArgs<S> pa{};
  pa.K = p.K; pa.w_inh = d->no_inh ? nullptr : pr->w_inh; pa.w_exc = pr->w_exc;
  for (int i = 0; i < 6; ++i) {
    pa.g[i] = pr->gate_w[i];
    pa.gf[i] = (S*)((char*)saved + p.o_g[i]);
    pa.gt[i] = (S*)((char*)saved + p.o_g[6 + i]);
  }
  pa.wf_inh = (S*)((char*)saved + p.o_wf[0]); pa.wf_exc = (S*)((char*)saved + p.o_wf[1]);
  pa.wt_inh = (S*)((char*)saved + p.o_wf[2]); pa.wt_exc = (S*)((char*)saved + p.o_wf[3]);
  HIPCHK(hipMemsetAsync((char*)ws + p.o_bnacc, 0, (size_t)p.T * 2 * 96 * 8, st));
  timed(PT_K_PREP, st, [&] { hipLaunchKernelGGL(k_prep<S>, dim3(256), dim3(256), 0, st, pa); });
  const size_t lds = cell_lds_bytes<S>();
  for (int t = 0; t <= p.T; ++t) {
    a.t = t;
    timed(PT_K_FWD_A, st, [&] { hipLaunchKernelGGL(k_fwd_a<S>, dim3(p.B), dim3(NT), lds, st, a); });
    if (t < p.T) timed(PT_K_FWD_B, st, [&] { hipLaunchKernelGGL(k_fwd_b<S>, dim3(p.B), dim3(NT), lds, st, a); });
  }
  if (e_last)
    hipLaunchKernelGGL(k_to_nchw<S>, dim3(256), dim3(256), 0, st,
                       (const S*)a.E + (size_t)(p.T - 1) * p.frame, e_last, p.B, 1, 0);
  HIPCHK(hipGetLastError());
  return 0;
}

template <class S>
int run_backward(const pt_cell_desc* d, const float* x, const pt_cell_params* pr,
                 const void* saved, void* ws, const float* d_e_last, const pt_cell_grads* g,
                 hipStream_t st) {
  const Plan p = plan(d);
  if (int rc = set_lds_attrs<S>()) return rc;
  CellArgs<S> a;
  fill_args<S>(a, d, p, x, pr, (char*)saved, (char*)ws);
  HIPCHK(hipMemsetAsync((char*)ws + p.o_slab, 0, (size_t)p.B * SLAB * 4, st));
  HIPCHK(hipMemsetAsync((char*)ws + p.o_bnbacc, 0, (size_t)p.T * 2 * 64 * 8, st));
  hipLaunchKernelGGL(k_from_nchw, dim3(256), dim3(256), 0, st, d_e_last,
                     (float*)((char*)ws + p.o_tr[8]), p.B);
  const size_t lds = cell_lds_bytes<S>();
  a.t = p.T - 1;
  timed(PT_K_BWD_A, st, [&] { hipLaunchKernelGGL(k_bwd_a<S>, dim3(p.B), dim3(NT), lds, st, a); });
  for (int t = p.T - 1; t >= 0; --t) {
    a.t = t;
    timed(PT_K_BWD_B, st, [&] { hipLaunchKernelGGL(k_bwd_b<S>, dim3(p.B), dim3(NT), lds, st, a); });
    a.t = t - 1;
    timed(PT_K_BWD_A, st, [&] { hipLaunchKernelGGL(k_bwd_a<S>, dim3(p.B), dim3(NT), lds, st, a); });
  }
  float* wslab = (float*)((char*)ws + p.o_wslab);
  if (!d->no_inh) {
    timed(PT_K_WGRAD, st, [&] { hipLaunchKernelGGL(k_wgrad<S>, dim3(p.nwg, 2), dim3(NT), wgrad_lds_bytes<S>(), st, a, wslab, p.nwg); });
  } else {
    HIPCHK(hipMemsetAsync(wslab, 0, (size_t)p.nwg * MAXTAP * 1024 * 4, st));
    // conv 1 only (w_exc); conv 0 slab stays zero
    CellArgs<S> a2 = a;
    hipLaunchKernelGGL(k_wgrad<S>, dim3(p.nwg, 2), dim3(NT), wgrad_lds_bytes<S>(), st, a2, wslab, p.nwg);
  }
  ReduceArgs r;
  r.B = p.B; r.K = p.K; r.nwg = p.nwg;
  r.slab = (const float*)((char*)ws + p.o_slab);
  r.wslab = wslab;
  r.g = *g;
  if (d->no_inh) { r.g.w_inh = nullptr; r.g.alpha = nullptr; r.g.mu = nullptr;
                   r.g.bn_w[0] = nullptr; r.g.bn_b[0] = nullptr;
                   r.g.gate_w[2] = r.g.gate_w[3] = nullptr; r.g.gate_b[2] = r.g.gate_b[3] = nullptr; }
  timed(PT_K_REDUCE, st, [&] { hipLaunchKernelGGL(k_reduce, dim3(256), dim3(256), 0, st, r); });
  HIPCHK(hipGetLastError());
  return 0;
}

}  // namespace

extern "C" {

size_t pt_cell_saved_bytes(const pt_cell_desc* d) {
  if (check(d)) return 0;
  return plan(d).saved;
}
size_t pt_cell_workspace_bytes(const pt_cell_desc* d) {
  if (check(d)) return 0;
  return plan(d).ws;
}

int pt_cell_forward(const pt_cell_desc* d, const float* x, const pt_cell_params* p, void* saved,
                    void* ws, float* e_last, float* gates, pt_stream_t stream) {
  if (int rc = check(d)) return rc;
  if (!x || !p || !saved || !ws) return fail(PT_ERR_ARG, "null pointer argument%s%ld");
  if (d->dtype == PT_DTYPE_BF16)
    return run_forward<bf16_t>(d, x, p, saved, ws, e_last, gates, (hipStream_t)stream);
  return run_forward<float>(d, x, p, saved, ws, e_last, gates, (hipStream_t)stream);
}

int pt_cell_export_exc(const pt_cell_desc* d, const void* saved, float* e_seq, pt_stream_t stream) {
  if (int rc = check(d)) return rc;
  if (!saved || !e_seq) return fail(PT_ERR_ARG, "null pointer argument%s%ld");
  const Plan p = plan(d);
  for (int t = 0; t < p.T; ++t) {
    if (d->dtype == PT_DTYPE_BF16)
      hipLaunchKernelGGL(k_to_nchw<bf16_t>, dim3(256), dim3(256), 0, (hipStream_t)stream,
                         (const bf16_t*)((const char*)saved + p.o_E) + (size_t)t * p.frame, e_seq, p.B, p.T, t);
    else
      hipLaunchKernelGGL(k_to_nchw<float>, dim3(256), dim3(256), 0, (hipStream_t)stream,
                         (const float*)((const char*)saved + p.o_E) + (size_t)t * p.frame, e_seq, p.B, p.T, t);
  }
  HIPCHK(hipGetLastError());
  return 0;
}

int pt_cell_backward(const pt_cell_desc* d, const float* x, const pt_cell_params* p,
                     const void* saved, void* ws, const float* d_e_last, const pt_cell_grads* g,
                     pt_stream_t stream) {
  if (int rc = check(d)) return rc;
  if (!x || !p || !saved || !ws || !d_e_last || !g) return fail(PT_ERR_ARG, "null pointer argument%s%ld");
  if (d->dtype == PT_DTYPE_BF16)
    return run_backward<bf16_t>(d, x, p, saved, ws, d_e_last, g, (hipStream_t)stream);
  return run_backward<float>(d, x, p, saved, ws, d_e_last, g, (hipStream_t)stream);
}

int pt_cell_timing_enable(uint32_t kind_mask) {
  __atomic_store_n(&g_tm.mask, kind_mask, __ATOMIC_RELAXED);
  return 0;
}

int pt_cell_timing_read(int kind, double* total_ms, int64_t* launches) {
  if (!total_ms || !launches) return fail(PT_ERR_ARG, "null pointer argument%s%ld");
  std::lock_guard<std::mutex> lk(g_tm.mu);
  double tot = 0.0;
  int64_t n = 0;
  for (size_t i = 0; i < g_tm.ev.size(); ++i) {
    if (g_tm.kind[i] != kind) continue;
    HIPCHK(hipEventSynchronize(g_tm.ev[i].second));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, g_tm.ev[i].first, g_tm.ev[i].second));
    tot += ms;
    ++n;
  }
  *total_ms = tot;
  *launches = n;
  return 0;
}

int pt_cell_timing_reset(void) {
  std::lock_guard<std::mutex> lk(g_tm.mu);
  for (auto& e : g_tm.ev) { (void)hipEventSynchronize(e.second); }
  g_tm.ev.clear();
  g_tm.kind.clear();
  g_tm.used = 0;
  return 0;
}

const char* pt_last_error(void) { return g_err; }
const char* pt_version(void) { return "pt_cell 0.1 gfx950"; }

}  // extern "C"
