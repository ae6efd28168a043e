// pt_cell.hip — InT recurrent cell, forward + BPTT backward, for MI355X (gfx950).
//
// Reference path replaced (paths relative to the reference repo):
//   stem + frame loop  models/InT.py:212-235   -> per frame: k_pw_fa, k_conv (inh),
//                                                 k_pw_fb, k_conv (exc)
//   rCell.forward      models/InT.py:145-179   -> split at the two BatchNorms
//   autograd BPTT      mainclean.py:204        -> per frame: k_conv (BN1 bwd + conv^T exc),
//                                                 k_pw_bb, k_conv (BN0 bwd + conv^T inh),
//                                                 k_pw_ba; then k_wgrad (7x7 weight
//                                                 grads), k_reduce
//
// Conv kernels: one workgroup owns one clip; the 32x32 image is exactly one
// 38x38 zero-halo LDS tile, so the k x k convolutions need no halo exchange.
// Point-wise kernels: several 8-wave workgroups per clip, one or two image rows
// per wave.  The only cross-clip coupling is BatchNorm's batch statistics
// (track_running_stats=False, models/InT.py:102): a kernel publishes per-clip
// partial sums (fp64 atomics), the next kernel finalises them (kernel boundary
// = grid-wide sync).  See DESIGN.md §3.
#include "pt_device.h"
#include "pt_pr.h"
#include "pt_graph.h"
#include "../../include/pt_cell.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <mutex>
#include <type_traits>
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
constexpr int NTRANS = 12;                       // backward transients incl. dAt, GEfin
// BatchNorm batch sums.  PT_BN_MODE selects the reduction (compile time):
//  3 as 2, but only the group's last member by index waits (for the
//    others' counts, bounded poll) and sums; the others count in with a
//    no-return atomic after their store's acknowledgement (bn_publish_finish).
//  2 (default) bitwise reproducible, no floating-point atomics: every producer
//    (forward: the conv workgroup of one clip / tile; backward: a point-wise
//    workgroup) stores its 64 partial sums in its own slot with write-through
//    (sc1) stores, its wave 0 drains them and takes an arrival ticket (one
//    relaxed agent-scope vector atomic; no release fence, so no L2 write-back);
//    the last producer to arrive in its group of bn_gsize() adds the group's
//    partials in slot order, reading them with sc1 loads (never a stale L1
//    line), and stores the group sum; a consumer adds the <= NGRP group sums in
//    group order.  Every sum has one fixed association, whatever the dispatch
//    order or XCD placement: runs and hipGraph replays agree bit for bit.
//  1 the same ticket with plain stores + an agent-scope release / acquire
//    fence pair (measured: the per-workgroup release, an L2 write-back, made
//    k_pw_bb 2x slower).
//  0 fp64 atomics into NGRP copies (order-dependent rounding).
#ifndef PT_BN_MODE
#define PT_BN_MODE 2
#endif
#ifndef PT_SLAB_DMA
#define PT_SLAB_DMA 1     // slab prefetch by LDS-DMA (0: through registers)
#endif
#ifndef PT_SLAB_WAIT
#define PT_SLAB_WAIT 0
#endif
#ifndef PT_WG_NOP
#define PT_WG_NOP 0
#endif
constexpr int NGRP = 16;
constexpr int BNB_WG_PER_CLIP = 8;     // backward producers per clip at most (PW_PARTS)
__host__ __device__ inline int bn_gsize(int nprod) { return (nprod + NGRP - 1) / NGRP; }
__host__ __device__ inline int bn_ngrp(int nprod) {
  if (PT_BN_MODE == 0) return NGRP;    // copies, all read (unused ones stay zero)
  const int g = bn_gsize(nprod);
  return (nprod + g - 1) / g;
}
struct BnSlot {       // one (frame, BatchNorm) reduction
  float* part;        // [nprod][64] per-producer partials
  double* grp;        // [NGRP][NV] group sums (NV: 96 forward, 64 backward)
  unsigned* cnt;      // [NGRP] arrival tickets, zeroed before every call
  int nprod;          // producers in the launch
  unsigned* done;     // persistent forward: groups summed so far (the grid wait's
                      // counter); the group sums then go out write-through
};

__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// 16-B agent-coherent (sc1) loads, as the 4-B relaxed agent-scope atomic load
// above is lowered (there is no 16-B atomic load): eight in flight, then one
// wait inside the same asm, so no result is read before it has landed.
__device__ __forceinline__ void ld16_sc1x8(f32x4 (&x)[8], const f32x4* const (&p)[8]) {
  asm volatile(
      "global_load_dwordx4 %0, %8, off sc1\n\t"
      "global_load_dwordx4 %1, %9, off sc1\n\t"
      "global_load_dwordx4 %2, %10, off sc1\n\t"
      "global_load_dwordx4 %3, %11, off sc1\n\t"
      "global_load_dwordx4 %4, %12, off sc1\n\t"
      "global_load_dwordx4 %5, %13, off sc1\n\t"
      "global_load_dwordx4 %6, %14, off sc1\n\t"
      "global_load_dwordx4 %7, %15, off sc1\n\t"
      "s_waitcnt vmcnt(0)"
      : "=&v"(x[0]), "=&v"(x[1]), "=&v"(x[2]), "=&v"(x[3]), "=&v"(x[4]), "=&v"(x[5]), "=&v"(x[6]), "=&v"(x[7])
      : "v"(p[0]), "v"(p[1]), "v"(p[2]), "v"(p[3]), "v"(p[4]), "v"(p[5]), "v"(p[6]), "v"(p[7])
      : "memory");
}
__device__ __forceinline__ f32x4 ld16_sc1(const f32x4* p) {
  f32x4 x;
  asm volatile("global_load_dwordx4 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=&v"(x) : "v"(p) : "memory");
  return x;
}

#ifndef PT_GS_4B
#define PT_GS_4B 0
#endif
// The last arriver of group g: sums of the group's partials in slot order, fp64.
// Thread (v = tid & 63, q = tid >> 6) adds members q, q + Q, ...; the Q
// quarter sums are then added in q order.  FWD: partial = (mean_b[32], M2_b[32])
// -> grp = (sum mean_b, sum mean_b^2, sum M2_b); else grp = sum of the 64 values.
// scr: NTH * (FWD ? 2 : 1) doubles of LDS.
template <int NTH, bool FWD>
__device__ void bn_group_sum_4b(const BnSlot& s, int g, int tid, double* scr) {
  constexpr int Q = NTH / 64;
  const int G = bn_gsize(s.nprod), m0 = g * G, m1 = min(s.nprod, m0 + G);
  const int v = tid & 63, q = tid >> 6;
  double a = 0.0, b = 0.0;
  // every load of this thread in flight at once (the tail of the launch waits
  // on this one workgroup), then added in member order
  // G / Q at B = 256: k_pw_bb 128 / 4, k_pw_ba 32 / 4, the convs 16 / 8
#ifndef PT_GS_PER
#define PT_GS_PER 0       // 32 (all loads in flight): k_pw_bb 69.7 -> 78.8 us; 8: 70.2
#endif
  constexpr int MAXPER = Q <= 4 ? PT_GS_PER : (PT_GS_PER < 4 ? PT_GS_PER : 4);
  float xv[MAXPER > 0 ? MAXPER : 1];
#pragma unroll
  for (int k = 0; k < MAXPER; ++k) {
    const int m = m0 + q + k * Q;
    xv[k] = 0.f;
    if (m < m1) {
      const float* pp = s.part + (size_t)m * 64 + v;
      xv[k] = PT_BN_MODE == 2 ? ld_sc1(pp) : *pp;
    }
  }
#pragma unroll
  for (int k = 0; k < MAXPER; ++k) {
    if (m0 + q + k * Q < m1) {
      const double x = (double)xv[k];
      a += x;
      b += x * x;
    }
  }
#pragma unroll 8
  for (int m = m0 + q + MAXPER * Q; m < m1; m += Q) {   // larger groups than planned for
    const float* pp = s.part + (size_t)m * 64 + v;
    const double x = (double)(PT_BN_MODE == 2 ? ld_sc1(pp) : *pp);
    a += x;
    b += x * x;
  }
  constexpr int W = FWD ? 2 : 1;
  scr[W * tid] = a;
  if (FWD) scr[W * tid + 1] = b;
  __syncthreads();
  if (tid < 64) {
    double sa = 0.0, sb = 0.0;
#pragma unroll
    for (int k = 0; k < Q; ++k) {
      sa += scr[W * (k * 64 + tid)];
      if (FWD) sb += scr[W * (k * 64 + tid) + 1];
    }
    double* o = s.grp + (size_t)g * (FWD ? 96 : 64);
    auto put = [&](int i, double v) {
      if (s.done) __hip_atomic_store(o + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else o[i] = v;
    };
    if (FWD) {
      if (tid < 32) { put(tid, sa); put(32 + tid, sb); }
      else put(32 + tid, sa);                          // sum M2_b at 64 + (tid - 32)
    } else {
      put(tid, sa);
    }
    if (s.done) {                   // the group sum is in L2: count it
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (tid == 0) __hip_atomic_fetch_add(s.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// The last arriver of group g: sums of the group's partials, fp64, in one
// fixed association.  Thread (v4 = tid & 15, q = tid >> 4) reads values
// 4 v4 .. 4 v4 + 3 of members q, q + NTH/16, ... as 16-B sc1 loads, all
// in flight at once (one round trip; the 4-byte form took four, at the tail of
// the launch); the 4 q of a wave are added by a fixed xor butterfly, the wave
// sums in wave order.  FWD: partial = (mean_b[32], M2_b[32]) -> grp = (sum
// mean_b, sum mean_b^2, sum M2_b); else grp = sum of the 64 values.
// scr: (NTH / 64) * (FWD ? 96 : 64) doubles of LDS.
template <int NTH, bool FWD>
__device__ void bn_group_sum(const BnSlot& s, int g, int tid, double* scr) {
  constexpr int QW = NTH / 16, NW = NTH / 64;
  const int G = bn_gsize(s.nprod), m0 = g * G, m1 = min(s.nprod, m0 + G);
  const int v4 = tid & 15, q = tid >> 4, wave = tid >> 6;
  double a[4] = {0.0, 0.0, 0.0, 0.0}, sq[4] = {0.0, 0.0, 0.0, 0.0};
  // G / QW at B = 256: k_pw_bb 128 / 16, k_pw_ba 32 / 16, the convs 16 / 32
  constexpr int MAXPER = 8;
  f32x4 xv[MAXPER];
  const f32x4* pp[MAXPER];
#pragma unroll
  for (int k = 0; k < MAXPER; ++k) {
    const int m = m0 + q + k * QW;
    const int mc = m < m1 ? m : m0;                  // unconditional loads, masked below
    pp[k] = (const f32x4*)(s.part + (size_t)mc * 64) + v4;
  }
  ld16_sc1x8(xv, pp);
  auto add = [&](const f32x4& x) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const double d = (double)x[j];
      a[j] += d;
      if (FWD) sq[j] += d * d;
    }
  };
#pragma unroll
  for (int k = 0; k < MAXPER; ++k)
    if (m0 + q + k * QW < m1) add(xv[k]);
#pragma unroll 1
  for (int m = m0 + q + MAXPER * QW; m < m1; m += QW)   // larger groups than planned for
    add(ld16_sc1((const f32x4*)(s.part + (size_t)m * 64) + v4));
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    a[j] += __shfl_xor(a[j], 16);
    a[j] += __shfl_xor(a[j], 32);
    if (FWD) { sq[j] += __shfl_xor(sq[j], 16); sq[j] += __shfl_xor(sq[j], 32); }
  }
  if ((tid & 63) < 16) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      scr[wave * 64 + 4 * v4 + j] = a[j];
      if (FWD && v4 < 8) scr[NW * 64 + wave * 32 + 4 * v4 + j] = sq[j];
    }
  }
  __syncthreads();
  if (tid < 64) {
    double sa = 0.0, sb = 0.0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      sa += scr[w * 64 + tid];
      if (FWD && tid < 32) sb += scr[NW * 64 + w * 32 + tid];
    }
    double* o = s.grp + (size_t)g * (FWD ? 96 : 64);
    auto put = [&](int i, double v) {
      if (s.done) __hip_atomic_store(o + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else o[i] = v;
    };
    if (FWD) {
      if (tid < 32) { put(tid, sa); put(32 + tid, sb); }
      else put(32 + tid, sa);                          // sum M2_b at 64 + (tid - 32)
    } else {
      put(tid, sa);
    }
    if (s.done) {                   // the group sum is in L2: count it
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (tid == 0) __hip_atomic_fetch_add(s.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Persistent forward: the calling WAVE waits until `target` group sums of a
// reduction are in (its BnSlot::done counter); no workgroup barrier (the
// caller's next one publishes what the wave then computes).  Lane 0 polls with
// coherent loads; the spin is bounded (a grid that is not fully resident
// would otherwise never return): past the bound it gives up and flags *err,
// the results are then garbage.
__device__ __forceinline__ void wave_wait(const unsigned* done, unsigned target, unsigned* err, int lane) {
  if (lane == 0) {
    unsigned it = 0;
    while (__hip_atomic_load(done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(2);
      if ((++it & 1023) == 0 &&       // ~0.1 s, or another workgroup already gave up
          (it > (1u << 21) || __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
        __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
}

// Producer side: this workgroup's 64 partial values (lanes tid < 64 -- wave 0
// -- hold value tid) into the reduction, in two calls: bn_publish_store puts
// the values out, bn_publish_finish completes the protocol (a caller may run
// other work between the two; all threads call both).  flag: an LDS word no
// other code touches until the caller's next barrier; scr: see bn_group_sum.
//  mode 3: every member but the group's LAST by index (normally the last
//    dispatched) waits for its store's acknowledgement and counts in with one
//    no-return atomic -- no reply to wait for; the last member polls the count
//    (bounded) and sums the group.  Same sums as mode 2.
//  mode 2: every member takes a ticket (returning atomic) and the last to
//    ARRIVE sums the group.
template <int NTH, bool FWD>
__device__ __forceinline__ void bn_publish_store(const BnSlot& s, int prod, float val, int tid) {
#if PT_BN_MODE >= 2
  if (tid < 64)
    __hip_atomic_store(s.part + (size_t)prod * 64 + tid, val, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);                  // write-through
#else
  (void)s; (void)prod; (void)val; (void)tid;
#endif
}
template <int NTH, bool FWD>
__device__ __forceinline__ void bn_publish_finish(const BnSlot& s, int prod, float val, int tid, int* flag,
                                                  double* scr) {
#if PT_BN_MODE == 0
  if (tid < 64) {
    double* o = s.grp + (size_t)(prod % NGRP) * (FWD ? 96 : 64);
    const double d = (double)val;
    if (FWD && tid < 32) { unsafeAtomicAdd(o + tid, d); unsafeAtomicAdd(o + 32 + tid, d * d); }
    else unsafeAtomicAdd(o + (FWD ? 32 : 0) + tid, d);
  }
  (void)flag; (void)scr;
#else
  const int G = bn_gsize(s.nprod), g = prod / G;
  const int nmem = min(G, s.nprod - g * G);
#if PT_BN_MODE == 3
  (void)val; (void)flag;
  if (prod != g * G + nmem - 1) {                 // a member: acknowledged, then counted
    if (tid < 64) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (tid == 0) __hip_atomic_fetch_add(s.cnt + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  if (tid < 64) {                                 // the group's last member
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (tid == 0)
      for (unsigned it = 0; it < (1u << 22); ++it) {   // ~0.3 s bound: never a hang
        if (__hip_atomic_load(s.cnt + g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= (unsigned)(nmem - 1))
          break;
        __builtin_amdgcn_s_sleep(2);
      }
  }
  __syncthreads();
  bn_group_sum<NTH, FWD>(s, g, tid, scr);
#else
  if (tid < 64) {
#if PT_BN_MODE == 2
#ifndef PT_BN_NOWAIT
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");              // this wave's payload is in L2
#endif
    if (tid == 0) {
      const unsigned old = __hip_atomic_fetch_add(s.cnt + g, 1u, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
      *flag = old == (unsigned)(nmem - 1);
    }
#else
    s.part[(size_t)prod * 64 + tid] = val;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned old = __hip_atomic_fetch_add(s.cnt + g, 1u, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
      const int last = old == (unsigned)(nmem - 1);
      if (last) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      *flag = last;
    }
#endif
  }
  __syncthreads();
  if (*flag) {
    if (PT_GS_4B) bn_group_sum_4b<NTH, FWD>(s, g, tid, scr);
    else bn_group_sum<NTH, FWD>(s, g, tid, scr);
  }
#endif
#endif
}
template <int NTH, bool FWD>
__device__ __forceinline__ void bn_publish(const BnSlot& s, int prod, float val, int tid, int* flag,
                                           double* scr) {
  bn_publish_store<NTH, FWD>(s, prod, val, tid);
  bn_publish_finish<NTH, FWD>(s, prod, val, tid, flag, scr);
}

// Diagnostic precision bits (PT_DIAG builds; the f32 cell then stores or uses
// a value as the bf16 cell would, tools/bf16_attrib.py): 2048 E, 4096 I,
// 8192 gE + eg, 524288 c_i / c_e (pre-BN conv outputs), 1048576 the conv and
// 1x1 weight fragments, 2097152 the backward transients, 4194304 the 1x1 gate
// operands.
#define RND_G(a) (sizeof(S) == 4 && (PT_ABL((a).ablate) & 4194304))
#define RND_T(a) (sizeof(S) == 4 && (PT_ABL((a).ablate) & 2097152))
#define RND_C(a) (sizeof(S) == 4 && (PT_ABL((a).ablate) & 524288))
__device__ __forceinline__ f32x16 rb16(bool on, f32x16 v) {
  if (on)
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = rbf(true, v[r]);
  return v;
}

// ----------------------------------------------------------------- arguments
template <class S>
struct CellArgs {
  using F = typename Tr<S>::frag;
  int B, T, K, act, no_inh;
  int Cu;         // the caller's channel count (<= 32; the kernels run 32, padded, see k_pad_params)
  int hgru;       // hConvGRUCell: the gated inhibition is the attention map (ffhgru_hierarchy.py:147)
  float eps;
  int t;
  int ntx, nty;   // frames of (32 nty) x (32 ntx) px as nty x ntx tiles of 32x32 ("virtual
                  // clips": B counts tiles, B = clips * ntx * nty); 1 x 1 at 32x32
  unsigned long long* trace;   // diagnostics (pt_cell_trace): per-workgroup phase stamps of frame trace_t
  int trace_t;
  int ablate;     // timing experiments only (env PT_CELL_ABLATE): 1 skip conv MFMAs,
                  // 256 skip the conv epilogue, 512 return at entry (launch floor),
                  // 2 skip tile fill, 4 skip point-wise row loops, 8 skip BN fp64
                  // atomics, 16 skip the 1x1 weight-gradient LDS reductions,
                  // 32 skip slab flush, 16384 skip the conv weight-slice staging,
                  // 32768 skip only the conv's BN fp64 atomics, 65536 / 131072
                  // skip k_pw_fa's BN1 finalisation / x staging; precision diagnostics (f32 path only): 2048 round
                  // the stored E_t to bf16, 4096 the stored I_t, 8192 the stored gE_t, eg_t
  const void* x;                        // f32 [B][3][T][H][W] or u8 [B][T][H][W][3] (xu8)
  int xu8;
  const float *wpre, *bpre;             // [32][3], [32]
  const float *alpha, *mu, *gamma, *kappa;
  const float *bnw0, *bnb0, *bnw1, *bnb1;
  const float* gb[6];                   // gate biases
  const F *wf_inh, *wf_exc, *wt_inh, *wt_exc;   // conv fragments (fwd, transposed)
  const F* gf[6];                       // 1x1 fragments, forward
  const F* gt[6];                       // 1x1 fragments, transposed (backward)
  using F16 = typename T16<S>::frag;
  const F16* g16f[6];                   // the same as 16x16 B operands (k_pw_bb2, pt_pr.h)
  const F16* g16t[6];
  // Saved per frame [T][B][32][32][32].  E is f32 in both modes: stored in
  // bf16 it stagnates once the excitation settles (|eg (Ehat - E)| below half
  // a bf16 ulp of E), and the gate gradients, which measure that slow
  // movement, lost ~25 % of their norm at B=256, T=64 (attention-gate cosine
  // 0.97 vs the f32 cell; rounding I, gE, eg, c_i or c_e instead moved none of
  // them below 0.998: tools/bf16_diag2.py).
  float* E;
  // I is f32 in both modes too (r04): stored in bf16 it carried most of the bf16
  // cell's deviation from the f32 cell at the headline size with trained
  // parameters (logits 2.1e-3 of 2.2e-3, i-gate bias gradient cosine 0.990;
  // profiles/r04_bf16_attrib_trained.json).  Ic is I_t in the storage type, the
  // exc conv's input and k_wgrad's X operand (bf16: a copy written beside I;
  // f32: I itself).
  float* I;
  S* Ic;
  // bf16 cell (r05): E and I are stored as two 16-bit planes each instead of
  // f32 + a bf16 copy -- hi = the value rounded half-up to bf16 (Eh; Ih IS Ic,
  // the exc conv's input and k_wgrad's X operand) and lo = the low 16 bits of
  // (f32 bits - hi << 16), so hi + lo restores the f32 value EXACTLY (ldE /
  // ldI) while a reader that only needs the bf16 value reads half the bytes
  // (ldEh / ldIh).  f32 cell: E and I above, these null.
  S* Eh;
  uint16_t *El, *Il;
  S *gE, *ci, *ce, *eg;
  S* at;                                // hGRU only: attention map per frame (the gated inhibition)
  float* bnstat;                        // [T][4][32] mean0, rstd0, mean1, rstd1
  // BatchNorm reductions (see BnSlot), slot (t, bn) = t * 2 + bn:
  float* bnf_part;                      // fwd [T][2][B][64] per-clip (mean_b, M2_b)
  double* bnf_grp;                      // fwd [T][2][NGRP][96] sum mean_b, sum mean_b^2, sum M2_b
  unsigned* bnf_cnt;                    // fwd [T][2][NGRP] tickets
  float* gates;                         // [B][T][C][32][32] or null
  // backward transients, channels-last [B][32][32][32] in the storage type
  S *dEn, *dcE, *dIl, *dEp, *dcI, *GI, *dgEp, *dxp, *dgE, *dIt;
  S* dAt;                               // hGRU: d loss / d att_t through the gated inhibition
  const float* GEfin;                   // dE of the last frame (channels-last)
  S *dci_s, *dce_s;                     // [T][B][32][32][32] conv-output grads (for k_wgrad)
  float* bnb_part;                      // bwd [T][2][PW_PARTS B][64] per-workgroup (sum dy, sum dy*xhat)
  double* bnb_grp;                      // bwd [T][2][NGRP][64]
  unsigned* bnb_cnt;                    // bwd [T][2][NGRP]
  // SyncBN (pt_cell_dist): the batch totals all-reduced over bn_world replicas,
  // fwd [T][2][96] then bwd [T][2][64]; null = per-replica statistics
  const double* bnsync;
  int bn_world;                         // replicas sharing the statistics (1 = per replica)
  float* slab;                          // [B][PW_PARTS][SLAB]
  int conv_done;                        // k_pw_ba: dgE holds conv^T(w_inh) + dgEp
  int xmap;                             // XCD-affine workgroup order (wg_split)
  // fused forward on tiled frames (xb_exchange): each tile's 348 border pixels
  // of its conv input [B][348][32], the per-segment flags [2][B] (t + 1 once
  // published; zeroed per call) and the give-up word
  S* xch;
  unsigned* xflag;
  unsigned* xerr;
};

// Workgroup j of a launch with nper workgroups per clip -> (clip b, part).
// xmap (default, PT_XCD_MAP != 0): b = j % B, part = j / B, so that every
// kernel of a step places clip b on the same XCD (workgroups go to XCDs
// round-robin, j % 8; B a multiple of 8) and a clip's tensors written by one
// launch are read by the next one from the same XCD's L2; else b = j / nper.
__device__ __forceinline__ void wg_split(int j, int nper, int B, int xmap, int& b, int& part) {
  if (xmap) { b = j % B; part = j / B; }
  else { b = j / nper; part = j % nper; }
}

// Phase stamp (diagnostics, pt_cell_trace): thread 0 of every
// (gridDim.x / TRACE_WG)-th workgroup of the traced frame writes the 100 MHz
// real-time counter into slot `slot` (< 32) of its record
// trace[kind][blockIdx.x / stride][32]; the entry stamp (slot 0) also stores
// where the workgroup runs (slot 7: XCC_ID << 32 | HW_ID: SE, SH, CU, SIMD,
// wave slot).  PT_TRW: lane 0 of EVERY wave stamps slot base + wave (r06:
// per-wave row ends in slots 8-15, per-wave conv ends in 16-23).  Off (a null pointer) in every normal run.
constexpr int TRACE_WG = 2048, TRACE_SLOTS = 32;
#if PT_DIAG
__device__ __forceinline__ unsigned long long tr_hwid() {
  unsigned id, xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(id));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  return ((unsigned long long)(xcc & 0xf) << 32) | id | (1ull << 40);
}
#define PT_TR_IDX(a, kind, slot)                                                               \
  (((size_t)(kind) * TRACE_WG + blockIdx.x / (gridDim.x > TRACE_WG ? gridDim.x / TRACE_WG : 1)) * TRACE_SLOTS + (slot))
#define PT_TR_ON(a)                                                                            \
  ((a).trace && (a).t == (a).trace_t && blockIdx.x % (gridDim.x > TRACE_WG ? gridDim.x / TRACE_WG : 1) == 0 && \
   blockIdx.x / (gridDim.x > TRACE_WG ? gridDim.x / TRACE_WG : 1) < TRACE_WG)
#define PT_TR(a, kind, slot) PT_TRT(a, kind, slot, 0)
#define PT_TRT(a, kind, slot, th)                                                              \
  do {                                                                                         \
    if (PT_TR_ON(a) && threadIdx.x == (th)) {                                                  \
      (a).trace[PT_TR_IDX(a, kind, slot)] = __builtin_amdgcn_s_memrealtime();                  \
      if ((slot) == 0) (a).trace[PT_TR_IDX(a, kind, 7)] = tr_hwid();                           \
    }                                                                                          \
  } while (0)
#define PT_TRW(a, kind, base)                                                                  \
  do {                                                                                         \
    if (PT_TR_ON(a) && (threadIdx.x & 63) == 0)                                                \
      (a).trace[PT_TR_IDX(a, kind, (base) + (threadIdx.x >> 6))] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define PT_TR(a, kind, slot) do { } while (0)
#define PT_TRT(a, kind, slot, th) do { } while (0)
#define PT_TRW(a, kind, base) do { } while (0)
#endif
__device__ __forceinline__ size_t fr_off(int t, int B) { return (size_t)t * B * NPIX * C; }

// (frame t, BatchNorm bn) reduction slots; nprod of the backward ones: the
// launch's workgroups (k_pw_bb -> bn 0, k_pw_ba -> bn 1)
template <class S>
__host__ __device__ inline BnSlot bnf_slot(const CellArgs<S>& a, int t, int bn) {
  const size_t k = (size_t)t * 2 + bn;
  return {a.bnf_part + k * a.B * 64, a.bnf_grp + k * NGRP * 96, a.bnf_cnt + k * NGRP, a.B};
}
// what the forward consumers finalise: the group sums, or (SyncBN) the totals
template <class S>
__host__ __device__ inline const double* bnf_src(const CellArgs<S>& a, int t, int bn) {
  return a.bnsync ? a.bnsync + ((size_t)t * 2 + bn) * 96 : a.bnf_grp + ((size_t)t * 2 + bn) * NGRP * 96;
}
template <class S>
__host__ __device__ inline int bnf_nsrc(const CellArgs<S>& a) { return a.bnsync ? 1 : bn_ngrp(a.B); }
template <class S>
__host__ __device__ inline BnSlot bnb_slot(const CellArgs<S>& a, int t, int bn, int nprod) {
  const size_t k = (size_t)t * 2 + bn;
  return {a.bnb_part + k * (size_t)a.B * BNB_WG_PER_CLIP * 64, a.bnb_grp + k * NGRP * 64, a.bnb_cnt + k * NGRP,
          nprod};
}
__device__ __forceinline__ size_t clip_off(int b) { return (size_t)b * NPIX * C; }

// ------------------------------------------------------ the f32 states E, I
// (CellArgs::Eh / El / Il).  Split: hi = (bits + 0x8000) >> 16 (rounded half
// up in magnitude), lo = bits - (hi << 16) as 16 bits, in [-0x8000, 0x7fff]:
// bits = (hi << 16) + sext(lo) exactly.  The bf16 MFMA operands taken from E
// and I in the forward are rounded the same way (op_round), so the hi plane
// the backward reads is the operand the forward used.
// NaN: the carry of the half-up add can leave a NaN's exponent
// (0x7fff8000 -> -0.0), so a NaN's hi is its truncated bits with the quiet bit
// forced (a NaN whose upper mantissa bits are zero would truncate to Inf) and
// its lo is 0: NaN stays NaN in both the operand and hi + lo (payload not
// kept); +-Inf and every finite value are unchanged (hi + lo exact).
__host__ __device__ __forceinline__ uint32_t split_hh(uint32_t b) {
  const uint32_t r = (b + 0x8000u) & 0xffff0000u, q = (b | 0x00400000u) & 0xffff0000u;
  return (b & 0x7fffffffu) > 0x7f800000u ? q : r;
}
__host__ __device__ __forceinline__ uint16_t split_lo(uint32_t b, uint32_t hh) {
  return (b & 0x7fffffffu) > 0x7f800000u ? (uint16_t)0 : (uint16_t)(b - hh);
}
__device__ __forceinline__ uint32_t split_hi(float v) { return split_hh(__float_as_uint(v)) >> 16; }
__device__ __forceinline__ float hi_f(float v) { return __uint_as_float(split_hi(v) << 16); }
template <class S>
__device__ __forceinline__ f32x16 op_round(const f32x16& v) {
  if constexpr (sizeof(S) == 4) {
    return v;
  } else {
    f32x16 o;
#pragma unroll
    for (int r = 0; r < 16; ++r) o[r] = hi_f(v[r]);
    return o;
  }
}
// CL row tile of a split state (4-B loads of the channel pair, as load_cl)
__device__ __forceinline__ f32x16 load_cl_split(const bf16_t* __restrict__ hi, const uint16_t* __restrict__ lo,
                                                int c, int h) {
  const uint32_t* wh = (const uint32_t*)(hi + (c & ~1));
  const uint32_t* wl = (const uint32_t*)(lo + (c & ~1));
  const uint32_t sel = bf16_sel(c);
  const int sh = (c & 1) ? 0 : 16;
  f32x16 v;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const uint32_t x = wh[cl_x(r, h) * (C / 2)], y = wl[cl_x(r, h) * (C / 2)];
    v[r] = __uint_as_float(__builtin_amdgcn_perm(x, x, sel) + (uint32_t)((int32_t)(y << sh) >> 16));
  }
  return v;
}
// stores the split and returns the hi plane's values (the bf16 operand value,
// so a caller that also needs it does not round a second time)
__device__ __forceinline__ f32x16 store_cl_split(bf16_t* __restrict__ hi, uint16_t* __restrict__ lo, int c, int h,
                                                 const f32x16& v) {
  uint16_t* hp = (uint16_t*)hi;
  f32x16 hv;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const uint32_t b = __float_as_uint(v[r]), hh = split_hh(b);
    hp[cl_x(r, h) * C + c] = (uint16_t)(hh >> 16);
    lo[cl_x(r, h) * C + c] = split_lo(b, hh);
    hv[r] = __uint_as_float(hh);
  }
  return hv;
}
// PR (pt_pr.h) half-row tile of a split state: the lane's channel pair is one
// dword per plane
__device__ __forceinline__ f32x8 pr_load_split(const bf16_t* __restrict__ hseg, const uint16_t* __restrict__ lseg,
                                               int lane) {
  const int n = lane & 15, g = lane >> 4;
  const uint32_t* wh = (const uint32_t*)hseg + (4 * g) * (C / 2) + n;
  const uint32_t* wl = (const uint32_t*)lseg + (4 * g) * (C / 2) + n;
  f32x8 v;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t x = wh[i * (C / 2)], y = wl[i * (C / 2)];
    v[i] = __uint_as_float((x << 16) + (uint32_t)((int32_t)(y << 16) >> 16));
    v[4 + i] = __uint_as_float((x & 0xffff0000u) + (uint32_t)((int32_t)y >> 16));
  }
  return v;
}
// E_t / I_t of row offset ro: full precision (ld*), the bf16 operand value
// (ld*h: the hi plane; the f32 cell reads its f32 array either way), stores
template <class S>
__device__ __forceinline__ f32x16 ldE(const CellArgs<S>& a, int t, size_t ro, int c, int h) {
  const size_t o = fr_off(t, a.B) + ro;
  if constexpr (sizeof(S) == 2) return load_cl_split(a.Eh + o, a.El + o, c, h);
  else return load_cl(a.E + o, c, h);
}
template <class S>
__device__ __forceinline__ f32x16 ldEh(const CellArgs<S>& a, int t, size_t ro, int c, int h) {
  const size_t o = fr_off(t, a.B) + ro;
  if constexpr (sizeof(S) == 2) return load_cl(a.Eh + o, c, h);
  else return load_cl(a.E + o, c, h);
}
template <class S>
__device__ __forceinline__ f32x16 ldI(const CellArgs<S>& a, int t, size_t ro, int c, int h) {
  const size_t o = fr_off(t, a.B) + ro;
  if constexpr (sizeof(S) == 2) return load_cl_split(a.Ic + o, a.Il + o, c, h);
  else return load_cl(a.I + o, c, h);
}
template <class S>
__device__ __forceinline__ f32x16 ldIh(const CellArgs<S>& a, int t, size_t ro, int c, int h) {
  const size_t o = fr_off(t, a.B) + ro;
  if constexpr (sizeof(S) == 2) return load_cl(a.Ic + o, c, h);
  else return load_cl(a.I + o, c, h);
}
// (both return op_round<S>(v): the value the bf16 operands take)
template <class S>
__device__ __forceinline__ f32x16 stE(const CellArgs<S>& a, int t, size_t ro, int c, int h, const f32x16& v) {
  const size_t o = fr_off(t, a.B) + ro;
  if constexpr (sizeof(S) == 2) {
    return store_cl_split(a.Eh + o, a.El + o, c, h, v);
  } else {
    store_cl(a.E + o, c, h, v);
    return v;
  }
}
template <class S>
__device__ __forceinline__ f32x16 stI(const CellArgs<S>& a, int t, size_t ro, int c, int h, const f32x16& v) {
  const size_t o = fr_off(t, a.B) + ro;
  if constexpr (sizeof(S) == 2) {
    return store_cl_split(a.Ic + o, a.Il + o, c, h, v);
  } else {
    store_cl(a.I + o, c, h, v);
    return v;
  }
}
template <class S>
__device__ __forceinline__ f32x8 prE(const CellArgs<S>& a, int t, size_t ro, int lane) {
  const size_t o = fr_off(t, a.B) + ro;
  if constexpr (sizeof(S) == 2) return pr_load_split(a.Eh + o, a.El + o, lane);
  else return pr_load<float>(a.E + o, lane);
}
template <class S>
__device__ __forceinline__ f32x8 prEh(const CellArgs<S>& a, int t, size_t ro, int lane) {
  const size_t o = fr_off(t, a.B) + ro;
  if constexpr (sizeof(S) == 2) return pr_load<S>(a.Eh + o, lane);
  else return pr_load<float>(a.E + o, lane);
}
template <class S>
__device__ __forceinline__ f32x8 prI(const CellArgs<S>& a, int t, size_t ro, int lane) {
  const size_t o = fr_off(t, a.B) + ro;
  if constexpr (sizeof(S) == 2) return pr_load_split(a.Ic + o, a.Il + o, lane);
  else return pr_load<float>(a.I + o, lane);
}
template <class S>
__device__ __forceinline__ f32x8 prIh(const CellArgs<S>& a, int t, size_t ro, int lane) {
  const size_t o = fr_off(t, a.B) + ro;
  if constexpr (sizeof(S) == 2) return pr_load<S>(a.Ic + o, lane);
  else return pr_load<float>(a.I + o, lane);
}

// Spatial tiling.  A frame larger than 32x32 (H, W multiples of 32) is held as
// nty x ntx tiles of 32x32, each stored and processed like a clip of its own
// (tile v = (clip b, row ty, col tx), v = (b nty + ty) ntx + tx).  Point-wise
// work never looks at neighbours; the k x k convolutions take their 3-px halo
// from the neighbouring tiles (tile_halo, WBand); BatchNorm's (B, H, W)
// statistics are the same sums over tiles instead of clips.
struct TileLoc { int b, ty, tx; };
__device__ __forceinline__ TileLoc tile_loc(int v, int ntx, int nty) {
  const int ntl = ntx * nty, b = v / ntl, q = v - b * ntl, ty = q / ntx;
  return {b, ty, q - ty * ntx};
}

// Stage rows [y0, y0+nrows) of tile v of x[:, 0:3, t] as float4 per pixel.
// x is either the model input f32 [clips][3][T][H][W] or (xu8) the raw clip
// bytes u8 [clips][T][H][W][3] as the TFRecords hold them, converted here
// exactly as engine.prepare_data does (utils/engine.py:220-255: the float64
// quotient u / 255 rounded to f32), so the f32 tensor never has to exist.
__device__ void stage_x(const void* __restrict__ xv, int xu8, f32x4* xs, int v, int t, int T,
                        int y0, int nrows, int tid, int nthreads, int ntx, int nty) {
  const TileLoc L = tile_loc(v, ntx, nty);
  const int W = ntx * IMG;
  if (xu8) {
    const uint8_t* x = (const uint8_t*)xv +
                       (((size_t)L.b * T + t) * ((size_t)nty * IMG) + L.ty * IMG + y0) * W * 3 +
                       (size_t)L.tx * IMG * 3;
    for (int p = tid; p < nrows * IMG; p += nthreads) {
      const uint8_t* q = x + ((size_t)(p >> 5) * W + (p & 31)) * 3;
      // the 3 bytes from aligned dwords (no sub-dword global loads, see ld_bf16_bits)
      const uintptr_t qa = (uintptr_t)q;
      const uint32_t* qw = (const uint32_t*)(qa & ~(uintptr_t)3);
      const int sh = (int)(qa & 3) * 8;
      uint64_t w = qw[0];
      if (sh >= 16) w |= (uint64_t)qw[1] << 32;
      w >>= sh;
      f32x4 v4;
      v4[0] = (float)((double)(uint32_t)(w & 0xff) / 255.0);
      v4[1] = (float)((double)(uint32_t)((w >> 8) & 0xff) / 255.0);
      v4[2] = (float)((double)(uint32_t)((w >> 16) & 0xff) / 255.0);
      v4[3] = 0.f;
      xs[p] = v4;
    }
    return;
  }
  const float* x = (const float*)xv;
  const size_t plane = (size_t)nty * IMG * W;
  const size_t o = (size_t)(L.ty * IMG + y0) * W + L.tx * IMG;
  const float* x0 = x + ((size_t)(L.b * 3 + 0) * T + t) * plane + o;
  const float* x1 = x + ((size_t)(L.b * 3 + 1) * T + t) * plane + o;
  const float* x2 = x + ((size_t)(L.b * 3 + 2) * T + t) * plane + o;
  // up to 4 pixels per thread in flight before the first store (one HBM
  // round trip however many threads stage)
  const int n = nrows * IMG;
  for (int p0 = tid; p0 < n; p0 += 4 * nthreads) {
    f32x4 v4[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int p = p0 + k * nthreads;
      if (p < n) {
        const int q = (p >> 5) * W + (p & 31);
        v4[k] = f32x4{x0[q], x1[q], x2[q], 0.f};
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int p = p0 + k * nthreads;
      if (p < n) xs[p] = v4[k];
    }
  }
}

// Halo of tile v's zero-padded LDS image when the frame has several tiles: the
// 420 border pixels (3 rows above / below incl. corners, 3 columns left /
// right) are channel chunks of the neighbouring tiles (ld maps a chunk's
// element offset to its 16 B, e.g. applying BatchNorm backward); positions
// outside the frame keep the zeros of tile_zero.
template <class S, int PAD, int NTH = NT, class Ld>
__device__ __forceinline__ void tile_halo(S* __restrict__ tile, int v, int ntx, int nty, int pass,
                                          int tid, Ld&& ld) {
  constexpr int CPB = 16 / (int)sizeof(S);
  constexpr int NCH = Tr<S>::CP / CPB;
  constexpr int TW = tile_w<PAD>();
  constexpr int NHP = TW * TW - NPIX;                  // 420 (PAD 3) / 1092 (PAD 7)
  constexpr int PER = (NHP * NCH + NTH - 1) / NTH;
  constexpr int BATCH = 6;                             // loads in flight per thread
  const TileLoc L = tile_loc(v, ntx, nty);
#pragma unroll
  for (int k0 = 0; k0 < PER; k0 += BATCH) {
    u32x4 val[BATCH];
    int dst[BATCH];
#pragma unroll
    for (int kk = 0; kk < BATCH; ++kk) {
      const int k = k0 + kk;
      const int idx = tid + k * NTH;
      const int hp = idx / NCH, q = idx - hp * NCH;
      int hy, hx;
      if (hp < PAD * TW) { hy = hp / TW - PAD; hx = hp % TW - PAD; }
      else if (hp < 2 * PAD * TW) { const int j = hp - PAD * TW; hy = IMG + j / TW; hx = j % TW - PAD; }
      else if (hp < 2 * PAD * TW + PAD * IMG) { const int j = hp - 2 * PAD * TW; hy = j / PAD; hx = j % PAD - PAD; }
      else { const int j = hp - 2 * PAD * TW - PAD * IMG; hy = j / PAD; hx = IMG + j % PAD; }
      const int dy = hy < 0 ? -1 : (hy >= IMG ? 1 : 0), dx = hx < 0 ? -1 : (hx >= IMG ? 1 : 0);
      const bool ok = k < PER && idx < NHP * NCH && L.ty + dy >= 0 && L.ty + dy < nty &&
                      L.tx + dx >= 0 && L.tx + dx < ntx;
      const int ly = hy - dy * IMG, lx = hx - dx * IMG;
      const size_t e = clip_off(ok ? v + dy * ntx + dx : v) + (size_t)(ly * IMG + lx) * C +
                       pass * Tr<S>::CP + q * CPB;
      val[kk] = ld(ok ? e : clip_off(v), pass * Tr<S>::CP + q * CPB);
      dst[kk] = ok ? tile_off<S, PAD>(hy + PAD, hx + PAD, q * CPB) : -1;
    }
#pragma unroll
    for (int kk = 0; kk < BATCH; ++kk)
      if (dst[kk] >= 0) *(u32x4*)(tile + dst[kk]) = val[kk];
  }
}

// Fused forward on tiled frames (r06, VERDICT r05 next #5a).  The conv's 3-px
// halo is the point-wise output of the neighbouring tiles' workgroups in the
// SAME launch.  After its rows every tile workgroup copies the 348 border
// pixels of its conv input (rows 0-2 and 29-31, columns 0-2 and 29-31 of its
// LDS tile) to its slot of xch with write-through (agent-scope) stores and,
// once they are acknowledged, sets its flag to t + 1; it then waits for the
// flags of its (up to 8) neighbours and fills its halo from their slots with
// agent-coherent loads (a neighbour may run on another XCD: no L2 is shared,
// the same protocol as the BatchNorm partials).  No grid barrier and no
// co-residency requirement: each XCD dispatches its workgroups in index
// order, so every workgroup resident on the XCD of the lowest not-yet-resident
// tile belongs to a lower clip, all of whose tiles are resident or done --
// they finish and free the slot.  The waits are bounded all the same: a
// give-up sets *xerr and fills the halo with NaN, so a broken assumption shows
// up as NaN results, never as a hang.  Same bf16 values as tile_halo reads
// from the stored conv input: bitwise the split tiled forward.
constexpr int XB_PIX = 6 * IMG + 6 * (IMG - 6);   // 348 border pixels of a 32x32 tile
__device__ __forceinline__ int xb_index(int ly, int lx) {
  if (ly < 3) return ly * IMG + lx;
  if (ly >= IMG - 3) return 3 * IMG + (ly - (IMG - 3)) * IMG + lx;
  return 6 * IMG + (ly - 3) * 6 + (lx < 3 ? lx : lx - (IMG - 6));
}
__device__ __forceinline__ void xb_pixel(int i, int& ly, int& lx) {
  if (i < 3 * IMG) { ly = i / IMG; lx = i % IMG; return; }
  if (i < 6 * IMG) { const int j = i - 3 * IMG; ly = IMG - 3 + j / IMG; lx = j % IMG; return; }
  const int j = i - 6 * IMG, q = j % 6;
  ly = 3 + j / 6;
  lx = q < 3 ? q : IMG - 6 + q;
}
template <class S, int NTH>
__device__ void xb_exchange(const CellArgs<S>& a, S* tile, unsigned* flags, int v, int t, int tid) {
  static_assert(sizeof(S) == 2, "the fused forward is bf16");
  // publish: 348 px x 8 quads of 4 channels (8 B), write-through
  uint64_t* dst = (uint64_t*)(a.xch + (size_t)v * XB_PIX * C);
  for (int w = tid; w < XB_PIX * 8; w += NTH) {
    int ly, lx;
    xb_pixel(w >> 3, ly, lx);
    const uint64_t val = *(const uint64_t*)(tile + tile_off<S, PADMAX>(ly + PADMAX, lx + PADMAX, 4 * (w & 7)));
    __hip_atomic_store(dst + w, val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");            // acknowledged
  __syncthreads();
  if (tid == 0) __hip_atomic_store(flags + v, (unsigned)(t + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // wait: lane 3 (dy + 1) + (dx + 1) of wave 0 polls neighbour (dy, dx)
  const TileLoc L = tile_loc(v, a.ntx, a.nty);
  int bad = 0;
  if (tid < 9 && tid != 4) {
    const int dy = tid / 3 - 1, dx = tid % 3 - 1;
    if (L.ty + dy >= 0 && L.ty + dy < a.nty && L.tx + dx >= 0 && L.tx + dx < a.ntx) {
      const unsigned* f = flags + v + dy * a.ntx + dx;
      for (unsigned it = 1; __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)(t + 1);
           ++it) {
        if ((it & 255) == 0 &&         // ~0.3 s, or another workgroup already gave up
            (it > (1u << 18) || __hip_atomic_load(a.xerr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
          bad = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
  }
  const bool poison = __syncthreads_or(bad);
  if (poison && tid == 0) __hip_atomic_store(a.xerr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // the halo from the neighbours' slots (agent-coherent 8-B loads)
  const uint64_t* src = (const uint64_t*)a.xch;
  tile_halo<S, PADMAX, NTH>(tile, v, a.ntx, a.nty, 0, tid, [&](size_t e, int) {
    const size_t nb = e / ((size_t)NPIX * C);
    const int r = (int)(e - nb * NPIX * C), pix = r / C, ch = r % C;
    const uint64_t* p = src + ((nb * XB_PIX + xb_index(pix / IMG, pix % IMG)) * C + ch) / 4;
    if (poison) return u32x4{0x7fc07fc0u, 0x7fc07fc0u, 0x7fc07fc0u, 0x7fc07fc0u};
    const uint64_t lo = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t hi = __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return u32x4{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)};
  });
}

// Stem (models/InT.py:212-213): z = W_pre x + b; xbn = nl(z); CL layout.
struct Stem { float w0, w1, w2, b; };
// WANT_D: z returns nl'(z) instead of z (the backward's stem gradient needs
// only that; f and f' then share one exponential).
template <int ACT, bool WANT_D = false>
__device__ __forceinline__ void stem_cl(const f32x4* xs, int yl, int h, const Stem& st,
                                        f32x16& z, f32x16& xv) {
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const f32x4 v = xs[yl * IMG + cl_x(r, h)];
    const float zr = st.w0 * v[0] + st.w1 * v[1] + st.w2 * v[2] + st.b;
    if constexpr (WANT_D) {
      float f, d;
      Act<ACT>::fd(zr, f, d);
      xv[r] = f;
      z[r] = d;
    } else {
      z[r] = zr;
      xv[r] = Act<ACT>::f(zr);
    }
  }
}

// Forward BN: batch mean / rstd per channel (B = clips / tiles counted, all
// replicas' under SyncBN) from the fp64 sums (ng group sums, added in order) of per-clip
// (mean_b, mean_b^2, M2_b) (Chan et al.: M2 = sum M2_b + n (sum mean_b^2 -
// (sum mean_b)^2 / B)); all threads end with them in stat[0..63].
// Lanes fl < 32 of ONE wave finalise (the caller picks the wave; others pass
// fl >= 32); stat is read only after the caller's next workgroup barrier.
template <bool COH = false>           // COH: the sums were written in this launch (persistent)
__device__ void bn_fwd_finalize(const double* __restrict__ grp, int ng, int B, float eps,
                                float* stat, float* gstat, int fl) {
  if (fl < 32) {
    const int tid = fl;
    double s1 = 0.0, s2 = 0.0, s3 = 0.0;
    auto ld = [&](int i) {
      return COH ? __hip_atomic_load(grp + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : grp[i];
    };
    // every group's loads in flight at once, then added in group order (a
    // loop over the runtime count waited on each group in turn: ~5.5 us of
    // the consumer's prologue)
    double x1[NGRP], x2[NGRP], x3[NGRP];
#pragma unroll
    for (int k = 0; k < NGRP; ++k) {
      const int kk = k < ng ? k : 0;
      x1[k] = ld(kk * 96 + tid); x2[k] = ld(kk * 96 + 32 + tid); x3[k] = ld(kk * 96 + 64 + tid);
    }
#pragma unroll
    for (int k = 0; k < NGRP; ++k)
      if (k < ng) { s1 += x1[k]; s2 += x2[k]; s3 += x3[k]; }
    const double mean = s1 / B;
    double m2 = s3 + (double)NPIX * (s2 - s1 * s1 / B);
    m2 = m2 > 0.0 ? m2 : 0.0;
    const float var = (float)(m2 / ((double)B * NPIX));
    const float rstd = 1.0f / sqrtf(var + eps);
    stat[tid] = (float)mean;
    stat[32 + tid] = rstd;
    if (gstat) { gstat[tid] = (float)mean; gstat[32 + tid] = rstd; }
  }
}

// Per-clip (mean, M2) of the conv outputs held in acc (PL layout), published
// to the deterministic batch reduction (bn_publish; scr / flag: free LDS).  Each wave runs a two-pass (mean, M2) over its own
// RW rows (its per-channel means go through its own LDS slot, no workgroup
// barrier); one barrier, then Chan's combination over the NW equal-sized wave
// blocks: M2 = sum M2_w + n_w sum (mean_w - mean)^2.  red: 2 * NW * 32 floats.
// Block blk (RW rows held in acc by the calling wave): two-pass per-channel
// mean -> red[blk * 32 + ch], M2 -> red[NW * 32 + blk * 32 + ch] (the block's
// means go through its own LDS slot: no workgroup barrier).
template <int RW, int NW>
__device__ __forceinline__ void bn_block_stats(const f32x16 (&acc)[RW], float* red, int blk, int lane) {
  const int h = lane >> 5;
  const int ch = pl_ch(pl_sum_reg(lane), h);
  f32x16 s = acc[0];
#pragma unroll
  for (int i = 1; i < RW; ++i) s += acc[i];
  const float ts = pl_lane_sum(s, lane);
  float* rw = red + blk * 32;                        // this block's means
  if (!(lane & 16)) rw[ch] = ts * (1.f / (RW * IMG));
  wave_sync();
  f32x16 mean;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const f32x4 m = *(const f32x4*)(rw + 8 * g + 4 * h);
#pragma unroll
    for (int j = 0; j < 4; ++j) mean[4 * g + j] = m[j];
  }
  f32x16 q = zero16();
#pragma unroll
  for (int i = 0; i < RW; ++i) {
    const f32x16 d = acc[i] - mean;
    q += d * d;
  }
  const float tq = pl_lane_sum(q, lane);
  if (!(lane & 16)) red[NW * 32 + blk * 32 + ch] = tq;
}
// After a workgroup barrier: Chan's combination over the NW equal-sized blocks
// (M2 = sum M2_w + n_w sum (mean_w - mean)^2), published to the batch
// reduction.  All NW * 64 threads call it.
template <int RW, int NW>
__device__ __forceinline__ void bn_blocks_publish(const float* red, const BnSlot& out, int prod, int tid,
                                                  int* flag, double* scr) {
  // lanes 0-31: channel tid's block mean; lanes 32-63: its M2
  const int ch2 = tid & 31;
  float mn = 0.f;
#pragma unroll
  for (int w = 0; w < NW; ++w) mn += red[w * 32 + ch2];
  mn *= 1.f / NW;
  float v = 0.f, dv = 0.f;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    const float d = red[w * 32 + ch2] - mn;
    v += red[NW * 32 + w * 32 + ch2];
    dv += d * d;
  }
  v += dv * (float)(RW * IMG);
  bn_publish<NW * 64, true>(out, prod, tid < 32 ? mn : v, tid, flag, scr);
}
// Per-clip (mean, M2) of the conv outputs held in acc (PL layout), published
// to the deterministic batch reduction (bn_publish; scr / flag: free LDS): each
// wave's RW rows are one block (bn_block_stats), one barrier, then the
// combination (bn_blocks_publish).  red: 2 * NW * 32 floats.
template <int RW, int NW>
__device__ void bn_fwd_partial(const f32x16 (&acc)[RW], float* red, const BnSlot& out, int prod,
                               int lane, int wave, int tid, int ablate, int* flag, double* scr) {
  bn_block_stats<RW, NW>(acc, red, wave, lane);
  __syncthreads();
  if (PT_ABL(ablate) & 32768) return;
  bn_blocks_publish<RW, NW>(red, out, prod, tid, flag, scr);
}

// =========================================================================
// Conv kernels: one workgroup (4 waves x 8 rows) per clip; the whole 32x32
// clip image is one zero-halo LDS tile.  FILL: how the tile interior is
// produced; EPI: what happens to the conv result.
//   FILL_COPY   input image as stored (forward: gE_t or I_t)
//   FILL_BNBWD  BatchNorm backward applied on the fly (models/InT.py:161/:172
//               reversed): dx = rstd g (dy - mean(dy) - xhat mean(dy xhat)),
//               also written out (the k x k weight gradient's D operand)
//   EPI_FWD     store the pre-BN conv output + per-clip BN statistics
//   EPI_ADD     out = conv + add0 (+ add1), f32
//   EPI_NONE    fill only (frame 0's dci: needed by k_wgrad, conv^T dead)
// =========================================================================
enum { FILL_COPY = 0, FILL_BNBWD = 1 };
enum { EPI_FWD = 0, EPI_ADD = 1, EPI_NONE = 2 };

// Backward BN consumers: sum dy and sum dy*xhat of channel c over the ng (<=
// NGRP) group sums, added in group order with every load in flight at once.
__device__ __forceinline__ void bnb_sums(const double* __restrict__ g, int ng, int c, double& sd, double& sdx) {
  double x[NGRP], y[NGRP];
#pragma unroll
  for (int k = 0; k < NGRP; ++k) {
    const int kk = k < ng ? k : 0;
    x[k] = g[kk * 64 + c];
    y[k] = g[kk * 64 + 32 + c];
  }
#pragma unroll
  for (int k = 0; k < NGRP; ++k)
    if (k < ng) { sd += x[k]; sdx += y[k]; }
}

template <class S>
struct ConvArgs {
  using F = typename Tr<S>::frag;
  int B, K, ablate;
  int ntx, nty;                 // tiles per frame (halo from neighbours when > 1 x 1)
  int xmap;                     // XCD-affine workgroup order (wg_split)
  const S* src;                 // FILL_COPY: frame base [B][NPIX][C]
  const S* dc;                  // FILL_BNBWD: dy
  const S* raw;                 // FILL_BNBWD: pre-BN conv output of the forward
  const float* bnstat;          // FILL_BNBWD: mean[32], rstd[32]
  const double* bnb;            // FILL_BNBWD: group sums [ngrp][64] (sum dy[32], sum dy*xhat[32])
  int bnb_ngrp;
  int bnB;                      // FILL_BNBWD: clips / tiles in the statistics (all replicas' under SyncBN)
  const float* bnw;             // FILL_BNBWD: BN gamma
  S* fill_out;                  // FILL_BNBWD: dx written here too
  const F* wf;
  S* out_raw;                   // EPI_FWD
  BnSlot bnout;                 // EPI_FWD: per-clip BN partials
  S* out;                       // EPI_ADD
  const S *add0, *add1;         // EPI_ADD (add1 may be null)
  unsigned long long* trace;    // diagnostics (PT_TR): as CellArgs, stamped as trace_kind
  int trace_t, t, trace_kind;
};

constexpr int CONV_MISC = 512;  // floats: red[256] (bn-bwd table [3][32] aliases it)
// k <= 7: 38 x 38 tile + two weight slices; k > 7: 46 x 46 tile, weights from L2
template <class S, int PAD = PADMAX>
constexpr int conv_lds_bytes() {
  return tile_bytes<S, PAD>() + CONV_MISC * 4 + (PAD == PADMAX ? 2 * WSLICE_BYTES : 0);
}

// conv_run row hook of EPI_FWD: store a finished output row (PL layout)
template <class S>
struct StoreRow {
  S* base;
  int h;
  bool rnd;       // diagnostic rounding (RND_C)
  static constexpr bool active = true;
  static constexpr bool prefetch_active = false;
  // B fragments from L2 into registers one column ahead, no per-column
  // barrier (vs the LDS slice ring: 31.7 -> 30.1 us per launch)
  static constexpr bool wreg = true;
  __device__ __forceinline__ void prefetch() const {}
  __device__ __forceinline__ void operator()(int i, const f32x16& v) const {
    store_pl(base + (size_t)i * IMG * C, h, rb16(rnd, v));
  }
};

// conv_run row hook of EPI_ADD (bf16): the add0 / add1 rows of this wave are
// prefetched into registers under the MFMA loop (issued at the first column);
// each output row is summed and stored as soon as its last MFMA retires.
// (Loaded after the loop, the 256 workgroups' add/store burst cost conv_bb
// 11 us and conv_ba 7 us per launch.)
template <int RW>
struct AddRowBf16 {
  bf16_t* out;
  const bf16_t *add0, *add1;      // add1 may be null
  size_t po;                      // element offset of row 0 of this lane's pixel
  int h;
  bf16x4 (&p0)[RW][4];
  bf16x4 (&p1)[RW][4];
  static constexpr bool active = true;
  static constexpr bool prefetch_active = true;
  static constexpr bool wreg = false;
  __device__ __forceinline__ void prefetch() const {
#pragma unroll
    for (int i = 0; i < RW; ++i)
#pragma unroll
      for (int g = 0; g < 4; ++g) p0[i][g] = *(const bf16x4*)(add0 + po + (size_t)i * IMG * C + 8 * g + 4 * h);
    if (add1)
#pragma unroll
      for (int i = 0; i < RW; ++i)
#pragma unroll
        for (int g = 0; g < 4; ++g) p1[i][g] = *(const bf16x4*)(add1 + po + (size_t)i * IMG * C + 8 * g + 4 * h);
  }
  __device__ __forceinline__ void operator()(int i, const f32x16& acc) const {
    f32x16 v = acc;
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int j = 0; j < 4; ++j) v[4 * g + j] += (float)p0[i][g][j];
    if (add1)
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int j = 0; j < 4; ++j) v[4 * g + j] += (float)p1[i][g][j];
    store_pl(out + po + (size_t)i * IMG * C, h, v);
  }
};

template <class S, int FILL, int EPI, int PAD, int NTH = NT>
__device__ __forceinline__ void conv_body(const ConvArgs<S>& a, char* smem, int b) {
  constexpr int NW = NTH / 64, RW = IMG / NW;      // waves, image rows per wave
  static_assert(2 * NW * 32 <= CONV_MISC, "BN partial table");
  S* tile = (S*)smem;
  float* red = (float*)(smem + tile_bytes<S, PAD>());
  float* tbl = red + 128;       // FILL_BNBWD: per-channel A, Bc, Cc
  char* wbuf = (char*)(red + CONV_MISC);   // 2 weight slices
  const int tid = threadIdx.x, lane = tid & 63, c = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const size_t cb = clip_off(b);
  if (PT_ABL(a.ablate) & 512) return;

  if constexpr (FILL == FILL_BNBWD) {
    if (tid < 32) {
      // dx = A dy + Bc raw + Cc  with A = rstd g, xhat = (raw - mean) rstd
      const double inv = 1.0 / ((double)a.bnB * NPIX);
      double sd = 0.0, sdx = 0.0;
      bnb_sums(a.bnb, a.bnb_ngrp, tid, sd, sdx);
      const float md = (float)(sd * inv), mdx = (float)(sdx * inv);
      const float mean = a.bnstat[tid], rstd = a.bnstat[32 + tid];
      const float A = rstd * a.bnw[tid];
      tbl[tid] = A;
      tbl[32 + tid] = -A * mdx * rstd;
      tbl[64 + tid] = -A * md + A * mdx * rstd * mean;
    }
  }
  if constexpr (EPI != EPI_NONE) tile_zero<S, PAD, NTH>(tile, tid);
  __syncthreads();

  const bool tiled = a.ntx * a.nty > 1;
  auto bnbwd16 = [&](const u32x4& dv, const u32x4& rv, int ch0) {
    constexpr int CPB = 16 / (int)sizeof(S);
    const S* rr = (const S*)&rv;
    const S* dd = (const S*)&dv;
    u32x4 ov;
    S* oo = (S*)&ov;
#pragma unroll
    for (int j = 0; j < CPB; ++j) {
      const int ch = ch0 + j;
      oo[j] = (S)(tbl[ch] * ldf(dd + j) + tbl[32 + ch] * ldf(rr + j) + tbl[64 + ch]);
    }
    return ov;
  };
  auto ldc = [&](size_t e, int) { return *(const u32x4*)(a.src + e); };
  auto ldb = [&](size_t e, int ch0) {
    return bnbwd16(*(const u32x4*)(a.dc + e), *(const u32x4*)(a.raw + e), ch0);
  };
  auto fill = [&](int pass) {
    if constexpr (FILL == FILL_COPY) {
      if (tiled)
        tile_halo<S, PAD, NTH>(tile, b, a.ntx, a.nty, pass, tid, ldc);
      tile_fill<S, PAD, NTH>(tile, a.src + cb, pass, tid);
    } else if constexpr (FILL == FILL_BNBWD) {
      if (EPI != EPI_NONE && tiled)
        tile_halo<S, PAD, NTH>(tile, b, a.ntx, a.nty, pass, tid, ldb);
      constexpr int CPB = 16 / (int)sizeof(S);      // channels per 16-B chunk of S
      constexpr int NCH = Tr<S>::CP / CPB;
      constexpr int PER = NPIX * NCH / NTH;          // 16 chunks per thread at 256 threads
      constexpr int BATCH = 4;
#pragma unroll
      for (int k0 = 0; k0 < PER; k0 += BATCH) {
        uint4 dv[BATCH], rv[BATCH];
#pragma unroll
        for (int k = 0; k < BATCH; ++k) {
          const int idx = tid + (k0 + k) * NTH;
          const int pix = idx / NCH, q = idx % NCH;
          const size_t e = cb + (size_t)pix * C + pass * Tr<S>::CP + q * CPB;
          dv[k] = *(const uint4*)(a.dc + e);
          rv[k] = *(const uint4*)(a.raw + e);
        }
#pragma unroll
        for (int k = 0; k < BATCH; ++k) {
          const int idx = tid + (k0 + k) * NTH;
          const int pix = idx / NCH, q = idx % NCH;
          const int ch0 = pass * Tr<S>::CP + q * CPB;
          const S* rr = (const S*)&rv[k];
          const S* dd = (const S*)&dv[k];
          uint4 ov;
          S* oo = (S*)&ov;
#pragma unroll
          for (int j = 0; j < CPB; ++j) {
            const int ch = ch0 + j;
            const float v = tbl[ch] * ldf(dd + j) + tbl[32 + ch] * ldf(rr + j) + tbl[64 + ch];
            oo[j] = (S)rbf(RND_T(a), v);
          }
          *(uint4*)(a.fill_out + cb + (size_t)pix * C + ch0) = ov;
          if constexpr (EPI != EPI_NONE) {
            const int y = pix >> 5, x = pix & 31;
            *(uint4*)(tile + tile_off<S, PAD>(y + PAD, x + PAD, q * CPB)) = ov;
          }
        }
      }
    }
  };

  if constexpr (EPI == EPI_NONE) {
    for (int pass = 0; pass < Tr<S>::NPASS; ++pass) fill(pass);
    return;
  } else {
    f32x16 acc[RW];
#pragma unroll
    for (int i = 0; i < RW; ++i) acc[i] = zero16();
    const int px = lane & 31;
    if constexpr (EPI == EPI_FWD) {
      // each finished row is stored while the later rows' MFMAs still run
      // (all 256 workgroups storing at the very end took ~6.5 us per launch)
      const StoreRow<S> sr{a.out_raw + cb + ((size_t)(wave * RW) * IMG + px) * C, h, RND_C(a)};
      conv_run<S, PAD, RW, NTH>(acc, fill, a.wf, tile, wbuf, a.K, wave * RW, lane, tid, a.ablate, sr);
      if (PT_ABL(a.ablate) & 256) return;
      // the tile is free once every wave has passed bn_fwd_partial's barrier
      if (!(PT_ABL(a.ablate) & 8))
        bn_fwd_partial<RW, NW>(acc, red, a.bnout, b, lane, wave, tid, a.ablate,
                               (int*)(smem + NTH * 16), (double*)smem);
    } else if constexpr (sizeof(S) == 2) {
      bf16x4 p0[RW][4], p1[RW][4];
      const AddRowBf16<RW> ar{(bf16_t*)a.out, (const bf16_t*)a.add0, (const bf16_t*)a.add1,
                              cb + ((size_t)(wave * RW) * IMG + px) * C, h, p0, p1};
      conv_run<S, PAD, RW, NTH>(acc, fill, a.wf, tile, wbuf, a.K, wave * RW, lane, tid, a.ablate, ar);
    } else {
      conv_run<S, PAD, RW, NTH>(acc, fill, a.wf, tile, wbuf, a.K, wave * RW, lane, tid, a.ablate);
      if (PT_ABL(a.ablate) & 256) return;
#pragma unroll
      for (int i = 0; i < RW; ++i) {
        const size_t po = cb + ((size_t)(wave * RW + i) * IMG + px) * C;
        f32x16 v = acc[i];
        add_pl(a.add0 + po, h, v);
        if (a.add1) add_pl(a.add1 + po, h, v);
        if (PT_ABL(a.ablate) & 1024) store_pl_nt(a.out + po, h, v);
        else store_pl(a.out + po, h, rb16(RND_T(a), v));
      }
    }
  }
}
// SyncBN: the ngrp group sums of one reduction, added in group order, into the
// buffer the replicas all-reduce (pt_cell_dist.bn_buf).
__global__ void k_bn_total(const double* __restrict__ grp, int ngrp, int nv, double* __restrict__ out) {
  const int v = threadIdx.x;
  if (v >= nv) return;
  double s = 0.0;
  for (int k = 0; k < ngrp; ++k) s += grp[k * nv + v];
  out[v] = s;
}

// Distinct kernel names per role (rocprof summaries tell them apart).
template <class S, int PAD, int NTH = NT>
__global__ __launch_bounds__(NTH, 1) void k_conv_fwd(ConvArgs<S> a) {     // conv + BN partials
  extern __shared__ __attribute__((aligned(16))) char smem[];
  conv_body<S, FILL_COPY, EPI_FWD, PAD, NTH>(a, smem, blockIdx.x);
}
template <class S, int PAD, int NTH = NT>
__global__ __launch_bounds__(NTH, 1) void k_conv_bwd(ConvArgs<S> a) {     // BN bwd + conv^T + adds
  extern __shared__ __attribute__((aligned(16))) char smem[];
  conv_body<S, FILL_BNBWD, EPI_ADD, PAD, NTH>(a, smem, blockIdx.x);
}
// k <= 7: 8-wave workgroups, 4 image rows per wave (2 waves per SIMD; vs 4
// waves x 8 rows: conv_fwd 34.0 -> 33.4 us, conv_bwd of the BN1 side 42.2 ->
// 39.1 us at B=256 bf16); k > 7: 4 waves x 8 rows (the 46 x 46 tile)
constexpr int CONV_NT = 512;

// -------------------------------------------------------------------------
// Banded backward conv (bf16, 32x32 frames, k <= 7; PT_CONV_BAND=1): TWO
// workgroups per clip, each a 16-row band of the output (4 waves x 4 rows)
// over a 22 x 38 halo tile (55 KB of LDS, so two workgroups share a CU and one
// fills / finishes while the other's MFMAs run -- the whole-clip form is one
// workgroup per CU with its fill, slice ring and epilogue serial).  B
// fragments come from L2 into registers one column ahead (no slice ring, no
// per-column barrier); each finished output row adds its addends and is
// stored at once (no prefetch: the co-resident workgroup covers the latency).
// Per output row the MFMA order is that of k_conv_bwd: results bit-identical.
// Issue priority (r06, the HW_ID trace: profiles/r06_trace_phases.txt).  The
// SIMD arbiter favours the older wave at equal priority, so the half a kernel
// starts second runs starved and ends last: the band-1 waves (4-7) of the
// staggered segments and of k_conv_bwd_band2 -- the critical path of both --
// and the second workgroup on a CU in k_pw_bb2 / k_pw_ba (rows ending ~10 us
// after the first one's).  PT_PRIO bit 0: band-1 waves at priority 1 in the
// fused segments; bit 1: the same in k_conv_bwd_band2; bit 2: the backward
// point-wise kernels lower their priority as they progress (3 - set / row),
// so the workgroup that is ahead yields to the one behind; bit 3: and the
// workgroup dispatched first on a CU (the first half of a 2-per-CU grid:
// blocks j and j + grid/2 share a CU, the trace shows) one level lower at
// the same step, so at equal progress the younger one wins, not the older;
// bit 4: in k_fused_fb the band-1 waves drop back to 0 and the band-0 waves
// rise to 1 once the rows are in (band 0's conv ends last there); bit 5:
// k_conv_bwd_band2's band-1 waves drop to 0 after their fill.
// Default 7 (bits 0-2; bit 3 measured slower: k_pw_bb2 53.7 -> 55.4 us):
// with RA_FA = 3 the step's device time 21.38 -> 20.64 ms
// (profiles/r06_libab_prio_{a,b,c}.txt, interleaved in one process).
#ifndef PT_PRIO
#define PT_PRIO 7
#endif
__device__ __forceinline__ void prio_by_step(int step) {   // 3 - step, clamped; step wave-uniform
  if (step <= 0) __builtin_amdgcn_s_setprio(3);
  else if (step == 1) __builtin_amdgcn_s_setprio(2);
  else if (step == 2) __builtin_amdgcn_s_setprio(1);
  else __builtin_amdgcn_s_setprio(0);
}
// -------------------------------------------------------------------------
constexpr int BAND_ROWS = 16, BAND_NT = 256, BAND_TR = BAND_ROWS + 2 * PADMAX;
// r06: k_conv_bwd_band2's first fill loads issued before the BatchNorm table
// (band_fill_pre): bitwise, measured no faster (conv_bb 36.9 vs 36.6 us, the
// step 20.764 ms both, profiles/r06_libab_fillpre.txt -- the fill is bound by
// the launch's HBM burst, not by the table's latency); off by default
#ifndef PT_FILL_PRE
#define PT_FILL_PRE 0
#endif
constexpr int band_tile_bytes() { return BAND_TR * TILE * C * 2; }

template <int RW>
struct AddRowBand {
  bf16_t* out;
  const bf16_t *add0, *add1;
  size_t po;
  int h;
  bf16x4 (&p0)[RW][4];
  bf16x4 (&p1)[RW][4];
  static constexpr bool active = true;
  static constexpr bool prefetch_active = false;
  static constexpr bool wreg = true;
  // r05: row i's addends are loaded PT_BAND_LEAD tile-row steps before the
  // row's last MFMA (conv_run_k calls pre(i)), not at the row's store: the
  // four rows of a wave finish within its last kernel column, and each store
  // waited for its own loads in turn (XNOADD: -5.7 us of conv_bb's 39.5)
  static constexpr int row_pre_lead = PT_BAND_LEAD;
  __device__ __forceinline__ void prefetch() const {}
  __device__ __forceinline__ void pre(int i) const {
    if constexpr (PT_BAND_LEAD > 0) {
#pragma unroll
      for (int g = 0; g < 4; ++g) p0[i][g] = *(const bf16x4*)(add0 + po + (size_t)i * IMG * C + 8 * g + 4 * h);
      if (add1)
#pragma unroll
        for (int g = 0; g < 4; ++g) p1[i][g] = *(const bf16x4*)(add1 + po + (size_t)i * IMG * C + 8 * g + 4 * h);
    }
  }
  __device__ __forceinline__ void operator()(int i, const f32x16& acc) const {
    f32x16 v = acc;
#if !PT_BAND_XNOADD     // (timing experiments only: without the addends)
    if constexpr (PT_BAND_LEAD > 0) {
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int j = 0; j < 4; ++j) v[4 * g + j] += (float)p0[i][g][j];
      if (add1)
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int j = 0; j < 4; ++j) v[4 * g + j] += (float)p1[i][g][j];
    } else {
      add_pl(add0 + po + (size_t)i * IMG * C, h, v);
      if (add1) add_pl(add1 + po + (size_t)i * IMG * C, h, v);
    }
#endif
    store_pl(out + po + (size_t)i * IMG * C, h, v);
  }
};

// Frames of several 32x32 tiles (cfg4, r06): the band tile's border pixels
// that lie in the neighbouring tiles -- the 3 rows above band 0 / below band
// 1 (38 px each, corners included) and 3 columns either side of the band's 19
// image rows -- BatchNorm-backward mapped as band_fill maps the interior
// (positions outside the frame keep the tile's zeros).  The same values
// tile_halo gives the whole-clip conv.
template <int NTH>
__device__ __forceinline__ void band_halo(const ConvArgs<bf16_t>& a, const float* tbl, bf16_t* tile, int v,
                                          int band, int tid) {
  using S = bf16_t;
  constexpr int CPB = 8, NCH = C / CPB, NHP = PADMAX * TILE + 19 * 2 * PADMAX;   // 114 + 114 px
  constexpr int BATCH = 4;
  const TileLoc L = tile_loc(v, a.ntx, a.nty);
  const int y0 = band * BAND_ROWS;
  for (int i0 = tid; i0 < NHP * NCH; i0 += BATCH * NTH) {
    uint4 dv[BATCH], rv[BATCH];
    int dst[BATCH];
#pragma unroll
    for (int k = 0; k < BATCH; ++k) {
      const int idx = i0 + k * NTH;
      const int hp = idx / NCH, q = idx % NCH;
      int hy, hx;
      if (hp < PADMAX * TILE) {                         // the full rows beyond the band's image edge
        hy = (band == 0 ? -PADMAX : IMG) + hp / TILE;
        hx = hp % TILE - PADMAX;
      } else {                                          // the side columns of the band's image rows
        const int j = hp - PADMAX * TILE, sd = j % (2 * PADMAX);
        hy = (band == 0 ? 0 : IMG - 19) + j / (2 * PADMAX);
        hx = sd < PADMAX ? sd - PADMAX : IMG + sd - PADMAX;
      }
      const int dy = hy < 0 ? -1 : (hy >= IMG ? 1 : 0), dx = hx < 0 ? -1 : (hx >= IMG ? 1 : 0);
      const bool ok = idx < NHP * NCH && L.ty + dy >= 0 && L.ty + dy < a.nty && L.tx + dx >= 0 &&
                      L.tx + dx < a.ntx;
      const size_t e = clip_off(ok ? v + dy * a.ntx + dx : v) +
                       (size_t)(ok ? (hy - dy * IMG) * IMG + hx - dx * IMG : 0) * C + q * CPB;
      dv[k] = *(const uint4*)(a.dc + e);
      rv[k] = *(const uint4*)(a.raw + e);
      dst[k] = ok ? tile_off<S, PADMAX>(hy - y0 + PADMAX, hx + PADMAX, q * CPB) : -1;
    }
#pragma unroll
    for (int k = 0; k < BATCH; ++k) {
      if (dst[k] < 0) continue;
      const int ch0 = ((i0 + k * NTH) % NCH) * CPB;
      const S* rr = (const S*)&rv[k];
      const S* dd = (const S*)&dv[k];
      uint4 ov;
      S* oo = (S*)&ov;
#pragma unroll
      for (int j = 0; j < CPB; ++j) {
        const int ch = ch0 + j;
        oo[j] = (S)(tbl[ch] * ldf(dd + j) + tbl[32 + ch] * ldf(rr + j) + tbl[64 + ch]);
      }
      *(uint4*)(tile + dst[k]) = ov;
    }
  }
}

// One band's BatchNorm-backward fill (r05; the tile rows [y0 - PAD, y0 + 16 +
// PAD) within the image, each pixel of the band's own rows also written out).
// r06: the first batch of each thread's loads can be issued before the
// BatchNorm table exists (FillPre, band_fill_pre: the loads do not need it),
// so their HBM latency runs under the table's group-sum loads instead of
// after the barrier that publishes it -- by every wave but wave 0, which
// computes the table (vmcnt counts in order: its group-sum loads would wait
// behind the fill's).  Same values, same arithmetic.
constexpr int BFILL_BATCH = 4;
struct FillPre { u32x4 dv[BFILL_BATCH], rv[BFILL_BATCH]; };
__device__ __forceinline__ int band_fill_n(int y0) {
  const int r0 = y0 - PADMAX < 0 ? 0 : y0 - PADMAX;
  const int r1 = y0 + BAND_ROWS + PADMAX > IMG ? IMG : y0 + BAND_ROWS + PADMAX;
  return (r1 - r0) * IMG * (C / 8);
}
template <int NTH>
__device__ __forceinline__ void band_fill_ld(const ConvArgs<bf16_t>& a, size_t cb, int y0, int i0, int n,
                                             u32x4 (&dv)[BFILL_BATCH], u32x4 (&rv)[BFILL_BATCH]) {
  constexpr int NCH = C / 8;
  const int r0 = y0 - PADMAX < 0 ? 0 : y0 - PADMAX;
#pragma unroll
  for (int k = 0; k < BFILL_BATCH; ++k) {
    const int idx = i0 + k * NTH < n ? i0 + k * NTH : i0;
    const int pix = r0 * IMG + idx / NCH, q = idx % NCH;
    const size_t e = cb + (size_t)pix * C + q * 8;
#if PT_BAND_XNOFILL     // (timing experiments only: no fill loads)
    dv[k] = u32x4{(unsigned)e, 0u, 0u, 0u}; rv[k] = dv[k];
#else
    dv[k] = *(const u32x4*)(a.dc + e);
    rv[k] = *(const u32x4*)(a.raw + e);
#endif
  }
}
template <int NTH>
__device__ __forceinline__ void band_fill_pre(const ConvArgs<bf16_t>& a, size_t cb, int y0, int tid, FillPre& p) {
  band_fill_ld<NTH>(a, cb, y0, tid, band_fill_n(y0), p.dv, p.rv);
}
template <int NTH>
__device__ __forceinline__ void band_fill_st(const ConvArgs<bf16_t>& a, const float* tbl, bf16_t* tile,
                                             size_t cb, int y0, int i0, int n,
                                             const u32x4 (&dv)[BFILL_BATCH], const u32x4 (&rv)[BFILL_BATCH]) {
  using S = bf16_t;
  constexpr int CPB = 8, NCH = C / CPB;
  const int r0 = y0 - PADMAX < 0 ? 0 : y0 - PADMAX;
#pragma unroll
  for (int k = 0; k < BFILL_BATCH; ++k) {
    const int idx = i0 + k * NTH;
    if (idx >= n) break;
    const int pix = r0 * IMG + idx / NCH, q = idx % NCH, ch0 = q * CPB;
    const S* rr = (const S*)&rv[k];
    const S* dd = (const S*)&dv[k];
    uint4 ov;
    S* oo = (S*)&ov;
#pragma unroll
    for (int j = 0; j < CPB; ++j) {
      const int ch = ch0 + j;
      oo[j] = (S)(tbl[ch] * ldf(dd + j) + tbl[32 + ch] * ldf(rr + j) + tbl[64 + ch]);
    }
    const int y = pix >> 5, x = pix & 31;
    if (y >= y0 && y < y0 + BAND_ROWS)          // each pixel written out by one band
      *(uint4*)(a.fill_out + cb + (size_t)pix * C + ch0) = ov;
    *(uint4*)(tile + tile_off<S, PADMAX>(y - y0 + PADMAX, x + PADMAX, ch0)) = ov;
  }
}
template <int NTH, bool PRE = false>
__device__ __forceinline__ void band_fill(const ConvArgs<bf16_t>& a, const float* tbl, bf16_t* tile,
                                          size_t cb, int y0, int tid, const FillPre& pre = FillPre{},
                                          bool use_pre = false) {
  const int n = band_fill_n(y0);
  int i0 = tid;
  if constexpr (PRE) {          // the first batch: prefetched (use_pre) or loaded here
    u32x4 dv[BFILL_BATCH], rv[BFILL_BATCH];
    if (use_pre) {
#pragma unroll
      for (int k = 0; k < BFILL_BATCH; ++k) { dv[k] = pre.dv[k]; rv[k] = pre.rv[k]; }
    } else {
      band_fill_ld<NTH>(a, cb, y0, i0, n, dv, rv);
    }
    if (i0 < n) band_fill_st<NTH>(a, tbl, tile, cb, y0, i0, n, dv, rv);
    i0 += BFILL_BATCH * NTH;
  }
  for (; i0 < n; i0 += BFILL_BATCH * NTH) {
    u32x4 dv[BFILL_BATCH], rv[BFILL_BATCH];
    band_fill_ld<NTH>(a, cb, y0, i0, n, dv, rv);
    band_fill_st<NTH>(a, tbl, tile, cb, y0, i0, n, dv, rv);
  }
}

// The band's conv with a row hook (hook(i, acc): output row i finished;
// k_conv_bwd_band adds the addends and stores, k_conv_pw_ba keeps the row).
constexpr int BAND_RW = BAND_ROWS / (BAND_NT / 64);
template <class Hook>
__device__ __forceinline__ void band_conv_body(const ConvArgs<bf16_t>& a, char* smem, int b, int band,
                                               f32x16 (&acc)[BAND_RW], const Hook& ar) {
  using S = bf16_t;
  constexpr int RW = BAND_RW;
  S* tile = (S*)smem;
  float* tbl = (float*)(smem + band_tile_bytes());
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int y0 = band * BAND_ROWS;
  const size_t cb = clip_off(b);
  if (tid < 32) {     // BN backward as an affine map per channel (as conv_body)
    const double inv = 1.0 / ((double)a.bnB * NPIX);
    double sd = 0.0, sdx = 0.0;
    bnb_sums(a.bnb, a.bnb_ngrp, tid, sd, sdx);
    const float md = (float)(sd * inv), mdx = (float)(sdx * inv);
    const float mean = a.bnstat[tid], rstd = a.bnstat[32 + tid];
    const float A = rstd * a.bnw[tid];
    tbl[tid] = A;
    tbl[32 + tid] = -A * mdx * rstd;
    tbl[64 + tid] = -A * md + A * mdx * rstd * mean;
  }
  {
    uint4* z = (uint4*)tile;
    for (int i = tid; i < band_tile_bytes() / 16; i += BAND_NT) z[i] = make_uint4(0, 0, 0, 0);
  }
  auto fill = [&](int) {
    // (no prefetch here: beside the first weight column and the hook's addend
    // registers it spilled in k_conv_pw_ba)
    band_fill<BAND_NT>(a, tbl, tile, cb, y0, tid);
    if (a.ntx * a.nty > 1) band_halo<BAND_NT>(a, tbl, tile, b, band, tid);   // tiled frames (r06)
  };
#pragma unroll
  for (int i = 0; i < RW; ++i) acc[i] = zero16();
  conv_run<S, PADMAX, RW, BAND_NT>(acc, fill, a.wf, tile, nullptr, a.K, wave * RW, lane, tid, a.ablate, ar);
}
__global__ __launch_bounds__(BAND_NT, 2) void k_conv_bwd_band(ConvArgs<bf16_t> a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int RW = BAND_RW;
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, px = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int b, band;
  wg_split(blockIdx.x, 2, a.B, a.xmap, b, band);
  f32x16 acc[RW];
  bf16x4 p0[RW][4], p1[RW][4];
  const AddRowBand<RW> ar{(bf16_t*)a.out, (const bf16_t*)a.add0, (const bf16_t*)a.add1,
                          clip_off(b) + ((size_t)(band * BAND_ROWS + wave * RW) * IMG + px) * C, h, p0, p1};
  band_conv_body(a, smem, b, band, acc, ar);
}
// -------------------------------------------------------------------------
// Staggered two-band backward conv (r05, PT_CONV_BAND=3): the two 16-row
// bands of a clip in ONE 8-wave workgroup (both 22 x 38 tiles in LDS,
// 107 KB).  All 8 waves fill band 0; then waves 0-3 run band 0's conv while
// waves 4-7 fill band 1 (BN-backward loads + affine map: the HBM phase of one
// band under the MFMA phase of the other, on the same SIMDs), sync among
// themselves through an LDS counter and run band 1's conv.  In
// k_conv_bwd_band the two workgroups of a CU start together and stay in step,
// so neither fill is covered.  Per output row: k_conv_bwd_band's arithmetic
// (same fill values, same MFMA order, same addend order): bitwise equal.
// -------------------------------------------------------------------------
constexpr int BAND2_NT = 512;
constexpr int band2_lds_bytes() { return 2 * band_tile_bytes() + CONV_MISC * 4; }

__global__ __launch_bounds__(BAND2_NT, 1) void k_conv_bwd_band2(ConvArgs<bf16_t> a) {
  using S = bf16_t;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int RW = BAND_ROWS / 4;
  S* tile0 = (S*)smem;
  S* tile1 = (S*)(smem + band_tile_bytes());
  float* tbl = (float*)(smem + 2 * band_tile_bytes());
  int* ready = (int*)(tbl + 96);            // band 1's filler waves, counted in
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, px = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int b = blockIdx.x;
  const size_t cb = clip_off(b);
  PT_TR(a, a.trace_kind, 0);
  FillPre pre;
  const bool use_pre = PT_FILL_PRE != 0 && tid >= 64;    // (wave 0 computes the table)
  if (use_pre) band_fill_pre<BAND2_NT>(a, cb, 0, tid, pre);   // under the table's loads
  if (tid < 32) {     // BN backward as an affine map per channel (as conv_body)
    const double inv = 1.0 / ((double)a.bnB * NPIX);
    double sd = 0.0, sdx = 0.0;
    bnb_sums(a.bnb, a.bnb_ngrp, tid, sd, sdx);
    const float md = (float)(sd * inv), mdx = (float)(sdx * inv);
    const float mean = a.bnstat[tid], rstd = a.bnstat[32 + tid];
    const float A = rstd * a.bnw[tid];
    tbl[tid] = A;
    tbl[32 + tid] = -A * mdx * rstd;
    tbl[64 + tid] = -A * md + A * mdx * rstd * mean;
  }
  if (tid == 0) *ready = 0;
  {
    uint4* z = (uint4*)smem;
    for (int i = tid; i < 2 * band_tile_bytes() / 16; i += BAND2_NT) z[i] = make_uint4(0, 0, 0, 0);
  }
  __syncthreads();
  PT_TR(a, a.trace_kind, 1);
  band_fill<BAND2_NT, PT_FILL_PRE != 0>(a, tbl, tile0, cb, 0, tid, pre, use_pre);
  const bool tiled = a.ntx * a.nty > 1;
  if (tiled) band_halo<BAND2_NT>(a, tbl, tile0, b, 0, tid);
  __syncthreads();
  PT_TR(a, a.trace_kind, 2);
  const int wb = wave & 3, band = wave >> 2;
  if ((PT_PRIO & 2) && band == 1) __builtin_amdgcn_s_setprio(1);   // band 1's fill + conv: the critical path
  if (band == 1) {
    band_fill<BAND2_NT / 2>(a, tbl, tile1, cb, BAND_ROWS, tid - BAND2_NT / 2);
    if (tiled) band_halo<BAND2_NT / 2>(a, tbl, tile1, b, 1, tid - BAND2_NT / 2);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");     // this wave's tile stores are done
    if (lane == 0) atomicAdd(ready, 1);
    while (__hip_atomic_load(ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < 4)
      __builtin_amdgcn_s_sleep(1);
    PT_TRT(a, a.trace_kind, 3, BAND2_NT / 2);
    if constexpr ((PT_PRIO & 32) != 0) __builtin_amdgcn_s_setprio(0);   // band 1's conv: band 0 is critical
  }
  f32x16 acc[RW];
#pragma unroll
  for (int i = 0; i < RW; ++i) acc[i] = zero16();
  bf16x4 p0[RW][4], p1[RW][4];
  const int y0 = band * BAND_ROWS;
  const AddRowBand<RW> ar{(bf16_t*)a.out, (const bf16_t*)a.add0, (const bf16_t*)a.add1,
                          cb + ((size_t)(y0 + wb * RW) * IMG + px) * C, h, p0, p1};
  conv_run_nobar<S, RW, BAND2_NT>(acc, a.wf, band ? tile1 : tile0, a.K, wb * RW, lane, tid, a.ablate, ar);
  PT_TRW(a, a.trace_kind, 16);
}

template <class S>
__global__ __launch_bounds__(NT, 1) void k_bnbwd_fill(ConvArgs<S> a) {   // frame 0: BN bwd only
  extern __shared__ __attribute__((aligned(16))) char smem[];
  conv_body<S, FILL_BNBWD, EPI_NONE, PADMAX>(a, smem, blockIdx.x);
}

// =========================================================================
// Point-wise kernels: 4 waves per workgroup, each wave owns PW_RPP image rows
// (1 in k_pw_fa / k_pw_fb / k_pw_bb, 4 in k_pw_ba), several workgroups per CU:
// the long dependent element-wise / 1x1-gate chains and the workgroup barriers
// of one workgroup are hidden behind the others (the backward kernels need
// 256 VGPRs, i.e. 2 waves per SIMD: with 8-wave workgroups one workgroup
// filled a CU; 4-wave workgroups measured k_pw_bb 68.4 -> 66.0 us, k_pw_ba
// 57.7 -> 55.2 us).
// =========================================================================
constexpr int PW_NT = 256;
constexpr int PW_NW = PW_NT / 64;
constexpr int PWF_RPP = 1;                         // forward rows per wave
// k_pw_ba loops over 4 rows per wave: its fixed per-workgroup cost (slab
// prefetch / flush, x staging, LDS clears, reductions) is paid once per 16 rows.
// k_pw_bb stays at one row per wave: looping its body spills (~46 VGPRs) and
// doubled its row cost.
#ifndef PT_PWA_RPP
#define PT_PWA_RPP 4
#endif
constexpr int PWA_RPP = PT_PWA_RPP;                // k_pw_ba rows per wave
#ifndef PT_PWB_RPP
#define PT_PWB_RPP 1
#endif
constexpr int PWB_RPP = PT_PWB_RPP;                // k_pw_bb rows per wave (register bound)
constexpr int PWF_WGPC = IMG / (PW_NW * PWF_RPP);  // workgroups per clip (8)
constexpr int PWA_WGPC = IMG / (PW_NW * PWA_RPP);  // (2)
constexpr int PWB_WGPC = IMG / (PW_NW * PWB_RPP);  // (8)
constexpr int PW_PARTS = PWB_WGPC > PWA_WGPC ? PWB_WGPC : PWA_WGPC;   // slab partitions per clip
static_assert(PW_PARTS <= BNB_WG_PER_CLIP, "backward BN partial slots per clip");

constexpr int PW_NGACC = 4;   // 1x1 weight-gradient tiles accumulated in LDS per workgroup
template <int RPP, bool BWD>
constexpr int pw_lds_bytes() {   // forward point-wise kernels use xs, scr, stat only
  return !BWD
             ? PW_NW * RPP * IMG * 16 + PW_NW * SCR_FLOATS * 4 + 128 * 4
             : PW_NW * RPP * IMG * 16 /*xs*/ + PW_NW * SCR_FLOATS * 4 /*scr*/ + 128 * 4 /*stat*/ +
                   PW_NW * NSMALL * 32 * 4 /*small*/ + 512 * 4 /*red*/ +
                   PW_NGACC * 1024 * 4 /*gacc*/ + SLAB * 4 /*slab copy*/;
}
struct PLds {
  bf16x8* stage;  // k_pw_bb, bf16: [3 slots][PW_NW waves][2 k-steps][64 lanes] wgrad operands
  f32x4* xs;
  float* scr;     // [PW_NW][SCR_FLOATS]
  float* stat;    // [128]
  float* small;   // [PW_NW][NSMALL][32]
  float* red;     // [512]
  float* gacc;    // [PW_NGACC][1024]  (rows n, cols ci)
  float* flush;   // [PW_NW][SCR_FLOATS] per-wave weight-gradient tiles of one gate (aliases scr)
  float* slabl;   // [SLAB]            this workgroup's slab partition, prefetched
};
template <int RPP>
__device__ __forceinline__ PLds pcarve(char* smem) {
  PLds l;
  l.xs = (f32x4*)smem;
  l.scr = (float*)(smem + PW_NW * RPP * IMG * 16);
  l.stat = l.scr + PW_NW * SCR_FLOATS;
  l.small = l.stat + 128;
  l.red = l.small + PW_NW * NSMALL * 32;
  l.gacc = l.red + 512;
  l.flush = l.scr;       // gacc_row runs between a wave's transposes, fenced by barriers
  l.slabl = l.gacc + PW_NGACC * 1024;
  return l;
}

// k_pw_bb's layout.  bf16: the 1x1 weight gradients are formed by one wave
// per gate from operands the four waves stage in LDS (stage_wg / gate_wgrad
// below) instead of the per-row gacc reductions; the slab copy holds only the
// fields this kernel updates (gate tiles 2..5 and the per-channel block:
// slab offsets from 2 * 1024), slabl points 2048 floats before it.
constexpr int PWB_STAGE_SLOTS = 3;
constexpr int PWB_SLAB_LO = 2 * 1024;
template <class S>
constexpr int pwb_lds_bytes() {
  return PW_NW * PWB_RPP * IMG * 16 /*xs*/ + PW_NW * SCR_FLOATS * 4 /*scr*/ + 128 * 4 /*stat*/ +
         PW_NW * NSMALL * 32 * 4 /*small*/ + 512 * 4 /*red*/ +
         (sizeof(S) == 2 ? PWB_STAGE_SLOTS * PW_NW * 2 * 64 * 16 : PW_NGACC * 1024 * 4) +
         (SLAB - PWB_SLAB_LO) * 4 /*slab copy*/;
}
template <class S>
__device__ __forceinline__ PLds pcarve_bb(char* smem) {
  PLds l = pcarve<PWB_RPP>(smem);
  char* p = (char*)(l.red + 512);
  if constexpr (sizeof(S) == 2) {
    l.stage = (bf16x8*)p;
    l.gacc = nullptr;
    p += PWB_STAGE_SLOTS * PW_NW * 2 * 64 * 16;
  } else {
    l.stage = nullptr;
    l.gacc = (float*)p;
    p += PW_NGACC * 1024 * 4;
  }
  l.slabl = (float*)p - PWB_SLAB_LO;
  return l;
}
// PT_EI_FULL: the bf16 cell's kappa I + gamma (forward E update,
// k_pw_ba) and d att = dgE E_t (k_pw_ba) from the f32 values of I and E (both
// planes) instead of their hi planes; the gate operands stay the hi planes.
#ifndef PT_EI_FULL
#define PT_EI_FULL 0
#endif
// k_pw_ba's layout.  bf16 (r05): the a_w / a_u weight gradients are formed
// from operand tiles staged channel-major in LDS (CL rows -> [ch][128 px], the
// PR weight-gradient contraction of pt_pr.h) by one wave per (gate, output
// half) per set of 4 rows, accumulated in registers and added into the slab
// once at the end -- instead of two per-row cross-wave LDS reductions (4
// barriers a row) into a gacc tile; the slab copy holds only the per-channel
// block.  f32: pcarve (gacc).
// PT_PWA_PAIR (r06 A/B): the staged 1x1 weight-gradient operands of TWO
// row sets in LDS, contracted after every second row: one barrier pair per
// two rows instead of per row (the workgroup's 4 waves align less often)
#ifndef PT_PWA_PAIR
#define PT_PWA_PAIR 0
#endif
#ifndef PT_PWA_STAGE
#define PT_PWA_STAGE 1      // 0: the r04 per-row gacc reductions (A/B builds, tools/libab.py)
#endif
constexpr int PWA_NPX = PW_NW * IMG;            // pixels per set (one row per wave)
template <class S>
constexpr int pwa_lds_bytes() {
  return sizeof(S) == 2 && PT_PWA_STAGE
             ? PW_NW * PWA_RPP * IMG * 16 /*xs*/ + PW_NW * SCR_FLOATS * 4 /*scr*/ + 128 * 4 /*stat*/ +
                   PW_NW * NSMALL * 32 * 4 /*small*/ + 512 * 4 /*red*/ +
                   (PT_PWA_PAIR ? 6 : 3) * stg_bytes<S, PWA_NPX>() /*stage*/ +
                   NSMALL * 32 * 4 /*slab copy: per-channel block*/
             : pw_lds_bytes<PWA_RPP, true>();
}
template <class S>
__device__ __forceinline__ PLds pcarve_ba(char* smem) {
  PLds l = pcarve<PWA_RPP>(smem);
  if constexpr (sizeof(S) == 2 && PT_PWA_STAGE) {
    char* p = (char*)(l.red + 512);
    l.stage = (bf16x8*)p;
    l.gacc = nullptr;
    p += (PT_PWA_PAIR ? 6 : 3) * stg_bytes<S, PWA_NPX>();
    l.slabl = (float*)p - SLAB_G;
  }
  return l;
}
// A CL row tile (lane = channel c, half h; 16 pixels in 4 runs of 4) into a
// channel-major stage [ch][NPX + pad] at pixel offset px0, as bf16.
template <int NPX>
__device__ __forceinline__ void cl_stage(bf16_t* __restrict__ stg, const f32x16& v, int px0, int lane) {
  const int c = lane & 31, h = lane >> 5;
  bf16_t* row = stg + c * stg_stride<bf16_t, NPX>() + px0 + 4 * h;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    *(u32x2*)(row + 8 * k) = u32x2{pk_bf16(v[4 * k], v[4 * k + 1]), pk_bf16(v[4 * k + 2], v[4 * k + 3])};
}

// bf16 1x1 weight gradients without the per-row cross-wave reductions: every
// wave parks its row's operand tile (CL registers packed as the bf16 MFMA
// fragments of wgrad_cl) in a slot; after a barrier ONE wave contracts the
// four rows of its gate (8 MFMAs, k = 128 pixels) and adds the tile into the
// workgroup's slab (slabl holds the prefetched old values).
template <class V>
__device__ __forceinline__ void stage_wg(bf16x8* stage, int slot, const V& v, int wave, int lane) {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    bf16x8 f;
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = (bf16_t)(float)v[8 * s + j];
    stage[((slot * PW_NW + wave) * 2 + s) * 64 + lane] = f;
  }
}
__device__ __forceinline__ void gate_wgrad(const bf16x8* stage, int dslot, int xslot, int g,
                                           const float* slabl, float* slab_p, int lane) {
  // operands read one k-step ahead of their MFMA (a dependent LDS read per
  // MFMA exposed the LDS latency 8 times)
  constexpr int NK = PW_NW * 2;
  const bf16x8* dp = stage + dslot * NK * 64 + lane;
  const bf16x8* xp = stage + xslot * NK * 64 + lane;
  f32x16 acc = zero16();
  bf16x8 da = dp[0], xa = xp[0];
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    bf16x8 dn = da, xn = xa;
    if (k + 1 < NK) { dn = dp[(k + 1) * 64]; xn = xp[(k + 1) * 64]; }
    acc = Tr<bf16_t>::mma(da, xa, acc);
    da = dn; xa = xn;
  }
  // one base per lane + compile-time offsets (cl_x(r, h) = cl_x(r, 0) + 4 h)
  const int ci = lane & 31, h = lane >> 5;
  const int o = g * 1024 + 4 * h * 32 + ci;
  float* sp = slab_p + o;
  const float* sl = slabl + o;
#pragma unroll
  for (int r = 0; r < 16; ++r) sp[cl_x(r, 0) * 32] = sl[cl_x(r, 0) * 32] + acc[r];
}

// Add one row's 1x1 weight-gradient tile (dW[n][ci] = sum_p D[p][n] X[p][ci],
// one MFMA pair from CL registers) into the workgroup accumulator: every wave
// parks its tile in its own flush slot, then each thread sums its elements
// over the waves (plain stores, no atomics; all waves call this uniformly).
template <class S, class V>
__device__ __forceinline__ void gacc_row(float* gacc_g, float* flush, const f32x16& d,
                                         const V& x, int lane, int wave, int tid) {
  const f32x16 t = wgrad_cl<S>(d, x, zero16());
#if PT_WG_NOP
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 7\n s_nop 7\n s_nop 7" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
#endif
  const int ci = lane & 31, h = lane >> 5;
#pragma unroll
  for (int r = 0; r < 16; ++r) flush[wave * SCR_FLOATS + cl_x(r, h) * 32 + ci] = t[r];
  __syncthreads();
  for (int e = tid; e < 1024; e += PW_NT) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < PW_NW; ++w) s += flush[w * SCR_FLOATS + e];
    gacc_g[e] += s;
  }
  __syncthreads();
}
__device__ void gacc_zero(float* g, int n, int tid) {
  for (int e = tid; e < n * 1024; e += PW_NT) g[e] = 0.f;
}
// The workgroup's slab fields are copied into LDS by LDS-DMA at kernel start
// (their latency hides under the staging loads); the flushes at the end then
// store old + new without waiting on a global read-modify-write.  Only the
// fields this kernel updates are fetched: gate-weight tiles [g0, g0 + ng) and
// the per-channel block.
__device__ __forceinline__ void slab_range(const float* slab_p, float* slabl, int f0, int nf,
                                           int wave, int lane) {
  const int nchunk = nf / 4;                             // 16-B chunks
  for (int j = wave; j * 64 < nchunk; j += PW_NW)
    if (j * 64 + lane < nchunk) {
#if PT_SLAB_DMA
      __builtin_amdgcn_global_load_lds((const void*)(slab_p + f0 + (j * 64 + lane) * 4),
                                       (__attribute__((address_space(3))) void*)(slabl + f0 + j * 256),
                                       16, 0, 0);
#else
      *(f32x4*)(slabl + f0 + (j * 64 + lane) * 4) = *(const f32x4*)(slab_p + f0 + (j * 64 + lane) * 4);
#endif
    }
#if PT_SLAB_WAIT
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
}
__device__ __forceinline__ void slab_prefetch(const float* slab_p, float* slabl, int g0, int ng,
                                              int wave, int lane) {
  slab_range(slab_p, slabl, g0 * 1024, ng * 1024, wave, lane);
  slab_range(slab_p, slabl, SLAB_G, NSMALL * 32, wave, lane);
}
// slab[g0 + k] = slab copy + gacc[k] for k < n (after a barrier)
__device__ void gacc_flush(const float* g, const float* slabl, float* slab_p, int g0, int n, int tid) {
  for (int e = tid; e < n * 1024; e += PW_NT) {
    const int o = (g0 + e / 1024) * 1024 + e % 1024;
    slab_p[o] = slabl[o] + g[e];
  }
}

// Workgroup sum of per-lane channel values -> slab (this workgroup's
// partition only: no atomics).
template <int N>
__device__ void flush_small(float (&v)[N], const int (&slot)[N], float* small, const float* slabl,
                            float* slab_p, int lane, int wave, int tid) {
#pragma unroll
  for (int k = 0; k < N; ++k) {
    const float s = v[k] + __shfl_xor(v[k], 32);
    if (lane < 32) small[(wave * N + k) * 32 + lane] = s;
  }
  __syncthreads();
  for (int e = tid; e < N * 32; e += PW_NT) {
    const int k = e >> 5, c = e & 31;
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < PW_NW; ++w) s += small[(w * N + k) * 32 + c];
    const int o = SLAB_G + slot[k] * 32 + c;
    slab_p[o] = slabl[o] + s;
  }
  __syncthreads();
}

// Workgroup totals of two per-lane channel sums -> the deterministic batch
// reduction (bn_publish).  red: 512 floats (reused as the group-sum scratch);
// flag: an LDS word outside red.
// The caller completes the protocol (bn_publish_finish with the returned value)
// after its slab flush: the partial's store latency hides under the flush.
__device__ float bn_bwd_partial(float s0, float s1, float* red, const BnSlot& out, int lane,
                                int wave, int tid) {
  s0 += __shfl_xor(s0, 32);
  s1 += __shfl_xor(s1, 32);
  if (lane < 32) { red[wave * 32 + lane] = s0; red[256 + wave * 32 + lane] = s1; }
  __syncthreads();
  float a = 0.f;                        // lanes 0-31: sum dy; 32-63: sum dy * xhat
  if (tid < 64) {
    const int o = tid < 32 ? tid : 256 + tid - 32;
#pragma unroll
    for (int w = 0; w < PW_NW; ++w) a += red[o + w * 32];
  }
  bn_publish_store<PW_NT, false>(out, blockIdx.x, a, tid);
  return a;
}

// -------------------------------------------------------------------------
// Forward point-wise A (frame t, 0 <= t <= T):
//   t > 0 : close frame t-1: E_{t-1} = (1-eg) E_{t-2} + eg nl(BN1(ce) (kappa I_{t-1} + gamma))
//           (models/InT.py:172-175)
//   t < T : att = sig(a_w x_t + a_u E_{t-1}) (:148), gE = att*E_{t-1} (:153),
//           eg = sig(e_w I_{t-1} + e_u gE) (:171, uses the OLD inhibition;
//           no_inh: e_w E_{t-1}, :168)
// -------------------------------------------------------------------------
template <class S> struct FaIn { Pk<S> egv, cev; f32x16 Iv, Eo; };
template <class S>
__device__ __forceinline__ FaIn<S> fa_load(const CellArgs<S>& a, int t, size_t ro, int c, int h) {
  const size_t fs = fr_off(1, a.B);
  FaIn<S> w;
  w.Iv = zero16(); w.Eo = zero16(); w.egv = zero_pk<S>(); w.cev = zero_pk<S>();
  if (t > 0) {
    // I_{t-1} feeds kappa I + gamma and the e_w gate operand: the bf16 cell
    // reads its hi plane only (r05; PT_EI_FULL: both planes, the
    // f32 value in kappa I + gamma, its hi rounding as the operand); E_{t-2}
    // feeds the E update and is read in full precision
    w.Iv = PT_EI_FULL ? ldI(a, t - 1, ro, c, h) : ldIh(a, t - 1, ro, c, h);
    if (t >= 2) w.Eo = ldE(a, t - 2, ro, c, h);
    w.egv = load_pk(a.eg + (t - 1) * fs + ro, c, h);
    w.cev = load_pk(a.ce + (t - 1) * fs + ro, c, h);
  }
  return w;
}

// One image row of forward point-wise A (x of the row staged in xs, BN1 stats
// of frame t-1 in stat[64..127]).
// tile: the fused kernel's conv tile (bf16, 32x32 frames): gE_t of the row is
// also written into its interior, rounded as the store rounds it.
template <class S>
__device__ __forceinline__ void tile_put_cl(S* tile, int y, int c, int h, const f32x16& v) {
#pragma unroll
  for (int r = 0; r < 16; ++r) tile[tile_off<S, PADMAX>(y + PADMAX, cl_x(r, h) + PADMAX, c)] = (S)v[r];
}

template <class S, int ACT, int HG>
__device__ __forceinline__ void fa_row(const CellArgs<S>& a, int t, const float* stat, const f32x4* xs,
                                       int yl, float* wscr, int b, int y, size_t ro,
                                       const FaIn<S>& in, int lane, S* tile = nullptr) {
  using F = typename Tr<S>::frag;
  const int c = lane & 31, h = lane >> 5;
  const int T = a.T;
  const size_t fs = fr_off(1, a.B);
  const Stem st{a.wpre[c * 3 + 0], a.wpre[c * 3 + 1], a.wpre[c * 3 + 2], a.bpre[c]};
  const float kap = a.kappa[c], gam = a.gamma[c], bw1 = a.bnw1[c], bb1 = a.bnb1[c];
  const float m1 = stat[64 + c], rs1 = stat[96 + c];
  const float nba = sig_nb(a.gb[0][c] + a.gb[1][c]), nbe = sig_nb(a.gb[4][c] + a.gb[5][c]);

  // close frame t-1 (:172-175)
  f32x16 Ep = zero16(), Eop = zero16();   // Eop: E_{t-1} as the gates' bf16 operand (= its hi plane)
  if (t > 0) {
    const float A1 = bw1 * rs1, B1 = bb1 - bw1 * rs1 * m1;     // BN1 affine folded
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float cn = A1 * (float)in.cev[r] + B1;
      const float eh = Act<ACT>::f(cn * (kap * (float)in.Iv[r] + gam));
      const float e = (float)in.egv[r];
      Ep[r] = (1.f - e) * in.Eo[r] + e * eh;
    }
    if (sizeof(S) == 4 && (PT_ABL(a.ablate) & 2048))
#pragma unroll
      for (int r = 0; r < 16; ++r) Ep[r] = (float)(bf16_t)Ep[r];
    Eop = stE(a, t - 1, ro, c, h, Ep);
  }
  if (t == T) return;
  f32x16 z, xv;
  stem_cl<ACT>(xs, yl, h, st, z, xv);
  F pax[Tr<S>::KS], pae[Tr<S>::KS];
  cl_to_pa<S>(wscr, xv, lane, pax, RND_G(a));
  cl_to_pa<S>(wscr, Eop, lane, pae, RND_G(a));
  f32x16 acc = zero16();
  acc = gemm_pa<S>(pax, a.gf[0], acc, lane);
  acc = gemm_pa<S>(pae, a.gf[1], acc, lane);
  f32x16 att, gEv;
#pragma unroll
  for (int r = 0; r < 16; ++r) { att[r] = sigm_b(acc[r], nba); gEv[r] = att[r] * Ep[r]; }
  if (sizeof(S) == 4 && (PT_ABL(a.ablate) & 8192))
#pragma unroll
    for (int r = 0; r < 16; ++r) gEv[r] = (float)(bf16_t)gEv[r];
  store_cl(a.gE + t * fs + ro, c, h, gEv);
  if (tile) tile_put_cl(tile, y, c, h, gEv);
  if (a.gates && c < a.Cu) {
    const TileLoc tl = tile_loc(b, a.ntx, a.nty);
    const int W = a.ntx * IMG;
    float* gp = a.gates + (((size_t)tl.b * T + t) * a.Cu + c) * ((size_t)a.nty * IMG * W) +
                (size_t)(tl.ty * IMG + y) * W + tl.tx * IMG;
#pragma unroll
    for (int r = 0; r < 16; ++r) gp[cl_x(r, h)] = att[r];
  }
  F pag[Tr<S>::KS], pai[Tr<S>::KS];
  cl_to_pa<S>(wscr, gEv, lane, pag, RND_G(a));
  if constexpr (HG) {          // g_inh = att (ffhgru_hierarchy.py:147, :154)
    store_cl(a.at + t * fs + ro, c, h, att);
    cl_to_pa<S>(wscr, att, lane, pai, RND_G(a));
  } else if (a.no_inh) {
    cl_to_pa<S>(wscr, Eop, lane, pai, RND_G(a));
  } else {
    if constexpr (PT_EI_FULL) cl_to_pa<S>(wscr, op_round<S>(in.Iv), lane, pai, RND_G(a));
    else cl_to_pa<S>(wscr, in.Iv, lane, pai, RND_G(a));
  }
  acc = zero16();
  acc = gemm_pa<S>(pai, a.gf[4], acc, lane);
  acc = gemm_pa<S>(pag, a.gf[5], acc, lane);
  f32x16 egn;
#pragma unroll
  for (int r = 0; r < 16; ++r) egn[r] = sigm_b(acc[r], nbe);
  if (sizeof(S) == 4 && (PT_ABL(a.ablate) & 8192))
#pragma unroll
    for (int r = 0; r < 16; ++r) egn[r] = (float)(bf16_t)egn[r];
  store_cl(a.eg + t * fs + ro, c, h, egn);
}

template <class S, int ACT, int HG>
__global__ __launch_bounds__(PW_NT, 4) void k_pw_fa(CellArgs<S> a) {
  static_assert(PWF_RPP == 1, "forward point-wise kernels: one row per wave");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if (PT_ABL(a.ablate) & 512) return;
  const PLds L = pcarve<PWF_RPP>(smem);
  const int tid = threadIdx.x, lane = tid & 63, c = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int b, part;
  wg_split(blockIdx.x, PWF_WGPC, a.B, a.xmap, b, part);
  const int t = a.t, T = a.T, B = a.B;
  const int y0 = part * PW_NW;
  const int yl = wave, y = y0 + yl;
  const size_t ro = clip_off(b) + (size_t)y * IMG * C;
  // The BN1 finalisation is wave PW_NW-1's first work: loads complete in
  // order per wave, so behind its own row tiles it would wait for all of them
  // (and the barrier below for it); the other waves' row tiles go out first.
  const bool finw = wave == PW_NW - 1;
  if (finw && t > 0 && !(PT_ABL(a.ablate) & 65536))
    bn_fwd_finalize(bnf_src(a, t - 1, 1), bnf_nsrc(a), B * a.bn_world, a.eps, L.stat + 64,
                    blockIdx.x == 0 ? a.bnstat + (size_t)(t - 1) * 128 + 64 : nullptr, lane);
  const FaIn<S> in = fa_load(a, t, ro, c, h);
  if (t < T && !(PT_ABL(a.ablate) & 131072)) stage_x(a.x, a.xu8, L.xs, b, t, T, y0, PW_NW, tid, PW_NT, a.ntx, a.nty);
  __syncthreads();
  if (PT_ABL(a.ablate) & 4) return;
  fa_row<S, ACT, HG>(a, t, L.stat, L.xs, yl, L.scr + wave * SCR_FLOATS, b, y, ro, in, lane);
}

// -------------------------------------------------------------------------
// Forward point-wise B (frame t): BN0 -> Ihat = nl(x - nl(c_i (alpha I + mu)))
//   (:162), ig = sig(i_w x + i_u I) (:165), I_t = (1-ig) I + ig Ihat (:166)
//   [no_inh: I_t = gE (:168)]
// -------------------------------------------------------------------------
template <class S> struct FbIn { Pk<S> civ, gi; f32x16 Iv; };
template <class S, int HG>
__device__ __forceinline__ FbIn<S> fb_load(const CellArgs<S>& a, int t, size_t ro, int c, int h) {
  const size_t fs = fr_off(1, a.B);
  FbIn<S> w;
  w.civ = load_pk(a.ci + t * fs + ro, c, h);
  w.Iv = t > 0 ? ldI(a, t - 1, ro, c, h) : zero16();     // full precision: the I update
  if constexpr (HG) w.gi = load_pk(a.at + t * fs + ro, c, h);   // gated inhibition att_t
  else w.gi = zero_pk<S>();                                     // InT: I_{t-1} (Iv, f32)
  return w;
}

// One image row of forward point-wise B (BN0 stats of frame t in stat[0..63]).
template <class S, int ACT, int HG>
__device__ __forceinline__ void fb_row(const CellArgs<S>& a, int t, const float* stat, const f32x4* xs,
                                       int yl, float* wscr, int y, size_t ro, const FbIn<S>& in,
                                       int lane, S* tile = nullptr) {
  using F = typename Tr<S>::frag;
  const int c = lane & 31, h = lane >> 5;
  const size_t fs = fr_off(1, a.B);
  const Stem st{a.wpre[c * 3 + 0], a.wpre[c * 3 + 1], a.wpre[c * 3 + 2], a.bpre[c]};
  const float al = a.alpha[c], mu = a.mu[c], bw0 = a.bnw0[c], bb0 = a.bnb0[c];
  const float m0 = stat[c], rs0 = stat[32 + c];
  const float A0 = bw0 * rs0, B0 = bb0 - bw0 * rs0 * m0;     // BN0 affine folded
  const float nbi = sig_nb(a.gb[2][c] + a.gb[3][c]);

  f32x16 z, xv, ih;
  stem_cl<ACT>(xs, yl, h, st, z, xv);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const float cn = A0 * (float)in.civ[r] + B0;
    const float gv = HG ? (float)in.gi[r] : in.Iv[r];
    ih[r] = Act<ACT>::f(xv[r] - Act<ACT>::f(cn * (al * gv + mu)));
  }
  F pax[Tr<S>::KS], pai[Tr<S>::KS];
  cl_to_pa<S>(wscr, xv, lane, pax, RND_G(a));
  if constexpr (HG) cl_to_pa<S>(wscr, in.gi, lane, pai, RND_G(a));
  else cl_to_pa<S>(wscr, in.Iv, lane, pai, RND_G(a));
  f32x16 acc = zero16();
  acc = gemm_pa<S>(pax, a.gf[2], acc, lane);
  acc = gemm_pa<S>(pai, a.gf[3], acc, lane);
  f32x16 In;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const float ig = sigm_b(acc[r], nbi);
    In[r] = (1.f - ig) * in.Iv[r] + ig * ih[r];
  }
  if (sizeof(S) == 4 && (PT_ABL(a.ablate) & 4096))
#pragma unroll
    for (int r = 0; r < 16; ++r) In[r] = (float)(bf16_t)In[r];
  const f32x16 Ih = stI(a, t, ro, c, h, In);   // bf16: the hi plane is Ic, the exc conv's input
  if (tile) tile_put_cl(tile, y, c, h, Ih);
}

template <class S, int ACT, int HG>
__global__ __launch_bounds__(PW_NT, 4) void k_pw_fb(CellArgs<S> a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if (PT_ABL(a.ablate) & 512) return;
  const PLds L = pcarve<PWF_RPP>(smem);
  const int tid = threadIdx.x, lane = tid & 63, c = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int b, part;
  wg_split(blockIdx.x, PWF_WGPC, a.B, a.xmap, b, part);
  const int t = a.t, T = a.T, B = a.B;
  const int y0 = part * PW_NW;
  const int yl = wave, y = y0 + yl;
  const size_t fs = fr_off(1, B), ro = clip_off(b) + (size_t)y * IMG * C;

  if (a.no_inh) {      // I_t = gE_t (:168)
    if (!(PT_ABL(a.ablate) & 4)) {
      const Pk<S> g = load_pk(a.gE + t * fs + ro, c, h);
      f32x16 v;
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = (float)g[r];
      stI(a, t, ro, c, h, v);
    }
    return;
  }
  const FbIn<S> in = fb_load<S, HG>(a, t, ro, c, h);
  stage_x(a.x, a.xu8, L.xs, b, t, T, y0, PW_NW, tid, PW_NT, a.ntx, a.nty);
  // (finalising first in a separate wave, as k_pw_fa does, measured no gain here)
  bn_fwd_finalize(bnf_src(a, t, 0), bnf_nsrc(a), B * a.bn_world, a.eps, L.stat,
                  blockIdx.x == 0 ? a.bnstat + (size_t)t * 128 : nullptr, tid);
  __syncthreads();
  if (PT_ABL(a.ablate) & 4) return;
  fb_row<S, ACT, HG>(a, t, L.stat, L.xs, yl, L.scr + wave * SCR_FLOATS, y, ro, in, lane);
}


// =========================================================================
// Fused forward segments (bf16, 32x32 frames, k <= 7): ONE workgroup per clip
// (8 waves, 4 rows each) runs the point-wise step of all 32 rows and writes
// the conv input straight into the LDS tile, then the k x k conv and its BN
// partials -- one launch per BatchNorm segment instead of two, and the conv
// never re-reads its input from HBM (the input is still stored: the backward
// needs it).  Arithmetic identical to k_pw_fa / k_pw_fb + k_conv_fwd: the
// tile holds the same bf16-rounded values the split conv would load.
//   k_fused_fa(t): fa_row (close E_{t-1}; att, gE_t, eg_t) -> conv(gE_t, w_inh)
//   k_fused_fb(t): fb_row (BN0, I_t)                        -> conv(I_t, w_exc)
// LDS: conv tile | red | x of the clip frame | per-wave transpose scratch | stat
// (the conv's B fragments come from L2 into registers: no weight slices).
// =========================================================================
constexpr int FUSED_NW = CONV_NT / 64, FUSED_RW = IMG / FUSED_NW;
template <class S> constexpr int fused_lds_bytes() {
  return tile_bytes<S, PADMAX>() + CONV_MISC * 4 + NPIX * 16 + FUSED_NW * SCR_FLOATS * 4 + 128 * 4 + 8 * 4;
}
struct FusedLds { char* tile; float* red; f32x4* xs; float* scr; float* stat; int* cnt; };
template <class S>
__device__ __forceinline__ FusedLds fused_carve(char* smem) {
  FusedLds l;
  l.tile = smem;
  l.red = (float*)(smem + tile_bytes<S, PADMAX>());
  l.xs = (f32x4*)(l.red + CONV_MISC);
  l.scr = (float*)(l.xs + NPIX);
  l.stat = l.scr + FUSED_NW * SCR_FLOATS;
  l.cnt = (int*)(l.stat + 128);             // the staggered segments' row counters
  return l;
}

// The conv half: conv(tile, wf) for this wave's rows, rows stored as they
// finish (out_raw), then the per-clip BN partials (bnout).
template <class S, bool NOBAR = false, bool XB = false>
__device__ __forceinline__ void fused_conv(const CellArgs<S>& a, const ConvArgs<S>& c, S* out_raw,
                                           const BnSlot& bnout, char* smem, const FusedLds& L, int b,
                                           int wave, int lane, int tid, int kind, unsigned* xflags = nullptr) {
  constexpr int RW = FUSED_RW;
  f32x16 acc[RW];
#pragma unroll
  for (int i = 0; i < RW; ++i) acc[i] = zero16();
  const int h = lane >> 5, px = lane & 31;
  const StoreRow<S> sr{out_raw + clip_off(b) + ((size_t)(wave * RW) * IMG + px) * C, h, false};
  // the point-wise half filled the tile's interior; tiled frames: the halo
  // from the neighbouring tiles' workgroups (xb_exchange), between the
  // conv's two barriers
  auto fill = [&](int) {
    if constexpr (XB && sizeof(S) == 2) xb_exchange<S, CONV_NT>(a, (S*)L.tile, xflags, b, a.t, tid);
  };
  if constexpr (NOBAR)                      // (the caller waited for this wave's input rows)
    conv_run_nobar<S, RW, CONV_NT>(acc, c.wf, (S*)L.tile, a.K, wave * RW, lane, tid, PT_ABL(a.ablate) & 1, sr);
  else
    conv_run<S, PADMAX, RW, CONV_NT>(acc, fill, c.wf, (S*)L.tile, nullptr, a.K, wave * RW, lane,
                                     tid, PT_ABL(a.ablate) & 1, sr);
  PT_TR(a, kind, 4);
  PT_TRW(a, kind, 16);
  if (PT_ABL(a.ablate) & 8) return;
  bn_block_stats<RW, FUSED_NW>(acc, L.red, wave, lane);       // = bn_fwd_partial, stamped
  __syncthreads();
  PT_TR(a, kind, 5);
  bn_blocks_publish<RW, FUSED_NW>(L.red, bnout, b, tid, (int*)(smem + CONV_NT * 16), (double*)smem);
}

// Staggered fused segments (r05, PT_FUSED_STAG, bf16 k <= 7): waves 0-3 (band
// 0, conv output rows 0-15) run 3 point-wise rows each (rows 0-11), waves 4-7
// run 5 (rows 12-31, round r of wave 4 + j is row 12 + 4 r + j), so band 0's
// conv input (rows 0-18) is complete after waves 4-7's second round and waves
// 0-3 start their conv while waves 4-7 are still in their point-wise rows;
// waves 4-7 convolve once their own rows are done (band 1 needs rows 13-31
// only).  LDS counters replace the workgroup barrier between the halves.  Per
// row and per output row the arithmetic and the MFMA order are unchanged:
// bitwise the unstaggered segment.
#ifndef PT_FUSED_STAG
#define PT_FUSED_STAG 3     // bit 0: k_fused_fb, bit 1: k_fused_fa
#endif
// RA point-wise rows per band-0 wave (rows 0 .. 4 RA - 1), 8 - RA per band-1
// wave (round r of wave 4 + j: row 4 RA + 4 r + j)
template <int RA> __device__ __forceinline__ int stag_rows(int wave) { return wave < 4 ? RA : 8 - RA; }
template <int RA> __device__ __forceinline__ int stag_row(int wave, int i) {
  return wave < 4 ? wave * RA + i : 4 * RA + 4 * i + (wave - 4);
}
// after row i of this wave is in the tile: count it (cnt[0]: band-0 waves'
// rows, cnt[1 + i]: round i of the band-1 waves)
__device__ __forceinline__ void stag_done(int* cnt, int wave, int i, int lane) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (lane == 0) atomicAdd(wave < 4 ? cnt : cnt + 1 + i, 1);
}
template <int RA>
__device__ __forceinline__ void stag_wait(const int* cnt, int wave) {
  auto ld = [&](int k) { return __hip_atomic_load(cnt + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); };
  constexpr int RB = 8 - RA;
  // band 0 needs image rows 0-18: every band-0 row and the band-1 rounds up
  // to the one holding row 18; band 1 needs rows 13-31: every band-1 round
  // and, when band-0 waves own any of rows 13-15, theirs
  constexpr int R0 = (18 - 4 * RA) / 4;     // last band-1 round band 0 needs (RA <= 4)
  if (wave < 4) {
    while (ld(0) < 4 * RA || ld(1 + R0) < 4) __builtin_amdgcn_s_sleep(1);
  } else {
    while (ld(RB) < 4 || (4 * RA > 13 && ld(0) < 4 * RA)) __builtin_amdgcn_s_sleep(1);
  }
  asm volatile("" ::: "memory");
}
// r06: the persistent forward (k_persist_fwd, COH) on the staggered segments
// too (N2 re-measured on the r05 segments)
#ifndef PT_PERSIST_STAG
#define PT_PERSIST_STAG 1
#endif
// r06: 3 (band 0 three rows per wave, band 1 five) with the band-1 waves at
// issue priority 1 (PT_PRIO bit 0): k_fused_fa 64.8 -> 62.0 us; 4 / 4 with
// the priority 66.6, 2 / 6 65.3, 5 / 3 67.6 (profiles/r06_libab_prio_*.txt)
#ifndef PT_FUSED_STAG_RA_FA
#define PT_FUSED_STAG_RA_FA 3
#endif
#ifndef PT_FUSED_STAG_RA_FB
#define PT_FUSED_STAG_RA_FB 3
#endif

template <class S, int ACT, int HG, bool COH, bool TL = false>
__device__ __forceinline__ void fused_fa_body(const CellArgs<S>& a, const ConvArgs<S>& c, int t, S* out_raw,
                                              const BnSlot& bnout, char* smem, int tid,
                                              const unsigned* wcnt = nullptr, unsigned wtarget = 0,
                                              unsigned* err = nullptr) {
  const FusedLds L = fused_carve<S>(smem);
  const int lane = tid & 63, cl = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int b = blockIdx.x;
  PT_TR(a, PT_K_FUSED_FA, 0);
  if constexpr (COH) __syncthreads();      // the previous segment's LDS use is over
  // persistent: only the finalising wave waits for the batch sums (COH); the
  // others' row loads and the x staging below go out meanwhile
  if (COH && wave == FUSED_NW - 1 && t > 0) wave_wait(wcnt, wtarget, err, lane);
  if (!(PT_ABL(a.ablate) & 65536) && wave == FUSED_NW - 1 && t > 0)
    bn_fwd_finalize<COH>(bnf_src(a, t - 1, 1), bnf_nsrc(a), a.B * a.bn_world, a.eps, L.stat + 64,
                         b == 0 ? a.bnstat + (size_t)(t - 1) * 128 + 64 : nullptr, lane);
  // this wave's first row's tiles go out before the staging and the barrier
  // (fa with 3 / 5 rows: 64.1 -> 64.6 us, its heavier rows do not hide under
  // the band-0 conv; with 4 / 4 -- each half convolves as soon as its rows
  // and the rows it borrows are in, no workgroup barrier -- 65.5 -> 64.2 us;
  // fb 3 / 5: 55.4 -> 52.4 us, 4 / 4: 54.6: profiles/r05_libab_fused_stag*.txt)
  constexpr bool STAG = (PT_FUSED_STAG & 2) && (!COH || PT_PERSIST_STAG) && sizeof(S) == 2;
  // tiled frames (r06, TL): the unstaggered rows, then the border exchange
  // (xb_exchange); separate instantiations, so the 32x32 kernels keep their
  // registers (the exchange beside the staggered form spilled)
  static_assert(!(TL && COH), "the persistent forward runs single-tile frames");
  constexpr bool stag = STAG && !TL;
  FaIn<S> nxt = fa_load(a, t, clip_off(b) + (size_t)(stag ? stag_row<PT_FUSED_STAG_RA_FA>(wave, 0) : wave * FUSED_RW) * IMG * C, cl, h);
  tile_zero_halo<S, PADMAX, CONV_NT>((S*)L.tile, tid);   // rows fill the interior
  // (r05) the finalising wave 7 stages no x: its BN loads and the others' x
  // loads are one HBM round trip each, side by side
  if (!(PT_ABL(a.ablate) & 131072) && (COH || wave < FUSED_NW - 1))
    stage_x(a.x, a.xu8, L.xs, b, t, a.T, 0, IMG, tid, COH ? CONV_NT : CONV_NT - 64, TL ? a.ntx : 1, TL ? a.nty : 1);
  if constexpr (stag) {
    int* cnt = L.cnt;
    if (tid < 8) cnt[tid] = 0;
    __syncthreads();
    PT_TR(a, PT_K_FUSED_FA, 2);
    const int nr = stag_rows<PT_FUSED_STAG_RA_FA>(wave);
    if ((PT_PRIO & 1) && wave >= 4) __builtin_amdgcn_s_setprio(1);   // band 1: the critical path
#pragma unroll 1
    for (int i = 0; i < nr; ++i) {
      const int y = stag_row<PT_FUSED_STAG_RA_FA>(wave, i);
      const size_t ro = clip_off(b) + (size_t)y * IMG * C;
      const FaIn<S> cur = nxt;
      if (i + 1 < nr) nxt = fa_load(a, t, clip_off(b) + (size_t)stag_row<PT_FUSED_STAG_RA_FA>(wave, i + 1) * IMG * C, cl, h);
      if (!(PT_ABL(a.ablate) & 4))
        fa_row<S, ACT, HG>(a, t, L.stat, L.xs, y, L.scr + wave * SCR_FLOATS, b, y, ro, cur, lane,
                           (S*)L.tile);
      stag_done(cnt, wave, i, lane);
    }
    PT_TRW(a, PT_K_FUSED_FA, 8);
    stag_wait<PT_FUSED_STAG_RA_FA>(cnt, wave);
    PT_TR(a, PT_K_FUSED_FA, 3);
    fused_conv<S, true>(a, c, out_raw, bnout, smem, L, b, wave, lane, tid, PT_K_FUSED_FA);
    PT_TR(a, PT_K_FUSED_FA, 6);
    return;
  }
  __syncthreads();
  PT_TR(a, PT_K_FUSED_FA, 2);
#pragma unroll 1
  for (int i = 0; i < FUSED_RW; ++i) {
    const int y = wave * FUSED_RW + i;
    const size_t ro = clip_off(b) + (size_t)y * IMG * C;
    const FaIn<S> cur = nxt;
    if (i + 1 < FUSED_RW) nxt = fa_load(a, t, ro + (size_t)IMG * C, cl, h);   // next row in flight
    if (!(PT_ABL(a.ablate) & 4))
      fa_row<S, ACT, HG>(a, t, L.stat, L.xs, y, L.scr + wave * SCR_FLOATS, b, y, ro, cur, lane,
                         (S*)L.tile);
  }
  PT_TR(a, PT_K_FUSED_FA, 3);
  fused_conv<S, false, TL>(a, c, out_raw, bnout, smem, L, b, wave, lane, tid, PT_K_FUSED_FA, a.xflag);
  PT_TR(a, PT_K_FUSED_FA, 6);
}

template <class S, int ACT, int HG, bool COH, bool TL = false>
__device__ __forceinline__ void fused_fb_body(const CellArgs<S>& a, const ConvArgs<S>& c, int t, S* out_raw,
                                              const BnSlot& bnout, char* smem, int tid,
                                              const unsigned* wcnt = nullptr, unsigned wtarget = 0,
                                              unsigned* err = nullptr) {
  const FusedLds L = fused_carve<S>(smem);
  const int lane = tid & 63, cl = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int b = blockIdx.x;
  PT_TR(a, PT_K_FUSED_FB, 0);
  if constexpr (COH) __syncthreads();
  if (COH && wave == FUSED_NW - 1) wave_wait(wcnt, wtarget, err, lane);
  if (!(PT_ABL(a.ablate) & 65536) && wave == FUSED_NW - 1)
    bn_fwd_finalize<COH>(bnf_src(a, t, 0), bnf_nsrc(a), a.B * a.bn_world, a.eps, L.stat,
                         b == 0 ? a.bnstat + (size_t)t * 128 : nullptr, lane);
  constexpr bool STAG = (PT_FUSED_STAG & 1) && (!COH || PT_PERSIST_STAG) && sizeof(S) == 2;   // (bf16: the barrier-free conv form)
  static_assert(!(TL && COH), "the persistent forward runs single-tile frames");
  constexpr bool stag = STAG && !TL;
  FbIn<S> nxt = fb_load<S, HG>(a, t, clip_off(b) + (size_t)(stag ? stag_row<PT_FUSED_STAG_RA_FB>(wave, 0) : wave * FUSED_RW) * IMG * C, cl, h);
  tile_zero_halo<S, PADMAX, CONV_NT>((S*)L.tile, tid);   // rows fill the interior
  // (r05) the finalising wave 7 stages no x: its BN loads and the others' x
  // loads are one HBM round trip each, side by side
  if (!(PT_ABL(a.ablate) & 131072) && (COH || wave < FUSED_NW - 1))
    stage_x(a.x, a.xu8, L.xs, b, t, a.T, 0, IMG, tid, COH ? CONV_NT : CONV_NT - 64, TL ? a.ntx : 1, TL ? a.nty : 1);
  if constexpr (stag) {
    int* cnt = L.cnt;
    if (tid < 8) cnt[tid] = 0;
    __syncthreads();
    PT_TR(a, PT_K_FUSED_FB, 2);
    const int nr = stag_rows<PT_FUSED_STAG_RA_FB>(wave);
    if ((PT_PRIO & 1) && wave >= 4) __builtin_amdgcn_s_setprio(1);   // band 1: the critical path
#pragma unroll 1
    for (int i = 0; i < nr; ++i) {
      const int y = stag_row<PT_FUSED_STAG_RA_FB>(wave, i);
      const size_t ro = clip_off(b) + (size_t)y * IMG * C;
      const FbIn<S> cur = nxt;
      if (i + 1 < nr) nxt = fb_load<S, HG>(a, t, clip_off(b) + (size_t)stag_row<PT_FUSED_STAG_RA_FB>(wave, i + 1) * IMG * C, cl, h);
      if (!(PT_ABL(a.ablate) & 4))
        fb_row<S, ACT, HG>(a, t, L.stat, L.xs, y, L.scr + wave * SCR_FLOATS, y, ro, cur, lane,
                           (S*)L.tile);
      stag_done(cnt, wave, i, lane);
    }
    PT_TRW(a, PT_K_FUSED_FB, 8);
    stag_wait<PT_FUSED_STAG_RA_FB>(cnt, wave);
    if constexpr ((PT_PRIO & 16) != 0) {   // fb: band 0's conv is the critical path once band 1's rows are done
      if (wave >= 4) __builtin_amdgcn_s_setprio(0);
      else __builtin_amdgcn_s_setprio(1);
    }
    PT_TR(a, PT_K_FUSED_FB, 3);
    fused_conv<S, true>(a, c, out_raw, bnout, smem, L, b, wave, lane, tid, PT_K_FUSED_FB);
    PT_TR(a, PT_K_FUSED_FB, 6);
    return;
  }
  __syncthreads();
  PT_TR(a, PT_K_FUSED_FB, 2);
#pragma unroll 1
  for (int i = 0; i < FUSED_RW; ++i) {
    const int y = wave * FUSED_RW + i;
    const size_t ro = clip_off(b) + (size_t)y * IMG * C;
    const FbIn<S> cur = nxt;
    if (i + 1 < FUSED_RW) nxt = fb_load<S, HG>(a, t, ro + (size_t)IMG * C, cl, h);
    if (!(PT_ABL(a.ablate) & 4))
      fb_row<S, ACT, HG>(a, t, L.stat, L.xs, y, L.scr + wave * SCR_FLOATS, y, ro, cur, lane,
                         (S*)L.tile);
  }
  PT_TR(a, PT_K_FUSED_FB, 3);
  fused_conv<S, false, TL>(a, c, out_raw, bnout, smem, L, b, wave, lane, tid, PT_K_FUSED_FB,
                           a.xflag + a.B);
  PT_TR(a, PT_K_FUSED_FB, 6);
}

template <class S, int ACT, int HG, bool TL = false>
__global__ __launch_bounds__(CONV_NT, 1) void k_fused_fa(CellArgs<S> a, ConvArgs<S> c) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  fused_fa_body<S, ACT, HG, false, TL>(a, c, a.t, c.out_raw, c.bnout, smem, threadIdx.x);
}
template <class S, int ACT, int HG, bool TL = false>
__global__ __launch_bounds__(CONV_NT, 1) void k_fused_fb(CellArgs<S> a, ConvArgs<S> c) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  fused_fb_body<S, ACT, HG, false, TL>(a, c, a.t, c.out_raw, c.bnout, smem, threadIdx.x);
}

// Persistent forward (PT_CELL_PERSIST=1): the fused segments of all T frames
// in ONE launch of B workgroups, all resident (one per CU; the host checks
// the occupancy).  The two BatchNorm syncs per frame become in-launch waits:
// every workgroup publishes its partials (write-through + ticket), the last of
// each group stores the group sum write-through and counts it in done[t][bn];
// every workgroup's finalising wave waits for all groups (wave_wait).  Same
// arithmetic and reduction order as the per-segment launches.
template <class S, int ACT, int HG>
__global__ __launch_bounds__(CONV_NT, 1) void k_persist_fwd(const CellArgs<S> a, const ConvArgs<S> ca,
                                                            const ConvArgs<S> cb, unsigned* done,
                                                            unsigned* err) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const size_t fs = fr_off(1, a.B);
  const unsigned ng = (unsigned)bn_ngrp(a.B);
#pragma unroll 1
  for (int t = 0; t < a.T; ++t) {
    // the weight pointers and the thread index laundered per frame: hoisted
    // out of the frame loop, the per-lane weight-fragment and LDS addresses
    // pinned ~130 VGPRs (2 KB of spills)
    ConvArgs<S> cx = ca;
    asm volatile("" : "+s"(cx.wf));
    int tl = tid;
    asm volatile("" : "+v"(tl));
    BnSlot s0 = bnf_slot(a, t, 0);
    s0.done = done + 2 * t;
    fused_fa_body<S, ACT, HG, true>(a, cx, t, a.ci + t * fs, s0, smem, tl,
                                    done + 2 * (t - 1) + 1, ng, err);   // waits for BN1 of t-1
    ConvArgs<S> cy = cb;
    asm volatile("" : "+s"(cy.wf));
    tl = tid;
    asm volatile("" : "+v"(tl));
    BnSlot s1 = bnf_slot(a, t, 1);
    s1.done = done + 2 * t + 1;
    fused_fb_body<S, ACT, HG, true>(a, cy, t, a.ce + t * fs, s1, smem, tl,
                                    done + 2 * t, ng, err);             // waits for BN0 of t
  }
}

// -------------------------------------------------------------------------
// Backward point-wise A (t from T-1 down to -1).  Two halves:
//  tail (frame tt = t+1, if tt <= T-1): dgE (= conv^T(dci, w_inh) + e_u^T d_e_pre,
//     prepared by k_conv), attention-gate backward (a_w, a_u grads),
//     dE_t complete, dx_tt complete -> stem gradients.
//  head (frame t, if t >= 0): with dE_t: excitation update backward
//     (:175, :173) -> d_eg, dc_e (-> BN1 bwd sums), kappa/gamma grads,
//     dI_t (local), dE_{t-1} partial = (1-eg) dE_t.
// -------------------------------------------------------------------------
// Body of k_pw_ba (RPP = PWA_RPP rows per wave, PWA_WGPC workgroups per clip).
template <class S, int ACT, int HG, int RPP>
__device__ __forceinline__ void pw_ba_body(const CellArgs<S>& a, char* smem, int b, int part) {
  using F = typename Tr<S>::frag;
  constexpr bool BF = sizeof(S) == 2 && PT_PWA_STAGE;   // staged wave-per-tile 1x1 weight gradients (pcarve_ba)
  const PLds L = pcarve_ba<S>(smem);
  const int tid = threadIdx.x, lane = tid & 63, c = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int t = a.t, T = a.T, B = a.B;
  const int y0 = part * PW_NW * RPP;
  float* wscr = L.scr + wave * SCR_FLOATS;
  const size_t fs = fr_off(1, B), cb = clip_off(b);
  const int tt = t + 1;
  const bool tail = tt <= T - 1, head = t >= 0;
  float* slab_p = a.slab + ((size_t)b * PW_PARTS + part) * SLAB;

  PT_TR(a, PT_K_PW_BA, 0);
  if constexpr (BF) slab_range(slab_p, L.slabl, SLAB_G, NSMALL * 32, wave, lane);   // per-channel block
  else slab_prefetch(slab_p, L.slabl, 0, 2, wave, lane);                           // a_w, a_u
  if (tail) stage_x(a.x, a.xu8, L.xs, b, tt, T, y0, PW_NW * RPP, tid, PW_NT, a.ntx, a.nty);
  if constexpr (!BF) gacc_zero(L.gacc, 2, tid);
  __syncthreads();
  // BF: wave w forms output half mt = w & 1 of gate gi = w >> 1 (a_w: X = xbn,
  // a_u: X = E_t) over each set's staged 128 pixels
  const bool att_wg = tail && (head || HG) && !(PT_ABL(a.ablate) & 16);
  const int gi = wave >> 1, mt = wave & 1;
  f32x4 wacc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  constexpr int SE = stg_bytes<S, PWA_NPX>() / (int)sizeof(S);
  PT_TR(a, PT_K_PW_BA, 2);

  const Stem st{a.wpre[c * 3 + 0], a.wpre[c * 3 + 1], a.wpre[c * 3 + 2], a.bpre[c]};
  float sm[9] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int slots[9] = {SM_GBA, SM_KAPPA, SM_GAMMA, SM_BN1W, SM_BN1B, SM_PW0, SM_PW1, SM_PW2, SM_PB};
  float bs0 = 0.f, bs1 = 0.f;   // BN1 bwd partial sums

  const float nba = sig_nb(a.gb[0][c] + a.gb[1][c]);
  const float kap = a.kappa[c], gam = a.gamma[c], bw1 = a.bnw1[c], bb1 = a.bnb1[c];
  float m1 = 0.f, rs1 = 0.f;
  if (head) { m1 = a.bnstat[(size_t)t * 128 + 64 + c]; rs1 = a.bnstat[(size_t)t * 128 + 96 + c]; }
  const S* dgsrc = a.conv_done ? a.dgE : a.dgEp;

#pragma unroll 1
  for (int i = 0; i < RPP && !(PT_ABL(a.ablate) & 4); ++i) {
    if constexpr ((PT_PRIO & 4) != 0)
      prio_by_step(i + ((PT_PRIO & 8) && blockIdx.x < gridDim.x / 2 ? 1 : 0));
    const int yl = wave * RPP + i, y = y0 + yl;
    const size_t ro = cb + (size_t)y * IMG * C;
    S* st_dap = (S*)L.stage + (PT_PWA_PAIR ? (i & 1) * 3 * SE : 0);
    S* st_xv = st_dap + SE;
    S* st_E = st_dap + 2 * SE;
    f32x16 GE;
    if (tail) {
      f32x16 z, xv;                          // z: nl'(stem pre-activation)
      stem_cl<ACT, true>(L.xs, yl, h, st, z, xv);
      // this kernel's share of d xbn_tt (a_w^T d_att_pre); k_pw_bb adds the
      // inhibition path's share to the same stem-gradient sums itself (the
      // stem gradient is linear in d xbn), so no d xbn tile crosses HBM
      f32x16 dx = zero16();
      // attention backward of frame tt.  InT at tt = 0 has none (gE_0 =
      // att * E_{-1} = 0); hGRU's att_0 still feeds the gated inhibition.
      if (head || HG) {
        const f32x16 dgE = head ? load_cl(dgsrc + ro, c, h) : zero16();
        const Pk<S> dAt = HG ? load_pk(a.dAt + ro, c, h) : zero_pk<S>();
        // E_t as the a_u gate operand and in d att = dgE E_t: the hi plane
        // (bf16 cell; PT_EI_FULL: d att from the f32 value, as the forward's
        // gE = att E_t)
        const f32x16 Ef = head ? (PT_EI_FULL ? ldE(a, t, ro, c, h) : ldEh(a, t, ro, c, h)) : zero16();
        const f32x16 Et = PT_EI_FULL ? op_round<S>(Ef) : Ef;
        F pax[Tr<S>::KS], pae[Tr<S>::KS];
        cl_to_pa<S>(wscr, xv, lane, pax, RND_G(a));
        cl_to_pa<S>(wscr, Et, lane, pae, RND_G(a));
        f32x16 g = zero16();
        g = gemm_pa<S>(pax, a.gf[0], g, lane);
        g = gemm_pa<S>(pae, a.gf[1], g, lane);
        f32x16 att, dap;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          att[r] = sigm_b(g[r], nba);
          const float datt = HG ? dgE[r] * Ef[r] + (float)dAt[r] : dgE[r] * Ef[r];
          dap[r] = datt * att[r] * (1.f - att[r]);
          sm[0] += dap[r];
        }
        if constexpr (BF) {
          if (att_wg) {             // this set's operands; contracted after the barrier below
            cl_stage<PWA_NPX>((bf16_t*)st_dap, dap, wave * IMG, lane);
            cl_stage<PWA_NPX>((bf16_t*)st_xv, xv, wave * IMG, lane);
            cl_stage<PWA_NPX>((bf16_t*)st_E, Et, wave * IMG, lane);
          }
        } else {
          if (!(PT_ABL(a.ablate) & 16)) gacc_row<S>(L.gacc + 0 * 1024, L.flush, dap, xv, lane, wave, tid);
          if (!(PT_ABL(a.ablate) & 16)) gacc_row<S>(L.gacc + 1 * 1024, L.flush, dap, Et, lane, wave, tid);
        }
        F pad[Tr<S>::KS];
        cl_to_pa<S>(wscr, dap, lane, pad, RND_G(a));
        if (head) {
          GE = load_cl(a.dEn + ro, c, h);
#pragma unroll
          for (int r = 0; r < 16; ++r) GE[r] += dgE[r] * att[r];
          GE = gemm_pa<S>(pad, a.gt[1], GE, lane);
        }
        dx = gemm_pa<S>(pad, a.gt[0], dx, lane);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const f32x4 xin = L.xs[yl * IMG + cl_x(r, h)];
        const float dz = dx[r] * z[r];
        sm[5] += dz * xin[0]; sm[6] += dz * xin[1]; sm[7] += dz * xin[2]; sm[8] += dz;
      }
    } else {
      GE = load_cl(a.GEfin + ro, c, h);
    }
    if (head) {
      // kappa I + gamma as the forward formed it
      const f32x16 Iv = PT_EI_FULL ? ldI(a, t, ro, c, h) : ldIh(a, t, ro, c, h);
      const f32x16 cev = load_cl(a.ce + t * fs + ro, c, h);
      const f32x16 egv = load_cl(a.eg + t * fs + ro, c, h);
      const f32x16 Eo = t > 0 ? ldE(a, t - 1, ro, c, h) : zero16();   // full: eh - E_{t-1}
      f32x16 dIl, dEn, dEp, dcE;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float xe = (cev[r] - m1) * rs1;
        const float cn = bw1 * xe + bb1;
        const float w = kap * Iv[r] + gam;
        const float pe = cn * w;
        float eh, ehd;
        Act<ACT>::fd(pe, eh, ehd);
        const float deg = GE[r] * (eh - Eo[r]);
        const float dpe = GE[r] * egv[r] * ehd;
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
      store_cl(a.dIl + ro, c, h, rb16(RND_T(a), dIl));
      store_cl(a.dEn + ro, c, h, rb16(RND_T(a), dEn));
      store_cl(a.dEp + ro, c, h, rb16(RND_T(a), dEp));
      store_cl(a.dcE + ro, c, h, rb16(RND_T(a), dcE));
    }
    if constexpr (BF) {
      if (att_wg && (!PT_PWA_PAIR || (i & 1) || i + 1 == RPP)) {
        __syncthreads();                  // the set's 4 rows are staged (PAIR: two sets)
        for (int q = PT_PWA_PAIR && (i & 1) ? 1 : 0; q >= 0; --q) {
          const S* sd = st_dap - q * 3 * SE;
          pr_wgrad_acc<S, PWA_NPX>(sd, gi == 0 ? sd + SE : sd + 2 * SE, mt, wacc, lane);
        }
        __syncthreads();                  // before the next set restages
      }
    }
  }
  float wold[2][4];
  float* sp = slab_p + gi * 1024 + (16 * mt + 4 * (lane >> 4)) * 32 + (lane & 15);
  if constexpr (BF) {
    if (att_wg && !(PT_ABL(a.ablate) & 32))    // the gate tiles' old slab values
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int i = 0; i < 4; ++i) wold[nt][i] = sp[i * 32 + 16 * nt];
  }
  sm[3] = bs1;   // d bn1.weight = sum dy * xhat
  sm[4] = bs0;   // d bn1.bias   = sum dy
  PT_TR(a, PT_K_PW_BA, 3);
  PT_TRW(a, PT_K_PW_BA, 8);
  const bool bn = head && !(PT_ABL(a.ablate) & 8);
  const BnSlot bo = bnb_slot(a, t, 1, B * PWA_WGPC);
  float bv = 0.f;
  if (bn) bv = bn_bwd_partial(bs0, bs1, L.red, bo, lane, wave, tid);
  PT_TR(a, PT_K_PW_BA, 4);
  if (!(PT_ABL(a.ablate) & 32)) flush_small<9>(sm, slots, L.small, L.slabl, slab_p, lane, wave, tid);   // ends with a barrier
  if constexpr (BF) {
    if (att_wg && !(PT_ABL(a.ablate) & 32))
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int i = 0; i < 4; ++i) sp[i * 32 + 16 * nt] = wold[nt][i] + wacc[nt][i];
  } else {
    if (tail && (head || HG) && !(PT_ABL(a.ablate) & 32)) gacc_flush(L.gacc, L.slabl, slab_p, 0, 2, tid);
  }
  PT_TR(a, PT_K_PW_BA, 5);
  // L.stat is unused by the backward kernels: mode 2's ticket flag word
  if (bn) bn_publish_finish<PW_NT, false>(bo, blockIdx.x, bv, tid, (int*)L.stat, (double*)L.red);
  PT_TR(a, PT_K_PW_BA, 6);
}
template <class S, int ACT, int HG>
__global__ __launch_bounds__(PW_NT, 2) void k_pw_ba(CellArgs<S> a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if (PT_ABL(a.ablate) & 512) return;
  int b, part;
  wg_split(blockIdx.x, PWA_WGPC, a.B, a.xmap, b, part);
  pw_ba_body<S, ACT, HG, PWA_RPP>(a, smem, b, part);
}

// -------------------------------------------------------------------------
// Fused backward A (r06; PT_CPA): k_conv_ba(t) and
// k_pw_ba(t-1) as ONE launch of 2B workgroups.  Workgroup (clip b, part p)
// first runs band p of the BN0-backward conv^T (k_conv_bwd_band: 16 output
// rows, 4 waves x 4 rows; dgE_t = conv + dgEp stored as in the split form),
// then k_pw_ba(t-1)'s rows of the same band -- k_pw_ba's workgroup (b, p)
// owns image rows 16 p .. 16 p + 15 with wave w on rows 16 p + 4 w + i,
// exactly the rows wave w just convolved, so every dgE row is read back by
// the wave that stored it (program order; no barrier or flag between
// workgroups) and the launch boundary between the two kernels goes.  The
// two workgroups of a clip share a CU (blocks j and j + B), each at two waves
// per SIMD.  Arithmetic, reduction slots and orders: those of
// k_conv_bwd_band (bitwise k_conv_bwd_band2) and k_pw_ba -- bitwise the
// split pair (tests/test_gpu_fused.py).
// -------------------------------------------------------------------------
static_assert(BAND_NT == PW_NT && PWA_RPP == BAND_RW && PW_NW * PWA_RPP == BAND_ROWS && PWA_WGPC == 2,
              "a k_pw_ba workgroup's rows are one band of the banded conv");
template <class S> constexpr int cpa_lds_bytes() {
  return pwa_lds_bytes<S>() > band_tile_bytes() + CONV_MISC * 4 ? pwa_lds_bytes<S>()
                                                               : band_tile_bytes() + CONV_MISC * 4;
}
template <int ACT, int HG>
__global__ __launch_bounds__(PW_NT, 2) void k_conv_pw_ba(CellArgs<bf16_t> a, ConvArgs<bf16_t> c) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if (PT_ABL(a.ablate) & 512) return;
  int b, part;
  wg_split(blockIdx.x, PWA_WGPC, a.B, a.xmap, b, part);
  {
    constexpr int RW = BAND_RW;
    const int lane = threadIdx.x & 63, h = lane >> 5, px = lane & 31;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if constexpr ((PT_PRIO & 64) != 0) {      // the clip's part 1 lags: its conv beside part 0's rows
      if (part == 1) __builtin_amdgcn_s_setprio(0);
      else __builtin_amdgcn_s_setprio(2);
    }
    f32x16 acc[RW];
    bf16x4 p0[RW][4], p1[RW][4];
    const AddRowBand<RW> ar{(bf16_t*)c.out, (const bf16_t*)c.add0, (const bf16_t*)c.add1,
                            clip_off(b) + ((size_t)(part * BAND_ROWS + wave * RW) * IMG + px) * C, h, p0, p1};
    band_conv_body(c, smem, b, part, acc, ar);
  }
  __syncthreads();              // the conv tile's LDS becomes k_pw_ba's
  pw_ba_body<bf16_t, ACT, HG, PWA_RPP>(a, smem, b, part);
}

// -------------------------------------------------------------------------
// Backward point-wise B (frame t): with dI_t (= conv^T(dce, w_exc) + local
//   + from frame t+1, prepared by k_conv): inhibition update backward
//   (:166, :165, :162) -> i_w/i_u, alpha, mu, dc_i (-> BN0 bwd sums),
//   dx_t partial, dI_{t-1}; exc gate backward (:171) -> e_w/e_u grads,
//   dI_{t-1}, dgE partial.
// -------------------------------------------------------------------------
template <class S>
struct BbRow { f32x16 ginh, Iprev; Pk<S> dep, gEv, dIt, civ; };

// Body of k_pw_bb (RPP = 1 row per wave, PWB_WGPC workgroups per clip).
template <class S, int ACT, int HG, int RPP>
__device__ __forceinline__ void pw_bb_body(const CellArgs<S>& a, char* smem, int b, int part) {
  using F = typename Tr<S>::frag;
  constexpr bool BF = sizeof(S) == 2;      // staged wave-per-gate 1x1 weight gradients
  const PLds L = pcarve_bb<S>(smem);
  const int tid = threadIdx.x, lane = tid & 63, c = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int t = a.t, T = a.T, B = a.B;
  const int y0 = part * PW_NW * RPP;
  float* wscr = L.scr + wave * SCR_FLOATS;
  const size_t fs = fr_off(1, B);
  float* slab_p = a.slab + ((size_t)b * PW_PARTS + part) * SLAB;

  // row tiles: g_inh = I_{t-1} (InT) / E_{t-1} (no_inh) and gE_t feed the exc
  // gate (:171), dI_t and c_i the inhibition backward.  Kept packed; e_w^T
  // d_e_pre is folded into dI_{t-1} at the end from its A fragments (pe)
  // rather than kept as a tile.  hGRU: g_inh = att_t (ffhgru_hierarchy.py:147)
  // and I_{t-1} is a separate tile.
  auto load_row = [&](size_t ro, int c, int h) {
    BbRow<S> w;
    w.Iprev = zero16();
    if constexpr (HG) {
      w.ginh = load_cl(a.at + t * fs + ro, c, h);
      if (t > 0) w.Iprev = ldI(a, t - 1, ro, c, h);
    } else {
      if (t == 0) w.ginh = zero16();
      else if (a.no_inh) w.ginh = ldE(a, t - 1, ro, c, h);
      else w.ginh = ldI(a, t - 1, ro, c, h);
    }
    w.dep = load_pk(a.dEp + ro, c, h);
    w.gEv = load_pk(a.gE + t * fs + ro, c, h);
    w.dIt = zero_pk<S>();
    w.civ = zero_pk<S>();
    if (!a.no_inh) {
      w.dIt = load_pk(a.dIt + ro, c, h);
      w.civ = load_pk(a.ci + t * fs + ro, c, h);
    }
    return w;
  };
  PT_TR(a, PT_K_PW_BB, 0);
  // one row per wave: its tiles are loaded first, their latency overlaps the staging
  BbRow<S> pre;
  if constexpr (RPP == 1) pre = load_row(clip_off(b) + (size_t)(y0 + wave) * IMG * C, c, h);
  if (!(PT_ABL(a.ablate) & 262144)) slab_prefetch(slab_p, L.slabl, 2, 4, wave, lane);   // i_w, i_u, e_w, e_u
  stage_x(a.x, a.xu8, L.xs, b, t, T, y0, PW_NW * RPP, tid, PW_NT, a.ntx, a.nty);
  if constexpr (!BF) gacc_zero(L.gacc, 4, tid);
  PT_TR(a, PT_K_PW_BB, 1);
  __syncthreads();
  PT_TR(a, PT_K_PW_BB, 2);

  const float* bs = a.bnstat + (size_t)t * 128;
  float sm[10] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int slots[10] = {SM_ALPHA, SM_MU, SM_GBI, SM_GBE, SM_BN0W, SM_BN0B,
                         SM_PW0, SM_PW1, SM_PW2, SM_PB};
  float bs0 = 0.f, bs1 = 0.f;

#pragma unroll 1
  for (int i = 0; i < RPP && !(PT_ABL(a.ablate) & 4); ++i) {
    // several rows per wave: the lane index laundered per row, so that the
    // per-lane parameters and addresses are formed in the row instead of
    // staying live across the loop as invariants (RPP 2: 161 VGPRs of spills)
    int tl = tid;
    if constexpr (RPP > 1) asm volatile("" : "+v"(tl));
    const int lane = tl & 63, c = lane & 31, h = lane >> 5;
    const Stem st{a.wpre[c * 3 + 0], a.wpre[c * 3 + 1], a.wpre[c * 3 + 2], a.bpre[c]};
    const float al = a.alpha[c], mu = a.mu[c], bw0 = a.bnw0[c], bb0 = a.bnb0[c];
    const float m0 = bs[c], rs0 = bs[32 + c];
    const float nbi = sig_nb(a.gb[2][c] + a.gb[3][c]);
    const int yl = wave * RPP + i, y = y0 + yl;
    const size_t ro = clip_off(b) + (size_t)y * IMG * C;
    BbRow<S> w;
    if constexpr (RPP == 1) w = pre;
    else w = load_row(ro, c, h);
    const f32x16& ginh = w.ginh;
    const Pk<S>& dIt = w.dIt;
    const Pk<S>& civ = w.civ;
    f32x16& Iprev = w.Iprev;
    F pe[Tr<S>::KS];
    {
      f32x16 depf;
#pragma unroll
      for (int r = 0; r < 16; ++r) depf[r] = (float)w.dep[r];
      if constexpr (BF) {
        // slots: 0 d_e_pre, 1 g_inh, 2 gE_t; waves 0 / 1 form e_w / e_u (slab gates 4, 5)
        stage_wg(L.stage, 0, depf, wave, lane);
        stage_wg(L.stage, 1, ginh, wave, lane);
        stage_wg(L.stage, 2, w.gEv, wave, lane);
        __syncthreads();
        if (wave < 2 && !(PT_ABL(a.ablate) & 16))
          gate_wgrad(L.stage, 0, 1 + wave, 4 + wave, L.slabl, slab_p, lane);
      } else {
        if (!(PT_ABL(a.ablate) & 16)) gacc_row<S>(L.gacc + 2 * 1024, L.flush, depf, ginh, lane, wave, tid);
        if (!(PT_ABL(a.ablate) & 16)) gacc_row<S>(L.gacc + 3 * 1024, L.flush, depf, w.gEv, lane, wave, tid);
      }
      sm[3] += hsum16(depf);
      cl_to_pa<S>(wscr, depf, lane, pe, RND_G(a));
      const f32x16 dIt0 = a.no_inh ? load_cl(a.dIt + ro, c, h) : zero16();
      const f32x16 dg = gemm_pa<S>(pe, a.gt[5], dIt0, lane);   // no_inh: I_t = gE_t
      store_cl(a.dgEp + ro, c, h, rb16(RND_T(a), dg));
    }
    if (a.no_inh) {
      const f32x16 dEn = gemm_pa<S>(pe, a.gt[4], load_cl(a.dEn + ro, c, h), lane);
      store_cl(a.dEn + ro, c, h, dEn);
    } else {
      // z: nl'(stem pre-activation); hGRU keeps z itself and forms nl' at
      // its use (its register schedule: 15.75 vs 15.4 ms/step at cfg4)
      f32x16 z, xv;
      stem_cl<ACT, !HG>(L.xs, yl, h, st, z, xv);
      f32x16 g = zero16();
      {
        F pax[Tr<S>::KS], pai[Tr<S>::KS];
        cl_to_pa<S>(wscr, xv, lane, pax, RND_G(a));
        g = gemm_pa<S>(pax, a.gf[2], g, lane);
        cl_to_pa<S>(wscr, ginh, lane, pai, RND_G(a));
        g = gemm_pa<S>(pai, a.gf[3], g, lane);
      }
      const float A0 = bw0 * rs0, B0 = bb0 - bw0 * rs0 * m0;    // BN0 affine folded
      f32x16 dIp, dip, dx;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float Ir = ginh[r], dIr = (float)dIt[r];
        const float Ip = HG ? Iprev[r] : Ir;             // I_{t-1} of the update (:166)
        const float xi = ((float)civ[r] - m0) * rs0;
        const float cn = A0 * (float)civ[r] + B0;
        const float u = al * Ir + mu;
        const float p = cn * u;
        float fp, dfp, ih, dfq;
        Act<ACT>::fd(p, fp, dfp);
        const float q = xv[r] - fp;
        Act<ACT>::fd(q, ih, dfq);
        const float ig = sigm_b(g[r], nbi);
        const float dih = dIr * ig;
        dip[r] = dIr * (ih - Ip) * ig * (1.f - ig);
        const float dq = dih * dfq;
        const float dp = -dq * dfp;
        const float du = dp * cn;
        const float dci = dp * u;
        stf(a.dcI + ro + cl_x(r, h) * C + c, rbf(RND_T(a), dci));
        dx[r] = dq;
        // InT: dI_{t-1} collects the update and the gated-inhibition terms;
        // hGRU: the gated-inhibition terms go to att (dA, kept in dIp's slot)
        dIp[r] = HG ? du * al : dIr * (1.f - ig) + du * al;
        if constexpr (HG) Iprev[r] = dIr * (1.f - ig);
        sm[0] += du * Ir;
        sm[1] += du;
        sm[2] += dip[r];
        bs0 += dci;
        bs1 += dci * xi;
      }
      if constexpr (BF) {
        // slots 0 / 2 are free once waves 0 / 1 have read them: d_i_pre -> 0, x -> 2;
        // waves 2 / 3 form i_w (x) / i_u (g_inh) (slab gates 2, 3)
        __syncthreads();
        stage_wg(L.stage, 0, dip, wave, lane);
        stage_wg(L.stage, 2, xv, wave, lane);
        __syncthreads();
        if (wave >= 2 && !(PT_ABL(a.ablate) & 16))
          gate_wgrad(L.stage, 0, wave == 2 ? 2 : 1, wave, L.slabl, slab_p, lane);
      } else {
        if (!(PT_ABL(a.ablate) & 16)) gacc_row<S>(L.gacc + 0 * 1024, L.flush, dip, xv, lane, wave, tid);
        if (!(PT_ABL(a.ablate) & 16)) gacc_row<S>(L.gacc + 1 * 1024, L.flush, dip, ginh, lane, wave, tid);
      }
      F pd[Tr<S>::KS];
      cl_to_pa<S>(wscr, dip, lane, pd, RND_G(a));
      dx = gemm_pa<S>(pd, a.gt[2], dx, lane);
      // stem backward of this share (models/InT.py:212-213): dz = dx nl'(z)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const f32x4 xin = L.xs[yl * IMG + cl_x(r, h)];
        const float dz = dx[r] * (HG ? Act<ACT>::d(z[r]) : z[r]);
        sm[6] += dz * xin[0]; sm[7] += dz * xin[1]; sm[8] += dz * xin[2]; sm[9] += dz;
      }
      dIp = gemm_pa<S>(pd, a.gt[3], dIp, lane);
      dIp = gemm_pa<S>(pe, a.gt[4], dIp, lane);
      if constexpr (HG) {
        store_cl(a.dAt + ro, c, h, dIp);
        f32x16 gi;
#pragma unroll
        for (int r = 0; r < 16; ++r) gi[r] = Iprev[r];
        store_cl(a.GI + ro, c, h, gi);
      } else {
        store_cl(a.GI + ro, c, h, rb16(RND_T(a), dIp));
      }
    }
  }
  sm[4] = bs1;
  sm[5] = bs0;
  PT_TR(a, PT_K_PW_BB, 3);
  const bool bn = !a.no_inh && !(PT_ABL(a.ablate) & 8);
  const BnSlot bo = bnb_slot(a, t, 0, B * PWB_WGPC);
  float bv = 0.f;
  if (bn) bv = bn_bwd_partial(bs0, bs1, L.red, bo, lane, wave, tid);
  PT_TR(a, PT_K_PW_BB, 4);
  if (!(PT_ABL(a.ablate) & 32)) flush_small<10>(sm, slots, L.small, L.slabl, slab_p, lane, wave, tid);  // ends with a barrier
  PT_TR(a, PT_K_PW_BB, 5);
  if (bn) bn_publish_finish<PW_NT, false>(bo, blockIdx.x, bv, tid, (int*)L.stat, (double*)L.red);
  PT_TR(a, PT_K_PW_BB, 6);
  if (PT_ABL(a.ablate) & 32) return;
  // gacc: 0 i_w, 1 i_u, 2 e_w, 3 e_u  ->  slab gates 2..5 (bf16: written by gate_wgrad)
  if constexpr (!BF) {
    if (!a.no_inh) gacc_flush(L.gacc, L.slabl, slab_p, 2, 2, tid);
    gacc_flush(L.gacc + 2 * 1024, L.slabl, slab_p, 4, 2, tid);
  }
}
template <class S, int ACT, int HG>
__global__ __launch_bounds__(PW_NT, 2) void k_pw_bb(CellArgs<S> a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if (PT_ABL(a.ablate) & 512) return;
  int b, part;
  wg_split(blockIdx.x, PWB_WGPC, a.B, a.xmap, b, part);
  pw_bb_body<S, ACT, HG, PWB_RPP>(a, smem, b, part);
}

// =========================================================================
// k_pw_bb2 (r04): backward point-wise B in the half-row PR layout (pt_pr.h).
// Same arithmetic as k_pw_bb (models/InT.py:162-171 differentiated, the
// reference's autograd of rCell.forward).  A workgroup = 8 waves owns 8 image
// rows of one clip, in two sets of 4 rows; in each set wave w takes one half
// row (row w >> 1 of the set, pixels 16 (w & 1) .. +15), 8 values per lane,
// <= 128 VGPRs: 4 waves per SIMD (k_pw_bb: 2) and half the workgroups of
// k_pw_bb, so a launch is two rounds of workgroups instead of four and each
// workgroup's prologue and epilogue serve twice the rows.  Per half row: the
// tiles loaded once, the 1x1 gates as 16x16x32 MFMAs (A operand
// transposed through a per-wave LDS scratch), the 1x1 weight-gradient
// operands staged channel-major; after each set wave w contracts output tile
// row (w & 1) of gate w >> 1 (i_w, i_u, e_w, e_u) over the set's 128 pixels
// into registers.  At the end the per-channel sums (lane-local, xor 16 / 32,
// then the 8 waves in order) and the gate tiles go to the slab (old values
// loaded at entry).  BatchNorm producers: PB2_WGPC workgroups per clip.
// =========================================================================
constexpr int PB2_NT = 512, PB2_NW = PB2_NT / 64;
constexpr int PB2_SET = 4;                    // rows per set
// sets per workgroup / workgroups per clip: bf16 4 / 2 (B = 256: 512
// workgroups, one round at two per CU); f32 (the parity path, twice the
// registers per operand) 1 / 8
#ifndef PT_PB2_NSET
#define PT_PB2_NSET 4
#endif
// (hGRU, bf16: 2 sets -- its extra I_{t-1} tile spilled 33 VGPRs at 4)
template <class S, int HG = 0> constexpr int pb2_nset() {
  return sizeof(S) == 2 ? (HG ? 2 : PT_PB2_NSET) : 1;
}
template <class S, int HG = 0> constexpr int pb2_wgpc() { return IMG / (4 * pb2_nset<S, HG>()); }
constexpr int PB2_NPX = PB2_SET * IMG;        // 128 pixels per set
constexpr int PB2_NQ = 10;                    // per-channel sums
static_assert(PB2_NW == 2 * PB2_SET, "one half row per wave and set");
static_assert(IMG / 4 <= PW_PARTS && IMG / 4 <= BNB_WG_PER_CLIP, "slab / BN slots per clip");
template <class S> constexpr int pb2_lds_bytes() {
  return pb2_nset<S>() * PB2_NPX * 16 /*xs*/ + PB2_NW * prs_bytes<S>() /*transpose scratch*/ +
         5 * stg_bytes<S, PB2_NPX>() /*weight-gradient operands*/ + PB2_NW * PB2_NQ * 32 * 4 /*sums*/ +
         (PB2_NT / 64) * 64 * 8 /*group-sum scratch (fp64)*/ + 16 /*flag*/;
}
// slab slots of the 10 sums, in this order: q 0 / 1 are the BatchNorm
// partial (sum dy, sum dy xhat), so threads 0..63 hold the values to publish
__constant__ int kPb2Slot[PB2_NQ] = {SM_BN0B, SM_BN0W, SM_ALPHA, SM_MU, SM_GBI, SM_GBE,
                                     SM_PW0, SM_PW1, SM_PW2, SM_PB};

__device__ __forceinline__ f32x2 lsum8(const f32x8& v) {
  return f32x2{v[0] + v[1] + v[2] + v[3], v[4] + v[5] + v[6] + v[7]};
}
__device__ __forceinline__ f32x8 rb8(bool on, f32x8 v) {
  if (on)
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = rbf(true, v[e]);
  return v;
}
template <class S> struct Pb2In { f32x8 ginh, Iprev; PrPk<S> dep, gE, dIt, ci; };
template <class S, int HG>
__device__ __forceinline__ Pb2In<S> pb2_load(const CellArgs<S>& a, int t, size_t ro, int lane) {
  const size_t fs = fr_off(1, a.B);
  Pb2In<S> w;
  w.Iprev = zero8();
  if constexpr (HG) {
    w.ginh = pr_load<S>(a.at + t * fs + ro, lane);                    // g_inh = att_t
    if (t > 0) w.Iprev = prI(a, t - 1, ro, lane);
  } else {
    if (t == 0) w.ginh = zero8();
    else if (a.no_inh) w.ginh = prE(a, t - 1, ro, lane);
    else w.ginh = prI(a, t - 1, ro, lane);
  }
  w.dep = pr_load_pk<S>(a.dEp + ro, lane);
  w.gE = pr_load_pk<S>(a.gE + t * fs + ro, lane);
  w.dIt = pr_load_pk<S>(a.dIt + ro, lane);
  w.ci = PrPk<S>{};
  if (!a.no_inh) w.ci = pr_load_pk<S>(a.ci + t * fs + ro, lane);
  return w;
}

template <class S, int ACT, int HG>
__global__ __launch_bounds__(PB2_NT, 4) void k_pw_bb2(CellArgs<S> a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if (PT_ABL(a.ablate) & 512) return;
  const int tid = threadIdx.x, lane = tid & 63, n = lane & 15, g4 = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  constexpr int NSET = pb2_nset<S, HG>(), WGPC = pb2_wgpc<S, HG>();
  int b, part;
  wg_split(blockIdx.x, WGPC, a.B, a.xmap, b, part);
  const int t = a.t, T = a.T, B = a.B;
  const int y0 = part * PB2_SET * NSET;
  const int px0 = (wave >> 1) * IMG + (wave & 1) * HR;       // first pixel of the half row in its set
  float* slab_p = a.slab + ((size_t)b * PW_PARTS + part) * SLAB;
  f32x4* xs = (f32x4*)smem;                                  // [2 sets][128 px]
  char* p = smem + NSET * PB2_NPX * 16;
  S* scr = (S*)(p + wave * prs_bytes<S>());
  p += PB2_NW * prs_bytes<S>();
  constexpr int SE = stg_bytes<S, PB2_NPX>() / (int)sizeof(S);
  S* st_dep = (S*)p;
  S* st_ginh = st_dep + SE;
  S* st_gE = st_dep + 2 * SE;
  S* st_dip = st_dep + 3 * SE;
  S* st_xv = st_dep + 4 * SE;
  float* wsum = (float*)(p + 5 * stg_bytes<S, PB2_NPX>());
  double* gscr = (double*)(wsum + PB2_NW * PB2_NQ * 32);
  int* flag = (int*)(gscr + (PB2_NT / 64) * 64);
  const int gi = wave >> 1, mt = wave & 1;                  // this wave's weight-gradient tile row
  const bool do_wg = !(a.no_inh && gi < 2) && !(PT_ABL(a.ablate) & 16);
  PT_TR(a, PT_K_PW_BB, 0);

  auto row_off = [&](int set) {
    return clip_off(b) + ((size_t)(y0 + set * PB2_SET) * IMG + px0) * C;
  };
  // set 0's tiles first (their latency overlaps the x staging), then the
  // old values of the slab's sums
  const Pb2In<S> in = pb2_load<S, HG>(a, t, row_off(0), lane);
  float* sp = slab_p + (2 + gi) * 1024 + (16 * mt + 4 * g4) * 32 + n;
  float wold[2][4];
  const int so = tid < PB2_NQ * 32 ? SLAB_G + kPb2Slot[tid >> 5] * 32 + (tid & 31) : 0;
  const float sold = tid < PB2_NQ * 32 ? slab_p[so] : 0.f;
  PT_TR(a, PT_K_PW_BB, 1);
  stage_x(a.x, a.xu8, xs, b, t, T, y0, PB2_SET * NSET, tid, PB2_NT, a.ntx, a.nty);
  __syncthreads();
  PT_TR(a, PT_K_PW_BB, 2);

  f32x4 wacc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};

  // one set (inlined once per set); the next set's tiles are loaded once this
  // set's element-wise temporaries are dead, before its barriers
  Pb2In<S> in1;
  auto set_body = [&](const int set, const Pb2In<S> in) {
    if constexpr ((PT_PRIO & 4) != 0)
      prio_by_step(set + ((PT_PRIO & 8) && blockIdx.x < gridDim.x / 2 ? 1 : 0));
    // the lane index laundered per set: the per-lane parameters and addresses
    // are formed in the set instead of living across both as invariants
    int tl = tid;
    if constexpr (NSET > 1) asm volatile("" : "+v"(tl));
    const int lane = tl & 63, n = lane & 15, g4 = lane >> 4;
    const size_t ro = row_off(set);
    f32x2 sm[PB2_NQ];
#pragma unroll
    for (int q = 0; q < PB2_NQ; ++q) sm[q] = f32x2{-0.f, -0.f};   // -0: the first add folds away
    const f32x4* xr = xs + set * PB2_NPX + px0 + 4 * g4;
    // this lane's channels 2n, 2n + 1
    float w0[2], w1[2], w2[2], bp[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int c = 2 * n + k;
      w0[k] = a.wpre[c * 3 + 0]; w1[k] = a.wpre[c * 3 + 1]; w2[k] = a.wpre[c * 3 + 2]; bp[k] = a.bpre[c];
    }
    const f32x8 depf = pr_widen(in.dep);
    const f32x8 ginh = in.ginh;
    f32x8 Iprev = in.Iprev;
    sm[5] += lsum8(depf);                                              // e-gate biases
    pr_stage<S, PB2_NPX>(st_dep, depf, px0, lane);
    pr_stage<S, PB2_NPX>(st_ginh, ginh, px0, lane);
    pr_stage<S, PB2_NPX>(st_gE, pr_widen(in.gE), px0, lane);
    const f32x8 dIt = pr_widen(in.dIt);
    const PrA<S> pe = pr_to_a<S>(scr, rb8(RND_G(a), depf), lane);
    {
      const f32x8 dg = pr_mm<S>(pe, a.g16t[5], a.no_inh ? dIt : zero8(), lane);   // no_inh: I_t = gE_t
      pr_store<S>(a.dgEp + ro, lane, rb8(RND_T(a), dg));
    }
    if (a.no_inh) {
      const f32x8 dEn = pr_mm<S>(pe, a.g16t[4], pr_load<S>(a.dEn + ro, lane), lane);
      pr_store<S>(a.dEn + ro, lane, dEn);
    } else {
      const float* bs = a.bnstat + (size_t)t * 128;
      const f32x2 al = pr_par(a.alpha, lane), mu = pr_par(a.mu, lane);
      const f32x2 bw0 = pr_par(a.bnw0, lane), bb0 = pr_par(a.bnb0, lane);
      const f32x2 m0 = pr_par(bs, lane), rs0 = pr_par(bs + 32, lane);
      const f32x2 gb2 = pr_par(a.gb[2], lane), gb3 = pr_par(a.gb[3], lane);
      // stem (models/InT.py:212-213) of the lane's 4 pixels; z: nl'(pre-activation)
      // (hGRU keeps the pre-activation and forms nl' at its use, as k_pw_bb)
      f32x8 z, xv;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f32x4 xin = xr[i];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const float zr = w0[k] * xin[0] + w1[k] * xin[1] + w2[k] * xin[2] + bp[k];
          if constexpr (HG) {
            z[4 * k + i] = zr;
            xv[4 * k + i] = Act<ACT>::f(zr);
          } else {
            float f, d;
            Act<ACT>::fd(zr, f, d);
            xv[4 * k + i] = f;
            z[4 * k + i] = d;
          }
        }
      }
      f32x8 gpre;
      {
        const PrA<S> ax = pr_to_a<S>(scr, rb8(RND_G(a), xv), lane);
        const PrA<S> ai = pr_to_a<S>(scr, rb8(RND_G(a), ginh), lane);
        gpre = pr_mm<S>(ax, a.g16f[2], zero8(), lane);
        gpre = pr_mm<S>(ai, a.g16f[3], gpre, lane);
      }
      const f32x8 civ = pr_widen(in.ci);
      f32x8 dIp, dip, dx, dci;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = e >> 2;
        const float A0 = bw0[k] * rs0[k], B0 = bb0[k] - bw0[k] * rs0[k] * m0[k];   // BN0 affine folded
        const float Ir = ginh[e], dIr = dIt[e];
        const float Ip = HG ? Iprev[e] : Ir;               // I_{t-1} of the update (:166)
        const float xi = (civ[e] - m0[k]) * rs0[k];
        const float cn = A0 * civ[e] + B0;
        const float u = al[k] * Ir + mu[k];
        const float pp = cn * u;
        float fp, dfp, ih, dfq;
        Act<ACT>::fd(pp, fp, dfp);
        const float q = xv[e] - fp;
        Act<ACT>::fd(q, ih, dfq);
        const float ig = sigm_b(gpre[e], sig_nb(gb2[k] + gb3[k]));
        const float dih = dIr * ig;
        dip[e] = dIr * (ih - Ip) * ig * (1.f - ig);
        const float dq = dih * dfq;
        const float dp = -dq * dfp;
        const float du = dp * cn;
        dci[e] = dp * u;
        dx[e] = dq;
        // InT: dI_{t-1} collects the update and the gated-inhibition terms;
        // hGRU: the gated-inhibition terms go to att (dA, kept in dIp)
        dIp[e] = HG ? du * al[k] : dIr * (1.f - ig) + du * al[k];
        if constexpr (HG) Iprev[e] = dIr * (1.f - ig);
        sm[2][k] += du * Ir;
        sm[3][k] += du;
        sm[4][k] += dip[e];
        sm[0][k] += dci[e];
        sm[1][k] += dci[e] * xi;
      }
      pr_store<S>(a.dcI + ro, lane, rb8(RND_T(a), dci));
      pr_stage<S, PB2_NPX>(st_dip, dip, px0, lane);
      pr_stage<S, PB2_NPX>(st_xv, xv, px0, lane);
      const PrA<S> pd = pr_to_a<S>(scr, rb8(RND_G(a), dip), lane);
      dx = pr_mm<S>(pd, a.g16t[2], dx, lane);
      // stem backward of this share (models/InT.py:212-213): dz = dx nl'(z)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f32x4 xin = xr[i];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const int e = 4 * k + i;
          const float dz = dx[e] * (HG ? Act<ACT>::d(z[e]) : z[e]);
          sm[6][k] += dz * xin[0];
          sm[7][k] += dz * xin[1];
          sm[8][k] += dz * xin[2];
          sm[9][k] += dz;
        }
      }
      dIp = pr_mm<S>(pd, a.g16t[3], dIp, lane);
      dIp = pr_mm<S>(pe, a.g16t[4], dIp, lane);
      if constexpr (HG) {
        pr_store<S>(a.dAt + ro, lane, dIp);
        pr_store<S>(a.GI + ro, lane, Iprev);
      } else {
        pr_store<S>(a.GI + ro, lane, rb8(RND_T(a), dIp));
      }
    }
    if (set + 1 < NSET) in1 = pb2_load<S, HG>(a, t, row_off(set + 1), lane);
    // this set's per-channel sums over the half row -> the wave's LDS slots
#pragma unroll
    for (int q = 0; q < PB2_NQ; ++q) {
      f32x2 v = sm[q];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        v[k] += __shfl_xor(v[k], 16);
        v[k] += __shfl_xor(v[k], 32);
      }
      f32x2* ws = (f32x2*)(wsum + (wave * PB2_NQ + q) * 32 + 2 * n);
      if (lane < 16) *ws = set == 0 ? v : *ws + v;
    }
    __syncthreads();
    if (do_wg) {
      const S* D = gi < 2 ? st_dip : st_dep;
      const S* X = gi == 0 ? st_xv : gi == 3 ? st_gE : st_ginh;
      pr_wgrad_acc<S, PB2_NPX>(D, X, mt, wacc, lane);
    }
    if (set + 1 < NSET) __syncthreads();                  // the operand slots are reused
  };
  set_body(0, in);
  if constexpr (NSET > 1) set_body(1, in1);
  if constexpr (NSET > 2) set_body(2, in1);
  if constexpr (NSET > 3) set_body(3, in1);
  static_assert(NSET <= 4, "set bodies");
  PT_TR(a, PT_K_PW_BB, 3);
  PT_TRW(a, PT_K_PW_BB, 8);
  if (do_wg) {                            // the gate tiles' old slab values
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int i = 0; i < 4; ++i) wold[nt][i] = sp[i * 32 + 16 * nt];
  }
  // (the last set's barrier before its contraction published the sums)
  PT_TR(a, PT_K_PW_BB, 4);
  // sums over the 8 waves (wave order) -> slab; threads 0..63: the BatchNorm partial
  const bool bn = !a.no_inh && !(PT_ABL(a.ablate) & 8);
  const BnSlot bo = bnb_slot(a, t, 0, B * WGPC);
  float bv = 0.f;
  if (tid < PB2_NQ * 32) {
    const int q = tid >> 5, c = tid & 31;
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < PB2_NW; ++w) s += wsum[(w * PB2_NQ + q) * 32 + c];
    bv = s;
    if (!(PT_ABL(a.ablate) & 32)) slab_p[so] = sold + s;
  }
  if (do_wg) {
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int i = 0; i < 4; ++i) sp[i * 32 + 16 * nt] = wold[nt][i] + wacc[nt][i];
  }
  PT_TR(a, PT_K_PW_BB, 5);
  if (bn) bn_publish<PB2_NT, false>(bo, blockIdx.x, bv, tid, flag, gscr);
  PT_TR(a, PT_K_PW_BB, 6);
}

// =========================================================================
// k_pw_ba2 (r04): backward point-wise A in the half-row PR layout (pt_pr.h),
// the same arithmetic as k_pw_ba (models/InT.py:148-153 and :172-175
// differentiated): tail = the attention backward of frame t + 1 and the stem
// gradient; head = the excitation update backward of frame t.  Workgroup
// structure as k_pw_bb2: 8 waves, one half row each per set of 4 rows, bf16
// 4 sets (16 rows, 2 workgroups per clip: the same BatchNorm producer split
// and slab partitions as k_pw_ba) / f32 1 set; after each set waves 0-3
// contract the a_w / a_u weight-gradient tiles (D = d att_pre, X = x / E_t)
// over the set's 128 pixels into registers.
// =========================================================================
constexpr int PA2_NQ = 9;
template <class S> constexpr int pa2_nset() { return sizeof(S) == 2 ? 4 : 1; }
template <class S> constexpr int pa2_wgpc() { return IMG / (4 * pa2_nset<S>()); }
template <class S> constexpr int pa2_lds_bytes() {
  return pa2_nset<S>() * PB2_NPX * 16 /*xs*/ + PB2_NW * prs_bytes<S>() /*transpose scratch*/ +
         3 * stg_bytes<S, PB2_NPX>() /*weight-gradient operands*/ + PB2_NW * PA2_NQ * 32 * 4 /*sums*/ +
         (PB2_NT / 64) * 64 * 8 /*group-sum scratch (fp64)*/ + 16 /*flag*/;
}
// slab slots of the 9 sums; q 0 / 1 = the BatchNorm partial (sum dy, sum dy xhat)
__constant__ int kPa2Slot[PA2_NQ] = {SM_BN1B, SM_BN1W, SM_GBA, SM_KAPPA, SM_GAMMA,
                                     SM_PW0, SM_PW1, SM_PW2, SM_PB};
template <class S> struct Pa2In { PrPk<S> dgE, dAt, ce, eg, dEn; f32x8 Et, Iv, Eo; };

template <class S, int ACT, int HG>
__global__ __launch_bounds__(PB2_NT, 4) void k_pw_ba2(CellArgs<S> a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if (PT_ABL(a.ablate) & 512) return;
  constexpr int NSET = pa2_nset<S>(), WGPC = pa2_wgpc<S>();
  const int tid = threadIdx.x, lane = tid & 63, n = lane & 15, g4 = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int b, part;
  wg_split(blockIdx.x, WGPC, a.B, a.xmap, b, part);
  const int t = a.t, T = a.T, B = a.B;
  const int tt = t + 1;
  const bool tail = tt <= T - 1, head = t >= 0;
  const bool att_bwd = tail && (head || HG);      // InT at tt = 0 has none (gE_0 = att * E_{-1} = 0)
  const int y0 = part * 4 * NSET;
  const int px0 = (wave >> 1) * IMG + (wave & 1) * HR;
  const size_t fs = fr_off(1, B);
  float* slab_p = a.slab + ((size_t)b * PW_PARTS + part) * SLAB;
  f32x4* xs = (f32x4*)smem;                                  // [NSET][128 px]
  char* p = smem + NSET * PB2_NPX * 16;
  S* scr = (S*)(p + wave * prs_bytes<S>());
  p += PB2_NW * prs_bytes<S>();
  constexpr int SE = stg_bytes<S, PB2_NPX>() / (int)sizeof(S);
  S* st_dap = (S*)p;
  S* st_xv = st_dap + SE;
  S* st_E = st_dap + 2 * SE;
  float* wsum = (float*)(p + 3 * stg_bytes<S, PB2_NPX>());
  double* gscr = (double*)(wsum + PB2_NW * PA2_NQ * 32);
  int* flag = (int*)(gscr + (PB2_NT / 64) * 64);
  const int gi = wave >> 1, mt = wave & 1;                  // waves 0-3: a_w / a_u tile rows
  const bool do_wg = att_bwd && wave < 4 && !(PT_ABL(a.ablate) & 16);
  const S* dgsrc = a.conv_done ? a.dgE : a.dgEp;
  PT_TR(a, PT_K_PW_BA, 0);

  auto row_off = [&](int set) { return clip_off(b) + ((size_t)(y0 + set * 4) * IMG + px0) * C; };
  auto tail_load = [&](int set, int ln) {
    Pa2In<S> w;
    const size_t ro = row_off(set);
    w.dgE = PrPk<S>{};
    w.dAt = PrPk<S>{};
    w.Et = zero8();
    if (att_bwd) {
      if (head) {
        w.dgE = pr_load_pk<S>(dgsrc + ro, ln);
        w.Et = prEh(a, t, ro, ln);
      }
      if constexpr (HG) w.dAt = pr_load_pk<S>(a.dAt + ro, ln);
    }
    w.Iv = zero8(); w.Eo = zero8();
    w.ce = PrPk<S>{}; w.eg = PrPk<S>{}; w.dEn = PrPk<S>{};
    if (head) {
      w.Iv = prIh(a, t, ro, ln);
      w.ce = pr_load_pk<S>(a.ce + t * fs + ro, ln);
      w.eg = pr_load_pk<S>(a.eg + t * fs + ro, ln);
      if (t > 0) w.Eo = prE(a, t - 1, ro, ln);
      if (tail) w.dEn = pr_load_pk<S>(a.dEn + ro, ln);
    }
    return w;
  };
  const Pa2In<S> in = tail_load(0, lane);
  float* sp = slab_p + gi * 1024 + (16 * mt + 4 * g4) * 32 + n;     // slab gates 0 (a_w), 1 (a_u)
  float wold[2][4];
  const int so = tid < PA2_NQ * 32 ? SLAB_G + kPa2Slot[tid >> 5] * 32 + (tid & 31) : 0;
  const float sold = tid < PA2_NQ * 32 ? slab_p[so] : 0.f;
  if (tail) stage_x(a.x, a.xu8, xs, b, tt, T, y0, 4 * NSET, tid, PB2_NT, a.ntx, a.nty);
  __syncthreads();
  PT_TR(a, PT_K_PW_BA, 2);
  f32x4 wacc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  Pa2In<S> in1;

  auto set_body = [&](const int set, const Pa2In<S> in) {
    if constexpr ((PT_PRIO & 4) != 0) prio_by_step(set);
    int tl = tid;
    if constexpr (NSET > 1) asm volatile("" : "+v"(tl));
    const int lane = tl & 63, n = lane & 15, g4 = lane >> 4;
    const size_t ro = row_off(set);
    const f32x8& Iv = in.Iv;
    const f32x8& Eo = in.Eo;
    f32x8 GE = zero8();
    if (!tail) GE = pr_load<float>(a.GEfin + ro, lane);
    f32x2 sm[PA2_NQ];
#pragma unroll
    for (int q = 0; q < PA2_NQ; ++q) sm[q] = f32x2{-0.f, -0.f};
    if (tail) {
      const f32x4* xr = xs + set * PB2_NPX + px0 + 4 * g4;
      float w0[2], w1[2], w2[2], bp[2];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int c = 2 * n + k;
        w0[k] = a.wpre[c * 3 + 0]; w1[k] = a.wpre[c * 3 + 1]; w2[k] = a.wpre[c * 3 + 2]; bp[k] = a.bpre[c];
      }
      f32x8 z, xv;                           // z: nl'(stem pre-activation)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f32x4 xin = xr[i];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const float zr = w0[k] * xin[0] + w1[k] * xin[1] + w2[k] * xin[2] + bp[k];
          float f, d;
          Act<ACT>::fd(zr, f, d);
          xv[4 * k + i] = f;
          z[4 * k + i] = d;
        }
      }
      // this kernel's share of d xbn_tt (a_w^T d_att_pre); k_pw_bb adds the
      // inhibition path's share to the same stem-gradient sums itself
      f32x8 dx = zero8();
      if (head || HG) {
        const f32x8 dgE = pr_widen(in.dgE);
        const f32x8 dAt = pr_widen(in.dAt);
        const f32x8& Et = in.Et;
        const f32x2 gb0 = pr_par(a.gb[0], lane), gb1 = pr_par(a.gb[1], lane);
        f32x8 gpre;
        {
          const PrA<S> ax = pr_to_a<S>(scr, rb8(RND_G(a), xv), lane);
          const PrA<S> ae = pr_to_a<S>(scr, rb8(RND_G(a), Et), lane);
          gpre = pr_mm<S>(ax, a.g16f[0], zero8(), lane);
          gpre = pr_mm<S>(ae, a.g16f[1], gpre, lane);
        }
        f32x8 att, dap;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int k = e >> 2;
          att[e] = sigm_b(gpre[e], sig_nb(gb0[k] + gb1[k]));
          const float datt = HG ? dgE[e] * Et[e] + dAt[e] : dgE[e] * Et[e];
          dap[e] = datt * att[e] * (1.f - att[e]);
          sm[2][k] += dap[e];
        }
        pr_stage<S, PB2_NPX>(st_dap, dap, px0, lane);
        pr_stage<S, PB2_NPX>(st_xv, xv, px0, lane);
        pr_stage<S, PB2_NPX>(st_E, Et, px0, lane);
        const PrA<S> pd = pr_to_a<S>(scr, rb8(RND_G(a), dap), lane);
        if (head) {
          const f32x8 dEn = pr_widen(in.dEn);
#pragma unroll
          for (int e = 0; e < 8; ++e) GE[e] = dEn[e] + dgE[e] * att[e];
          GE = pr_mm<S>(pd, a.g16t[1], GE, lane);
        }
        dx = pr_mm<S>(pd, a.g16t[0], dx, lane);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f32x4 xin = xr[i];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const float dz = dx[4 * k + i] * z[4 * k + i];
          sm[5][k] += dz * xin[0];
          sm[6][k] += dz * xin[1];
          sm[7][k] += dz * xin[2];
          sm[8][k] += dz;
        }
      }
    }
    if (head) {
      const float* bst = a.bnstat + (size_t)t * 128;
      const f32x2 m1 = pr_par(bst + 64, lane), rs1 = pr_par(bst + 96, lane);
      const f32x2 kap = pr_par(a.kappa, lane), gam = pr_par(a.gamma, lane);
      const f32x2 bw1 = pr_par(a.bnw1, lane), bb1 = pr_par(a.bnb1, lane);
      const f32x8 cev = pr_widen(in.ce), egv = pr_widen(in.eg);
      f32x8 dIl, dEn, dEp, dcE;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = e >> 2;
        const float xe = (cev[e] - m1[k]) * rs1[k];
        const float cn = bw1[k] * xe + bb1[k];
        const float w = kap[k] * Iv[e] + gam[k];
        const float pe = cn * w;
        float eh, ehd;
        Act<ACT>::fd(pe, eh, ehd);
        const float deg = GE[e] * (eh - Eo[e]);
        const float dpe = GE[e] * egv[e] * ehd;
        const float dce = dpe * w;
        const float dw = dpe * cn;
        sm[3][k] += dw * Iv[e];
        sm[4][k] += dw;
        dIl[e] = dw * kap[k];
        dEn[e] = (1.f - egv[e]) * GE[e];
        dEp[e] = deg * egv[e] * (1.f - egv[e]);
        dcE[e] = dce;
        sm[0][k] += dce;
        sm[1][k] += dce * xe;
      }
      pr_store<S>(a.dIl + ro, lane, rb8(RND_T(a), dIl));
      pr_store<S>(a.dEn + ro, lane, rb8(RND_T(a), dEn));
      pr_store<S>(a.dEp + ro, lane, rb8(RND_T(a), dEp));
      pr_store<S>(a.dcE + ro, lane, rb8(RND_T(a), dcE));
    }
    if (set + 1 < NSET) in1 = tail_load(set + 1, lane);
#pragma unroll
    for (int q = 0; q < PA2_NQ; ++q) {
      f32x2 v = sm[q];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        v[k] += __shfl_xor(v[k], 16);
        v[k] += __shfl_xor(v[k], 32);
      }
      f32x2* ws = (f32x2*)(wsum + (wave * PA2_NQ + q) * 32 + 2 * n);
      if (lane < 16) *ws = set == 0 ? v : *ws + v;
    }
    __syncthreads();
    if (do_wg) pr_wgrad_acc<S, PB2_NPX>(st_dap, gi == 0 ? st_xv : st_E, mt, wacc, lane);
    if (set + 1 < NSET) __syncthreads();                  // the operand slots are reused
  };
  set_body(0, in);
  if constexpr (NSET > 1) set_body(1, in1);
  if constexpr (NSET > 2) set_body(2, in1);
  if constexpr (NSET > 3) set_body(3, in1);
  static_assert(NSET <= 4, "set bodies");
  PT_TR(a, PT_K_PW_BA, 3);
  if (do_wg) {
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int i = 0; i < 4; ++i) wold[nt][i] = sp[i * 32 + 16 * nt];
  }
  PT_TR(a, PT_K_PW_BA, 4);
  const bool bn = head && !(PT_ABL(a.ablate) & 8);
  const BnSlot bo = bnb_slot(a, t, 1, B * WGPC);
  float bv = 0.f;
  if (tid < PA2_NQ * 32) {
    const int q = tid >> 5, c = tid & 31;
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < PB2_NW; ++w) s += wsum[(w * PA2_NQ + q) * 32 + c];
    bv = s;
    if (!(PT_ABL(a.ablate) & 32)) slab_p[so] = sold + s;
  }
  if (do_wg) {
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int i = 0; i < 4; ++i) sp[i * 32 + 16 * nt] = wold[nt][i] + wacc[nt][i];
  }
  PT_TR(a, PT_K_PW_BA, 5);
  if (bn) bn_publish<PB2_NT, false>(bo, blockIdx.x, bv, tid, flag, gscr);
  PT_TR(a, PT_K_PW_BA, 6);
}


// Band geometry by halo width PAD (k <= 7: 3, k > 7: 7): D rows per band (so
// that the band buffers fit in LDS) and buffers (2 = double-buffered; f32 at
// PAD 7 has room for one).
template <class S, int PAD> constexpr int wg_rb() {
  return sizeof(S) == 2 ? (PAD == PADMAX ? 8 : 4) : (PAD == PADMAX ? 4 : 2);
}
template <class S, int PAD> constexpr int wg_nbuf() { return sizeof(S) == 4 && PAD != PADMAX ? 1 : 2; }
template <class S, int PAD> constexpr int wg_xr() { return wg_rb<S, PAD>() + 2 * PAD; }
constexpr int WG_NACC = 13;            // f32: accumulator tiles per wave (taps tap0 + wave + 4 m)
// f32 taps per wave and group actually used: 13 at PAD 3 (49 taps, one
// group); 8 at PAD 7 (the single-buffered band needs the registers)
template <int PAD> constexpr int wg_nacc() { return PAD == PADMAX ? WG_NACC : 8; }
template <class S, int PAD>
constexpr int wgrad_band_elems() {
  return wg_xr<S, PAD>() * tile_w<PAD>() * C + wg_rb<S, PAD>() * IMG * C;
}
template <class S, int PAD>
constexpr int wgrad_lds_bytes() {
  return wg_nbuf<S, PAD>() * wgrad_band_elems<S, PAD>() * (int)sizeof(S);
}
// Tap groups (grid.z): the accumulator tiles of one pass cover at most 7 x 8
// taps (bf16: 7 kernel rows x 2 columns per wave) / 52 taps (f32); k > 7
// makes several passes over the data, one per group.
inline int wgrad_groups(int K, bool bf16) {
  if (K <= 2 * PADMAX + 1) return 1;
  return bf16 ? ((K + 6) / 7) * ((K + 7) / 8) : (K * K + 4 * wg_nacc<PADBIG>() - 1) / (4 * wg_nacc<PADBIG>());
}

// Unswizzled channels-last band images: the transposed 4x16 block reads
// (ds_read_b64_tr_b16) and the f32 row reads are bank-conflict free on them,
// and every tap is a constant element offset from a per-lane base.
template <int PAD>
__device__ __forceinline__ int wx_off(int row, int col, int ch) { return (row * tile_w<PAD>() + col) * C + ch; }
__device__ __forceinline__ int wd_off(int row, int col, int ch) { return (row * IMG + col) * C + ch; }

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
__device__ __forceinline__ bf16x4 tr_read(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(p));
}
__device__ __forceinline__ bf16x8 tr_read8(const bf16_t* p) {
  return __builtin_shufflevector(tr_read(p), tr_read(p + 4 * C), 0, 1, 2, 3, 4, 5, 6, 7);
}

// One band = (frame, clip, RB D rows): the X rows y0-PAD .. y0+RB-1+PAD
// (interior columns; the PAD halo columns each side stay zero from the
// initial clear, rows outside the image are written as zeros) and the D rows.
template <class S, int PAD, int NTH = NT>
struct WBand {
  static constexpr int CPB = 16 / (int)sizeof(S);
  static constexpr int NCH = C / CPB;
  static constexpr int RB = wg_rb<S, PAD>(), XR = wg_xr<S, PAD>();
  static constexpr int XN = XR * IMG * NCH;            // X chunks (the last pass may be partial)
  static constexpr int XPER = (XN + NTH - 1) / NTH;    // 7 / 10 (PAD 3), 9 / 16 (PAD 7) at NT
  static constexpr int DPER = RB * IMG * NCH / NTH;    // 4 / 4, 2 / 2
  static_assert(RB * IMG * NCH % NTH == 0, "band split");
  // tiled frames only: the 2 PAD halo columns of the X rows come from the left /
  // right neighbour tiles (at 32x32 they stay zero from the initial clear)
  static constexpr int HN = XR * 2 * PAD * NCH;
  static constexpr int HPER = (HN + NTH - 1) / NTH;
  u32x4 x[XPER], d[DPER], hx[HPER];
  int xvalid;                                              // bit j: X chunk j inside the frame
  int hvalid;                                              // bit j: halo chunk j inside the frame

  __device__ __forceinline__ void load(const S* __restrict__ Xs, const S* __restrict__ Ds, int B,
                                       int f, int y0, int tid, int ntx, int nty) {
    const int t = f / B, b = f - t * B;
    const S* xfr = Xs + (size_t)t * B * NPIX * C;
    const S* dsrc = Ds + ((size_t)t * B + b) * NPIX * C;
    const TileLoc L = tile_loc(b, ntx, nty);
    xvalid = 0;
#pragma unroll
    for (int j = 0; j < XPER; ++j) {
      const bool in = XN % NTH == 0 || tid + j * NTH < XN;
      const int idx = in ? tid + j * NTH : 0;
      const int q = idx % NCH, pc = idx / NCH;
      const int col = pc % IMG, row = pc / IMG;
      const int iy = y0 + row - PAD;
      const int dy = iy < 0 ? -1 : (iy >= IMG ? 1 : 0);
      const bool ok = in && L.ty + dy >= 0 && L.ty + dy < nty;
      const int cy = ok ? iy - dy * IMG : 0;
      x[j] = *(const u32x4*)(xfr + clip_off(ok ? b + dy * ntx : b) + (cy * IMG + col) * C + q * CPB);
      xvalid |= ok << j;
    }
    hvalid = 0;
    if (ntx * nty > 1) {
#pragma unroll
      for (int j = 0; j < HPER; ++j) {
        const int idx = tid + j * NTH;
        const int q = idx % NCH, pc = idx / NCH;
        const int k = pc % (2 * PAD), row = pc / (2 * PAD);
        const int ix = k < PAD ? k - PAD : IMG + k - PAD;
        const int iy = y0 + row - PAD;
        const int dy = iy < 0 ? -1 : (iy >= IMG ? 1 : 0), dx = ix < 0 ? -1 : 1;
        const bool ok = idx < HN && L.ty + dy >= 0 && L.ty + dy < nty && L.tx + dx >= 0 &&
                        L.tx + dx < ntx;
        const int cy = ok ? iy - dy * IMG : 0, cx = ok ? ix - dx * IMG : 0;
        hx[j] = *(const u32x4*)(xfr + clip_off(ok ? b + dy * ntx + dx : b) + (cy * IMG + cx) * C +
                                q * CPB);
        hvalid |= ok << j;
      }
    }
#pragma unroll
    for (int j = 0; j < DPER; ++j) {
      const int idx = tid + j * NTH;
      const int q = idx % NCH, pc = idx / NCH;
      d[j] = *(const u32x4*)(dsrc + (y0 * IMG + pc) * C + q * CPB);
    }
  }
  __device__ __forceinline__ void store(S* xt, S* dt, int tid, bool tiled) const {
#pragma unroll
    for (int j = 0; j < XPER; ++j) {
      const int idx = tid + j * NTH;
      if (XN % NTH != 0 && idx >= XN) break;
      const int q = idx % NCH, pc = idx / NCH;
      const int col = pc % IMG, row = pc / IMG;
      const u32x4 z = {0u, 0u, 0u, 0u};
      *(u32x4*)(xt + wx_off<PAD>(row, col + PAD, q * CPB)) = (xvalid >> j) & 1 ? x[j] : z;
    }
    if (tiled) {
#pragma unroll
      for (int j = 0; j < HPER; ++j) {
        const int idx = tid + j * NTH;
        const int q = idx % NCH, pc = idx / NCH;
        const int k = pc % (2 * PAD), row = pc / (2 * PAD);
        const int col = k < PAD ? k : IMG + k;
        const u32x4 z = {0u, 0u, 0u, 0u};
        if (idx < HN) *(u32x4*)(xt + wx_off<PAD>(row, col, q * CPB)) = (hvalid >> j) & 1 ? hx[j] : z;
      }
    }
#pragma unroll
    for (int j = 0; j < DPER; ++j) {
      const int idx = tid + j * NTH;
      const int q = idx % NCH, pc = idx / NCH;
      *(u32x4*)(dt + pc * C + q * CPB) = d[j];
    }
  }
};

// f32: MFMAs of one band for this wave's taps (element offsets toff).
template <int K, int PAD>
__device__ __forceinline__ void wgrad_band(f32x16 (&acc)[WG_NACC], const float* xt, const float* dt,
                                           const int (&toff)[WG_NACC], int lane) {
  constexpr int NACC = wg_nacc<PAD>();
  constexpr int off = PAD - K / 2;
  // k-step = 2 pixels (x0 + h); lane&31 is ci for A, n for B
  const int ch = lane & 31, h = lane >> 5;
  for (int yd = 0; yd < wg_rb<float, PAD>(); ++yd) {
    const int xb = wx_off<PAD>(yd + off, h + off, ch), db = wd_off(yd, h, ch);
    for (int x0 = 0; x0 < IMG; x0 += 2) {
      const float bv = dt[db + x0 * C];
#pragma unroll
      for (int m = 0; m < NACC; ++m) acc[m] = Tr<float>::mma(xt[xb + x0 * C + toff[m]], bv, acc[m]);
    }
  }
}

// bf16: tap-column blocking.  Wave w owns kernel columns kw0 = kwb + 2w, +1
// and the kernel rows kh0 .. kh0+6 (< K) of its group (14 accumulator tiles).
// The band's 16 B fragments (RB D rows x 2 pixel blocks) are read once into
// registers; then for every X row r of the band ONE A fragment per column
// feeds the MFMAs of all taps kh with D row r - kh.  LDS reads per MFMA: 1/7
// for A (was 1 with one tap per A read) -- the old tap-scattered assignment
// was bound by the transposing LDS reads.
constexpr int WG2_NACC = 14;             // acc[j * 7 + kh - kh0]: tap (kh, kw0 + j)
template <int K, int NKW, int PAD>
__device__ __forceinline__ void wgrad_band2(f32x16 (&acc)[WG2_NACC], const bf16_t* xt,
                                           const bf16_t* dt, int kw0, int kh0, int lane) {
  constexpr int off = PAD - K / 2;
  constexpr int RB = wg_rb<bf16_t, PAD>();
  constexpr int NKH = K < 7 ? K : 7;               // kernel rows per group
  const int nkh = K - kh0 < NKH ? K - kh0 : NKH;   // valid in this group (uniform)
  const int grp = lane >> 4, m16 = lane & 15, q = m16 >> 2, pp = m16 & 3;
  const int chb = 16 * (grp & 1) + 4 * pp;
  const int hh = grp >> 1;
  bf16x8 bv[RB][2];
#pragma unroll
  for (int yd = 0; yd < RB; ++yd)
#pragma unroll
    for (int blk = 0; blk < 2; ++blk) bv[yd][blk] = tr_read8(dt + wd_off(yd, blk * 16 + 8 * hh + q, chb));
  // steps st = (X row r, pixel block): A fragments read one step ahead; the
  // sched_barriers keep the compiler from hoisting every read of the unrolled
  // band to the top (which spilled)
  constexpr int NST = (RB + NKH - 1) * 2;
  const int nst = (RB + nkh - 1) * 2;              // X rows this group's taps touch
  auto xaddr = [&](int st) {
    return xt + wx_off<PAD>((st >> 1) + off + kh0, (st & 1) * 16 + 8 * hh + q + off + kw0, chb);
  };
  bf16x8 a0[2], a1[2];
  a0[0] = tr_read8(xaddr(0));
  if constexpr (NKW > 1) a1[0] = tr_read8(xaddr(0) + C);
#pragma unroll
  for (int st = 0; st < NST; ++st) {
    if (st >= nst) break;
    const int r = st >> 1, blk = st & 1, cur = st & 1, nxt = cur ^ 1;
    if (st + 1 < nst) {
      a0[nxt] = tr_read8(xaddr(st + 1));
      if constexpr (NKW > 1) a1[nxt] = tr_read8(xaddr(st + 1) + C);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kh = 0; kh < NKH; ++kh) {
      const int yd = r - kh;
      if (yd >= 0 && yd < RB && kh < nkh) {
        acc[kh] = Tr<bf16_t>::mma(a0[cur], bv[yd][blk], acc[kh]);
        if constexpr (NKW > 1) acc[7 + kh] = Tr<bf16_t>::mma(a1[cur], bv[yd][blk], acc[7 + kh]);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// NTH threads per workgroup, all of them staging the bands.
template <class S, int PAD, int NTH = NT, class Body>
__device__ __forceinline__ void wgrad_run(Body&& body, const S* __restrict__ Xs,
                                          const S* __restrict__ Ds, int B, int T, int g, int nwg,
                                          S* buf, int tid, int ablate, int ntx, int nty) {
  constexpr bool stager = true;                  // every thread stages its share
  const bool tiled = ntx * nty > 1;
  constexpr int BE = wgrad_band_elems<S, PAD>();
  constexpr int NBUF = wg_nbuf<S, PAD>();
  constexpr int RB = wg_rb<S, PAD>();
  constexpr int XE = wg_xr<S, PAD>() * tile_w<PAD>() * C;
  constexpr int NB = IMG / RB;                                  // bands per (frame, clip)
  const int npairs = (B * T - g + nwg - 1) / nwg;
  const int nunits = npairs * NB;
  // clear the buffers once (the X halo columns stay zero)
  for (int i = tid; i < NBUF * BE * (int)sizeof(S) / 16; i += NTH)
    ((u32x4*)buf)[i] = u32x4{0u, 0u, 0u, 0u};
  __syncthreads();
  WBand<S, PAD, NTH> band;
  if (nunits > 0 && stager) {
    band.load(Xs, Ds, B, g, 0, tid, ntx, nty);
    band.store(buf, buf + XE, tid, tiled);
  }
  __syncthreads();
  for (int u = 0; u < nunits; ++u) {
    S* xt = buf + (NBUF == 2 ? (u & 1) * BE : 0);
    S* dt = xt + XE;
    const bool more = u + 1 < nunits;
    // two buffers: the next band's loads are in flight under this band's MFMAs;
    // one buffer (f32, PAD 7): load it after (the staged band would not fit
    // in registers beside the accumulators)
    if constexpr (NBUF == 2)
      if (more && stager && !(PT_ABL(ablate) & 128))
        band.load(Xs, Ds, B, g + ((u + 1) / NB) * nwg, ((u + 1) % NB) * RB, tid, ntx, nty);
    if (!(PT_ABL(ablate) & 64)) body(xt, dt);
    if (more) {
      S* xn = buf + (NBUF == 2 ? ((u + 1) & 1) * BE : 0);
      if constexpr (NBUF == 1) {
        __syncthreads();                              // every wave is done reading the buffer
        if (stager && !(PT_ABL(ablate) & 128))
          band.load(Xs, Ds, B, g + ((u + 1) / NB) * nwg, ((u + 1) % NB) * RB, tid, ntx, nty);
      }
      if (stager && !(PT_ABL(ablate) & 128)) band.store(xn, xn + XE, tid, tiled);
      __syncthreads();
    }
  }
}

// =========================================================================
// k x k weight gradients over all (frame, clip) pairs:
//   dW[n][ci][tap] = sum_{t,b,p} D_t[b][p][n] X_t[b][p + tap][ci]
//   conv 0: (D, X) = (d ci_raw, gE)  -> w_inh;  conv 1: (d ce_raw, I_t) -> w_exc
// The D / X row bands are staged in LDS; per-workgroup partials go to wslab
// [2][nwg][K*K][1024].  grid = (nwg, convs, tap groups).
// =========================================================================
// bf16, k <= 7: 8 waves (WG8_NT threads), wave w owns kernel column w (7
// accumulator tiles), two waves per SIMD hide each other's LDS waits; the
// 4-wave form (two columns per wave, one wave per SIMD) serves k > 7 and f32.
constexpr int WG8_NT = 512;
template <class S, int PAD> constexpr int wgrad_nt() { return sizeof(S) == 2 && PAD == PADMAX ? WG8_NT : NT; }
template <class S, int PAD>
__global__ __launch_bounds__((wgrad_nt<S, PAD>()), 1) void k_wgrad(CellArgs<S> a, float* wslab, int nwg, int conv0) {
  constexpr int NTH = wgrad_nt<S, PAD>();
  constexpr int NKW = NTH == WG8_NT ? 1 : 2;        // kernel columns per wave
  extern __shared__ __attribute__((aligned(16))) char smem[];
  S* buf = (S*)smem;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = blockIdx.x, conv = blockIdx.y + conv0, grp = blockIdx.z;
  const int KK = a.K * a.K;
  const S* Xs = conv == 0 ? a.gE : a.Ic;
  const S* Ds = conv == 0 ? a.dci_s : a.dce_s;

  float* dst = wslab + ((size_t)conv * nwg + g) * KK * 1024;
  if constexpr (sizeof(S) == 2) {
    f32x16 acc[WG2_NACC];
#pragma unroll
    for (int m = 0; m < WG2_NACC; ++m) acc[m] = zero16();
    const int nkwg = (a.K + 7) / 8;                  // column groups (1 for k <= 7)
    const int kh0 = PAD == PADMAX ? 0 : (grp / nkwg) * 7;
    const int kw0 = (PAD == PADMAX ? 0 : (grp % nkwg) * 8) + NKW * wave;
    auto run = [&](auto kc) {
      constexpr int K = decltype(kc)::value;
      // 4 waves: every wave runs two columns; a column kw >= K (wave 3's
      // second at K = 7) reads in-bounds LDS and its tiles are never stored.
      // 8 waves: a wave whose column is >= K only stages and syncs.
      wgrad_run<S, PAD, NTH>(
          [&](const S* xt, const S* dt) {
            if (NKW == 1 && kw0 >= K) return;
            wgrad_band2<K, NKW, PAD>(acc, xt, dt, kw0, kh0, lane);
          },
          Xs, Ds, a.B, a.T, g, nwg, buf, tid, a.ablate, a.ntx, a.nty);
    };
    if constexpr (PAD == PADMAX) {
      switch (a.K) {
        case 7: run(std::integral_constant<int, 7>{}); break;
        case 5: run(std::integral_constant<int, 5>{}); break;
        case 3: run(std::integral_constant<int, 3>{}); break;
        default: run(std::integral_constant<int, 1>{}); break;
      }
    } else {
      switch (a.K) {
        case 15: run(std::integral_constant<int, 15>{}); break;
        case 13: run(std::integral_constant<int, 13>{}); break;
        case 11: run(std::integral_constant<int, 11>{}); break;
        default: run(std::integral_constant<int, 9>{}); break;
      }
    }
    // acc[j * 7 + kh - kh0]: rows ci = cl_x(r,h), cols n = lane&31
#pragma unroll
    for (int m = 0; m < 7 * NKW; ++m) {
      const int kh = kh0 + m % 7, kw = kw0 + m / 7;
      if (kh < a.K && kw < a.K) {
#pragma unroll
        for (int r = 0; r < 16; ++r) dst[(kh * a.K + kw) * 1024 + r * 64 + lane] = acc[m][r];
      }
    }
  } else {
    f32x16 acc[WG_NACC];
#pragma unroll
    for (int m = 0; m < WG_NACC; ++m) acc[m] = zero16();
    constexpr int NACC = wg_nacc<PAD>();
    const int tap0 = grp * 4 * NACC;
    // wave-uniform element offset of each tap; taps beyond K*K (the 13th slot
    // of waves 1-3 at K=7) read tap 0 and their accumulator is never stored,
    // so every MFMA is unconditional (no accumulator copies around branches)
    auto run = [&](auto kc) {
      constexpr int K = decltype(kc)::value;
      int toff[WG_NACC];
#pragma unroll
      for (int m = 0; m < WG_NACC; ++m) {
        const int tap = m < NACC && tap0 + wave + 4 * m < K * K ? tap0 + wave + 4 * m : 0;
        const int kh = tap / K, kw = tap - kh * K;
        toff[m] = (kh * tile_w<PAD>() + kw) * C;
      }
      wgrad_run<S, PAD>(
          [&](const S* xt, const S* dt) { wgrad_band<K, PAD>(acc, (const float*)xt, (const float*)dt, toff, lane); },
          Xs, Ds, a.B, a.T, g, nwg, buf, tid, a.ablate, a.ntx, a.nty);
    };
    if constexpr (PAD == PADMAX) {
      switch (a.K) {
        case 7: run(std::integral_constant<int, 7>{}); break;
        case 5: run(std::integral_constant<int, 5>{}); break;
        case 3: run(std::integral_constant<int, 3>{}); break;
        default: run(std::integral_constant<int, 1>{}); break;
      }
    } else {
      switch (a.K) {
        case 15: run(std::integral_constant<int, 15>{}); break;
        case 13: run(std::integral_constant<int, 13>{}); break;
        case 11: run(std::integral_constant<int, 11>{}); break;
        default: run(std::integral_constant<int, 9>{}); break;
      }
    }
    // acc[m]: rows ci = cl_x(r,h), cols n = lane&31
#pragma unroll
    for (int m = 0; m < NACC; ++m) {
      const int tap = tap0 + wave + 4 * m;
      if (tap < KK) {
#pragma unroll
        for (int r = 0; r < 16; ++r) dst[tap * 1024 + r * 64 + lane] = acc[m][r];
      }
    }
  }
}

// -------------------------------------------------------------------------
// bf16, k = 7, 16 waves (r04, default; PT_WG16=0 selects the 8-wave form).
// The 8-wave form gives wave w kernel column w (7 tiles): SIMD s runs waves s
// and s + 4, so SIMDs 0-2 carry 14 tiles and SIMD 3 seven (wave 7 only
// stages) -- 87.5 % of the MFMA rate at best, and two waves per SIMD hide
// little.  Here the 49 tiles are (column, kernel rows 0-3) and (column,
// kernel rows 4-6) units on 14 of 16 waves, placed so that the SIMDs carry
// 13 / 12 / 12 / 12 tiles (wave w on SIMD w & 3): four waves per SIMD at
// <= 128 VGPRs.  Per band and pixel block the wave streams the X rows of its
// kernel rows once (one A fragment per X row, reused over its 3-4 taps) and
// keeps a 5-row window of D fragments (one read ahead) instead of all 8.
// -------------------------------------------------------------------------
constexpr int WG16_NT = 1024;
constexpr unsigned WG16_BIG = 0x0CCDu;                    // waves with kernel rows 0-3
constexpr unsigned long long WG16_KW = 0xFF65654343212100ull;   // nibble w: column (15: stager)
template <int KH0, int NKH>
__device__ __forceinline__ void wgrad_band16(f32x16 (&acc)[4], const bf16_t* xt, const bf16_t* dt,
                                             int kw, int lane) {
  constexpr int PAD = PADMAX, off = PAD - 3;
  constexpr int RB = wg_rb<bf16_t, PAD>();
  constexpr int ns = RB + NKH - 1;                 // X rows of the unit
  const int grp = lane >> 4, m16 = lane & 15, q = m16 >> 2, pp = m16 & 3;
  const int chb = 16 * (grp & 1) + 4 * pp;
  const int hh = grp >> 1;
#pragma unroll
  for (int blk = 0; blk < 2; ++blk) {
    const bf16_t* xb = xt + wx_off<PAD>(off + KH0, blk * 16 + 8 * hh + q + off + kw, chb);
    const bf16_t* db = dt + wd_off(0, blk * 16 + 8 * hh + q, chb);
    bf16x8 dw[5], av[2];
    dw[0] = tr_read8(db);
    av[0] = tr_read8(xb);
#pragma unroll
    for (int s = 0; s < ns; ++s) {
      const int cur = s & 1;
      // one step ahead: X row s + 1 of this unit, D row s + 1 of the band
      if (s + 1 < ns) av[cur ^ 1] = tr_read8(xb + (s + 1) * tile_w<PAD>() * C);
      if (s + 1 < RB) dw[(s + 1) % 5] = tr_read8(db + (s + 1) * IMG * C);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < NKH; ++j) {              // tap (KH0 + j, kw) pairs X row s with D row s - j
        if (s - j >= 0 && s - j < RB) acc[j] = Tr<bf16_t>::mma(av[cur], dw[(s - j) % 5], acc[j]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// LDS-DMA band staging (untiled frames): three band buffers; band u + 2's rows
// are copied global -> LDS (global_load_lds_dwordx4, 1 KiB per wave-instruction,
// lane-linear: one half interior row) while band u's MFMAs run, and a counted
// vmcnt retires band u + 1 before a raw barrier.  With register staging
// (wgrad_run) the band loads and the MFMAs measured additive
// (profiles/r04_wgrad_ablate.txt).  44 chunks per band (28 X, 16 D), issued
// by the two stager waves (below).
constexpr int WG16_DMA_BUFS = 3;
constexpr int wgrad16_dma_lds_bytes() {
  return WG16_DMA_BUFS * wgrad_band_elems<bf16_t, PADMAX>() * 2 + 1024;
}
template <bool TILED, class Body>
__device__ __forceinline__ void wgrad_run_dma(Body&& body, const bf16_t* __restrict__ Xs,
                                              const bf16_t* __restrict__ Ds, int B, int T, int g, int nwg,
                                              bf16_t* buf, int tid, int wave, int lane, int ablate, int ntx,
                                              int nty) {
  constexpr int PAD = PADMAX;
  constexpr int BE = wgrad_band_elems<bf16_t, PAD>();
  constexpr int RB = wg_rb<bf16_t, PAD>(), XR = wg_xr<bf16_t, PAD>(), NB = IMG / RB;
  constexpr int XE = XR * tile_w<PAD>() * C;
  const int npairs = (B * T - g + nwg - 1) / nwg;
  const int nunits = npairs * NB;
  for (int i = tid; i < WG16_DMA_BUFS * BE * 2 / 16; i += WG16_NT) ((u32x4*)buf)[i] = u32x4{0u, 0u, 0u, 0u};
  __syncthreads();
  // The DMAs are inline asm: the compiler's own LDS-DMA bookkeeping waits
  // vmcnt(0) before every global_load_lds (it cannot tell the destinations
  // apart), which would serialise them.  Addresses are wave-uniform (SGPR base,
  // M0 = LDS byte offset) plus the lane's 16 B.
  const unsigned lds0 = (unsigned)(size_t)(__attribute__((address_space(3))) bf16_t*)buf;
  const unsigned voff = lane * 16;
  auto dma = [&](const bf16_t* src, unsigned ldst) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(src), "s"(ldst) : "memory");
  };
  // Only the two waves without MFMA work (14: the 28 X chunks, 15: the 16 D
  // chunks) stage: the scalar unit is shared by the CU's waves, and the
  // per-chunk address / M0 work on all 16 waves cost ~0.8 us per band.  A row
  // outside the image is zeroed by ds_write and its DMA goes to the scratch
  // KiB, so that each stager has a fixed count in flight (its vmcnt).
  // tiled frames (TILED): the X halo rows come from the tiles above / below,
  // and each row's 3 + 3 halo pixels (192 B each side) from the left / right
  // neighbours as 12-lane DMAs -- wave 14 the left, wave 15 the right ones
  constexpr int NXD = 2 * XR + (TILED ? XR : 0), NDD = 2 * RB + (TILED ? XR : 0);
  const unsigned scr = lds0 + WG16_DMA_BUFS * BE * 2;
  auto issue = [&](int u) {
    if (u >= nunits || wave < 14 || (PT_ABL(ablate) & 128)) return;
    const unsigned xt = lds0 + (unsigned)((u % WG16_DMA_BUFS) * BE * 2);
    const int f = g + (u / NB) * nwg, y0 = (u % NB) * RB;   // frame-clip f = t * B + b
    int ty = 0, tx = 0;
    if constexpr (TILED) {
      const TileLoc L = tile_loc(f % B, ntx, nty);
      ty = L.ty; tx = L.tx;
    }
    // halo pixels of X row `row` on side sd (0 left, 1 right): 12 lanes x 16 B
    auto halo = [&](int row, int sd) {
      const int iy = y0 + row - PAD, dy = iy < 0 ? -1 : (iy >= IMG ? 1 : 0), dx = sd ? 1 : -1;
      const bool ok = ty + dy >= 0 && ty + dy < nty && tx + dx >= 0 && tx + dx < ntx;
      const unsigned d = xt + wx_off<PAD>(row, sd ? IMG + PAD : 0, 0) * 2;
      if (lane < 3 * C * 2 / 16) {
        if (ok) {
          dma(Xs + ((size_t)f + dy * ntx + dx) * NPIX * C + ((iy - dy * IMG) * IMG + (sd ? 0 : IMG - PAD)) * C, d);
        } else {
          *(__attribute__((address_space(3))) u32x4*)(size_t)(d + voff) = u32x4{0u, 0u, 0u, 0u};
          dma(Ds, scr);
        }
      }
    };
    if (wave == 14) {
#pragma unroll
      for (int row = 0; row < XR; ++row) {
        const int iy = y0 + row - PAD, dy = iy < 0 ? -1 : (iy >= IMG ? 1 : 0);
        const bool in = TILED ? (ty + dy >= 0 && ty + dy < nty) : dy == 0;
        const bf16_t* xb = Xs + ((size_t)f + dy * ntx) * NPIX * C + (size_t)(iy - dy * IMG) * IMG * C;
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          const unsigned d = xt + wx_off<PAD>(row, PAD + half * 16, 0) * 2;
          if (in) {
            dma(xb + half * 16 * C, d);
          } else {
            *(__attribute__((address_space(3))) u32x4*)(size_t)(d + voff) = u32x4{0u, 0u, 0u, 0u};
            dma(Ds, scr);
          }
        }
        if constexpr (TILED) halo(row, 0);
      }
    } else {
      const bf16_t* db = Ds + (size_t)f * NPIX * C + (size_t)y0 * IMG * C;
#pragma unroll
      for (int k = 0; k < 2 * RB; ++k) dma(db + k * 16 * C, xt + (XE + k * 16 * C) * 2);
      if constexpr (TILED) {
#pragma unroll
        for (int row = 0; row < XR; ++row) halo(row, 1);
      }
    }
  };
  // retire band v's DMAs: this stager's count for a band still in flight behind it
  auto retire = [&](bool more) {
    if (more && wave == 14) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NXD) : "memory");
    else if (more && wave == 15) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NDD) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };
  issue(0);
  issue(1);
  retire(1 < nunits);                     // band 0 landed
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  for (int u = 0; u < nunits; ++u) {
    issue(u + 2);
    int bo = (u % WG16_DMA_BUFS) * BE;
    asm volatile("" : "+s"(bo));          // opaque: no per-buffer address sets hoisted out of the loop
    bf16_t* xt = buf + bo;
    if (!(PT_ABL(ablate) & 64)) body(xt, xt + XE);
    retire(u + 2 < nunits);               // band u + 1 landed
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <bool DMA>
__global__ __launch_bounds__(WG16_NT, 1) void k_wgrad16(CellArgs<bf16_t> a, float* wslab, int nwg, int conv0) {
  constexpr int PAD = PADMAX;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* buf = (bf16_t*)smem;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = blockIdx.x, conv = blockIdx.y + conv0;
  const bf16_t* Xs = conv == 0 ? a.gE : a.Ic;
  const bf16_t* Ds = conv == 0 ? a.dci_s : a.dce_s;
  float* dst = wslab + ((size_t)conv * nwg + g) * 49 * 1024;
  const int kw = (int)((WG16_KW >> (4 * wave)) & 15);
  // one full copy of the band loop per unit shape (a shape branch inside the
  // loop spilled 180 VGPRs)
  auto unit = [&](auto kh0c, auto nkhc) {
    constexpr int KH0 = decltype(kh0c)::value, NKH = decltype(nkhc)::value;
    f32x16 acc[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) acc[m] = zero16();
    auto body = [&](const bf16_t* xt, const bf16_t* dt) {
      if (kw >= 7) return;
      wgrad_band16<KH0, NKH>(acc, xt, dt, kw, lane);
    };
    if constexpr (DMA) {
      if (a.ntx * a.nty > 1)
        wgrad_run_dma<true>(body, Xs, Ds, a.B, a.T, g, nwg, buf, tid, wave, lane, a.ablate, a.ntx, a.nty);
      else
        wgrad_run_dma<false>(body, Xs, Ds, a.B, a.T, g, nwg, buf, tid, wave, lane, a.ablate, 1, 1);
    }
    else wgrad_run<bf16_t, PAD, WG16_NT>(body, Xs, Ds, a.B, a.T, g, nwg, buf, tid, a.ablate, a.ntx, a.nty);
    if (kw >= 7) return;
#pragma unroll
    for (int j = 0; j < NKH; ++j) {
#pragma unroll
      for (int r = 0; r < 16; ++r) dst[((KH0 + j) * 7 + kw) * 1024 + r * 64 + lane] = acc[j][r];
    }
  };
  if ((WG16_BIG >> wave) & 1) unit(std::integral_constant<int, 0>{}, std::integral_constant<int, 4>{});
  else unit(std::integral_constant<int, 4>{}, std::integral_constant<int, 3>{});
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
  S* g16f[6];     // 16x16 B-operand forms for k_pw_bb2 (pt_pr.h): [k 2][KS][64 lanes]
  S* g16t[6];
  int rnd;        // diagnostic: weights rounded to bf16 (f32 path, bit 1048576)
};

template <class S>
__global__ void k_prep(PrepArgs<S> p) {
  using TT = Tr<S>;
  const int K = p.K, KK = K * K;
  const int nconv = KK * TT::KS * 64 * TT::EPL;   // == C*C*K*K
  const int ngate = TT::KS * 64 * TT::EPL;        // == C*C
  const int total = 4 * nconv + 24 * ngate;
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
        dst[r] = (S)rbf(p.rnd, v);
      }
    } else if (e >= 4 * nconv + 12 * ngate) {
      // 16x16 forms: column n of output tile k is channel o = 2n + k; K index =
      // bf16: 8 (lane >> 4) + j, f32 (step s): 4 s + (lane >> 4) (pt_pr.h pr_mm)
      const int e2 = e - 4 * nconv - 12 * ngate;
      const int gi = e2 / ngate, r = e2 % ngate;
      const int gate = gi % 6, tr = gi / 6;
      int lane, kk;
      if constexpr (sizeof(S) == 2) {
        const int j = r % 8;
        lane = (r / 8) % 64;
        kk = 8 * (lane >> 4) + j;
      } else {
        lane = r % 64;
        kk = 4 * ((r / 64) % 8) + (lane >> 4);
      }
      const int o = 2 * (lane & 15) + r / 512;
      const float* G = p.g[gate];
      const float v = tr == 0 ? G[o * C + kk] : G[kk * C + o];
      (tr == 0 ? p.g16f[gate] : p.g16t[gate])[r] = (S)rbf(p.rnd, v);
    } else {
      const int e2 = e - 4 * nconv;
      const int gi = e2 / ngate, r = e2 % ngate;
      const int gate = gi % 6, tr = gi / 6;
      const int j = r % TT::EPL, l = (r / TT::EPL) % 64, ks = r / (TT::EPL * 64);
      const int n = l & 31, h = l >> 5, kc = frag_chan<S>(ks, h, j);
      const float* G = p.g[gate];
      const float v = tr == 0 ? G[n * C + kc] : G[kc * C + n];
      (tr == 0 ? p.gf[gate] : p.gt[gate])[r] = (S)rbf(p.rnd, v);
    }
  }
}

// ---------------------------------------------------------------- reductions
struct ReduceArgs {
  int B, K, nwg;
  int part;             // 0: the per-clip slabs (all but the k x k weights); 1: the k x k weights
  int Cu;               // the caller's channel count (<= 32); padded channels are dropped
  const float* slab;    // [rows][SLAB]
  const float* wslab;   // [2][nwg][K*K][16 r][64 lanes] (accumulator tiles, lane-linear)
  pt_cell_grads g;
};

// Deterministic strided sum of n floats (stride in floats) with 16 loads in
// flight per thread (a serial chain of dependent loads made this kernel
// latency-bound at ~0.6 ms).
__device__ __forceinline__ float strided_sum(const float* __restrict__ p, size_t stride, int n) {
  float acc[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) acc[j] = 0.f;
  int i = 0;
  for (; i + 16 <= n; i += 16) {
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] += p[(size_t)(i + j) * stride];
  }
  for (; i < n; ++i) acc[0] += p[(size_t)i * stride];
#pragma unroll
  for (int w = 8; w >= 1; w >>= 1)
#pragma unroll
    for (int j = 0; j < w; ++j) acc[j] += acc[j + w];
  return acc[0];
}

// k_reduce part 0 in two levels: the B * PW_PARTS slab partitions summed in
// RED_NG contiguous groups (fixed order), then the group sums (k_reduce on
// the RED_NG rows).  One level had 26 workgroups each walking 2048
// partitions: ~100 us, latency-bound.
constexpr int RED_NG = 32;
__global__ void k_slab_partial(const float* __restrict__ slab, float* __restrict__ tmp, int rows) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x, g = blockIdx.y;
  if (e >= SLAB) return;
  const int r0 = (int)((long)g * rows / RED_NG), r1 = (int)((long)(g + 1) * rows / RED_NG);
  tmp[(size_t)g * SLAB + e] = strided_sum(slab + (size_t)r0 * SLAB + e, SLAB, r1 - r0);
}
__global__ void k_reduce(ReduceArgs r) {
  const int KK = r.K * r.K;
  const int n_small = SLAB;                  // slab entries
  const int n_w = 2 * KK * 1024;             // conv weights
  // part 1: both k x k weights; 2: w_inh only; 3: w_exc only (the three-part
  // gradient exchange, pt_cell_dist.grads_mid_event)
  const int e0 = r.part == 0 ? 0 : n_small + (r.part == 3 ? KK * 1024 : 0);
  const int e1 = r.part == 0 ? n_small : n_small + (r.part == 2 ? KK * 1024 : n_w);
  for (int e = e0 + blockIdx.x * blockDim.x + threadIdx.x; e < e1; e += gridDim.x * blockDim.x) {
    if (e < n_small) {
      const float s = strided_sum(r.slab + e, SLAB, r.B);
      if (e < SLAB_G) {
        const int gate = e / 1024, n = (e % 1024) / 32, ci = e % 32;
        if (r.g.gate_w[gate] && n < r.Cu && ci < r.Cu) r.g.gate_w[gate][n * r.Cu + ci] = s;
      } else {
        const int slot = (e - SLAB_G) / 32, c = (e - SLAB_G) % 32;
        if (c >= r.Cu) continue;
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
      // wslab tiles are stored lane-linear (k_wgrad: [r][lane] of the 32x32
      // accumulator, 256-B stores): n = lane & 31, ci = cl_x(r, lane >> 5)
      const int tap = rem / 1024, nc = rem % 1024, n = nc & 31, ci = cl_x(nc >> 6, (nc >> 5) & 1);
      const float s = strided_sum(r.wslab + ((size_t)conv * r.nwg * KK + tap) * 1024 + nc,
                                  (size_t)KK * 1024, r.nwg);
      float* W = conv == 0 ? r.g.w_inh : r.g.w_exc;
      if (W && n < r.Cu && ci < r.Cu) W[(n * r.Cu + ci) * KK + tap] = s;
    }
  }
}

// channels-last tiles [B tiles][32][32][C] (S)  <->  NCHW fp32 frames of the
// caller's Cu <= 32 channels (the padded channels are dropped / zero)
__device__ __forceinline__ size_t nchw_off(int v, int pix, int c, int T, int t, int ntx, int nty,
                                           int Cu) {
  const TileLoc L = tile_loc(v, ntx, nty);
  const int W = ntx * IMG;
  return (((size_t)L.b * T + t) * Cu + c) * ((size_t)nty * IMG * W) +
         (size_t)(L.ty * IMG + (pix >> 5)) * W + L.tx * IMG + (pix & 31);
}
// CL rows <-> NCHW: one workgroup per (tile, image row), the 32 px x 32 ch
// row transposed through LDS so both sides are read / written contiguously.
// grid = tiles * IMG, 256 threads.
template <class S>
__global__ __launch_bounds__(256) void k_to_nchw(const S* __restrict__ src, float* __restrict__ dst, int B,
                                                 int T, int t, int ntx, int nty, int Cu) {
  // dst [clips][T][Cu][H][W] (T=1,t=0 for a single frame); B = tiles
  __shared__ float tl[IMG][C + 1];
  const int v = blockIdx.x / IMG, y = blockIdx.x % IMG;
  const S* row = src + ((size_t)v * NPIX + (size_t)y * IMG) * C;
  for (int i = threadIdx.x; i < IMG * C; i += 256) tl[i / C][i % C] = ldg(row + i);
  __syncthreads();
  for (int i = threadIdx.x; i < IMG * C; i += 256) {
    const int c = i / IMG, px = i % IMG;
    if (c < Cu) dst[nchw_off(v, y * IMG + px, c, T, t, ntx, nty, Cu)] = tl[px][c];
  }
}
// The same for a state (E) of the bf16 cell: f32 restored from its hi / lo
// planes (CellArgs::Eh / El), a channel pair per 4-B load of each plane.
__global__ __launch_bounds__(256) void k_split_to_nchw(const uint16_t* __restrict__ hi,
                                                       const uint16_t* __restrict__ lo, float* __restrict__ dst,
                                                       int B, int T, int t, int ntx, int nty, int Cu) {
  __shared__ float tl[IMG][C + 1];
  const int v = blockIdx.x / IMG, y = blockIdx.x % IMG;
  const size_t o = ((size_t)v * NPIX + (size_t)y * IMG) * C;
  const uint32_t* wh = (const uint32_t*)(hi + o);
  const uint32_t* wl = (const uint32_t*)(lo + o);
  for (int i = threadIdx.x; i < IMG * C / 2; i += 256) {
    const uint32_t x = wh[i], w = wl[i];
    tl[(2 * i) / C][(2 * i) % C] = __uint_as_float((x << 16) + (uint32_t)((int32_t)(w << 16) >> 16));
    tl[(2 * i) / C][(2 * i) % C + 1] = __uint_as_float((x & 0xffff0000u) + (uint32_t)((int32_t)w >> 16));
  }
  __syncthreads();
  for (int i = threadIdx.x; i < IMG * C; i += 256) {
    const int c = i / IMG, px = i % IMG;
    if (c < Cu) dst[nchw_off(v, y * IMG + px, c, T, t, ntx, nty, Cu)] = tl[px][c];
  }
}
__global__ __launch_bounds__(256) void k_from_nchw(const float* __restrict__ src, float* __restrict__ dst,
                                                   int B, int ntx, int nty, int Cu) {
  __shared__ float tl[IMG][C + 1];
  const int v = blockIdx.x / IMG, y = blockIdx.x % IMG;
  for (int i = threadIdx.x; i < IMG * C; i += 256) {
    const int c = i / IMG, px = i % IMG;
    tl[px][c] = c < Cu ? src[nchw_off(v, y * IMG + px, c, 1, 0, ntx, nty, Cu)] : 0.f;
  }
  __syncthreads();
  float* row = dst + ((size_t)v * NPIX + (size_t)y * IMG) * C;
  for (int i = threadIdx.x; i < IMG * C; i += 256) row[i] = tl[i / C][i % C];
}

// Channel padding (Cu < 32): the caller's parameters copied into 32-channel
// buffers, zero outside [0, Cu) (rows and columns of every weight, biases,
// per-channel and BatchNorm parameters).  A padded channel receives no input
// from a real one (zero weight columns) and sends none (zero weight rows), so
// the real channels compute exactly the Cu-channel model; the padded ones
// stay finite (BatchNorm of an all-zero conv output is 0) and their
// gradients are dropped by k_reduce.  The padded tensors live in the saved
// blob: the backward reads the same values.
struct PadArgs {
  int Cu, KK;
  pt_cell_params src;   // caller layout ([Cu]..., [Cu][Cu][K][K], ...)
  float* dst;           // packed 32-channel copies, layout of pad_layout()
};
struct PadLayout {      // float offsets into PadArgs::dst
  size_t pw, pb, w_exc, w_inh, alpha, mu, gamma, kappa, gw[6], gb[6], bnw[2], bnb[2], total;
};
__host__ __device__ inline PadLayout pad_layout(int KK) {
  PadLayout l{};
  size_t o = 0;
  l.pw = o; o += 32 * 3;
  l.pb = o; o += 32;
  l.w_exc = o; o += (size_t)32 * 32 * KK;
  l.w_inh = o; o += (size_t)32 * 32 * KK;
  l.alpha = o; o += 32; l.mu = o; o += 32; l.gamma = o; o += 32; l.kappa = o; o += 32;
  for (int i = 0; i < 6; ++i) { l.gw[i] = o; o += 1024; }
  for (int i = 0; i < 6; ++i) { l.gb[i] = o; o += 32; }
  for (int i = 0; i < 2; ++i) { l.bnw[i] = o; o += 32; }
  for (int i = 0; i < 2; ++i) { l.bnb[i] = o; o += 32; }
  l.total = o;
  return l;
}
__global__ void k_pad_params(PadArgs a) {
  const PadLayout l = pad_layout(a.KK);
  const int Cu = a.Cu, KK = a.KK;
  auto vec = [&](const float* s, size_t off, size_t e) {       // [32] <- [Cu]
    a.dst[off + e] = s && (int)e < Cu ? s[e] : 0.f;
  };
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < l.total;
       e += (size_t)gridDim.x * blockDim.x) {
    if (e < l.pb) {                                    // preproc [32][3]
      const int c = (int)(e / 3), k = (int)(e % 3);
      a.dst[e] = c < Cu ? a.src.preproc_w[c * 3 + k] : 0.f;
    } else if (e < l.w_exc) {
      vec(a.src.preproc_b, l.pb, e - l.pb);
    } else if (e < l.alpha) {                          // w_exc, w_inh [32][32][KK]
      const bool inh = e >= l.w_inh;
      const size_t r = e - (inh ? l.w_inh : l.w_exc);
      const int n = (int)(r / (32 * KK)), ci = (int)(r / KK % 32), tap = (int)(r % KK);
      const float* W = inh ? a.src.w_inh : a.src.w_exc;
      a.dst[e] = W && n < Cu && ci < Cu ? W[((size_t)n * Cu + ci) * KK + tap] : 0.f;
    } else if (e < l.gw[0]) {                          // alpha, mu, gamma, kappa
      const int which = (int)((e - l.alpha) / 32);
      const float* p4[4] = {a.src.alpha, a.src.mu, a.src.gamma, a.src.kappa};
      vec(p4[which], l.alpha + which * 32, (e - l.alpha) % 32);
    } else if (e < l.gb[0]) {                          // gate weights [32][32]
      const int gi = (int)((e - l.gw[0]) / 1024), r = (int)((e - l.gw[0]) % 1024);
      const int n = r / 32, ci = r % 32;
      a.dst[e] = n < Cu && ci < Cu ? a.src.gate_w[gi][n * Cu + ci] : 0.f;
    } else if (e < l.bnw[0]) {
      const int gi = (int)((e - l.gb[0]) / 32);
      vec(a.src.gate_b[gi], l.gb[gi], (e - l.gb[0]) % 32);
    } else {                                           // bn weights / biases
      const int k = (int)((e - l.bnw[0]) / 32);
      const float* src = k < 2 ? a.src.bn_w[k] : a.src.bn_b[k - 2];
      vec(src, l.bnw[0] + k * 32, (e - l.bnw[0]) % 32);
    }
  }
}
// pt_cell_params view of the padded copies
inline pt_cell_params padded_params(const float* base, int KK, bool no_inh) {
  const PadLayout l = pad_layout(KK);
  pt_cell_params p{};
  p.preproc_w = base + l.pw; p.preproc_b = base + l.pb;
  p.w_exc = base + l.w_exc; p.w_inh = no_inh ? nullptr : base + l.w_inh;
  p.alpha = base + l.alpha; p.mu = base + l.mu; p.gamma = base + l.gamma; p.kappa = base + l.kappa;
  for (int i = 0; i < 6; ++i) { p.gate_w[i] = base + l.gw[i]; p.gate_b[i] = base + l.gb[i]; }
  for (int i = 0; i < 2; ++i) { p.bn_w[i] = base + l.bnw[i]; p.bn_b[i] = base + l.bnb[i]; }
  return p;
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
// the library's other translation units (pt_readout.hip) report through here
__attribute__((visibility("hidden"))) int pt_set_error(int code, const char* msg) {
  snprintf(g_err, sizeof(g_err), "%s", msg);
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
// pt_cell_trace: phase stamps of one frame's launches (diagnostics)
unsigned long long* g_trace = nullptr;
int g_trace_t = -1;

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

// Diagnostic switches (PT_DIAG builds only): PT_CELL_ABLATE
// (phase / precision bits, CellArgs::ablate) and PT_CELL_DEBUG_STOP (end the
// backward sweep after n launches).  The release library never reads them.
int ablate_env() {
#if PT_DIAG
  const char* ab = getenv("PT_CELL_ABLATE");
  return ab ? atoi(ab) : 0;
#else
  return 0;
#endif
}
int debug_stop_env() {
#if PT_DIAG
  const char* e = getenv("PT_CELL_DEBUG_STOP");
  return e ? atoi(e) : 0;
#else
  return 0;
#endif
}

// PT_XCD_MAP=0 (diagnostic builds only, read per call) selects the clip-major workgroup order (wg_split)
int xmap_env() { return PT_SW("PT_XCD_MAP", 1); }

constexpr size_t ALIGN = 256;
inline size_t al(size_t x) { return (x + ALIGN - 1) / ALIGN * ALIGN; }

struct Plan {
  int B, T, K, dt;
  int Cu;             // caller's channels (<= 32); < 32: padded parameter copies at o_pad
  int ntx, nty;       // tiles per frame; B counts tiles (clips * ntx * nty)
  size_t es;          // element size of S
  size_t frame;       // elements per frame tensor (B*NPIX*C)
  // saved offsets
  size_t o_E, o_I, o_Ic, o_gE, o_ci, o_ce, o_eg, o_at, o_bnstat, o_wf[4], o_g[12], o_g16[12], o_pad, saved;
  // workspace offsets
  size_t o_bnf_cnt, o_bnf_part, o_bnf_grp, o_bnb_cnt, o_bnb_part, o_bnb_grp;   // BnSlot storage
  size_t o_bnf_done, o_err;   // persistent forward: group-sum counters [T][2], give-up flag
  size_t o_xflag;             // fused tiled forward: border flags [2][B] (xb_exchange)
  size_t bnf_cnt_bytes, bnb_cnt_bytes;
  size_t o_tr[NTRANS], o_dci, o_dce, o_slab, o_wslab, ws;
  int nwg;
};

int check(const pt_cell_desc* d) {
  if (!d) return fail(PT_ERR_ARG, "null descriptor%s%ld");
  if (d->channels < 1 || d->channels > 32)
    return fail(PT_ERR_UNSUPPORTED, "channels must be in [1, 32]%s (got %ld)", "", d->channels);
  if (d->height < 32 || d->height % 32 || d->height > 1024)
    return fail(PT_ERR_UNSUPPORTED, "height must be a multiple of 32 in [32, 1024]%s (got %ld)", "", d->height);
  if (d->width < 32 || d->width % 32 || d->width > 1024)
    return fail(PT_ERR_UNSUPPORTED, "width must be a multiple of 32 in [32, 1024]%s (got %ld)", "", d->width);
  if (d->ksize < 1 || d->ksize > 15 || (d->ksize & 1) == 0)
    return fail(PT_ERR_UNSUPPORTED, "ksize must be odd and <= 15%s (got %ld)", "", d->ksize);
  if (d->batch < 1 || d->frames < 1) return fail(PT_ERR_ARG, "batch and frames must be >= 1%s%ld");
  if (d->act != PT_ACT_SOFTPLUS && d->act != PT_ACT_TANH) return fail(PT_ERR_ARG, "bad act%s%ld");
  if (d->dtype != PT_DTYPE_F32 && d->dtype != PT_DTYPE_BF16) return fail(PT_ERR_ARG, "bad dtype%s%ld");
  if (d->cell != PT_CELL_INT && d->cell != PT_CELL_HGRU) return fail(PT_ERR_ARG, "bad cell%s%ld");
  if (d->cell == PT_CELL_HGRU && d->no_inh) return fail(PT_ERR_ARG, "no_inh is an InT option%s%ld");
  if (d->x_format != PT_X_F32_NCTHW && d->x_format != PT_X_U8_NTHWC)
    return fail(PT_ERR_ARG, "bad x_format%s (got %ld)", "", d->x_format);
  return 0;
}

inline size_t fbytes_of(const Plan& p) { return al(p.frame * p.T * p.es); }

Plan plan(const pt_cell_desc* d) {
  Plan p{};
  p.ntx = d->width / IMG; p.nty = d->height / IMG;
  p.B = d->batch * p.ntx * p.nty; p.T = d->frames; p.K = d->ksize; p.dt = d->dtype;
  p.es = d->dtype == PT_DTYPE_BF16 ? 2 : 4;
  p.frame = (size_t)p.B * NPIX * C;
  const size_t fbytes = al(p.frame * p.T * p.es);
  size_t o = 0;
  // E, I: f32 cell: f32 arrays; bf16 cell: hi plane then lo plane (CellArgs::Eh /
  // El, Ic / Il), the same 4 bytes per element, and I's hi plane is Ic
  p.o_E = o; o += p.es == 2 ? 2 * fbytes : al(p.frame * p.T * 4);
  p.o_I = o; o += p.es == 2 ? 2 * fbytes : al(p.frame * p.T * 4);
  p.o_gE = o; o += fbytes;
  p.o_ci = o; o += fbytes;
  p.o_ce = o; o += fbytes;
  p.o_eg = o; o += fbytes;
  p.o_at = o; o += d->cell == PT_CELL_HGRU ? fbytes : 0;
  p.o_Ic = p.o_I;                                 // bf16: I's hi plane; f32: I itself
  p.o_bnstat = o; o += al((size_t)p.T * 128 * 4);
  for (int i = 0; i < 4; ++i) { p.o_wf[i] = o; o += al((size_t)C * C * p.K * p.K * p.es); }
  for (int i = 0; i < 12; ++i) { p.o_g[i] = o; o += al((size_t)C * C * p.es); }
  for (int i = 0; i < 12; ++i) { p.o_g16[i] = o; o += al((size_t)C * C * p.es); }
  p.Cu = d->channels;
  p.o_pad = o; o += p.Cu < C ? al(pad_layout(p.K * p.K).total * 4) : 0;
  p.saved = o;
  o = 0;
  // tickets first (the only words cleared per call), then partials and group sums
  // (PT_BN_MODE 0 accumulates into the group sums: they are cleared too)
  p.o_bnf_cnt = o; o += al((size_t)p.T * 2 * NGRP * 4);
  p.o_bnf_done = o; o += al((size_t)p.T * 2 * 4);
  p.o_err = o; o += al(4);
  p.o_xflag = o; o += al((size_t)2 * p.B * 4);
  p.o_bnf_grp = o; o += al((size_t)p.T * 2 * NGRP * 96 * 8);
  p.bnf_cnt_bytes = PT_BN_MODE == 0 ? o - p.o_bnf_cnt : p.o_bnf_grp - p.o_bnf_cnt;
  p.o_bnf_part = o; o += al((size_t)p.T * 2 * p.B * 64 * 4);
  p.o_bnb_cnt = o; o += al((size_t)p.T * 2 * NGRP * 4);
  p.o_bnb_grp = o; o += al((size_t)p.T * 2 * NGRP * 64 * 8);
  p.bnb_cnt_bytes = PT_BN_MODE == 0 ? o - p.o_bnb_cnt : p.o_bnb_grp - p.o_bnb_cnt;
  p.o_bnb_part = o; o += al((size_t)p.T * 2 * p.B * BNB_WG_PER_CLIP * 64 * 4);
  for (int i = 0; i < NTRANS; ++i) { p.o_tr[i] = o; o += al(p.frame * 4); }   // GEfin f32
  p.o_dci = o; o += fbytes;
  p.o_dce = o; o += fbytes;
  p.o_slab = o; o += al((size_t)p.B * PW_PARTS * SLAB * 4);
  p.nwg = p.B * p.T < 256 ? p.B * p.T : 256;
  p.o_wslab = o;              // also k_reduce's group sums (k_slab_partial) before k_wgrad
  o += al(std::max((size_t)2 * p.nwg * p.K * p.K * 1024 * 4, (size_t)RED_NG * SLAB * 4));
  p.ws = o;
  return p;
}

template <class S>
void fill_args(CellArgs<S>& a, const pt_cell_desc* d, const Plan& p, const void* x,
               const pt_cell_params* pr, char* saved, char* ws) {
  using F = typename Tr<S>::frag;
  memset(&a, 0, sizeof(a));
  a.B = p.B; a.T = p.T; a.K = p.K; a.act = d->act; a.no_inh = d->no_inh; a.eps = d->eps;
  a.Cu = p.Cu;
  a.ntx = p.ntx; a.nty = p.nty;
  a.hgru = d->cell == PT_CELL_HGRU;
  a.bn_world = 1;
  a.xmap = xmap_env();
  a.trace = g_trace;
  a.trace_t = g_trace_t;
  a.x = x;
  a.xu8 = d->x_format == PT_X_U8_NTHWC;
  a.ablate = ablate_env();                       // diagnostic builds only
  a.wpre = pr->preproc_w; a.bpre = pr->preproc_b;
  a.alpha = pr->alpha; a.mu = pr->mu; a.gamma = pr->gamma; a.kappa = pr->kappa;
  a.bnw0 = pr->bn_w[0]; a.bnb0 = pr->bn_b[0]; a.bnw1 = pr->bn_w[1]; a.bnb1 = pr->bn_b[1];
  for (int i = 0; i < 6; ++i) a.gb[i] = pr->gate_b[i];
  a.wf_inh = (const F*)(saved + p.o_wf[0]); a.wf_exc = (const F*)(saved + p.o_wf[1]);
  a.wt_inh = (const F*)(saved + p.o_wf[2]); a.wt_exc = (const F*)(saved + p.o_wf[3]);
  for (int i = 0; i < 6; ++i) {
    a.gf[i] = (const F*)(saved + p.o_g[i]);
    a.gt[i] = (const F*)(saved + p.o_g[6 + i]);
    a.g16f[i] = (const typename CellArgs<S>::F16*)(saved + p.o_g16[i]);
    a.g16t[i] = (const typename CellArgs<S>::F16*)(saved + p.o_g16[6 + i]);
  }
  if (p.es == 2) {            // bf16: split planes (CellArgs::Eh); no f32 arrays
    a.E = nullptr; a.I = nullptr;
    a.Eh = (S*)(saved + p.o_E); a.El = (uint16_t*)(saved + p.o_E + fbytes_of(p));
    a.Ic = (S*)(saved + p.o_I); a.Il = (uint16_t*)(saved + p.o_I + fbytes_of(p));
  } else {
    a.E = (float*)(saved + p.o_E); a.I = (float*)(saved + p.o_I);
    a.Eh = nullptr; a.El = nullptr; a.Il = nullptr;
    a.Ic = (S*)(saved + p.o_I);
  }
  a.gE = (S*)(saved + p.o_gE);
  a.ci = (S*)(saved + p.o_ci); a.ce = (S*)(saved + p.o_ce); a.eg = (S*)(saved + p.o_eg);
  a.at = a.hgru ? (S*)(saved + p.o_at) : nullptr;
  a.bnstat = (float*)(saved + p.o_bnstat);
  if (ws) {
    a.bnf_cnt = (unsigned*)(ws + p.o_bnf_cnt);
    a.bnf_part = (float*)(ws + p.o_bnf_part);
    a.bnf_grp = (double*)(ws + p.o_bnf_grp);
    a.bnb_cnt = (unsigned*)(ws + p.o_bnb_cnt);
    a.bnb_part = (float*)(ws + p.o_bnb_part);
    a.bnb_grp = (double*)(ws + p.o_bnb_grp);
    S** tr[NTRANS] = {&a.dEn, &a.dcE, &a.dIl, &a.dEp, &a.dcI, &a.GI, &a.dgEp, &a.dxp,
                      &a.dgE, &a.dIt, &a.dAt, nullptr};
    for (int i = 0; i < NTRANS - 1; ++i) *tr[i] = (S*)(ws + p.o_tr[i]);
    a.GEfin = (const float*)(ws + p.o_tr[NTRANS - 1]);
    a.dci_s = (S*)(ws + p.o_dci); a.dce_s = (S*)(ws + p.o_dce);
    a.slab = (float*)(ws + p.o_slab);
    // (the forward has no backward transients live: the border slots use dEn's)
    a.xch = (S*)(ws + p.o_tr[0]);
    a.xflag = (unsigned*)(ws + p.o_xflag);
    a.xerr = (unsigned*)(ws + p.o_err);
  }
}

#define HIPCHK(expr)                                                              \
  do {                                                                            \
    hipError_t e_ = (expr);                                                       \
    if (e_ != hipSuccess) return fail(PT_ERR_HIP, "HIP error %s at line %ld", hipGetErrorString(e_), __LINE__); \
  } while (0)

template <class K, class A>
void launch_pw(K kern, dim3 grid, size_t lds, hipStream_t st, const A& a, int nt = PW_NT) {
  hipLaunchKernelGGL(kern, grid, dim3(nt), lds, st, a);
}

// (activation, cell) -> kernel instantiation
#define PW_LAUNCH_NT(kern, grid, lds, nt)                                       \
  (a.hgru ? (a.act ? launch_pw(kern<S, 1, 1>, grid, lds, st, a, nt)              \
                   : launch_pw(kern<S, 0, 1>, grid, lds, st, a, nt))             \
          : (a.act ? launch_pw(kern<S, 1, 0>, grid, lds, st, a, nt)              \
                   : launch_pw(kern<S, 0, 0>, grid, lds, st, a, nt)))
#define PW_LAUNCH(kern, grid, lds) PW_LAUNCH_NT(kern, grid, lds, PW_NT)


// (activation, cell) -> fused kernel instantiation: grid = clips, CONV_NT threads
template <class K, class A, class Cv>
void launch_fused(K kern, int nclip, size_t lds, hipStream_t st, const A& a, const Cv& c) {
  hipLaunchKernelGGL(kern, dim3(nclip), dim3(CONV_NT), lds, st, a, c);
}
#define FUSED_LAUNCH_TL(kern, c, TL)                                                                \
  (a.hgru ? (a.act ? launch_fused(kern<S, 1, 1, TL>, p.B, fused_lds_bytes<S>(), st, a, c)             \
                   : launch_fused(kern<S, 0, 1, TL>, p.B, fused_lds_bytes<S>(), st, a, c))            \
          : (a.act ? launch_fused(kern<S, 1, 0, TL>, p.B, fused_lds_bytes<S>(), st, a, c)             \
                   : launch_fused(kern<S, 0, 0, TL>, p.B, fused_lds_bytes<S>(), st, a, c)))
// tiled frames: the border-exchange instantiations (xb_exchange)
#define FUSED_LAUNCH(kern, c) \
  (p.ntx * p.nty > 1 ? FUSED_LAUNCH_TL(kern, c, true) : FUSED_LAUNCH_TL(kern, c, false))

#define SETLDS(kern, bytes) \
  HIPCHK(hipFuncSetAttribute((const void*)(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (bytes)))

template <class S>
int set_lds_attrs() {
  static thread_local bool done = false;   // per host thread; cheap either way
  if (done) return 0;
  SETLDS((k_conv_fwd<S, PADMAX, CONV_NT>), (conv_lds_bytes<S, PADMAX>()));
  SETLDS((k_conv_bwd<S, PADMAX, CONV_NT>), (conv_lds_bytes<S, PADMAX>()));
  SETLDS((k_conv_fwd<S, PADBIG>), (conv_lds_bytes<S, PADBIG>()));
  SETLDS((k_conv_bwd<S, PADBIG>), (conv_lds_bytes<S, PADBIG>()));
  SETLDS((k_bnbwd_fill<S>), conv_lds_bytes<S>());
  SETLDS(k_conv_bwd_band2, band2_lds_bytes());
  SETLDS((k_conv_pw_ba<0, 0>), cpa_lds_bytes<bf16_t>());
  SETLDS((k_conv_pw_ba<0, 1>), cpa_lds_bytes<bf16_t>());
  SETLDS((k_conv_pw_ba<1, 0>), cpa_lds_bytes<bf16_t>());
  SETLDS((k_conv_pw_ba<1, 1>), cpa_lds_bytes<bf16_t>());
  SETLDS((k_pw_fa<S, 0, 0>), (pw_lds_bytes<PWF_RPP, false>()));
  SETLDS((k_pw_fb<S, 0, 0>), (pw_lds_bytes<PWF_RPP, false>()));
  SETLDS((k_pw_ba<S, 0, 0>), (pwa_lds_bytes<S>()));
  SETLDS((k_pw_bb<S, 0, 0>), (pwb_lds_bytes<S>()));
  SETLDS((k_pw_fa<S, 0, 1>), (pw_lds_bytes<PWF_RPP, false>()));
  SETLDS((k_pw_fb<S, 0, 1>), (pw_lds_bytes<PWF_RPP, false>()));
  SETLDS((k_pw_ba<S, 0, 1>), (pwa_lds_bytes<S>()));
  SETLDS((k_pw_bb<S, 0, 1>), (pwb_lds_bytes<S>()));
  SETLDS((k_pw_fa<S, 1, 0>), (pw_lds_bytes<PWF_RPP, false>()));
  SETLDS((k_pw_fb<S, 1, 0>), (pw_lds_bytes<PWF_RPP, false>()));
  SETLDS((k_pw_ba<S, 1, 0>), (pwa_lds_bytes<S>()));
  SETLDS((k_pw_bb<S, 1, 0>), (pwb_lds_bytes<S>()));
  SETLDS((k_pw_fa<S, 1, 1>), (pw_lds_bytes<PWF_RPP, false>()));
  SETLDS((k_pw_fb<S, 1, 1>), (pw_lds_bytes<PWF_RPP, false>()));
  SETLDS((k_pw_ba<S, 1, 1>), (pwa_lds_bytes<S>()));
  SETLDS((k_pw_bb<S, 1, 1>), (pwb_lds_bytes<S>()));
  SETLDS((k_pw_bb2<S, 0, 0>), (pb2_lds_bytes<S>()));
  SETLDS((k_pw_bb2<S, 0, 1>), (pb2_lds_bytes<S>()));
  SETLDS((k_pw_bb2<S, 1, 0>), (pb2_lds_bytes<S>()));
  SETLDS((k_pw_bb2<S, 1, 1>), (pb2_lds_bytes<S>()));
  SETLDS((k_pw_ba2<S, 0, 0>), (pa2_lds_bytes<S>()));
  SETLDS((k_pw_ba2<S, 0, 1>), (pa2_lds_bytes<S>()));
  SETLDS((k_pw_ba2<S, 1, 0>), (pa2_lds_bytes<S>()));
  SETLDS((k_pw_ba2<S, 1, 1>), (pa2_lds_bytes<S>()));
  SETLDS((k_fused_fa<S, 0, 0>), fused_lds_bytes<S>());
  SETLDS((k_fused_fa<S, 0, 0, true>), fused_lds_bytes<S>());
  SETLDS((k_fused_fa<S, 0, 1>), fused_lds_bytes<S>());
  SETLDS((k_fused_fa<S, 0, 1, true>), fused_lds_bytes<S>());
  SETLDS((k_fused_fa<S, 1, 0>), fused_lds_bytes<S>());
  SETLDS((k_fused_fa<S, 1, 0, true>), fused_lds_bytes<S>());
  SETLDS((k_fused_fa<S, 1, 1>), fused_lds_bytes<S>());
  SETLDS((k_fused_fa<S, 1, 1, true>), fused_lds_bytes<S>());
  SETLDS((k_fused_fb<S, 0, 0>), fused_lds_bytes<S>());
  SETLDS((k_fused_fb<S, 0, 0, true>), fused_lds_bytes<S>());
  SETLDS((k_fused_fb<S, 0, 1>), fused_lds_bytes<S>());
  SETLDS((k_fused_fb<S, 0, 1, true>), fused_lds_bytes<S>());
  SETLDS((k_fused_fb<S, 1, 0>), fused_lds_bytes<S>());
  SETLDS((k_fused_fb<S, 1, 0, true>), fused_lds_bytes<S>());
  SETLDS((k_fused_fb<S, 1, 1>), fused_lds_bytes<S>());
  SETLDS((k_fused_fb<S, 1, 1, true>), fused_lds_bytes<S>());
  SETLDS((k_persist_fwd<S, 0, 0>), fused_lds_bytes<S>());
  SETLDS((k_persist_fwd<S, 0, 1>), fused_lds_bytes<S>());
  SETLDS((k_persist_fwd<S, 1, 0>), fused_lds_bytes<S>());
  SETLDS((k_persist_fwd<S, 1, 1>), fused_lds_bytes<S>());
  SETLDS((k_wgrad<S, PADMAX>), (wgrad_lds_bytes<S, PADMAX>()));
  SETLDS((k_wgrad<S, PADBIG>), (wgrad_lds_bytes<S, PADBIG>()));
  if constexpr (sizeof(S) == 2) {
    SETLDS(k_wgrad16<false>, (wgrad_lds_bytes<S, PADMAX>()));
    SETLDS(k_wgrad16<true>, wgrad16_dma_lds_bytes());
  }
  done = true;
  return 0;
}

// conv launches: the 38 x 38-tile kernels for k <= 7, the 46 x 46 ones above
template <class S>
void launch_conv_fwd(const Plan& p, hipStream_t st, const ConvArgs<S>& c) {
  if (p.K <= 2 * PADMAX + 1)
    hipLaunchKernelGGL((k_conv_fwd<S, PADMAX, CONV_NT>), dim3(p.B), dim3(CONV_NT), (conv_lds_bytes<S, PADMAX>()), st, c);
  else
    hipLaunchKernelGGL((k_conv_fwd<S, PADBIG>), dim3(p.B), dim3(NT), (conv_lds_bytes<S, PADBIG>()), st, c);
}
// PT_CONV_BAND (diagnostic builds only, read per call): 0 never, 2 the one-addend launches only,
// 1 or unset: always.  First session of r03: k_conv_ba 38.9 -> 37.3 us banded,
// k_conv_bb 41.9 -> 42.8 us (profiles/r03_ablate_band.txt); with the flat
// conv pipeline k_conv_bb is equal either way (38.1 us) and the point-wise
// kernels after it run faster (k_pw_ba 58.5 -> 56.2, k_pw_bb 71.7 -> 69.2 us,
// interleaved; summed device time per step 23.10 -> 22.80 ms).
#ifndef PT_CONV_BAND_DEF
#define PT_CONV_BAND_DEF 3   // r05: k_conv_bwd_band2 (profiles/r05_libab_band2.txt)
#endif
// 3 (r05): the staggered two-band workgroup k_conv_bwd_band2
int band_env() { return PT_SW("PT_CONV_BAND", PT_CONV_BAND_DEF); }
// r06: k_conv_bwd_band2 on tiled frames too (band_halo; default); PT_BAND2_TILED=0
// in diag builds selects the whole-clip conv.  cfg4 (profiles/r06_bench_cpa.txt):
// conv_ba + conv_bb 17.94 -> 17.00 ms per step, 1,450 -> 1,469 clips/s
#ifndef PT_BAND2_TILED_DEF
#define PT_BAND2_TILED_DEF 1
#endif
bool band2_tiled_env() { return PT_SW("PT_BAND2_TILED", PT_BAND2_TILED_DEF) != 0; }
template <class S>
void launch_conv_bwd(const Plan& p, hipStream_t st, const ConvArgs<S>& c) {
  if constexpr (sizeof(S) == 2) {
    const int bm = band_env();
    if (bm == 3 && p.K <= 2 * PADMAX + 1 && (p.ntx * p.nty == 1 || band2_tiled_env())) {
      hipLaunchKernelGGL(k_conv_bwd_band2, dim3(p.B), dim3(BAND2_NT), band2_lds_bytes(), st, c);
      return;
    }
    if ((bm == 1 || (bm == 2 && !c.add1)) && p.K <= 2 * PADMAX + 1 && p.ntx * p.nty == 1) {
      hipLaunchKernelGGL(k_conv_bwd_band, dim3(2 * p.B), dim3(BAND_NT),
                         band_tile_bytes() + CONV_MISC * 4, st, c);
      return;
    }
  }
  if (p.K <= 2 * PADMAX + 1)
    hipLaunchKernelGGL((k_conv_bwd<S, PADMAX, CONV_NT>), dim3(p.B), dim3(CONV_NT), (conv_lds_bytes<S, PADMAX>()), st, c);
  else
    hipLaunchKernelGGL((k_conv_bwd<S, PADBIG>), dim3(p.B), dim3(NT), (conv_lds_bytes<S, PADBIG>()), st, c);
}

template <class S>
ConvArgs<S> conv_args(const CellArgs<S>& a) {
  ConvArgs<S> c;
  memset(&c, 0, sizeof(c));
  c.B = a.B; c.K = a.K; c.ablate = a.ablate;
  c.bnB = a.B * a.bn_world;
  c.ntx = a.ntx; c.nty = a.nty;
  c.xmap = a.xmap;
  c.trace = a.trace; c.trace_t = a.trace_t; c.t = a.t;
  return c;
}

// SyncBN step after a BatchNorm producer launch: the group sums of reduction
// `slot` added into bn_buf + off, then the caller's all-reduce of those nv
// doubles, enqueued on the same stream.
int bn_sync(const pt_cell_dist* dist, const double* grp, int ngrp, int nv, size_t off, hipStream_t st) {
  hipLaunchKernelGGL(k_bn_total, dim3(1), dim3(128), 0, st, grp, ngrp, nv, dist->bn_buf + off);
  HIPCHK(hipGetLastError());
  if (dist->allreduce(dist->user, (int64_t)off, (int64_t)nv) != 0)
    return fail(PT_ERR_ARG, "BatchNorm all-reduce callback failed%s%ld");
  return 0;
}
inline bool syncbn(const pt_cell_dist* dist) { return dist && dist->bn_world > 1; }
// The fused forward (k_fused_fa / k_fused_fb) covers the bf16 InT / hGRU cell
// on single-tile (32x32) frames with k <= 7 and the inhibition branch; other
// configurations, and PT_CELL_FUSED=0, run the split kernels.
bool fused_env() { return PT_SW("PT_CELL_FUSED", 1) != 0; }   // diag builds: read per call
// k_pw_bb2 (the half-row backward point-wise B, r04) by default;
// PT_PWB2=0 (diagnostic builds only, read per call) selects k_pw_bb.
bool pwb2_env() { return PT_SW("PT_PWB2", 1) != 0; }
// k_pw_ba2 (its PR-layout counterpart): opt-in (PT_PWA2=1).  Measured r04
// (B=256 T=64, interleaved): 59.9-60.1 vs 58.4-58.7 us for k_pw_ba, which
// already ran one round of workgroups (4 rows per wave); k_pw_bb2's gain came
// from halving the rounds, not from the layout.
// k_conv_pw_ba (r06, default): PT_CPA=0 in diag builds selects the split
// k_conv_bwd_band2 + k_pw_ba.  A/B (profiles/r06_libab_cpa.txt,
// r06_bench_cpa.txt): 81.4 us per launch vs 31.7 + 53.9 us split, bench
// 20.06 vs 20.11-20.17 ms per step on one box, alternating
#ifndef PT_CPA_DEF
#define PT_CPA_DEF 1
#endif
bool cpa_env() { return PT_SW("PT_CPA", PT_CPA_DEF) != 0; }
#ifndef PT_PWA2_DEF
#define PT_PWA2_DEF 0     // A/B builds: k_pw_ba2 by default
#endif
bool pwa2_env() { return PT_SW("PT_PWA2", PT_PWA2_DEF) == 1; }
// k_wgrad16 (bf16, k = 7) by default; PT_WG16=0 (diagnostic builds only, read per call) selects the
// 8-wave k_wgrad.
bool wg16_env() { return PT_SW("PT_WG16", 1) != 0; }
// its LDS-DMA band staging on untiled frames (PT_WGDMA=0: register staging)
bool wgdma_env() { return PT_SW("PT_WGDMA", 1) != 0; }
// r06: tiled frames through the fused segments too (the border exchange,
// xb_exchange; opt-in, PT_FUSED_TILED=1 in diag builds): bitwise the split
// forward, but at cfg4 (B = 128 clips of 2 x 2 tiles) k_fused_fa / fb take
// 135.4 / 114.3 us per frame against 76.4 + 55.9 / 57.1 + 56.0 us split
// (86.70 vs 87.06 ms per step, profiles/r06_libab_fused_tiled.txt): its
// 146 KB of LDS holds one workgroup per CU, so 512 tile workgroups run in two
// rounds, each as long as the 32x32 launch plus the exchange, while the split
// point-wise kernels run four workgroups per CU
#ifndef PT_FUSED_TILED_DEF
#define PT_FUSED_TILED_DEF 0
#endif
bool fused_tiled_env() { return PT_SW("PT_FUSED_TILED", PT_FUSED_TILED_DEF) != 0; }
bool use_fused(const pt_cell_desc* d, const Plan& p) {
  return fused_env() && d->dtype == PT_DTYPE_BF16 && (p.ntx * p.nty == 1 || fused_tiled_env()) &&
         p.K <= 2 * PADMAX + 1 && !d->no_inh;
}

// Persistent forward (k_persist_fwd): opt-in (PT_CELL_PERSIST=1, read per
// call) on the fused configurations without SyncBN, and only when the B
// workgroups are all resident at once (occupancy x CUs, checked per device).
#ifndef PT_PERSIST_DEF
#define PT_PERSIST_DEF 0     // A/B builds (tools/libab.py): the persistent forward by default
#endif
bool persist_env() { return PT_SW("PT_CELL_PERSIST", PT_PERSIST_DEF) == 1; }
template <class S>
bool persist_fits(int B) {
  static int cap[2] = {-1, -1};           // per storage type; one device per process
  int& c = cap[sizeof(S) == 2];
  if (c < 0) {
    int dev = 0, ncu = 0, per = 0;
    c = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_persist_fwd<S, 0, 0>, CONV_NT,
                                                     fused_lds_bytes<S>()) == hipSuccess)
      c = per * ncu;
  }
  return B <= c;
}

int check_dist(const pt_cell_dist* dist) {
  if (!dist) return 0;
  if (dist->bn_world < 1) return fail(PT_ERR_ARG, "bn_world must be >= 1%s (got %ld)", "", dist->bn_world);
  if (dist->bn_world > 1 && (!dist->bn_buf || !dist->allreduce))
    return fail(PT_ERR_ARG, "SyncBN (bn_world > 1) needs bn_buf and allreduce%s%ld");
  return 0;
}

template <class S>
int run_forward(const pt_cell_desc* d, const void* x, const pt_cell_params* pr, void* saved,
                void* ws, float* e_last, float* gates, const pt_cell_dist* dist, hipStream_t st) {
  const Plan p = plan(d);
  if (int rc = set_lds_attrs<S>()) return rc;
  pt_cell_params padded;
  if (p.Cu < C) {            // fewer channels than the MFMA tile: zero-padded copies (k_pad_params)
    PadArgs pad{p.Cu, p.K * p.K, *pr, (float*)((char*)saved + p.o_pad)};
    hipLaunchKernelGGL(k_pad_params, dim3(256), dim3(256), 0, st, pad);
    padded = padded_params(pad.dst, p.K * p.K, d->no_inh);
    pr = &padded;
  }
  CellArgs<S> a;
  fill_args<S>(a, d, p, x, pr, (char*)saved, (char*)ws);
  a.gates = gates;
  if (syncbn(dist)) { a.bnsync = dist->bn_buf; a.bn_world = dist->bn_world; }
  PrepArgs<S> pa{};
  pa.K = p.K; pa.w_inh = d->no_inh ? nullptr : pr->w_inh; pa.w_exc = pr->w_exc;
  pa.rnd = sizeof(S) == 4 && (a.ablate & 1048576);
  for (int i = 0; i < 6; ++i) {
    pa.g[i] = pr->gate_w[i];
    pa.gf[i] = (S*)((char*)saved + p.o_g[i]);
    pa.gt[i] = (S*)((char*)saved + p.o_g[6 + i]);
    pa.g16f[i] = (S*)((char*)saved + p.o_g16[i]);
    pa.g16t[i] = (S*)((char*)saved + p.o_g16[6 + i]);
  }
  pa.wf_inh = (S*)((char*)saved + p.o_wf[0]); pa.wf_exc = (S*)((char*)saved + p.o_wf[1]);
  pa.wt_inh = (S*)((char*)saved + p.o_wf[2]); pa.wt_exc = (S*)((char*)saved + p.o_wf[3]);
  HIPCHK(zero_async((char*)ws + p.o_bnf_cnt, p.bnf_cnt_bytes, st));     // BN tickets
  timed(PT_K_PREP, st, [&] { hipLaunchKernelGGL(k_prep<S>, dim3(256), dim3(256), 0, st, pa); });
  const dim3 gpf(p.B * PWF_WGPC);
  const size_t lpf = (pw_lds_bytes<PWF_RPP, false>());
  const size_t fs = p.frame;
  ConvArgs<S> ca = conv_args(a), cb = conv_args(a);
  ca.wf = a.wf_inh;
  cb.wf = a.wf_exc;
  if (use_fused(d, p) && p.ntx * p.nty == 1 && !syncbn(dist) && persist_env() && persist_fits<S>(p.B)) {
    // it reads its give-up flag back (a host sync below): illegal under an
    // outer stream capture, so refuse that case with a clear message
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    HIPCHK(hipStreamIsCapturing(st, &cs));
    if (cs != hipStreamCaptureStatusNone)
      return fail(PT_ERR_UNSUPPORTED,
                  "the persistent forward (PT_CELL_PERSIST=1, diagnostic build) cannot run under stream capture%s%ld");
    unsigned* done = (unsigned*)((char*)ws + p.o_bnf_done);
    unsigned* err = (unsigned*)((char*)ws + p.o_err);
    timed(PT_K_PERSIST, st, [&] {
      const size_t lds = fused_lds_bytes<S>();
      if (a.hgru) {
        if (a.act) hipLaunchKernelGGL((k_persist_fwd<S, 1, 1>), dim3(p.B), dim3(CONV_NT), lds, st, a, ca, cb, done, err);
        else hipLaunchKernelGGL((k_persist_fwd<S, 0, 1>), dim3(p.B), dim3(CONV_NT), lds, st, a, ca, cb, done, err);
      } else {
        if (a.act) hipLaunchKernelGGL((k_persist_fwd<S, 1, 0>), dim3(p.B), dim3(CONV_NT), lds, st, a, ca, cb, done, err);
        else hipLaunchKernelGGL((k_persist_fwd<S, 0, 0>), dim3(p.B), dim3(CONV_NT), lds, st, a, ca, cb, done, err);
      }
    });
    // a grid that was not fully resident (another stream holding CUs) gives up
    // its bounded waits and flags err: read it back and fail loudly (this
    // opt-in mode runs without hipGraph replay, pt_cell_forward_dist)
    unsigned herr = 0;
    HIPCHK(hipMemcpyAsync(&herr, err, sizeof(herr), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (herr)
      return fail(PT_ERR_HIP, "persistent forward: the grid was not co-resident (a BatchNorm wait gave up)%s%ld");
    a.t = p.T;
    timed(PT_K_PW_FA, st, [&] { PW_LAUNCH(k_pw_fa, gpf, lpf); });     // closes E_{T-1}
  } else if (use_fused(d, p)) {   // one launch per BatchNorm segment (k_fused_fa / k_fused_fb)
    for (int t = 0; t < p.T; ++t) {
      a.t = t;
      ca.out_raw = a.ci + t * fs; ca.bnout = bnf_slot(a, t, 0);
      timed(PT_K_FUSED_FA, st, [&] { FUSED_LAUNCH(k_fused_fa, ca); });
      if (syncbn(dist))
        if (int rc = bn_sync(dist, ca.bnout.grp, bn_ngrp(p.B), 96, ((size_t)t * 2 + 0) * 96, st)) return rc;
      cb.out_raw = a.ce + t * fs; cb.bnout = bnf_slot(a, t, 1);
      timed(PT_K_FUSED_FB, st, [&] { FUSED_LAUNCH(k_fused_fb, cb); });
      if (syncbn(dist))
        if (int rc = bn_sync(dist, cb.bnout.grp, bn_ngrp(p.B), 96, ((size_t)t * 2 + 1) * 96, st)) return rc;
    }
    a.t = p.T;
    timed(PT_K_PW_FA, st, [&] { PW_LAUNCH(k_pw_fa, gpf, lpf); });     // closes E_{T-1}
  } else
  for (int t = 0; t <= p.T; ++t) {
    a.t = t;
    timed(PT_K_PW_FA, st, [&] { PW_LAUNCH(k_pw_fa, gpf, lpf); });
    if (t == p.T) break;
    if (!d->no_inh) {
      ca.src = a.gE + t * fs; ca.out_raw = a.ci + t * fs; ca.bnout = bnf_slot(a, t, 0);
      timed(PT_K_CONV_FA, st, [&] {
        launch_conv_fwd<S>(p, st, ca); });
      if (syncbn(dist))
        if (int rc = bn_sync(dist, ca.bnout.grp, bn_ngrp(p.B), 96, ((size_t)t * 2 + 0) * 96, st)) return rc;
    }
    timed(PT_K_PW_FB, st, [&] { PW_LAUNCH(k_pw_fb, gpf, lpf); });
    cb.src = a.Ic + t * fs; cb.out_raw = a.ce + t * fs; cb.bnout = bnf_slot(a, t, 1);
    timed(PT_K_CONV_FB, st, [&] {
      launch_conv_fwd<S>(p, st, cb); });
    if (syncbn(dist))
      if (int rc = bn_sync(dist, cb.bnout.grp, bn_ngrp(p.B), 96, ((size_t)t * 2 + 1) * 96, st)) return rc;
  }
  if (e_last) {
    const size_t o = (size_t)(p.T - 1) * p.frame;
    if (p.es == 2)
      hipLaunchKernelGGL(k_split_to_nchw, dim3(p.B * IMG), dim3(256), 0, st, (const uint16_t*)a.Eh + o,
                         (const uint16_t*)a.El + o, e_last, p.B, 1, 0, p.ntx, p.nty, p.Cu);
    else
      hipLaunchKernelGGL(k_to_nchw<float>, dim3(p.B * IMG), dim3(256), 0, st, (const float*)a.E + o, e_last,
                         p.B, 1, 0, p.ntx, p.nty, p.Cu);
  }
  HIPCHK(hipGetLastError());
  return 0;
}

// The backward in phases: 0 = the BPTT sweep and every gradient except
// the two k x k weights (k_reduce part 0); 1 = k_wgrad and those two (part 1).
// pt_cell_dist.grads_early_event is recorded between them, so the caller can
// all-reduce the early gradients on another stream while k_wgrad runs.  With
// grads_mid_event (r06) phase 1 is split by weight: 1 = k_wgrad of w_inh
// alone and its reduction (part 2), the event, then 2 = w_exc (part 3), so
// w_inh's all-reduce runs under w_exc's weight gradient.
template <class S>
int run_backward(const pt_cell_desc* d, const void* x, const pt_cell_params* pr,
                 const void* saved, void* ws, const float* d_e_last, const pt_cell_grads* g,
                 const pt_cell_dist* dist, int phase, hipStream_t st, bool wsplit = false) {
  const Plan p = plan(d);
  if (int rc = set_lds_attrs<S>()) return rc;
  pt_cell_params padded;
  if (p.Cu < C) {            // the forward's padded copies
    padded = padded_params((const float*)((const char*)saved + p.o_pad), p.K * p.K, d->no_inh);
    pr = &padded;
  }
  CellArgs<S> a;
  fill_args<S>(a, d, p, x, pr, (char*)saved, (char*)ws);
  const bool sync = syncbn(dist);
  if (sync) { a.bnsync = dist->bn_buf; a.bn_world = dist->bn_world; }
  ReduceArgs r;
  r.B = p.B * PW_PARTS; r.K = p.K; r.nwg = p.nwg;
  r.slab = (const float*)((char*)ws + p.o_slab);
  r.wslab = (const float*)((char*)ws + p.o_wslab);
  r.g = *g;
  r.Cu = p.Cu;
  if (d->no_inh) { r.g.w_inh = nullptr; r.g.alpha = nullptr; r.g.mu = nullptr;
                   r.g.bn_w[0] = nullptr; r.g.bn_b[0] = nullptr;
                   r.g.gate_w[2] = r.g.gate_w[3] = nullptr; r.g.gate_b[2] = r.g.gate_b[3] = nullptr; }
  if (phase >= 1) {
    float* wslab = (float*)((char*)ws + p.o_wslab);
    // the weights this phase forms: [conv0, conv1]
    const int conv0 = wsplit ? phase - 1 : d->no_inh ? 1 : 0, conv1 = wsplit ? phase - 1 : 1;
    if (d->no_inh) HIPCHK(zero_async(wslab, (size_t)p.nwg * p.K * p.K * 1024 * 4, st));
    timed(PT_K_WGRAD, st, [&] {
      const dim3 grid(p.nwg, conv1 - conv0 + 1, wgrad_groups(p.K, sizeof(S) == 2));
      if constexpr (sizeof(S) == 2)
        if (p.K == 7 && wg16_env()) {
          if (wgdma_env())
            hipLaunchKernelGGL(k_wgrad16<true>, grid, dim3(WG16_NT), wgrad16_dma_lds_bytes(), st, a, wslab, p.nwg,
                               conv0);
          else
            hipLaunchKernelGGL(k_wgrad16<false>, grid, dim3(WG16_NT), (wgrad_lds_bytes<S, PADMAX>()), st, a, wslab,
                               p.nwg, conv0);
          return;
        }
      if (p.K <= 2 * PADMAX + 1)
        hipLaunchKernelGGL((k_wgrad<S, PADMAX>), grid, dim3(wgrad_nt<S, PADMAX>()), (wgrad_lds_bytes<S, PADMAX>()), st, a,
                           wslab, p.nwg, conv0);
      else
        hipLaunchKernelGGL((k_wgrad<S, PADBIG>), grid, dim3(NT), (wgrad_lds_bytes<S, PADBIG>()), st, a,
                           wslab, p.nwg, conv0); });
    r.part = wsplit ? 1 + phase : 1;
    const int n_w = (wsplit ? 1 : 2) * p.K * p.K * 1024;      // one thread per output element
    timed(PT_K_REDUCE, st, [&] {
      hipLaunchKernelGGL(k_reduce, dim3((n_w + 255) / 256), dim3(256), 0, st, r); });
    HIPCHK(hipGetLastError());
    return 0;
  }
  HIPCHK(zero_async((char*)ws + p.o_slab, (size_t)p.B * PW_PARTS * SLAB * 4, st));
  HIPCHK(zero_async((char*)ws + p.o_bnb_cnt, p.bnb_cnt_bytes, st));     // BN tickets
  hipLaunchKernelGGL(k_from_nchw, dim3(p.B * IMG), dim3(256), 0, st, d_e_last,
                     (float*)((char*)ws + p.o_tr[NTRANS - 1]), p.B, p.ntx, p.nty, p.Cu);
  const dim3 gpa(p.B * PWA_WGPC), gpb(p.B * PWB_WGPC);
  const size_t lpa = pwa_lds_bytes<S>(), lpb = pwb_lds_bytes<S>();
  const size_t lcv = conv_lds_bytes<S>();
  const size_t fs = p.frame;
  const float* bst = a.bnstat;
  const size_t sync_b = (size_t)p.T * 2 * 96;     // backward totals in bn_buf
  // SyncBN: the backward sums of reduction (t, bn) all-reduced after their producer
  auto sync_bwd = [&](int t, int bn, int nprod) {
    return sync ? bn_sync(dist, bnb_slot(a, t, bn, nprod).grp, bn_ngrp(nprod), 64,
                          sync_b + ((size_t)t * 2 + bn) * 64, st)
                : 0;
  };
  auto bwd_src = [&](ConvArgs<S>& c, int t, int bn, int nprod) {
    c.bnb = sync ? dist->bn_buf + sync_b + ((size_t)t * 2 + bn) * 64 : bnb_slot(a, t, bn, nprod).grp;
    c.bnb_ngrp = sync ? 1 : bn_ngrp(nprod);
  };
  // diagnostics only (env PT_CELL_DEBUG_STOP = n): return after the sweep's
  // first n launches, leaving the transients as that launch wrote them
  const bool pwb2 = pwb2_env(), pwa2 = pwa2_env();
  const int nprod_b = p.B * (pwb2 ? (a.hgru ? pb2_wgpc<S, 1>() : pb2_wgpc<S, 0>()) : PWB_WGPC);   // BN0 bwd producers
  const int nprod_a = p.B * (pwa2 ? pa2_wgpc<S>() : PWA_WGPC);     // BN1 backward producers
  // k_conv_pw_ba: bf16, 32x32 frames, k <= 7, the staged k_pw_ba (not k_pw_ba2)
  const bool cpa = cpa_env() && sizeof(S) == 2 && p.K <= 2 * PADMAX + 1 &&
                   (p.ntx * p.nty == 1 || band2_tiled_env()) && !pwa2 && PT_PWA_STAGE;
  auto launch_pwa = [&] {
    if (pwa2)
      timed(PT_K_PW_BA, st, [&] { PW_LAUNCH_NT(k_pw_ba2, dim3(nprod_a), (pa2_lds_bytes<S>()), PB2_NT); });
    else
      timed(PT_K_PW_BA, st, [&] { PW_LAUNCH(k_pw_ba, gpa, lpa); });
  };
  const int stop_at = debug_stop_env();
  int n_launch = 0;
  auto stop = [&] { return stop_at > 0 && ++n_launch >= stop_at; };
  a.t = p.T - 1;
  a.conv_done = 0;
  launch_pwa();
  if (stop()) return 0;
  if (int rc = sync_bwd(p.T - 1, 1, nprod_a)) return rc;
  for (int t = p.T - 1; t >= 0; --t) {
    // dI_t = conv^T(BN1-bwd(dcE), w_exc) + dI_local + dI from frame t+1
    ConvArgs<S> cb = conv_args(a);
    cb.t = t; cb.trace_kind = PT_K_CONV_BB;
    cb.dc = a.dcE; cb.raw = a.ce + t * fs; cb.bnstat = bst + (size_t)t * 128 + 64;
    bwd_src(cb, t, 1, nprod_a);
    cb.bnw = a.bnw1; cb.fill_out = a.dce_s + t * fs;
    cb.wf = a.wt_exc; cb.out = a.dIt; cb.add0 = a.dIl; cb.add1 = t < p.T - 1 && !d->no_inh ? a.GI : nullptr;
    timed(PT_K_CONV_BB, st, [&] {
      launch_conv_bwd<S>(p, st, cb); });
    if (stop()) return 0;
    a.t = t;
    if (pwb2)
      timed(PT_K_PW_BB, st, [&] { PW_LAUNCH_NT(k_pw_bb2, dim3(nprod_b), (pb2_lds_bytes<S>()), PB2_NT); });
    else
      timed(PT_K_PW_BB, st, [&] { PW_LAUNCH(k_pw_bb, gpb, lpb); });
    if (stop()) return 0;
    a.conv_done = 0;
    if (!d->no_inh) {
      if (int rc = sync_bwd(t, 0, nprod_b)) return rc;
      // dgE_t = conv^T(BN0-bwd(dcI), w_inh) + e_u^T d_e_pre ; frame 0's conv^T is dead (E_{-1}=0)
      ConvArgs<S> ca = conv_args(a);
      ca.t = t; ca.trace_kind = PT_K_CONV_BA;
      ca.dc = a.dcI; ca.raw = a.ci + t * fs; ca.bnstat = bst + (size_t)t * 128;
      bwd_src(ca, t, 0, nprod_b);
      ca.bnw = a.bnw0; ca.fill_out = a.dci_s + t * fs;
      ca.wf = a.wt_inh; ca.out = a.dgE; ca.add0 = a.dgEp; ca.add1 = nullptr;
      if (t >= 1 && cpa) {      // k_conv_ba(t) + k_pw_ba(t-1) in one launch
        a.conv_done = 1;
        a.t = t - 1;
        if constexpr (sizeof(S) == 2)
          timed(PT_K_CONV_PW_BA, st, [&] {
            const dim3 g(p.B * PWA_WGPC);
            const size_t l = cpa_lds_bytes<bf16_t>();
            if (a.hgru) {
              if (a.act) hipLaunchKernelGGL((k_conv_pw_ba<1, 1>), g, dim3(PW_NT), l, st, a, ca);
              else hipLaunchKernelGGL((k_conv_pw_ba<0, 1>), g, dim3(PW_NT), l, st, a, ca);
            } else {
              if (a.act) hipLaunchKernelGGL((k_conv_pw_ba<1, 0>), g, dim3(PW_NT), l, st, a, ca);
              else hipLaunchKernelGGL((k_conv_pw_ba<0, 0>), g, dim3(PW_NT), l, st, a, ca);
            } });
        if (stop()) return 0;
        if (int rc = sync_bwd(t - 1, 1, nprod_a)) return rc;
        continue;
      } else if (t >= 1) {
        timed(PT_K_CONV_BA, st, [&] {
          launch_conv_bwd<S>(p, st, ca); });
        a.conv_done = 1;
      } else {
        timed(PT_K_CONV_BA, st, [&] {
          hipLaunchKernelGGL((k_bnbwd_fill<S>), dim3(p.B), dim3(NT), lcv, st, ca); });
      }
      if (stop()) return 0;
    }
    a.t = t - 1;
    launch_pwa();
    if (stop()) return 0;
    if (t >= 1)
      if (int rc = sync_bwd(t - 1, 1, nprod_a)) return rc;
  }
  r.part = 0;
  timed(PT_K_REDUCE, st, [&] {
    float* tmp = (float*)((char*)ws + p.o_wslab);      // free until k_wgrad (phase 1)
    hipLaunchKernelGGL(k_slab_partial, dim3((SLAB + 255) / 256, RED_NG), dim3(256), 0, st, r.slab,
                       tmp, r.B);
    ReduceArgs r2 = r;
    r2.slab = tmp;
    r2.B = RED_NG;
    hipLaunchKernelGGL(k_reduce, dim3((SLAB + 255) / 256), dim3(256), 0, st, r2); });
  HIPCHK(hipGetLastError());
  return 0;
}

// Whole forward / backward launch sequences replayed as hipGraphs (pt_graph.h);
// off while kernel timing is enabled (that pass wants per-launch events).
ptg::GraphCache g_graphs;
bool use_graph() {
  return ptg::graphs_enabled() && __atomic_load_n(&g_tm.mask, __ATOMIC_RELAXED) == 0 &&
         !debug_stop_env() && !g_trace;
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

size_t pt_cell_bn_sync_doubles(const pt_cell_desc* d) {
  if (check(d)) return 0;
  return (size_t)d->frames * 2 * (96 + 64);
}

int pt_cell_forward_dist(const pt_cell_desc* d, const void* x, const pt_cell_params* p, void* saved,
                         void* ws, float* e_last, float* gates, const pt_cell_dist* dist,
                         pt_stream_t stream) {
  if (int rc = check(d)) return rc;
  if (!x || !p || !saved || !ws) return fail(PT_ERR_ARG, "null pointer argument%s%ld");
  if (int rc = check_dist(dist)) return rc;
  hipStream_t st = (hipStream_t)stream;
  const bool bf = d->dtype == PT_DTYPE_BF16;
  auto body = [&](hipStream_t s) {
    return bf ? run_forward<bf16_t>(d, x, p, saved, ws, e_last, gates, dist, s)
              : run_forward<float>(d, x, p, saved, ws, e_last, gates, dist, s);
  };
  // SyncBN calls back into the caller between launches, and the persistent
  // forward reads its give-up flag back: direct launches only
  if (!use_graph() || syncbn(dist) || persist_env()) return body(st);
  if (int rc = bf ? set_lds_attrs<bf16_t>() : set_lds_attrs<float>()) return rc;
  ptg::Key k;
  k.add(*d).add(x).add(*p).add(saved).add(ws).add(e_last).add(gates).add(ablate_env())
      .add(fused_env()).add(fused_tiled_env())
      .add(persist_env()).add(xmap_env());
  return g_graphs.run(k.b.data(), k.b.size(), st, PT_ERR_HIP, body);
}

int pt_cell_forward(const pt_cell_desc* d, const void* x, const pt_cell_params* p, void* saved,
                    void* ws, float* e_last, float* gates, pt_stream_t stream) {
  return pt_cell_forward_dist(d, x, p, saved, ws, e_last, gates, nullptr, stream);
}

int pt_cell_export_exc(const pt_cell_desc* d, const void* saved, float* e_seq, pt_stream_t stream) {
  if (int rc = check(d)) return rc;
  if (!saved || !e_seq) return fail(PT_ERR_ARG, "null pointer argument%s%ld");
  const Plan p = plan(d);
  for (int t = 0; t < p.T; ++t) {
    const size_t o = (size_t)t * p.frame;
    if (p.es == 2) {          // E_t restored exactly from its planes (CellArgs::Eh)
      const uint16_t* hi = (const uint16_t*)((const char*)saved + p.o_E);
      const uint16_t* lo = (const uint16_t*)((const char*)saved + p.o_E + fbytes_of(p));
      hipLaunchKernelGGL(k_split_to_nchw, dim3(p.B * IMG), dim3(256), 0, (hipStream_t)stream, hi + o, lo + o,
                         e_seq, p.B, p.T, t, p.ntx, p.nty, p.Cu);
    } else {
      hipLaunchKernelGGL(k_to_nchw<float>, dim3(p.B * IMG), dim3(256), 0, (hipStream_t)stream,
                         (const float*)((const char*)saved + p.o_E) + o, e_seq, p.B, p.T, t, p.ntx, p.nty, p.Cu);
    }
  }
  HIPCHK(hipGetLastError());
  return 0;
}

int pt_cell_backward_dist(const pt_cell_desc* d, const void* x, const pt_cell_params* p,
                          const void* saved, void* ws, const float* d_e_last,
                          const pt_cell_grads* g, const pt_cell_dist* dist, pt_stream_t stream) {
  if (int rc = check(d)) return rc;
  if (!x || !p || !saved || !ws || !d_e_last || !g) return fail(PT_ERR_ARG, "null pointer argument%s%ld");
  if (int rc = check_dist(dist)) return rc;
  hipStream_t st = (hipStream_t)stream;
  const bool bf = d->dtype == PT_DTYPE_BF16;
  const hipEvent_t early = dist ? (hipEvent_t)dist->grads_early_event : nullptr;
  const hipEvent_t mid = dist ? (hipEvent_t)dist->grads_mid_event : nullptr;
  const bool wsplit = mid && !d->no_inh;     // three phases: sweep, w_inh, w_exc
  for (int phase = 0; phase < (wsplit ? 3 : 2); ++phase) {
    auto body = [&](hipStream_t s) {
      return bf ? run_backward<bf16_t>(d, x, p, saved, ws, d_e_last, g, dist, phase, s, wsplit)
                : run_backward<float>(d, x, p, saved, ws, d_e_last, g, dist, phase, s, wsplit);
    };
    int rc;
    if (!use_graph() || syncbn(dist)) {
      rc = body(st);
    } else {
      if ((rc = bf ? set_lds_attrs<bf16_t>() : set_lds_attrs<float>())) return rc;
      ptg::Key k;
      k.add(phase).add(wsplit).add(*d).add(x).add(*p).add(saved).add(ws).add(d_e_last).add(*g).add(ablate_env())
          .add(band_env()).add(pwb2_env()).add(pwa2_env()).add(xmap_env()).add(wg16_env()).add(wgdma_env())
          .add(cpa_env()).add(band2_tiled_env());
      rc = g_graphs.run(k.b.data(), k.b.size(), st, PT_ERR_HIP, body);
    }
    if (rc) return rc;
    if (phase == 0 && early) HIPCHK(hipEventRecord(early, st));
    if (phase == 1 && wsplit) HIPCHK(hipEventRecord(mid, st));
  }
  return 0;
}

int pt_cell_backward(const pt_cell_desc* d, const void* x, const pt_cell_params* p,
                     const void* saved, void* ws, const float* d_e_last, const pt_cell_grads* g,
                     pt_stream_t stream) {
  return pt_cell_backward_dist(d, x, p, saved, ws, d_e_last, g, nullptr, stream);
}

int pt_cell_split_bits(const uint32_t* bits, uint16_t* hi, uint16_t* lo, int64_t n) {
  if (!bits || !hi || !lo || n < 0) return fail(PT_ERR_ARG, "pt_cell_split_bits: null buffer or n < 0%s%ld");
  for (int64_t i = 0; i < n; ++i) {
    const uint32_t hh = split_hh(bits[i]);
    hi[i] = (uint16_t)(hh >> 16);
    lo[i] = split_lo(bits[i], hh);
  }
  return 0;
}

int pt_cell_trace(void* buf, int frame) {
#if PT_DIAG
  g_trace = (unsigned long long*)buf;
  g_trace_t = frame;
  return 0;
#else
  (void)buf; (void)frame;
  return fail(PT_ERR_UNSUPPORTED, "pt_cell_trace needs the diagnostic build (libptcell_diag.so)%s%ld");
#endif
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
// PT_SRC_HASH: hash of the sources this library was built from (ptamd/build.py)
#ifndef PT_SRC_HASH
#define PT_SRC_HASH "unstamped"
#endif
#if PT_DIAG
const char* pt_version(void) { return "pt_cell 0.2 gfx950 diag src " PT_SRC_HASH; }
#else
const char* pt_version(void) { return "pt_cell 0.2 gfx950 src " PT_SRC_HASH; }
#endif

}  // extern "C"
