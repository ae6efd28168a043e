// pt_readout.hip — the readout head after the recurrent cell, fused (gfx950).
//
// Reference op chain (models/InT.py:236-241; ffhgru_hierarchy.py:258-272;
// convlstm.py ConvLSTMVideo): readout_conv (1x1, C -> 1) on E_T, concat with
// the target marker x[:, 2, 0], target_conv (5x5, 2 -> 1, pad 2), global
// average pool, readout_dense (Linear 1 -> 1).  As torch ops this is seven
// launches per forward and about as many per backward (MIOpen's naive 5x5
// conv, a 137 us single-thread-per-clip avg_pool2d); here one workgroup per
// clip does the forward, one the backward, and a last launch sums the
// per-clip parameter gradients in clip order (bitwise reproducible).
//
// Backward, with dy = w_d * dlogit / (H W) the same at every output pixel:
//   d target_b = w_d dlogit;  d target_w[ch][tap] = dy * sum_p z_ch[p + tap - 2]
//   dr[q] = dy * sum of target_w[0][tap] over the taps whose output pixel
//           q - (tap - 2) lies inside the frame
//   d E[c][q] = conv_w[c] dr[q];  d conv_w[c] = sum_q dr[q] E[c][q];  d conv_b = sum_q dr[q]
//   d dense_w = dlogit * pooled;  d dense_b = dlogit
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pt_readout.h"

__attribute__((visibility("hidden"))) int pt_set_error(int code, const char* msg);

namespace {

constexpr int RO_NT = 256;
constexpr int RO_MAXPW = 132;          // (H + 4), (W + 4) bound: the padded planes fit LDS

struct RoArgs {
  int B, C, H, W;
  const float* e;
  const float* tgt;
  pt_readout_params p;
  float* logits;
  float* pooled;
  const float* d_logits;
  float* d_e;
  float* part;        // [B][NPAR] per-clip partial gradients
};

__host__ __device__ inline int ro_npar(int C) { return C + 1 + 50 + 1 + 2; }

// Fixed-order workgroup sum (every thread gets the total).
__device__ float block_sum(float v, float* red, int tid) {
  red[tid] = v;
  __syncthreads();
  for (int s = RO_NT / 2; s > 0; s >>= 1) {
    if (tid < s) red[tid] += red[tid + s];
    __syncthreads();
  }
  const float r = red[0];
  __syncthreads();
  return r;
}

// z planes [2][H+4][W+4] with a zero 2-px halo: z0 = readout_conv(E), z1 = tgt
__device__ void ro_planes(const RoArgs& a, int b, float* z, int tid) {
  const int PW = a.W + 4, PH = a.H + 4, HW = a.H * a.W;
  for (int i = tid; i < 2 * PH * PW; i += RO_NT) z[i] = 0.f;
  __syncthreads();
  const float* eb = a.e + (size_t)b * a.C * HW;
  const float cb = a.p.conv_b[0];
  for (int p = tid; p < HW; p += RO_NT) {
    const int y = p / a.W, x = p - y * a.W;
    float r = cb;
    int c = 0;
    for (; c + 8 <= a.C; c += 8) {       // 8 channel loads in flight, then added in order
      float v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = eb[(size_t)(c + k) * HW + p];
#pragma unroll
      for (int k = 0; k < 8; ++k) r += a.p.conv_w[c + k] * v[k];
    }
    for (; c < a.C; ++c) r += a.p.conv_w[c] * eb[(size_t)c * HW + p];
    z[(y + 2) * PW + x + 2] = r;
    z[PH * PW + (y + 2) * PW + x + 2] = a.tgt[(size_t)b * HW + p];
  }
  __syncthreads();
}

__global__ __launch_bounds__(RO_NT) void k_ro_fwd(RoArgs a) {
  extern __shared__ float sm[];
  const int tid = threadIdx.x, b = blockIdx.x;
  const int PW = a.W + 4, PH = a.H + 4, HW = a.H * a.W;
  float* z = sm;
  float* red = sm + 2 * PH * PW;
  ro_planes(a, b, z, tid);
  float wt[50];
#pragma unroll
  for (int i = 0; i < 50; ++i) wt[i] = a.p.target_w[i];
  const float tb = a.p.target_b[0];
  float acc = 0.f;
  for (int p = tid; p < HW; p += RO_NT) {
    const int y = p / a.W, x = p - y * a.W;
    float v = tb;
#pragma unroll
    for (int ch = 0; ch < 2; ++ch)
#pragma unroll
      for (int kh = 0; kh < 5; ++kh)
#pragma unroll
        for (int kw = 0; kw < 5; ++kw) v += wt[ch * 25 + kh * 5 + kw] * z[ch * PH * PW + (y + kh) * PW + x + kw];
    acc += v;
  }
  const float s = block_sum(acc, red, tid) / (float)HW;
  if (tid == 0) {
    a.pooled[b] = s;
    a.logits[b] = a.p.dense_w[0] * s + a.p.dense_b[0];
  }
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// LDS: z planes | dr[HW] | per-wave partial sums [C + 51][RO_NT / 64]
__global__ __launch_bounds__(RO_NT) void k_ro_bwd(RoArgs a) {
  extern __shared__ float sm[];
  constexpr int NW = RO_NT / 64;
  const int tid = threadIdx.x, b = blockIdx.x, lane = tid & 63, wave = tid >> 6;
  const int PW = a.W + 4, PH = a.H + 4, HW = a.H * a.W, C = a.C;
  float* z = sm;
  float* drs = sm + 2 * PH * PW;
  float* wred = drs + HW;
  const float dl = a.d_logits[b];
  const float ds = a.p.dense_w[0] * dl;
  const float dy = ds / (float)HW;
  ro_planes(a, b, z, tid);
  float wt0[25];
#pragma unroll
  for (int i = 0; i < 25; ++i) wt0[i] = a.p.target_w[i];
  float gt[50];                          // window sums of the padded planes (d target_w / dy)
#pragma unroll
  for (int i = 0; i < 50; ++i) gt[i] = 0.f;
  float gcb = 0.f;
  for (int p = tid; p < HW; p += RO_NT) {
    const int y = p / a.W, x = p - y * a.W;
#pragma unroll
    for (int ch = 0; ch < 2; ++ch)
#pragma unroll
      for (int kh = 0; kh < 5; ++kh)
#pragma unroll
        for (int kw = 0; kw < 5; ++kw) gt[ch * 25 + kh * 5 + kw] += z[ch * PH * PW + (y + kh) * PW + x + kw];
    // dr at input pixel p: the taps whose output pixel p - (tap - 2) is inside
    float wsum = 0.f;
#pragma unroll
    for (int kh = 0; kh < 5; ++kh)
#pragma unroll
      for (int kw = 0; kw < 5; ++kw) {
        const int oy = y - (kh - 2), ox = x - (kw - 2);
        if (oy >= 0 && oy < a.H && ox >= 0 && ox < a.W) wsum += wt0[kh * 5 + kw];
      }
    const float dr = dy * wsum;
    drs[p] = dr;
    gcb += dr;
  }
  __syncthreads();
  const float* eb = a.e + (size_t)b * C * HW;
  float* deb = a.d_e + (size_t)b * C * HW;
  auto chan = [&](int c, const float (&ev)[4]) {    // ev: this thread's E[c][tid + k RO_NT], k < 4
    const float wc = a.p.conv_w[c];
    float g = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int p = tid + k * RO_NT;
      if (p < HW) {
        const float dr = drs[p];
        g += dr * ev[k];
        deb[(size_t)c * HW + p] = wc * dr;
      }
    }
    for (int p = tid + 4 * RO_NT; p < HW; p += RO_NT) {
      const float dr = drs[p];
      g += dr * eb[(size_t)c * HW + p];
      deb[(size_t)c * HW + p] = wc * dr;
    }
    g = wave_sum(g);
    if (lane == 0) wred[c * NW + wave] = g;
  };
  int c0 = 0;
  for (; c0 + 4 <= C; c0 += 4) {        // the first 4 pixels of 4 channels in flight at once
    float ev[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int p = tid + k * RO_NT;
        ev[j][k] = p < HW ? eb[(size_t)(c0 + j) * HW + p] : 0.f;
      }
#pragma unroll
    for (int j = 0; j < 4; ++j) chan(c0 + j, ev[j]);
  }
  for (; c0 < C; ++c0) {
    float ev[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int p = tid + k * RO_NT;
      ev[k] = p < HW ? eb[(size_t)c0 * HW + p] : 0.f;
    }
    chan(c0, ev);
  }
  gcb = wave_sum(gcb);
  if (lane == 0) wred[C * NW + wave] = gcb;
#pragma unroll
  for (int i = 0; i < 50; ++i) {
    const float t = wave_sum(gt[i]);
    if (lane == 0) wred[(C + 1 + i) * NW + wave] = t;
  }
  __syncthreads();
  float* prow = a.part + (size_t)b * ro_npar(C);
  for (int j = tid; j < C + 51; j += RO_NT) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) t += wred[j * NW + w];
    prow[j] = j > C ? dy * t : t;
  }
  if (tid == 0) {
    prow[C + 51] = ds;                    // target_b
    prow[C + 52] = dl * a.pooled[b];      // dense_w
    prow[C + 53] = dl;                    // dense_b
  }
}

// parameter gradients: per-clip partials summed in clip order
__global__ void k_ro_reduce(RoArgs a, pt_readout_grads g) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x, C = a.C, np = ro_npar(C);
  if (j >= np) return;
  float s = 0.f;
  int b = 0;
  for (; b + 32 <= a.B; b += 32) {       // 32 loads in flight, added in clip order
    float v[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) v[k] = a.part[(size_t)(b + k) * np + j];
#pragma unroll
    for (int k = 0; k < 32; ++k) s += v[k];
  }
  for (; b < a.B; ++b) s += a.part[(size_t)b * np + j];
  if (j < C) g.conv_w[j] = s;
  else if (j == C) g.conv_b[0] = s;
  else if (j < C + 51) g.target_w[j - C - 1] = s;
  else if (j == C + 51) g.target_b[0] = s;
  else if (j == C + 52) g.dense_w[0] = s;
  else g.dense_b[0] = s;
}

size_t lds_fwd(const pt_readout_desc* d) {
  return (size_t)(2 * (d->height + 4) * (d->width + 4) + RO_NT) * sizeof(float);
}
size_t lds_bwd(const pt_readout_desc* d) {
  return (size_t)(2 * (d->height + 4) * (d->width + 4) + d->height * d->width +
                  (d->channels + 51) * (RO_NT / 64)) * sizeof(float);
}

// One shape check for every entry point: a shape whose BACKWARD does not fit
// the 160 KB of LDS is refused up front (the forward alone would fit up to
// 128 x 128 and only the backward would then fail, mid training step).
int check(const pt_readout_desc* d) {
  if (!d) return pt_set_error(PT_ERR_ARG, "null readout descriptor");
  if (d->batch < 1 || d->channels < 1 || d->height < 1 || d->width < 1)
    return pt_set_error(PT_ERR_ARG, "readout: batch, channels, height, width must be >= 1");
  if (d->height + 4 > RO_MAXPW || d->width + 4 > RO_MAXPW || d->channels > 1024)
    return pt_set_error(PT_ERR_UNSUPPORTED, "readout: frames up to 128 x 128, channels up to 1024");
  if (lds_bwd(d) > 160 * 1024)
    return pt_set_error(PT_ERR_UNSUPPORTED, "readout: the backward's LDS tiles exceed 160 KB at this frame size");
  return 0;
}

int set_lds() {
  static bool done = false;
  if (!done) {
    const int mx = 160 * 1024;
    if (hipFuncSetAttribute((const void*)k_ro_fwd, hipFuncAttributeMaxDynamicSharedMemorySize, mx) != hipSuccess ||
        hipFuncSetAttribute((const void*)k_ro_bwd, hipFuncAttributeMaxDynamicSharedMemorySize, mx) != hipSuccess)
      return pt_set_error(PT_ERR_HIP, "readout: hipFuncSetAttribute failed");
    done = true;
  }
  return 0;
}

}  // namespace

extern "C" {

int64_t pt_readout_workspace_bytes(const pt_readout_desc* d) {
  if (check(d)) return -1;
  return (int64_t)d->batch * ro_npar(d->channels) * (int64_t)sizeof(float);
}

int pt_readout_forward(const pt_readout_desc* d, const float* e, const float* tgt,
                       const pt_readout_params* p, float* logits, float* pooled, pt_stream_t stream) {
  if (int rc = check(d)) return rc;
  if (!e || !tgt || !p || !logits || !pooled) return pt_set_error(PT_ERR_ARG, "readout: null pointer");
  const size_t lds = lds_fwd(d);
  if (int rc = set_lds()) return rc;
  RoArgs a{};
  a.B = d->batch; a.C = d->channels; a.H = d->height; a.W = d->width;
  a.e = e; a.tgt = tgt; a.p = *p; a.logits = logits; a.pooled = pooled;
  hipLaunchKernelGGL(k_ro_fwd, dim3(a.B), dim3(RO_NT), lds, (hipStream_t)stream, a);
  if (hipGetLastError() != hipSuccess) return pt_set_error(PT_ERR_HIP, "readout: forward launch failed");
  return 0;
}

int pt_readout_backward(const pt_readout_desc* d, const float* e, const float* tgt,
                        const pt_readout_params* p, const float* pooled, const float* d_logits,
                        float* d_e, const pt_readout_grads* g, void* workspace, pt_stream_t stream) {
  if (int rc = check(d)) return rc;
  if (!e || !tgt || !p || !pooled || !d_logits || !d_e || !g || !workspace)
    return pt_set_error(PT_ERR_ARG, "readout: null pointer");
  const size_t lds = lds_bwd(d);
  if (int rc = set_lds()) return rc;
  RoArgs a{};
  a.B = d->batch; a.C = d->channels; a.H = d->height; a.W = d->width;
  a.e = e; a.tgt = tgt; a.p = *p; a.pooled = (float*)pooled; a.d_logits = d_logits; a.d_e = d_e;
  a.part = (float*)workspace;
  hipLaunchKernelGGL(k_ro_bwd, dim3(a.B), dim3(RO_NT), lds, (hipStream_t)stream, a);
  const int np = ro_npar(a.C);
  hipLaunchKernelGGL(k_ro_reduce, dim3((np + 63) / 64), dim3(64), 0, (hipStream_t)stream, a, *g);
  if (hipGetLastError() != hipSuccess) return pt_set_error(PT_ERR_HIP, "readout: backward launch failed");
  return 0;
}

}  // extern "C"
