/*
 * pt_readout.h — C ABI of the fused readout head (gfx950), part of libptcell.so.
 *
 * Replaces the reference's per-model readout op chain, which runs after the
 * recurrent cell on its last excitation state E_T:
 *   models/InT.py:236-241, models/ffhgru_hierarchy.py:258-272,
 *   models/convlstm.py (ConvLSTMVideo readout, same ops):
 *     out = cat([readout_conv(E_T), x[:, 2, 0][:, None]], 1)   1x1 conv C->1
 *     out = target_conv(out)                                    5x5 conv 2->1, pad 2
 *     out = avg_pool2d(out, out.size()[2:])                     global mean
 *     logit = readout_dense(out.reshape(B, -1))                 Linear(1, 1)
 * as one forward kernel (one workgroup per clip) and one backward kernel plus a
 * fixed-order reduction of the parameter gradients (bitwise reproducible).
 *
 * Conventions as pt_cell.h: caller-allocated fp32 device buffers in their
 * PyTorch layouts, explicit stream, 0 or PT_ERR_* (the message from pt_last_error, pt_cell.h).
 */
#ifndef PT_READOUT_H
#define PT_READOUT_H

#include <stdint.h>

#include "pt_cell.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pt_readout_desc {
    int32_t batch;      /* B clips                                              */
    int32_t channels;   /* C channels of E_T (readout_conv in_channels), >= 1   */
    int32_t height;     /* H, W of the frames: (H + 4) * (W + 4) <= 132 * 132   */
    int32_t width;
} pt_readout_desc;

typedef struct pt_readout_params {
    const float* conv_w;    /* readout_conv.weight  [1][C][1][1]  */
    const float* conv_b;    /* readout_conv.bias    [1]           */
    const float* target_w;  /* target_conv.weight   [1][2][5][5]  */
    const float* target_b;  /* target_conv.bias     [1]           */
    const float* dense_w;   /* readout_dense.weight [1][1]        */
    const float* dense_b;   /* readout_dense.bias   [1]           */
} pt_readout_params;

typedef struct pt_readout_grads {   /* same shapes; written (not accumulated) */
    float* conv_w;
    float* conv_b;
    float* target_w;
    float* target_b;
    float* dense_w;
    float* dense_b;
} pt_readout_grads;

/* Bytes of the backward's scratch (per-clip partial gradients). */
int64_t pt_readout_workspace_bytes(const pt_readout_desc* d);

/* e: E_T f32 [B][C][H][W]; tgt: the target-marker channel x[:, 2, 0], f32
 * [B][H][W]; logits: f32 [B]; pooled: f32 [B], the global mean the backward
 * needs (kept by the caller between the two calls). */
int pt_readout_forward(const pt_readout_desc* d, const float* e, const float* tgt,
                       const pt_readout_params* p, float* logits, float* pooled,
                       pt_stream_t stream);

/* d_logits: f32 [B]; d_e: f32 [B][C][H][W] (written); g: parameter gradients
 * (written); workspace: pt_readout_workspace_bytes() bytes. */
int pt_readout_backward(const pt_readout_desc* d, const float* e, const float* tgt,
                        const pt_readout_params* p, const float* pooled, const float* d_logits,
                        float* d_e, const pt_readout_grads* g, void* workspace,
                        pt_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif
