/*
 * pt_lstm.h — C ABI of the MI355X (gfx950) ConvLSTM cell library (libptlstm.so).
 *
 * Drop-in boundary beneath the reference's ConvLSTM (models/convlstm.py):
 *   ConvLSTMCell.forward   models/convlstm.py:84-90   (one step, x/h/c given)
 *   ConvLSTM.forward loop  models/convlstm.py:137-143 (bptt: `timesteps` steps
 *                                                     on a static x, h0=c0=0)
 *   autograd BPTT through that loop, and the training-mode Jacobian penalty
 *   models/convlstm.py:150-161 (l1: two vector-Jacobian products).
 * conv0 + pow2 (:118-119), BN (:146) and conv6 (:147) stay in PyTorch; the
 * library takes the squared conv0 output x and returns h (and c).
 *
 * Conventions as include/pt_cell.h: plain C types, caller-owned buffers (fp32
 * NCHW tensors in their PyTorch layout, an opaque saved blob and workspace),
 * an explicit stream per call, no mutable global state, int status with a
 * thread-local message (pt_lstm_last_error()).
 *
 * Gate order everywhere is the reference's attribute order i, f, c, o
 * (Wxi/Whi, Wxf/Whf, Wxc/Whc, Wxo/Who, models/convlstm.py:63-73).
 */
#ifndef PT_LSTM_H
#define PT_LSTM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* pt_lstm_stream_t;   /* == hipStream_t */

enum { PT_LSTM_OK = 0, PT_LSTM_ERR_ARG = 1, PT_LSTM_ERR_UNSUPPORTED = 2, PT_LSTM_ERR_HIP = 3 };
enum { PT_LSTM_F32 = 0, PT_LSTM_BF16 = 1 };      /* storage + MFMA operand type */
enum { PT_LSTM_H0 = 1, PT_LSTM_C0 = 2 };         /* desc.init_state bits        */

typedef struct pt_lstm_desc {
    int32_t batch;        /* B images                                          */
    int32_t in_channels;  /* input_channels  (25 in ConvLSTM), <= 32           */
    int32_t channels;     /* hidden_channels (25 in ConvLSTM), <= 32           */
    int32_t height;       /* H (32)                                            */
    int32_t width;        /* W (32)                                            */
    int32_t ksize;        /* kernel_size, odd, <= 15 (filt_size, default 15)   */
    int32_t steps;        /* recurrent steps T (timesteps), >= 1               */
    int32_t dtype;        /* PT_LSTM_F32 / PT_LSTM_BF16                        */
    int32_t init_state;   /* PT_LSTM_H0 | PT_LSTM_C0: initial h / c are given  */
    int32_t x_seq;        /* 0: static x [B,cin,H,W] (the reference ConvLSTM,
                             convlstm.py:137-143, recurs on one image);
                             1: one input per step, x [B,cin,T,H,W], x_t =
                             x[:, :, t] (the video adaptation for PathTracker
                             clips)                           */
} pt_lstm_desc;

/* fp32, PyTorch layouts: wx[g] [ch,cin,k,k], bx[g] [ch], wh[g] [ch,ch,k,k]. */
typedef struct pt_lstm_params {
    const float* wx[4];
    const float* bx[4];
    const float* wh[4];
} pt_lstm_params;

/* Gradients (fp32, overwritten; any pointer may be NULL).  d_x shaped like x;
 * d_h0 / d_c0 [B,ch,H,W] (only meaningful when h0 / c0 were given). */
typedef struct pt_lstm_grads {
    float* wx[4];
    float* bx[4];
    float* wh[4];
    float* d_x;
    float* d_h0;
    float* d_c0;
} pt_lstm_grads;

size_t pt_lstm_saved_bytes(const pt_lstm_desc* d);
size_t pt_lstm_workspace_bytes(const pt_lstm_desc* d);

/* T steps of the cell on x (static [B,cin,H,W], or per step [B,cin,T,H,W] when
 * desc.x_seq) from (h0, c0) [B,ch,H,W]
 * (NULL = zeros, as convlstm.py:120-121; must agree with desc.init_state).
 * Writes h_T, c_T [B,ch,H,W] (either may be NULL) and keeps everything the
 * backward / jv calls need in `saved` (prepared weight fragments included). */
int pt_lstm_forward(const pt_lstm_desc* d, const float* x, const pt_lstm_params* p,
                    const float* h0, const float* c0, void* saved, float* h_out, float* c_out,
                    pt_lstm_stream_t stream);

/* BPTT from dL/dh_T (d_h, required) and dL/dc_T (d_c, NULL = 0), using the
 * `saved` blob of the matching forward. */
int pt_lstm_backward(const pt_lstm_desc* d, const void* saved, void* workspace,
                     const float* d_h, const float* d_c, const pt_lstm_grads* g,
                     pt_lstm_stream_t stream);

/* Training-mode Jacobian penalty of the last step (convlstm.py:150-161, l1):
 *   jv = clamp(J_h^T 1 - mu, 0)^2 + clamp(J_c^T 1 - mu, 0)^2      [B,ch,H,W]
 * J_h = dh_{T-1}/dh_{T-2}; J_c = dc_{T-1}/dc_{T-2} along every path (the forget
 * gate and the path through h_{T-2}).  Needs steps >= 2. */
int pt_lstm_jv_penalty(const pt_lstm_desc* d, const void* saved, void* workspace, float mu,
                       float* jv, pt_lstm_stream_t stream);

/* Per-step hidden states h_t, t = 0..T-1, of the forward that filled `saved`,
 * as fp32 [B,ch,T,H,W] (testmode outputs of the clip ConvLSTM: the reference
 * ConvLSTM's testmode collects the per-step h, models/convlstm.py:127-135). */
int pt_lstm_export_h(const pt_lstm_desc* d, const void* saved, float* h_seq,
                     pt_lstm_stream_t stream);

/* Frame stem of the clip ConvLSTM (the stem of InT.py:192,212-213
 * applied per frame): y = softplus(W x + b), a 1x1x1 channel mix over the n
 * voxels of the clip batch into y [B,cout,n] (n = T*H*W, a multiple of 4; cin
 * 1..4, cout 1..32; softplus as torch's F.softplus, beta 1, threshold 20).
 * x is the f32 model input [B,cin,n] (x_u8 = 0) or the raw clip bytes u8
 * [B,n,cin] as the TFRecords hold them (x_u8 = 1, [B,T,H,W,3]; converted
 * as engine.prepare_data does, u / 255 in float64 rounded to f32).
 * The backward recomputes W x + b and writes dW [cout,cin] and db [cout]
 * (either may be NULL) through a workspace of pt_lstm_stem_workspace_bytes(cin)
 * bytes; the stem input never needs a gradient (it is the clip). */
size_t pt_lstm_stem_workspace_bytes(int cin);
int pt_lstm_stem_forward(const void* x, int x_u8, const float* w, const float* b, int B, int cin,
                         int cout, long long n, float* y, pt_lstm_stream_t stream);
int pt_lstm_stem_backward(const void* x, int x_u8, const float* w, const float* b, const float* dy,
                          int B, int cin, int cout, long long n, void* workspace, float* dw,
                          float* db, pt_lstm_stream_t stream);

/* The clip ConvLSTM with its frame stem fused in: desc.x_seq
 * must be 1, desc.init_state 0, desc.in_channels = the stem's outputs.  x is
 * the raw clip batch the stem takes (f32 [B,cin_s,T,H,W], or x_u8 = 1: u8
 * [B,T,H,W,cin_s]; cin_s 1..4) and the recurrence's per-step input is
 * softplus(ws x + bs) (ws [in_channels,cin_s], bs [in_channels]), computed
 * exactly as pt_lstm_stem_forward does but written straight into the
 * recurrence's own buffer: the f32 [B,in_channels,T,H,W] stem output and its
 * layout conversion never exist.  The backward does pt_lstm_backward's work
 * and then the stem's dW (dws [in_channels,cin_s]) and db (dbs) straight from
 * the recurrence's d x_t (either may be NULL); g->d_x may be NULL.
 * Replaces pt_lstm_stem_forward + pt_lstm_forward (and the backward pair) for
 * models/convlstm.py's ConvLSTMVideo. */
int pt_lstm_forward_stem(const pt_lstm_desc* d, const void* x, int x_u8, int cin_s, const float* ws,
                         const float* bs, const pt_lstm_params* p, void* saved, float* h_out,
                         float* c_out, pt_lstm_stream_t stream);
int pt_lstm_backward_stem(const pt_lstm_desc* d, const void* x, int x_u8, int cin_s, const float* ws,
                          const float* bs, const void* saved, void* workspace, const float* d_h,
                          const float* d_c, const pt_lstm_grads* g, float* dws, float* dbs,
                          pt_lstm_stream_t stream);

const char* pt_lstm_last_error(void);
const char* pt_lstm_version(void);

#ifdef __cplusplus
}
#endif
#endif /* PT_LSTM_H */
