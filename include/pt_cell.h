/*
 * pt_cell.h — C ABI of the MI355X (gfx950) recurrent-cell library.
 *
 * This is the drop-in boundary beneath the reference's model API: the
 * reference runs InT / hGRU forward as a Python loop of torch ops
 * (models/InT.py:210-245, cell models/InT.py:145-179;
 *  models/ffhgru_hierarchy.py:211-276, cell :135-173) and its BPTT backward
 * through stock autograd (mainclean.py:204).  The Python module
 * `models/InT.py` of this repo keeps the reference's class / constructor /
 * forward / state_dict surface and reaches the GPU only through the entry
 * points below (loaded with ctypes).
 *
 * Conventions
 *  - Plain C types only: device pointers, sizes, an opaque hipStream_t.
 *  - All tensors are allocated by the caller (PyTorch).  The library keeps no
 *    allocation and no mutable global state across calls; every call names
 *    its stream explicitly, so concurrent calls from several host threads
 *    (the reference's DataParallel replicas) are safe.
 *  - Return value: 0 on success, non-zero PT_ERR_* on failure; the message is
 *    available from pt_last_error() (thread-local).
 *  - Parameters are fp32 device buffers in their PyTorch (state_dict) layout.
 */
#ifndef PT_CELL_H
#define PT_CELL_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* pt_stream_t;   /* == hipStream_t */

enum { PT_OK = 0, PT_ERR_ARG = 1, PT_ERR_UNSUPPORTED = 2, PT_ERR_HIP = 3 };
enum { PT_ACT_SOFTPLUS = 0, PT_ACT_TANH = 1 };      /* the model's `nl` (models/InT.py:184) */
enum { PT_CELL_INT = 0, PT_CELL_HGRU = 1 };         /* rCell / hConvGRUCell */
enum { PT_DTYPE_F32 = 0, PT_DTYPE_BF16 = 1 };       /* storage + MFMA operand type */

/* Input layouts (pt_cell_desc.x_format):
 *  PT_X_F32_NCTHW  x = f32 [B][3][T][H][W], the model input as
 *                  engine.prepare_data produces it (utils/engine.py:220-255);
 *  PT_X_U8_NTHWC   x = u8 [B][T][H][W][3], the raw clip bytes as the TFRecords
 *                  hold them (utils/TFRDataset.py:6-28); the kernels convert
 *                  each byte u to (float)(u / 255.0 in double), bit-identical to
 *                  prepare_data's plain branch, so the f32 tensor is never built. */
enum { PT_X_F32_NCTHW = 0, PT_X_U8_NTHWC = 1 };

/* Problem description. */
typedef struct pt_cell_desc {
    int32_t batch;      /* B  clips on this device                              */
    int32_t channels;   /* C  = `dimensions` (utils/engine.py:75); 1..32: C < 32
                           runs zero-padded to the 32-wide MFMA tile          */
    int32_t frames;     /* T  = x.shape[2]                                      */
    int32_t height;     /* H  multiple of 32 (32; 64 for hGRU cfg4)             */
    int32_t width;      /* W  multiple of 32; frames > 32x32 run as 32x32 tiles */
    int32_t ksize;      /* horizontal kernel size, odd, <= 15 (engine passes 7;
                           the constructors' default is 15)                  */
    int32_t act;        /* PT_ACT_*                                             */
    int32_t no_inh;     /* InT_no_inh (models/InT.py:168)                       */
    int32_t cell;       /* PT_CELL_*                                            */
    int32_t dtype;      /* PT_DTYPE_*                                           */
    float   eps;        /* BatchNorm eps (1e-3, models/InT.py:102)              */
    int32_t x_format;   /* PT_X_*                                               */
} pt_cell_desc;

/* Recurrent-cell parameters, fp32, PyTorch layouts.  Gate order everywhere:
 * 0 a_w, 1 a_u, 2 i_w, 3 i_u, 4 e_w, 5 e_u (models/InT.py:73-84). */
typedef struct pt_cell_params {
    const float* preproc_w;   /* [C,3,1,1,1] */
    const float* preproc_b;   /* [C]         */
    const float* w_exc;       /* [C,C,k,k]   */
    const float* w_inh;       /* [C,C,k,k]   (ignored when no_inh)              */
    const float* alpha;       /* [C,1,1]     */
    const float* mu;
    const float* gamma;
    const float* kappa;
    const float* gate_w[6];   /* [C,C,1,1]   */
    const float* gate_b[6];   /* [C]         */
    const float* bn_w[2];     /* [C]  bn.0 / bn.1 */
    const float* bn_b[2];
} pt_cell_params;

/* Gradient outputs (same shapes as pt_cell_params; fp32, overwritten).  Any
 * pointer may be NULL when the caller does not want that gradient. */
typedef struct pt_cell_grads {
    float* preproc_w; float* preproc_b;
    float* w_exc; float* w_inh;
    float* alpha; float* mu; float* gamma; float* kappa;
    float* gate_w[6]; float* gate_b[6];
    float* bn_w[2]; float* bn_b[2];
} pt_cell_grads;

/* Bytes the caller must keep alive from pt_cell_forward to pt_cell_backward
 * (per-frame states and conv pre-activations, BN statistics, prepared weight
 * fragments), and bytes of transient workspace (reusable between calls). */
size_t pt_cell_saved_bytes(const pt_cell_desc* d);
size_t pt_cell_workspace_bytes(const pt_cell_desc* d);

/* Forward over all T frames (replaces the frame loop models/InT.py:223-235).
 *   x       [B,3,T,H,W] fp32
 *   e_last  [B,C,H,W] fp32 out: the excitation after the last frame (input of
 *           the readout, models/InT.py:236)
 *   gates   [B,T,C,H,W] fp32 out or NULL: attention maps (testmode, :230-233)
 */
int pt_cell_forward(const pt_cell_desc* d, const void* x, const pt_cell_params* p,
                    void* saved, void* workspace, float* e_last, float* gates,
                    pt_stream_t stream);

/* Per-frame excitations E_t, t = 0..T-1, as [B,T,C,H,W] fp32 (testmode
 * `states` are readout_conv of these, models/InT.py:233). */
int pt_cell_export_exc(const pt_cell_desc* d, const void* saved, float* e_seq,
                       pt_stream_t stream);

/* BPTT backward (replaces autograd through the frame loop).
 *   d_e_last  [B,C,H,W] fp32: dLoss/d e_last from the readout.
 * Writes every parameter gradient (overwrite, not accumulate). */
int pt_cell_backward(const pt_cell_desc* d, const void* x, const pt_cell_params* p,
                     const void* saved, void* workspace, const float* d_e_last,
                     const pt_cell_grads* g, pt_stream_t stream);

/* Cross-replica hooks (one process per GPU).  Pass NULL for
 * the reference's DataParallel semantics (per-replica BatchNorm statistics,
 * mainclean.py:132-134) and a single-stream backward.
 *
 *  bn_world > 1: SyncBN.  After each BatchNorm reduction (2 per frame forward,
 *    2 per frame backward) the library writes the replica's batch totals to
 *    bn_buf[offset, offset + count) (device, caller-owned, at least
 *    pt_cell_bn_sync_doubles() doubles) and calls allreduce(user, offset,
 *    count), which must enqueue, on the call's stream, a SUM of those doubles
 *    over the bn_world replicas and return 0; the statistics then cover all
 *    replicas' clips (count B * bn_world), so the replicas together compute
 *    exactly the single-process batch's forward and gradients (each on its
 *    own clips).  The call is made from the thread that called the entry
 *    point, between kernel launches; hipGraph replay is off in this mode.
 *  grads_early_event (hipEvent_t or NULL): recorded on the stream by the
 *    backward once every gradient except w_exc / w_inh is written, before the
 *    k x k weight-gradient kernel: the caller can all-reduce those gradients
 *    on another stream while that kernel runs (pt_cell_backward_dist).
 *  grads_mid_event (hipEvent_t or NULL; r06): when set (and the inhibition
 *    branch is on), the k x k weight gradients run as two launches, w_inh's
 *    first; the event is recorded once w_inh's gradient is written, so its
 *    all-reduce overlaps w_exc's weight-gradient kernel.  The values are the
 *    same as with one launch (the same per-tile sums in the same order). */
typedef int (*pt_bn_allreduce_fn)(void* user, int64_t offset, int64_t count);
typedef struct pt_cell_dist {
    int32_t bn_world;
    double* bn_buf;
    pt_bn_allreduce_fn allreduce;
    void* user;
    void* grads_early_event;
    void* grads_mid_event;
} pt_cell_dist;

size_t pt_cell_bn_sync_doubles(const pt_cell_desc* d);
int pt_cell_forward_dist(const pt_cell_desc* d, const void* x, const pt_cell_params* p,
                         void* saved, void* workspace, float* e_last, float* gates,
                         const pt_cell_dist* dist, pt_stream_t stream);
int pt_cell_backward_dist(const pt_cell_desc* d, const void* x, const pt_cell_params* p,
                          const void* saved, void* workspace, const float* d_e_last,
                          const pt_cell_grads* g, const pt_cell_dist* dist, pt_stream_t stream);

/* Optional kernel timing for benchmarks (process-wide, off by default; the
 * only mutable library state, guarded by a mutex).  When enabled for a kernel
 * kind, every launch of that kind is bracketed by two hipEvents on its launch
 * stream.  Reading
 * synchronises on the recorded events and returns the summed device time and
 * the launch count since the last reset.  Kinds: */
enum { PT_K_PW_FA = 0, PT_K_CONV_FA = 1, PT_K_PW_FB = 2, PT_K_CONV_FB = 3,
       PT_K_PW_BA = 4, PT_K_CONV_BA = 5, PT_K_PW_BB = 6, PT_K_CONV_BB = 7,
       PT_K_WGRAD = 8, PT_K_PREP = 9, PT_K_REDUCE = 10,
       PT_K_FUSED_FA = 11, PT_K_FUSED_FB = 12,     /* bf16 32x32: point-wise + conv per launch */
       PT_K_PERSIST = 13,                          /* opt-in persistent forward, all frames */
       PT_K_CONV_PW_BA = 14,                       /* bf16 32x32: k_conv_ba(t) + k_pw_ba(t-1) per launch */
       PT_K_NKINDS = 15 };
int pt_cell_timing_enable(uint32_t kind_mask);      /* bit k enables kind k; 0 disables */
int pt_cell_timing_read(int kind, double* total_ms, int64_t* launches);
int pt_cell_timing_reset(void);

/* Diagnostics: per-workgroup phase stamps (100 MHz real-time counter) of the
 * launches of frame `frame`, written to buf as u64 [PT_K_NKINDS][2048][32]
 * (every (grid / 2048)-th workgroup; slot meanings in csrc/pt_cell.hip, PT_TR).  buf = NULL
 * turns it off.  hipGraph replay is off while a buffer is set. */
int pt_cell_trace(void* buf, int frame);

/* Test hook (host only, no device work): the bf16 cell's split of f32 state
 * values into a hi plane (the bf16 operand, rounded half up in magnitude) and
 * a lo plane (hi << 16 plus sign-extended lo == the f32 bits; a NaN keeps a
 * quiet-NaN hi and lo = 0), exactly as the kernels store E and I (DESIGN.md
 * §4).  No reference counterpart: the reference keeps E and I in f32. */
int pt_cell_split_bits(const uint32_t* bits, uint16_t* hi, uint16_t* lo, int64_t n);

const char* pt_last_error(void);
const char* pt_version(void);

#ifdef __cplusplus
}
#endif
#endif /* PT_CELL_H */
