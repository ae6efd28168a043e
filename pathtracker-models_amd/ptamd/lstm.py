"""ctypes binding of ``libptlstm.so`` (include/pt_lstm.h) and its autograd bridge.

``LSTMStepsFn`` runs ``steps`` ConvLSTM steps on a static input (the
reference's form) or on one input image per step (``x`` [B,cin,T,H,W], the
video adaptation for PathTracker clips) through the HIP library — forward, BPTT backward and (for the model's training mode) the
Jacobian penalty — with every buffer owned by torch and the library seeing raw
device pointers plus the current HIP stream.  It replaces, for the reference's
``models/convlstm.py``, the per-step Python loop (:137-143, cell :84-90) and
autograd through it.  There is no CPU fallback: CPU tensors or a missing
library raise.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch
from torch.autograd.function import once_differentiable

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libptlstm.so")

PT_LSTM_F32, PT_LSTM_BF16 = 0, 1
PT_LSTM_H0, PT_LSTM_C0 = 1, 2
PT_LSTM_OK, PT_LSTM_ERR_ARG, PT_LSTM_ERR_UNSUPPORTED, PT_LSTM_ERR_HIP = 0, 1, 2, 3

# Exported symbols declared in include/pt_lstm.h (tests check all are present).
EXPORTS = ("pt_lstm_saved_bytes", "pt_lstm_workspace_bytes", "pt_lstm_forward",
           "pt_lstm_backward", "pt_lstm_jv_penalty", "pt_lstm_export_h",
           "pt_lstm_stem_workspace_bytes",
           "pt_lstm_stem_forward", "pt_lstm_stem_backward", "pt_lstm_forward_stem",
           "pt_lstm_backward_stem", "pt_lstm_last_error", "pt_lstm_version")

_P = ctypes.c_void_p


class Desc(ctypes.Structure):
    _fields_ = [("batch", ctypes.c_int32), ("in_channels", ctypes.c_int32),
                ("channels", ctypes.c_int32), ("height", ctypes.c_int32),
                ("width", ctypes.c_int32), ("ksize", ctypes.c_int32),
                ("steps", ctypes.c_int32), ("dtype", ctypes.c_int32),
                ("init_state", ctypes.c_int32), ("x_seq", ctypes.c_int32)]


class Params(ctypes.Structure):
    _fields_ = [("wx", _P * 4), ("bx", _P * 4), ("wh", _P * 4)]


class Grads(ctypes.Structure):
    _fields_ = [("wx", _P * 4), ("bx", _P * 4), ("wh", _P * 4), ("d_x", _P), ("d_h0", _P),
                ("d_c0", _P)]


class PtLstmError(RuntimeError):
    pass


# The diagnostic build (-DPT_DIAG=1): also honours the kernel-variant switches
# PT_LCONV_FAST / PT_LCONVT8 / PT_LWGRAD2, which libptlstm.so compiles to their
# defaults; tests A/B the variants through diag_library().
DIAG_PATH = os.path.join(HERE, "libptlstm_diag.so")

_lock = threading.RLock()
_lib = None
_opened = {}
_override = None


class diag_library:
    """Context manager: calls inside the block go to libptlstm_diag.so
    (process-wide; see ptamd._lib.diag_library)."""

    def __enter__(self):
        global _override
        lib = _open(DIAG_PATH)
        with _lock:           # not held across the block: autograd's backward thread loads too
            self._prev = _override
            _override = DIAG_PATH
        return lib

    def __exit__(self, *exc):
        global _override
        with _lock:
            _override = self._prev
        return False


def load():
    """Load (once) and return the library; raise if it is not built."""
    global _lib
    with _lock:
        if _override is not None:
            return _open(_override)
        if _lib is None:
            _lib = _open(LIB_PATH)
        return _lib


def _open(path):
    with _lock:
        if path in _opened:
            return _opened[path]
        if not os.path.exists(path):
            raise PtLstmError(
                f"{path} is missing: build the HIP extensions first "
                "(python __graft_entry__.py build, or python -m ptamd.build)")
        lib = ctypes.CDLL(path)
        D = ctypes.POINTER(Desc)
        lib.pt_lstm_saved_bytes.restype = ctypes.c_size_t
        lib.pt_lstm_saved_bytes.argtypes = [D]
        lib.pt_lstm_workspace_bytes.restype = ctypes.c_size_t
        lib.pt_lstm_workspace_bytes.argtypes = [D]
        lib.pt_lstm_forward.restype = ctypes.c_int
        lib.pt_lstm_forward.argtypes = [D, _P, ctypes.POINTER(Params), _P, _P, _P, _P, _P, _P]
        lib.pt_lstm_backward.restype = ctypes.c_int
        lib.pt_lstm_backward.argtypes = [D, _P, _P, _P, _P, ctypes.POINTER(Grads), _P]
        lib.pt_lstm_jv_penalty.restype = ctypes.c_int
        lib.pt_lstm_jv_penalty.argtypes = [D, _P, _P, ctypes.c_float, _P, _P]
        lib.pt_lstm_export_h.restype = ctypes.c_int
        lib.pt_lstm_export_h.argtypes = [D, _P, _P, _P]
        lib.pt_lstm_stem_workspace_bytes.restype = ctypes.c_size_t
        lib.pt_lstm_stem_workspace_bytes.argtypes = [ctypes.c_int]
        _i, _ll = ctypes.c_int, ctypes.c_longlong
        lib.pt_lstm_stem_forward.restype = ctypes.c_int
        lib.pt_lstm_stem_forward.argtypes = [_P, _i, _P, _P, _i, _i, _i, _ll, _P, _P]
        lib.pt_lstm_stem_backward.restype = ctypes.c_int
        lib.pt_lstm_stem_backward.argtypes = [_P, _i, _P, _P, _P, _i, _i, _i, _ll, _P, _P, _P, _P]
        lib.pt_lstm_forward_stem.restype = ctypes.c_int
        lib.pt_lstm_forward_stem.argtypes = [D, _P, _i, _i, _P, _P, ctypes.POINTER(Params), _P, _P, _P, _P]
        lib.pt_lstm_backward_stem.restype = ctypes.c_int
        lib.pt_lstm_backward_stem.argtypes = [D, _P, _i, _i, _P, _P, _P, _P, _P, _P,
                                              ctypes.POINTER(Grads), _P, _P, _P]
        lib.pt_lstm_last_error.restype = ctypes.c_char_p
        lib.pt_lstm_version.restype = ctypes.c_char_p
        _opened[path] = lib
        return lib


def check(rc: int, lib=None):
    """Raise on a non-zero status; the message comes from ``lib``, the library
    that returned it (its error string is per library: the release and the
    diagnostic builds can both be open, ptamd.lstm.diag_library)."""
    if rc != 0:
        msg = (lib or load()).pt_lstm_last_error().decode(errors="replace")
        raise PtLstmError(f"pt_lstm error {rc}: {msg}")


def _chk(lib, rc: int):
    check(rc, lib)


DTYPES = {"f32": PT_LSTM_F32, "fp32": PT_LSTM_F32, "float32": PT_LSTM_F32,
          "bf16": PT_LSTM_BF16, "bfloat16": PT_LSTM_BF16}


def make_desc(x, channels: int, ksize: int, steps: int, dtype: str, h0=None, c0=None) -> Desc:
    """x: static [B,cin,H,W] or per step [B,cin,T,H,W] (T == steps)."""
    if x.dim() == 5:
        b, cin, t, h, w = x.shape
        if t != steps:
            raise ValueError(f"per-step input has {t} frames but steps={steps}")
    else:
        b, cin, h, w = x.shape
    return Desc(batch=b, in_channels=cin, channels=channels, height=h, width=w, ksize=ksize,
                steps=steps, dtype=DTYPES[dtype],
                init_state=(PT_LSTM_H0 if h0 is not None else 0)
                | (PT_LSTM_C0 if c0 is not None else 0), x_seq=int(x.dim() == 5))


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _require_device(x):
    if x.device.type != "cuda":
        raise RuntimeError("the ConvLSTM HIP cell runs on a ROCm device only (got a "
                           f"{x.device.type} tensor); there is no CPU fallback")


# weight order handed to the Function: Wx{i,f,c,o}, bx{i,f,c,o}, Wh{i,f,c,o}
GATES = ("i", "f", "c", "o")


class LSTMStepsFn(torch.autograd.Function):
    """(x, h0|None, c0|None, 12 weights) -> (h_T, c_T, jv, h_seq).

    ``jv`` (the training-mode Jacobian penalty, models/convlstm.py:150-161) is
    only computed when ``want_jv``; it is returned detached (the reference
    builds a graph for it only with ``jacobian_penalty=True``, and never puts
    it in the loss it returns).  ``h_seq`` [B,ch,T,H,W] holds every step's
    hidden state when ``want_seq`` (testmode), detached; otherwise it is empty.
    """

    @staticmethod
    def forward(ctx, x, h0, c0, ksize: int, steps: int, dtype: str, want_jv: bool, mu: float,
                want_seq: bool, *weights):
        _require_device(x)
        lib = load()
        x = x.contiguous().float()
        h0 = h0.contiguous().float() if h0 is not None else None
        c0 = c0.contiguous().float() if c0 is not None else None
        weights = [w.contiguous().float() for w in weights]
        ch = weights[0].shape[0]
        d = make_desc(x, ch, ksize, steps, dtype, h0, c0)
        nsaved = lib.pt_lstm_saved_bytes(ctypes.byref(d))
        if nsaved == 0:
            check(1, lib)
        saved = torch.empty(nsaved, dtype=torch.uint8, device=x.device)
        b, hh, ww = x.shape[0], x.shape[-2], x.shape[-1]
        h_out = torch.empty((b, ch, hh, ww), dtype=torch.float32, device=x.device)
        c_out = torch.empty_like(h_out)
        pp = Params()
        for g in range(4):
            pp.wx[g] = weights[g].data_ptr()
            pp.bx[g] = weights[4 + g].data_ptr()
            pp.wh[g] = weights[8 + g].data_ptr()
        st = _stream(x.device)
        _chk(lib, lib.pt_lstm_forward(ctypes.byref(d), _ptr(x), ctypes.byref(pp), _ptr(h0), _ptr(c0),
                                  _ptr(saved), _ptr(h_out), _ptr(c_out), st))
        jv = torch.empty((0,), device=x.device)
        if want_jv:
            ws = torch.empty(lib.pt_lstm_workspace_bytes(ctypes.byref(d)), dtype=torch.uint8,
                             device=x.device)
            jv = torch.empty_like(h_out)
            _chk(lib, lib.pt_lstm_jv_penalty(ctypes.byref(d), _ptr(saved), _ptr(ws), float(mu),
                                         _ptr(jv), st))
        h_seq = torch.empty((b, ch, steps, hh, ww) if want_seq else (0,), device=x.device)
        if want_seq:
            _chk(lib, lib.pt_lstm_export_h(ctypes.byref(d), _ptr(saved), _ptr(h_seq), st))
        ctx.meta = (ksize, steps, dtype, h0 is not None, c0 is not None, tuple(x.shape), ch)
        ctx.lib = lib
        ctx.desc = d
        ctx.saved_blob = saved
        ctx.wshapes = [w.shape for w in weights]
        ctx.mark_non_differentiable(jv, h_seq)
        return h_out, c_out, jv, h_seq

    @staticmethod
    @once_differentiable
    def backward(ctx, d_h, d_c, _d_jv, _d_seq):
        # may run several times on one graph (retain_graph: the rbp Neumann
        # series and the Jacobian-penalty VJPs, models/convlstm.py:35,155-160),
        # so the saved blob stays with ctx until autograd frees the graph; the
        # library that wrote it runs the backward
        lib = ctx.lib
        ksize, steps, dtype, has_h0, has_c0, xshape, ch = ctx.meta
        b, hh, ww = xshape[0], xshape[-2], xshape[-1]
        dev = ctx.saved_blob.device
        d = ctx.desc
        if d_h is None:
            d_h = torch.zeros((b, ch, hh, ww), device=dev)
        d_h = d_h.contiguous().float()
        d_c = d_c.contiguous().float() if d_c is not None else None
        ws = torch.empty(lib.pt_lstm_workspace_bytes(ctypes.byref(d)), dtype=torch.uint8,
                         device=dev)
        need = ctx.needs_input_grad
        grads = [torch.empty(s, device=dev) if need[9 + i] else None      # weights follow 9 args
                 for i, s in enumerate(ctx.wshapes)]
        dx = torch.empty(xshape, device=dev) if need[0] else None
        dh0 = torch.empty((b, ch, hh, ww), device=dev) if (has_h0 and need[1]) else None
        dc0 = torch.empty((b, ch, hh, ww), device=dev) if (has_c0 and need[2]) else None
        gg = Grads()
        for g in range(4):
            gg.wx[g] = grads[g].data_ptr() if grads[g] is not None else 0
            gg.bx[g] = grads[4 + g].data_ptr() if grads[4 + g] is not None else 0
            gg.wh[g] = grads[8 + g].data_ptr() if grads[8 + g] is not None else 0
        gg.d_x = dx.data_ptr() if dx is not None else 0
        gg.d_h0 = dh0.data_ptr() if dh0 is not None else 0
        gg.d_c0 = dc0.data_ptr() if dc0 is not None else 0
        _chk(lib, lib.pt_lstm_backward(ctypes.byref(d), _ptr(ctx.saved_blob), _ptr(ws), _ptr(d_h),
                                   _ptr(d_c), ctypes.byref(gg), _stream(dev)))
        return (dx, dh0, dc0, None, None, None, None, None, None, *grads)


def run_steps(x, weights, *, ksize: int, steps: int, h0=None, c0=None, dtype: str = "f32",
              want_jv: bool = False, mu: float = 0.9, want_seq: bool = False):
    """Apply ``steps`` ConvLSTM steps.  ``weights``: [Wx_i..o, bx_i..o, Wh_i..o].
    Returns (h_T, c_T, jv, h_seq) when ``want_seq``, else (h_T, c_T, jv)."""
    h, c, jv, seq = LSTMStepsFn.apply(x, h0, c0, ksize, steps, dtype, want_jv, mu, want_seq,
                                      *weights)
    return (h, c, jv, seq) if want_seq else (h, c, jv)


class StemStepsFn(torch.autograd.Function):
    """(raw clips x, stem weight, stem bias, 12 cell weights) -> (h_T, c_T, jv,
    h_seq): ConvLSTMVideo's stem ``softplus(Conv3d 1x1x1)`` and its ``steps``
    ConvLSTM steps (one frame per step, h0 = c0 = 0) in one library call
    (pt_lstm_forward_stem): the stem writes the recurrence's per-step input
    directly, so neither its f32 [B,C,T,H,W] output nor the gradient of it
    is ever materialised.  Same values as ``stem`` followed by
    ``run_steps`` (the stem output is rounded to the cell's storage type
    either way); x is the f32 model input [B,cin,T,H,W] or the raw u8 clips
    [B,T,H,W,cin] and gets no gradient."""

    @staticmethod
    def forward(ctx, x, sw, sb, ksize: int, dtype: str, want_jv: bool, mu: float, want_seq: bool,
                *weights):
        _require_device(x)
        if x.requires_grad:
            raise NotImplementedError("the stem gives no gradient for its input")
        lib = load()
        u8 = x.dtype == torch.uint8
        if u8:
            b, cin_s, steps, hh, ww = x.shape[0], x.shape[-1], x.shape[1], x.shape[2], x.shape[3]
            x = x.contiguous()
        else:
            b, cin_s, steps, hh, ww = x.shape
            x = x.contiguous().float()
        cs = sw.shape[0]
        w = sw.detach().reshape(cs, cin_s).contiguous().float()
        bb = sb.detach().contiguous().float()
        weights = [wt.contiguous().float() for wt in weights]
        ch = weights[0].shape[0]
        d = Desc(batch=b, in_channels=cs, channels=ch, height=hh, width=ww, ksize=ksize, steps=steps,
                 dtype=DTYPES[dtype], init_state=0, x_seq=1)
        nsaved = lib.pt_lstm_saved_bytes(ctypes.byref(d))
        if nsaved == 0:
            check(1, lib)
        saved = torch.empty(nsaved, dtype=torch.uint8, device=x.device)
        h_out = torch.empty((b, ch, hh, ww), dtype=torch.float32, device=x.device)
        c_out = torch.empty_like(h_out)
        pp = Params()
        for g in range(4):
            pp.wx[g] = weights[g].data_ptr()
            pp.bx[g] = weights[4 + g].data_ptr()
            pp.wh[g] = weights[8 + g].data_ptr()
        st = _stream(x.device)
        _chk(lib, lib.pt_lstm_forward_stem(ctypes.byref(d), _ptr(x), int(u8), cin_s, _ptr(w), _ptr(bb),
                                       ctypes.byref(pp), _ptr(saved), _ptr(h_out), _ptr(c_out), st))
        jv = torch.empty((0,), device=x.device)
        if want_jv:
            ws = torch.empty(lib.pt_lstm_workspace_bytes(ctypes.byref(d)), dtype=torch.uint8,
                             device=x.device)
            jv = torch.empty_like(h_out)
            _chk(lib, lib.pt_lstm_jv_penalty(ctypes.byref(d), _ptr(saved), _ptr(ws), float(mu),
                                         _ptr(jv), st))
        h_seq = torch.empty((b, ch, steps, hh, ww) if want_seq else (0,), device=x.device)
        if want_seq:
            _chk(lib, lib.pt_lstm_export_h(ctypes.byref(d), _ptr(saved), _ptr(h_seq), st))
        ctx.lib = lib
        ctx.desc = d
        ctx.saved_blob = saved
        ctx.stem = (x, w, bb, int(u8), cin_s)
        ctx.sshape = (sw.shape, sb.shape)
        ctx.wshapes = [wt.shape for wt in weights]
        ctx.ch = ch
        ctx.mark_non_differentiable(jv, h_seq)
        return h_out, c_out, jv, h_seq

    @staticmethod
    @once_differentiable
    def backward(ctx, d_h, d_c, _d_jv, _d_seq):
        lib = ctx.lib
        d = ctx.desc
        x, w, bb, u8, cin_s = ctx.stem
        dev = ctx.saved_blob.device
        if d_h is None:
            d_h = torch.zeros((d.batch, ctx.ch, d.height, d.width), device=dev)
        d_h = d_h.contiguous().float()
        d_c = d_c.contiguous().float() if d_c is not None else None
        ws = torch.empty(lib.pt_lstm_workspace_bytes(ctypes.byref(d)), dtype=torch.uint8, device=dev)
        need = ctx.needs_input_grad
        grads = [torch.empty(s, device=dev) if need[8 + i] else None      # weights follow 8 args
                 for i, s in enumerate(ctx.wshapes)]
        dsw = torch.empty(ctx.sshape[0], device=dev) if need[1] else None
        dsb = torch.empty(ctx.sshape[1], device=dev) if need[2] else None
        gg = Grads()
        for g in range(4):
            gg.wx[g] = grads[g].data_ptr() if grads[g] is not None else 0
            gg.bx[g] = grads[4 + g].data_ptr() if grads[4 + g] is not None else 0
            gg.wh[g] = grads[8 + g].data_ptr() if grads[8 + g] is not None else 0
        gg.d_x = gg.d_h0 = gg.d_c0 = 0
        _chk(lib, lib.pt_lstm_backward_stem(ctypes.byref(d), _ptr(x), u8, cin_s, _ptr(w), _ptr(bb),
                                        _ptr(ctx.saved_blob), _ptr(ws), _ptr(d_h), _ptr(d_c),
                                        ctypes.byref(gg), _ptr(dsw), _ptr(dsb), _stream(dev)))
        return (None, dsw, dsb, None, None, None, None, None, *grads)


def stem_steps(x, stem_weight, stem_bias, weights, *, ksize: int, dtype: str = "f32",
               want_jv: bool = False, mu: float = 0.9, want_seq: bool = False):
    """The clip ConvLSTM's stem + its per-frame steps in one library call
    (StemStepsFn).  Returns (h_T, c_T, jv, h_seq) when ``want_seq``, else (h_T, c_T, jv)."""
    h, c, jv, seq = StemStepsFn.apply(x, stem_weight, stem_bias, ksize, dtype, want_jv, mu, want_seq,
                                      *weights)
    return (h, c, jv, seq) if want_seq else (h, c, jv)


class StemFn(torch.autograd.Function):
    """softplus(Conv3d 1x1x1) of a clip batch through pt_lstm_stem_* (HIP).

    x: the f32 model input [B,cin,T,H,W] or the raw u8 clips [B,T,H,W,cin]
    (converted in the kernel as engine.prepare_data would; no gradient: it is
    the clip), weight [cout,cin,1,1,1], bias [cout] -> [B,cout,T,H,W]; the
    backward returns weight / bias grads.
    """

    @staticmethod
    def forward(ctx, x, weight, bias):
        _require_device(x)
        if x.requires_grad:
            raise NotImplementedError("the stem gives no gradient for its input")
        lib = load()
        u8 = x.dtype == torch.uint8
        if u8:
            b, cin, dims = x.shape[0], x.shape[-1], tuple(x.shape[1:4])
            x = x.contiguous()
        else:
            b, cin, dims = x.shape[0], x.shape[1], tuple(x.shape[2:])
            x = x.contiguous().float()
        n = dims[0] * dims[1] * dims[2]
        cout = weight.shape[0]
        w = weight.detach().reshape(cout, cin).contiguous().float()
        bb = bias.detach().contiguous().float()
        y = torch.empty((b, cout) + dims, device=x.device)
        _chk(lib, lib.pt_lstm_stem_forward(_ptr(x), int(u8), _ptr(w), _ptr(bb), b, cin, cout, n,
                                       _ptr(y), _stream(x.device)))
        ctx.save_for_backward(x, w, bb)
        ctx.lib = lib
        ctx.meta = (int(u8), b, cin, n)
        ctx.wshape = weight.shape
        return y

    @staticmethod
    @once_differentiable
    def backward(ctx, dy):
        lib = ctx.lib
        x, w, bb = ctx.saved_tensors
        u8, b, cin, n = ctx.meta
        cout = w.shape[0]
        dy = dy.contiguous().float()
        ws = torch.empty(lib.pt_lstm_stem_workspace_bytes(cin), dtype=torch.uint8, device=x.device)
        dw = torch.empty((cout, cin), device=x.device)
        db = torch.empty((cout,), device=x.device)
        _chk(lib, lib.pt_lstm_stem_backward(_ptr(x), u8, _ptr(w), _ptr(bb), _ptr(dy), b, cin, cout,
                                        n, _ptr(ws), _ptr(dw), _ptr(db), _stream(x.device)))
        return None, dw.reshape(ctx.wshape), db


def stem(x, weight, bias):
    """softplus(conv3d(x, weight, bias)) for a 1x1x1 ``weight`` (ConvLSTMVideo's stem)."""
    return StemFn.apply(x, weight, bias)
