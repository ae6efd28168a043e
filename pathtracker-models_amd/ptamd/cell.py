"""Autograd bridge: the whole-clip recurrent cell as one ``torch.autograd.Function``.

Forward and backward are single calls into the C-ABI HIP library
(``include/pt_cell.h``): torch owns every buffer (inputs, outputs, the saved
state blob, the workspace) and the library sees raw device pointers and the
current HIP stream.  This replaces, for the reference's InT
(models/InT.py:210-245), the Python frame loop (:223-235) and the autograd
BPTT through it (mainclean.py:204).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import torch
from torch.utils.weak import WeakTensorKeyDictionary

from . import _lib

# Parameter order handed to the Function (names are the reference state_dict keys).
GATES = ("a_w", "a_u", "i_w", "i_u", "e_w", "e_u")
PARAM_KEYS = (["preproc.weight", "preproc.bias", "unit1.w_exc", "unit1.w_inh",
               "unit1.alpha", "unit1.mu", "unit1.gamma", "unit1.kappa"]
              + [f"unit1.{g}_gate.weight" for g in GATES]
              + [f"unit1.{g}_gate.bias" for g in GATES]
              + ["unit1.bn.0.weight", "unit1.bn.1.weight", "unit1.bn.0.bias", "unit1.bn.1.bias"])

DTYPES = {"f32": _lib.PT_DTYPE_F32, "fp32": _lib.PT_DTYPE_F32, "float32": _lib.PT_DTYPE_F32,
          "bf16": _lib.PT_DTYPE_BF16, "bfloat16": _lib.PT_DTYPE_BF16}


@dataclass(frozen=True)
class CellConfig:
    ksize: int = 7
    act: str = "softplus"        # 'softplus' | 'tanh'
    no_inh: bool = False
    cell: str = "int"            # 'int' (rCell) | 'hgru' (hConvGRUCell)
    dtype: str = "f32"           # 'f32' (parity) | 'bf16' (throughput)
    eps: float = 1e-3


# Parameters the no_inh branch never reads (models/InT.py:168): the reference
# leaves their .grad None, so must we.
_UNUSED_NO_INH = {"unit1.w_inh", "unit1.alpha", "unit1.mu", "unit1.i_w_gate.weight",
                  "unit1.i_u_gate.weight", "unit1.i_w_gate.bias", "unit1.i_u_gate.bias",
                  "unit1.bn.0.weight", "unit1.bn.0.bias"}


def clip_dims(x: torch.Tensor):
    """(B, T, H, W) of a model input: f32 [B,3,T,H,W] or raw u8 clips [B,T,H,W,3]."""
    if x.dtype == torch.uint8:
        b, t, h, w, ch = x.shape
    else:
        b, ch, t, h, w = x.shape
    if ch != 3:
        raise ValueError(f"expected 3 input channels, got shape {tuple(x.shape)}")
    return b, t, h, w


def unit_values(x_u8: torch.Tensor) -> torch.Tensor:
    """u8 -> f32 exactly as engine.prepare_data (float64 u / 255 rounded to f32)."""
    return (x_u8.to(torch.float64) / 255.).to(torch.float32)


def target_channel(x: torch.Tensor) -> torch.Tensor:
    """x[:, 2, 0] of the f32 model input (the readout's target marker,
    models/InT.py:236) from either input layout."""
    if x.dtype == torch.uint8:
        return unit_values(x[:, 0, :, :, 2])
    return x[:, 2, 0]


def _desc(cfg: CellConfig, x: torch.Tensor, channels: int) -> _lib.Desc:
    b, t, h, w = clip_dims(x)
    return _lib.Desc(batch=b, channels=channels, frames=t, height=h, width=w, ksize=cfg.ksize,
                     act=_lib.PT_ACT_TANH if cfg.act == "tanh" else _lib.PT_ACT_SOFTPLUS,
                     no_inh=int(cfg.no_inh),
                     cell=_lib.PT_CELL_HGRU if cfg.cell == "hgru" else _lib.PT_CELL_INT,
                     dtype=DTYPES[cfg.dtype], eps=cfg.eps,
                     x_format=_lib.PT_X_U8_NTHWC if x.dtype == torch.uint8 else _lib.PT_X_F32_NCTHW)


# f32 contiguous staging copies of parameters that are not (e.g. a model moved
# to another dtype): one persistent buffer per parameter, refreshed in place
# each call, so the device pointers -- and with them the library's cached
# hipGraph (pt_graph.h, keyed by every pointer) -- stay the same from step to
# step instead of a fresh temporary forcing a re-capture per call.  Keys
# compare by identity (a plain WeakKeyDictionary would compare tensors
# element-wise on a hash collision and raise).
_STAGED = WeakTensorKeyDictionary()


def _as_f32(p):
    if p is None or (p.dtype == torch.float32 and p.is_contiguous()):
        return p
    buf = _STAGED.get(p)
    if buf is None or buf.shape != p.shape or buf.device != p.device:
        buf = torch.empty(p.shape, dtype=torch.float32, device=p.device)
        _STAGED[p] = buf
    with torch.no_grad():
        buf.copy_(p)
    return buf


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _pack(struct_cls, tensors):
    """Fill a Params/Grads struct from tensors in PARAM_KEYS order (None -> NULL)."""
    s = struct_cls()
    vals = [t.data_ptr() if t is not None else 0 for t in tensors]
    (s.preproc_w, s.preproc_b, s.w_exc, s.w_inh, s.alpha, s.mu, s.gamma, s.kappa) = vals[:8]
    for i in range(6):
        s.gate_w[i] = vals[8 + i]
        s.gate_b[i] = vals[14 + i]
    s.bn_w[0], s.bn_w[1], s.bn_b[0], s.bn_b[1] = vals[20:24]
    return s


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _require_device(x):
    if x.device.type != "cuda":
        raise RuntimeError("the InT HIP cell runs on a ROCm device only (got a "
                           f"{x.device.type} tensor); there is no CPU fallback")


class RecurrentCellFn(torch.autograd.Function):
    """(x, params...) -> (E_T [B,C,H,W], E_seq [B,T,C,H,W], att [B,T,C,H,W]).

    x is the f32 model input [B,3,T,H,W] or the raw u8 clips [B,T,H,W,3]
    (converted inside the kernels, bit-identical to engine.prepare_data).

    E_seq / att are only filled when ``want_seq`` (testmode); otherwise they
    are empty tensors.  Only E_T is differentiable.  ``cdist`` (a
    ptamd.dist.CellDist or None) selects SyncBN and the early-gradient
    all-reduce (pt_cell_dist).
    """

    @staticmethod
    def forward(ctx, x, cfg: CellConfig, want_seq: bool, cdist, *params):
        _require_device(x)
        lib = _lib.load()
        x = x.contiguous() if x.dtype == torch.uint8 else x.contiguous().float()
        ctx.param_ids = [id(p) if p is not None else None for p in params]
        params = [_as_f32(p) for p in params]
        c = params[0].shape[0]
        d = _desc(cfg, x, c)
        saved = torch.empty(lib.pt_cell_saved_bytes(ctypes.byref(d)), dtype=torch.uint8,
                            device=x.device)
        if saved.numel() == 0:
            _lib.check(1, lib)
        ws = torch.empty(lib.pt_cell_workspace_bytes(ctypes.byref(d)), dtype=torch.uint8,
                         device=x.device)
        b, t, h, w = clip_dims(x)
        e_last = torch.empty((b, c, h, w), dtype=torch.float32, device=x.device)
        gates = torch.empty((b, t, c, h, w) if want_seq else (0,), dtype=torch.float32,
                            device=x.device)
        pp = _pack(_lib.Params, params)
        st = _stream(x.device)
        dd = (cdist.struct(lib.pt_cell_bn_sync_doubles(ctypes.byref(d)), x.device)
              if cdist is not None else None)
        _lib.check_lib(lib, lib.pt_cell_forward_dist(ctypes.byref(d), _ptr(x), ctypes.byref(pp),
                                            _ptr(saved), _ptr(ws), _ptr(e_last),
                                            _ptr(gates) if want_seq else None,
                                            ctypes.byref(dd) if dd is not None else None, st))
        e_seq = torch.empty((b, t, c, h, w) if want_seq else (0,), dtype=torch.float32,
                            device=x.device)
        if want_seq:
            _lib.check_lib(lib, lib.pt_cell_export_exc(ctypes.byref(d), _ptr(saved), _ptr(e_seq), st))
        ctx.cfg = cfg
        ctx.cdist = cdist
        ctx.lib = lib                      # the backward runs on the library that wrote `saved`
        ctx.saved_blob = saved
        ctx.save_for_backward(x, *[p if p is not None else torch.empty(0) for p in params])
        ctx.has = [p is not None for p in params]
        ctx.mark_non_differentiable(e_seq, gates)
        return e_last, e_seq, gates

    @staticmethod
    def backward(ctx, d_e_last, _d_seq, _d_gates):
        lib = ctx.lib
        x, *params = ctx.saved_tensors
        params = [p if has else None for p, has in zip(params, ctx.has)]
        c = params[0].shape[0]
        d = _desc(ctx.cfg, x, c)
        if d_e_last is None:
            b, _, h, w = clip_dims(x)
            d_e_last = torch.zeros((b, c, h, w), device=x.device)
        d_e_last = d_e_last.contiguous().float()
        ws = torch.empty(lib.pt_cell_workspace_bytes(ctypes.byref(d)), dtype=torch.uint8,
                         device=x.device)
        need = list(ctx.needs_input_grad[4:])      # after x, cfg, want_seq, cdist
        if ctx.cfg.no_inh:
            need = [n and PARAM_KEYS[i] not in _UNUSED_NO_INH for i, n in enumerate(need)]
        grads = [torch.empty_like(p) if (p is not None and need[i]) else None
                 for i, p in enumerate(params)]
        pp = _pack(_lib.Params, params)
        gg = _pack(_lib.Grads, grads)
        cdist = ctx.cdist
        early = mid = None
        bucket = cdist.bucket if cdist is not None else None
        if bucket is not None and cdist.world() > 1:
            early = torch.cuda.Event()
            early.record()                  # creates the event; the library re-records it
            if not ctx.cfg.no_inh and bucket.three_part:
                mid = torch.cuda.Event()
                mid.record()
        dd = (cdist.struct(lib.pt_cell_bn_sync_doubles(ctypes.byref(d)), x.device,
                           early.cuda_event if early is not None else None,
                           mid.cuda_event if mid is not None else None)
              if cdist is not None else None)
        _lib.check_lib(lib, lib.pt_cell_backward_dist(ctypes.byref(d), _ptr(x), ctypes.byref(pp),
                                             _ptr(ctx.saved_blob), _ptr(ws), _ptr(d_e_last),
                                             ctypes.byref(gg),
                                             ctypes.byref(dd) if dd is not None else None,
                                             _stream(x.device)))
        if early is not None:
            # every gradient but the two k x k weights is final at `early`:
            # averaged on a side stream under the k x k weight-gradient kernel
            from .dist import LATE_KEYS, MID_KEYS
            bucket.reduce_early([(pid, g) for k, pid, g in zip(PARAM_KEYS, ctx.param_ids, grads)
                                 if g is not None and k not in LATE_KEYS], early)
            if mid is not None:
                # w_inh is final at `mid`: averaged under w_exc's weight-gradient launch
                bucket.reduce_early([(pid, g) for k, pid, g in zip(PARAM_KEYS, ctx.param_ids, grads)
                                     if g is not None and k in MID_KEYS], mid)
        ctx.saved_blob = None
        return (None, None, None, None, *grads)


def run_cell(x, params, cfg: CellConfig, want_seq: bool = False, cdist=None):
    """Apply the HIP recurrent cell.  ``params`` is a list in PARAM_KEYS order;
    ``cdist``: optional ptamd.dist.CellDist (SyncBN / early-gradient overlap)."""
    return RecurrentCellFn.apply(x, cfg, want_seq, cdist, *params)
