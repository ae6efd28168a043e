"""The readout head as one HIP forward / backward (include/pt_readout.h, in
``libptcell.so``), behind the reference's module parameters.

Reference (models/InT.py:236-241, ffhgru_hierarchy.py:258-272, the
ConvLSTMVideo readout):
``readout_dense(avg_pool2d(target_conv(cat([readout_conv(E_T), x[:, 2, 0]]))))``.
On ROCm tensors ``readout()`` runs the fused kernels (parameter gradients
reduced in clip order); on CPU tensors -- the reference's per-step API that
``rCell.forward`` / ``hConvGRUCell.forward`` keep for callers stepping the cell
themselves -- it is the reference's op chain.
"""
from __future__ import annotations

import ctypes

import torch
import torch.nn.functional as F

from . import _lib

EXPORTS = ("pt_readout_backward", "pt_readout_forward", "pt_readout_workspace_bytes")

_P = ctypes.c_void_p


class RoDesc(ctypes.Structure):
    _fields_ = [("batch", ctypes.c_int32), ("channels", ctypes.c_int32),
                ("height", ctypes.c_int32), ("width", ctypes.c_int32)]


class RoParams(ctypes.Structure):
    _fields_ = [("conv_w", _P), ("conv_b", _P), ("target_w", _P), ("target_b", _P),
                ("dense_w", _P), ("dense_b", _P)]


class RoGrads(ctypes.Structure):
    _fields_ = RoParams._fields_


_bound = None


def load():
    """The cell library with the readout entry points typed."""
    global _bound
    lib = _lib.load()
    if _bound is not lib:
        lib.pt_readout_workspace_bytes.restype = ctypes.c_int64
        lib.pt_readout_workspace_bytes.argtypes = [ctypes.POINTER(RoDesc)]
        lib.pt_readout_forward.restype = ctypes.c_int
        lib.pt_readout_forward.argtypes = [ctypes.POINTER(RoDesc), _P, _P, ctypes.POINTER(RoParams),
                                           _P, _P, _P]
        lib.pt_readout_backward.restype = ctypes.c_int
        lib.pt_readout_backward.argtypes = [ctypes.POINTER(RoDesc), _P, _P, ctypes.POINTER(RoParams),
                                            _P, _P, _P, ctypes.POINTER(RoGrads), _P, _P]
        _bound = lib
    return lib


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr())


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _params(ws):
    return RoParams(*[_ptr(w) for w in ws])


class ReadoutFn(torch.autograd.Function):
    """logits [B, 1] = readout(e [B, C, H, W] f32, tgt [B, H, W] f32; 6 parameters)."""

    @staticmethod
    def forward(ctx, e, tgt, *ws):
        lib = load()
        b, c, h, w = e.shape
        d = RoDesc(b, c, h, w)
        ws = [p.detach().contiguous().float() for p in ws]
        logits = torch.empty(b, device=e.device, dtype=torch.float32)
        pooled = torch.empty(b, device=e.device, dtype=torch.float32)
        pp = _params(ws)
        _lib.check_lib(lib, lib.pt_readout_forward(ctypes.byref(d), _ptr(e), _ptr(tgt), ctypes.byref(pp),
                                          _ptr(logits), _ptr(pooled), _stream(e.device)))
        ctx.save_for_backward(e, tgt, pooled, *ws)
        ctx.lib = lib                       # the backward runs in the same library
        return logits.reshape(b, 1)

    @staticmethod
    def backward(ctx, d_logits):
        lib = ctx.lib
        e, tgt, pooled, *ws = ctx.saved_tensors
        b, c, h, w = e.shape
        d = RoDesc(b, c, h, w)
        dl = d_logits.reshape(b).contiguous().float()
        d_e = torch.empty_like(e)
        grads = [torch.empty_like(p) for p in ws]
        scratch = torch.empty(int(lib.pt_readout_workspace_bytes(ctypes.byref(d))),
                              dtype=torch.uint8, device=e.device)
        pp = _params(ws)
        gg = RoGrads(*[_ptr(g) for g in grads])
        _lib.check_lib(lib, lib.pt_readout_backward(ctypes.byref(d), _ptr(e), _ptr(tgt), ctypes.byref(pp),
                                           _ptr(pooled), _ptr(dl), _ptr(d_e), ctypes.byref(gg),
                                           _ptr(scratch), _stream(e.device)))
        need = ctx.needs_input_grad
        return (d_e if need[0] else None, None,
                *[g if n else None for g, n in zip(grads, need[2:])])


def readout(e, tgt, readout_conv, target_conv, readout_dense):
    """The reference's readout chain; the fused HIP kernels on ROCm tensors."""
    if e.is_cuda:
        return ReadoutFn.apply(e.contiguous().float(), tgt.contiguous().float(),
                               readout_conv.weight, readout_conv.bias, target_conv.weight,
                               target_conv.bias, readout_dense.weight, readout_dense.bias)
    out = torch.cat([readout_conv(e), tgt[:, None]], 1)
    out = target_conv(out)
    out = F.avg_pool2d(out, kernel_size=out.size()[2:])
    return readout_dense(out.reshape(e.shape[0], -1))
