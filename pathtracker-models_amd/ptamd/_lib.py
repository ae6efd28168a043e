"""ctypes binding of the C-ABI library ``libptcell.so`` (include/pt_cell.h).

The shared library is built in-tree (``__graft_entry__.build()`` or
``python -m ptamd.build``) next to this file.  There is no fallback: if the
library or a ROCm device is missing, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libptcell.so")
# The diagnostic build (-DPT_DIAG=1: PT_CELL_ABLATE, PT_CELL_DEBUG_STOP,
# pt_cell_trace), for tools/ only; selected by use_diag() before the first
# load, or PT_CELL_DIAG=1 in the environment of a tool's process.
DIAG_PATH = os.path.join(HERE, "libptcell_diag.so")
if os.environ.get("PT_CELL_DIAG") == "1":
    LIB_PATH = DIAG_PATH

PT_ACT_SOFTPLUS, PT_ACT_TANH = 0, 1
PT_CELL_INT, PT_CELL_HGRU = 0, 1
PT_DTYPE_F32, PT_DTYPE_BF16 = 0, 1
PT_X_F32_NCTHW, PT_X_U8_NTHWC = 0, 1

# Exported symbols declared in include/pt_cell.h (tests check all are present).
EXPORTS = ("pt_cell_saved_bytes", "pt_cell_workspace_bytes", "pt_cell_forward",
           "pt_cell_export_exc", "pt_cell_backward", "pt_cell_bn_sync_doubles",
           "pt_cell_forward_dist", "pt_cell_backward_dist", "pt_cell_timing_enable",
           "pt_cell_timing_read", "pt_cell_timing_reset", "pt_cell_trace", "pt_cell_split_bits",
           "pt_last_error", "pt_version")

# kernel kinds for pt_cell_timing_* (include/pt_cell.h)
KIND_NAMES = ("k_pw_fa", "k_conv_fa", "k_pw_fb", "k_conv_fb", "k_pw_ba", "k_conv_ba",
              "k_pw_bb", "k_conv_bb", "k_wgrad", "k_prep", "k_reduce", "k_fused_fa",
              "k_fused_fb", "k_persist_fwd", "k_conv_pw_ba")
NKINDS = len(KIND_NAMES)
TRACE_WG, TRACE_SLOTS = 2048, 32      # pt_cell_trace record layout (csrc/pt_cell.hip PT_TR)

_P = ctypes.c_void_p


class Desc(ctypes.Structure):
    _fields_ = [("batch", ctypes.c_int32), ("channels", ctypes.c_int32),
                ("frames", ctypes.c_int32), ("height", ctypes.c_int32),
                ("width", ctypes.c_int32), ("ksize", ctypes.c_int32),
                ("act", ctypes.c_int32), ("no_inh", ctypes.c_int32),
                ("cell", ctypes.c_int32), ("dtype", ctypes.c_int32),
                ("eps", ctypes.c_float), ("x_format", ctypes.c_int32)]


class Params(ctypes.Structure):
    _fields_ = [("preproc_w", _P), ("preproc_b", _P), ("w_exc", _P), ("w_inh", _P),
                ("alpha", _P), ("mu", _P), ("gamma", _P), ("kappa", _P),
                ("gate_w", _P * 6), ("gate_b", _P * 6), ("bn_w", _P * 2), ("bn_b", _P * 2)]


class Grads(ctypes.Structure):
    _fields_ = Params._fields_


# int (*)(void* user, int64_t offset, int64_t count): SyncBN all-reduce hook
ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64)


class Dist(ctypes.Structure):
    """pt_cell_dist (include/pt_cell.h): SyncBN hook and the early-gradient event."""
    _fields_ = [("bn_world", ctypes.c_int32), ("bn_buf", _P), ("allreduce", ALLREDUCE_FN),
                ("user", _P), ("grads_early_event", _P), ("grads_mid_event", _P)]


class PtCellError(RuntimeError):
    pass


_lock = threading.RLock()
_lib = None
_opened = {}          # path -> CDLL (the release and the diagnostic library may both be open)
_override = None      # path of the library diag_library() made current, process-wide


def use_diag():
    """Load the diagnostic library instead of the release one (tools only)."""
    global LIB_PATH
    with _lock:
        if _lib is not None and LIB_PATH != DIAG_PATH:
            raise PtCellError("the release library is already loaded in this process")
        LIB_PATH = DIAG_PATH


class diag_library:
    """Context manager: every call into the cell library inside the block goes
    to the diagnostic build (libptcell_diag.so), opened beside the release one.
    For the kernel-variant A/B tests, which set PT_CELL_FUSED, PT_PWB2, ... in
    the environment: only the diagnostic build reads them.  Process-wide (the
    autograd backward runs on another thread), not re-entrant across threads;
    the forward and backward of one step must both run inside the block."""

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
            raise PtCellError(
                f"{path} is missing: build the HIP extension first "
                "(python __graft_entry__.py build, or python -m ptamd.build)")
        lib = ctypes.CDLL(path)
        lib.pt_cell_saved_bytes.restype = ctypes.c_size_t
        lib.pt_cell_saved_bytes.argtypes = [ctypes.POINTER(Desc)]
        lib.pt_cell_workspace_bytes.restype = ctypes.c_size_t
        lib.pt_cell_workspace_bytes.argtypes = [ctypes.POINTER(Desc)]
        lib.pt_cell_forward.restype = ctypes.c_int
        lib.pt_cell_forward.argtypes = [ctypes.POINTER(Desc), _P, ctypes.POINTER(Params), _P, _P,
                                        _P, _P, _P]
        lib.pt_cell_export_exc.restype = ctypes.c_int
        lib.pt_cell_export_exc.argtypes = [ctypes.POINTER(Desc), _P, _P, _P]
        lib.pt_cell_backward.restype = ctypes.c_int
        lib.pt_cell_backward.argtypes = [ctypes.POINTER(Desc), _P, ctypes.POINTER(Params), _P, _P,
                                         _P, ctypes.POINTER(Grads), _P]
        lib.pt_cell_bn_sync_doubles.restype = ctypes.c_size_t
        lib.pt_cell_bn_sync_doubles.argtypes = [ctypes.POINTER(Desc)]
        lib.pt_cell_forward_dist.restype = ctypes.c_int
        lib.pt_cell_forward_dist.argtypes = [ctypes.POINTER(Desc), _P, ctypes.POINTER(Params), _P,
                                             _P, _P, _P, ctypes.POINTER(Dist), _P]
        lib.pt_cell_backward_dist.restype = ctypes.c_int
        lib.pt_cell_backward_dist.argtypes = [ctypes.POINTER(Desc), _P, ctypes.POINTER(Params), _P,
                                              _P, _P, ctypes.POINTER(Grads), ctypes.POINTER(Dist),
                                              _P]
        lib.pt_cell_timing_enable.restype = ctypes.c_int
        lib.pt_cell_timing_enable.argtypes = [ctypes.c_uint32]
        lib.pt_cell_timing_read.restype = ctypes.c_int
        lib.pt_cell_timing_read.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                            ctypes.POINTER(ctypes.c_int64)]
        lib.pt_cell_split_bits.restype = ctypes.c_int
        lib.pt_cell_split_bits.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
        lib.pt_cell_trace.restype = ctypes.c_int
        lib.pt_cell_trace.argtypes = [ctypes.c_void_p, ctypes.c_int]
        lib.pt_cell_timing_reset.restype = ctypes.c_int
        lib.pt_last_error.restype = ctypes.c_char_p
        lib.pt_version.restype = ctypes.c_char_p
        _opened[path] = lib
        return lib


def check(rc: int, lib=None):
    """Raise on a non-zero status with the error string of ``lib``, the library
    that returned it (release and diagnostic builds can both be open)."""
    if rc != 0:
        msg = (lib or load()).pt_last_error().decode(errors="replace")
        raise PtCellError(f"pt_cell error {rc}: {msg}")


def check_lib(lib, rc: int):
    check(rc, lib)


def timing_read(kind: int):
    """(total_ms, launches) of kernel kind since the last reset (synchronises)."""
    lib = load()
    ms = ctypes.c_double()
    n = ctypes.c_int64()
    check_lib(lib, lib.pt_cell_timing_read(kind, ctypes.byref(ms), ctypes.byref(n)))
    return ms.value, n.value
