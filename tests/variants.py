"""Kernel-variant switches for the A/B tests (PT_CELL_FUSED, PT_PWB2, PT_WG16,
PT_LCONV_FAST, ...): the release libraries compile them to their defaults
(csrc/pt_device.h PT_SW), so a test that compares a variant with the default
runs BOTH sides on the diagnostic builds (libptcell_diag.so,
libptlstm_diag.so), opened beside the release ones in the same process.
test_gpu_trace.py checks that the diagnostic build's defaults equal the
release library bit for bit, which ties these comparisons to the kernels the
release library runs."""
import contextlib
import os


@contextlib.contextmanager
def variants(**env):
    """Run the block on the diagnostic libraries with the given switches set
    (values as strings or ints; restored on exit)."""
    from ptamd import _lib, lstm
    old = {k: os.environ.get(k) for k in env}
    with _lib.diag_library(), lstm.diag_library():
        os.environ.update({k: str(v) for k, v in env.items()})
        try:
            yield
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
