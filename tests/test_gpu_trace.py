"""Diagnostic switches (include/pt_cell.h).

* The release library (libptcell.so) ignores them: with PT_CELL_ABLATE
  (phase-skipping bits whose results are garbage) and PT_CELL_DEBUG_STOP set
  in the environment, forward and backward are bit-identical to a run without
  them, and pt_cell_trace is refused.
* The diagnostic build (libptcell_diag.so, -DPT_DIAG=1, loaded by tools/ with
  ptamd._lib.use_diag()): with a trace buffer set, one frame's point-wise and
  fused-forward launches stamp their phases with the 100 MHz real-time
  counter, per sampled workgroup, in order; with the buffer cleared nothing is
  written and the results are unchanged (tools/trace.py reads the same
  records).  Run in a child process, which loads the diagnostic library.
"""
import ctypes
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _setup():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from models import InT
    dev = torch.device("cuda:0")
    torch.manual_seed(5)
    m = InT.InT(dimensions=32, timesteps=4, kernel_size=7).to(dev)
    m.cell_dtype = "bf16"
    x = torch.rand(8, 3, 4, 32, 32, device=dev)

    def run():
        m.zero_grad(set_to_none=True)
        out, _ = m(x)
        out.sum().backward()
        torch.cuda.synchronize()
        return out.detach().clone(), {k: p.grad.detach().clone() for k, p in m.named_parameters()
                                      if p.grad is not None}
    return run


# every switch at a non-default value (phase-skipping ablations, a debug stop
# and the kernel-variant A/B switches)
NON_DEFAULT = dict(PT_CELL_ABLATE=str(1 | 4 | 8 | 32 | 512), PT_CELL_DEBUG_STOP="2",
                   PT_CELL_FUSED="0", PT_PWB2="0", PT_PWA2="1", PT_WG16="0", PT_WGDMA="0",
                   PT_CELL_PERSIST="1", PT_XCD_MAP="0", PT_CONV_BAND="0", PT_CPA="0", PT_BAND2_TILED="0",
                   PT_FUSED_TILED="1")


def test_release_library_ignores_the_diagnostic_switches():
    """With every diagnostic and kernel-variant switch set to a non-default
    value the release library's forward and backward are bit-identical to a
    run without them; and the diagnostic build at its defaults equals the
    release library bit for bit (so the A/B tests, which compare variants on
    the diagnostic build, compare against the release kernels)."""
    from ptamd import _lib
    run = _setup()
    lib = _lib.load()
    assert "diag" not in lib.pt_version().decode()
    o0, g0 = run()
    os.environ.update(NON_DEFAULT)
    try:
        o1, g1 = run()
    finally:
        for k in NON_DEFAULT:
            os.environ.pop(k)
    assert torch.equal(o0, o1)
    for k in g0:
        assert torch.equal(g0[k], g1[k]), k
    assert lib.pt_cell_trace(None, -1) == 2                  # PT_ERR_UNSUPPORTED
    assert b"diagnostic build" in lib.pt_last_error()
    with _lib.diag_library() as dl:
        assert "diag" in dl.pt_version().decode()
        o2, g2 = run()
    assert torch.equal(o0, o2)
    for k in g0:
        assert torch.equal(g0[k], g2[k]), ("diag build at its defaults", k)


_CHILD = r"""
import ctypes, os, sys
sys.path[:0] = [{repo!r}, os.path.join({repo!r}, "pathtracker-models_amd"), os.path.join({repo!r}, "tests")]
import torch
from ptamd import _lib
_lib.use_diag()
from test_gpu_trace import _setup
run = _setup()
lib = _lib.load()
assert "diag" in lib.pt_version().decode()
o0, g0 = run()
dev = torch.device("cuda:0")
buf = torch.zeros(_lib.NKINDS * _lib.TRACE_WG * _lib.TRACE_SLOTS, dtype=torch.int64, device=dev)
assert lib.pt_cell_trace(ctypes.c_void_p(buf.data_ptr()), 1) == 0
try:
    o1, g1 = run()
finally:
    lib.pt_cell_trace(None, -1)
assert torch.equal(o0, o1) and all(torch.equal(g0[k], g1[k]) for k in g0)
tr = buf.view(_lib.NKINDS, _lib.TRACE_WG, _lib.TRACE_SLOTS).cpu()
# (kind, ordered phase slots, per-wave slot base, waves): r06 adds the workgroup's
# XCC / HW_ID word (slot 7, bit 40 set) and per-wave stamps
for kind, slots, wbase, nw in (("k_pw_bb", [0, 1, 2, 3, 4, 5, 6], 8, 8), ("k_pw_ba", [0, 2, 3, 4, 5, 6], 8, 4),
                               ("k_fused_fa", [0, 2, 3, 4, 5, 6], 16, 8),
                               ("k_fused_fb", [0, 2, 3, 4, 5, 6], 16, 8), ("k_conv_bb", [0, 1, 2], 16, 8)):
    r = tr[_lib.KIND_NAMES.index(kind)]
    live = r[:, 0] > 0
    assert live.any(), kind
    assert ((r[live][:, 7] >> 40) == 1).all(), kind
    w = r[live][:, wbase:wbase + nw]
    assert (w > 0).all() and (w >= r[live][:, slots[0]:slots[0] + 1]).all(), kind
    r = r[live][:, slots]
    assert (r > 0).all(), kind
    assert (r[:, 1:] >= r[:, :-1]).all(), kind            # phases in order per workgroup
buf.zero_()
run()                                                     # cleared: no stamps
assert int(buf.abs().sum()) == 0
print("trace ok")
"""


@pytest.mark.timeout(240)
def test_diag_build_phase_stamps_are_written_in_order_and_change_nothing():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    env = dict(os.environ)
    env.pop("PT_CELL_ABLATE", None)
    r = subprocess.run([sys.executable, "-c", _CHILD.format(repo=REPO)], env=env, cwd=REPO,
                       capture_output=True, text=True, timeout=220)
    assert r.returncode == 0 and "trace ok" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]
