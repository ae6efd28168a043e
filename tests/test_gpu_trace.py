"""pt_cell_trace (diagnostics C-ABI, include/pt_cell.h): with a buffer set,
one frame's point-wise and fused-forward launches stamp their phases with the
100 MHz real-time counter, per sampled workgroup, in order; with the buffer
cleared nothing is written and the results are unchanged (tools/trace.py
reads the same records)."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_phase_stamps_are_written_in_order_and_change_nothing():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from models import InT
    from ptamd import _lib
    dev = torch.device("cuda:0")
    lib = _lib.load()
    torch.manual_seed(5)
    m = InT.InT(dimensions=32, timesteps=4, kernel_size=7).to(dev)
    m.cell_dtype = "bf16"
    x = torch.rand(8, 3, 4, 32, 32, device=dev)

    def run():
        m.zero_grad(set_to_none=True)
        out, _ = m(x)
        out.sum().backward()
        torch.cuda.synchronize()
        return out.detach().clone(), m.unit1.w_exc.grad.detach().clone()

    o0, g0 = run()
    buf = torch.zeros(_lib.NKINDS * 256 * 16, dtype=torch.int64, device=dev)
    lib.pt_cell_trace(ctypes.c_void_p(buf.data_ptr()), 1)
    try:
        o1, g1 = run()
    finally:
        lib.pt_cell_trace(None, -1)
    assert torch.equal(o0, o1) and torch.equal(g0, g1)
    tr = buf.view(_lib.NKINDS, 256, 16).cpu()
    for kind, slots in (("k_pw_bb", [0, 1, 2, 3, 4, 5, 6]), ("k_pw_ba", [0, 2, 3, 4, 5, 6]),
                        ("k_fused_fa", [0, 2, 3, 4, 5, 6]), ("k_fused_fb", [0, 2, 3, 4, 5, 6])):
        r = tr[_lib.KIND_NAMES.index(kind)]
        live = r[:, 0] > 0
        assert live.any(), kind
        r = r[live][:, slots]
        assert (r > 0).all(), kind
        assert (r[:, 1:] >= r[:, :-1]).all(), kind            # phases in order per workgroup
    buf.zero_()
    run()                                                     # cleared: no stamps
    assert int(buf.abs().sum()) == 0
