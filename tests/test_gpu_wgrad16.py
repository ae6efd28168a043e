"""k_wgrad16 (the 16-wave k x k weight-gradient kernel, r04, bf16 k = 7)
against the 8-wave k_wgrad it replaces (PT_WG16=0), in one process: every
parameter gradient of one forward + backward.  Both read the same bf16 D / X
bands and accumulate in f32; only the order of the per-tile MFMA sums differs
(the 16-wave kernel takes a band's two pixel blocks one after the other), so
the two k x k weight gradients agree to 1e-5 relative and every other gradient
is bitwise equal.  Also: two runs of the default are bitwise equal, the
LDS-DMA band staging (default on untiled frames) equals the register staging
(PT_WGDMA=0) bitwise, also on 64x64 (tiled) hGRU frames, whose X halo rows
and columns come from the neighbouring tiles."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F
from variants import variants

pytestmark = pytest.mark.gpu


def _grads(m, x, y):
    m.zero_grad(set_to_none=True)
    out, _ = m(x)
    F.binary_cross_entropy_with_logits(out, y.reshape(-1, 1)).backward()
    torch.cuda.synchronize()
    return {k: p.grad.detach().double().flatten().cpu() for k, p in m.named_parameters() if p.grad is not None}


def _with_env(key, val, fn):
    """fn() on the diagnostic library with switch key = val (tests/variants.py)."""
    with variants(**{key: val}):
        return fn()


@pytest.mark.parametrize("kind", ["int", "int_noinh", "hgru", "hgru64"])
def test_wgrad16_matches_wgrad8(kind):
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from models import InT, ffhgru_hierarchy
    from ptamd import synth
    dev = torch.device("cuda:0")
    torch.manual_seed(7)
    t, b, hw = 10, 24, 32
    if kind.startswith("hgru"):
        m = ffhgru_hierarchy.FFhGRU(dimensions=32, timesteps=t, kernel_size=7)
        if kind == "hgru64":
            b, hw = 6, 64
    else:
        m = InT.InT(dimensions=32, timesteps=t, kernel_size=7, no_inh=(kind == "int_noinh"))
    with torch.no_grad():
        for n, p in m.named_parameters():
            if n.endswith(("alpha", "kappa")):
                p.uniform_(0.5, 1.5)
            elif n.startswith("readout") or n.startswith("target"):
                p.mul_(4.0)
    m = m.to(dev)
    m.cell_dtype = "bf16"
    clips, labels = synth.make_batch(41, b, t, h=hw, w=hw)
    x = torch.from_numpy(np.ascontiguousarray(clips.transpose(0, 4, 1, 2, 3), dtype=np.float32) / 255.0).to(dev)
    y = torch.tensor([ord(v) for v in labels], dtype=torch.float32, device=dev)
    g8 = _with_env("PT_WG16", "0", lambda: _grads(m, x, y))
    g16 = _with_env("PT_WG16", "1", lambda: _grads(m, x, y))
    g16b = _with_env("PT_WG16", "1", lambda: _grads(m, x, y))
    greg = _with_env("PT_WGDMA", "0", lambda: _grads(m, x, y))
    assert g8.keys() == g16.keys()
    nk = 0
    for k in g8:
        a, ref = g16[k], g8[k]
        assert torch.isfinite(a).all(), k
        assert torch.equal(a, g16b[k]), ("not reproducible", k)
        assert torch.equal(a, greg[k]), ("DMA vs register staging", k)
        if torch.equal(a, ref):
            continue
        nk += 1
        assert a.numel() == 32 * 32 * 49, ("only the k x k weights may differ", k)
        err = float((a - ref).abs().max())
        assert err <= 1e-5 * float(ref.abs().max()), (k, err)
    assert nk <= 2


@pytest.mark.parametrize("kind,b,t", [("int", 1, 1), ("int", 3, 2), ("int", 2, 3), ("hgru64", 1, 1),
                                      ("hgru64", 1, 2)])
def test_wgrad16_smallest_shapes(kind, b, t):
    """Fewer (frame, clip) pairs than workgroups (B*T = 1..6): one or two band
    units per workgroup, so the LDS-DMA prologue and drain run with nothing or
    one band behind them; equal to the 8-wave kernel as above."""
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from models import InT, ffhgru_hierarchy
    from ptamd import synth
    dev = torch.device("cuda:0")
    torch.manual_seed(b * 10 + t)
    hw = 64 if kind == "hgru64" else 32
    if kind == "hgru64":
        m = ffhgru_hierarchy.FFhGRU(dimensions=32, timesteps=t, kernel_size=7)
    else:
        m = InT.InT(dimensions=32, timesteps=t, kernel_size=7)
    m = m.to(dev)
    m.cell_dtype = "bf16"
    clips, labels = synth.make_batch(50 + b + t, b, t, h=hw, w=hw)
    x = torch.from_numpy(np.ascontiguousarray(clips.transpose(0, 4, 1, 2, 3), dtype=np.float32) / 255.0).to(dev)
    y = torch.tensor([ord(v) for v in labels], dtype=torch.float32, device=dev)
    g8 = _with_env("PT_WG16", "0", lambda: _grads(m, x, y))
    g16 = _with_env("PT_WG16", "1", lambda: _grads(m, x, y))
    greg = _with_env("PT_WGDMA", "0", lambda: _grads(m, x, y))
    for k in g8:
        a, ref = g16[k], g8[k]
        assert torch.isfinite(a).all(), k
        assert torch.equal(a, greg[k]), ("DMA vs register staging", k)
        err = float((a - ref).abs().max())
        assert err <= 1e-5 * float(ref.abs().max()) + 1e-12, (k, err)
