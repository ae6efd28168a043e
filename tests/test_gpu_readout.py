"""The fused readout head (include/pt_readout.h, ptamd/readout.py) against the
reference's op chain (models/InT.py:236-241: readout_conv 1x1 -> cat target
channel -> target_conv 5x5 pad 2 -> global average pool -> readout_dense),
evaluated in float64 on the CPU: logits, d E_T and all six parameter
gradients; two runs bit-identical (the parameter gradients are reduced in
clip order)."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda:0")


def _heads(c, seed):
    torch.manual_seed(seed)
    conv, target, dense = nn.Conv2d(c, 1, 1), nn.Conv2d(2, 1, 5, padding=2), nn.Linear(1, 1)
    with torch.no_grad():
        target.bias.uniform_(-0.5, 0.5)
    return conv, target, dense


def _reference(e, tgt, conv, target, dense, d_logits):
    mods = [m.double() for m in (conv, target, dense)]
    e = e.double().requires_grad_(True)
    out = torch.cat([mods[0](e), tgt.double()[:, None]], 1)
    out = F.avg_pool2d(mods[1](out), kernel_size=out.size()[2:])
    lo = mods[2](out.reshape(e.shape[0], -1))
    lo.backward(d_logits.double())
    grads = [p.grad for m in mods for p in (m.weight, m.bias)]
    return lo.detach(), e.grad, grads


@pytest.mark.parametrize("b,c,h,w", [(256, 32, 32, 32), (5, 32, 64, 64), (3, 7, 32, 32), (2, 16, 20, 36)])
def test_readout_matches_reference_chain(b, c, h, w):
    from ptamd import readout as ro
    dev = _dev()
    g = torch.Generator().manual_seed(b * 131 + c)
    e = torch.randn(b, c, h, w, generator=g)
    tgt = (torch.rand(b, h, w, generator=g) > 0.9).float()
    d_logits = torch.randn(b, 1, generator=g)
    conv, target, dense = _heads(c, b + h)
    lo_ref, de_ref, g_ref = _reference(e, tgt, *(m for m in _heads(c, b + h)), d_logits)
    runs = []
    for _ in range(2):
        mods = [m.to(dev) for m in (conv, target, dense)]
        for m in mods:
            m.zero_grad(set_to_none=True)
        ed = e.to(dev).requires_grad_(True)
        lo = ro.readout(ed, tgt.to(dev), *mods)
        lo.backward(d_logits.to(dev))
        torch.cuda.synchronize()
        runs.append((lo.detach().cpu(), ed.grad.cpu(),
                     [p.grad.cpu() for m in mods for p in (m.weight, m.bias)]))
    lo, de, grads = runs[0]
    torch.testing.assert_close(lo.double(), lo_ref, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(de.double(), de_ref, rtol=1e-5, atol=1e-9)
    for gg, gr in zip(grads, g_ref):
        torch.testing.assert_close(gg.double(), gr, rtol=1e-4, atol=1e-6)
    lo2, de2, grads2 = runs[1]
    assert torch.equal(lo, lo2) and torch.equal(de, de2)
    assert all(torch.equal(a, b2) for a, b2 in zip(grads, grads2))
