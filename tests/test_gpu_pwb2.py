"""k_pw_bb2 / k_pw_ba2 (the half-row backward point-wise kernels, r04, pt_pr.h)
against the CL-layout k_pw_bb / k_pw_ba they replace (PT_PWB2=0 PT_PWA2=0), in
one process: every parameter
gradient of one forward + backward, f32 (different summation order only:
1e-5 relative) and bf16 (its own rounding of the 1x1 gate and weight-gradient
operands: gradient cosine), for InT, InT no_inh and hGRU.  The reference
goldens (test_gpu_parity.py) run k_pw_bb2 too: it is the default.  Both
sides run on the diagnostic library, which reads the switches
(tests/variants.py)."""
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


@pytest.mark.parametrize("kind", ["int", "int_noinh", "hgru"])
@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_pwb2_matches_pwb(kind, dtype):
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from models import InT, ffhgru_hierarchy
    import bench
    dev = torch.device("cuda:0")
    torch.manual_seed(5)
    t = 12
    if kind == "hgru":
        m = ffhgru_hierarchy.FFhGRU(dimensions=32, timesteps=t, kernel_size=7)
    else:
        m = InT.InT(dimensions=32, timesteps=t, kernel_size=7, no_inh=(kind == "int_noinh"))
    with torch.no_grad():
        for n, p in m.named_parameters():
            if (n.startswith("unit1.bn") and n.endswith("weight")) or n.endswith(("alpha", "kappa")):
                p.uniform_(0.5, 1.5)
            elif n.endswith(("mu", "gamma")):
                p.uniform_(-0.5, 0.5)
            elif n.startswith("readout") or n.startswith("target"):
                p.mul_(4.0)
    m = m.to(dev)
    m.cell_dtype = dtype
    x, y = bench.make_data(77, 24, t, dev)
    with variants(PT_PWB2=0, PT_PWA2=0):
        g0 = _grads(m, x, y)
    with variants(PT_PWB2=1, PT_PWA2=1):
        g1 = _grads(m, x, y)
    assert g0.keys() == g1.keys()
    for k in g0:
        a, b = g1[k], g0[k]
        assert torch.isfinite(a).all(), k
        if dtype == "f32":
            assert float((a - b).abs().max()) <= 1e-7 + 1e-5 * float(b.abs().max()), (k, float((a - b).abs().max()))
        elif b.norm() > 0:
            cos = float(a @ b / (a.norm() * b.norm()))
            assert cos >= 0.999, (k, cos)
