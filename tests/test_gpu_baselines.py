"""Comparison baselines on the GPU (stock PyTorch-ROCm, fp32): same golden
vectors as tests/test_baselines_cpu.py, looser bounds for the MIOpen
convolution algorithms: outputs within 1e-4 (max-relative); gradients within
2e-2 in norm, ||g - g_ref|| / ||g_ref|| (MIOpen's Conv3d backward-weight
kernels on gfx950 measured up to 1.4e-2 max-relative on single entries of the
R3D's deeper layers; the reference fp32 CPU values are the golden ones).
These are stock-PyTorch comparison baselines, not the HIP hot path."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from goldens import load, prepared_input

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda:0")


def _close(name, a, b, rtol, atol=1e-6):
    a = np.asarray(a.detach().float().cpu(), np.float64)
    b = np.asarray(b, np.float64)
    err = np.abs(a - b).max()
    assert err <= atol + rtol * np.abs(b).max(), f"{name}: {err:.3e}"


@pytest.mark.parametrize("tag", ["gru_c16", "r3d_small"])
def test_baseline_on_gpu(tag):
    dev = _dev()
    torch.backends.cudnn.allow_tf32 = False
    g = load(tag)
    if tag == "gru_c16":
        from models import kys
        m = kys.GRU(dimensions=int(g["cfg_dims"]), timesteps=4, kernel_size=7)
        m.load_state_dict({k[6:]: torch.from_numpy(v.copy()) for k, v in g.items() if k.startswith("param.")})
    else:
        from models import nostridetv_cc_smallest as r3d
        m = r3d.r3d_18(timesteps=4)
        m.load_state_dict({k[5:]: torch.from_numpy(v.copy()) for k, v in g.items() if k.startswith("init.")})
    m = m.to(dev)
    x, y = prepared_input(g)
    m.train()
    logits, _ = m(x.to(dev))
    F.binary_cross_entropy_with_logits(logits, y.to(dev).reshape(-1, 1)).backward()
    _close("train logits", logits, g["train_logits"], 1e-4)
    for k, p in m.named_parameters():
        if "grad." + k in g:
            a = p.grad.detach().double().cpu().flatten()
            b = torch.from_numpy(g["grad." + k]).double().flatten()
            rel = float((a - b).norm() / (b.norm() + 1e-30))
            assert rel < 2e-2, f"grad {k}: relative norm error {rel:.3e}"
