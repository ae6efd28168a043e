"""Edge cases and size-independent properties of the HIP cell (InT / hGRU).

* smallest shapes against the CPU oracle (f32, 1e-3): one clip, one frame;
  an odd batch with two frames; a single-clip 64x64 hGRU (tiles, B=1); the
  same shapes through the bf16 path (logits 2e-2, gradient cosine > 0.99,
  r06); kernel sizes 5, 3, 1 (no golden holds one) in f32 and bf16;
* a 520-clip batch (more than one dispatch round) bf16 against f32;
* raw u8 clips [B,T,H,W,3] as the cell input (PT_X_U8_NTHWC) against the
  f32 tensor engine.prepare_data builds from them: same values, so the cell's
  outputs and gradients agree bit for bit (InT f32 / bf16, tiled hGRU);
* at the headline size (B=256, T=64, bf16) where the oracle is too slow:
  permutation equivariance (BatchNorm's batch statistics are symmetric in the
  clips, so permuting the clips permutes the logits, up to the rounding of the
  fp64 statistics sums taken in the permuted order) and bitwise run-to-run
  reproducibility.
"""

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda:0")


def _perturbed(cls, t, seed, k=7, **kw):
    torch.manual_seed(seed)
    m = cls(dimensions=32, timesteps=t, kernel_size=k, **kw)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if (n.startswith("unit1.bn") and n.endswith("weight")) or n.endswith(("alpha", "kappa")):
                p.uniform_(0.5, 1.5)
            elif n.endswith(("mu", "gamma")):
                p.uniform_(-0.5, 0.5)
    return m


def _close(name, a, b, atol, rtol=0.0):
    a = np.asarray(a.detach().cpu() if torch.is_tensor(a) else a, np.float64)
    b = np.asarray(b.detach().cpu() if torch.is_tensor(b) else b, np.float64)
    err = np.abs(a - b).max()
    assert err <= atol + rtol * np.abs(b).max(), f"{name}: {err:.3e}"


def _vs_oracle(m, x, y, hgru=False):
    from oracle import cells
    dev = _dev()
    sd = {k: v.detach().clone().requires_grad_(k != "unit1.w") for k, v in m.named_parameters()}
    lo, _, _ = cells.recurrent_forward(sd, x, hgru=hgru)
    cells.bce_logits(lo, y).backward()
    m = m.to(dev)
    out, _ = m(x.to(dev))
    F.binary_cross_entropy_with_logits(out, y.to(dev).reshape(-1, 1)).backward()
    _close("logits", out, lo, 1e-3)
    for k, p in m.named_parameters():
        if p.grad is not None:
            _close(f"grad {k}", p.grad, sd[k].grad, 1e-6, 1e-3)


def _batch(seed, b, t, hw=32):
    from ptamd import synth
    clips, labels = synth.make_batch(seed, b, t, h=hw, w=hw)
    x = torch.from_numpy(clips.transpose(0, 4, 1, 2, 3) / 255.0).float()
    return x, torch.tensor([ord(v) for v in labels], dtype=torch.float32)


@pytest.mark.parametrize("k", [5, 3, 1])
def test_int_small_kernels_vs_oracle(k):
    """k < 7 (no golden holds one): the f32 cell at 1e-3 against the oracle,
    and the bf16 cell (fused forward, banded backward convs with their
    pre-loaded addends) within the bf16 golden bounds: logits 2e-2, gradient
    cosine > 0.99 per tensor."""
    from models import InT
    x, y = _batch(60 + k, 3, 4)
    m = _perturbed(InT.InT, 4, seed=k, k=k)
    _vs_oracle(m, x, y)
    _vs_oracle_bf16(m, x, y)


def _vs_oracle_bf16(m, x, y, hgru=False):
    """The bf16 cell against the oracle within the bf16 golden bounds: logits
    2e-2, gradient cosine > 0.99 per tensor with a non-trivial gradient."""
    from oracle import cells
    dev = _dev()
    sd = {n: v.detach().cpu().clone().requires_grad_(n != "unit1.w") for n, v in m.named_parameters()}
    lo, _, _ = cells.recurrent_forward(sd, x, hgru=hgru)
    cells.bce_logits(lo, y).backward()
    m = m.to(dev)
    m.zero_grad(set_to_none=True)
    m.cell_dtype = "bf16"
    out, _ = m(x.to(dev))
    F.binary_cross_entropy_with_logits(out, y.to(dev).reshape(-1, 1)).backward()
    _close("bf16 logits", out, lo, 2e-2)
    for n, p in m.named_parameters():
        if p.grad is None or sd[n].grad is None or sd[n].grad.norm() < 1e-8:
            continue
        a, b = p.grad.detach().cpu().double().flatten(), sd[n].grad.double().flatten()
        cos = float(a @ b / (a.norm() * b.norm() + 1e-30))
        assert cos > 0.99, f"bf16 {n}: cosine {cos:.4f}"


def test_int_large_batch_bf16_vs_f32():
    """B = 520 clips (past the 256 / 512 workgroups of one dispatch round, not
    a multiple of 8 clips per XCD): the bf16 cell against the f32 cell on the
    same clips -- logits within 2e-2, gradient cosine > 0.99 per tensor -- and
    the bf16 step bitwise reproducible."""
    from models import InT
    dev = _dev()
    x, y = _batch(91, 520, 6)
    x, y = x.to(dev), y.to(dev)
    m = _perturbed(InT.InT, 6, seed=17).to(dev)

    def run(dtype):
        m.cell_dtype = dtype
        m.zero_grad(set_to_none=True)
        out, _ = m(x)
        F.binary_cross_entropy_with_logits(out, y.reshape(-1, 1)).backward()
        return out.detach().clone(), {n: p.grad.detach().clone() for n, p in m.named_parameters()
                                      if p.grad is not None}
    o32, g32 = run("f32")
    o16, g16 = run("bf16")
    o16b, g16b = run("bf16")
    assert torch.equal(o16, o16b) and all(torch.equal(g16[n], g16b[n]) for n in g16)
    _close("bf16 logits", o16, o32, 2e-2)
    for n in g32:
        a, b = g16[n].double().flatten(), g32[n].double().flatten()
        if b.norm() < 1e-8:
            continue
        cos = float(a @ b / (a.norm() * b.norm() + 1e-30))
        assert cos > 0.99, f"{n}: cosine {cos:.4f}"


@pytest.mark.parametrize("b,t", [(1, 1), (3, 2), (2, 1)])
def test_int_smallest_shapes(b, t):
    from models import InT
    x, y = _batch(20 + b + t, b, t)
    _vs_oracle(_perturbed(InT.InT, t, seed=b * 10 + t), x, y)


@pytest.mark.parametrize("b,t", [(1, 1), (3, 2), (2, 3)])
def test_int_smallest_shapes_bf16(b, t):
    """The bf16 path (fused forward, the fused backward A from frame 1, the
    first / last frame's k_pw_ba) at one and two frames."""
    from models import InT
    x, y = _batch(40 + b + t, b, t)
    _vs_oracle_bf16(_perturbed(InT.InT, t, seed=b * 10 + t + 1), x, y)


def test_hgru_single_clip_tiled():
    from models import ffhgru_hierarchy as hg
    x, y = _batch(31, 1, 3, hw=64)
    _vs_oracle(_perturbed(hg.FFhGRU, 3, seed=5), x, y, hgru=True)
    _vs_oracle_bf16(_perturbed(hg.FFhGRU, 3, seed=5), x, y, hgru=True)


@pytest.mark.parametrize("cell,dtype,hw", [("int", "f32", 32), ("int", "bf16", 32),
                                           ("hgru", "bf16", 64)])
def test_u8_input_matches_f32_input(cell, dtype, hw):
    import types
    from models import InT, ffhgru_hierarchy as hg
    from ptamd import synth
    from utils import engine
    dev = _dev()
    clips, labels = synth.make_batch(47, 4, 5, h=hw, w=hw)
    args = types.SimpleNamespace(pretrained=False)
    x, y = engine.prepare_data(clips, labels, args, dev, False)
    xu, _ = engine.prepare_data(clips, labels, args, dev, False, keep_u8=True)
    assert xu.dtype == torch.uint8
    m = _perturbed(hg.FFhGRU if cell == "hgru" else InT.InT, 5, seed=13).to(dev)
    m.cell_dtype = dtype
    res = []
    for inp in (x, xu):
        m.zero_grad(set_to_none=True)
        out, _ = m(inp)
        F.binary_cross_entropy_with_logits(out, y.reshape(-1, 1)).backward()
        res.append((out.detach().clone(), {k: p.grad.detach().clone()
                                           for k, p in m.named_parameters() if p.grad is not None}))
    (o0, g0), (o1, g1) = res
    assert torch.isfinite(o1).all()
    assert torch.equal(o1, o0)
    assert g0.keys() == g1.keys()
    for k in g0:
        if k.startswith(("unit1.", "preproc.")):      # the library's own gradients
            assert torch.equal(g1[k], g0[k]), k
        else:                                          # readout: MIOpen / hipBLASLt
            _close(f"grad {k}", g1[k], g0[k], 1e-7, 1e-5)


def _headline_model(dev):
    from models import InT
    torch.manual_seed(1234)
    m = InT.InT(dimensions=32, timesteps=64, kernel_size=7).to(dev)
    m.cell_dtype = "bf16"
    return m


def test_headline_size_permutation_and_reproducibility():
    dev = _dev()
    import bench
    x, y = bench.make_data(77, 256, 64, dev)
    m = _headline_model(dev)
    perm = torch.randperm(256, generator=torch.Generator().manual_seed(3)).to(dev)
    out1, _ = m(x)
    F.binary_cross_entropy_with_logits(out1, y.reshape(-1, 1)).backward()
    g1 = {k: p.grad.detach().clone() for k, p in m.named_parameters() if p.grad is not None}
    m.zero_grad(set_to_none=True)
    out2, _ = m(x)                                       # same input again
    F.binary_cross_entropy_with_logits(out2, y.reshape(-1, 1)).backward()
    # the cell is bitwise reproducible (deterministic BatchNorm sums); the
    # readout's MIOpen/hipBLASLt gradients need not be, so only the cell's
    # parameters (the library's own output) are compared bit for bit
    assert torch.equal(out2, out1)
    for k, p in m.named_parameters():
        if p.grad is not None:
            if k.startswith(("unit1.", "preproc.")):
                assert torch.equal(p.grad, g1[k]), k
            else:
                _close(f"rerun grad {k}", p.grad, g1[k], 1e-7, 1e-5)
    m.zero_grad(set_to_none=True)
    out3, _ = m(x[perm].contiguous())                    # clips permuted
    F.binary_cross_entropy_with_logits(out3, y[perm].reshape(-1, 1)).backward()
    _close("permuted logits", out3, out1[perm], 1e-4)
    for k, p in m.named_parameters():
        if p.grad is not None:                           # the mean loss is permutation invariant
            _close(f"permuted grad {k}", p.grad, g1[k], 1e-6, 2e-3)


@pytest.mark.parametrize("cls,kw,hw", [("int", {}, 32), ("int", {"dimensions": 20, "kernel_size": 11}, 32),
                                      ("hgru", {"kernel_size": 13}, 64)])
def test_constructor_defaults_and_other_sizes(cls, kw, hw):
    """The reference constructors' defaults (kernel_size=15, InT.py:184 /
    ffhgru_hierarchy.py:178) and other (C, k) pairs against the CPU oracle."""
    from models import InT, ffhgru_hierarchy as hg
    mod = hg.FFhGRU if cls == "hgru" else InT.InT
    args = {"dimensions": 32, **kw}
    torch.manual_seed(17)
    m = mod(args.pop("dimensions"), 3, **args)
    assert m.kernel_size == kw.get("kernel_size", 15)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if (n.startswith("unit1.bn") and n.endswith("weight")) or n.endswith(("alpha", "kappa")):
                p.uniform_(0.5, 1.5)
            elif n.endswith(("mu", "gamma")):
                p.uniform_(-0.5, 0.5)
    x, y = _batch(61, 2, 3, hw=hw)
    _vs_oracle(m, x, y, hgru=cls == "hgru")


def test_k15_bf16_close_to_f32():
    """bf16 cell at the constructors' default k = 15: logits and gradient
    directions against the f32 cell (same parameters and clips)."""
    from models import InT
    dev = _dev()
    torch.manual_seed(19)
    m = InT.InT(32, 6).to(dev)
    x, y = _batch(63, 8, 6)
    x, y = x.to(dev), y.to(dev).reshape(-1, 1)
    res = {}
    for dt in ("f32", "bf16"):
        m.cell_dtype = dt
        m.zero_grad(set_to_none=True)
        out, _ = m(x)
        F.binary_cross_entropy_with_logits(out, y).backward()
        res[dt] = (out.detach().double(), {k: p.grad.detach().double().flatten()
                                           for k, p in m.named_parameters() if p.grad is not None})
    (o32, g32), (o16, g16) = res["f32"], res["bf16"]
    assert float((o16 - o32).abs().max()) < 5e-2
    for k in g32:
        if g32[k].norm() > 1e-12:
            cos = float(g16[k] @ g32[k] / (g16[k].norm() * g32[k].norm()))
            assert cos > 0.99, (k, cos)
