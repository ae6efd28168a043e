"""BASELINE configs[3]'s horizon: hGRU (models/ffhgru_hierarchy.py:135-173,
211-276) on 64 x 64 frames (2 x 2 tiles of 32 x 32), T = 128, and the training
guards at the headline / cfg4 sizes.

* f32 HIP vs the CPU oracle over all 128 frames (B=1: the oracle's cost),
  logits 1e-3, every gradient 1e-6 + 1e-3 max|g| (north_star bound);
* bf16 vs f32 at cfg4's per-GPU batch (B=128 clips, T=128): logits within
  BF16_LOGIT_TOL, identical 0.5 / 0 decisions outside that band, per-tensor
  gradient cosine >= 0.99;
* bf16 training at the headline (InT B=256 T=64) and cfg4 (hGRU B=128, 64 x 64,
  T=128) sizes through the cached hipGraphs: loss and gradients finite.
Measured numbers go to gpurun_out/parity_records.json (goldens.record).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from goldens import record

pytestmark = pytest.mark.gpu

BF16_LOGIT_TOL = 2e-3


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda:0")


def _perturbed(cls, t, seed):
    torch.manual_seed(seed)
    m = cls(dimensions=32, timesteps=t, kernel_size=7)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if (n.startswith("unit1.bn") and n.endswith("weight")) or n.endswith(("alpha", "kappa")):
                p.uniform_(0.5, 1.5)
            elif n.endswith(("mu", "gamma")):
                p.uniform_(-0.5, 0.5)
    return m


def _batch(seed, b, t, hw):
    from ptamd import synth
    clips, labels = synth.make_batch(seed, b, t, h=hw, w=hw)
    x = torch.from_numpy(clips.transpose(0, 4, 1, 2, 3).astype(np.float32) / 255.0)
    return x, torch.tensor([ord(v) for v in labels], dtype=torch.float32)


@pytest.mark.timeout(600)
def test_hgru_cfg4_f32_matches_oracle_over_128_frames():
    from models import ffhgru_hierarchy as hg
    from oracle import cells
    dev = _dev()
    m = _perturbed(hg.FFhGRU, 128, 41)
    x, y = _batch(42, 1, 128, 64)
    sd = {k: v.detach().clone().requires_grad_() for k, v in m.named_parameters()}
    lo, _, _ = cells.recurrent_forward(sd, x, hgru=True)
    cells.bce_logits(lo, y).backward()
    m = m.to(dev)
    m.cell_dtype = "f32"
    out, _ = m(x.to(dev))
    F.binary_cross_entropy_with_logits(out, y.to(dev).reshape(-1, 1)).backward()
    lerr = float((out.detach().cpu() - lo.detach()).abs().max())
    worst, worst_k = 0.0, None
    for k, p in m.named_parameters():
        if p.grad is None:
            continue
        r = sd[k].grad
        e = float((p.grad.cpu() - r).abs().max())
        rel = e / (float(r.abs().max()) + 1e-30)
        if rel > worst:
            worst, worst_k = rel, k
        assert e <= 1e-6 + 1e-3 * float(r.abs().max()), (k, e, rel)
    record("hgru_64x64_T128_f32_vs_oracle_B1",
           {"logit_max_abs_err": lerr, "grad_max_rel_err": worst, "grad_worst_tensor": worst_k})
    assert lerr <= 1e-3


@pytest.mark.timeout(600)
def test_hgru_cfg4_bf16_vs_f32_at_per_gpu_batch():
    from models import ffhgru_hierarchy as hg
    dev = _dev()
    m = _perturbed(hg.FFhGRU, 128, 43).to(dev)
    x, y = _batch(44, 128, 128, 64)
    x, y = x.to(dev), y.to(dev).reshape(-1, 1)
    res = {}
    for dt in ("f32", "bf16"):
        m.cell_dtype = dt
        m.zero_grad(set_to_none=True)
        out, _ = m(x)
        F.binary_cross_entropy_with_logits(out, y).backward()
        torch.cuda.synchronize()
        res[dt] = (out.detach().double().flatten().cpu(),
                   {k: p.grad.detach().double().flatten().cpu() for k, p in m.named_parameters()
                    if p.grad is not None})
    (o32, g32), (o16, g16) = res["f32"], res["bf16"]
    err = (o16 - o32).abs()
    rec = {"logit_max_abs_err": float(err.max()), "logit_mean_abs_err": float(err.mean()),
           "logit_spread": float(o32.max() - o32.min())}
    for name, thr in (("train_0.5", 0.5), ("eval_0", 0.0)):
        far = (o32 - thr).abs() > BF16_LOGIT_TOL
        rec[f"flips_{name}"] = int(((o16 > thr) != (o32 > thr))[far].sum())
        rec[f"in_band_{name}"] = int((~far).sum())
    cos = {k: float(g16[k] @ g32[k] / (g16[k].norm() * g32[k].norm()))
           for k in g32 if g32[k].norm() > 1e-12}
    rec["grad_cosine_min"] = min(cos.values())
    rec["grad_cosine_min_tensor"] = min(cos, key=cos.get)
    record("hgru_64x64_T128_B128_bf16_vs_f32", rec)
    assert torch.isfinite(o16).all()
    assert rec["logit_max_abs_err"] <= BF16_LOGIT_TOL, rec
    assert rec["flips_train_0.5"] == 0 and rec["flips_eval_0"] == 0, rec
    assert rec["grad_cosine_min"] >= 0.99, rec


@pytest.mark.timeout(600)
@pytest.mark.parametrize("cell,b,t,hw,steps", [("int", 256, 64, 32, 40), ("hgru", 128, 128, 64, 12)])
def test_bf16_training_stays_finite_at_bench_sizes(cell, b, t, hw, steps):
    """The headline (BASELINE configs[1]) and cfg4 (configs[3], per GPU) bf16
    training steps through the cached hipGraphs: finite loss and gradients."""
    from models import InT, ffhgru_hierarchy as hg
    dev = _dev()
    torch.manual_seed(9)
    m = (hg.FFhGRU if cell == "hgru" else InT.InT)(dimensions=32, timesteps=t, kernel_size=7).to(dev)
    m.cell_dtype = "bf16"
    opt = torch.optim.Adam(m.parameters(), lr=3e-4)
    data = [tuple(v.to(dev) for v in _batch(200 + i, b, t, hw)) for i in range(2)]
    losses = []
    for s in range(steps):
        x, y = data[s % 2]
        out, _ = m(x.clone())
        loss = F.binary_cross_entropy_with_logits(out, y.reshape(-1, 1))
        loss.backward()
        bad = [k for k, p in m.named_parameters() if p.grad is not None and not torch.isfinite(p.grad).all()]
        assert torch.isfinite(loss) and not bad, (s, float(loss), bad)
        losses.append(float(loss))
        opt.step()
        opt.zero_grad(set_to_none=True)
    record(f"bf16_training_{cell}_B{b}_T{t}_{hw}x{hw}", {"steps": steps, "loss_first": losses[0],
                                                       "loss_last": losses[-1]})
