"""GPU parity: the HIP InT cell (through the drop-in ``models.InT``) against the
reference's golden vectors and the CPU oracle.

f32 mode is the parity path (exact-f32 MFMA): logits / per-frame states / gates
/ every parameter gradient / post-Adam parameters within 1e-3 of the reference
(the north_star bound), accuracy decisions bit-identical.  bf16 mode is the
throughput path and gets its own, stated, looser bound.
"""
import numpy as np
import pytest
import torch

from goldens import cfg, load, params, prepared_input

pytestmark = pytest.mark.gpu

# k = 7 (the engine's), the constructors' default k = 15 and k = 9; C = 32 and
# C < 32 (zero-padded to the MFMA tile inside the library)
INT_TAGS = ["int_c32", "int_tanh", "int_lesion", "int_noinh", "int_cfg1", "int_64x96",
            "int_tiny_c8", "int_k15", "int_k9_c16"]
HGRU_TAGS = ["hgru_c32", "hgru_b4t16", "hgru_64", "hgru_k15_64", "hgru_c24"]


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda:0")


def _model(g, dtype="f32"):
    from models import InT as int_mod
    import torch.nn.functional as F
    c = cfg(g)
    if c["cell"] == "hgru":
        from models import ffhgru_hierarchy as hg
        m = hg.FFhGRU(dimensions=c["dims"], timesteps=8, kernel_size=c["k"])
        m.load_state_dict(params(g), strict=True)
        m.cell_dtype = dtype
        return m
    kw = dict(dimensions=c["dims"], timesteps=8, kernel_size=c["k"], no_inh=c["no_inh"],
              nl=F.tanh if c["act"] == "tanh" else F.softplus)
    for les in c["lesion"]:
        kw["lesion_" + les] = True
    m = int_mod.InT(**kw)
    sd = params(g)
    m.load_state_dict(sd, strict=True)
    m.cell_dtype = dtype
    return m


def _err(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    assert a.shape == b.shape, (a.shape, b.shape)
    return float(np.abs(a - b).max()), float(np.abs(b).max())


def _assert_close(name, a, b, atol, rtol=0.0):
    e, s = _err(a, b)
    assert e <= atol + rtol * s, f"{name}: max|err| {e:.3e} > {atol:.1e} + {rtol:.1e}*{s:.3e}"


@pytest.mark.parametrize("tag", INT_TAGS + HGRU_TAGS)
def test_forward_testmode_f32(tag):
    dev = _dev()
    g = load(tag)
    m = _model(g).to(dev)
    x, _ = prepared_input(g)
    m.eval()
    with torch.no_grad():
        logits, states, gates = m(x.to(dev), testmode=True)
    _assert_close("logits", logits.cpu(), g["logits"], 1e-3)
    _assert_close("states", states.cpu(), g["states"], 1e-3)
    if "gates" in g:
        _assert_close("gates", gates.cpu(), g["gates"], 1e-3)
    # eval accuracy (logit > 0, test_model.py:127) bit-identical
    assert np.array_equal(logits.cpu().numpy() > 0, g["logits"] > 0)


@pytest.mark.parametrize("tag", INT_TAGS + HGRU_TAGS)
def test_bptt_grads_and_adam_f32(tag):
    dev = _dev()
    g = load(tag)
    m = _model(g).to(dev)
    x, y = prepared_input(g)
    m.train()
    out, jv = m(x.to(dev))
    loss = torch.nn.functional.binary_cross_entropy_with_logits(out, y.to(dev).reshape(-1, 1))
    loss.backward()
    _assert_close("train logits", out.detach().cpu(), g["train_logits"], 1e-3)
    assert abs(loss.item() - float(g["loss"])) < 1e-4
    # training accuracy decision (acc_scores thresholds logits at 0.5, misc_functions.py:41)
    assert np.array_equal(out.detach().cpu().numpy() > 0.5, g["train_logits"] > 0.5)
    ref_grads = {k[len("grad."):]: v for k, v in g.items() if k.startswith("grad.")}
    got = {k: p.grad for k, p in m.named_parameters() if p.grad is not None}
    assert set(got) == set(ref_grads), set(got) ^ set(ref_grads)
    for k, v in ref_grads.items():
        _assert_close(f"grad {k}", got[k].cpu(), v, 1e-6, 1e-3)
    opt = torch.optim.Adam(m.parameters(), lr=3e-4)
    opt.step()
    for k, p in m.named_parameters():
        if k == "unit1.w":
            continue
        _assert_close(f"adam {k}", p.detach().cpu(), g["adam." + k], 1e-6, 1e-3)


# bf16 cell vs the reference goldens (perturbed parameters, up to 32 frames):
# the measured errors are recorded (gpurun_out/parity_records.json)
BF16_GOLDEN_TOL = 2e-2


@pytest.mark.parametrize("tag", INT_TAGS + HGRU_TAGS)
def test_forward_bf16_tolerance(tag):
    """bf16 operands / saved states, f32 accumulation: logits within
    BF16_GOLDEN_TOL and per-frame states within BF16_GOLDEN_TOL (absolute +
    relative to max|state|) of the reference after up to 32 recurrent steps."""
    dev = _dev()
    g = load(tag)
    m = _model(g, "bf16").to(dev)
    x, _ = prepared_input(g)
    with torch.no_grad():
        logits, states, _ = m(x.to(dev), testmode=True)
    from goldens import record
    lerr, _ = _err(logits.cpu(), g["logits"])
    serr, sscale = _err(states.cpu(), g["states"])
    record(f"bf16_vs_reference_{tag}", {"logit_max_abs_err": lerr, "state_max_abs_err": serr,
                                        "state_max_abs": sscale})
    _assert_close("bf16 logits", logits.cpu(), g["logits"], BF16_GOLDEN_TOL)
    _assert_close("bf16 states", states.cpu(), g["states"], BF16_GOLDEN_TOL, BF16_GOLDEN_TOL)


@pytest.mark.parametrize("tag", INT_TAGS + HGRU_TAGS)
def test_bf16_grads_direction(tag):
    """bf16 BPTT gradients point the same way as the reference's (cosine > 0.99
    per parameter tensor with a non-trivial gradient), on every InT / hGRU
    golden (r06: all of them -- k = 15 / 9, C < 32, tanh, lesions, no_inh,
    tiled frames -- not only the k = 7, C = 32 ones)."""
    dev = _dev()
    g = load(tag)
    m = _model(g, "bf16").to(dev)
    x, y = prepared_input(g)
    out, _ = m(x.to(dev))
    torch.nn.functional.binary_cross_entropy_with_logits(out, y.to(dev).reshape(-1, 1)).backward()
    from goldens import record
    cosines = {}
    for k, p in m.named_parameters():
        if p.grad is None:
            continue
        a = p.grad.detach().cpu().double().flatten()
        b = torch.from_numpy(g["grad." + k]).double().flatten()
        if b.norm() < 1e-8:
            continue
        cosines[k] = float(a @ b / (a.norm() * b.norm() + 1e-30))
    worst = min(cosines, key=cosines.get)
    record(f"bf16_grad_cosine_{tag}", {"min_cosine": cosines[worst], "tensor": worst})
    for k, cos in cosines.items():
        assert cos > 0.99, f"{k}: cosine {cos:.4f}"


def test_oracle_agrees_on_device_sized_batch():
    """Size-independent cross-check beyond the fixtures: a fresh seeded batch
    (B=8, T=16), HIP f32 vs the CPU oracle, logits and all grads."""
    from oracle import cells
    from ptamd import synth
    from models import InT as int_mod
    dev = _dev()
    torch.manual_seed(7)
    m = int_mod.InT(dimensions=32, timesteps=16, kernel_size=7)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if n.startswith("unit1.bn") and n.endswith("weight"):
                p.uniform_(0.5, 1.5)
            elif n.endswith(("alpha", "kappa")):
                p.uniform_(0.5, 1.5)
            elif n.endswith(("mu", "gamma")):
                p.uniform_(-0.5, 0.5)
    clips, labels = synth.make_batch(11, 8, 16)
    x = torch.from_numpy(clips.transpose(0, 4, 1, 2, 3) / 255.0).float()
    y = torch.tensor([ord(b) for b in labels], dtype=torch.float32)
    sd = {k: v.detach().clone().requires_grad_(v.requires_grad) for k, v in m.named_parameters()}
    sd["unit1.w"].requires_grad_(False)
    lo, _, _ = cells.recurrent_forward(sd, x)
    cells.bce_logits(lo, y).backward()
    m = m.to(dev)
    out, _ = m(x.to(dev))
    torch.nn.functional.binary_cross_entropy_with_logits(out, y.to(dev).reshape(-1, 1)).backward()
    _assert_close("logits", out.detach().cpu(), lo.detach(), 1e-3)
    for k, p in m.named_parameters():
        if p.grad is not None:
            _assert_close(f"grad {k}", p.grad.cpu(), sd[k].grad, 1e-6, 1e-3)


@pytest.mark.parametrize("tag", ["int_c32", "hgru_c32"])
def test_step_api_on_gpu_matches_fused_cell(tag):
    """The per-step cell API (rCell / hConvGRUCell.forward, torch ops on the
    device) stepped over the clip agrees with the fused HIP recurrence."""
    dev = _dev()
    g = load(tag)
    m = _model(g).to(dev)
    x, _ = prepared_input(g)
    x = x.to(dev)
    with torch.no_grad():
        fused, fstates, fgates = m(x, testmode=True)
        xbn = m.nl(m.preproc(x))
        b, c, t_len, h, w = xbn.shape
        inh = torch.zeros((b, c, h, w), device=dev)
        exc = torch.zeros((b, c, h, w), device=dev)
        states = []
        for t in range(t_len):
            inh, exc, att = m.unit1(xbn[:, :, t], inh, exc, activ=m.nl, testmode=True)
            states.append(m.readout_conv(exc))
        stepped = m.readout(exc, x)
    _assert_close("logits", stepped.cpu(), fused.cpu(), 1e-3)
    _assert_close("states", torch.stack(states, 1).cpu(), fstates.cpu(), 1e-3)
