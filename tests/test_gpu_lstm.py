"""GPU parity of the HIP ConvLSTM cell (models/convlstm.py drop-in) against the
reference's golden vectors and the CPU oracle.

f32 mode (exact-f32 MFMA) is the parity path: outputs, loss, the Jacobian
penalty and every parameter gradient within 1e-3 (relative to each tensor's
scale for gradients, the north_star bound).  bf16 is the throughput path with
its own, stated, looser bound.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from goldens import load, params

pytestmark = pytest.mark.gpu

LSTM_TAGS = ["convlstm_k7", "convlstm_k15", "convlstm_t2"]


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda:0")


def _model(g, dtype="f32"):
    from models import convlstm as cl
    m = cl.ConvLSTM(timesteps=int(g["cfg_timesteps"]), filt_size=int(g["cfg_filt"]))
    m.load_state_dict(params(g), strict=True)
    m.cell_dtype = dtype
    return m


def _assert_close(name, a, b, atol, rtol=0.0):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    assert a.shape == b.shape, (name, a.shape, b.shape)
    e, s = float(np.abs(a - b).max()), float(np.abs(b).max())
    assert e <= atol + rtol * s, f"{name}: max|err| {e:.3e} > {atol:.1e} + {rtol:.1e}*{s:.3e}"


@pytest.mark.parametrize("tag", LSTM_TAGS)
def test_convlstm_eval_f32(tag):
    dev = _dev()
    g = load(tag)
    m = _model(g).to(dev).eval()
    img = torch.from_numpy(g["img"]).to(dev)
    tgt = torch.from_numpy(g["target"]).to(dev)
    with torch.no_grad():
        out, jv, loss = m(img, 0, 0, tgt, torch.nn.CrossEntropyLoss())
    _assert_close("eval output", out.cpu(), g["eval_output"], 1e-3)
    assert abs(loss.item() - float(g["eval_loss"])) < 1e-4
    assert jv.shape == (1,) and jv.item() == 1.0          # eval: constant (convlstm.py:151)
    # per-pixel decisions bit-identical
    assert np.array_equal(out.argmax(1).cpu().numpy(), g["eval_output"].argmax(1))


@pytest.mark.parametrize("tag", LSTM_TAGS)
def test_convlstm_bptt_grads_and_jv_f32(tag):
    dev = _dev()
    g = load(tag)
    m = _model(g).to(dev).train()
    img = torch.from_numpy(g["img"]).to(dev)
    tgt = torch.from_numpy(g["target"]).to(dev)
    out, jv, loss = m(img, 0, 0, tgt, torch.nn.CrossEntropyLoss())
    loss.backward()
    _assert_close("train output", out.detach().cpu(), g["output"], 1e-3)
    assert abs(loss.item() - float(g["loss"])) < 1e-4
    _assert_close("jv_penalty", jv.cpu(), g["jv_penalty"], 1e-4, 1e-3)
    ref = {k[len("grad."):]: v for k, v in g.items() if k.startswith("grad.")}
    got = {k: p.grad for k, p in m.named_parameters() if p.grad is not None}
    assert set(got) == set(ref), set(got) ^ set(ref)
    for k, v in ref.items():
        _assert_close(f"grad {k}", got[k].cpu(), v, 1e-6, 1e-3)


@pytest.mark.parametrize("tag", ["convlstm_jvp", "convlstm_jvp_t2", "convlstm_rbp_jvp"])
def test_convlstm_jacobian_penalty_with_graph_f32(tag):
    """jacobian_penalty=True: the penalty carries its graph (convlstm.py:158-162)
    and the loss is loss + 10 mean(jv_penalty) (mainclean.py:191-195); the
    reference's gradients of that sum within 1e-3 (golden from the reference
    with the flag set).  convlstm_rbp_jvp: the same with grad_method='rbp'
    (create_graph applies to both methods; the Neumann-series backward of
    dummyhgru, 5 terms)."""
    from models import convlstm as cl
    dev = _dev()
    g = load(tag)
    rbp = "cfg_rbp" in g and int(g["cfg_rbp"]) == 1
    m = cl.ConvLSTM(timesteps=int(g["cfg_timesteps"]), filt_size=int(g["cfg_filt"]),
                    jacobian_penalty=True, grad_method="rbp" if rbp else "bptt",
                    num_iter=int(g["cfg_num_iter"]) if rbp else 50)
    m.load_state_dict(params(g), strict=True)
    m = m.to(dev).train()
    img = torch.from_numpy(g["img"]).to(dev)
    tgt = torch.from_numpy(g["target"]).to(dev)
    out, jv, loss = m(img, 0, 0, tgt, torch.nn.CrossEntropyLoss())
    assert jv.requires_grad
    (loss + jv.mean() * 1e1).backward()
    _assert_close("train output", out.detach().cpu(), g["output"], 1e-3)
    assert abs(loss.item() - float(g["loss"])) < 1e-4
    _assert_close("jv_penalty", jv.detach().cpu(), g["jv_penalty"], 1e-4, 1e-3)
    ref = {k[len("grad."):]: v for k, v in g.items() if k.startswith("grad.")}
    got = {k: p.grad for k, p in m.named_parameters() if p.grad is not None}
    assert set(got) == set(ref), set(got) ^ set(ref)
    for k, v in ref.items():
        _assert_close(f"grad {k}", got[k].cpu(), v, 1e-6, 1e-3)


def test_convlstm_jacobian_penalty_bf16_vs_f32():
    """jacobian_penalty=True with the bf16 cell: the library's first T-2 steps
    store bf16 states, which feed the last two steps' f32 torch ops and their
    double backward.  Against the f32 run (itself pinned to the reference
    golden above): the penalty within 5 % relative RMS, the output within 1 %,
    gradient cosine > 0.999 per tensor (r06: the static x-conv in three bf16
    passes, see test_convlstm_bf16_tolerance; r05 measured 0.966 with the
    single-pass bf16 x-conv and asserted 0.95); measured values recorded
    (gpurun_out/parity_records.json)."""
    from goldens import record
    from models import convlstm as cl
    dev = _dev()
    g = load("convlstm_jvp")
    img = torch.from_numpy(g["img"]).to(dev)
    tgt = torch.from_numpy(g["target"]).to(dev)
    res = {}
    for dt in ("f32", "bf16"):
        m = cl.ConvLSTM(timesteps=int(g["cfg_timesteps"]), filt_size=int(g["cfg_filt"]),
                        jacobian_penalty=True)
        m.load_state_dict(params(g), strict=True)
        m = m.to(dev).train()
        m.cell_dtype = dt
        out, jv, loss = m(img, 0, 0, tgt, torch.nn.CrossEntropyLoss())
        assert jv.requires_grad
        (loss + jv.mean() * 1e1).backward()
        res[dt] = (out.detach().double().cpu(), jv.detach().double().cpu(),
                   {k: p.grad.detach().double().flatten().cpu() for k, p in m.named_parameters()
                    if p.grad is not None})
    (o32, j32, g32), (o16, j16, g16) = res["f32"], res["bf16"]
    rel = lambda a, b: float((a - b).norm() / b.norm().clamp_min(1e-30))
    worst = 1.0
    for k in g32:
        if g32[k].norm() > 0:
            cos = float(g16[k] @ g32[k] / (g16[k].norm() * g32[k].norm()))
            worst = min(worst, cos)
    record("convlstm_jvp_bf16_vs_f32", {"penalty_rel_rms": rel(j16, j32), "output_rel_rms": rel(o16, o32),
                                        "min_grad_cos": worst})
    for k in g32:
        if g32[k].norm() > 0:
            cos = float(g16[k] @ g32[k] / (g16[k].norm() * g32[k].norm()))
            assert cos > 0.999, (k, cos)
    assert rel(j16, j32) < 5e-2, rel(j16, j32)
    assert rel(o16, o32) < 1e-2, rel(o16, o32)


@pytest.mark.parametrize("tag", ["convlstm_k15", "convlstm_k7", "convlstm_t2"])
def test_convlstm_bf16_tolerance(tag):
    """bf16 operands / saved h, f32 gate math and accumulation, k=15 (and r06:
    the k=7 prefetching loops, and the two-step unroll): outputs
    (after the batch-statistics BN, which amplifies h's rounding) within 1 %
    relative RMS of the reference; gradient cosine > 0.999 per tensor.  Until
    r05 the static x-conv (xg = Wx x + b, once per forward) ran with bf16 x and
    Wx: the Gabor-squared input's pre-activations saturate tanh(P_c), where
    1 - g^2 is exponentially sensitive to P_c's error, and the c-gate
    gradients measured cosine 0.96-0.97 (asserted 0.95).  The CPU attribution
    (tools/lstm_bf16_attrib.py, profiles/r06_lstm_bf16_attrib.json) puts all of
    it on that x-conv's forward value -- x and Wx rounding, not h, dP, Wh or the
    weight gradient's X operand -- and predicts 0.99999 once that value is
    near f32; r06 computes it in three bf16 passes (hi x hi + lo x hi + hi x
    lo).  Measured values recorded (gpurun_out/parity_records.json)."""
    dev = _dev()
    g = load(tag)
    m = _model(g, "bf16").to(dev).train()
    img = torch.from_numpy(g["img"]).to(dev)
    tgt = torch.from_numpy(g["target"]).to(dev)
    out, _, loss = m(img, 0, 0, tgt, torch.nn.CrossEntropyLoss())
    loss.backward()
    a = out.detach().cpu().double()
    b = torch.from_numpy(g["output"]).double()
    rel = float((a - b).norm() / b.norm())
    assert rel < 1e-2, f"bf16 output relative RMS error {rel:.3e}"
    cos = {}
    for k, p in m.named_parameters():
        b = torch.from_numpy(g["grad." + k]).double().flatten()
        if b.norm() < 1e-8:
            continue
        a = p.grad.detach().cpu().double().flatten()
        cos[k] = float(a @ b / (a.norm() * b.norm() + 1e-30))
    from goldens import record
    record(f"{tag}_bf16_vs_reference", {"output_rel_rms": rel, "min_grad_cos": min(cos.values()),
                                         "min_grad_cos_tensor": min(cos, key=cos.get)})
    bad = {k: round(v, 6) for k, v in cos.items() if v <= 0.999}
    assert not bad, f"gradient cosine <= 0.999: {bad} (all: {cos})"


def _oracle_cell_step(sd, x, h, c, k):
    pad = k // 2

    def conv(name, v, bias=True):
        return F.conv2d(v, sd[f"W{name}.weight"], sd[f"W{name}.bias"] if bias else None,
                        padding=pad)
    i = torch.sigmoid(conv("xi", x) + conv("hi", h, False))
    f = torch.sigmoid(conv("xf", x) + conv("hf", h, False))
    c2 = f * c + i * torch.tanh(conv("xc", x) + conv("hc", h, False))
    o = torch.sigmoid(conv("xo", x) + conv("ho", h, False))
    return o * torch.tanh(c2), c2


@pytest.mark.parametrize("k,cin,ch", [(15, 25, 25), (5, 7, 19), (1, 32, 32)])
def test_cell_step_with_states(k, cin, ch):
    """ConvLSTMCell.forward(x, h, c) (convlstm.py:84-90) with non-zero states:
    h', c' and the grads of x, h, c and every weight vs the oracle step."""
    from models import convlstm as cl
    dev = _dev()
    torch.manual_seed(k + cin)
    cell = cl.ConvLSTMCell(cin, ch, k)
    x = torch.rand(3, cin, 32, 32)
    h = torch.randn(3, ch, 32, 32) * 0.5
    c = torch.randn(3, ch, 32, 32) * 0.5
    wh = torch.randn(3, ch, 32, 32)
    wc = torch.randn(3, ch, 32, 32)
    sd = {n: p.detach().clone().requires_grad_() for n, p in cell.named_parameters()}
    xr, hr, cr = (t.clone().requires_grad_() for t in (x, h, c))
    h2, c2 = _oracle_cell_step(sd, xr, hr, cr, k)
    ((h2 * wh).sum() + (c2 * wc).sum()).backward()

    cell = cell.to(dev)
    xg, hg, cg = (t.to(dev).requires_grad_() for t in (x, h, c))
    h3, c3 = cell(xg, hg, cg)
    ((h3 * wh.to(dev)).sum() + (c3 * wc.to(dev)).sum()).backward()
    _assert_close("h'", h3.detach().cpu(), h2.detach(), 1e-4)
    _assert_close("c'", c3.detach().cpu(), c2.detach(), 1e-4)
    for name, a, b in (("dx", xg.grad, xr.grad), ("dh", hg.grad, hr.grad), ("dc", cg.grad, cr.grad)):
        _assert_close(name, a.cpu(), b, 1e-5, 1e-3)
    for n, p in cell.named_parameters():
        _assert_close(f"grad {n}", p.grad.cpu(), sd[n].grad, 1e-5, 1e-3)


def test_convlstm_longer_unroll_vs_oracle():
    """A fresh seeded batch beyond the fixtures (B=6, T=8, k=7): outputs, jv and
    every gradient vs the CPU oracle."""
    from oracle import cells
    from models import convlstm as cl
    dev = _dev()
    torch.manual_seed(5)
    m = cl.ConvLSTM(timesteps=8, filt_size=7)
    img = torch.rand(6, 1, 32, 32)
    tgt = torch.randint(0, 2, (6, 32, 32))
    sd = {n: p.detach().clone().requires_grad_() for n, p in m.named_parameters()}
    out_r, _, _, jv_r = cells.convlstm_forward(sd, img, 8, with_jv=True)
    F.cross_entropy(out_r, tgt).backward()
    m = m.to(dev).train()
    out, jv, loss = m(img.to(dev), 0, 0, tgt.to(dev), torch.nn.CrossEntropyLoss())
    loss.backward()
    _assert_close("output", out.detach().cpu(), out_r.detach(), 1e-3)
    _assert_close("jv", jv.cpu(), jv_r, 1e-4, 1e-3)
    for n, p in m.named_parameters():
        _assert_close(f"grad {n}", p.grad.cpu(), sd[n].grad, 1e-6, 1e-3)


def test_convlstm_rbp_runs_on_the_cell():
    """grad_method='rbp' (convlstm.py:124-135) composes the one-step cell and the
    Neumann-series backward; its grads reach every parameter of the last step."""
    from models import convlstm as cl
    dev = _dev()
    torch.manual_seed(3)
    m = cl.ConvLSTM(timesteps=4, filt_size=7, num_iter=5, grad_method="rbp").to(dev).train()
    img = torch.rand(2, 1, 32, 32, device=dev)
    tgt = torch.randint(0, 2, (2, 32, 32), device=dev)
    out, jv, loss = m(img, 0, 0, tgt, torch.nn.CrossEntropyLoss())
    loss.backward()
    assert jv.shape == (2, 25, 32, 32) and torch.isfinite(jv).all()
    assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in m.parameters())
