"""ConvLSTM on PathTracker clips (BASELINE configs[2], models/convlstm.py
ConvLSTMVideo): the library's per-step-input mode (x_seq)
against the CPU restatement oracle/cells.py:convlstm_video_forward (f32,
1e-3), the Jacobian penalty on that same trajectory, and bf16 within the
stated tolerance.  Parity of the video model itself is against this repo's
definition (the reference has no clip ConvLSTM); its cell step is the
reference's and is pinned by the convlstm_* goldens (test_gpu_lstm.py)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda:0")


def _clips(seed, b, t):
    from ptamd import synth
    clips, labels = synth.make_batch(seed, b, t)
    x = torch.from_numpy(clips.transpose(0, 4, 1, 2, 3) / 255.0).float()
    return x, torch.tensor([ord(v) for v in labels], dtype=torch.float32)


def _model(k, seed):
    from models import convlstm
    torch.manual_seed(seed)
    m = convlstm.ConvLSTMVideo(dimensions=25, timesteps=6, kernel_size=k)
    with torch.no_grad():                                  # off the near-constant init
        m.readout_conv.weight.mul_(8.0)
        m.preproc.weight.mul_(2.0)
    return m


@pytest.mark.parametrize("k,b,t", [(7, 3, 6), (15, 2, 4), (3, 4, 2)])
def test_video_convlstm_matches_oracle(k, b, t):
    from oracle import cells
    dev = _dev()
    m = _model(k, 30 + k)
    x, y = _clips(40 + k, b, t)
    sd = {n: p.detach().clone().requires_grad_() for n, p in m.named_parameters()}
    lo, _, hs, cs = cells.convlstm_video_forward(sd, x)
    jr = cells.convlstm_jv_penalty(hs, cs) if t >= 2 else None
    F.binary_cross_entropy_with_logits(lo, y.reshape(-1, 1)).backward()
    m = m.to(dev).train()
    out, jv = m(x.to(dev))
    F.binary_cross_entropy_with_logits(out, y.to(dev).reshape(-1, 1)).backward()
    assert float((out.detach().cpu() - lo.detach()).abs().max()) < 1e-3
    for n, p in m.named_parameters():
        r = sd[n].grad
        err = float((p.grad.cpu() - r).abs().max())
        assert err <= 1e-6 + 1e-3 * float(r.abs().max()), (n, err)
    # the reference ConvLSTM's Jacobian penalty of the last step, on this trajectory
    if t >= 2:
        assert jv.shape == jr.shape
        err = float((jv.cpu() - jr).abs().max())
        assert err <= 1e-3 * (1.0 + float(jr.abs().max())), err


@pytest.mark.parametrize("k", [7, 5, 3, 15])
def test_video_convlstm_bf16_tolerance(k):
    """The bf16 library against the f32 one on the same clips (r06: every
    kernel-size path -- the k <= 7 prefetching loops at 7 / 5 / 3, the plain
    loop at 15): logits within 2e-2, gradient cosine > 0.99 per tensor."""
    dev = _dev()
    m = _model(k, 5).to(dev).train()
    x, y = _clips(9, 16, 8)
    x, y = x.to(dev), y.to(dev).reshape(-1, 1)
    res = {}
    for dt in ("f32", "bf16"):
        m.cell_dtype = dt
        m.zero_grad(set_to_none=True)
        out, _ = m(x)
        F.binary_cross_entropy_with_logits(out, y).backward()
        res[dt] = (out.detach().double(), {n: p.grad.detach().double().flatten()
                                           for n, p in m.named_parameters()})
    (o32, g32), (o16, g16) = res["f32"], res["bf16"]
    assert float((o16 - o32).abs().max()) < 2e-2
    for n in g32:
        if g32[n].norm() > 1e-12:
            cos = float(g16[n] @ g32[n] / (g16[n].norm() * g32[n].norm()))
            assert cos > 0.99, (n, cos)


@pytest.mark.parametrize("switch", ["PT_LCONV_FAST", "PT_LWGRAD2", "PT_LCONVT8", "PT_LPW_FUSE"])
def test_lconv_prefetch_loop_is_bitwise_the_plain_loop(switch):
    """r04 bf16 k <= 7 kernels against the forms they replace, switched off per
    call: k_lconv's prefetching column loop (PT_LCONV_FAST=0: the plain loop)
    the column-owned weight gradients k_lwgrad2 (PT_LWGRAD2=1) and the
    8-wave transposed conv (PT_LCONVT8=1), and (r05) the per-step point-wise
    update in the two-source conv's epilogue against its own launch
    (PT_LPW_FUSE=0), each against the default.
    Same MFMA order per accumulator, so logits, the Jacobian penalty and every
    gradient are bitwise equal (k=7, 5 and 3)."""
    from variants import variants
    dev = _dev()
    for k in (7, 5, 3):
        m = _model(k, 11 + k).to(dev).train()
        m.cell_dtype = "bf16"
        x, y = _clips(13 + k, 6, 5)
        x, y = x.to(dev), y.to(dev).reshape(-1, 1)
        res = []
        for v in ("0", "1"):
            with variants(**{switch: v}):          # the diagnostic library reads the switch
                m.zero_grad(set_to_none=True)
                out, jv = m(x)
                F.binary_cross_entropy_with_logits(out, y).backward()
                torch.cuda.synchronize()
                res.append((out.detach().clone(), jv.detach().clone(),
                            {n: p.grad.detach().clone() for n, p in m.named_parameters()}))
        (o0, j0, g0), (o1, j1, g1) = res
        assert torch.equal(o0, o1) and torch.equal(j0, j1), k
        for n in g0:
            assert torch.equal(g0[n], g1[n]), (k, n)


def test_registry_builds_it():
    import types
    from utils import engine
    m = engine.model_selector(types.SimpleNamespace(model="convlstm"), timesteps=8, device="cpu")
    assert type(m).__name__ == "ConvLSTMVideo" and m.kernel_size == 7


@pytest.mark.parametrize("cin,cout,b,t", [(3, 25, 3, 6), (1, 32, 2, 4), (4, 7, 5, 2)])
def test_stem_matches_torch(cin, cout, b, t):
    """pt_lstm_stem_* (softplus of a 1x1x1 Conv3d) against torch in f32,
    including pre-activations past softplus's threshold (20) where it is linear."""
    from ptamd import lstm
    dev = _dev()
    g = torch.Generator().manual_seed(cin * 100 + cout)
    x = torch.rand((b, cin, t, 32, 32), generator=g).to(dev)
    w = (torch.randn((cout, cin, 1, 1, 1), generator=g) * 4).to(dev).requires_grad_()
    bias = torch.randn((cout,), generator=g) * 8
    bias[0] = 21.0                                          # straddles the threshold
    bias = bias.to(dev).requires_grad_()
    dy = torch.randn((b, cout, t, 32, 32), generator=g).to(dev)
    y = lstm.stem(x, w, bias)
    (y * dy).sum().backward()
    w2, b2 = w.detach().clone().requires_grad_(), bias.detach().clone().requires_grad_()
    yr = F.softplus(F.conv3d(x.double(), w2.double(), b2.double()))
    (yr * dy.double()).sum().backward()
    assert (yr.detach() > 20).any()
    torch.testing.assert_close(y.double(), yr.detach(), rtol=1e-5, atol=1e-5)
    for a, r in ((w.grad, w2.grad), (bias.grad, b2.grad)):
        assert float((a.double() - r).abs().max()) <= 1e-4 * float(r.abs().max()) + 1e-6


def test_u8_clips_match_f32_input():
    """Raw u8 clips [B,T,H,W,3] through the stem kernel give the same model
    outputs, bit for bit, as engine.prepare_data's f32 input, and the same
    gradients (to 1e-5: MIOpen's readout weight gradient is not bitwise
    reproducible between two identical calls)."""
    from ptamd import synth
    from ptamd.cell import unit_values
    dev = _dev()
    clips, labels = synth.make_batch(77, 3, 6)
    xu8 = torch.from_numpy(clips).to(dev)                       # [B,T,H,W,3]
    x32 = unit_values(xu8).permute(0, 4, 1, 2, 3).contiguous()  # [B,3,T,H,W]
    y = torch.tensor([ord(v) for v in labels], dtype=torch.float32, device=dev).reshape(-1, 1)
    m = _model(7, 11).to(dev).train()
    res = []
    for x in (x32, xu8):
        m.zero_grad(set_to_none=True)
        out, jv = m(x)
        F.binary_cross_entropy_with_logits(out, y).backward()
        res.append((out.detach().clone(), jv.clone(),
                    {n: p.grad.detach().clone() for n, p in m.named_parameters()}))
    (o1, j1, g1), (o2, j2, g2) = res
    assert torch.equal(o1, o2) and torch.equal(j1, j2)
    for n in g1:
        torch.testing.assert_close(g2[n], g1[n], rtol=1e-5, atol=1e-8, msg=n)


def test_bf16_matches_f32_at_cfg3_size():
    """The clip ConvLSTM at its bench size (B=256, T=64, k=7): the bf16 cell
    against the f32 cell (itself pinned to the oracle above) on the bench's
    clips — logits within 1e-3 (north_star's bound; measured 3.4e-4), identical
    0.5 / 0 decisions for every clip (in-band ones included), per-tensor
    gradient cosine >= 0.99."""
    from models import convlstm
    dev = _dev()
    x, y = _clips(1000, 256, 64)
    x, y = x.to(dev), y.to(dev).reshape(-1, 1)
    torch.manual_seed(1234)
    m = convlstm.ConvLSTMVideo(dimensions=25, timesteps=64, kernel_size=7).to(dev).train()
    with torch.no_grad():                                   # off the near-constant init
        m.readout_conv.weight.mul_(8.0)
    res = {}
    for dt in ("f32", "bf16"):
        m.cell_dtype = dt
        m.zero_grad(set_to_none=True)
        out, _ = m(x)
        F.binary_cross_entropy_with_logits(out, y).backward()
        torch.cuda.synchronize()
        res[dt] = (out.detach().double().flatten().cpu(),
                   {n: p.grad.detach().double().flatten().cpu() for n, p in m.named_parameters()})
    (o32, g32), (o16, g16) = res["f32"], res["bf16"]
    tol = 1e-3
    err = float((o16 - o32).abs().max())
    cos = {n: float(g16[n] @ g32[n] / (g16[n].norm() * g32[n].norm()))
           for n in g32 if g32[n].norm() > 1e-12}
    flips = {}
    for name, thr in (("train_0.5", 0.5), ("eval_0", 0.0)):
        flips[name] = int(((o16 > thr) != (o32 > thr)).sum())
    rec = {"logit_max_abs_err": err, "logit_spread": float(o32.max() - o32.min()),
           "grad_cosine_min": min(cos.values()), "grad_cosine_min_tensor": min(cos, key=cos.get),
           "flips_all_clips": flips}
    from goldens import record
    record("convlstm_video_bf16_vs_f32_B256_T64", rec)
    assert err <= tol, rec
    assert flips == {"train_0.5": 0, "eval_0": 0}, rec
    bad = {n: v for n, v in cos.items() if v < 0.99}
    assert not bad, (bad, rec)


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_testmode_per_frame_outputs(dtype):
    """testmode returns InT's triple (InT.py:230-233,244): logits, per-frame
    states = readout_conv(h_t) [B,T,1,H,W] and the per-frame hidden states
    h_t [B,T,C,H,W] (what the reference ConvLSTM's testmode collects,
    convlstm.py:127-135), each frame against the oracle's trajectory (f32:
    1e-3; bf16: the stated bf16 tolerance, 2e-2 absolute on states/logits)."""
    from oracle import cells
    dev = _dev()
    m = _model(7, 21)
    x, _ = _clips(22, 3, 6)
    sd = {n: p.detach().clone() for n, p in m.named_parameters()}
    with torch.no_grad():
        lo, _, hs, _ = cells.convlstm_video_forward(sd, x)
        ref_h = torch.stack(hs, 1)                                   # [B,T,C,H,W]
        ref_states = torch.stack([F.conv2d(h, sd["readout_conv.weight"], sd["readout_conv.bias"])
                                  for h in hs], 1)
    m = m.to(dev).eval()
    m.cell_dtype = dtype
    with torch.no_grad():
        out, states, hidden = m(x.to(dev), testmode=True)
        out2, _ = m(x.to(dev))
    assert states.shape == (3, 6, 1, 32, 32) and hidden.shape == (3, 6, 25, 32, 32)
    tol = 1e-3 if dtype == "f32" else 2e-2
    assert float((out.cpu() - lo).abs().max()) < tol
    assert torch.equal(out, out2)                       # testmode does not change the logits
    for t in range(6):
        assert float((hidden[:, t].cpu() - ref_h[:, t]).abs().max()) < tol, t
        assert float((states[:, t].cpu() - ref_states[:, t]).abs().max()) < tol, t
    # engine.model_step(test=True) path (utils/engine.py:64-72)
    from utils import engine
    res = engine.model_step(m, x.to(dev), "convlstm", test=True)
    assert len(res) == 3 and torch.equal(res[0], out)


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("u8", [False, True])
def test_fused_stem_equals_stem_then_steps(dtype, u8):
    """pt_lstm_forward_stem / pt_lstm_backward_stem (r05: the stem written
    straight into the recurrence's per-step input, its dW / db straight from
    d x_t) against the separate pt_lstm_stem_* + pt_lstm_forward / backward
    the model used before: the per-step input is the same values rounded the
    same way, so logits, the Jacobian penalty and every cell gradient are
    bitwise equal; the stem's weight / bias gradients are the same per-voxel
    terms summed in another block order (1e-6 relative)."""
    from ptamd import lstm
    from ptamd import readout as ro
    from ptamd.cell import target_channel
    dev = _dev()
    m = _model(7, 61).to(dev).train()
    m.cell_dtype = dtype
    x, y = _clips(62, 3, 6)
    x = x.to(dev)
    if u8:                                     # the raw clip bytes [B,T,H,W,3]
        x = (x * 255.0).round().to(torch.uint8).permute(0, 2, 3, 4, 1).contiguous()
    y = y.to(dev).reshape(-1, 1)

    def run(fused):
        m.zero_grad(set_to_none=True)
        if fused:
            out, jv = m(x)
        else:                                  # the r04 composition of the same model
            xbn = lstm.stem(x, m.preproc.weight, m.preproc.bias)
            h_t, _, jv = m.unit1.steps(xbn, xbn.shape[2], want_jv=True)
            out = ro.readout(h_t, target_channel(x), m.readout_conv, m.target_conv, m.readout_dense)
        F.binary_cross_entropy_with_logits(out, y).backward()
        torch.cuda.synchronize()
        return out.detach().clone(), jv.detach().clone(), {n: p.grad.detach().clone()
                                                           for n, p in m.named_parameters()}

    o0, j0, g0 = run(False)
    o1, j1, g1 = run(True)
    assert torch.equal(o0, o1) and torch.equal(j0, j1)
    for n in g0:
        if n.startswith("preproc."):
            err = float((g1[n] - g0[n]).abs().max())
            assert err <= 1e-6 * float(g0[n].abs().max()) + 1e-12, (n, err)
        else:
            assert torch.equal(g0[n], g1[n]), n
