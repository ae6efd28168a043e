"""The fused forward (k_fused_fa / k_fused_fb: the point-wise step of a clip's
32 rows and the k x k conv in ONE launch per BatchNorm segment, bf16, 32 x 32
frames) against the split kernels (k_pw_fa, k_conv_fwd, k_pw_fb, k_conv_fwd):
the arithmetic is the same operation for operation (the LDS tile holds the
bf16 values the split conv would load), so logits, per-frame testmode outputs
and every gradient must agree bit for bit.  PT_CELL_FUSED=0 selects the split
path (read per call by the diagnostic library: tests/variants.py).

The persistent forward (k_persist_fwd, PT_CELL_PERSIST=1: all T frames of the
fused segments in one launch, the BatchNorm syncs as in-launch waits on the
deterministic group sums) is the same arithmetic in the same reduction order,
so it too must reproduce the per-segment launches bit for bit.  So must the
banded backward convs (PT_CONV_BAND=1, and the staggered two-band workgroup,
PT_CONV_BAND=3): per output row the same MFMA order.  r06: the fused
backward A (k_conv_pw_ba, the default; PT_CPA=0 selects the split pair) and
the two-band conv on tiled frames (PT_BAND2_TILED) likewise.  The baseline
of every comparison is the library's defaults with the whole-clip backward
conv (PT_CONV_BAND=0)."""
import pytest
import torch
import torch.nn.functional as F
from variants import variants

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda:0")


def _run(m, x, y, fused, persist=False, band=False, cpa=1, band2_tiled=1, fused_tiled=0):
    with variants(PT_CELL_FUSED=int(fused), PT_CELL_PERSIST=int(persist), PT_CONV_BAND=int(band),
                  PT_CPA=int(cpa), PT_BAND2_TILED=int(band2_tiled), PT_FUSED_TILED=int(fused_tiled)):
        m.zero_grad(set_to_none=True)
        out, _ = m(x)
        F.binary_cross_entropy_with_logits(out, y.reshape(-1, 1)).backward()
        with torch.no_grad():
            lo, states, gates = m(x, testmode=True)
        torch.cuda.synchronize()
        return (out.detach().clone(), states.clone(), gates.clone(),
                {k: p.grad.detach().clone() for k, p in m.named_parameters() if p.grad is not None})


@pytest.mark.parametrize("cell,act,b,t", [("int", "softplus", 24, 8), ("int", "tanh", 5, 3),
                                          ("hgru", "softplus", 16, 6), ("int", "softplus", 256, 64)])
def test_fused_forward_is_bitwise_the_split_forward(cell, act, b, t):
    _compare(cell, act, b, t, dict(fused=False))


@pytest.mark.parametrize("cell,act,b,t", [("int", "softplus", 24, 8), ("int", "tanh", 5, 3),
                                          ("hgru", "softplus", 16, 6), ("int", "softplus", 256, 64)])
def test_persistent_forward_is_bitwise_the_fused_forward(cell, act, b, t):
    _compare(cell, act, b, t, dict(fused=True, persist=True))


@pytest.mark.parametrize("cell,act,b,t", [("int", "softplus", 24, 8), ("hgru", "softplus", 16, 6),
                                          ("int", "softplus", 256, 64)])
def test_banded_backward_conv_is_bitwise_the_whole_clip_conv(cell, act, b, t):
    """k_conv_bwd_band (PT_CONV_BAND=1: two 16-row workgroups per clip, B
    fragments in registers) against k_conv_bwd (one workgroup per clip)."""
    _compare(cell, act, b, t, dict(fused=True, band=True))


@pytest.mark.parametrize("cell,act,b,t", [("int", "softplus", 24, 8), ("hgru", "softplus", 16, 6),
                                          ("int", "softplus", 256, 64)])
def test_staggered_two_band_conv_is_bitwise_the_whole_clip_conv(cell, act, b, t):
    """k_conv_bwd_band2 (PT_CONV_BAND=3, r05: both bands of a clip in one
    8-wave workgroup, band 1 filled under band 0's MFMAs, an LDS counter
    instead of a workgroup barrier for band 1's waves) against k_conv_bwd."""
    _compare(cell, act, b, t, dict(fused=True, band=3))


@pytest.mark.parametrize("cell,act,b,t", [("int", "softplus", 24, 8), ("int", "tanh", 5, 3),
                                          ("hgru", "softplus", 16, 6), ("int", "softplus", 256, 64)])
def test_fused_backward_a_is_bitwise_the_split_pair(cell, act, b, t):
    """k_conv_pw_ba (the r06 default: k_conv_ba(t)'s band p and k_pw_ba(t-1)'s
    rows of that band in one workgroup, one launch per frame) against the
    split k_conv_bwd_band2 + k_pw_ba (PT_CPA=0): the same arithmetic and
    reduction slots."""
    _compare(cell, act, b, t, dict(fused=True, cpa=0))


@pytest.mark.parametrize("hw,b,t,cpa", [(64, 4, 6, 0), (64, 4, 6, 1), (96, 2, 4, 1)])
def test_staggered_two_band_conv_on_tiled_frames_is_bitwise_the_whole_clip_conv(hw, b, t, cpa):
    """k_conv_bwd_band2 on frames of several 32x32 tiles (PT_BAND2_TILED=1,
    r06: the band tile's border from the neighbouring tiles, band_halo), and
    with cpa the fused backward A on them too, against the whole-clip convs
    with tile_halo and the split k_pw_ba (hGRU, cfg4's 64x64 and a 3x3-tile
    96x96 frame whose middle tile has neighbours on every side)."""
    from models import ffhgru_hierarchy as hg
    dev = _dev()
    torch.manual_seed(hw + b)
    m = hg.FFhGRU(dimensions=32, timesteps=t, kernel_size=7)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if (n.startswith("unit1.bn") and n.endswith("weight")) or n.endswith(("alpha", "kappa")):
                p.uniform_(0.5, 1.5)
            elif n.endswith(("mu", "gamma")):
                p.uniform_(-0.5, 0.5)
    m = m.to(dev)
    m.cell_dtype = "bf16"
    x = torch.rand(b, 3, t, hw, hw, device=dev)
    y = (torch.arange(b, device=dev) % 2).float()
    o1, s1, g1, gr1 = _run(m, x, y, fused=True, band=0, band2_tiled=0, cpa=0)
    o0, s0, g0, gr0 = _run(m, x, y, fused=True, band=3, band2_tiled=1, cpa=cpa)
    assert torch.isfinite(o1).all()
    assert torch.equal(o1, o0), (o1 - o0).abs().max().item()
    bad = {k: ((gr1[k] - gr0[k]).abs().max() / gr0[k].abs().max().clamp_min(1e-30)).item()
           for k in gr0 if k.startswith(("unit1.", "preproc.")) and not torch.equal(gr1[k], gr0[k])}
    assert not bad, bad


@pytest.mark.parametrize("cell,h,w,b,t", [("hgru", 64, 64, 4, 6), ("hgru", 96, 96, 2, 4), ("int", 64, 96, 3, 5),
                                          ("hgru", 64, 64, 128, 8)])
def test_fused_forward_on_tiled_frames_is_bitwise_the_split_forward(cell, h, w, b, t):
    """k_fused_fa / k_fused_fb on frames of several 32x32 tiles (r06, opt-in
    PT_FUSED_TILED=1: each tile workgroup publishes its conv input's border
    and takes its halo from the neighbouring tiles' workgroups of the same
    launch, xb_exchange) against the split forward (k_pw_fa, k_conv_fwd with
    tile_halo, ...): logits, per-frame states and gates, every gradient; the
    3x3-tile frame's middle tile has all 8 neighbours, and (128, 64x64) is
    cfg4's launch of 512 tile workgroups."""
    from models import InT, ffhgru_hierarchy as hg
    dev = _dev()
    torch.manual_seed(h + w + b)
    m = (hg.FFhGRU(dimensions=32, timesteps=t, kernel_size=7) if cell == "hgru"
         else InT.InT(dimensions=32, timesteps=t, kernel_size=7))
    with torch.no_grad():
        for n, p in m.named_parameters():
            if (n.startswith("unit1.bn") and n.endswith("weight")) or n.endswith(("alpha", "kappa")):
                p.uniform_(0.5, 1.5)
            elif n.endswith(("mu", "gamma")):
                p.uniform_(-0.5, 0.5)
    m = m.to(dev)
    m.cell_dtype = "bf16"
    x = torch.rand(b, 3, t, h, w, device=dev)
    y = (torch.arange(b, device=dev) % 2).float()
    o1, s1, g1, gr1 = _run(m, x, y, fused=True, fused_tiled=1)
    o0, s0, g0, gr0 = _run(m, x, y, fused=True, fused_tiled=0)
    assert torch.isfinite(o1).all() and torch.isfinite(s1).all()
    for name, u, v in (("logits", o1, o0), ("states", s1, s0), ("gates", g1, g0)):
        assert torch.equal(u, v), (name, (u - v).abs().max().item(), (u != v).sum().item())
    bad = {k: ((gr1[k] - gr0[k]).abs().max() / gr0[k].abs().max().clamp_min(1e-30)).item()
           for k in gr0 if k.startswith(("unit1.", "preproc.")) and not torch.equal(gr1[k], gr0[k])}
    assert not bad, bad


@pytest.mark.parametrize("cell,k,hw", [("int", 5, 32), ("int", 3, 32), ("int", 1, 32), ("hgru", 5, 32),
                                        ("hgru", 5, 64)])
def test_banded_backward_convs_at_small_kernels_are_bitwise_the_whole_clip_conv(cell, k, hw):
    """k < 7 through the banded backward convs (k_conv_bwd_band2 and the fused
    backward A, whose addends are pre-loaded PT_BAND_LEAD tile-row steps
    ahead in the last kernel column: r06 fix -- for k < lead + 2 the first
    rows' pre-loads fell before the column's first step and were never
    issued) against the whole-clip k_conv_bwd (no pre-load) with the split
    k_pw_ba; and the fused forward against the split one at the same k (64 x
    64: the tiled frames' halos at k = 5)."""
    from models import InT, ffhgru_hierarchy as hg
    dev = _dev()
    torch.manual_seed(k + 11)
    m = (hg.FFhGRU(dimensions=32, timesteps=6, kernel_size=k) if cell == "hgru"
         else InT.InT(dimensions=32, timesteps=6, kernel_size=k))
    with torch.no_grad():
        for n, p in m.named_parameters():
            if (n.startswith("unit1.bn") and n.endswith("weight")) or n.endswith(("alpha", "kappa")):
                p.uniform_(0.5, 1.5)
            elif n.endswith(("mu", "gamma")):
                p.uniform_(-0.5, 0.5)
    m = m.to(dev)
    m.cell_dtype = "bf16"
    x = torch.rand(24 if hw == 32 else 4, 3, 6, hw, hw, device=dev)
    y = (torch.arange(x.shape[0], device=dev) % 2).float()
    o1, s1, g1, gr1 = _run(m, x, y, fused=True)                      # band2 + k_conv_pw_ba
    assert torch.isfinite(o1).all()
    for other in (dict(fused=True, band=0, cpa=0),                   # k_conv_bwd + k_pw_ba
                  dict(fused=False, band=0, cpa=0)):                 # and the split forward
        o0, s0, g0, gr0 = _run(m, x, y, **other)
        for name, u, v in (("logits", o1, o0), ("states", s1, s0), ("gates", g1, g0)):
            assert torch.equal(u, v), (other, name, (u - v).abs().max().item())
        bad = {k2: ((gr1[k2] - gr0[k2]).abs().max() / gr0[k2].abs().max().clamp_min(1e-30)).item()
               for k2 in gr0 if k2.startswith(("unit1.", "preproc.")) and not torch.equal(gr1[k2], gr0[k2])}
        assert not bad, (other, bad)


def _compare(cell, act, b, t, other):
    from models import InT, ffhgru_hierarchy as hg
    from ptamd import synth
    dev = _dev()
    torch.manual_seed(b + t)
    if cell == "hgru":
        m = hg.FFhGRU(dimensions=32, timesteps=t, kernel_size=7)
    else:
        m = InT.InT(dimensions=32, timesteps=t, kernel_size=7,
                    nl=torch.tanh if act == "tanh" else F.softplus)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if (n.startswith("unit1.bn") and n.endswith("weight")) or n.endswith(("alpha", "kappa")):
                p.uniform_(0.5, 1.5)
            elif n.endswith(("mu", "gamma")):
                p.uniform_(-0.5, 0.5)
    m = m.to(dev)
    m.cell_dtype = "bf16"
    clips, labels = synth.make_batch(b * 7 + t, b, t)
    x = torch.from_numpy(clips.transpose(0, 4, 1, 2, 3) / 255.0).float().to(dev)
    y = torch.tensor([ord(v) for v in labels], dtype=torch.float32, device=dev)
    o1, s1, g1, gr1 = _run(m, x, y, fused=True)        # the library defaults
    o0, s0, g0, gr0 = _run(m, x, y, **other)
    assert torch.isfinite(o1).all()
    for name, u, v in (("logits", o1, o0), ("states", s1, s0), ("gates", g1, g0)):
        assert torch.equal(u, v), (name, (u - v).abs().max().item(), (u != v).sum().item())
    bad = {}
    for k in gr0:
        if k.startswith(("unit1.", "preproc.")):      # the library's gradients: bitwise
            if not torch.equal(gr1[k], gr0[k]):
                bad[k] = ((gr1[k] - gr0[k]).abs().max() / gr0[k].abs().max().clamp_min(1e-30)).item()
        else:                                          # readout (MIOpen): same inputs
            torch.testing.assert_close(gr1[k], gr0[k], rtol=1e-5, atol=1e-8)
    assert not bad, bad
