"""Comparison baselines of BASELINE.json configs[4]:
the kys ConvGRU ('gru') and the stride-free R3D ('nostride_video_cc_small'),
stock-PyTorch modules, against golden vectors produced by the reference's own
modules (tests/golden/make_golden.py): init under the same seed (exact),
outputs, loss, every gradient and one Adam step (fp32 CPU, 1e-5 relative)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from goldens import load, prepared_input


def _close(name, a, b, rtol=1e-5, atol=1e-6):
    a = np.asarray(a.detach().cpu() if torch.is_tensor(a) else a, np.float64)
    b = np.asarray(b, np.float64)
    assert a.shape == b.shape, (name, a.shape, b.shape)
    err = np.abs(a - b).max()
    assert err <= atol + rtol * np.abs(b).max(), f"{name}: {err:.3e}"


def _state(g, prefix):
    return {k[len(prefix):]: torch.from_numpy(v.copy()) for k, v in g.items() if k.startswith(prefix)}


def _check_init(model, g):
    init = _state(g, "init.")
    sd = model.state_dict()
    assert list(sd) == list(init)
    for k, v in sd.items():
        assert torch.equal(v, init[k]), k


def _train_and_check(model, g, x, y, dev="cpu", tol=1e-5):
    model.train()
    logits, _ = model(x.to(dev))
    loss = F.binary_cross_entropy_with_logits(logits, y.to(dev).reshape(-1, 1))
    loss.backward()
    _close("train logits", logits, g["train_logits"], tol)
    assert abs(loss.item() - float(g["loss"])) < 10 * tol
    for k, p in model.named_parameters():
        if "grad." + k not in g:          # registered but unused (kys.GRU.bn): no grad there either
            assert p.grad is None, k
            continue
        _close("grad " + k, p.grad, g["grad." + k], 10 * tol, 1e-7)
    opt = torch.optim.Adam(model.parameters(), lr=3e-4)
    opt.step()
    for k, p in model.named_parameters():
        _close("adam " + k, p, g["adam." + k], 10 * tol, 1e-7)


def test_gru_matches_reference():
    from models import kys
    g = load("gru_c16")
    torch.manual_seed(int(g["cfg_seed"]))
    m = kys.GRU(dimensions=int(g["cfg_dims"]), timesteps=4, kernel_size=7)
    _check_init(m, g)
    m.load_state_dict(_state(g, "param."))
    x, y = prepared_input(g)
    m.eval()
    with torch.no_grad():
        logits, states, gates = m(x, testmode=True)
    _close("logits", logits, g["logits"])
    _close("states", states, g["states"])
    _close("gates", gates, g["gates"])
    _train_and_check(m, g, x, y)


def test_r3d_small_matches_reference():
    from models import nostridetv_cc_smallest as r3d
    g = load("r3d_small")
    torch.manual_seed(int(g["cfg_seed"]))
    m = r3d.r3d_18(timesteps=4)
    _check_init(m, g)
    x, y = prepared_input(g)
    m.eval()
    with torch.no_grad():
        _close("eval logits", m(x)[0], g["logits"])
    _train_and_check(m, g, x, y)
    for k, v in m.state_dict().items():
        if "running" in k:
            _close("running " + k, v, g["after." + k])


def test_registry_builds_baselines():
    from types import SimpleNamespace
    from utils import engine
    gru = engine.model_selector(SimpleNamespace(model="gru"), timesteps=8, device="cpu")
    assert gru.hgru_size == 64 and gru.unit1.conv_reset.kernel_size == (7, 7)   # 2 x dims, k=7
    r3d = engine.model_selector(SimpleNamespace(model="nostride_video_cc_small", pretrained=False),
                                timesteps=8, device="cpu")
    assert sum(p.numel() for p in r3d.parameters()) > 0
    with pytest.raises(NotImplementedError):
        engine.model_selector(SimpleNamespace(model="nostride_video_cc_small", pretrained=True),
                              timesteps=8, device="cpu")
