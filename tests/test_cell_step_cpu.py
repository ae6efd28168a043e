"""Per-step cell API (``rCell.forward`` / ``hConvGRUCell.forward``, reference
models/InT.py:145-179, models/ffhgru_hierarchy.py:135-173) against the
reference's golden vectors: stepping the drop-in cell frame by frame from
I = E = 0 (InT.py:217-235) reproduces the reference's logits, per-frame states
and gates, and its BPTT gradients.  These run on the CPU; the fused HIP path
(``InT.forward``) is pinned by the GPU parity tests."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from goldens import cfg, load, params, prepared_input


def _model(g):
    from models import InT as int_mod
    from models import ffhgru_hierarchy as hg
    c = cfg(g)
    if c["cell"] == "hgru":
        m = hg.FFhGRU(dimensions=c["dims"], timesteps=8, kernel_size=c["k"])
    else:
        kw = dict(dimensions=c["dims"], timesteps=8, kernel_size=c["k"], no_inh=c["no_inh"],
                  nl=F.tanh if c["act"] == "tanh" else F.softplus)
        for les in c["lesion"]:
            kw["lesion_" + les] = True
        m = int_mod.InT(**kw)
    m.load_state_dict(params(g), strict=True)
    return m


def _step_forward(m, x):
    """The reference's frame loop around the per-step cell (InT.py:210-245)."""
    xbn = m.nl(m.preproc(x))
    b, c, t_len, h, w = xbn.shape
    inh = torch.zeros((b, c, h, w))
    exc = torch.zeros((b, c, h, w))
    states, gates = [], []
    for t in range(t_len):
        inh, exc, att = m.unit1(xbn[:, :, t], inh, exc, activ=m.nl, testmode=True)
        states.append(m.readout_conv(exc))
        gates.append(att)
    return m.readout(exc, x), torch.stack(states, 1), torch.stack(gates, 1)


def _close(name, a, b, rtol=2e-5, atol=2e-6):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    assert a.shape == b.shape, (name, a.shape, b.shape)
    err = np.abs(a - b).max()
    tol = atol + rtol * np.abs(b).max()
    assert err <= tol, f"{name}: max err {err:.3e} > {tol:.3e}"


@pytest.mark.parametrize("tag", ["int_c32", "int_tanh", "int_noinh", "int_lesion", "hgru_c32"])
def test_step_api_matches_reference(tag):
    g = load(tag)
    m = _model(g)
    x, y = prepared_input(g)
    with torch.no_grad():
        logits, states, gates = _step_forward(m, x)
    _close("logits", logits, g["logits"])
    _close("states", states, g["states"])
    if "gates" in g and not cfg(g)["no_inh"]:
        _close("gates", gates, g["gates"])
    logits, _, _ = _step_forward(m, x)
    F.binary_cross_entropy_with_logits(logits, y.reshape(-1, 1)).backward()
    _close("train_logits", logits.detach(), g["train_logits"])
    for n, p in m.named_parameters():
        key = "grad." + n
        if key in g:
            _close(key, p.grad, g[key], rtol=1e-4, atol=1e-7)


def test_hgru_step_requires_attention():
    from models import ffhgru_hierarchy as hg
    cell = hg.hConvGRUCell(hidden_size=4, kernel_size=3, use_attention=False, timesteps=4)
    z = torch.zeros(1, 4, 8, 8)
    with pytest.raises(ValueError):
        cell(z, z, z)
