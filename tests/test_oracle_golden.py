"""Pin the CPU oracle (oracle/cells.py) to the reference's own outputs.

The golden vectors were produced by importing the reference model files in the
build container (tests/golden/make_golden.py).  Tolerances: the oracle runs the
same fp32 torch CPU ops, so agreement is at rounding level (<=1e-5 relative).
"""
import numpy as np
import pytest
import torch

from oracle import cells
from goldens import cfg, load, params, prepared_input

RECURRENT = ["int_tiny_c8", "int_c32", "int_noinh", "int_tanh", "int_lesion", "int_cfg1",
             "hgru_c32", "hgru_b4t16", "hgru_64", "int_64x96", "int_k15", "int_k9_c16",
             "hgru_k15_64", "hgru_c24"]


def _close(a, b, rtol=2e-5, atol=2e-6):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    assert a.shape == b.shape, (a.shape, b.shape)
    err = np.abs(a - b)
    tol = atol + rtol * np.abs(b).max()
    assert err.max() <= tol, f"max err {err.max():.3e} > {tol:.3e}"


@pytest.mark.parametrize("tag", RECURRENT)
def test_recurrent_forward_testmode(tag):
    g = load(tag)
    c = cfg(g)
    sd = params(g)
    x, _ = prepared_input(g)
    with torch.no_grad():
        logits, exc_seq, att_seq = cells.recurrent_forward(
            sd, x, act=c["act"], no_inh=c["no_inh"], hgru=c["cell"] == "hgru", testmode=True)
        states, gates = cells.testmode_outputs(sd, exc_seq, att_seq)
    _close(logits, g["logits"])
    _close(states, g["states"])
    if "gates" in g:
        _close(gates, g["gates"])


@pytest.mark.parametrize("tag", RECURRENT)
def test_recurrent_bptt_grads_and_adam(tag):
    g = load(tag)
    c = cfg(g)
    sd = params(g)
    frozen = {f"unit1.{n}" for n in c["lesion"]} | {"unit1.w"}
    if c["cell"] == "hgru":
        frozen |= {"bn.weight", "bn.bias"}          # FFhGRU.bn is registered but unused
    if c["no_inh"]:
        frozen |= {"unit1.alpha", "unit1.mu"}       # unused in the no_inh branch
    leaf = {k: v.clone().requires_grad_(k not in frozen) for k, v in sd.items()}
    x, y = prepared_input(g)
    logits, _, _ = cells.recurrent_forward(leaf, x, act=c["act"], no_inh=c["no_inh"],
                                           hgru=c["cell"] == "hgru")
    loss = cells.bce_logits(logits, y)
    loss.backward()
    _close(logits.detach(), g["train_logits"])
    _close(loss.item(), float(g["loss"]))
    grads = {k: v.grad for k, v in leaf.items() if v.grad is not None}
    ref_grads = {k[len("grad."):]: v for k, v in g.items() if k.startswith("grad.")}
    # every parameter the reference differentiates, and no other, gets a grad
    assert set(grads) == set(ref_grads), set(grads) ^ set(ref_grads)
    for k, v in ref_grads.items():
        _close(grads[k], v, rtol=1e-4, atol=1e-7)
    stepped = cells.adam_step({k: v.detach() for k, v in leaf.items()}, grads)
    for k in sd:
        if k.startswith("unit1.w") and k == "unit1.w":
            continue
        _close(stepped[k], g["adam." + k], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("tag", ["convlstm_k7", "convlstm_k15", "convlstm_t2"])
def test_convlstm_static(tag):
    g = load(tag)
    sd = params(g)
    img = torch.from_numpy(g["img"])
    target = torch.from_numpy(g["target"])
    steps = int(g["cfg_timesteps"])
    with torch.no_grad():
        out, _, _ = cells.convlstm_forward(sd, img, steps)
    _close(out, g["eval_output"])
    leaf = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    out, _, _, jv = cells.convlstm_forward(leaf, img, steps, with_jv=True)
    _close(jv, g["jv_penalty"], rtol=1e-4, atol=1e-6)
    loss = torch.nn.functional.cross_entropy(out, target)
    loss.backward()
    _close(loss.item(), float(g["loss"]))
    for k in (k for k in g if k.startswith("grad.")):
        _close(leaf[k[len("grad."):]].grad, g[k], rtol=1e-4, atol=1e-7)


@pytest.mark.parametrize("tag", ["convlstm_jvp", "convlstm_jvp_t2"])
def test_convlstm_jacobian_penalty_with_graph(tag):
    """jacobian_penalty=True (models/convlstm.py:158-162, create_graph): the
    gradients of loss + 10 mean(jv_penalty) (mainclean.py:191-195)."""
    g = load(tag)
    assert int(g["cfg_jacobian_penalty"]) == 1
    sd = params(g)
    img = torch.from_numpy(g["img"])
    target = torch.from_numpy(g["target"])
    steps = int(g["cfg_timesteps"])
    leaf = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    out, _, _, jv = cells.convlstm_forward(leaf, img, steps, with_jv=True, create_graph=True)
    _close(jv.detach(), g["jv_penalty"], rtol=1e-4, atol=1e-6)
    loss = torch.nn.functional.cross_entropy(out, target)
    (loss + jv.mean() * 1e1).backward()
    _close(loss.item(), float(g["loss"]))
    for k in (k for k in g if k.startswith("grad.")):
        _close(leaf[k[len("grad."):]].grad, g[k], rtol=1e-4, atol=1e-7)


def test_flop_model():
    # 218,103,808 FLOP per clip-frame forward at C=32, 32x32, k=7
    assert cells.flops_per_clip_frame() == 218_103_808
