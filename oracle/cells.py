"""CPU oracle for the recurrent-cell hot path — TEST INFRASTRUCTURE ONLY.

Clean-room restatement, in plain PyTorch fp32 on the CPU, of the reference's
InT / hGRU / ConvLSTM forward passes (and, through torch autograd, their BPTT
backward).  It is written functionally over a ``state_dict``-shaped dict so
that it shares no structure with the reference classes; every step cites the
reference line it restates (paths relative to the reference repo root).

Who may use this module: ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` — as the checker / the CPU baseline,
never as the thing measured or shipped.  The product path
(``pathtracker-models_amd``) never imports it.

Pinning: ``tests/golden/make_golden.py`` imports the reference itself (in the
build container only) and writes golden vectors under ``tests/golden/``;
``tests/test_oracle_golden.py`` checks this restatement against them.

Op graph: the per-frame slice ``xbn[:, :, t]`` on the 5-D stem output is kept
(reference ``models/InT.py:225``) so that the CPU timing of this oracle stays
representative of the reference (its O(T^2) SelectBackward zero-fill included).
"""
from __future__ import annotations

import math
from typing import Callable, Dict

import torch
import torch.nn.functional as F

Tensor = torch.Tensor
Params = Dict[str, Tensor]


def activation(name: str) -> Callable[[Tensor], Tensor]:
    """The model's ``nl``: softplus (beta 1, threshold 20) or tanh.

    Reference: ``models/InT.py:184`` (``nl=F.softplus`` default) and
    ``utils/engine.py:138-146`` (``InT_tanh`` passes ``nl=F.tanh``).
    """
    if name == "softplus":
        return F.softplus
    if name == "tanh":
        return torch.tanh
    raise ValueError(f"unknown activation {name!r}")


def _gate(sd: Params, prefix: str, name: str, v: Tensor) -> Tensor:
    # 1x1 Conv2d with bias (models/InT.py:73-84).
    return F.conv2d(v, sd[f"{prefix}{name}_gate.weight"], sd[f"{prefix}{name}_gate.bias"])


def _bn_batch(v: Tensor, w: Tensor, b: Tensor, eps: float) -> Tensor:
    # BatchNorm2d(eps=1e-3, affine, track_running_stats=False): batch statistics
    # in train AND eval mode (models/InT.py:102).
    return F.batch_norm(v, None, None, w, b, training=True, eps=eps)


def sync_batch_norm(group=None) -> Callable[[Tensor, Tensor, Tensor, float], Tensor]:
    """SyncBN: BatchNorm with batch statistics over the clips of every rank of
    ``group`` (the opt-in mode of the HIP cell).  Per-channel
    sums and sums of squares are all-reduced with the differentiable
    ``torch.distributed.nn`` all-reduce, so autograd gives the matching
    backward (the all-reduced sum dy and sum dy * xhat of the HIP backward)."""
    from torch.distributed.nn.functional import all_reduce

    def bn(v: Tensor, w: Tensor, b: Tensor, eps: float) -> Tensor:
        vd = v.double()                                  # fp64 sums: no cancellation in var
        n = torch.tensor([float(v.shape[0] * v.shape[2] * v.shape[3])], dtype=torch.float64)
        s1 = all_reduce(vd.sum((0, 2, 3)), group=group)
        s2 = all_reduce((vd * vd).sum((0, 2, 3)), group=group)
        cnt = all_reduce(n, group=group)
        mean = s1 / cnt
        var = s2 / cnt - mean * mean
        xhat = (vd - mean[None, :, None, None]) / torch.sqrt(var + eps)[None, :, None, None]
        return (xhat * w[None, :, None, None] + b[None, :, None, None]).to(v.dtype)
    return bn


def horizontal_frame(sd: Params, prefix: str, x_t: Tensor, inh: Tensor, exc: Tensor,
                     act: Callable[[Tensor], Tensor], *, no_inh: bool = False,
                     hgru: bool = False, eps: float = 1e-3, bn=None):
    """One recurrent step.  Returns ``(inh_new, exc_new, att)``.

    InT ``rCell.forward`` (models/InT.py:145-179) with ``use_attention=True``
    (hard-wired by ``InT.__init__`` at models/InT.py:196); ``hgru=True`` gives
    ``hConvGRUCell.forward`` (models/ffhgru_hierarchy.py:135-173), whose only
    difference is that the gated inhibition is the attention map itself
    (models/ffhgru_hierarchy.py:147).  ``bn``: the BatchNorm (default: batch
    statistics of this process's clips, as the reference's DataParallel
    replicas; :func:`sync_batch_norm` for SyncBN).
    """
    bnf = bn or _bn_batch
    k = sd[f"{prefix}w_exc"].shape[-1]
    pad = k // 2
    att = torch.sigmoid(_gate(sd, prefix, "a_w", x_t) + _gate(sd, prefix, "a_u", exc))  # InT.py:148
    g_exc = att * exc                                                                   # InT.py:153
    g_inh = att if hgru else inh                                                        # InT.py:157 / ffhgru:147
    if not no_inh:
        c_i = bnf(F.conv2d(g_exc, sd[f"{prefix}w_inh"], padding=pad),
                        sd[f"{prefix}bn.0.weight"], sd[f"{prefix}bn.0.bias"], eps)      # InT.py:161
        i_hat = act(x_t - act(c_i * (sd[f"{prefix}alpha"] * g_inh + sd[f"{prefix}mu"])))  # InT.py:162
        i_g = torch.sigmoid(_gate(sd, prefix, "i_w", x_t) + _gate(sd, prefix, "i_u", g_inh))  # InT.py:165
        inh_new = (1 - i_g) * inh + i_g * i_hat                                          # InT.py:166
    else:
        inh_new, g_inh = g_exc, exc                                                      # InT.py:168
    e_g = torch.sigmoid(_gate(sd, prefix, "e_w", g_inh) + _gate(sd, prefix, "e_u", g_exc))  # InT.py:171
    c_e = bnf(F.conv2d(inh_new, sd[f"{prefix}w_exc"], padding=pad),
                    sd[f"{prefix}bn.1.weight"], sd[f"{prefix}bn.1.bias"], eps)            # InT.py:172
    e_hat = act(c_e * (sd[f"{prefix}kappa"] * inh_new + sd[f"{prefix}gamma"]))         # InT.py:173
    exc_new = (1 - e_g) * exc + e_g * e_hat                                              # InT.py:175
    return inh_new, exc_new, att


def stem(sd: Params, x: Tensor, act: Callable[[Tensor], Tensor]) -> Tensor:
    """1x1x1 Conv3d 3->C then ``nl`` (models/InT.py:212-213)."""
    return act(F.conv3d(x, sd["preproc.weight"], sd["preproc.bias"]))


def readout(sd: Params, exc: Tensor, x: Tensor) -> Tensor:
    """Readout on the last excitation (models/InT.py:236-241).

    ``cat([readout_conv(E_T), x[:, 2, 0]])`` -> 5x5 ``target_conv`` (pad 2) ->
    global average pool -> ``Linear(1, 1)``.
    """
    r = F.conv2d(exc, sd["readout_conv.weight"], sd["readout_conv.bias"])
    o = torch.cat([r, x[:, 2, 0][:, None]], 1)
    o = F.conv2d(o, sd["target_conv.weight"], sd["target_conv.bias"], padding=2)
    o = F.avg_pool2d(o, kernel_size=o.shape[2:]).reshape(x.shape[0], -1)
    return F.linear(o, sd["readout_dense.weight"], sd["readout_dense.bias"])


def recurrent_forward(sd: Params, x: Tensor, *, act: str = "softplus", no_inh: bool = False,
                      hgru: bool = False, testmode: bool = False, eps: float = 1e-3, bn=None):
    """Whole-clip forward of InT (models/InT.py:210-245) or FFhGRU
    (models/ffhgru_hierarchy.py:211-276).

    Returns ``(logits [B,1], exc_seq list[T] of [B,C,H,W], att_seq list[T])``;
    ``states``/``gates`` of testmode are ``readout_conv(E_t)`` / ``att_t``
    stacked on dim 1 (InT.py:230-233,244) — see :func:`testmode_outputs`.
    """
    nl = activation(act)
    xbn = stem(sd, x, nl)
    b, c, t_len, h, w = xbn.shape
    exc = torch.zeros((b, c, h, w), dtype=xbn.dtype)   # InT.py:217-218
    inh = torch.zeros((b, c, h, w), dtype=xbn.dtype)
    exc_seq, att_seq = [], []
    for t in range(t_len):                               # InT.py:223
        inh, exc, att = horizontal_frame(sd, "unit1.", xbn[:, :, t], inh, exc, nl,
                                         no_inh=no_inh, hgru=hgru, eps=eps, bn=bn)
        if testmode:
            exc_seq.append(exc)
            att_seq.append(att)
    logits = readout(sd, exc, x)
    if not testmode:
        exc_seq = [exc]
    return logits, exc_seq, att_seq


def testmode_outputs(sd: Params, exc_seq, att_seq):
    """``(states [B,T,1,H,W], gates [B,T,C,H,W])`` as InT.forward(testmode=True)."""
    states = torch.stack([F.conv2d(e, sd["readout_conv.weight"], sd["readout_conv.bias"])
                          for e in exc_seq], 1)
    return states, torch.stack(att_seq, 1)


def bce_logits(logits: Tensor, labels: Tensor) -> Tensor:
    """``BCEWithLogitsLoss()(output, target.reshape(-1, 1))`` (mainclean.py:156,190)."""
    return F.binary_cross_entropy_with_logits(logits, labels.float().reshape(-1, 1))


def adam_step(params: Params, grads: Params, lr: float = 3e-4, betas=(0.9, 0.999),
              eps: float = 1e-8) -> Params:
    """First Adam step from zero moments (torch.optim.Adam defaults, mainclean.py:157).

    At step 1: m = (1-b1) g, v = (1-b2) g^2, update = lr * m_hat / (sqrt(v_hat) + eps)
    with m_hat = g and v_hat = g^2.  Parameters without a grad are unchanged.
    """
    out = {}
    b1, b2 = betas
    for k, p in params.items():
        g = grads.get(k)
        if g is None:
            out[k] = p.clone()
            continue
        m = (1 - b1) * g
        v = (1 - b2) * g * g
        m_hat = m / (1 - b1)
        v_hat = v / (1 - b2)
        out[k] = p - lr * m_hat / (v_hat.sqrt() + eps)
    return out


# ----------------------------------------------------------------------------- ConvLSTM

def convlstm_forward(sd: Params, img: Tensor, timesteps: int, eps: float = 1e-3,
                     with_jv: bool = False, mu: float = 0.9, create_graph: bool = False):
    """ConvLSTM on a static single-channel image (models/convlstm.py:116-147, bptt).

    conv0 (Gabor 7x7, 1->25, bias) then ``pow 2`` (:118-119); ``timesteps``
    iterations of the 4-gate cell on the same x (:137-139, cell :84-90; x-convs
    with bias, h-convs without); ``BN(h)`` (batch stats, :111,146) -> 1x1
    ``conv6`` 25->2 (:112,147).  Returns ``(output [B,2,H,W], h_T, c_T)``, or
    ``(output, h_T, c_T, jv_penalty)`` with ``with_jv`` (see
    :func:`convlstm_jv_penalty`; ``create_graph``: the penalty keeps its graph,
    as the reference's ``jacobian_penalty=True`` builds it, :158-162).
    """
    x = F.conv2d(img, sd["conv0.weight"], sd["conv0.bias"], padding=3).pow(2)
    k = sd["unit1.Wxi.weight"].shape[-1]
    pad = (k - 1) // 2
    h = torch.zeros_like(x)
    c = torch.zeros_like(x)

    def xconv(g, v):
        return F.conv2d(v, sd[f"unit1.Wx{g}.weight"], sd[f"unit1.Wx{g}.bias"], padding=pad)

    def hconv(g, v):
        return F.conv2d(v, sd[f"unit1.Wh{g}.weight"], None, padding=pad)

    hs, cs = [], []
    for _ in range(timesteps):
        i_t = torch.sigmoid(xconv("i", x) + hconv("i", h))
        f_t = torch.sigmoid(xconv("f", x) + hconv("f", h))
        c = f_t * c + i_t * torch.tanh(xconv("c", x) + hconv("c", h))
        o_t = torch.sigmoid(xconv("o", x) + hconv("o", h))
        h = o_t * torch.tanh(c)
        hs.append(h)
        cs.append(c)
    out = F.batch_norm(h, None, None, sd["bn.weight"], sd["bn.bias"], training=True, eps=eps)
    out = F.conv2d(out, sd["conv6.weight"], sd["conv6.bias"])
    if not with_jv:
        return out, h, c
    return out, h, c, convlstm_jv_penalty(hs, cs, mu, create_graph)


def convlstm_jv_penalty(hs, cs, mu: float = 0.9, create_graph: bool = False) -> Tensor:
    """Training-mode Jacobian penalty of ConvLSTM (models/convlstm.py:150-161, l1):

        jv = clamp(J_h^T 1 - mu, 0)^2 + clamp(J_c^T 1 - mu, 0)^2

    with J_h = d h_{T-1} / d h_{T-2} (the one-step path through the h-convs) and
    J_c = d c_{T-1} / d c_{T-2}, which autograd takes along EVERY path: the
    direct forget-gate term f_{T-1} and the path through h_{T-2} = o tanh(c_{T-2})
    into the next step's gates.  ``hs`` / ``cs`` are the per-step states of a
    graph that requires grad; needs ``timesteps >= 2`` (the reference's
    ``state_2nd_last`` is unbound otherwise).  ``create_graph`` (the reference's
    ``jacobian_penalty=True``, :158-162): the penalty is returned with its graph,
    so its parameter gradients (through the last step's Jacobian and, via
    h_{T-2} / c_{T-2}, the earlier steps) reach a loss that adds it.
    """
    ones = torch.ones_like(hs[-1])
    jh = torch.autograd.grad(hs[-1], hs[-2], ones, retain_graph=True, create_graph=create_graph)[0]
    jc = torch.autograd.grad(cs[-1], cs[-2], ones, retain_graph=True, create_graph=create_graph)[0]
    jv = (jh - mu).clamp(0) ** 2 + (jc - mu).clamp(0) ** 2
    return jv if create_graph else jv.detach()


def flops_per_clip_frame(c: int = 32, h: int = 32, w: int = 32, k: int = 7) -> int:
    """Algorithmic forward FLOPs of one InT frame for one clip:
    two kxk CxC convs + six 1x1 CxC gates."""
    return 2 * (2 * c * c * k * k * h * w) + 6 * (2 * c * c * h * w)


def param_count(sd: Params) -> int:
    return int(sum(math.prod(v.shape) for v in sd.values()))


def convlstm_video_forward(sd: Params, x: Tensor, act: str = "softplus"):
    """The ConvLSTM clip model (repo models/convlstm.py ConvLSTMVideo, DESIGN.md
    §10), restated with stock torch ops: the InT stem per frame
    (models/InT.py:212-213), the reference ConvLSTMCell step
    (models/convlstm.py:84-90) with the frame as its input, and InT's readout
    (models/InT.py:236-241) on h_T.  Returns ``(logits [B,1], h_T, hs, cs)``."""
    nl = F.softplus if act == "softplus" else torch.tanh
    xbn = nl(F.conv3d(x, sd["preproc.weight"], sd["preproc.bias"]))
    k = sd["unit1.Wxi.weight"].shape[-1]
    pad = (k - 1) // 2
    b, ch, t_len, hh, ww = xbn.shape
    h = torch.zeros((b, ch, hh, ww), dtype=x.dtype)
    c = torch.zeros_like(h)

    def xconv(g, v):
        return F.conv2d(v, sd[f"unit1.Wx{g}.weight"], sd[f"unit1.Wx{g}.bias"], padding=pad)

    def hconv(g, v):
        return F.conv2d(v, sd[f"unit1.Wh{g}.weight"], None, padding=pad)

    hs, cs = [], []
    for t in range(t_len):
        xt = xbn[:, :, t]
        i_t = torch.sigmoid(xconv("i", xt) + hconv("i", h))
        f_t = torch.sigmoid(xconv("f", xt) + hconv("f", h))
        c = f_t * c + i_t * torch.tanh(xconv("c", xt) + hconv("c", h))
        o_t = torch.sigmoid(xconv("o", xt) + hconv("o", h))
        h = o_t * torch.tanh(c)
        hs.append(h)
        cs.append(c)
    o = torch.cat([F.conv2d(h, sd["readout_conv.weight"], sd["readout_conv.bias"]),
                   x[:, 2, 0][:, None]], 1)
    o = F.conv2d(o, sd["target_conv.weight"], sd["target_conv.bias"], padding=2)
    o = F.avg_pool2d(o, kernel_size=o.size()[2:])
    o = F.linear(o.reshape(b, -1), sd["readout_dense.weight"], sd["readout_dense.bias"])
    return o, h, hs, cs
