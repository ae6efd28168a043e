#!/usr/bin/env python3
"""where the static ConvLSTM's bf16 gradient deviation
comes from (CPU, test infrastructure: the oracle's ConvLSTM with chosen
values rounded as the bf16 library rounds them).

The library (csrc/pt_lstm.hip) keeps the gate
pre-activations P, the cell state c and all gate math in f32 and rounds to
bf16: the conv operands x (the Gabor-squared input), h (the stored hidden
state, also the returned h_T), the conv weights, and in the backward dP (the
transposed conv's input and the weight gradient's D operand; the bias
gradients are the f32 sums).  Each class is rounded alone, then all at once,
on the reference golden of test_convlstm_bf16_tolerance (convlstm_k15:
k = 15, T = 3, B = 2) and of the Jacobian-penalty test (convlstm_jvp); per
tensor gradient cosine against the unrounded oracle, which equals the
reference golden at 1e-6.  x is split into its forward value (xf) and the
weight gradient's X operand (xg), the weights into Wx and Wh; the last row
("split") is the library after r06's fix: every class rounded except the
forward x-conv's value (three bf16 passes, hi/lo splits of x and Wx).  Writes profiles/r06_lstm_bf16_attrib.json."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "pathtracker-models_amd"), os.path.join(REPO, "tests")]

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from goldens import load, params  # noqa: E402
from oracle import cells  # noqa: E402


def rb(v):
    return v.to(torch.bfloat16).float()


class _RoundGrad(torch.autograd.Function):
    @staticmethod
    def forward(ctx, v):
        return v.view_as(v)

    @staticmethod
    def backward(ctx, g):
        return rb(g)


def forward(sd, img, T, what, with_jv=False):
    """cells.convlstm_forward with the classes in ``what`` rounded."""
    x = F.conv2d(img, sd["conv0.weight"], sd["conv0.bias"], padding=3).pow(2)
    k = sd["unit1.Wxi.weight"].shape[-1]
    pad = (k - 1) // 2
    W = (lambda w: w + (rb(w) - w).detach()) if "w" in what else (lambda w: w)   # value rounded, grad identity
    xo = x + (rb(x) - x).detach() if "x" in what else x
    h = torch.zeros_like(x)
    c = torch.zeros_like(x)

    Wx = (lambda w: w + (rb(w) - w).detach()) if ("w" in what or "wx" in what) else (lambda w: w)
    Wh = (lambda w: w + (rb(w) - w).detach()) if ("w" in what or "wh" in what) else (lambda w: w)

    def xconv(g):
        w, b = Wx(sd[f"unit1.Wx{g}.weight"]), sd[f"unit1.Wx{g}.bias"]
        if "xf" in what:      # x rounded in the forward value only (the weight gradient's X in f32)
            return F.conv2d(x, w, b, padding=pad) + (F.conv2d(rb(x), w, b, padding=pad)
                                                     - F.conv2d(x, w, b, padding=pad)).detach()
        if "xg" in what or "split" in what:
            # the forward value in f32 (split: the library's three-pass x-conv,
            # hi x hi + lo x hi + hi x lo, exact to ~2^-16); the weight gradient's
            # X operand bf16 (xg, split); split: d x through the bf16 Wx too
            w0 = sd[f"unit1.Wx{g}.weight"]
            p = F.conv2d(x.detach(), w0.detach(), b, padding=pad)
            p = p + F.conv2d(rb(x).detach(), w0, None, padding=pad) - F.conv2d(rb(x).detach(), w0.detach(), None, padding=pad)
            wd = rb(w0).detach() if "split" in what else w0.detach()
            return p + F.conv2d(x, wd, None, padding=pad) - F.conv2d(x.detach(), wd, None, padding=pad)
        return F.conv2d(xo, w, b, padding=pad)

    def P(g, hv):
        p = xconv(g)
        p = p + F.conv2d(hv, Wh(sd[f"unit1.Wh{g}.weight"]), None, padding=pad)
        return _RoundGrad.apply(p) if "dP" in what else p

    hs, cs = [], []
    for _ in range(T):
        i_t = torch.sigmoid(P("i", h))
        f_t = torch.sigmoid(P("f", h))
        c = f_t * c + i_t * torch.tanh(P("c", h))
        o_t = torch.sigmoid(P("o", h))
        h = o_t * torch.tanh(c)
        if "h" in what:
            h = h + (rb(h) - h).detach()
        hs.append(h)
        cs.append(c)
    out = F.batch_norm(h, None, None, sd["bn.weight"], sd["bn.bias"], training=True, eps=1e-3)
    out = F.conv2d(out, sd["conv6.weight"], sd["conv6.bias"])
    if not with_jv:
        return out, None
    return out, cells.convlstm_jv_penalty(hs, cs, 0.9, True)


def run(g, what, with_jv):
    sd = {k: v.clone().requires_grad_(True) for k, v in params(g).items()}
    img = torch.from_numpy(g["img"]).float()
    tgt = torch.from_numpy(g["target"]).long()
    out, jv = forward(sd, img, int(g["cfg_timesteps"]), what, with_jv)
    loss = torch.nn.CrossEntropyLoss()(out, tgt)
    if jv is not None:
        loss = loss + jv.mean() * 1e1
    loss.backward()
    return out.detach().double(), {k: v.grad.detach().double().flatten() for k, v in sd.items()
                                   if v.grad is not None}


def main():
    torch.set_num_threads(8)
    res = {}
    for name, with_jv in (("convlstm_k15", False), ("convlstm_jvp", True)):
        g = load(name)
        o0, g0 = run(g, (), with_jv)
        rec = {}
        for what in (("x",), ("xf",), ("xg",), ("w",), ("wx",), ("wh",), ("h",), ("dP",), ("x", "w"),
                     ("x", "w", "h", "dP"), ("split", "wh", "h", "dP")):
            o, gg = run(g, what, with_jv)
            cos = {}
            for k in g0:
                if g0[k].norm() > 0:
                    cos[k] = float(gg[k] @ g0[k] / (gg[k].norm() * g0[k].norm()))
            worst = sorted(cos, key=cos.get)[:4]
            rec["+".join(what)] = {"output_rel_rms": float((o - o0).norm() / o0.norm()),
                                   "grad_cos_min": min(cos.values()),
                                   "worst": {k: round(cos[k], 5) for k in worst}}
            print(name, "+".join(what), json.dumps(rec["+".join(what)]), flush=True)
        res[name] = rec
    path = os.path.join(REPO, "profiles", "r06_lstm_bf16_attrib.json")
    with open(path, "w") as f:
        json.dump(res, f, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
