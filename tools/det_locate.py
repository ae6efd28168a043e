#!/usr/bin/env python3
"""Locate a run-to-run difference in the cell's backward: run forward +
backward twice on the same inputs and compare the BatchNorm reduction slots
the workspace keeps for every frame (per-producer partials and group sums,
forward and backward; layout of pt_cell.hip plan()).  The latest frame whose
partials differ is where the backward first diverged (the sweep runs t = T-1
down to 0); partials equal with group sums different point at the reduction
itself.  Diagnostic only."""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "pathtracker-models_amd")]
import torch  # noqa: E402

from ptamd import _lib  # noqa: E402
_lib.use_diag()         # the PT_DIAG build (libptcell_diag.so) honours the switches
from ptamd.cell import _desc, _pack, _ptr, _stream  # noqa: E402
from models import InT  # noqa: E402

NGRP, ALIGN, WGPC = 16, 256, 8


def al(x):
    return (x + ALIGN - 1) // ALIGN * ALIGN


def layout(B, T, es):
    o, r = 0, {}
    r["bnf_cnt"] = o; o += al(T * 2 * NGRP * 4)
    r["bnf_done"] = o; o += al(T * 2 * 4)          # persistent forward counters (pt_cell.hip plan())
    r["err"] = o; o += al(4)
    r["bnf_grp"] = o; o += al(T * 2 * NGRP * 96 * 8)
    r["bnf_part"] = o; o += al(T * 2 * B * 64 * 4)
    r["bnb_cnt"] = o; o += al(T * 2 * NGRP * 4)
    r["bnb_grp"] = o; o += al(T * 2 * NGRP * 64 * 8)
    r["bnb_part"] = o; o += al(T * 2 * B * WGPC * 64 * 4)
    frame = B * 1024 * 32
    for n in TR:
        r[n] = o; o += al(frame * 4)
    r["dci_s"] = o; o += al(frame * T * es)
    r["dce_s"] = o; o += al(frame * T * es)
    r["slab"] = o; o += al(B * WGPC * SLAB * 4)
    r["end"] = o
    return r


TR = ["dEn", "dcE", "dIl", "dEp", "dcI", "GI", "dgEp", "dxp", "dgE", "dIt", "dAt", "GEfin"]
SLAB = 6 * 1024 + 15 * 32


def region_diff(w0, w1, L, B, es):
    """per transient: differing clips (the tensors are [B][1024 px][32 ch] in S)"""
    res = {}
    for n in TR:
        nb = B * 1024 * 32 * (4 if n == "GEfin" else es)
        a, b = w0[L[n]:L[n] + nb], w1[L[n]:L[n] + nb]
        if not torch.equal(a, b):
            d = (a.view(B, -1) != b.view(B, -1))
            clips = d.any(1).nonzero().flatten().tolist()
            rows = (d.view(B, 32, -1).any(2)).nonzero().tolist()[:8]
            res[n] = {"clips": clips[:12], "n_clips": len(clips), "clip_rows": rows}
    a, b = w0[L["slab"]:L["end"]].view(torch.float32), w1[L["slab"]:L["end"]].view(torch.float32)
    if not torch.equal(a, b):
        d = (a.view(B * WGPC, SLAB) != b.view(B * WGPC, SLAB))
        parts = d.any(1).nonzero().flatten().tolist()
        res["slab"] = {"parts": parts[:12], "n_parts": len(parts),
                       "fields": d.any(0).nonzero().flatten().tolist()[:20]}
    return res


def explain(w0, w1, saved, L, B, T, m, t):
    """k_pw_ba head (frame t) recomputed on the host for the rows whose dcE
    differ: which run matches the saved inputs, and where the other deviates."""
    es = 2
    frame = B * 1024 * 32
    fb = al(frame * T * es)
    o_E = 0
    o_I = al(frame * T * 4)                 # I f32 (r04), then gE, ci, ce, eg, [at], Ic (bf16)
    o_ce = o_I + al(frame * T * 4) + 2 * fb
    o_eg = o_ce + fb
    o_bn = o_eg + fb + (fb if es == 2 else 0)
    bf = lambda buf, off, n: buf[off:off + n * 2].view(torch.bfloat16).float()
    nb = frame * es
    d0 = w0[L["dcE"]:L["dcE"] + nb].view(torch.bfloat16).float().view(B, 32, 32, 32)
    d1 = w1[L["dcE"]:L["dcE"] + nb].view(torch.bfloat16).float().view(B, 32, 32, 32)
    dEn = w1[L["dEn"]:L["dEn"] + nb].view(torch.bfloat16).float().view(B, 32, 32, 32)
    I = saved[o_I + t * frame * 4:o_I + (t + 1) * frame * 4].view(torch.float32).view(B, 32, 32, 32)
    ce = bf(saved, o_ce + t * nb, frame).view(B, 32, 32, 32)
    eg = bf(saved, o_eg + t * nb, frame).view(B, 32, 32, 32)
    st = saved[o_bn:o_bn + T * 128 * 4].view(torch.float32).view(T, 128)[t]
    m1, rs1 = st[64:96], st[96:128]
    sd = {k: v.detach().float().flatten() for k, v in m.named_parameters()}
    kap, gam = sd["unit1.kappa"], sd["unit1.gamma"]
    bw1, bb1 = sd["unit1.bn.1.weight"], sd["unit1.bn.1.bias"]
    out = []
    for b, y in (d0 != d1).any(3).any(2).nonzero().tolist()[:4]:
        GE = dEn[b, y] / (1 - eg[b, y])
        xe = (ce[b, y] - m1) * rs1
        cn = bw1 * xe + bb1
        w = kap * I[b, y] + gam
        pe = cn * w
        exp_ = GE * eg[b, y] * torch.sigmoid(pe) * w
        diff = (d0[b, y] != d1[b, y]).nonzero().tolist()
        e0 = float((d0[b, y] - exp_).abs().max())
        e1 = float((d1[b, y] - exp_).abs().max())
        px = sorted({p for p, _ in diff})
        ch = sorted({c for _, c in diff})
        samp = [(p, c, float(d0[b, y, p, c]), float(d1[b, y, p, c]), float(exp_[p, c])) for p, c in diff[:6]]
        # raw per-element record of every differing element (tools: which input
        # of the head, if replaced, reproduces the deviating run's outputs)
        E_prev = saved[o_E + (t - 1) * frame * 4:o_E + t * frame * 4].view(torch.float32).view(B, 32, 32, 32)
        tr = {n: (w0[L[n]:L[n] + nb].view(torch.bfloat16).float().view(B, 32, 32, 32),
                  w1[L[n]:L[n] + nb].view(torch.bfloat16).float().view(B, 32, 32, 32)) for n in ("dcE", "dIl", "dEp", "dEn")}
        raw = []
        for p, c in diff[:16]:
            raw.append({"p": p, "c": c, "I": float(I[b, y, p, c]), "ce": float(ce[b, y, p, c]),
                        "eg": float(eg[b, y, p, c]), "Eo": float(E_prev[b, y, p, c]),
                        "kap": float(kap[c]), "gam": float(gam[c]), "bw1": float(bw1[c]), "bb1": float(bb1[c]),
                        "m1": float(m1[c]), "rs1": float(rs1[c]),
                        "I_row": I[b, y, :, c].tolist(), "ce_row": ce[b, y, :, c].tolist(),
                        **{f"{n}_{k}": float(v[k][b, y, p, c]) for n, v in tr.items() for k in (0, 1)}})
        out.append({"clip": b, "row": y, "n_diff": len(diff), "px": px, "ch": ch,
                    "maxerr_run0": e0, "maxerr_run1": e1, "samples": samp, "raw": raw})
    return out


def main():
    b, t = int(os.environ.get("B", 256)), int(os.environ.get("T", 64))
    reps = int(os.environ.get("REPS", 3))
    dev = torch.device("cuda:0")
    lib = _lib.load()
    torch.manual_seed(3)
    m = InT.InT(dimensions=32, timesteps=t, kernel_size=7).to(dev)
    m.cell_dtype = os.environ.get("DTYPE", "bf16")
    x = torch.rand(b, 3, t, 32, 32, device=dev)
    d = _desc(m.cell_config(), x, 32)
    saved = torch.empty(lib.pt_cell_saved_bytes(ctypes.byref(d)), dtype=torch.uint8, device=dev)
    ws = torch.empty(lib.pt_cell_workspace_bytes(ctypes.byref(d)), dtype=torch.uint8, device=dev)
    d_e = torch.randn((b, 32, 32, 32), device=dev, generator=torch.Generator(device=dev).manual_seed(1)) * 1e-3
    params = [p.detach().contiguous() if p is not None else None for p in m.cell_params()]
    pp = _pack(_lib.Params, params)
    st = _stream(dev)
    es = 2 if m.cell_dtype == "bf16" else 4
    L = layout(b, t, es)
    snaps = []
    for _ in range(reps):
        e = torch.empty((b, 32, 32, 32), device=dev)
        _lib.check(lib.pt_cell_forward(ctypes.byref(d), _ptr(x), ctypes.byref(pp), _ptr(saved), _ptr(ws),
                                       _ptr(e), None, st))
        gr = [torch.empty_like(p) if p is not None else None for p in params]
        gg = _pack(_lib.Grads, gr)
        _lib.check(lib.pt_cell_backward(ctypes.byref(d), _ptr(x), ctypes.byref(pp), _ptr(saved), _ptr(ws),
                                        _ptr(d_e), ctypes.byref(gg), st))
        torch.cuda.synchronize()
        w = ws[:L["end"]].clone()
        snaps.append((w, saved.clone()))
    out = {"stop": os.environ.get("PT_CELL_DEBUG_STOP"), "B": b, "T": t, "dtype": m.cell_dtype, "lib": lib.pt_version().decode(), "pairs": []}
    w0, s0 = snaps[0]
    for w1, s1 in snaps[1:]:
        rec = {"saved_equal": bool(torch.equal(s0, s1)), "frames": [],
               "transients": region_diff(w0, w1, L, b, es)}
        fg0 = w0[L["bnf_grp"]:L["bnf_part"]].view(torch.float64).view(t, 2, NGRP, 96)
        fg1 = w1[L["bnf_grp"]:L["bnf_part"]].view(torch.float64).view(t, 2, NGRP, 96)
        bg0 = w0[L["bnb_grp"]:L["bnb_part"]].view(torch.float64).view(t, 2, NGRP, 64)
        bg1 = w1[L["bnb_grp"]:L["bnb_part"]].view(torch.float64).view(t, 2, NGRP, 64)
        bp0 = w0[L["bnb_part"]:L["bnb_part"] + t * 2 * b * WGPC * 256].view(torch.float32).view(t, 2, b * WGPC, 64)
        bp1 = w1[L["bnb_part"]:L["bnb_part"] + t * 2 * b * WGPC * 256].view(torch.float32).view(t, 2, b * WGPC, 64)
        for tt in range(t - 1, -1, -1):
            for bn in (0, 1):
                pb2 = os.environ.get("PT_PWB2", "1") != "0"     # k_pw_bb2: 2 (bf16) / 8 (f32) producers per clip (InT; hGRU bf16 uses 4)
                nprod = b * (((2 if es == 2 else 8) if pb2 else WGPC) if bn == 0 else 2)
                pd = (bp0[tt, bn, :nprod] != bp1[tt, bn, :nprod]).any(1).nonzero().flatten().tolist()
                gd = (bg0[tt, bn] != bg1[tt, bn]).any(1).nonzero().flatten().tolist()
                fd = (fg0[tt, bn] != fg1[tt, bn]).any(1).nonzero().flatten().tolist()
                if pd or gd or fd:
                    rec["frames"].append({"t": tt, "bn": bn, "bwd_part_rows": pd[:16], "n_part": len(pd),
                                          "bwd_grp": gd, "fwd_grp": fd})
        rec["frames"] = rec["frames"][:12]
        if "dcE" in rec["transients"] and os.environ.get("PT_CELL_DEBUG_STOP"):
            rec["explain"] = explain(w0, w1, s0, L, b, t, m, int(os.environ.get("EXPLAIN_T", t - 2)))
        out["pairs"].append(rec)
        print(json.dumps(rec), flush=True)
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    tag = os.environ.get("PT_CELL_DEBUG_STOP", "all")
    json.dump(out, open(os.path.join(REPO, "gpurun_out", f"det_locate_{tag}.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
