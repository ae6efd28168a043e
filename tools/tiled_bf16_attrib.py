#!/usr/bin/env python3
"""r06: why the bf16 cell's w_exc gradient on the tiled hgru_64 golden sits
at cosine 0.994 against the reference (every untiled golden: >= 0.9997).
The golden's gradients against: the f32 cell, the bf16 cell, and the f32
cell with every bf16 rounding class applied (PT_DIAG precision bits, as
tools/bf16_attrib.py) -- if the last reproduces the bf16 figure the deviation
is the rounding, not the tiled kernels.  Diagnostic library only."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "pathtracker-models_amd"), os.path.join(REPO, "tests")]
os.environ["PT_CELL_DIAG"] = "1"

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from goldens import load, prepared_input  # noqa: E402
from test_gpu_parity import _model  # noqa: E402

ALL_RND = 2048 | 4096 | 8192 | 524288 | 1048576 | 2097152 | 4194304


def cosines(m, g, x, y, dtype):
    m.cell_dtype = dtype
    m.zero_grad(set_to_none=True)
    out, _ = m(x)
    F.binary_cross_entropy_with_logits(out, y.reshape(-1, 1)).backward()
    res = {}
    for k, p in m.named_parameters():
        if p.grad is None:
            continue
        a = p.grad.detach().cpu().double().flatten()
        b = torch.from_numpy(g["grad." + k]).double().flatten()
        if b.norm() > 1e-8:
            res[k] = round(float(a @ b / (a.norm() * b.norm())), 6)
    return res


def main():
    dev = torch.device("cuda:0")
    out = {}
    for tag in os.environ.get("TAGS", "hgru_64,hgru_c32,int_64x96,int_c32").split(","):
        g = load(tag)
        x, y = prepared_input(g)
        x, y = x.to(dev), y.to(dev)
        m = _model(g, "f32").to(dev)
        rec = {"f32": cosines(m, g, x, y, "f32"), "bf16": cosines(m, g, x, y, "bf16")}
        os.environ["PT_CELL_ABLATE"] = str(ALL_RND)
        rec["f32_all_rounding"] = cosines(m, g, x, y, "f32")
        os.environ.pop("PT_CELL_ABLATE")
        out[tag] = {k: {"min": min(v.values()), "argmin": min(v, key=v.get),
                        "w_exc": v.get("unit1.w_exc"), "w_inh": v.get("unit1.w_inh")} for k, v in rec.items()}
        print(tag, json.dumps(out[tag]), flush=True)
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", "tiled_bf16_attrib.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
