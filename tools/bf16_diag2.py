#!/usr/bin/env python3
"""Which bf16-rounded saved state moves the gradient?  The f32 (exact) cell
with selected stored states rounded to bf16 (PT_CELL_ABLATE diagnostic bits
2048 E, 4096 I, 8192 gE+eg) against the plain f32 cell, B=256, T=64, init."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "pathtracker-models_amd"), os.path.join(REPO, "tests")]

os.environ["PT_CELL_DIAG"] = "1"     # the PT_DIAG build honours PT_CELL_ABLATE
import torch  # noqa: E402

import bench  # noqa: E402
from test_gpu_headline import _model, _run  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    t = int(os.environ.get("DIAG_T", 64))
    x, y = bench.make_data(1000, 256, t, dev)
    m = _model(1234, False, t=t).to(dev)
    _, g0 = _run(m, "f32", x, y)
    out = {}
    for name, bits in (("E", 2048), ("I", 4096), ("gE_eg", 8192), ("all", 2048 | 4096 | 8192)):
        os.environ["PT_CELL_ABLATE"] = str(bits)
        _, g = _run(m, "f32", x, y)
        os.environ.pop("PT_CELL_ABLATE")
        row = {}
        for k in g0:
            a, c = g[k], g0[k]
            if c.norm() > 0:
                row[k.replace("unit1.", "")] = round(float(a @ c / (a.norm() * c.norm())), 5)
        out[name] = row
        print(name, json.dumps({k: v for k, v in row.items() if v < 0.999}), flush=True)
    _, g16 = _run(m, "bf16", x, y)
    out["bf16"] = {k.replace("unit1.", ""): round(float(g16[k] @ g0[k] / (g16[k].norm() * g0[k].norm())), 5)
                   for k in g0 if g0[k].norm() > 0}
    print("bf16", json.dumps({k: v for k, v in out["bf16"].items() if v < 0.999}), flush=True)
    json.dump(out, open(os.path.join(REPO, "gpurun_out", "bf16_diag2.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
