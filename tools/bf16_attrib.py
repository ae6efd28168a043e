#!/usr/bin/env python3
"""Attribution of the bf16 cell's deviation from the f32 cell at the headline
size (B=256, T=64) on chosen parameters (default: the 300-step trained ones,
tests/golden/int_trained_headline.npz): the f32 cell with ONE class of values
rounded as the bf16 cell rounds it (PT_DIAG precision bits, pt_cell.hip
RND_*), then cumulative combinations, each against the plain f32 cell --
logit max |err| and per-tensor gradient cosine.  Diagnostic only (the
diagnostic library, libptcell_diag.so)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "pathtracker-models_amd"), os.path.join(REPO, "tests")]

os.environ["PT_CELL_DIAG"] = "1"     # the PT_DIAG build honours PT_CELL_ABLATE
import torch  # noqa: E402

import bench  # noqa: E402
from test_gpu_headline import _model, _run  # noqa: E402

BITS = {"E": 2048, "I": 4096, "gE_eg": 8192, "ci_ce": 524288, "weights": 1048576,
        "bwd_transients": 2097152, "gate_operands": 4194304}


def main():
    dev = torch.device("cuda:0")
    t = int(os.environ.get("DIAG_T", 64))
    b = int(os.environ.get("DIAG_B", 256))
    which = os.environ.get("DIAG_PARAMS", "trained")
    x, y = bench.make_data(1000, b, t, dev)
    m = _model(1234, which if which == "trained" else which == "perturbed", t=t).to(dev)
    lo0, g0 = _run(m, "f32", x, y)

    def compare(lo, g):
        row = {"logit_max_abs_err": float((lo - lo0).abs().max())}
        cos = {}
        for k in g0:
            a, c = g[k], g0[k]
            if c.norm() > 0:
                cos[k.replace("unit1.", "")] = round(float(a @ c / (a.norm() * c.norm())), 5)
        row["cos_min"] = min(cos.values())
        row["cos_min_tensor"] = min(cos, key=cos.get)
        row["cos_below_0.999"] = {k: v for k, v in cos.items() if v < 0.999}
        return row

    out = {"B": b, "T": t, "params": which}
    combos = [(k, v) for k, v in BITS.items()]
    acc = 0
    for k in ("E", "I", "gE_eg", "ci_ce", "weights", "gate_operands", "bwd_transients"):
        acc |= BITS[k]
        combos.append((f"cum_to_{k}", acc))
    for name, bits in combos:
        os.environ["PT_CELL_ABLATE"] = str(bits)
        lo, g = _run(m, "f32", x, y)
        os.environ.pop("PT_CELL_ABLATE")
        out[name] = compare(lo, g)
        print(name, json.dumps(out[name]), flush=True)
    lo, g = _run(m, "bf16", x, y)
    out["bf16"] = compare(lo, g)
    print("bf16", json.dumps(out["bf16"]), flush=True)
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    json.dump(out, open(os.path.join(REPO, "gpurun_out", f"bf16_attrib_{which}.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
