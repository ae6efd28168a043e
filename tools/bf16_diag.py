#!/usr/bin/env python3
"""bf16-vs-f32 gradient agreement of the InT cell over frame counts and
parameter regimes (diagnostic for DESIGN §4): per tensor, cosine and relative
error norm |g16 - g32| / |g32|, and logit errors."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "pathtracker-models_amd"), os.path.join(REPO, "tests")]

import torch  # noqa: E402

import bench  # noqa: E402
from test_gpu_headline import _model, _run  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    b = int(os.environ.get("DIAG_B", 256))
    out = {}
    for t in [int(v) for v in os.environ.get("DIAG_T", "8,32,64").split(",")]:
        x, y = bench.make_data(1000, b, t, dev)
        for perturb in (False, True):
            m = _model(1234, perturb, t=t).to(dev)
            lo32, g32 = _run(m, "f32", x, y)
            lo16, g16 = _run(m, "bf16", x, y)
            row = {"logit_err": float((lo16 - lo32).abs().max()),
                   "logit_spread": float(lo32.max() - lo32.min())}
            for k in g32:
                a, c = g16[k], g32[k]
                if c.norm() > 0:
                    row[k] = [round(float(a @ c / (a.norm() * c.norm())), 5),
                              round(float((a - c).norm() / c.norm()), 5), float(c.norm())]
            out[f"T{t}_{'pert' if perturb else 'init'}"] = row
            print(t, perturb, json.dumps(row), flush=True)
    json.dump(out, open(os.path.join(REPO, "gpurun_out", "bf16_diag.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
