#!/usr/bin/env python3
"""what reading only the hi planes of E / I costs in
accuracy.  The bf16 cell forms kappa I + gamma (forward E update, k_pw_ba)
and d att = dgE E_t (k_pw_ba) from the hi (bf16) plane of I / E; the
PT_EI_FULL=1 build (ptamd/ab/libptcell_eifull.so) reads both planes there.
For each library in LIBS (default: release, eifull) the bf16 step is compared
with the f32 cell (release library) at the headline size B=256, T=64 on the
bench's clips, with the parameters of tests/test_gpu_headline.py (perturbed,
trained), as that test measures; plus the two bf16 builds against each other.
Writes gpurun_out/ei_drift.json."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "pathtracker-models_amd"), os.path.join(REPO, "tests")]

import torch  # noqa: E402

import bench  # noqa: E402
from ptamd import _lib  # noqa: E402
import test_gpu_headline as th  # noqa: E402

B, T = 256, 64


def stats(lo, g, lo32, g32):
    err = (lo - lo32).abs()
    cos = {}
    for k in g32:
        a, b = g[k], g32[k]
        if b.norm() > 1e-12:
            cos[k] = float(a @ b / (a.norm() * b.norm()))
    flips = {n: int(((lo > t) != (lo32 > t)).sum()) for n, t in (("train_0.5", 0.5), ("eval_0", 0.0))}
    return {"logit_max_abs_err": float(err.max()), "logit_mean_abs_err": float(err.mean()),
            "grad_cosine_min": min(cos.values()), "grad_cosine_min_tensor": min(cos, key=cos.get),
            "flips": flips}


def main():
    libs = os.environ.get("LIBS")
    libs = libs.split(",") if libs else [_lib.LIB_PATH, os.path.join(REPO, "pathtracker-models_amd", "ptamd",
                                                                      "ab", "libptcell_eifull.so")]
    dev = torch.device("cuda:0")
    x, y = bench.make_data(1000, B, T, dev)
    out = {}
    for perturb in (True, "trained"):
        tag = "trained" if perturb == "trained" else "perturbed"
        m = th._model(1234, perturb).to(dev)
        lo32, g32 = th._run(m, "f32", x, y)
        res = {}
        for p in libs:
            _lib.DIAG_PATH = p
            with _lib.diag_library():
                res[p] = th._run(m, "bf16", x, y)
        rec = {os.path.basename(p): stats(*res[p], lo32, g32) for p in libs}
        if len(libs) == 2:
            rec["between_builds"] = stats(*res[libs[1]], *res[libs[0]])
        out[tag] = rec
        print(tag, json.dumps(rec, indent=1), flush=True)
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", "ei_drift.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
