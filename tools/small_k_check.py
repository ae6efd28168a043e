#!/usr/bin/env python3
"""r06: the banded backward convs at k < 7 against the whole-clip conv on the
diagnostic library LIB (default: the in-tree build): max |diff| of the logits
and per-parameter gradients, k = 7, 5, 3, 1 (InT, B=24, T=6, bf16).  Shows
the pre-load schedule bug of the r05-r06 banded convs (rows whose addend
pre-load fell before the last column's first step) and its fix."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "pathtracker-models_amd"), os.path.join(REPO, "tests")]

import torch  # noqa: E402

from ptamd import _lib  # noqa: E402
if os.environ.get("LIB"):
    _lib.DIAG_PATH = os.environ["LIB"]
import test_gpu_fused as tf  # noqa: E402
from models import InT  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    for k in (7, 5, 3, 1):
        torch.manual_seed(k + 11)
        m = InT.InT(dimensions=32, timesteps=6, kernel_size=k).to(dev)
        m.cell_dtype = "bf16"
        x = torch.rand(24, 3, 6, 32, 32, device=dev)
        y = (torch.arange(24, device=dev) % 2).float()
        o1, _, _, g1 = tf._run(m, x, y, fused=True)
        o0, _, _, g0 = tf._run(m, x, y, fused=True, band=0, cpa=0)
        worst = max(((g1[n] - g0[n]).abs().max() / g0[n].abs().max().clamp_min(1e-30)).item()
                    for n in g0 if n.startswith("unit1."))
        print(f"k={k}: logits max|diff| {(o1 - o0).abs().max().item():.3e}, "
              f"worst gradient rel diff {worst:.3e}", flush=True)


if __name__ == "__main__":
    main()
