#!/usr/bin/env python3
"""Per-workgroup phase timeline of one frame's launches (pt_cell_trace):
forward + backward at B, T (default 256, 64) with frame FRAME traced; prints
per kernel the launch span and, per phase, the median / max time since the
workgroup's first stamp (100 MHz counter: 10 ns ticks).  Diagnostics only."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "pathtracker-models_amd")]
import torch  # noqa: E402

from ptamd import _lib  # noqa: E402
_lib.use_diag()         # the PT_DIAG build (libptcell_diag.so) honours the switches
from models import InT  # noqa: E402

SLOTS = {"k_pw_bb": ["entry", "issued", "prologue", "rows", "bn_partial", "flush", "publish"],
         "k_pw_ba": ["entry", "-", "prologue", "rows", "bn_partial", "flush", "publish"],
         "k_fused_fa": ["entry", "-", "prologue", "pw_rows", "conv", "bn_stats", "bn_publish"],
         "k_fused_fb": ["entry", "-", "prologue", "pw_rows", "conv", "bn_stats", "bn_publish"]}


def main():
    b, t, fr = int(os.environ.get("B", 256)), int(os.environ.get("T", 64)), int(os.environ.get("FRAME", 30))
    dev = torch.device("cuda:0")
    lib = _lib.load()
    torch.manual_seed(0)
    m = InT.InT(dimensions=32, timesteps=t, kernel_size=7).to(dev)
    m.cell_dtype = "bf16"
    x = torch.rand(b, 3, t, 32, 32, device=dev)
    for _ in range(2):                       # warm-up, then the traced pass
        buf = torch.zeros(_lib.NKINDS * 256 * 16, dtype=torch.int64, device=dev)
        lib.pt_cell_trace(ctypes.c_void_p(buf.data_ptr()), fr)
        out, _ = m(x)
        out.sum().backward()
        torch.cuda.synchronize()
        lib.pt_cell_trace(None, -1)
    tr = buf.view(_lib.NKINDS, 256, 16).cpu()
    for k, names in SLOTS.items():
        r = tr[_lib.KIND_NAMES.index(k)]
        ok = r[:, 0] > 0
        if not ok.any():
            continue
        r = r[ok].double()
        t0 = r[:, 0].min()
        print(f"{k}: {int(ok.sum())} workgroups, first entry -> last end {(r[:, 6].max() - t0) / 100:.1f} us, "
              f"entries spread {(r[:, 0].max() - t0) / 100:.1f} us")
        for j, nm in enumerate(names):
            if nm == "-" or j == 0:
                continue
            d = (r[:, j] - r[:, 0]) / 100
            d = d[r[:, j] > 0]
            if len(d):
                print(f"   {nm:11s} since entry: median {d.median():7.2f}  max {d.max():7.2f} us")


if __name__ == "__main__":
    main()
