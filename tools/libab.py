#!/usr/bin/env python3
"""A/B timing of cell-library BUILDS in one process: every library file in
LIBS (comma-separated paths; default: the release library and the A/B builds
under ptamd/ab/) is opened beside the others (ptamd._lib.diag_library routes
the model's calls to it) and runs the same forward + backward, interleaved
round by round (cdna_hip_programming.md §5.4 rule 24: compare on one box, in
one process); per-kind average launch times from each library's own launch
events (pt_cell_timing_*) and the summed device ms per step, medians over the
rounds.  B, T, DT as tools/ablate.py; CELL=hgru with HW=64 runs cfg4's FFhGRU
on 64x64 frames (tiled)."""
import glob
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "pathtracker-models_amd")]

import torch  # noqa: E402

from ptamd import _lib  # noqa: E402
from models import InT as int_mod, ffhgru_hierarchy as hg  # noqa: E402


def main():
    b = int(os.environ.get("B", 256))
    t = int(os.environ.get("T", 64))
    dtype = os.environ.get("DT", "bf16")
    rounds = int(os.environ.get("ROUNDS", 3))
    libs = os.environ.get("LIBS")
    libs = libs.split(",") if libs else [_lib.LIB_PATH] + sorted(
        glob.glob(os.path.join(REPO, "pathtracker-models_amd", "ptamd", "ab", "*.so")))
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    hw = int(os.environ.get("HW", 32))
    if os.environ.get("CELL", "int") == "hgru":
        m = hg.FFhGRU(dimensions=32, timesteps=t, kernel_size=7).to(dev)
    else:
        m = int_mod.InT(dimensions=32, timesteps=t, kernel_size=7).to(dev)
    m.cell_dtype = dtype
    x = torch.rand(b, 3, t, hw, hw, device=dev)
    kinds = [k for k in _lib.KIND_NAMES if k not in ("k_prep", "k_reduce")]
    res = {p: {k: [] for k in kinds} for p in libs}
    tot = {p: [] for p in libs}
    for r in range(rounds + 1):
        for p in libs:
            _lib.DIAG_PATH = p
            with _lib.diag_library() as lib:
                torch.cuda.synchronize()
                lib.pt_cell_timing_reset()
                lib.pt_cell_timing_enable((1 << _lib.NKINDS) - 1)
                out, _ = m(x)
                out.sum().backward()
                torch.cuda.synchronize()
                lib.pt_cell_timing_enable(0)
                if r == 0:
                    continue
                s = 0.0
                for name in _lib.KIND_NAMES:
                    ms, n = _lib.timing_read(_lib.KIND_NAMES.index(name))
                    if n and name in kinds:
                        res[p][name].append(1e3 * ms / n)
                    s += ms
                tot[p].append(s)
    med = lambda v: sorted(v)[len(v) // 2] if v else float("nan")
    print(f"avg launch us (B={b} T={t} {dtype}), median of {rounds} rounds")
    print(f"{'library':28s}" + "".join(f"{k[2:]:>10}" for k in kinds) + "   step ms")
    for p in libs:
        print(f"{os.path.basename(p)[:28]:28s}" + "".join(
            f"{med(res[p][k]):10.1f}" if res[p][k] else " " * 10 for k in kinds) + f"  {med(tot[p]):8.3f}")


if __name__ == "__main__":
    main()
