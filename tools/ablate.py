#!/usr/bin/env python3
"""Kernel-phase ablation timing (timing experiments only; outputs are garbage
under ablation).  PT_CELL_ABLATE bits: 1 skip conv MFMA loop, 2 skip conv tile
fill, 4 skip per-row element-wise loops.  Masks are interleaved in one process
(cdna_hip_programming.md §5.4 rule 24).  A mask may carry variant switches,
e.g. MASKS="0:PT_CELL_BB_RPP=1,0:PT_CELL_BB_RPP=8" (env NAME=VALUE pairs after
':' separated by '+'), interleaved the same way."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "pathtracker-models_amd")]

import torch  # noqa: E402

from ptamd import _lib  # noqa: E402
_lib.use_diag()         # the PT_DIAG build (libptcell_diag.so) honours the switches
from models import InT as int_mod  # noqa: E402


def main():
    b = int(os.environ.get("B", 256))
    t = int(os.environ.get("T", 64))
    dtype = os.environ.get("DT", "bf16")
    masks = os.environ.get("MASKS", "0,1,2,3,4,7").split(",")
    rounds = int(os.environ.get("ROUNDS", 3))
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    m = int_mod.InT(dimensions=32, timesteps=t, kernel_size=7).to(dev)
    m.cell_dtype = dtype
    x = torch.rand(b, 3, t, 32, 32, device=dev)
    lib = _lib.load()
    kinds = [k for k in _lib.KIND_NAMES if k not in ("k_prep", "k_reduce")]
    res = {mk: {k: [] for k in kinds} for mk in masks}
    tot = {mk: {"fwd": [], "bwd": [], "all": []} for mk in masks}     # summed device ms per step
    fwd_kinds = {"k_pw_fa", "k_conv_fa", "k_pw_fb", "k_conv_fb", "k_fused_fa", "k_fused_fb", "k_persist_fwd"}
    for r in range(rounds + 1):
        for mk in masks:
            bits, _, env = mk.partition(":")
            os.environ["PT_CELL_ABLATE"] = bits
            extra = dict(kv.split("=", 1) for kv in env.split("+") if kv)
            os.environ.update(extra)
            torch.cuda.synchronize()
            lib.pt_cell_timing_reset()
            lib.pt_cell_timing_enable((1 << _lib.NKINDS) - 1)
            out, _ = m(x)
            out.sum().backward()
            torch.cuda.synchronize()
            lib.pt_cell_timing_enable(0)
            for k in extra:
                os.environ.pop(k)
            if r == 0:
                continue
            sums = {"fwd": 0.0, "bwd": 0.0, "all": 0.0}
            for name in _lib.KIND_NAMES:
                ms, n = _lib.timing_read(_lib.KIND_NAMES.index(name))
                if n and name in kinds:
                    res[mk][name].append(1e3 * ms / n)
                sums["all"] += ms
                sums["fwd" if name in fwd_kinds else "bwd"] += ms
            for k, v in sums.items():
                tot[mk][k].append(v)
    os.environ.pop("PT_CELL_ABLATE")
    print(f"avg launch us (B={b} T={t} {dtype}), median of {rounds} rounds")
    print("mask  " + "  ".join(f"{k[2:]:>8}" for k in kinds))
    for mk in masks:
        row = []
        for k in kinds:
            v = sorted(res[mk][k])
            row.append(f"{v[len(v) // 2]:8.1f}" if v else " " * 8)
        print(f"{mk:>4}  " + "  ".join(row))
    print("summed device ms per step (median): " + "; ".join(
        f"{mk}: fwd {sorted(tot[mk]['fwd'])[len(tot[mk]['fwd']) // 2]:.3f} "
        f"bwd {sorted(tot[mk]['bwd'])[len(tot[mk]['bwd']) // 2]:.3f} "
        f"all {sorted(tot[mk]['all'])[len(tot[mk]['all']) // 2]:.3f}" for mk in masks))


if __name__ == "__main__":
    main()
