#!/usr/bin/env python3
"""A/B timing of ConvLSTM library BUILDS in one process (the cfg3 clip step:
ConvLSTMVideo k=7, 32x32x64f, B=256, bf16, fwd + BPTT + jv + Adam).  Every
library in LIBS (comma-separated; default: the release libptlstm.so and the
A/B builds under ptamd/ab/libptlstm_*.so) is routed to through
ptamd.lstm.diag_library() in turn, interleaved round by round (one box, one
process: cdna_hip_programming.md §5.4 rule 24); median ms per step."""
import glob
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "pathtracker-models_amd"), os.path.join(REPO, "tools")]

import torch  # noqa: E402

from ptamd import lstm  # noqa: E402
from models import convlstm as cl  # noqa: E402
from bench_convlstm import make_clips  # noqa: E402


def main():
    b = int(os.environ.get("B", 256))
    t = int(os.environ.get("T", 64))
    rounds = int(os.environ.get("ROUNDS", 5))
    steps = int(os.environ.get("STEPS", 4))
    libs = os.environ.get("LIBS")
    libs = libs.split(",") if libs else [lstm.LIB_PATH] + sorted(
        glob.glob(os.path.join(REPO, "pathtracker-models_amd", "ptamd", "ab", "libptlstm_*.so")))
    dev = torch.device("cuda:0")
    torch.manual_seed(1234)
    m = cl.ConvLSTMVideo(dimensions=25, timesteps=t, kernel_size=7).to(dev).train()
    m.cell_dtype = "bf16"
    opt = torch.optim.Adam(m.parameters(), lr=3e-4)
    crit = torch.nn.BCEWithLogitsLoss()
    x, y = make_clips(b, t, seed=1000)
    x, y = x.to(dev), y.to(dev).reshape(-1, 1)

    def step():
        out, _ = m(x)
        crit(out, y).backward()
        opt.step()
        opt.zero_grad(set_to_none=True)

    res = {p: [] for p in libs}
    for r in range(rounds + 1):
        for p in libs:
            lstm.DIAG_PATH = p
            with lstm.diag_library():
                step()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(steps):
                    step()
                torch.cuda.synchronize()
                if r:
                    res[p].append((time.perf_counter() - t0) / steps * 1e3)
        print(f"round {r}", flush=True)
    med = lambda v: sorted(v)[len(v) // 2]
    print(f"ms per step (B={b} T={t} bf16 k=7), median of {rounds} rounds x {steps} steps")
    for p in libs:
        print(f"{os.path.basename(p):36s} {med(res[p]):8.3f}   {b / med(res[p]) * 1e3:8.1f} clips/s   "
              + " ".join(f"{v:.2f}" for v in res[p]))


if __name__ == "__main__":
    main()
