#!/usr/bin/env python3
"""ConvLSTM training throughput on MI355X (BASELINE.json configs[2], cfg3).

Workload: the reference ConvLSTM (models/convlstm.py) at its defaults —
timesteps=8, filt_size=15, 25 channels — on 32x32 single-channel images,
B images per GPU, one step = conv0 + pow + 8 recurrent steps + BN + conv6 +
CrossEntropy + the training-mode Jacobian penalty + BPTT backward + Adam.
The reference form is a static image recurred `timesteps` times (there is no
video form of this model in the reference); the synthetic images are frame 0
of the PathTracker clips (channel mean), targets the per-pixel target-marker
mask.  Prints one JSON line (not the headline metric: bench.py is).

FLOP model (algorithmic, 25 real channels, the reference's op graph minus the
x-conv recomputation it does every step): forward = 4 Wx convs once +
4 Wh convs x (T-1) (h_0 = 0); backward = 2 x forward (data + weight grads);
Jacobian penalty = 2 conv^T of one step.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "pathtracker-models_amd")
for _p in (REPO, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

PEAK_TFLOPS = {"bf16": 2500.0, "f32": 157.3}


def conv_flops(k, c=25, hw=32):
    return 2 * 4 * c * c * k * k * hw * hw          # the 4 gate convs of one family


def flops_per_image(k, t):
    fwd = conv_flops(k) * (1 + (t - 1))
    return 3 * fwd + 2 * conv_flops(k)     # + jv: two conv^T (4 gates in) of one step


def make_images(batch, seed=0):
    from ptamd import synth
    clips, _ = synth.make_batch(seed, batch, 1)
    img = clips[:, 0].astype(np.float32).mean(-1, keepdims=True) / 255.0     # [B,32,32,1]
    img = torch.from_numpy(img.transpose(0, 3, 1, 2).copy())
    tgt = torch.from_numpy((clips[:, 0, :, :, 2] > 127).astype(np.int64))
    return img, tgt


def cpu_baseline(seconds, k, t, batch=2):
    from oracle import cells
    torch.manual_seed(0)
    from models import convlstm as cl
    m = cl.ConvLSTM(timesteps=t, filt_size=k)
    sd = {n: p.detach().clone().requires_grad_() for n, p in m.named_parameters()}
    img, tgt = make_images(batch, 5)
    opt = torch.optim.Adam(list(sd.values()), lr=3e-4)

    def step():
        out, _, _, _ = cells.convlstm_forward(sd, img, t, with_jv=True)
        torch.nn.functional.cross_entropy(out, tgt).backward()
        opt.step()
        opt.zero_grad(set_to_none=True)

    step()
    n, t0 = 0, time.perf_counter()
    while True:
        step()
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds or n >= 50:
            break
    return {"value": round(batch * n / el, 3), "unit": "images/s", "cores": torch.get_num_threads(),
            "kind": "port",
            "sample": f"oracle/cells.py ConvLSTM fwd+jv+BPTT+Adam, B={batch} T={t} k={k} "
                      f"32x32 fp32, {n} steps in {el:.1f}s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--timesteps", type=int, default=8)
    ap.add_argument("--filt", type=int, default=15)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()
    from models import convlstm as cl

    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    m = cl.ConvLSTM(timesteps=args.timesteps, filt_size=args.filt).to(dev).train()
    m.cell_dtype = args.dtype
    opt = torch.optim.Adam(m.parameters(), lr=3e-4)
    crit = torch.nn.CrossEntropyLoss()
    img, tgt = make_images(args.batch)
    img, tgt = img.to(dev), tgt.to(dev)

    def step():
        out, jv, loss = m(img, 0, 0, tgt, crit)
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
        return loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    value = args.batch * args.steps / el
    fl = flops_per_image(args.filt, args.timesteps) * value
    line = {"metric": "images/sec/GPU fwd+BPTT+jv, ConvLSTM 32x32 static image (cfg3)",
            "value": round(value, 2), "unit": "images/s", "n_gpus": 1, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3),
            "higher_is_better": True, "dtype": args.dtype, "data": "synthetic",
            "config": {"workload": f"ConvLSTM timesteps={args.timesteps} filt_size={args.filt} "
                                   f"25ch, {args.batch} images/GPU, {args.dtype} cell"},
            "step_tflops": round(fl / 1e12, 2),
            "step_frac_of_mfma_peak": round(fl / 1e12 / PEAK_TFLOPS[args.dtype], 4),
            "loss": round(float(loss.item()), 5)}
    if not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(args.cpu_seconds, args.filt, args.timesteps)
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
