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

--video: the clip form (models/convlstm.py ConvLSTMVideo) on
the headline's 32x32x64-frame PathTracker clips, B clips per GPU, k = 7 (the
engine's fb_kernel_size), 25 channels: stem + 64 recurrent steps with a new
frame each + readout + BCE + the Jacobian penalty + BPTT + Adam -> clips/s.
FLOP model: per frame 4 Wx + 4 Wh convs (frame 0: no Wh, h_0 = 0), x 3 for
the backward, + the penalty's 2 conv^T.
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


def video_flops_per_clip(k, t):
    fwd = conv_flops(k) * (t + (t - 1))
    return 3 * fwd + 2 * conv_flops(k)


def make_clips(batch, frames, seed=0):
    from ptamd import synth
    clips, labels = synth.make_batch(seed, batch, frames)
    x = torch.from_numpy(clips.transpose(0, 4, 1, 2, 3).astype(np.float32) / 255.0)
    return x, torch.tensor([ord(v) for v in labels], dtype=torch.float32)


def cpu_baseline_video(seconds, k, t, batch=2):
    from oracle import cells
    from models import convlstm as cl
    torch.manual_seed(0)
    m = cl.ConvLSTMVideo(dimensions=25, timesteps=t, kernel_size=k)
    sd = {n: p.detach().clone().requires_grad_() for n, p in m.named_parameters()}
    x, y = make_clips(batch, t, seed=3)
    opt = torch.optim.Adam(list(sd.values()), lr=3e-4)

    def step():
        lo, _, hs, cs = cells.convlstm_video_forward(sd, x)
        cells.convlstm_jv_penalty(hs, cs)
        torch.nn.functional.binary_cross_entropy_with_logits(lo, y.reshape(-1, 1)).backward()
        opt.step()
        opt.zero_grad(set_to_none=True)

    t0 = time.perf_counter()
    step()
    n, el = 1, time.perf_counter() - t0
    while el < seconds and n < 20:
        step()
        n += 1
        el = time.perf_counter() - t0
    return {"value": round(batch * n / el, 4), "unit": "clips/s", "cores": torch.get_num_threads(),
            "kind": "port",
            "sample": f"oracle/cells.py convlstm_video_forward fwd+jv+BPTT+Adam, B={batch} T={t} "
                      f"k={k} fp32, {n} steps in {el:.1f}s"}


def main_video(args):
    from models import convlstm as cl
    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    m = cl.ConvLSTMVideo(dimensions=25, timesteps=args.frames, kernel_size=args.filt).to(dev).train()
    m.cell_dtype = args.dtype
    opt = torch.optim.Adam(m.parameters(), lr=3e-4)
    crit = torch.nn.BCEWithLogitsLoss()
    x, y = make_clips(args.batch, args.frames, seed=1000)
    if args.input == "u8":       # the same clips as raw bytes [B,T,H,W,3]
        x = (x * 255.0).round().to(torch.uint8).permute(0, 2, 3, 4, 1).contiguous()
    x, y = x.to(dev), y.to(dev).reshape(-1, 1)

    def step():
        out, _ = m(x)
        loss = crit(out, y)
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
    fl = video_flops_per_clip(args.filt, args.frames) * value
    line = {"metric": "clips/sec/GPU fwd+BPTT+jv, ConvLSTM on 32x32x64f PathTracker clips (cfg3)",
            "value": round(value, 2), "unit": "clips/s", "n_gpus": 1, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3),
            "higher_is_better": True, "dtype": args.dtype, "data": "synthetic",
            "config": {"workload": f"ConvLSTMVideo 32x32x{args.frames}f k={args.filt} 25ch, "
                                   f"{args.batch} clips/GPU, {args.dtype} cell, {args.input} input"},
            "step_tflops": round(fl / 1e12, 2),
            "step_frac_of_mfma_peak": round(fl / 1e12 / PEAK_TFLOPS[args.dtype], 4),
            "loss": round(float(loss.item()), 5)}
    if not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline_video(args.cpu_seconds, args.filt, args.frames)
    print(json.dumps(line), flush=True)


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
    ap.add_argument("--video", action="store_true", help="cfg3 on the 32x32x64f clips")
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--input", default="f32", choices=["f32", "u8"],
                    help="--video: the f32 model input, or the raw u8 clips the TFRecords hold")
    args = ap.parse_args()
    if args.video:
        if args.filt == 15 and "--filt" not in sys.argv:
            args.filt = 7
        return main_video(args)
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
