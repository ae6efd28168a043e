#!/usr/bin/env python3
"""Comparison baselines on MI355X (BASELINE.json configs[4]; SURVEY.md §8(f)
item 4): the kys ConvGRU ('gru': 64 channels, k=7, three 128->64 convs per
frame) and the stride-free R3D-18 ('nostride_video_cc_small': 17 Conv3d of
32 channels over the whole clip) on the same 32x32x64-frame clips, trained
with the same step as bench.py (forward + BCE + backward + Adam), stock
PyTorch-ROCm (MIOpen convolutions, bf16 autocast, channels-last).  The
reference's resnet_TSM and transformer baselines need un-vendored packages
(spatial_correlation_sampler, timesformer/performer/lambda) and are not built.

Prints one JSON line per model: clips/s, ms/step, algorithmic model TFLOP/s.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "pathtracker-models_amd")]

import torch  # noqa: E402

import bench  # noqa: E402


def flops_per_clip(name, frames, hw=32):
    px = hw * hw
    if name == "gru":                       # 3 convs (64+64)->64, 7x7, per frame; x3 for fwd+bwd
        return 3 * frames * 3 * 2 * 128 * 64 * 49 * px
    # stem 3->32 (3x7x7) + 16 convs 32->32 (3x3x3), every voxel; x3 for fwd+bwd
    return 3 * frames * px * (2 * 3 * 32 * 147 + 16 * 2 * 32 * 32 * 27)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="gru,nostride_video_cc_small")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    args = ap.parse_args()
    from types import SimpleNamespace
    from utils import engine
    dev = torch.device("cuda:0")
    torch.backends.cudnn.benchmark = True
    x, y = bench.make_data(1000, args.batch, args.frames, dev)
    for name in args.models.split(","):
        torch.manual_seed(0)
        model = engine.model_selector(SimpleNamespace(model=name, pretrained=False),
                                      timesteps=args.frames, device=dev).to(dev)
        opt = torch.optim.Adam(model.parameters(), lr=3e-4)
        crit = torch.nn.BCEWithLogitsLoss()
        xin = x.contiguous(memory_format=torch.channels_last_3d) if name != "gru" else x

        def step():
            with torch.autocast("cuda", dtype=torch.bfloat16):
                out, _ = model(xin)
                loss = crit(out.float(), y.reshape(-1, 1))
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
        f = flops_per_clip(name, args.frames) * args.batch * args.steps
        print(json.dumps({
            "metric": f"clips/sec/GPU fwd+BPTT, 32x32x{args.frames}f, comparison baseline '{name}'",
            "value": round(args.batch * args.steps / el, 2), "unit": "clips/s",
            "ms_per_step": round(el / args.steps * 1e3, 2), "batch": args.batch,
            "dtype": "bf16 autocast", "model_tflops": round(f / el / 1e12, 1),
            "loss": round(float(loss.item()), 5), "data": "synthetic"}), flush=True)
        del model, opt
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
