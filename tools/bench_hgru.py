#!/usr/bin/env python3
"""hGRU long-range training throughput on MI355X (BASELINE.json configs[3], cfg4).

Workload: FFhGRU (models/ffhgru_hierarchy.py:176-276, drop-in
models/ffhgru_hierarchy.py here) on 64x64-pixel x 128-frame PathTracker clips,
C=32, k=7, B clips per GPU (default 128: global batch 1024 over the 8 GPUs of a
node), bf16 cell.  One step = forward over all frames + readout + BCE + BPTT +
[one RCCL all-reduce of the flat gradient bucket when N>1] + Adam — the same
step as bench.py.  The 64x64 frames run as 2x2 tiles of 32x32 (halo rows /
columns read from the neighbouring tiles by the conv kernels),
so the kernels see 4B "tile clips" of bench.py's shape.

Usage:  python tools/bench_hgru.py [--gpus N] [--steps K] [--warmup W]
        (N>1: one rank per GPU over RCCL; started by torch.distributed.run, or
        launched by this script itself as bench.py does).
Prints one JSON line; not the headline metric (bench.py is).
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
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402  (algorithmic FLOP / byte model per 32x32 tile-frame)


def make_data(seed, batch, frames, hw, device):
    from ptamd import synth
    clips, labels = synth.make_batch(seed, batch, frames, h=hw, w=hw)
    x = torch.from_numpy(clips.transpose(0, 4, 1, 2, 3).astype(np.float32) / 255.0)
    y = torch.tensor([ord(b) for b in labels], dtype=torch.float32)
    return x.to(device), y.to(device)


def cpu_baseline(seconds, frames, hw, batch=1):
    """Oracle (reference op graph, fp32 CPU) hGRU fwd+BPTT+Adam on one clip."""
    from oracle import cells
    from models import ffhgru_hierarchy as hg
    torch.manual_seed(0)
    m = hg.FFhGRU(dimensions=32, timesteps=frames, kernel_size=7)
    sd = {k: v.detach().clone().requires_grad_() for k, v in m.state_dict().items()}
    x, y = make_data(99, batch, frames, hw, "cpu")
    opt = torch.optim.Adam(list(sd.values()), lr=3e-4)

    def step():
        logits, _, _ = cells.recurrent_forward(sd, x, hgru=True)
        cells.bce_logits(logits, y).backward()
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
            "sample": f"oracle/cells.py FFhGRU fwd+BPTT+Adam, B={batch} T={frames} {hw}x{hw} fp32, "
                      f"{n} steps in {el:.1f}s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=128, help="clips per GPU")
    ap.add_argument("--frames", type=int, default=128)
    ap.add_argument("--hw", type=int, default=64)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    rc = bench.launch_ranks(sys.argv[1:], args.gpus, script=__file__)
    if rc is not None:
        sys.exit(rc)
    from ptamd import _lib
    from ptamd.dist import GradBucket, env_rank
    from models import ffhgru_hierarchy as hg

    rank, local_rank, world = env_rank()
    if world != args.gpus:
        sys.exit(f"bench_hgru.py: --gpus {args.gpus} but the launcher started {world} rank(s)")
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        assert dist.get_world_size() == args.gpus
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    torch.manual_seed(1234)
    model = hg.FFhGRU(dimensions=32, timesteps=args.frames, kernel_size=7).to(dev)
    model.cell_dtype = args.dtype
    if world > 1:
        for p in model.parameters():
            dist.broadcast(p.data, 0)
    bucket = GradBucket(model.parameters(), dev)
    opt = torch.optim.Adam(model.parameters(), lr=3e-4)
    crit = torch.nn.BCEWithLogitsLoss()
    x, y = make_data(2000 + rank, args.batch, args.frames, args.hw, dev)

    def step():
        out, _ = model(x)
        loss = crit(out, y.reshape(-1, 1))
        loss.backward()
        bucket.allreduce_mean()
        opt.step()
        opt.zero_grad(set_to_none=True)
        return loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    lib = _lib.load()
    lib.pt_cell_timing_reset()
    lib.pt_cell_timing_enable((1 << _lib.NKINDS) - 1)
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    lib.pt_cell_timing_enable(0)
    kern = {name: _lib.timing_read(kind) for kind, name in enumerate(_lib.KIND_NAMES)}
    lib.pt_cell_timing_reset()
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    if rank == 0:
        tiles = args.batch * (args.hw // 32) ** 2
        elt = 2 if args.dtype == "bf16" else 4
        flops = sum(bench.algorithmic_flops(k, tiles, args.frames) for k in kern)
        dom = max(kern, key=lambda k: kern[k][0])
        dom_ms, dom_n = kern[dom]
        avg_ms = dom_ms / max(dom_n, 1)
        f_l = bench.algorithmic_flops(dom, tiles, args.frames) * args.steps / max(dom_n, 1)
        b_l = bench.algorithmic_bytes(dom, tiles, args.frames, elt) * args.steps / max(dom_n, 1)
        peak_f = bench.PEAK_TFLOPS[args.dtype]
        if f_l / (peak_f * 1e12) >= b_l / (bench.PEAK_HBM_GBS * 1e9):
            roof = {"bound": "mfma", "achieved": round(f_l / (avg_ms * 1e-3) / 1e12, 2),
                    "peak": peak_f, "unit": "TFLOP/s"}
        else:
            roof = {"bound": "hbm", "achieved": round(b_l / (avg_ms * 1e-3) / 1e9, 1),
                    "peak": bench.PEAK_HBM_GBS, "unit": "GB/s"}
        roof["frac"] = round(roof["achieved"] / roof["peak"], 4)
        roof.update({"kernel": dom, "avg_launch_ms": round(avg_ms, 4), "launches": dom_n})
        line = {
            "metric": "clips/sec/GPU fwd+BPTT, hGRU 64x64x128f long-range (cfg4)",
            "value": round(world * args.batch * args.steps / el, 2),
            "unit": "clips/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.dtype, "data": "synthetic",
            "config": {"workload": f"FFhGRU {args.hw}x{args.hw}x{args.frames}f fwd+BPTT+Adam, "
                                   f"{args.batch} clips/GPU, {args.dtype} cell",
                       "batch_per_gpu": args.batch, "global_batch": args.batch * world,
                       "parallelism": f"dp{world}"},
            "model_tflops_per_gpu": round(flops * args.steps / el / 1e12, 1),
            "roofline": roof,
            "kernels_ms_per_step": {k: round(v[0] / args.steps, 3) for k, v in kern.items()},
            "loss": round(float(loss.item()), 5),
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args.cpu_seconds, args.frames, args.hw)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
