#!/usr/bin/env python3
"""bench.py — InT training throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]): InT, 32x32 frames x 64, C=32, k=7,
B=256 clips per GPU, bf16 cell (bf16 operands / saved states, f32 accumulate),
one step = forward over all frames + readout + BCE loss + BPTT backward
[+ one RCCL all-reduce of the flat gradient bucket when N>1] + Adam step.
Synthetic seeded PathTracker clips (ptamd.synth), resident in HBM before the
timed region; random init (no checkpoints offline).

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W]
N>1 is launched by torch.distributed.run (one rank per GPU, RCCL); rank 0
prints ONE JSON line.  value = clips/s of the whole job (all ranks) =
N * B * K / max-over-ranks(time of K steps).  Scaling is weak (B fixed per GPU).

roofline: the dominant kernel (largest summed device time over K further,
instrumented steps, measured with HIP events the library records around its
own launches on the launch stream) against whichever roofline binds it — dense MFMA peak or
HBM bandwidth — using the algorithmic FLOPs / bytes per launch of DESIGN.md §3;
traffic = PMC-measured HBM bytes per launch from profiles/ (or null).
cpu_baseline: the CPU oracle
(oracle/cells.py, plain PyTorch fp32, the reference's own op graph) timed on
this host for a bounded sample (rank 0, N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "pathtracker-models_amd")
for _p in (REPO, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = json.load(open(os.path.join(REPO, "BASELINE.json")))["metric"]
C, HW, K = 32, 32, 7
PEAK_TFLOPS = {"bf16": 2500.0, "f32": 157.3}     # dense MFMA peaks, MI355X_MICROARCH.md
PEAK_HBM_GBS = 8000.0


def conv_flops():          # one k x k C->C conv over one 32x32 clip frame
    return 2 * C * C * K * K * HW * HW


def gate_flops():          # one 1x1 C->C gate conv over one clip frame
    return 2 * C * C * HW * HW


def algorithmic_flops(kind, batch, frames, fused_fwd=False):
    """Algorithmic FLOPs of ALL launches of one kernel kind in one step.

    Counts the model's contractions only (no recompute): forward conv + gates;
    backward data-gradients + 1x1 weight-gradients; the k x k weight gradients
    in k_wgrad.  Sum over kinds = 3 x forward (41.9 GFLOP/clip
    at T=64, minus the stem's 12.6 MFLOP which is counted nowhere)."""
    cf, gf = conv_flops(), gate_flops()
    per_clip = {
        "k_conv_fa": frames * cf,                   # conv(gE, w_inh)
        "k_conv_fb": frames * cf,                   # conv(I, w_exc)
        "k_pw_fa": frames * 4 * gf,                 # a_w, a_u, e_w, e_u
        "k_pw_fb": frames * 2 * gf,                 # i_w, i_u
        "k_conv_bb": frames * cf,                   # conv^T(w_exc)
        "k_conv_ba": (frames - 1) * cf,             # conv^T(w_inh) (frame 0's is dead)
        "k_pw_ba": (frames - 1) * 4 * gf,           # a_* dgrad + wgrad
        "k_pw_bb": frames * 8 * gf,                 # i_*, e_* dgrad + wgrad
        "k_wgrad": frames * 2 * cf,                 # dW_inh + dW_exc
    }
    # fused backward steps = their two halves
    per_clip["k_conv_pw_bb"] = per_clip["k_conv_bb"] + per_clip["k_pw_bb"]
    per_clip["k_conv_pw_ba"] = per_clip["k_conv_ba"] + per_clip["k_pw_ba"]
    # fused forward steps (k_pw_conv_fa / k_pw_conv_fb; k_pw_fa then only closes frame T-1)
    per_clip["k_pw_conv_fa"] = per_clip["k_pw_fa"] + per_clip["k_conv_fa"]
    per_clip["k_pw_conv_fb"] = per_clip["k_pw_fb"] + per_clip["k_conv_fb"]
    if fused_fwd:
        per_clip["k_pw_fa"] = 0
    return per_clip.get(kind, 0) * batch


def algorithmic_bytes(kind, batch, frames, elt, fused_fwd=False, xb=4):
    """Algorithmic HBM bytes of ALL launches of one kernel kind in one step
    (DESIGN.md §3 table): F = one clip-frame state tensor (32x32x32 elements),
    XF = one clip-frame of the input (3x32x32; xb = 4 B f32, 1 B raw u8 clips)."""
    F, XF = C * HW * HW * elt, 3 * HW * HW * xb
    per_clip = {
        "k_pw_fa": frames * (XF + 7 * F),
        "k_conv_fa": frames * 2 * F,
        "k_pw_fb": frames * (XF + 3 * F),
        "k_conv_fb": frames * 2 * F,
        "k_pw_ba": frames * (XF + 11 * F),
        "k_conv_ba": (frames - 1) * 5 * F + 3 * F,
        "k_pw_bb": frames * (XF + 8 * F),
        "k_conv_bb": frames * 6 * F,
        "k_wgrad": frames * 4 * F,
    }
    # fused backward steps: both halves minus the hand-off tensor (dI_t / dgE_t)
    # that the point-wise half re-reads from L2 in the same workgroup
    per_clip["k_conv_pw_bb"] = per_clip["k_conv_bb"] + per_clip["k_pw_bb"] - frames * F
    per_clip["k_conv_pw_ba"] = per_clip["k_conv_ba"] + per_clip["k_pw_ba"] - (frames - 1) * F
    # fused forward steps: the conv takes its input from the prologue's LDS tile
    # (gE_t / I_t still go to HBM for the backward); frame 0 has nothing to
    # close, which the standalone k_pw_fa(T) (reads I, E, eg, ce; writes E) does
    per_clip["k_pw_conv_fa"] = frames * (XF + 8 * F) - 5 * F
    per_clip["k_pw_conv_fb"] = frames * (XF + 4 * F)
    if fused_fwd:
        per_clip["k_pw_fa"] = 5 * F
    return per_clip.get(kind, 0) * batch


def pmc_traffic(kernel, batch, frames, dtype):
    """HBM bytes per launch of `kernel` from the committed PMC summary
    (profiles/*_pmc_traffic.json, written by tools/pmc_traffic.py from
    rocprofv3 FETCH_SIZE / WRITE_SIZE passes of this same workload), or None."""
    import glob
    tag = f"B={batch} T={frames} {dtype}"
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc_traffic.json")), reverse=True):
        d = json.load(open(f))
        if d.get("note") == tag and kernel in d.get("kernels", {}):
            return d["kernels"][kernel]["traffic_bytes"]
    return None


def make_data(seed, batch, frames, device, u8=False):
    """Synthetic clips: the f32 model input [B,3,T,32,32], or (u8) the raw
    clip bytes [B,T,32,32,3] the cell converts while staging each frame."""
    from ptamd import synth
    clips, labels = synth.make_batch(seed, batch, frames)
    x = (torch.from_numpy(clips) if u8 else
         torch.from_numpy(clips.transpose(0, 4, 1, 2, 3).astype(np.float32) / 255.0))
    y = torch.tensor([ord(b) for b in labels], dtype=torch.float32)
    return x.to(device), y.to(device)


def cpu_baseline(seconds, frames=64, batch=4):
    """Oracle (reference op graph, fp32 CPU) fwd+BPTT+Adam on B=4 clips."""
    from oracle import cells
    from ptamd import synth
    torch.manual_seed(0)
    from models import InT as int_mod
    m = int_mod.InT(dimensions=C, timesteps=frames, kernel_size=K)
    sd = {k: v.detach().clone().requires_grad_(k != "unit1.w") for k, v in m.state_dict().items()}
    clips, labels = synth.make_batch(99, batch, frames)
    x = torch.from_numpy(clips.transpose(0, 4, 1, 2, 3) / 255.0).float()
    y = torch.tensor([ord(b) for b in labels], dtype=torch.float32)
    opt = torch.optim.Adam([v for v in sd.values() if v.requires_grad], lr=3e-4)

    def step():
        logits, _, _ = cells.recurrent_forward(sd, x)
        cells.bce_logits(logits, y).backward()
        opt.step()
        opt.zero_grad(set_to_none=True)

    step()                                   # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        step()
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds or n >= 50:
            break
    return {"value": round(batch * n / el, 3), "unit": "clips/s", "cores": torch.get_num_threads(),
            "kind": "port",
            "sample": f"oracle/cells.py InT fwd+BPTT+Adam, B={batch} T={frames} 32x32 fp32, "
                      f"{n} steps in {el:.1f}s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256, help="clips per GPU")
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--input", default="f32", choices=["u8", "f32"],
                    help="cell input: raw u8 clips (converted in-kernel) or the f32 tensor")
    args = ap.parse_args()

    from ptamd import _lib
    from ptamd.dist import GradBucket, env_rank
    from models import InT as int_mod

    rank, local_rank, world = env_rank()
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)

    torch.manual_seed(1234)
    model = int_mod.InT(dimensions=C, timesteps=args.frames, kernel_size=K).to(dev)
    model.cell_dtype = args.dtype
    if world > 1:                       # identical init on every rank
        for p in model.parameters():
            dist.broadcast(p.data, 0)
    bucket = GradBucket(model.parameters(), dev)
    opt = torch.optim.Adam(model.parameters(), lr=3e-4)
    crit = torch.nn.BCEWithLogitsLoss()
    x, y = make_data(1000 + rank, args.batch, args.frames, dev, u8=args.input == "u8")

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
    lib = _lib.load()
    # timed region: no instrumentation (the per-launch HIP events of the
    # kernel-timing pass below add ~1 us of stream work per launch)
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
    # kernel-timing pass (same steps, HIP events around every library launch)
    lib.pt_cell_timing_reset()
    lib.pt_cell_timing_enable((1 << _lib.NKINDS) - 1)
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    lib.pt_cell_timing_enable(0)
    kern = {}
    for kind, name in enumerate(_lib.KIND_NAMES):
        ms, n = _lib.timing_read(kind)
        kern[name] = (ms, n)
    lib.pt_cell_timing_reset()
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())

    if rank == 0:
        value = world * args.batch * args.steps / el
        dom = max(kern, key=lambda k: kern[k][0])
        dom_ms, dom_n = kern[dom]
        avg_ms = dom_ms / max(dom_n, 1)
        elt = 2 if args.dtype == "bf16" else 4
        ffw = kern["k_pw_conv_fa"][1] > 0
        xb = 1 if args.input == "u8" else 4
        flop_launch = algorithmic_flops(dom, args.batch, args.frames, ffw) * args.steps / max(dom_n, 1)
        byte_launch = algorithmic_bytes(dom, args.batch, args.frames, elt, ffw, xb) * args.steps / max(dom_n, 1)
        peak_f = PEAK_TFLOPS[args.dtype]
        # the binding roofline: the larger of the two ideal times
        if flop_launch / (peak_f * 1e12) >= byte_launch / (PEAK_HBM_GBS * 1e9):
            roof = {"bound": "mfma", "achieved": round(flop_launch / (avg_ms * 1e-3) / 1e12, 2),
                    "peak": peak_f, "unit": "TFLOP/s"}
        else:
            roof = {"bound": "hbm", "achieved": round(byte_launch / (avg_ms * 1e-3) / 1e9, 1),
                    "peak": PEAK_HBM_GBS, "unit": "GB/s"}
        roof["frac"] = round(roof["achieved"] / roof["peak"], 4)
        roof.update({"traffic": pmc_traffic(dom, args.batch, args.frames, args.dtype),
                     "kernel": dom, "avg_launch_ms": round(avg_ms, 4), "launches": dom_n,
                     "algorithmic_flop_per_launch": int(flop_launch),
                     "algorithmic_bytes_per_launch": int(byte_launch)})
        # every kernel kind against its own binding roofline (context for the
        # dominant one above): conv / wgrad are MFMA-bound, point-wise HBM-bound
        per_kind = {}
        for k, (ms, n) in kern.items():
            fl = algorithmic_flops(k, args.batch, args.frames, ffw) * args.steps
            by = algorithmic_bytes(k, args.batch, args.frames, elt, ffw, xb) * args.steps
            if n == 0 or ms <= 0 or (fl == 0 and by == 0):
                continue
            sec = ms * 1e-3
            if fl / (peak_f * 1e12) >= by / (PEAK_HBM_GBS * 1e9):
                per_kind[k] = {"bound": "mfma", "achieved_tflops": round(fl / sec / 1e12, 1),
                               "frac": round(fl / sec / 1e12 / peak_f, 3)}
            else:
                per_kind[k] = {"bound": "hbm", "achieved_gbs": round(by / sec / 1e9, 1),
                               "frac": round(by / sec / 1e9 / PEAK_HBM_GBS, 3)}
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "clips/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic",
            "config": {"workload": f"InT 32x32x{args.frames}f fwd+BPTT+Adam, "
                                   f"{args.batch} clips/GPU, {args.dtype} cell, {args.input} input",
                       "batch_per_gpu": args.batch, "global_batch": args.batch * world,
                       "frames": args.frames, "channels": C, "kernel": K, "input": args.input,
                       "parallelism": f"dp{world}"},
            "roofline": roof,
            "roofline_per_kernel": per_kind,
            "kernels_ms_per_step": {k: round(v[0] / args.steps, 3) for k, v in kern.items()},
            "loss": round(float(loss.item()), 5),
        }
        if not np.isfinite(line["loss"]):
            print("bench.py: WARNING non-finite training loss", file=sys.stderr, flush=True)
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args.cpu_seconds, frames=args.frames)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
