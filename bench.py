#!/usr/bin/env python3
"""bench.py — InT training throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]): InT, 32x32 frames x 64, C=32, k=7,
B=256 clips per GPU, bf16 cell (bf16 operands / saved states, f32 accumulate),
one step = forward over all frames + readout + BCE loss + BPTT backward
[+ one RCCL all-reduce of the flat gradient bucket when N>1] + Adam step.
Synthetic seeded PathTracker clips (ptamd.synth), resident in HBM before the
timed region; random init (no checkpoints offline).

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W]
N>1: one rank per GPU over RCCL.  Under torch.distributed.run the ranks come
from the environment (WORLD_SIZE must equal N); run directly, bench.py starts
torch.distributed.run itself as a child process before touching the GPU.  Rank
0 prints ONE JSON line.  value = clips/s of the whole job (all ranks) =
N * B * K / max-over-ranks(time of K steps).  Scaling is weak (B fixed per GPU).
allreduce_ms_per_step: device time of the gradient all-reduce left after
backward (the exposed part: by default the cell's early gradients -- all but
the two k x k weights -- are averaged on a side stream under the k x k
weight-gradient kernel; --no-grad-overlap averages everything here).

roofline: the dominant kernel (largest summed device time over K further,
instrumented steps, measured with HIP events the library records around its
own launches on the launch stream) against the roofline SURVEY.md §8(d) binds
it to: MFMA for every kernel with a k x k conv (§8(d) FLOPs per launch / launch
time / dense bf16 peak), HBM for the point-wise-only kernels (DESIGN.md §3
bytes); mfma_frac and hbm_frac_design_bytes (the design's own byte count, a
secondary figure) for every kernel; traffic = PMC-measured HBM bytes per launch
from profiles/ (or null).  step_vs_8d: the whole step's §8(d) FLOPs against the
MFMA peak (step_mfma_frac) and its PMC-measured bytes against §8(d)'s minimum
(step_traffic_vs_8d).
cpu_baseline: the CPU oracle
(oracle/cells.py, plain PyTorch fp32, the reference's own op graph) timed on
this host for a bounded sample (rank 0, N=1 only): B=4 clips of the workload's
64 frames, and (cpu_baseline_cfg1) BASELINE configs[0]'s B=4 x 32 frames.
f32_cell: the same step with the f32 cell (the reference's arithmetic and the
parity path) at the same size, a precision-matched figure beside the bf16 value.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
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


def algorithmic_flops(kind, batch, frames, fused=False, cpa=False):
    """Algorithmic FLOPs of ALL launches of one kernel kind in one step.

    Counts the model's contractions only (no recompute): forward conv + gates;
    backward data-gradients + 1x1 weight-gradients; the k x k weight gradients
    in k_wgrad.  Sum over kinds = 3 x forward (41.9 GFLOP/clip
    at T=64, minus the stem's 12.6 MFLOP which is counted nowhere).  fused: the
    forward runs as k_fused_fa / k_fused_fb (point-wise + conv per launch) and
    one k_pw_fa that only closes the last frame.  cpa (r06): k_conv_ba(t) and
    k_pw_ba(t-1) run as one k_conv_pw_ba launch for t = T-1 .. 1; k_pw_ba
    keeps the first (head only) and last (frame 0's tail: no attention gates
    for InT, gE_0 = 0) launches."""
    cf, gf = conv_flops(), gate_flops()
    if cpa and kind in ("k_conv_pw_ba", "k_conv_ba", "k_pw_ba"):
        return {"k_conv_pw_ba": (frames - 1) * (cf + 4 * gf)}.get(kind, 0) * batch
    if fused:
        fwd = {"k_fused_fa": frames * (cf + 4 * gf), "k_fused_fb": frames * (cf + 2 * gf)}
        if kind in fwd or kind in ("k_pw_fa", "k_pw_fb", "k_conv_fa", "k_conv_fb"):
            return fwd.get(kind, 0) * batch
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
    return per_clip.get(kind, 0) * batch


def algorithmic_bytes(kind, batch, frames, elt, xb=4, fused=False, cpa=False):
    """Algorithmic HBM bytes of ALL launches of one kernel kind in one step
    (DESIGN.md §3 table): F = one clip-frame state tensor (32x32x32 elements),
    XF = one clip-frame of the input (3x32x32; xb = 4 B f32, 1 B raw u8 clips).
    The excitation E and the inhibition I keep their f32 values in both cell
    dtypes: a full-precision E or I tile counts F + dE bytes
    (dE: the extra 2 B per element in bf16: the f32 array, or (r05) the hi +
    lo planes), a read of only its bf16 operand value F (the hi plane; I's
    hi plane is the exc conv's input and k_wgrad's X).  Implementation
    overhead (the per-workgroup gradient partials, BatchNorm sums) is not
    algorithmic and is not counted."""
    F, XF = C * HW * HW * elt, 3 * HW * HW * xb
    dE = C * HW * HW * (4 - elt)
    if fused:       # the conv reads its input from the LDS tile the point-wise half wrote
        # fa: E_{t-2} full, I_{t-1} hi, eg, ce in; E_{t-1} full, gE, eg, ci out
        # fb: c_i, I_{t-1} full in; I_t full, c_e out
        fwd = {"k_fused_fa": frames * (XF + 8 * F + 2 * dE),
               "k_fused_fb": frames * (XF + 4 * F + 2 * dE),
               "k_pw_fa": 5 * F + 2 * dE}                # closes E_{T-1} only
        if kind in fwd or kind in ("k_pw_fb", "k_conv_fa", "k_conv_fb"):
            return fwd.get(kind, 0) * batch
    if cpa and kind in ("k_conv_pw_ba", "k_conv_ba", "k_pw_ba"):
        # k_conv_pw_ba: the two kernels' bytes (dgE still stored and read back,
        # by the same wave); k_pw_ba: its first and last launches ~ one frame;
        # k_conv_ba: frame 0's BatchNorm-backward fill (dc, raw in, dci out)
        return {"k_conv_pw_ba": (frames - 1) * (5 * F + XF + 11 * F + dE),
                "k_pw_ba": XF + 11 * F + dE, "k_conv_ba": 3 * F}[kind] * batch
    per_clip = {
        "k_pw_fa": frames * (XF + 7 * F + 2 * dE),
        "k_conv_fa": frames * 2 * F,
        "k_pw_fb": frames * (XF + 4 * F + 2 * dE),
        "k_conv_fb": frames * 2 * F,
        # dgE, E_t hi, dEn, I_t hi, ce, eg, E_{t-1} full in; dIl, dEn, dEp, dcE out
        "k_pw_ba": frames * (XF + 11 * F + dE),
        "k_conv_ba": (frames - 1) * 5 * F + 3 * F,
        "k_pw_bb": frames * (XF + 8 * F + dE),
        "k_conv_bb": frames * 6 * F,
        "k_wgrad": frames * 4 * F,
    }
    return per_clip.get(kind, 0) * batch


# forward per clip-frame 2 k x k convs + 6 gates = 218,103,808 FLOP,
# the stem 2*3*32*1024 per frame; fwd + bwd = 3 x forward (41.91 GFLOP / clip at
# T = 64).  Minimal HBM bytes: 17.2 MB per 64-frame clip (268.75 KB per clip-frame).
FLOP_8D_FRAME = 2 * conv_flops() + 6 * gate_flops()
FLOP_8D_STEM = 2 * 3 * C * HW * HW
BYTES_8D_FRAME = 17.2e6 / 64
CONV_KINDS = ("k_fused_fa", "k_fused_fb", "k_conv_fa", "k_conv_fb", "k_conv_ba", "k_conv_bb", "k_wgrad",
              "k_persist_fwd", "k_conv_pw_ba")


def step_flops_8d(batch, frames):
    return 3 * batch * frames * (FLOP_8D_FRAME + FLOP_8D_STEM)


def _pmc_summary(batch, frames, dtype, lib_version):
    import glob
    tag = f"B={batch} T={frames} {dtype}"
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc_traffic.json")), reverse=True):
        d = json.load(open(f))
        if d.get("note") == tag and d.get("lib_version") == lib_version:
            return d
    return None


def pmc_step_bytes(batch, frames, dtype, lib_version):
    """HBM bytes of one whole step from the matching PMC summary: every kernel's
    per-launch traffic times its launches per profiled step (the summary's
    `steps`, else the fused forward's launches / frames), or None."""
    d = _pmc_summary(batch, frames, dtype, lib_version)
    if d is None:
        return None
    k = d["kernels"]
    steps = d.get("steps") or (k["k_fused_fa"]["launches"] / frames if "k_fused_fa" in k else None)
    if not steps:
        return None
    return sum(v["traffic_bytes"] * v["launches"] for v in k.values()) / steps


def pmc_traffic(kernel, batch, frames, dtype, lib_version):
    """HBM bytes per launch of `kernel` from the committed PMC summary
    (profiles/*_pmc_traffic.json, written by tools/pmc_traffic.py from
    rocprofv3 FETCH_SIZE / WRITE_SIZE passes of this same workload), or None.
    Only a summary stamped with the loaded library's version (which carries the
    hash of the kernel sources, ptamd/build.py) counts: counters of other
    kernels say nothing about these."""
    import glob
    tag = f"B={batch} T={frames} {dtype}"
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc_traffic.json")), reverse=True):
        d = json.load(open(f))
        if (d.get("note") == tag and d.get("lib_version") == lib_version
                and kernel in d.get("kernels", {})):
            return d["kernels"][kernel]["traffic_bytes"]
    return None


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(argv, gpus, script=None):
    """--gpus N > 1 outside a torch.distributed.run launch: start N ranks of
    `script` (default: this file) on this node as a child process (before this
    process touches the GPU) and return its exit code; None when this process
    is already a rank or N = 1."""
    if gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={gpus}", "--master-addr", "127.0.0.1",
           f"--master-port={_free_port()}", os.path.abspath(script or __file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def dry_run(world, rank):
    """--dry-run: the launcher and rendezvous path with gloo on CPU, no GPU:
    every rank checks the world size and joins one all-reduce."""
    if world > 1:
        dist.init_process_group("gloo")
        assert dist.get_world_size() == world
        t = torch.ones(1)
        dist.all_reduce(t)
        assert int(t.item()) == world
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def make_data(seed, batch, frames, device, u8=False):
    """Synthetic clips: the f32 model input [B,3,T,32,32], or (u8) the raw
    clip bytes [B,T,32,32,3] the cell converts while staging each frame."""
    from ptamd import synth
    clips, labels = synth.make_batch(seed, batch, frames)
    # C-contiguous [B,3,T,H,W] as prepare_data hands it over (the transposed
    # numpy view kept its strides through astype / .to(device), and the cell
    # then made a 201 MB contiguous copy inside every timed step: 81 us)
    x = (torch.from_numpy(clips) if u8 else
         torch.from_numpy(np.ascontiguousarray(clips.transpose(0, 4, 1, 2, 3), dtype=np.float32) / 255.0))
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


def kernel_roofline(kind, ms, n, batch, frames, steps, dtype, xb, fused=False, cpa=False):
    """One kernel kind against the roofline SURVEY.md §8(d) binds it to: every
    kernel that runs a k x k conv (the fused cell segments, the backward convs,
    the weight gradients) is MFMA-bound -- achieved = §8(d) FLOPs per launch /
    average launch time vs the dense MFMA peak; the point-wise-only kernels
    are HBM-bound on this design's algorithmic bytes.  Also
    returned for every kernel: its MFMA fraction and, labelled as the
    design's own byte count, its HBM fraction."""
    elt = 2 if dtype == "bf16" else 4
    fl = algorithmic_flops(kind, batch, frames, fused, cpa) * steps / max(n, 1)
    by = algorithmic_bytes(kind, batch, frames, elt, xb, fused, cpa) * steps / max(n, 1)
    avg = ms / max(n, 1) * 1e-3
    peak_f = PEAK_TFLOPS[dtype]
    mf = fl / avg / 1e12
    hb = by / avg / 1e9
    if kind in CONV_KINDS:
        r = {"bound": "mfma", "achieved": round(mf, 2), "peak": peak_f, "unit": "TFLOP/s"}
    else:
        r = {"bound": "hbm", "achieved": round(hb, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s"}
    r["frac"] = round(r["achieved"] / r["peak"], 4)
    r["mfma_frac"] = round(mf / peak_f, 4)
    r["hbm_frac_design_bytes"] = round(hb / PEAK_HBM_GBS, 4)
    return r, int(fl), int(by), avg * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256, help="clips per GPU")
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-f32", action="store_true", help="skip the f32-cell figure")
    ap.add_argument("--f32-steps", type=int, default=3)
    ap.add_argument("--input", default="f32", choices=["u8", "f32"],
                    help="cell input: raw u8 clips (converted in-kernel) or the f32 tensor")
    ap.add_argument("--sync-bn", action="store_true",
                    help="N>1: BatchNorm statistics over all ranks' clips (SyncBN, opt-in)")
    ap.add_argument("--no-grad-overlap", action="store_true",
                    help="N>1: all-reduce every gradient after backward (default: the cell's "
                         "early gradients on a side stream under the k x k weight-gradient kernel)")
    ap.add_argument("--rehearse", action="store_true",
                    help="N>1 on a ONE-GPU box: every rank on cuda:0, gloo instead of RCCL -- "
                         "exercises the multi-rank step (broadcast, the three-part gradient "
                         "exchange, the MAX over ranks); not a measurement")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher / rendezvous check on CPU (gloo), no GPU work")
    args = ap.parse_args()

    rc = launch_ranks(sys.argv[1:], args.gpus)
    if rc is not None:
        sys.exit(rc)
    from ptamd.dist import CellDist, GradBucket, env_rank
    rank, local_rank, world = env_rank()
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but the launcher started {world} rank(s)")
    if args.dry_run:
        dry_run(world, rank)
        return

    from ptamd import _lib
    from models import InT as int_mod

    if args.rehearse:
        local_rank = 0
    if world > 1:
        if args.rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
            assert dist.get_world_size() == args.gpus and dist.get_backend() == "nccl"
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)

    def build(dtype):
        torch.manual_seed(1234)
        model = int_mod.InT(dimensions=C, timesteps=args.frames, kernel_size=K).to(dev)
        model.cell_dtype = dtype
        if world > 1:                       # identical init on every rank
            for p in model.parameters():
                dist.broadcast(p.data, 0)
        bucket = GradBucket(model.parameters(), dev)
        if world > 1:
            model.cell_dist = CellDist(sync_bn=args.sync_bn,
                                       bucket=None if args.no_grad_overlap else bucket)
        # the same Adam update as one fused kernel over all parameters (the
        # default multi-tensor form launched seven kernels, ~0.1 ms per step)
        return model, bucket, torch.optim.Adam(model.parameters(), lr=3e-4, fused=True)

    model, bucket, opt = build(args.dtype)
    crit = torch.nn.BCEWithLogitsLoss()
    x, y = make_data(1000 + rank, args.batch, args.frames, dev, u8=args.input == "u8")
    ar_ev = []                               # (start, end) events around the all-reduce

    def step(model, bucket, opt, time_ar=False):
        out, _ = model(x)
        loss = crit(out, y.reshape(-1, 1))
        loss.backward()
        if time_ar and world > 1:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            bucket.allreduce_mean()
            e1.record()
            ar_ev.append((e0, e1))
        else:
            bucket.allreduce_mean()
        opt.step()
        opt.zero_grad(set_to_none=True)
        return loss

    for _ in range(args.warmup):
        step(model, bucket, opt)
    torch.cuda.synchronize()
    lib = _lib.load()
    # timed region: no instrumentation (the per-launch HIP events of the
    # kernel-timing pass below add ~1 us of stream work per launch)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step(model, bucket, opt)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    # kernel-timing pass (same steps, HIP events around every library launch
    # on its launch stream, and around the all-reduce)
    lib.pt_cell_timing_reset()
    lib.pt_cell_timing_enable((1 << _lib.NKINDS) - 1)
    for _ in range(args.steps):
        step(model, bucket, opt, time_ar=True)
    torch.cuda.synchronize()
    lib.pt_cell_timing_enable(0)
    kern = {name: _lib.timing_read(kind) for kind, name in enumerate(_lib.KIND_NAMES)}
    lib.pt_cell_timing_reset()
    ar_ms = sum(a.elapsed_time(b) for a, b in ar_ev) / args.steps if ar_ev else 0.0
    if world > 1:
        t = torch.tensor([el, ar_ms], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el, ar_ms = float(t[0]), float(t[1])
    version = lib.pt_version().decode()
    f32 = None
    if world == 1 and args.dtype == "bf16" and not args.no_f32:
        del model, bucket, opt
        torch.cuda.empty_cache()
        m32, b32, o32 = build("f32")
        step(m32, b32, o32)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.f32_steps):
            step(m32, b32, o32)
        torch.cuda.synchronize()
        e32 = time.perf_counter() - t1
        f32 = {"value": round(args.batch * args.f32_steps / e32, 2), "unit": "clips/s",
               "ms_per_step": round(e32 / args.f32_steps * 1e3, 3), "steps": args.f32_steps,
               "dtype": "f32",
               "note": "same step with the f32 cell (exact-f32 MFMA, f32 saved states): the "
                       "reference's arithmetic and the oracle-pinned parity path"}
        del m32, b32, o32

    if rank == 0:
        xb = 1 if args.input == "u8" else 4
        value = world * args.batch * args.steps / el
        fused = kern["k_fused_fa"][1] > 0
        cpa = kern.get("k_conv_pw_ba", (0.0, 0))[1] > 0
        dom = max(kern, key=lambda k: kern[k][0])
        dom_ms, dom_n = kern[dom]
        roof, fl, by, avg_ms = kernel_roofline(dom, dom_ms, dom_n, args.batch, args.frames,
                                               args.steps, args.dtype, xb, fused, cpa)
        roof.update({"traffic": pmc_traffic(dom, args.batch, args.frames, args.dtype, version),
                     "kernel": dom, "avg_launch_ms": round(avg_ms, 4), "launches": dom_n,
                     "algorithmic_flop_per_launch": fl, "algorithmic_bytes_per_launch": by})
        # every kernel kind against its own binding roofline (context for the
        # dominant one above): conv / wgrad are MFMA-bound, point-wise HBM-bound
        per_kind = {}
        for k, (ms, n) in kern.items():
            if n == 0 or ms <= 0 or (algorithmic_flops(k, 1, args.frames, fused, cpa) == 0 and
                                     algorithmic_bytes(k, 1, args.frames, 2, 4, fused, cpa) == 0):
                continue
            r, _, _, a = kernel_roofline(k, ms, n, args.batch, args.frames, args.steps,
                                         args.dtype, xb, fused, cpa)
            per_kind[k] = {"bound": r["bound"], "achieved": r["achieved"], "unit": r["unit"],
                           "frac": r["frac"], "mfma_frac": r["mfma_frac"],
                           "hbm_frac_design_bytes": r["hbm_frac_design_bytes"],
                           "avg_launch_us": round(a * 1e3, 2)}
        # the whole step against SURVEY.md §8(d): its FLOPs vs the MFMA peak, and
        # the PMC-measured HBM bytes of every kernel of the step vs §8(d)'s minimum
        sf = step_flops_8d(world * args.batch, args.frames) / world
        step_s = el / args.steps
        sb = pmc_step_bytes(args.batch, args.frames, args.dtype, version)
        step_8d = {"flop_per_step": int(sf), "step_mfma_frac": round(sf / step_s / (PEAK_TFLOPS[args.dtype] * 1e12), 4),
                   "min_bytes_per_step_8d": int(args.batch * args.frames * BYTES_8D_FRAME),
                   "pmc_bytes_per_step": None if sb is None else int(sb),
                   "step_traffic_vs_8d": None if sb is None else
                   round(sb / (args.batch * args.frames * BYTES_8D_FRAME), 2)}
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
                       "parallelism": f"dp{world}",
                       "batchnorm": "sync" if (args.sync_bn and world > 1) else "per-replica",
                       "grad_overlap": world > 1 and not args.no_grad_overlap},
            "roofline": roof,
            "roofline_per_kernel": per_kind,
            "step_vs_8d": step_8d,
            "kernels_ms_per_step": {k: round(v[0] / args.steps, 3) for k, v in kern.items()},
            "allreduce_ms_per_step": round(ar_ms, 4),
            "lib_version": version,
            "loss": round(float(loss.item()), 5),
        }
        if f32 is not None:
            line["f32_cell"] = f32
        if args.rehearse:
            line["rehearsal"] = "all ranks on one GPU over gloo: a path check, not a measurement"
        if not np.isfinite(line["loss"]):
            print("bench.py: WARNING non-finite training loss", file=sys.stderr, flush=True)
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args.cpu_seconds, frames=args.frames)
            line["cpu_baseline_cfg1"] = cpu_baseline(args.cpu_seconds, frames=32)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
