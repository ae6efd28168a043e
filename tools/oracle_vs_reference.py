#!/usr/bin/env python3
"""Step time of the CPU oracle against the reference itself (build container only).

SURVEY.md §8(d): the bench's cpu_baseline times the repo's CPU restatement
(oracle/cells.py) because the reference cannot travel to the GPU box; this
script checks, where the reference IS importable (/root/reference, with the
two NameError aliases and the no-op ``.cuda()`` of tests/golden/make_golden.py),
that the oracle is a faithful stand-in for its step time: InT fwd + BPTT +
Adam on the same seeded clips, same parameters, same thread count, at
BASELINE configs[0] (B=4, T=32) and at the workload's T=64.  The two must
agree in time (ratio ~1) and in output (logits / loss / gradients).

Writes profiles/<tag>_oracle_vs_reference.json.
Usage:  python tools/oracle_vs_reference.py [--tag r02] [--steps 5]
"""
from __future__ import annotations

import argparse
import importlib.util
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
sys.path[:0] = [REPO, os.path.join(REPO, "pathtracker-models_amd")]

import torch  # noqa: E402


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _time(step, n):
    step()                                   # warm-up
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    return (time.perf_counter() - t0) / n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="r02")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--threads", type=int, default=os.cpu_count())
    args = ap.parse_args()
    if not os.path.isdir(REF):
        sys.exit("the reference is not mounted here; this check runs in the build container only")
    torch.set_num_threads(args.threads)
    from oracle import cells
    from ptamd import synth
    torch.Tensor.cuda = lambda self, *a, **k: self       # shim, this process only
    ref_int = _load("ref_InT", os.path.join(REF, "models", "InT.py"))
    ref_int.hConvGRUCell = ref_int.rCell                 # NameError aliases (InT.py:64,187)
    ref_int.FFhGRU = ref_int.InT
    out = {"threads": args.threads, "steps": args.steps, "configs": {}}
    for b, t in ((4, 32), (4, 64)):
        torch.manual_seed(0)
        ref = ref_int.InT(dimensions=32, timesteps=t, kernel_size=7)
        clips, labels = synth.make_batch(99, b, t)
        x = torch.from_numpy(clips.transpose(0, 4, 1, 2, 3) / 255.0).float()
        y = torch.tensor([ord(v) for v in labels], dtype=torch.float32).reshape(-1, 1)
        sd = {k: v.detach().clone().requires_grad_(k != "unit1.w")
              for k, v in ref.named_parameters()}
        opt_r = torch.optim.Adam(ref.parameters(), lr=3e-4)
        opt_o = torch.optim.Adam([v for v in sd.values() if v.requires_grad], lr=3e-4)
        crit = torch.nn.BCEWithLogitsLoss()

        # one step each from the same parameters: outputs must agree
        lr, _ = ref(x)
        crit(lr, y).backward()
        lo, _, _ = cells.recurrent_forward(sd, x)
        cells.bce_logits(lo, y.flatten()).backward()
        gerr = max(float((p.grad - sd[k].grad).abs().max() / (sd[k].grad.abs().max() + 1e-30))
                   for k, p in ref.named_parameters() if p.grad is not None)
        lerr = float((lr.detach().flatten() - lo.detach().flatten()).abs().max())

        def step_ref():
            o, _ = ref(x)
            crit(o, y).backward()
            opt_r.step()
            opt_r.zero_grad(set_to_none=True)

        def step_oracle():
            o, _, _ = cells.recurrent_forward(sd, x)
            cells.bce_logits(o, y.flatten()).backward()
            opt_o.step()
            opt_o.zero_grad(set_to_none=True)

        tr = _time(step_ref, args.steps)
        to = _time(step_oracle, args.steps)
        out["configs"][f"B{b}_T{t}"] = {
            "reference_s_per_step": round(tr, 4), "oracle_s_per_step": round(to, 4),
            "oracle_over_reference": round(to / tr, 3),
            "logit_max_abs_err": lerr, "grad_max_rel_err": gerr}
        print(f"B={b} T={t}: reference {tr:.3f} s/step, oracle {to:.3f} s/step, "
              f"ratio {to / tr:.3f}; logits {lerr:.1e}, grads {gerr:.1e}", flush=True)
    p = os.path.join(REPO, "profiles", f"{args.tag}_oracle_vs_reference.json")
    json.dump(out, open(p, "w"), indent=1)
    print("wrote", p)


if __name__ == "__main__":
    main()
