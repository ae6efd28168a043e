#!/usr/bin/env python3
"""Run the cell's forward + backward several times on the same inputs (direct
launches and hipGraph replays) and report, per parameter gradient, whether the
runs agree bit for bit and the largest relative difference.  Diagnostic for
the deterministic BatchNorm reduction (pt_cell.hip PT_BN_MODE)."""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "pathtracker-models_amd")]
import torch  # noqa: E402

from ptamd import _lib  # noqa: E402
from ptamd.cell import PARAM_KEYS, _desc, _pack, _ptr, _stream  # noqa: E402
from models import InT  # noqa: E402


def run(m, x, d_e, saved, ws, lib):
    params = [p.detach().contiguous() if p is not None else None for p in m.cell_params()]
    d = _desc(m.cell_config(), x, 32)
    e = torch.empty((x.shape[0], 32, 32, 32), device=x.device)
    pp = _pack(_lib.Params, params)
    st = _stream(x.device)
    _lib.check(lib.pt_cell_forward(ctypes.byref(d), _ptr(x), ctypes.byref(pp), _ptr(saved), _ptr(ws),
                                   _ptr(e), None, st))
    gr = [torch.empty_like(p) if p is not None else None for p in params]
    gg = _pack(_lib.Grads, gr)
    _lib.check(lib.pt_cell_backward(ctypes.byref(d), _ptr(x), ctypes.byref(pp), _ptr(saved), _ptr(ws),
                                    _ptr(d_e), ctypes.byref(gg), st))
    torch.cuda.synchronize()
    return e.clone(), [g.clone() if g is not None else None for g in gr]


def main():
    b, t = int(os.environ.get("B", 64)), int(os.environ.get("T", 16))
    dev = torch.device("cuda:0")
    lib = _lib.load()
    out = {"lib": lib.pt_version().decode()}
    for dtype in ("bf16", "f32"):
        torch.manual_seed(3)
        m = InT.InT(dimensions=32, timesteps=t, kernel_size=7).to(dev)
        m.cell_dtype = dtype
        x = torch.rand(b, 3, t, 32, 32, device=dev)
        d = _desc(m.cell_config(), x, 32)
        saved = torch.empty(lib.pt_cell_saved_bytes(ctypes.byref(d)), dtype=torch.uint8, device=dev)
        ws = torch.empty(lib.pt_cell_workspace_bytes(ctypes.byref(d)), dtype=torch.uint8, device=dev)
        d_e = torch.randn((b, 32, 32, 32), device=dev, generator=torch.Generator(device=dev).manual_seed(1)) * 1e-3
        runs = []
        for mode in ("direct", "direct", "graph", "graph"):
            lib.pt_cell_timing_enable((1 << _lib.NKINDS) - 1 if mode == "direct" else 0)
            runs.append(run(m, x, d_e, saved, ws, lib))
            lib.pt_cell_timing_enable(0)
            lib.pt_cell_timing_reset()
        e0, g0 = runs[0]
        res = {}
        for i, (e, g) in enumerate(runs[1:], 1):
            r = {"e_last_equal": bool(torch.equal(e, e0))}
            for k, a, c in zip(PARAM_KEYS, g, g0):
                if a is None:
                    continue
                if not torch.equal(a, c):
                    r[k] = float((a - c).abs().max()) / (float(c.abs().max()) + 1e-30)
            res[f"run{i}"] = r
        out[dtype] = res
        print(dtype, json.dumps(res), flush=True)
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    json.dump(out, open(os.path.join(REPO, "gpurun_out", "determinism.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
