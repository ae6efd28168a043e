#!/usr/bin/env python3
"""Per-workgroup phase timeline of one frame's launches (pt_cell_trace):
forward + backward at B, T (default 256, 64) with frame FRAME traced.

Per kernel: the launch span, per phase the median / max time since the
workgroup's entry, and (r06) the per-wave row ends (slots 8-15) and conv ends
(slots 16-23) against the kernel's first entry, broken down by where the
workgroup ran (slot 7: XCC_ID and HW_ID -> SE / SH / CU / SIMD), by its entry
order on its CU (first or second co-resident workgroup) and by clip.  The raw
records are saved to gpurun_out/trace_<tag>.npy for offline analysis
(100 MHz counter: 10 ns ticks).  Diagnostics only (libptcell_diag.so)."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "pathtracker-models_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from ptamd import _lib  # noqa: E402
if os.environ.get("TRACE_LIB"):          # a diagnostic A/B build (tools/build_ab.sh ... -DPT_DIAG=1)
    _lib.DIAG_PATH = os.environ["TRACE_LIB"]
_lib.use_diag()         # the PT_DIAG build (libptcell_diag.so) honours the switches
from models import InT  # noqa: E402

NWG, NSLOT = _lib.TRACE_WG, _lib.TRACE_SLOTS
SLOTS = {"k_pw_bb": ["entry", "issued", "prologue", "rows", "bn_partial", "flush", "publish"],
         "k_pw_ba": ["entry", "-", "prologue", "rows", "bn_partial", "flush", "publish"],
         "k_fused_fa": ["entry", "-", "prologue", "pw_rows", "conv", "bn_stats", "bn_publish"],
         "k_fused_fb": ["entry", "-", "prologue", "pw_rows", "conv", "bn_stats", "bn_publish"],
         "k_conv_bb": ["entry", "bn_table", "band0_fill", "band1_fill", "-", "-", "-"],
         "k_conv_ba": ["entry", "bn_table", "band0_fill", "band1_fill", "-", "-", "-"]}


def decode(idw):
    """slot-7 word -> (xcc, se, sh, cu, simd, wave slot)"""
    hw = idw & 0xffffffff
    return ((idw >> 32) & 0xf, (hw >> 13) & 0x7, (hw >> 12) & 1, (hw >> 8) & 0xf, (hw >> 4) & 3, hw & 0xf)


def analyse(name, r, names):
    ok = (r[:, 0] > 0) & (r[:, 7] >> 40 == 1)
    if not ok.any():
        return
    idx = np.nonzero(ok)[0]
    r = r[ok].astype(np.int64)
    t0 = r[:, 0].min()
    us = lambda v: (v - t0) / 100.0
    end = max(r[:, 6].max(), r[:, 8:24].max())
    print(f"\n{name}: {len(r)} workgroups traced, first entry -> last stamp {us(end):.1f} us, "
          f"entries spread {us(r[:, 0].max()):.1f} us")
    for j, nm in enumerate(names):
        if nm == "-" or j == 0:
            continue
        m = r[:, j] > 0
        if m.any():
            d = (r[m, j] - r[m, 0]) / 100
            print(f"   {nm:11s} since entry: median {np.median(d):7.2f}  max {d.max():7.2f} us")
    ids = [decode(int(v)) for v in r[:, 7]]
    xcc = np.array([i[0] for i in ids])
    cukey = np.array([(i[0] << 8) | (i[1] << 5) | (i[2] << 4) | i[3] for i in ids])
    for base, what in ((8, "row end"), (16, "conv end")):
        w = r[:, base:base + 8]
        m = w > 0
        if not m.any():
            continue
        wmax = np.where(m, w, 0).max(1)          # the workgroup's last wave
        wmin = np.where(m, w, np.iinfo(np.int64).max).min(1)
        has = m.any(1)
        e = us(wmax[has])
        print(f"   per-wave {what} (vs first entry): WG last wave median {np.median(e):6.2f} "
              f"p90 {np.percentile(e, 90):6.2f} max {e.max():6.2f} us; within-WG wave spread median "
              f"{np.median((wmax - wmin)[has]) / 100:5.2f} max {((wmax - wmin)[has]).max() / 100:5.2f} us")
        # by XCC
        row = "      by XCC (median / max of WG last wave):"
        for x in range(8):
            s = has & (xcc == x)
            if s.any():
                row += f"  {x}: {np.median(us(wmax[s])):5.1f}/{us(wmax[s]).max():5.1f}"
        print(row)
        # co-resident order on a CU: rank by entry among WGs sharing the CU key
        rank = np.zeros(len(r), int)
        ncu = {}
        for k in np.unique(cukey):
            s = np.nonzero(cukey == k)[0]
            order = s[np.argsort(r[s, 0])]
            rank[order] = np.arange(len(order))
            ncu[k] = len(s)
        for q in range(rank.max() + 1):
            s = has & (rank == q)
            if s.any():
                print(f"      entry rank {q} on its CU: {s.sum():4d} WGs, last wave median "
                      f"{np.median(us(wmax[s])):6.2f} max {us(wmax[s]).max():6.2f} us, entry median "
                      f"{np.median(us(r[s, 0])):5.2f}")
        cnt = np.array([ncu[k] for k in cukey])
        for q in sorted(set(cnt)):
            s = has & (cnt == q)
            print(f"      CUs holding {q} traced WGs: {s.sum():4d} WGs, last wave median "
                  f"{np.median(us(wmax[s])):6.2f} max {us(wmax[s]).max():6.2f} us")
        late = np.argsort(-wmax)[:8]
        print("      latest 8 WGs (wg index, xcc, se, sh, cu, simd, entry us, last wave us, spread us): " +
              "; ".join(f"{idx[i]} x{ids[i][0]} s{ids[i][1]} h{ids[i][2]} c{ids[i][3]} m{ids[i][4]} "
                        f"{us(r[i, 0]):.1f} {us(wmax[i]):.1f} {(wmax[i] - wmin[i]) / 100:.1f}" for i in late))


def main():
    b, t, fr = int(os.environ.get("B", 256)), int(os.environ.get("T", 64)), int(os.environ.get("FRAME", 30))
    tag = os.environ.get("TAG", "head")
    dev = torch.device("cuda:0")
    lib = _lib.load()
    torch.manual_seed(0)
    m = InT.InT(dimensions=32, timesteps=t, kernel_size=7).to(dev)
    m.cell_dtype = "bf16"
    x = torch.rand(b, 3, t, 32, 32, device=dev)
    for _ in range(2):                       # warm-up, then the traced pass
        buf = torch.zeros(_lib.NKINDS * NWG * NSLOT, dtype=torch.int64, device=dev)
        lib.pt_cell_trace(ctypes.c_void_p(buf.data_ptr()), fr)
        out, _ = m(x)
        out.sum().backward()
        torch.cuda.synchronize()
        lib.pt_cell_trace(None, -1)
    tr = buf.view(_lib.NKINDS, NWG, NSLOT).cpu().numpy()
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    np.save(os.path.join(REPO, "gpurun_out", f"trace_{tag}.npy"), tr)
    for k, names in SLOTS.items():
        analyse(k, tr[_lib.KIND_NAMES.index(k)], names)


if __name__ == "__main__":
    main()
