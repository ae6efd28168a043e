"""Build the HIP extensions in-tree for gfx950: ``python -m ptamd.build``.

One compiler line per library (run in parallel): ``hipcc`` for the gfx950
kernels — ``libptcell.so`` (InT / hGRU cell, include/pt_cell.h) and
``libptlstm.so`` (ConvLSTM cell, include/pt_lstm.h) — and ``g++`` for the host
TFRecord reader ``libpttfr.so`` (include/pt_tfrecord.h, zlib).  They sit next
to the ctypes bindings so they travel with the repository snapshot to the GPU
box.  ``libptcell_diag.so`` is the same cell library built with -DPT_DIAG=1
(the PT_CELL_ABLATE / PT_CELL_DEBUG_STOP switches and pt_cell_trace, for
tools/ only: ``ptamd._lib.use_diag()``); the release ``libptcell.so`` ignores
those switches; ``libptlstm_diag.so`` is the same for the ConvLSTM library.
The diagnostic builds also honour the kernel-variant switches (PT_CELL_FUSED,
PT_PWB2, PT_WG16, PT_LCONV_FAST, ...: ``PT_SW`` in csrc/pt_device.h), which the
release libraries compile to their defaults.
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INC = os.path.join(REPO, "include")

# library -> (sources, extra dependencies[, extra compiler flags])
_CELL = ([os.path.join(CSRC, "pt_cell.hip"), os.path.join(CSRC, "pt_readout.hip")],
         [os.path.join(CSRC, "pt_device.h"), os.path.join(CSRC, "pt_graph.h"),
          os.path.join(INC, "pt_cell.h"), os.path.join(INC, "pt_readout.h")])
_LSTM = ([os.path.join(CSRC, "pt_lstm.hip")],
         [os.path.join(CSRC, "pt_device.h"), os.path.join(CSRC, "pt_graph.h"),
          os.path.join(INC, "pt_lstm.h")])
LIBS = {
    "libptcell.so": _CELL,
    "libptcell_diag.so": _CELL + (["-DPT_DIAG=1"],),
    "libpttfr.so": ([os.path.join(CSRC, "pt_tfrecord.cpp")], [os.path.join(INC, "pt_tfrecord.h")]),
    "libptlstm.so": _LSTM,
    "libptlstm_diag.so": _LSTM + (["-DPT_DIAG=1"],),
}
OUT = os.path.join(HERE, "libptcell.so")      # kept for callers of the old single-library API
# The compiler line of the HIP libraries; part of the source stamp.
# -fno-slp-vectorize (r04): no packed-FP32 (v_pk_fma / v_pk_mul / v_pk_add_f32)
# math formed by the SLP vectorizer.  With it, hipcc (ROCm 7.2) issues a
# packed op right after the VALU instruction that wrote the HIGH register of
# its source pair (968 such pairs in the cell library); now and then the
# packed op read that register stale in the wave's last 16 lanes, so the bf16
# backward differed run to run (the deviating elements were
# always the high element of a pair, lanes 48-63; determinism_check bitwise
# with this flag in both the default and the -ffp-contract=on builds, never
# without it).
HIP_FLAGS = "--offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize"


def _out(lib: str) -> str:
    return os.path.join(HERE, lib)


def up_to_date(lib: str = "libptcell.so") -> bool:
    out = _out(lib)
    if not os.path.exists(out):
        return False
    t = os.path.getmtime(out)
    srcs, deps = LIBS[lib][:2]
    return all(os.path.getmtime(d) <= t for d in srcs + deps)


def src_hash(lib: str) -> str:
    """sha256 (first 12 hex digits) of a library's sources and headers: compiled
    into its version string, so measurements (profiles/*_pmc_traffic.json) can
    be matched to the exact kernels that produced them."""
    h = hashlib.sha256(HIP_FLAGS.encode())
    srcs, deps = LIBS[lib][:2]
    for flag in (LIBS[lib][2] if len(LIBS[lib]) > 2 else []):
        h.update(flag.encode())
    for f in srcs + deps:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:12]


def build(force: bool = False, verbose: bool = True) -> str:
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    procs = []
    for lib, spec in LIBS.items():
        srcs, extra = spec[0], (spec[2] if len(spec) > 2 else [])
        if not force and up_to_date(lib):
            continue
        out = _out(lib)
        if srcs[0].endswith(".cpp"):
            cmd = [os.environ.get("CXX", "g++"), "-O2", "-std=c++17", "-fPIC", "-shared",
                   "-pthread", "-Wall", "-I", INC, "-o", out + ".tmp", *srcs, "-lz", "-ldl"]
        else:
            cmd = [hipcc, *HIP_FLAGS.split(), *extra, "-fPIC", "-shared",
                   f'-DPT_SRC_HASH="{src_hash(lib)}"', "-I", INC, "-o", out + ".tmp", *srcs]
        if verbose:
            print(" ".join(cmd), flush=True)
        procs.append((lib, out, subprocess.Popen(cmd)))
    failed = []
    for lib, out, p in procs:
        if p.wait() != 0:
            failed.append(lib)
        else:
            os.replace(out + ".tmp", out)
    if failed:
        raise RuntimeError(f"hipcc failed for {', '.join(failed)}")
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
