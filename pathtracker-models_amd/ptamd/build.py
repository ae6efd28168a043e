"""Build the HIP extension in-tree for gfx950: ``python -m ptamd.build``.

One ``hipcc -shared -fPIC`` line; the resulting ``libptcell.so`` sits next to
``_lib.py`` so it travels with the repository snapshot to the GPU box.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
OUT = os.path.join(HERE, "libptcell.so")
SOURCES = [os.path.join(CSRC, "pt_cell.hip")]
DEPS = SOURCES + [os.path.join(CSRC, "pt_device.h"), os.path.join(REPO, "include", "pt_cell.h")]


def up_to_date() -> bool:
    if not os.path.exists(OUT):
        return False
    t = os.path.getmtime(OUT)
    return all(os.path.getmtime(d) <= t for d in DEPS)


def build(force: bool = False, verbose: bool = True) -> str:
    if not force and up_to_date():
        return OUT
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-I", os.path.join(REPO, "include"), "-o", OUT + ".tmp", *SOURCES]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
