#!/usr/bin/env python3
"""gfx950 listing of a BUILT library: the device code object is unbundled from
the .so's .hip_fatbin section (clang-offload-bundler), disassembled with
llvm-objdump, and rewritten in the form of a `hipcc -S` listing that
waitcnt_check.py / pk_hazard_scan.py / trans_hazard_scan.py read: one
`name: ; @name` header per kernel, `.LBB_<offset>:` labels at branch targets
(branch operands rewritten to them), `.Lfunc_end` after the last instruction.
So the static checks run on exactly the machine code that ships (and on the
CPU: tests/test_lib_cpu.py), not on a separate compile.
Usage: isa_listing.py lib.so > listing.s"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
FUNC = re.compile(r"^([0-9a-f]+) <(\S+)>:\s*$")
INS = re.compile(r"^\s+(\S.*?)\s*//\s*([0-9A-F]+):")
BTARGET = re.compile(r"<(\S+)\+0x([0-9a-f]+)>\s*$")


def disassemble(so_path: str) -> str:
    with tempfile.TemporaryDirectory() as d:
        fb, co = os.path.join(d, "fb.bin"), os.path.join(d, "co.o")
        subprocess.run(["objcopy", "--dump-section", f".hip_fatbin={fb}", so_path], check=True,
                       capture_output=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--targets={TARGET}",
                        f"--input={fb}", f"--output={co}"], check=True, capture_output=True)
        return subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co], check=True,
                              capture_output=True, text=True).stdout


def listing(so_path: str) -> str:
    out = []
    funcs = []                              # (name, base, [(addr, text, target)])
    cur = None
    for ln in disassemble(so_path).split("\n"):
        m = FUNC.match(ln)
        if m:
            cur = (m.group(2), int(m.group(1), 16), [])
            funcs.append(cur)
            continue
        if cur is None:
            continue
        m = INS.match(ln)
        if not m:
            continue
        text, addr = m.group(1), int(m.group(2), 16)
        tgt = None
        b = BTARGET.search(ln)
        if b and b.group(1) == cur[0] and text.split()[0].startswith(("s_branch", "s_cbranch")):
            tgt = int(b.group(2), 16)
        cur[2].append((addr, text, tgt))
    for n, (name, base, ins) in enumerate(funcs):
        targets = {t for _, _, t in ins if t is not None}
        out.append(f"{name}:   ; @{name}")
        for addr, text, tgt in ins:
            off = addr - base
            if off in targets:
                out.append(f".LBB_{off:x}:")
            if tgt is not None:
                op = text.split()[0]
                text = f"{op} .LBB_{tgt:x}"
            out.append("\t" + text)
        out.append(f".Lfunc_end{n}:")
    return "\n".join(out) + "\n"


if __name__ == "__main__":
    sys.stdout.write(listing(sys.argv[1]))
