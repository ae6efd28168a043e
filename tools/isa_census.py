#!/usr/bin/env python3
"""Static instruction census of one kernel in a gfx950 assembly listing
(hipcc --cuda-device-only -S): opcode counts, VALU split into transcendental
(quarter rate: v_exp / v_log / v_rcp / v_sqrt / v_rsq / v_sin / v_cos),
conversion / permute, packed and plain arithmetic.  Usage:
  isa_census.py listing.s <mangled-name-substring> [top]"""
import collections
import re
import sys

TRANS = ("v_exp_", "v_log_", "v_rcp_", "v_sqrt_", "v_rsq_", "v_sin_", "v_cos_")
CONV = ("v_cvt_", "v_perm_", "v_bfe_", "v_lshl", "v_lshr", "v_and_", "v_or_", "v_alignbit", "v_mov_", "v_cndmask")


def body(lines, name):
    out, on = [], False
    for ln in lines:
        if re.match(r"^_Z\S*:", ln):
            on = name in ln.split(":")[0]
            continue
        if on and ln.startswith(".Lfunc_end"):
            break
        s = ln.strip()
        if on and s and not s.startswith((".", ";")) and not s.endswith(":"):
            out.append(s)
    return out


def main():
    lines = open(sys.argv[1]).read().split("\n")
    b = body(lines, sys.argv[2])
    ops = collections.Counter(s.split()[0] for s in b)
    valu = {k: v for k, v in ops.items() if k.startswith("v_") and not k.startswith(("v_mfma", "v_accvgpr", "v_readlane", "v_writelane", "v_readfirstlane"))}
    tr = sum(v for k, v in valu.items() if k.startswith(TRANS))
    cv = sum(v for k, v in valu.items() if k.startswith(CONV))
    pk = sum(v for k, v in valu.items() if k.startswith("v_pk_"))
    tot = sum(valu.values())
    print(f"instructions {len(b)}  VALU {tot}: transcendental {tr}, convert/move/select/bit {cv}, "
          f"packed {pk}, other {tot - tr - cv - pk}")
    print("mfma", sum(v for k, v in ops.items() if k.startswith("v_mfma")),
          "global", sum(v for k, v in ops.items() if k.startswith("global_")),
          "ds", sum(v for k, v in ops.items() if k.startswith("ds_")),
          "s_waitcnt", ops.get("s_waitcnt", 0), "s_barrier", ops.get("s_barrier", 0))
    for k, v in ops.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 40):
        print(f"  {k:28s} {v}")


if __name__ == "__main__":
    main()
