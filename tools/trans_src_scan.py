#!/usr/bin/env python3
"""For every transcendental VALU instruction (v_exp / v_log / v_rcp / ...) in
a gfx950 listing: distance, in issued instructions (s_nop n counted as n + 1),
from the latest writer of its source VGPR, with the writer's opcode.  A
histogram per kernel, and the closest cases.
Usage: trans_src_scan.py listing.s [kernel-substring] [N]"""
import collections
import re
import sys

sys.path.insert(0, __import__("os").path.dirname(__file__))
from waitcnt_check import functions, regs, split_ops  # noqa: E402
from trans_hazard_scan import TRANS, instrs  # noqa: E402


def dst_of(s):
    op = s.split()[0]
    if not op.startswith("v_") or op.startswith(("v_cmp", "v_readlane", "v_readfirstlane")):
        return set()
    ops = split_ops(s[len(op):])
    return regs(ops[0]) if ops else set()


def main():
    lines = open(sys.argv[1]).read().split("\n")
    want = sys.argv[2] if len(sys.argv) > 2 and sys.argv[2] != "-" else None
    nshow = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    tot = collections.Counter()
    for name, body in functions(lines, want):
        ins = instrs(body)
        hist = collections.Counter()
        shown = []
        for i, s in enumerate(ins):
            op = s.split()[0]
            if not TRANS.match(op):
                continue
            ops = split_ops(s[len(op):])
            src = set()
            for tok in ops[1:]:
                src |= regs(tok)
            src = {r for r in src if r[0] == "v"}
            if not src:
                continue
            ws = 0
            for j in range(i - 1, max(-1, i - 16), -1):
                t = ins[j]
                top = t.split()[0]
                if top.endswith(":") or top.startswith(("s_branch", "s_cbranch")):
                    break
                m = re.match(r"s_nop\s+(\d+)", t)
                ws += int(m.group(1)) + 1 if m else 1
                if dst_of(t) & src:
                    hist[(ws, top)] += 1
                    if ws <= nshow and len(shown) < 16:
                        shown.append((ws, ins[max(0, j - 1):i + 1]))
                    break
        tot.update(hist)
        h = collections.Counter()
        for (w, _), c in hist.items():
            h[w] += c
        print(f"{name[:70]}: writer->trans distance {dict(sorted(h.items()))}")
        for w, ctx in shown:
            print(f"    d={w}: " + "  |  ".join(ctx))
    h = collections.Counter()
    for (w, top), c in tot.items():
        h[w] += c
    print("total", dict(sorted(h.items())))
    print("writers at distance 1:", collections.Counter(top for (w, top), c in tot.items() for _ in range(c) if w == 1).most_common(12))


if __name__ == "__main__":
    main()
