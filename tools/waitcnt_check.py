#!/usr/bin/env python3
"""Static check of the memory-counter waits in a gfx950 assembly listing
(hipcc --cuda-device-only -S): for every kernel, a data-flow pass over the
basic blocks tracks which registers are the destinations of loads still
outstanding (vmcnt: global / buffer / flat / scratch, returned in issue order;
lgkmcnt: LDS in issue order, scalar loads out of order) and flags every
instruction that reads or writes such a register before an `s_waitcnt` has
retired the load -- the hazard that reads a register while the memory return
is still landing (a missing wait would show up at run time as stale values in
part of a wave).  Inline-asm instructions are checked like the compiler's own.
Usage: waitcnt_check.py listing.s [kernel-substring]"""
import re
import sys

VMEM = ("global_", "buffer_", "flat_", "scratch_")
SMEM = ("s_load_", "s_buffer_load_", "s_scratch_load_")
BR = re.compile(r"^s_(c?branch\S*|setpc_b64|endpgm)")
REG = re.compile(r"\b([vas])(?:(\d+)|\[(\d+):(\d+)\])")
MAXQ = 64


def regs(tok):
    out = set()
    for m in REG.finditer(tok):
        k = m.group(1)
        if m.group(2) is not None:
            out.add((k, int(m.group(2))))
        else:
            for r in range(int(m.group(3)), int(m.group(4)) + 1):
                out.add((k, r))
    return out


def split_ops(rest):
    rest = rest.split(";")[0]
    return [t.strip() for t in rest.split(",") if t.strip()]


def functions(lines, want):
    cur, body = None, []
    for ln in lines:
        m = re.match(r"^(_Z\S*|[A-Za-z_]\w*):\s*(;.*)?$", ln)
        if m and not ln.startswith(".") and "@" in ln:
            cur, body = m.group(1), []
            continue
        if cur and ln.startswith(".Lfunc_end"):
            if want is None or want in cur:
                yield cur, body
            cur = None
            continue
        if cur is not None:
            body.append(ln)


def blocks(body):
    """[(label, [instr lines])], successor map"""
    blks, cur = [], ["<entry>", []]
    for ln in body:
        s = ln.strip()
        if not s or s.startswith((";", ".")) and not s.startswith(".LBB"):
            continue
        if re.match(r"^\.LBB\S*:", s) or re.match(r"^\.Ltmp\S*:", s):
            blks.append(cur)
            cur = [s[:-1], []]
            continue
        if s.startswith("."):
            continue
        cur[1].append(s)
        if BR.match(s):
            blks.append(cur)
            cur = [f"<after {len(blks)}>", []]
    blks.append(cur)
    blks = [b for b in blks if b[1] or b[0].startswith(".LBB")]
    idx = {b[0]: i for i, b in enumerate(blks)}
    succ = []
    for i, (lab, ins) in enumerate(blks):
        s = []
        last = ins[-1] if ins else ""
        op = last.split()[0] if last else ""
        if op == "s_branch":
            s.append(idx.get(last.split()[1]))
        elif op.startswith("s_cbranch"):
            s.append(idx.get(last.split()[1]))
            s.append(i + 1 if i + 1 < len(blks) else None)
        elif op in ("s_endpgm", "s_setpc_b64"):
            pass
        else:
            s.append(i + 1 if i + 1 < len(blks) else None)
        succ.append([x for x in s if x is not None])
    return blks, succ


def parse_wait(s):
    vm = lg = None
    m = re.search(r"vmcnt\((\d+)\)", s)
    if m:
        vm = int(m.group(1))
    m = re.search(r"lgkmcnt\((\d+)\)", s)
    if m:
        lg = int(m.group(1))
    m = re.match(r"s_waitcnt\s+(\d+)\s*$", s)
    if m:
        v = int(m.group(1))
        vm = (v & 0xF) | ((v >> 14) & 3) << 4
        lg = (v >> 8) & 0xF
    return vm, lg


class State:
    __slots__ = ("vm", "lg", "smem")

    def __init__(self, vm=(), lg=(), smem=False):
        self.vm, self.lg, self.smem = tuple(vm), tuple(lg), smem   # newest first

    def key(self):
        return (self.vm, self.lg, self.smem)

    @staticmethod
    def merge(a, b):
        def m(x, y):
            n = max(len(x), len(y))
            return tuple((x[i] if i < len(x) else frozenset()) | (y[i] if i < len(y) else frozenset())
                         for i in range(n))
        return State(m(a.vm, b.vm), m(a.lg, b.lg), a.smem or b.smem)


def step(st, s, report, where):
    op = s.split()[0]
    rest = s[len(op):]
    ops = split_ops(rest)
    if op == "s_waitcnt":
        vm, lg = parse_wait(s)
        vmq, lgq, smem = st.vm, st.lg, st.smem
        if vm is not None:
            vmq = vmq[:vm]
        if lg is not None:
            if lg == 0:
                lgq, smem = (), False
            elif not smem:
                lgq = lgq[:lg]
        return State(vmq, lgq, smem)
    pending_vm = set().union(*st.vm) if st.vm else set()
    pending_lg = set().union(*st.lg) if st.lg else set()
    is_vmem = op.startswith(VMEM)
    is_ds = op.startswith("ds_")
    is_smem = op.startswith(SMEM)
    loads = (is_vmem and ("load" in op or "atomic" in op and " glc" in s or "_lds" in op)) or \
            (is_ds and ("read" in op or "bpermute" in op or "permute" in op or "swizzle" in op or
                        "_rtn" in op or "consume" in op or "append" in op)) or is_smem
    dest = set()
    srcs = set()
    if ops:
        if loads and not ("_lds" in op) and not op.startswith("global_load_lds"):
            dest = regs(ops[0])
            for t in ops[1:]:
                srcs |= regs(t)
        else:
            for t in ops:
                srcs |= regs(t)
            if not (is_vmem or is_ds or is_smem) and op.startswith(("v_", "s_")):
                dest = regs(ops[0])
                srcs -= set()   # sources include the dest for read-modify-write ops; fine
    # hazards: any operand (read or written) of a non-memory instruction that a
    # pending load will still write; for memory instructions their address /
    # data operands (sources)
    touched = srcs | (dest if not (loads and (is_vmem or is_ds or is_smem)) else set())
    bad_vm = touched & pending_vm
    bad_lg = touched & pending_lg
    if bad_vm or bad_lg:
        report.append((where, s, sorted(bad_vm), sorted(bad_lg)))
    vmq, lgq, smem = st.vm, st.lg, st.smem
    if is_vmem:
        ev = frozenset(dest) if loads else frozenset()
        vmq = (ev,) + vmq[:MAXQ - 1]
        if op.startswith("flat_"):
            lgq = (ev,) + lgq[:MAXQ - 1]
    elif is_ds:
        if "gws" not in op:
            lgq = (frozenset(dest) if loads else frozenset(),) + lgq[:MAXQ - 1]
    elif is_smem:
        lgq = (frozenset(dest),) + lgq[:MAXQ - 1]
        smem = True
    else:
        # a write of a register by a non-memory instruction removes nothing
        # pending (the load still lands later: that is the WAW hazard above)
        pass
    return State(vmq, lgq, smem)


def check(body):
    blks, succ = blocks(body)
    ins = [None] * len(blks)
    ins[0] = State()
    work = [0]
    out_cache = {}
    reports = {}
    it = 0
    while work:
        it += 1
        if it > 200000:
            raise RuntimeError("no fixpoint")
        i = work.pop()
        st = ins[i]
        rep = []
        for k, s in enumerate(blks[i][1]):
            st = step(st, s, rep, (blks[i][0], k))
        reports[i] = rep
        if out_cache.get(i) == st.key():
            continue
        out_cache[i] = st.key()
        for j in succ[i]:
            new = st if ins[j] is None else State.merge(ins[j], st)
            if ins[j] is None or new.key() != ins[j].key():
                ins[j] = new
                work.append(j)
    return [r for i in sorted(reports) for r in reports[i]]


def main():
    lines = open(sys.argv[1]).read().split("\n")
    want = sys.argv[2] if len(sys.argv) > 2 else None
    total = 0
    for name, body in functions(lines, want):
        rep = check(body)
        total += len(rep)
        print(f"{name}: {len(rep)} hazard(s)")
        for where, s, bv, bl in rep[:20]:
            print(f"   {where[0]}#{where[1]}: {s}   vm={bv[:6]} lgkm={bl[:6]}")
    print("total", total)
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main())
