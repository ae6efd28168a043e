#!/usr/bin/env python3
"""Per-kernel means of every counter in rocprofv3 --pmc run directories.

Writes OUT_JSON {kernel: {counter: mean per dispatch, "dispatches": n}}, prints
the table, and with --rm deletes the raw CSVs (a full bench pass can exceed
gpurun's 64 MiB copy-back limit).  Kernels are keyed by their ptc::/ptl::
short name plus the workgroup size, so variants stay apart.

usage: pmc_summary.py OUT_JSON RUN_DIR [RUN_DIR ...] [--rm]
"""
import collections
import csv
import glob
import json
import re
import shutil
import sys


def _key(row):
    m = re.search(r"(k_[a-z_0-9]+)", row["Kernel_Name"])
    base = m.group(1) if m else row["Kernel_Name"][:50]
    # template arguments (mangled Li..E / demangled <...>) keep instantiations apart
    tail = row["Kernel_Name"][m.end():m.end() + 48] if m else ""
    targs = re.findall(r"Li(\d+)E|Lb(\d)E|, (\d+|true|false)", tail)
    ta = ",".join(next(x for x in t if x) for t in targs)
    return f"{base}<{ta}>/wg{row['Workgroup_Size']}" if ta else f"{base}/wg{row['Workgroup_Size']}"


def main():
    args = [a for a in sys.argv[1:] if a != "--rm"]
    out, dirs = args[0], args[1:]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            for row in csv.DictReader(open(f)):
                acc[_key(row)][row["Counter_Name"]].append(float(row["Counter_Value"]))
    res = {}
    for k, cs in sorted(acc.items()):
        res[k] = {c: sum(v) / len(v) for c, v in cs.items()}
        res[k]["dispatches"] = max(len(v) for v in cs.values())
    json.dump(res, open(out, "w"), indent=1)
    for k, cs in res.items():
        if k.startswith("k_"):
            print(k)
            for c, v in sorted(cs.items()):
                print(f"   {c:32s} {v:16.1f}")
    if "--rm" in sys.argv:
        for d in dirs:
            shutil.rmtree(d)
    print(f"{len(res)} kernels -> {out}")


if __name__ == "__main__":
    main()
