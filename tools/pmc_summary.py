#!/usr/bin/env python3
"""Average rocprofv3 --pmc counters per kernel (short names) over one or more
counter_collection.csv directories.  usage: pmc_summary.py DIR [DIR ...]"""
import collections
import csv
import glob
import re
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            m = re.search(r"(k_[a-z_0-9]+)", row["Kernel_Name"])
            if not m:
                continue
            acc[m.group(1)][row["Counter_Name"]].append(float(row["Counter_Value"]))
names = sorted({c for k in acc.values() for c in k})
for k, cs in sorted(acc.items()):
    print(k)
    for c in names:
        if c in cs:
            v = cs[c]
            print(f"   {c:32s} {sum(v) / len(v):16.1f}  (n={len(v)})")
