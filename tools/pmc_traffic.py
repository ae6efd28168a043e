#!/usr/bin/env python3
"""Per-kernel HBM traffic from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

Correction per /opt/skills/guides/MI355X_MICROARCH.md §HBM: counters are in KB;
on gfx950 FETCH_SIZE reports half the bytes of wide coalesced streaming reads,
so fetched bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE x 1024 is exact for
16-B/lane stores.  Writes profiles/<out>.json: {kernel: {launches,
fetch_bytes, write_bytes, traffic_bytes}} averaged per launch.

usage: pmc_traffic.py FETCH_DIR WRITE_DIR OUT_JSON [note]

The summary is stamped with the version string of the in-tree libptcell.so
(it carries the hash of the kernel sources): bench.py only uses a summary whose
stamp matches the library it runs.
"""
import collections
import csv
import glob
import json
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pathtracker-models_amd"))


def _short(name):
    m = re.search(r"(k_[a-z_0-9]+)", name)
    return m.group(1) if m else name[:60]


def _read(d, counter):
    acc = collections.defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] == counter:
                acc[_short(row["Kernel_Name"])].append(float(row["Counter_Value"]))
    return acc


def main():
    fd, wd, out = sys.argv[1:4]
    note = sys.argv[4] if len(sys.argv) > 4 else ""
    fe, wr = _read(fd, "FETCH_SIZE"), _read(wd, "WRITE_SIZE")
    from ptamd import _lib
    res = {"note": note, "lib_version": _lib.load().pt_version().decode(),
           "correction": "fetch_bytes = 2*FETCH_SIZE*1024; write_bytes = WRITE_SIZE*1024",
           "kernels": {}}
    for k in sorted(set(fe) | set(wr)):
        f = 2 * 1024 * sum(fe.get(k, [0])) / max(len(fe.get(k, [])), 1)
        w = 1024 * sum(wr.get(k, [0])) / max(len(wr.get(k, [])), 1)
        res["kernels"][k] = {"launches": max(len(fe.get(k, [])), len(wr.get(k, []))),
                             "fetch_bytes": round(f), "write_bytes": round(w), "traffic_bytes": round(f + w)}
    json.dump(res, open(out, "w"), indent=1)
    for k, v in res["kernels"].items():
        print(f"{k:28s} n={v['launches']:5d} fetch {v['fetch_bytes']/1e6:9.2f} MB  write {v['write_bytes']/1e6:9.2f} MB")


if __name__ == "__main__":
    main()
