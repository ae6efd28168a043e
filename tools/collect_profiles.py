#!/usr/bin/env python3
"""Copy measured GPU-test records into profiles/ (tracked) unedited.

The -m gpu tests write their measured parity numbers, stamped with the loaded
libraries' source-hash versions, to gpurun_out/parity_records.json
(tests/goldens.py record); gpurun merges gpurun_out/ back from the box.  This
copies that file to profiles/<tag>_parity_records.json byte for byte, plus the
pytest summary line of the run's log when one is given.

usage: python tools/collect_profiles.py TAG [pytest-log]
"""
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    tag = sys.argv[1]
    src = os.path.join(REPO, "gpurun_out", "parity_records.json")
    dst = os.path.join(REPO, "profiles", f"{tag}_parity_records.json")
    shutil.copyfile(src, dst)
    print("copied", src, "->", dst, f"({len(json.load(open(dst)))} records)")
    if len(sys.argv) > 2:
        lines = [ln for ln in open(sys.argv[2]) if " passed" in ln or " failed" in ln]
        with open(os.path.join(REPO, "profiles", f"{tag}_gpu_tests_summary.txt"), "w") as f:
            f.write(lines[-1] if lines else "no summary line\n")


if __name__ == "__main__":
    main()
