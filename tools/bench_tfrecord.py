#!/usr/bin/env python3
"""Native TFRecord reader throughput (clips/s and decompressed GB/s) on
synthetic GZIP shards, per decoder-thread count.  One GPU consumes ~11k
clips/s x 196 KB at the InT headline (bench.py); the reader must keep ahead."""
import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "pathtracker-models_amd")]

from ptamd import tfrecord  # noqa: E402


def main():
    t = int(os.environ.get("T", 64))
    shards = int(os.environ.get("SHARDS", 16))
    per = int(os.environ.get("PER", 256))
    with tempfile.TemporaryDirectory() as d:
        paths = tfrecord.write_synthetic_shards(d, shards, per, t, seed=7)
        mb = sum(os.path.getsize(p) for p in paths) / 1e6
        res = {}
        for th in [int(x) for x in os.environ.get("THREADS", "1,2,4,8").split(",")]:
            t0 = time.perf_counter()
            n = 0
            with tfrecord.Reader(paths, t, threads=th, shuffle_buffer=0) as rd:
                for clips, _ in rd.batches(256, reuse=True):
                    n += len(clips)
            el = time.perf_counter() - t0
            res[th] = {"clips_per_s": round(n / el), "GB_per_s": round(n * t * 3072 / el / 1e9, 2)}
        print(json.dumps({"clips": shards * per, "frames": t, "gz_MB": round(mb, 1),
                          "threads": res}))


if __name__ == "__main__":
    main()
