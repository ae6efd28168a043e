#!/usr/bin/env python3
"""utils/TFRDataset.tfr_data_loader throughput (what mainclean.py sees): clips/s
with / without the shuffle buffer, pinned ring on or off."""
import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "pathtracker-models_amd")]

from ptamd import tfrecord  # noqa: E402
from utils.TFRDataset import tfr_data_loader  # noqa: E402


def main():
    shards, per, t, b = (int(os.environ.get(k, v)) for k, v in
                         (("SHARDS", 16), ("PER", 256), ("T", 64), ("B", 256)))
    with tempfile.TemporaryDirectory() as d:
        tfrecord.write_synthetic_shards(d, shards, per, t, seed=7, prefix="train")
        res = {}
        for name, kw in (("shuffle1000_pinned", dict(shuffle_buffer=1000, pin_memory=True)),
                         ("shuffle1000", dict(shuffle_buffer=1000, pin_memory=False)),
                         ("noshuffle", dict(shuffle_buffer=0, pin_memory=False))):
            try:
                ld = tfr_data_loader(d + "/train-*", b, timesteps=t, **kw)
                t0, n = time.perf_counter(), 0
                for x, y in ld:
                    n += len(y)
                res[name] = round(n / (time.perf_counter() - t0))
            except Exception as e:               # e.g. no device to pin for
                res[name] = repr(e)[:80]
        print(json.dumps({"clips": shards * per, "batch": b, "clips_per_s": res}))


if __name__ == "__main__":
    main()
