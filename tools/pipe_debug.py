#!/usr/bin/env python3
"""Where does the input pipeline's time go inside a training process?  Times
the native Reader.next calls (producer thread) and the consumer's waits while
InT training steps run on the GPU."""
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "pathtracker-models_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from ptamd import tfrecord  # noqa: E402
from utils import TFRDataset  # noqa: E402


def main():
    b, t = 256, 64
    d = tempfile.mkdtemp()
    tfrecord.write_synthetic_shards(d, 16, 256, t, seed=3, prefix="train")
    times = []
    orig = tfrecord.Reader.next

    def timed_next(self, batch, out=None):
        t0 = time.perf_counter()
        r = orig(self, batch, out)
        times.append(time.perf_counter() - t0)
        return r
    tfrecord.Reader.next = timed_next
    mode = os.environ.get("MODE", "gpu")
    if mode == "gpu":
        from models import InT
        m = InT.InT(dimensions=32, timesteps=t, kernel_size=7).cuda()
        m.cell_dtype = "bf16"
        opt = torch.optim.Adam(m.parameters(), lr=3e-4)
    waits = []
    ld = TFRDataset.tfr_data_loader(d + "/train-*", b, timesteps=t)
    t_end = time.perf_counter()
    for i, (x, y) in enumerate(ld):
        waits.append(time.perf_counter() - t_end)
        if mode == "gpu":
            xx = torch.from_numpy(np.asarray(x)).cuda().permute(0, 4, 1, 2, 3).float().div_(255)
            out, _ = m(xx)
            out.sum().backward()
            opt.step()
            opt.zero_grad()
            torch.cuda.synchronize()
        elif mode == "sleep":
            time.sleep(0.03)
        t_end = time.perf_counter()
        if i >= 14:
            break
    print(mode, "reader.next ms", [round(1e3 * v, 1) for v in times[:16]])
    print(mode, "consumer wait ms", [round(1e3 * v, 1) for v in waits])


if __name__ == "__main__":
    main()
