#!/usr/bin/env python3
"""One cell forward+backward (no optimizer) for counter collection under rocprofv3."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "pathtracker-models_amd")]
import torch  # noqa: E402
from models import InT as int_mod  # noqa: E402

b = int(os.environ.get("B", 256)); t = int(os.environ.get("T", 8))
dev = torch.device("cuda:0")
torch.manual_seed(0)
m = int_mod.InT(dimensions=32, timesteps=t, kernel_size=7).to(dev)
m.cell_dtype = os.environ.get("DT", "bf16")
x = torch.rand(b, 3, t, 32, 32, device=dev)
for _ in range(2):
    out, _ = m(x)
    out.sum().backward()
torch.cuda.synchronize()
print("ok")
