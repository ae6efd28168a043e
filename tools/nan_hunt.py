#!/usr/bin/env python3
"""Train the bf16 InT cell on changing synthetic batches (as mainclean.py does)
and stop at the first non-finite loss or gradient: report the step, which
gradients are bad, and whether replaying that step (same parameters, same
batch) reproduces it with and without hipGraph replay."""
import copy
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "pathtracker-models_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from models import InT  # noqa: E402


def main():
    steps, b, t = int(os.environ.get("STEPS", 60)), 256, 64
    dev = torch.device("cuda:0")
    torch.manual_seed(1234)
    m = InT.InT(dimensions=32, timesteps=t, kernel_size=7).to(dev)
    m.cell_dtype = os.environ.get("DT", "bf16")
    opt = torch.optim.Adam(m.parameters(), lr=3e-4)
    crit = torch.nn.BCEWithLogitsLoss()
    nb = int(os.environ.get("NB", 8))
    data = [bench.make_data(500 + i, b, t, dev) for i in range(nb)]

    def run(x, y):
        out, _ = m(x)
        loss = crit(out, y.reshape(-1, 1))
        loss.backward()
        return loss, out

    for s in range(steps):
        x, y = data[s % nb]
        snap = (copy.deepcopy(m.state_dict()), copy.deepcopy(opt.state_dict()))
        loss, out = run(x, y)
        bad = [k for k, p in m.named_parameters() if p.grad is not None and not torch.isfinite(p.grad).all()]
        if not torch.isfinite(loss) or bad:
            print(f"step {s}: loss {loss.item()} logits finite {bool(torch.isfinite(out).all())} "
                  f"bad grads {bad}", flush=True)
            for mode in ("graph", "nograph", "graph"):
                os.environ["PT_CELL_GRAPH"] = "0" if mode == "nograph" else "1"
                m.load_state_dict(snap[0])
                opt.zero_grad(set_to_none=True)
                loss2, out2 = run(x, y)
                bad2 = [k for k, p in m.named_parameters()
                        if p.grad is not None and not torch.isfinite(p.grad).all()]
                print(f"  replay ({mode}): loss {loss2.item()} bad grads {bad2}", flush=True)
            return
        opt.step()
        opt.zero_grad(set_to_none=True)
        if s % 10 == 0:
            print(f"step {s}: loss {loss.item():.5f}", flush=True)
    print("no non-finite values in", steps, "steps")


if __name__ == "__main__":
    main()
