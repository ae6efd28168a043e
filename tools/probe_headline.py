"""Probe: what parameters give headline-size (B=256, T=64) logits that
straddle the accuracy thresholds, and how far bf16 sits from f32 there.

Trains the InT model for --steps Adam steps on the bench's clips (bf16 or f32
cell), printing the logit distribution as it goes, then compares the f32 and
bf16 cells at the trained parameters.  Investigation tool (GPU box)."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "pathtracker-models_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def stats(lo):
    lo = lo.double().flatten()
    return {"min": float(lo.min()), "max": float(lo.max()), "mean": float(lo.mean()),
            "gt0": int((lo > 0).sum()), "gt05": int((lo > 0.5).sum())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--nbatches", type=int, default=4)
    ap.add_argument("--out", default="gpurun_out/probe_headline.json")
    a = ap.parse_args()
    import bench
    from models import InT
    dev = torch.device("cuda:0")
    data = [bench.make_data(1000 + i, 256, 64, dev) for i in range(a.nbatches)]
    torch.manual_seed(1234)
    m = InT.InT(dimensions=32, timesteps=64, kernel_size=7).to(dev)
    m.cell_dtype = a.dtype
    opt = torch.optim.Adam(m.parameters(), lr=a.lr)
    log = []
    t0 = time.time()
    for s in range(a.steps):
        x, y = data[s % len(data)]
        out, _ = m(x)
        loss = F.binary_cross_entropy_with_logits(out, y.reshape(-1, 1))
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
        if s % 25 == 0 or s == a.steps - 1:
            acc = float(((out.detach() > 0).float().flatten() == y).float().mean())
            e = {"step": s, "loss": float(loss), "acc0": acc, **stats(out.detach())}
            log.append(e)
            print(json.dumps(e), f"{time.time() - t0:.1f}s", flush=True)
    x, y = data[0]
    res = {"train": log}
    with torch.no_grad():
        los = {}
        for dt in ("f32", "bf16"):
            m.cell_dtype = dt
            los[dt] = m(x)[0].double().flatten()
    err = (los["bf16"] - los["f32"]).abs()
    res["f32"] = stats(los["f32"])
    res["bf16_err_max"] = float(err.max())
    res["bf16_err_mean"] = float(err.mean())
    for thr in (0.0, 0.5):
        d = los["f32"] - thr
        res[f"flips_{thr}"] = int(((los["bf16"] > thr) != (los["f32"] > thr)).sum())
        res[f"near_{thr}_1e-2"] = int((d.abs() < 1e-2).sum())
    print(json.dumps(res), flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    torch.save({k: v.detach().cpu() for k, v in m.state_dict().items()},
               a.out.replace(".json", ".pt"))
    json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
