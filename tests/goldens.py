"""Helpers to read the committed golden fixtures (data only; see tests/golden/make_golden.py)."""
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(tag):
    z = np.load(os.path.join(GOLDEN, f"{tag}.npz"), allow_pickle=False)
    return {k: z[k] for k in z.files}


def params(g, prefix="param."):
    return {k[len(prefix):]: torch.from_numpy(v.copy()) for k, v in g.items() if k.startswith(prefix)}


def prepared_input(g):
    """engine.prepare_data semantics (utils/engine.py:220-245): uint8 [B,T,H,W,3] ->
    float32 [B,3,T,H,W] / 255 (divide in float64 as numpy does, then cast)."""
    x = torch.from_numpy(g["clip_u8"].transpose(0, 4, 1, 2, 3) / 255.0).float()
    y = torch.from_numpy(g["label_u8"].astype(np.float64)).float()
    return x, y


def cfg(g):
    return dict(cell=str(g["cfg_cell"]), act=str(g["cfg_act"]), no_inh=bool(g["cfg_no_inh"]),
                lesion=[s for s in str(g["cfg_lesion"]).split(",") if s],
                dims=int(g["cfg_dims"]), k=int(g["cfg_k"]) if "cfg_k" in g else 7)


REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RECORDS = os.path.join(REPO, "gpurun_out", "parity_records.json")


def record(key, val):
    """Measured parity numbers of a GPU test -> gpurun_out/parity_records.json
    (merged per key, stamped with the loaded libraries' source-hash versions);
    tools/collect_profiles.py copies the file into profiles/ unedited."""
    import json
    import time
    stamp = {}
    try:
        from ptamd import _lib, lstm
        stamp = {"pt_cell": _lib.load().pt_version().decode(),
                 "pt_lstm": lstm.load().pt_lstm_version().decode()}
    except Exception:                  # a record never fails its test
        pass
    os.makedirs(os.path.dirname(RECORDS), exist_ok=True)
    cur = json.load(open(RECORDS)) if os.path.exists(RECORDS) else {}
    cur[key] = {**val, "lib": stamp, "utc": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())}
    with open(RECORDS, "w") as f:
        json.dump(cur, f, indent=1, sort_keys=True)
