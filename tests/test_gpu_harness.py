"""The training harness end to end on the GPU: synthetic GZIP TFRecord shards
-> native reader -> prepare_data -> InT / FFhGRU (HIP cell) -> BCE -> BPTT ->
Adam -> 4-batch validation -> EarlyStopping checkpoint (mainclean.py)."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("model", ["InT", "ffhgru"])
def test_mainclean_two_epochs(tmp_path, model):
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    import mainclean
    data, res = tmp_path / "data", tmp_path / "res"
    out = mainclean.main(["--model", model, "--name", "smoke", "--dist", "14", "--speed", "1",
                          "--length", "8", "-b", "4", "--epochs", "2", "--print-freq", "1",
                          "--data-root", str(data), "--synthetic", "16",
                          "--results-root", str(res), "--max-iters", "3"])
    tr, va = out["train"], out["val"]
    assert len(tr["loss"]) == 6 and all(np.isfinite(tr["loss"]))
    assert len(va["loss"]) == 2 and all(np.isfinite(va["loss"]))
    assert all(0.0 <= a <= 100.0 for a in tr["balacc"])
    folder = out["results_folder"]
    assert os.path.exists(os.path.join(folder, "hp_dict.npz"))
    assert os.path.exists(folder + "train.npz") and os.path.exists(folder + "smoke.txt")
    ck = [f for f in os.listdir(folder) if f.endswith("_checkpoint.pth.tar")]
    assert ck, os.listdir(folder)
    sd = torch.load(os.path.join(folder, ck[0]), map_location="cpu", weights_only=True)
    assert "unit1.w_exc" in sd and all(torch.isfinite(v).all() for k, v in sd.items() if k != "unit1.w")
