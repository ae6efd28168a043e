"""The training harness around the hot path (mainclean.py, utils/opts.py,
utils/engine.py dataset_selector / load_ckpt, utils/earlystopping.py,
AverageMeter), host logic only.  The loop itself runs on the GPU
(tests/test_gpu_harness.py): the cell has no CPU path."""
import os

import numpy as np
import pytest
import torch

from utils import engine
from utils.earlystopping import EarlyStopping
from utils.misc_functions import AverageMeter
from utils.opts import parser


def test_reference_launcher_flags_parse():
    # train_InT.sh:3
    a = parser.parse_args("-b 180 --model InT --length 64 --speed 1 --dist 14 --parallel".split())
    assert (a.batch_size, a.model, a.length, a.speed, a.dist, a.parallel) == (180, "InT", 64, 1, 14, True)
    assert (a.lr, a.dimensions, a.fb_kernel_size, a.epochs, a.print_freq) == (3e-4, 32, 7, 30, 100)
    assert a.data_root is None and a.synthetic == 0


def test_dataset_selector_table():
    # remote paths (no /gpfs here): timesteps = length; unknown keys fall through to None
    for (d, s, l) in [(14, 1, 128), (25, 1, 64), (14, 2, 64), (14, 4, 64), (14, 1, 64), (5, 1, 32)]:
        root, t, ntr, nva = engine.dataset_selector(d, s, l)
        assert t == l and (ntr, nva) == (20000, 20000) and root.endswith("/")
    assert "skip_param_4" in engine.dataset_selector(14, 4, 64)[0]
    assert "/5_dist/" in engine.dataset_selector(14, 1, 64)[0]      # the reference's fallback
    assert engine.dataset_selector(3, 3, 3) is None
    assert engine.dataset_selector(14, 1, 64, data_root="/tmp/pt")[:2] == ("/tmp/pt/", 64)


def test_average_meter():
    m = AverageMeter()
    for v in (1.0, 2.0, 6.0):
        m.update(v)
    assert (m.val, m.avg, m.count, m.history) == (6.0, 3.0, 3, [1.0, 2.0, 6.0])


def test_early_stopping_and_checkpoint_roundtrip(tmp_path):
    from models import InT as int_mod
    m = int_mod.InT(dimensions=32, timesteps=8, kernel_size=7)
    es = EarlyStopping(patience=2, results_folder=str(tmp_path), trace_func=lambda *_: None)
    es(50.0, m, 0)                      # first call saves
    es(40.0, m, 1)                      # worse: counter 1
    es(55.5, m, 2)                      # better: saves, counter reset
    es(10.0, m, 3)
    assert not es.early_stop
    es(10.0, m, 4)
    assert es.early_stop
    files = sorted(os.listdir(tmp_path))
    assert files == ["model_val_acc_0050_epoch_00_checkpoint.pth.tar",
                     "model_val_acc_0055_epoch_02_checkpoint.pth.tar"]
    # load_ckpt accepts the EarlyStopping file (bare state_dict; the reference's
    # own load_ckpt wants a 'state_dict' key) and the wrapped / DataParallel forms
    m2 = int_mod.InT(dimensions=32, timesteps=8, kernel_size=7)
    engine.load_ckpt(m2, str(tmp_path / files[-1]))
    for (k, v), (_, w) in zip(m.state_dict().items(), m2.state_dict().items()):
        if k != "unit1.w":              # torch.empty, never initialised (InT.py:100)
            assert torch.equal(v, w), k
    wrapped = tmp_path / "wrapped.pth"
    torch.save({"state_dict": {"module." + k: v for k, v in m.state_dict().items()}}, wrapped)
    engine.load_ckpt(int_mod.InT(dimensions=32, timesteps=8, kernel_size=7), str(wrapped))


def test_harness_requires_pt_config():
    import mainclean
    with pytest.raises(AssertionError):
        mainclean.main(["--model", "InT", "--speed", "1", "--length", "8"])
