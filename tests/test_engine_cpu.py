"""The hot path's callers (utils/engine.py, utils/misc_functions.py mirrors) on CPU.

Checked bit-for-bit against oracle/harness.py (numpy restatement of
reference utils/engine.py:220-255 and utils/misc_functions.py:12-45) and, for
the model registry, against the reference's constructor arguments
(utils/engine.py:77-146).
"""
import types

import numpy as np
import pytest
import torch

from oracle import harness
from ptamd import synth
from utils import engine
from utils.misc_functions import acc_scores


def _args(model, pretrained=False):
    return types.SimpleNamespace(model=model, algo="bptt", penalty=False, pretrained=pretrained)


@pytest.mark.parametrize("disentangle", [False, True])
@pytest.mark.parametrize("pretrained", [False, True])
def test_prepare_data_bit_exact(disentangle, pretrained):
    clips, labels = synth.make_batch(7, 3, 5)
    rng = np.random.default_rng(0)
    clips[0] = rng.integers(0, 256, clips[0].shape, dtype=np.uint8)    # every byte value
    x, y = engine.prepare_data(clips, labels, _args("InT", pretrained), "cpu", disentangle)
    xr, yr = harness.prepare_data(clips, labels, disentangle, pretrained)
    assert x.dtype == torch.float32 and tuple(x.shape) == xr.shape
    np.testing.assert_array_equal(x.numpy(), xr)
    np.testing.assert_array_equal(y.numpy(), yr)


def test_prepare_data_all_byte_values():
    u = np.arange(256, dtype=np.uint8).reshape(1, 1, 16, 16, 1).repeat(3, 4)
    x, _ = engine.prepare_data(u, np.array([b"\x01"], dtype=object), _args("InT"), "cpu", False)
    np.testing.assert_array_equal(x.numpy(), harness.prepare_data(u, np.array([b"\x01"], dtype=object))[0])


def test_acc_scores_matches_reference_loop():
    rng = np.random.default_rng(3)
    for b in (1, 7, 64):
        logits = rng.normal(0.5, 1.0, (b, 1)).astype(np.float32)
        logits[0, 0] = 0.5                                   # exactly at the threshold: not positive
        y = rng.integers(0, 2, b)
        got = [float(v) for v in acc_scores(torch.from_numpy(y).float(), torch.from_numpy(logits))]
        ref = harness.acc_scores(y, logits)
        np.testing.assert_allclose(got, ref, rtol=1e-6)
    # no positive predictions: precision divides by 1e-6 as in the reference
    got = acc_scores(torch.ones(4), torch.full((4, 1), -1.0))
    assert float(got[1]) == 0.0 and float(got[0]) == 0.0


@pytest.mark.parametrize("name", sorted(engine.INT_VARIANTS))
def test_model_selector_variants(name):
    torch.manual_seed(0)
    m = engine.model_selector(_args(name), timesteps=8, device="cpu")
    keys = list(m.state_dict())
    assert ("unit1.w_inh" in keys) == (name != "InT_no_inh")
    frozen = {n for n, p in m.named_parameters() if not p.requires_grad}
    lesions = {k for k, v in engine.INT_VARIANTS[name].items() if k.startswith("lesion") and v}
    assert frozen == {"unit1." + k[len("lesion_"):] for k in lesions}


def test_model_selector_unknown():
    with pytest.raises(NotImplementedError):
        engine.model_selector(_args("r3d"), timesteps=8, device="cpu")
