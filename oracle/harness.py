"""CPU oracle for the hot path's callers — TEST INFRASTRUCTURE ONLY.

Literal numpy / Python-loop restatements of the reference's batch preparation
and training metrics, which the reference cannot import here (tensorflow,
torchvision, ``torch._six`` are absent).  Used by tests/ to
check ``pathtracker-models_amd/utils`` bit-for-bit.
"""
import numpy as np


def prepare_data(imgs_u8, target_bytes, disentangle_channels=False, pretrained=False):
    """utils/engine.py:220-255 (numpy half; the result is cast to float32 as ``.to(float)``)."""
    imgs = imgs_u8.transpose(0, 4, 1, 2, 3)                      # :223
    target = np.vectorize(ord)(target_bytes).astype(np.float32)   # :224-225
    imgs = imgs / 255.                                            # :226 (float64)
    if disentangle_channels:                                      # :228-233
        mask = imgs.sum(1).round()
        proc = np.zeros_like(imgs)
        proc[:, 1] = (mask == 1).astype(imgs.dtype)
        proc[:, 2] = (mask == 2).astype(imgs.dtype)
        proc[:, 0] = (mask == 3).astype(imgs.dtype)
    else:
        proc = imgs
    out = proc.astype(np.float32)                                 # :239-240
    if pretrained:                                                # :241-244 (float32 on device)
        mu = np.array([0.43216, 0.394666, 0.37645], np.float32)[None, :, None, None, None]
        sd = np.array([0.22803, 0.22145, 0.216989], np.float32)[None, :, None, None, None]
        out = (out - mu) / sd
    return out, target


def acc_scores(target, logits):
    """utils/misc_functions.py:32-45 with metric_scores :12-29, per-sample loop as written."""
    target = np.asarray(target).astype(np.uint8)
    pred = np.array([1 if float(v) > 0.5 else 0 for v in np.asarray(logits).reshape(-1)], np.uint8)
    correct = pred == target
    tp = float(correct[target == 1].sum())
    p = target.shape[0]
    tpfp = float(pred.sum())
    if tpfp == 0:
        tpfp = 1e-6
    return 100 * correct.sum() / float(p), tp / tpfp, tp / p, 2 * tp / (p + tpfp)
