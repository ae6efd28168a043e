"""Training metrics (reference utils/misc_functions.py:12-45), vectorised.

Same definitions as the reference, without its per-sample Python loop and its
hard ``.cuda()``: everything stays on the logits' device.
  pred     = logit > 0.5            (misc_functions.py:41; eval uses > 0, test_model.py:127)
  balacc   = #correct / B           (:25, the reference's "bacc" is plain accuracy)
  precision= tp / max(#pred, 1e-6)  (:19-24)
  recall   = tp / B                 (:18,22 — P is the batch size, not #positives)
  f1       = 2 tp / (B + #pred)     (:26)
"""
import torch


def metric_scores(target, pred):
    """target, pred: uint8 {0,1} tensors of shape [B] on the same device."""
    correct = pred.eq(target)
    tp = correct[target == 1].sum().float()
    p = target.shape[0]
    tpfp = pred.sum().float()
    if tpfp.item() == 0:
        tpfp = torch.tensor(1e-6, device=pred.device)
    recall = tp / p
    precision = tp / tpfp
    bacc = correct.sum() / float(p)
    f1s = (2 * tp) / (p + tpfp)
    return bacc, precision, recall, f1s


def acc_scores(target, prediction, threshold=0.5):
    """(balacc*100, precision, recall, f1) of logits ``prediction`` [B,1] vs labels [B]."""
    target = target.reshape(-1).to(prediction.device).byte()
    pred = (prediction.reshape(-1) > threshold).byte()
    balacc, precision, recall, f1s = metric_scores(target, pred)
    return balacc * 100, precision, recall, f1s


class AverageMeter(object):
    """Current value, running average and history (misc_functions.py:117-135)."""

    def __init__(self):
        self.reset()

    def reset(self):
        self.history = []
        self.val = 0
        self.avg = 0
        self.sum = 0
        self.count = 0

    def update(self, val, n=1):
        self.history.append(val)
        self.val = val
        self.sum += val * n
        self.count += n
        self.avg = self.sum / self.count
