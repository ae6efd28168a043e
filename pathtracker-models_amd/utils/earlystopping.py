"""Validation-accuracy checkpointing with patience (the
reference's ``utils/earlystopping.py:6-57`` is the behaviour matched, the
code here is written from that description).

Behaviour kept for drop-in use by ``mainclean.py`` (reference call site
``mainclean.py:125,253``):

* ``EarlyStopping(patience, verbose, delta, results_folder, trace_func)``;
  the instance is called as ``es(acc, model, epoch)`` once per validation.
* A call "improves" unless ``acc < best + delta``: the first call and every
  improving call (an equal accuracy included) write ``model.state_dict()`` to
  ``<results_folder>/model_val_acc_{int(acc):04d}_epoch_{epoch:02d}_checkpoint.pth.tar``
  and reset the counter; any other call counts one strike, and ``patience``
  strikes in a row set ``early_stop``.
* Only the state_dict is stored (no optimizer state), as in the reference.
"""
import os

import torch

CKPT_NAME = "model_val_acc_{acc:04d}_epoch_{epoch:02d}_checkpoint.pth.tar"


class EarlyStopping:
    def __init__(self, patience=7, verbose=False, delta=0, results_folder="checkpoint.pt",
                 trace_func=print):
        self.patience, self.verbose, self.delta = patience, verbose, delta
        self.path = results_folder
        self.trace_func = trace_func
        self.best_score = None       # best accuracy seen (None before the first call)
        self.counter = 0             # consecutive non-improving calls
        self.early_stop = False
        self.last_saved = float("inf")   # accuracy of the last checkpoint (log line only)
        os.makedirs(self.path, exist_ok=True)

    def _improves(self, acc):
        return self.best_score is None or not acc < self.best_score + self.delta

    def __call__(self, acc, model, epoch):
        if self._improves(acc):
            self.best_score = acc
            self.counter = 0
            self.save_checkpoint(acc, model, epoch)
            return
        self.counter += 1
        self.trace_func(f"EarlyStopping counter: {self.counter} out of {self.patience}")
        self.early_stop = self.early_stop or self.counter >= self.patience

    def checkpoint_path(self, acc, epoch):
        return os.path.join(self.path, CKPT_NAME.format(acc=int(acc), epoch=epoch))

    def save_checkpoint(self, acc, model, epoch):
        if self.verbose:
            self.trace_func(f"Validation acc increased ({self.last_saved:.6f} --> {acc:.6f}).  "
                            "Saving model ...")
        torch.save(model.state_dict(), self.checkpoint_path(acc, epoch))
        self.last_saved = acc
