"""EarlyStopping (reference utils/earlystopping.py:6-57), same semantics.

Called once per validation with the accuracy: the first call and every call
that does not fall below ``best + delta`` saves ``model.state_dict()`` as
``model_val_acc_{int(acc):04d}_epoch_{epoch:02d}_checkpoint.pth.tar`` in the
results folder; ``patience`` consecutive worse calls set ``early_stop``.
(``score < best + delta`` counts as worse, so an equal score re-saves, as in
the reference.)
"""
import os

import numpy as np
import torch


class EarlyStopping:
    def __init__(self, patience=7, verbose=False, delta=0, results_folder='checkpoint.pt',
                 trace_func=print):
        self.patience = patience
        self.verbose = verbose
        self.counter = 0
        self.best_score = None
        self.early_stop = False
        self.acc_min = np.inf
        self.delta = delta
        self.path = results_folder
        self.trace_func = trace_func
        os.makedirs(self.path, exist_ok=True)

    def __call__(self, acc, model, epoch):
        score = acc
        if self.best_score is None:
            self.best_score = score
            self.save_checkpoint(acc, model, epoch)
        elif score < self.best_score + self.delta:
            self.counter += 1
            self.trace_func(f'EarlyStopping counter: {self.counter} out of {self.patience}')
            if self.counter >= self.patience:
                self.early_stop = True
        else:
            self.best_score = score
            self.save_checkpoint(acc, model, epoch)
            self.counter = 0

    def save_checkpoint(self, acc, model, epoch):
        if self.verbose:
            self.trace_func(f'Validation acc increased ({self.acc_min:.6f} --> {acc:.6f}).  Saving model ...')
        filename = 'model_val_acc_{0:04d}_epoch_{1:02d}_checkpoint.pth.tar'.format(int(acc), epoch)
        torch.save(model.state_dict(), os.path.join(self.path, filename))
        self.acc_min = acc
