"""InT — drop-in for the reference ``models/InT.py`` on MI355X.

Same class names, constructor signatures, ``forward`` signature / return
tuple and ``state_dict`` keys as the reference (``rCell`` models/InT.py:58-143,
``InT`` :182-245), and the same parameter initialisation performed in the same
RNG order, so a given ``torch.manual_seed`` yields the reference's initial
weights and checkpoints interchange.  What differs is the execution: the
T-frame recurrence and its BPTT run as hand-written gfx950 kernels behind the
C-ABI of ``include/pt_cell.h`` (see ``ptamd/cell.py``), and so does the readout
head (:236-241: ``readout_conv``, the target channel, ``target_conv``, the
global mean and ``readout_dense`` as one forward and one backward kernel per
clip, ``include/pt_readout.h`` / ``ptamd/readout.py``); the loss and the
optimizer stay in PyTorch.

Precision: ``InT.cell_dtype`` selects the cell's storage / MFMA operand type:
``'f32'`` (exact-f32 MFMA, the parity path; default, or env PT_CELL_DTYPE) or
``'bf16'`` (bf16 operands and saved states, f32 accumulation and f32
element-wise math; the throughput path).
"""
import os

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.nn import init

from ptamd import readout as ro
from ptamd.cell import PARAM_KEYS, CellConfig, run_cell, target_channel

_DEFAULT_DTYPE = os.environ.get("PT_CELL_DTYPE", "f32")


def _act_name(nl):
    if nl in (F.softplus,):
        return "softplus"
    if nl in (F.tanh, torch.tanh):
        return "tanh"
    raise NotImplementedError(f"nl={nl!r}: the HIP cell implements softplus and tanh")


class rCell(nn.Module):
    """InT recurrent cell parameters (reference models/InT.py:58-143).

    Registration and RNG order follow the reference: attention gates, the four
    E/I gates, w_exc, w_inh, the per-channel parameters, the two BatchNorms,
    then the orthogonal re-initialisations and bias constants.
    """

    def __init__(self, hidden_size, kernel_size, timesteps, batchnorm=True, grad_method='bptt',
                 use_attention=False, no_inh=False, lesion_alpha=False, lesion_gamma=False,
                 lesion_mu=False, lesion_kappa=False):
        super().__init__()
        self.padding = kernel_size // 2
        self.hidden_size = hidden_size
        self.batchnorm = batchnorm
        self.timesteps = timesteps
        self.use_attention = use_attention
        self.no_inh = no_inh
        self.h_padding = kernel_size // 2
        c = hidden_size

        if use_attention:
            self.a_w_gate = nn.Conv2d(c, c, 1)
            self.a_u_gate = nn.Conv2d(c, c, 1)
            for g in (self.a_w_gate, self.a_u_gate):
                init.orthogonal_(g.weight)
            for g in (self.a_w_gate, self.a_u_gate):
                init.constant_(g.bias, 1.)
        for name in ("i_w_gate", "i_u_gate", "e_w_gate", "e_u_gate"):
            setattr(self, name, nn.Conv2d(c, c, 1))

        self.w_exc = nn.Parameter(torch.empty(c, c, kernel_size, kernel_size))
        init.orthogonal_(self.w_exc)
        if not no_inh:
            self.w_inh = nn.Parameter(torch.empty(c, c, kernel_size, kernel_size))
            init.orthogonal_(self.w_inh)
        # per-channel parameters, shape [C,1,1]; `w` is registered but unused
        # by the reference (torch.empty there; zero-filled here, it gets no grad)
        for name in ("alpha", "mu", "gamma", "kappa", "w"):
            setattr(self, name, nn.Parameter(torch.zeros((c, 1, 1))))
        self.bn = nn.ModuleList([nn.BatchNorm2d(c, eps=1e-03, affine=True,
                                                track_running_stats=False) for _ in range(2)])
        for g in (self.i_w_gate, self.i_u_gate, self.e_w_gate, self.e_u_gate):
            init.orthogonal_(g.weight)
        for bn in self.bn:
            init.constant_(bn.weight, 0.1)
        if not no_inh:
            init.constant_(self.alpha, 1.)
            init.constant_(self.mu, 0.)
        init.constant_(self.gamma, 0.)
        init.constant_(self.kappa, 1.)
        if use_attention:
            self.i_w_gate.bias.data = -self.a_w_gate.bias.data
            self.e_w_gate.bias.data = -self.a_w_gate.bias.data
            self.i_u_gate.bias.data = -self.a_u_gate.bias.data
            self.e_u_gate.bias.data = -self.a_u_gate.bias.data
        else:
            init.uniform_(self.i_w_gate.bias.data, 1, self.timesteps - 1)
            self.e_w_gate.bias.data = -self.i_w_gate.bias.data
            self.e_u_gate.bias.data = -self.i_u_gate.bias.data
        # lesions only freeze the parameter (the reference's `.weight = 0.` is an
        # inert attribute; values stay at their init, models/InT.py:132-143)
        for flag, name in ((lesion_alpha, "alpha"), (lesion_mu, "mu"),
                           (lesion_gamma, "gamma"), (lesion_kappa, "kappa")):
            if flag:
                getattr(self, name).requires_grad = False

    def forward(self, input_, inhibition, excitation, activ=F.softplus, testmode=False):
        """One frame step (reference models/InT.py:145-179), for callers that
        step the cell themselves.  ``InT.forward`` never calls this: its whole
        T-frame recurrence and BPTT run fused in the HIP library.  The step is
        the reference's own op graph (1x1 gate convs, k x k convs, batch-stat
        BatchNorm) as device-agnostic torch ops, so it runs wherever its
        arguments live and autograd differentiates it."""
        if self.use_attention:
            att_gate = torch.sigmoid(self.a_w_gate(input_) + self.a_u_gate(excitation))
            gated_excitation = att_gate * excitation
        else:
            att_gate = None
            gated_excitation = excitation
        gated_input = input_
        gated_inhibition = inhibition
        if not self.no_inh:
            inh_intx = self.bn[0](F.conv2d(gated_excitation, self.w_inh, padding=self.h_padding))
            inhibition_hat = activ(input_ - activ(inh_intx * (self.alpha * gated_inhibition + self.mu)))
            inh_gate = torch.sigmoid(self.i_w_gate(gated_input) + self.i_u_gate(gated_inhibition))
            inhibition = (1 - inh_gate) * inhibition + inh_gate * inhibition_hat
        else:
            inhibition, gated_inhibition = gated_excitation, excitation
        exc_gate = torch.sigmoid(self.e_w_gate(gated_inhibition) + self.e_u_gate(gated_excitation))
        exc_intx = self.bn[1](F.conv2d(inhibition, self.w_exc, padding=self.h_padding))
        excitation_hat = activ(exc_intx * (self.kappa * inhibition + self.gamma))
        excitation = (1 - exc_gate) * excitation + exc_gate * excitation_hat
        if testmode:
            return inhibition, excitation, att_gate
        return inhibition, excitation


class InT(nn.Module):
    """InT model (reference models/InT.py:182-245)."""

    def __init__(self, dimensions, timesteps=8, kernel_size=15, jacobian_penalty=False,
                 grad_method='bptt', no_inh=False, lesion_alpha=False, lesion_mu=False,
                 lesion_gamma=False, lesion_kappa=False, nl=F.softplus):
        super().__init__()
        self.timesteps = timesteps
        self.jacobian_penalty = jacobian_penalty
        self.grad_method = grad_method
        self.hgru_size = dimensions
        self.preproc = nn.Conv3d(3, dimensions, kernel_size=1)
        self.unit1 = rCell(hidden_size=dimensions, kernel_size=kernel_size, use_attention=True,
                           no_inh=no_inh, lesion_alpha=lesion_alpha, lesion_mu=lesion_mu,
                           lesion_gamma=lesion_gamma, lesion_kappa=lesion_kappa,
                           timesteps=timesteps)
        self.readout_conv = nn.Conv2d(dimensions, 1, 1)
        self.target_conv = nn.Conv2d(2, 1, 5, padding=2)
        torch.nn.init.zeros_(self.target_conv.bias)
        self.readout_dense = nn.Linear(1, 1)
        self.nl = nl
        self.kernel_size = kernel_size
        self.no_inh = no_inh
        self.cell_dtype = _DEFAULT_DTYPE
        # ptamd.dist.CellDist: SyncBN / early-gradient all-reduce (None: per-replica BN)
        self.cell_dist = None

    def cell_config(self):
        return CellConfig(ksize=self.kernel_size, act=_act_name(self.nl), no_inh=self.no_inh,
                          cell="int", dtype=self.cell_dtype)

    def cell_params(self):
        sd = dict(self.named_parameters())
        return [sd.get(k) for k in PARAM_KEYS]

    def readout(self, e_last, x):
        """models/InT.py:236-241 (fused HIP kernels on ROCm tensors: ptamd/readout.py)"""
        return ro.readout(e_last, target_channel(x), self.readout_conv, self.target_conv,
                          self.readout_dense)

    # forward also takes the raw u8 clips [B,T,H,W,3] (engine.prepare_data
    # keep_u8): the kernels convert them exactly as prepare_data would
    accepts_u8 = True

    def forward(self, x, testmode=False):
        e_last, e_seq, gates = run_cell(x, self.cell_params(), self.cell_config(),
                                        want_seq=testmode,
                                        cdist=self.cell_dist)
        output = self.readout(e_last, x)
        if testmode:
            b, t, c, h, w = e_seq.shape
            states = self.readout_conv(e_seq.reshape(b * t, c, h, w)).reshape(b, t, 1, h, w)
            return output, states, gates
        jv_penalty = torch.ones(1, device=x.device)
        return output, jv_penalty


class FC(nn.Module):
    """Feed-forward control of the reference (models/InT.py:248-271; registry
    'fc', utils/engine.py:154-161): 1x1x1 conv stem, BatchNorm3d with batch
    statistics, one Linear over the whole clip.  Plain PyTorch (MIOpen /
    hipBLASLt on the GPU): it is a comparison model, not the recurrent hot
    path.  The Linear is sized for 64-frame 32x32 clips with 32 channels, as in
    the reference (``nn.Linear(64*32*32*32, 1)``, :260)."""

    def __init__(self, dimensions, timesteps=8, kernel_size=15, jacobian_penalty=False,
                 grad_method='bptt'):
        super().__init__()
        self.timesteps = timesteps
        self.jacobian_penalty = jacobian_penalty
        self.grad_method = grad_method
        self.hgru_size = dimensions
        self.bn = nn.BatchNorm3d(self.hgru_size, eps=1e-03, track_running_stats=False)
        self.preproc = nn.Conv3d(3, dimensions, kernel_size=1)
        self.readout = nn.Linear(64 * 32 * 32 * 32, 1)

    def forward(self, x, testmode=False):
        x = self.preproc(x)
        x = self.bn(x)
        x = self.readout(x.reshape(x.shape[0], -1))
        jv_penalty = torch.ones(1, device=x.device)
        return x, jv_penalty
