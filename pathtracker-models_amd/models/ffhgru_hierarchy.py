"""FFhGRU — drop-in for the reference ``models/ffhgru_hierarchy.py`` on MI355X.

Same class names, constructor signatures, ``forward`` signature / return tuple
and ``state_dict`` keys as the reference (``hConvGRUCell`` :58-173, ``FFhGRU``
:176-276), and the same parameter initialisation in the same RNG order.  The
cell differs from InT's only in its gated inhibition, which is the attention
map itself (:147); it runs through the same fused HIP kernels (``cell='hgru'``
in the C ABI), the readout (:258-272) stays in PyTorch.

The reference's Neumann-series ``dummyhgru`` Function (:11-57) is reachable
only through ``grad_method='rbp'``, which ``FFhGRU`` never wires in; BPTT is
the gradient here as there.
"""
import os

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.nn import init

from ptamd import readout as ro
from ptamd.cell import PARAM_KEYS, CellConfig, run_cell, target_channel

_DEFAULT_DTYPE = os.environ.get("PT_CELL_DTYPE", "f32")


class hConvGRUCell(nn.Module):
    """hGRU cell parameters (reference models/ffhgru_hierarchy.py:58-133).

    Registration and RNG order follow the reference: attention gates (+ their
    orthogonal init and bias 1), the four E/I gates (default init), w_exc,
    w_inh, the per-channel parameters, the two BatchNorms, then the orthogonal
    re-initialisations, constants and the bias ties of :127-131.
    """

    def __init__(self, hidden_size, kernel_size, timesteps, batchnorm=True, grad_method='bptt',
                 use_attention=False):
        super().__init__()
        self.padding = kernel_size // 2
        self.hidden_size = hidden_size
        self.batchnorm = batchnorm
        self.timesteps = timesteps
        self.use_attention = use_attention
        c = hidden_size
        if use_attention:
            self.a_w_gate = nn.Conv2d(c, c, 1)
            self.a_u_gate = nn.Conv2d(c, c, 1)
            init.orthogonal_(self.a_w_gate.weight)
            init.orthogonal_(self.a_u_gate.weight)
            init.constant_(self.a_w_gate.bias, 1.)
            init.constant_(self.a_u_gate.bias, 1.)
        for name in ("i_w_gate", "i_u_gate", "e_w_gate", "e_u_gate"):
            setattr(self, name, nn.Conv2d(c, c, 1))
        self.h_padding = kernel_size // 2
        self.w_exc = nn.Parameter(torch.empty(c, c, kernel_size, kernel_size))
        self.w_inh = nn.Parameter(torch.empty(c, c, kernel_size, kernel_size))
        # registered in the reference's order; `w` is unused by the cell
        for name in ("alpha", "gamma", "kappa", "w", "mu"):
            setattr(self, name, nn.Parameter(torch.zeros((c, 1, 1))))
        self.bn = nn.ModuleList([nn.BatchNorm2d(c, eps=1e-03, affine=True,
                                                track_running_stats=False) for _ in range(2)])
        init.orthogonal_(self.w_inh)
        init.orthogonal_(self.w_exc)
        for g in (self.i_w_gate, self.i_u_gate, self.e_w_gate, self.e_u_gate):
            init.orthogonal_(g.weight)
        for bn in self.bn:
            init.constant_(bn.weight, 0.1)
        init.constant_(self.alpha, 1.)
        init.constant_(self.mu, 0.)
        init.constant_(self.gamma, 0.)
        init.constant_(self.w, 1.)
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

    def forward(self, input_, inhibition, excitation, activ=F.softplus, testmode=False):
        """One frame step (reference models/ffhgru_hierarchy.py:135-173), for
        callers that step the cell themselves; ``FFhGRU.forward`` runs the
        fused HIP recurrence instead and never calls this.  Device-agnostic
        torch ops (the reference's op graph), differentiable by autograd.  The
        gated inhibition is the attention map itself (:147)."""
        if not self.use_attention:
            raise ValueError("hConvGRUCell.forward needs use_attention=True (the reference "
                             "leaves the gated tensors undefined otherwise, :141-148)")
        att_gate = torch.sigmoid(self.a_w_gate(input_) + self.a_u_gate(excitation))
        gated_input = input_
        gated_excitation = att_gate * excitation
        gated_inhibition = att_gate
        inh_intx = self.bn[0](F.conv2d(gated_excitation, self.w_inh, padding=self.h_padding))
        inhibition_hat = activ(input_ - activ(inh_intx * (self.alpha * gated_inhibition + self.mu)))
        inh_gate = torch.sigmoid(self.i_w_gate(gated_input) + self.i_u_gate(gated_inhibition))
        inhibition = (1 - inh_gate) * inhibition + inh_gate * inhibition_hat
        exc_gate = torch.sigmoid(self.e_w_gate(gated_inhibition) + self.e_u_gate(gated_excitation))
        exc_intx = self.bn[1](F.conv2d(inhibition, self.w_exc, padding=self.h_padding))
        excitation_hat = activ(exc_intx * (self.kappa * inhibition + self.gamma))
        excitation = (1 - exc_gate) * excitation + exc_gate * excitation_hat
        if testmode:
            return inhibition, excitation, att_gate
        return inhibition, excitation


class FFhGRU(nn.Module):
    """FFhGRU model (reference models/ffhgru_hierarchy.py:176-276)."""

    def __init__(self, dimensions, timesteps=8, kernel_size=15, jacobian_penalty=False,
                 grad_method='bptt'):
        super().__init__()
        self.timesteps = timesteps
        self.jacobian_penalty = jacobian_penalty
        self.grad_method = grad_method
        self.hgru_size = dimensions
        # registered (and initialised) but never applied by the reference (:215)
        self.bn = nn.BatchNorm3d(self.hgru_size, eps=1e-03, track_running_stats=False)
        self.preproc = nn.Conv3d(3, dimensions, kernel_size=1)
        self.unit1 = hConvGRUCell(hidden_size=dimensions, kernel_size=kernel_size,
                                  use_attention=True, timesteps=timesteps)
        self.readout_conv = nn.Conv2d(dimensions, 1, 1)
        self.target_conv = nn.Conv2d(2, 1, 5, padding=2)
        torch.nn.init.zeros_(self.target_conv.bias)
        self.readout_dense = nn.Linear(1, 1)
        self.nl = F.softplus
        self.kernel_size = kernel_size
        self.cell_dtype = _DEFAULT_DTYPE
        # ptamd.dist.CellDist: SyncBN / early-gradient all-reduce (None: per-replica BN)
        self.cell_dist = None

    def cell_config(self):
        return CellConfig(ksize=self.kernel_size, act="softplus", no_inh=False, cell="hgru",
                          dtype=self.cell_dtype)

    def cell_params(self):
        sd = dict(self.named_parameters())
        return [sd.get(k) for k in PARAM_KEYS]

    def readout(self, e_last, x):
        """models/ffhgru_hierarchy.py:258-272 (fused HIP kernels on ROCm tensors)"""
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
