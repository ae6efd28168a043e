"""ConvLSTM — drop-in for the reference ``models/convlstm.py`` on MI355X.

Same class names, constructor signatures, ``forward`` signatures / return
tuples and ``state_dict`` keys as the reference (``dummyhgru`` :9-54,
``ConvLSTMCell`` :57-90, ``ConvLSTM`` :93-166), and the same parameter
initialisation in the same RNG order (conv0 is registered, then overwritten
by the Gabor bank, :103-106; conv6 gets xavier-normal weights and a
log(99) bias, :112-114).

The recurrence runs in the HIP library ``libptlstm.so`` (include/pt_lstm.h)
through ``ptamd.lstm.LSTMStepsFn``: with ``grad_method='bptt'`` the whole
``timesteps``-step loop (:137-143) and its BPTT are two library calls, and
the training-mode Jacobian penalty (:150-161) a third.  conv0 + pow (:118-119),
BN (:146), conv6 (:147) and the criterion stay in PyTorch.  The cell-level
``ConvLSTMCell.forward(x, h, c)`` is one library step with given states, so
``grad_method='rbp'`` (:124-135, Neumann-series backward in ``dummyhgru``)
works unchanged on top of it.

``jacobian_penalty=True`` (training, bptt): the reference builds the penalty
with ``create_graph`` (:158-162), so a loss that adds it (mainclean.py:195)
differentiates through the Jacobian of the last step.  The library runs the
first T-2 steps; the last two run as PyTorch ops (``ConvLSTMCell.torch_step``,
the reference's own cell arithmetic, :84-90) so that autograd holds the graph
the penalty needs: J_h = d h_T / d h_{T-1} and J_c = d c_T / d c_{T-1}, the
latter along every path (through h_{T-1} = o tanh c_{T-1} too), and their
parameter gradients reach the earlier steps through h_{T-2}, c_{T-2} (the
library's BPTT).  With the flag off ``jv_penalty`` is the library's detached
value, as the reference's (create_graph=False).  The image must be 32x32 and
``filt_size`` odd <= 15.
"""
import os

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.autograd import Function
from torch.nn import init

from ptamd import lstm
from ptamd import readout as ro
from ptamd.cell import target_channel
from ptamd.lstm import run_steps

_DEFAULT_DTYPE = os.environ.get("PT_CELL_DTYPE", "f32")
_GABOR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "utils",
                      "gabor_serre.npy")


class dummyhgru(Function):
    """Neumann-series recurrent back-propagation (reference models/convlstm.py:9-54).

    Forward passes ``last_state`` through; backward replaces its gradient by
    sum_k (J^T)^k g, J = d last_state / d state_2nd_last, truncated at
    ``truncate_iter`` terms or as soon as the series stops contracting
    (norm > 1, a growing term, or a vanishing one).
    """

    @staticmethod
    def forward(ctx, state_2nd_last, last_state, *args):
        ctx.save_for_backward(state_2nd_last, last_state)
        ctx.args = args
        return last_state

    @staticmethod
    def backward(ctx, grad):
        state_2nd_last, last_state = ctx.saved_tensors
        truncate_iter = ctx.args[-1]
        g_prev = grad.clone()
        v_prev = grad.clone()
        norm_v = [torch.norm(g_prev).item()]
        g = g_prev
        for _ in range(truncate_iter):
            v = torch.autograd.grad(last_state, state_2nd_last, grad_outputs=v_prev,
                                    retain_graph=True, allow_unused=True)[0]
            nv = torch.norm(v)
            g = g_prev + v
            ng = torch.norm(g)
            if ng > 1 or nv > norm_v[-1] or nv < 1e-9:
                g = g_prev
                break
            v_prev, g_prev = v, g
            norm_v.append(nv.item())
        return (None, g, None, None, None, None)


class ConvLSTMCell(nn.Module):
    """ConvLSTM cell parameters and one step (reference models/convlstm.py:57-90).

    x-convs carry a bias, h-convs do not; peephole weights Wci/Wcf/Wco are None
    as in the reference.  ``forward(x, h, c)`` runs one step on the device.
    """

    def __init__(self, input_channels, hidden_channels, kernel_size):
        super().__init__()
        self.input_channels = input_channels
        self.hidden_channels = hidden_channels
        self.kernel_size = kernel_size
        self.num_features = 4
        self.padding = int((kernel_size - 1) / 2)
        for g in ("i", "f", "c", "o"):
            setattr(self, f"Wx{g}", nn.Conv2d(self.input_channels, self.hidden_channels,
                                               self.kernel_size, 1, self.padding, bias=True))
            setattr(self, f"Wh{g}", nn.Conv2d(self.hidden_channels, self.hidden_channels,
                                               self.kernel_size, 1, self.padding, bias=False))
        self.Wci = None
        self.Wcf = None
        self.Wco = None
        self.cell_dtype = _DEFAULT_DTYPE

    def cell_weights(self):
        """[Wx_i..o, bx_i..o, Wh_i..o] in the order ptamd.lstm expects."""
        gs = ("i", "f", "c", "o")
        return ([getattr(self, f"Wx{g}").weight for g in gs]
                + [getattr(self, f"Wx{g}").bias for g in gs]
                + [getattr(self, f"Wh{g}").weight for g in gs])

    def steps(self, x, timesteps, h=None, c=None, want_jv=False, mu=0.9, want_seq=False):
        """``timesteps`` steps from (h, c) (None = zeros): (h_T, c_T, jv), plus
        every step's h [B,C,T,H,W] when ``want_seq``."""
        return run_steps(x, self.cell_weights(), ksize=self.kernel_size, steps=timesteps,
                         h0=h, c0=c, dtype=self.cell_dtype, want_jv=want_jv, mu=mu,
                         want_seq=want_seq)

    def forward(self, x, h, c):
        h_t, c_t, _ = self.steps(x, 1, h, c)
        return h_t, c_t

    def torch_step(self, x, h, c):
        """One step as PyTorch ops (reference convlstm.py:84-90): the graph the
        ``jacobian_penalty=True`` penalty differentiates (double backward)."""
        def gate(g, f):
            return f(getattr(self, f"Wx{g}")(x) + getattr(self, f"Wh{g}")(h))
        i_t = gate("i", torch.sigmoid)
        f_t = gate("f", torch.sigmoid)
        c_t = f_t * c + i_t * gate("c", torch.tanh)
        o_t = gate("o", torch.sigmoid)
        return o_t * torch.tanh(c_t), c_t


class ConvLSTM(nn.Module):
    """Reference models/convlstm.py:93-166 (static-image ConvLSTM, 25 channels)."""

    def __init__(self, timesteps=8, filt_size=15, num_iter=50, exp_name='exp1',
                 jacobian_penalty=False, grad_method='bptt'):
        super().__init__()
        self.timesteps = timesteps
        self.num_iter = num_iter
        self.exp_name = exp_name
        self.jacobian_penalty = jacobian_penalty
        self.grad_method = grad_method
        self.conv0 = nn.Conv2d(1, 25, kernel_size=7, padding=3)
        part1 = np.load(_GABOR, allow_pickle=False)
        self.conv0.weight.data = torch.FloatTensor(part1)
        self.unit1 = ConvLSTMCell(25, 25, filt_size)
        print("Training with filter size:", filt_size, "x", filt_size)
        self.bn = nn.BatchNorm2d(25, eps=1e-03, track_running_stats=False)
        self.conv6 = nn.Conv2d(25, 2, kernel_size=1)
        init.xavier_normal_(self.conv6.weight)
        init.constant_(self.conv6.bias, torch.log(torch.tensor((1 - 0.01) / 0.01)))

    @property
    def cell_dtype(self):
        return self.unit1.cell_dtype

    @cell_dtype.setter
    def cell_dtype(self, v):
        self.unit1.cell_dtype = v

    def forward(self, x, epoch, itr, target, criterion, testmode=False):
        x = self.conv0(x)
        x = torch.pow(x, 2)
        states = []
        jv_penalty = None
        if self.grad_method == 'rbp':
            internal_h = torch.zeros_like(x)
            internal_c = torch.zeros_like(x)
            with torch.no_grad():
                for _ in range(self.timesteps - 1):
                    if testmode:
                        states.append(internal_h)
                    internal_h, internal_c = self.unit1(x, internal_h, internal_c)
            if testmode:
                states.append(internal_h)
            state_2nd_last = internal_h.detach().requires_grad_()
            state_2nd_last_c = internal_c.detach().requires_grad_()
            # with jacobian_penalty the penalty keeps its graph (create_graph,
            # reference :158-162, both grad methods): that is a double backward
            # through the last step, so it runs as torch ops (torch_step), as
            # the bptt branch's last two steps do
            graph = self.training and self.jacobian_penalty
            step = self.unit1.torch_step if graph else self.unit1
            last_state, internal_c = step(x, state_2nd_last, state_2nd_last_c)
            internal_h = dummyhgru.apply(state_2nd_last, last_state, epoch, itr, self.exp_name,
                                         self.num_iter)
            if testmode:
                states.append(internal_h)
            if self.training:
                ones = torch.ones_like(last_state)
                jv = torch.autograd.grad(last_state, state_2nd_last, grad_outputs=[ones],
                                         retain_graph=True, create_graph=graph, allow_unused=True)[0]
                jv_penalty = (jv - 0.90).clamp(0) ** 2
                jv = torch.autograd.grad(internal_c, state_2nd_last_c, grad_outputs=[ones],
                                         retain_graph=True, create_graph=graph, allow_unused=True)[0]
                jv_penalty = jv_penalty + (jv - 0.90).clamp(0) ** 2
        elif self.grad_method == 'bptt':
            if self.training and self.timesteps < 2:
                raise RuntimeError("ConvLSTM training needs timesteps >= 2 (the reference's "
                                   "state_2nd_last is unbound otherwise, convlstm.py:140-161)")
            if self.training and self.jacobian_penalty:
                jv_penalty, internal_h = self._penalty_with_graph(x)
            else:
                internal_h, _, jv = self.unit1.steps(x, self.timesteps, want_jv=self.training)
                if self.training:
                    jv_penalty = jv
        else:
            raise ValueError(f"unknown grad_method {self.grad_method!r}")

        output = self.bn(internal_h)
        output = self.conv6(output)
        loss = criterion(output, target)
        if jv_penalty is None:
            jv_penalty = torch.tensor([1]).float().to(output.device)
        if testmode:
            return output, states, loss
        return output, jv_penalty, loss

    def _penalty_with_graph(self, x):
        """(jv_penalty with its graph, h_T): steps 1..T-2 in the library, the
        last two in PyTorch ops (module docstring; reference :137-162)."""
        lstm._require_device(x)              # the HIP path's rule: no CPU run of the model
        t = self.timesteps
        if t > 2:
            h, c, _ = self.unit1.steps(x, t - 2)
        else:
            h = c = torch.zeros_like(x)
        state_2nd_last, state_2nd_last_c = self.unit1.torch_step(x, h, c)
        last_state, internal_c = self.unit1.torch_step(x, state_2nd_last, state_2nd_last_c)
        ones = torch.ones_like(last_state)
        jv = torch.autograd.grad(last_state, state_2nd_last, grad_outputs=[ones],
                                 retain_graph=True, create_graph=True)[0]
        jv_penalty = (jv - 0.90).clamp(0) ** 2
        jv = torch.autograd.grad(internal_c, state_2nd_last_c, grad_outputs=[ones],
                                 retain_graph=True, create_graph=True)[0]
        return jv_penalty + (jv - 0.90).clamp(0) ** 2, last_state


class ConvLSTMVideo(nn.Module):
    """ConvLSTM on PathTracker clips: BASELINE configs[2] ("ConvLSTM ... same
    clips").  Not a reference class: the reference ConvLSTM recurs on ONE static
    image (convlstm.py:116-147), so the clip version is defined here
     from the reference's own parts:

    * stem      ``nl(Conv3d 1x1x1 3->C)`` per frame, as InT (InT.py:192,212-213);
    * recurrence ``ConvLSTMCell`` (convlstm.py:84-90) with the frame as input:
                 h_t, c_t = cell(x_t, h_{t-1}, c_{t-1}), h_0 = c_0 = 0; the
                 x-convs see a new frame each step (the library's x_seq mode);
    * readout   InT's (InT.py:236-241) on h_T: readout_conv C->1, the target
                 marker x[:, 2, 0], target_conv 5x5, global average, Linear(1,1);
    * jv_penalty the reference ConvLSTM's training-mode Jacobian penalty of the
                 last step (convlstm.py:150-161), detached, as ``ConvLSTM``.

    ``forward(x, testmode=False)`` has InT's signature and returns
    ``(logits [B,1], jv_penalty)``, so engine.model_step / mainclean.py run it
    (registry name ``convlstm``).  ``testmode=True`` returns, as InT's
    (InT.py:230-233,244), ``(logits, states [B,T,1,H,W], hidden [B,T,C,H,W])``:
    ``states`` = readout_conv(h_t) per frame; the third element, InT's
    attention maps there, is the per-frame hidden state h_t here (the
    reference ConvLSTM's testmode collects exactly those, convlstm.py:127-135;
    the cell has no attention gate).
    """

    def __init__(self, dimensions=25, timesteps=8, kernel_size=7, jacobian_penalty=False,
                 grad_method='bptt', nl=F.softplus):
        super().__init__()
        if grad_method != 'bptt':
            raise NotImplementedError("ConvLSTMVideo trains with BPTT only")
        if nl is not F.softplus:
            raise NotImplementedError("the HIP stem fuses F.softplus (InT's default nl)")
        self.timesteps = timesteps
        self.jacobian_penalty = jacobian_penalty
        self.grad_method = grad_method
        self.hgru_size = dimensions
        self.kernel_size = kernel_size
        self.nl = nl
        self.preproc = nn.Conv3d(3, dimensions, kernel_size=1)
        self.unit1 = ConvLSTMCell(dimensions, dimensions, kernel_size)
        self.readout_conv = nn.Conv2d(dimensions, 1, 1)
        self.target_conv = nn.Conv2d(2, 1, 5, padding=2)
        init.zeros_(self.target_conv.bias)
        self.readout_dense = nn.Linear(1, 1)

    @property
    def cell_dtype(self):
        return self.unit1.cell_dtype

    @cell_dtype.setter
    def cell_dtype(self, v):
        self.unit1.cell_dtype = v

    # forward also takes the raw u8 clips [B,T,H,W,3] (engine.prepare_data
    # keep_u8): the stem kernel converts them exactly as prepare_data would
    accepts_u8 = True

    def forward(self, x, testmode=False):
        # the 1x1x1 stem + softplus written straight into the recurrence's
        # per-step input (pt_lstm_forward_stem; r05: the f32 stem output and its
        # layout conversions, ~3 ms of a 45 ms step, no longer exist)
        steps = x.shape[1] if x.dtype == torch.uint8 else x.shape[2]
        want_jv = self.training and steps >= 2
        lstm._require_device(x)
        res = lstm.stem_steps(x, self.preproc.weight, self.preproc.bias, self.unit1.cell_weights(),
                              ksize=self.kernel_size, dtype=self.cell_dtype, want_jv=want_jv,
                              want_seq=testmode)
        h_t, jv = res[0], res[2]
        out = ro.readout(h_t, target_channel(x), self.readout_conv, self.target_conv,
                         self.readout_dense)                         # ptamd/readout.py
        if testmode:
            hidden = res[3].permute(0, 2, 1, 3, 4)                  # [B, T, C, H, W]
            b, t, c, h, w = hidden.shape
            states = self.readout_conv(hidden.reshape(b * t, c, h, w)).reshape(b, t, 1, h, w)
            return out, states, hidden
        jv_penalty = jv if want_jv else torch.ones(1, device=x.device)
        return out, jv_penalty
