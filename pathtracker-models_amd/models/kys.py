"""ConvGRU comparison baseline (reference models/kys.py; registry name 'gru').

A stock-PyTorch module (the convolutions run on MIOpen on MI355X): this is the
feedforward/recurrent *comparison* path of BASELINE.json configs[4]
(SURVEY.md §8(f) item 4), not the hand-written hot path.  Same class names,
constructor arguments, submodule names (so ``state_dict`` keys match the
reference's), forward signature and return values.

  ConvGRUCell (kys.py:7-48): r = sig(W_r*[x,h]), z = sig(W_z*[x,h]),
      n = tanh(W_n*[x, r*h]), h' = (1-z) h + z n     (k x k convs with bias)
  GRU (kys.py:70-135): xbn = softplus(Conv3d_1x1x1(x)); h_0 = 0; the cell over
      the T frames; readout exactly as InT: readout_conv(h_T) ++ x[:,2,0] ->
      target_conv 5x5 -> global mean -> Linear(1, 1).  The registry builds it
      with 2 x dimensions channels and the engine's kernel size (engine.py:147-153).
"""
import torch
import torch.nn.functional as F
from torch import nn


class ConvGRUCell(nn.Module):
    def __init__(self, input_dim, hidden_dim, kernel_size, padding_mode='zeros'):
        super().__init__()
        if padding_mode != 'zeros':
            raise NotImplementedError("only zero padding (the GRU's own setting, kys.py:79) "
                                      "is provided")
        self.hidden_dim = hidden_dim
        k = kernel_size if isinstance(kernel_size, (list, tuple)) else (kernel_size, kernel_size)
        pad = (k[0] // 2, k[1] // 2)
        cin = input_dim + hidden_dim
        self.conv_reset = nn.Conv2d(cin, hidden_dim, k, padding=pad)
        self.conv_update = nn.Conv2d(cin, hidden_dim, k, padding=pad)
        self.conv_state_new = nn.Conv2d(cin, hidden_dim, k, padding=pad)

    def forward(self, input, state_cur, testmode=False):
        xh = torch.cat([input, state_cur], dim=1)
        reset_gate = torch.sigmoid(self.conv_reset(xh))
        update_gate = torch.sigmoid(self.conv_update(xh))
        cand = torch.tanh(self.conv_state_new(torch.cat([input, reset_gate * state_cur], dim=1)))
        state_next = (1.0 - update_gate) * state_cur + update_gate * cand
        return (state_next, reset_gate) if testmode else state_next


class GRU(nn.Module):
    def __init__(self, dimensions, timesteps=8, kernel_size=15, jacobian_penalty=False,
                 grad_method='bptt'):
        super().__init__()
        self.timesteps = timesteps
        self.jacobian_penalty = jacobian_penalty
        self.grad_method = grad_method
        self.hgru_size = dimensions
        # registered but unused by forward (kys.py:79), kept for state_dict parity
        self.bn = nn.BatchNorm3d(dimensions, eps=1e-03, track_running_stats=False)
        self.preproc = nn.Conv3d(3, dimensions, kernel_size=1)
        self.unit1 = ConvGRUCell(input_dim=dimensions, hidden_dim=dimensions,
                                 kernel_size=kernel_size)
        self.readout_conv = nn.Conv2d(dimensions, 1, 1)
        self.target_conv = nn.Conv2d(2, 1, 5, padding=2)
        nn.init.zeros_(self.target_conv.bias)
        self.readout_dense = nn.Linear(1, 1)
        self.nl = F.softplus

    def forward(self, x, testmode=False):
        xbn = self.nl(self.preproc(x))
        b, c, t_len, h, w = xbn.shape
        exc = torch.zeros((b, c, h, w), dtype=xbn.dtype, device=x.device)
        states, gates = [], []
        for t in range(t_len):
            out = self.unit1(input=xbn[:, :, t], state_cur=exc, testmode=testmode)
            if testmode:
                exc, gate = out
                gates.append(gate)
                states.append(self.readout_conv(exc))
            else:
                exc = out
        output = torch.cat([self.readout_conv(exc), x[:, 2, 0][:, None]], 1)
        output = self.target_conv(output)
        output = F.avg_pool2d(output, kernel_size=output.size()[2:]).reshape(b, -1)
        output = self.readout_dense(output)
        jv_penalty = torch.ones(1, dtype=torch.float32, device=x.device)
        if testmode:
            return output, torch.stack(states, 1), torch.stack(gates, 1)
        return output, jv_penalty
