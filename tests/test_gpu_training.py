"""Many bf16 training steps through the cached hipGraphs (as mainclean.py runs
them): loss and every gradient stay finite.  Guards the class of bug where a
captured launch sequence replays differently from direct launches (a
hipMemsetAsync captured into the backward graph was not reliably ordered
before the kernels accumulating into the cleared buffer: non-finite
slab-derived gradients at step ~50 of a B=256 run; now a kernel node)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_bf16_training_stays_finite():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from models import InT
    from ptamd import synth
    dev = torch.device("cuda:0")
    torch.manual_seed(7)
    b, t = 128, 16
    m = InT.InT(dimensions=32, timesteps=t, kernel_size=7).to(dev)
    m.cell_dtype = "bf16"
    opt = torch.optim.Adam(m.parameters(), lr=3e-4)
    data = []
    for i in range(4):
        clips, labels = synth.make_batch(100 + i, b, t)
        x = torch.from_numpy(clips.transpose(0, 4, 1, 2, 3).astype(np.float32) / 255.0).to(dev)
        y = torch.tensor([ord(v) for v in labels], dtype=torch.float32, device=dev)
        data.append((x, y))
    for s in range(80):
        x, y = data[s % 4]
        x = x.clone()                      # fresh allocations, as prepare_data makes each step
        out, _ = m(x)
        loss = torch.nn.functional.binary_cross_entropy_with_logits(out, y.reshape(-1, 1))
        loss.backward()
        assert torch.isfinite(loss), f"step {s}: loss {loss.item()}"
        bad = [k for k, p in m.named_parameters() if p.grad is not None and not torch.isfinite(p.grad).all()]
        assert not bad, f"step {s}: non-finite grads {bad}"
        opt.step()
        opt.zero_grad(set_to_none=True)
