"""Multi-rank paths of the HIP cell on ONE GPU (2 processes, gloo on device
tensors): the cross-replica hooks of include/pt_cell.h (pt_cell_dist) through
ptamd.dist.CellDist, against the single-process HIP cell.

* SyncBN: 2 ranks x 2 clips with BatchNorm statistics all-reduced between
  the cell's launches reproduce the single process on all 4 clips (logits per
  clip, rank-averaged gradients) -- the library's per-reduction callback, the
  SyncBN totals kernel and the global clip count in every consumer; for the
  f32 cell (split forward kernels) and the bf16 cell (the fused forward
  segments, which read the all-rank totals through bnf_src; the banded
  backward convs).  bf16 tolerance: the two-rank totals are the same fp64
  sums in another association, so a bf16-stored value may round the other
  way.  r06: also the tiled hGRU (64 x 64, BatchNorm over clips x tiles).
* early-gradient overlap: with per-replica BatchNorm (the default) the
  gradients averaged in two parts -- the cell's early gradients on a side
  stream behind the event the backward records before its k x k
  weight-gradient kernel, the rest after backward -- or in three (r06: w_inh
  on the side stream behind the event recorded between w_inh's and w_exc's
  weight-gradient launches) equal the mean of the per-shard single-process
  gradients.
"""
import os
import socket

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model(tiled=False):
    from models import InT, ffhgru_hierarchy as hg
    torch.manual_seed(21)
    m = (hg.FFhGRU(dimensions=32, timesteps=4, kernel_size=7) if tiled
         else InT.InT(dimensions=32, timesteps=6, kernel_size=7))
    with torch.no_grad():
        for n, p in m.named_parameters():
            if (n.startswith("unit1.bn") and n.endswith("weight")) or n.endswith(("alpha", "kappa")):
                p.uniform_(0.5, 1.5)
            elif n.endswith(("mu", "gamma")):
                p.uniform_(-0.5, 0.5)
    return m


def _batch(tiled=False):
    from ptamd import synth
    clips, labels = (synth.make_batch(5, 4, 4, h=64, w=64) if tiled else synth.make_batch(5, 4, 6))
    x = torch.from_numpy(clips.transpose(0, 4, 1, 2, 3) / 255.0).float()
    return x, torch.tensor([ord(v) for v in labels], dtype=torch.float32)


def _worker(rank, world, port, sync_bn, out_q, dtype="f32", three_part=True, tiled=False):
    import sys
    sys.path[:0] = [os.path.join(REPO, "tests"), REPO, os.path.join(REPO, "pathtracker-models_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from ptamd.dist import CellDist, GradBucket
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m = _model(tiled).to(dev)
    m.cell_dtype = dtype
    x, y = _batch(tiled)
    sh = slice(2 * rank, 2 * rank + 2)
    bucket = GradBucket(m.parameters(), dev, three_part=three_part)
    m.cell_dist = CellDist(sync_bn=sync_bn, bucket=bucket)
    out, _ = m(x[sh].to(dev))
    F.binary_cross_entropy_with_logits(out, y[sh].to(dev).reshape(-1, 1)).backward()
    early = len(bucket._early_done)
    bucket.allreduce_mean()
    torch.cuda.synchronize()
    out_q.put((rank, out.detach().cpu().numpy(), early,
               {k: p.grad.detach().cpu().numpy() for k, p in m.named_parameters()
                if p.grad is not None}))
    dist.barrier()
    dist.destroy_process_group()


def _run_ranks(sync_bn, dtype="f32", three_part=True, tiled=False):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, sync_bn, q, dtype, three_part, tiled))
             for r in range(2)]
    for p in procs:
        p.start()
    res = {r: rest for r, *rest in (q.get(timeout=200) for _ in range(2))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def _single(x, y, dtype="f32", tiled=False):
    dev = torch.device("cuda:0")
    m = _model(tiled).to(dev)
    m.cell_dtype = dtype
    out, _ = m(x.to(dev))
    F.binary_cross_entropy_with_logits(out, y.to(dev).reshape(-1, 1)).backward()
    return out.detach().cpu(), {k: p.grad.detach().cpu() for k, p in m.named_parameters()
                                if p.grad is not None}


def _close_grads(got, ref, rel, min_cos=None, tag=None):
    """max |err| <= 1e-7 + rel * max|ref| per tensor; bf16 (min_cos): also the
    per-tensor gradient cosine, which a wrong all-rank BatchNorm total would
    pull far below 1 even where the max-error bound is loose; the measured
    worst values go to gpurun_out/parity_records.json."""
    assert set(got) == set(ref)
    worst_rel, worst_cos = 0.0, 1.0
    for k, v in got.items():
        a = torch.from_numpy(v).double().flatten()
        b = ref[k].double().flatten()
        err = float((a - b).abs().max())
        scale = float(b.abs().max())
        assert err <= 1e-7 + rel * scale, (k, err)
        worst_rel = max(worst_rel, err / max(scale, 1e-30))
        if min_cos is not None and float(b.norm()) > 0:
            cos = float(a @ b / (a.norm() * b.norm()))
            worst_cos = min(worst_cos, cos)
            assert cos >= min_cos, (k, cos)
    if tag:
        from goldens import record
        record(tag, {"max_rel_err": worst_rel, "min_grad_cos": worst_cos})


@pytest.mark.timeout(300)
# bf16 bounds from the measured worst case (r05: max relative error 3.4e-6,
# gradient cosine 1 - 5e-12, logits equal to 1e-6): the fp64 BatchNorm sums
# added in another order move a value by at most a rounding step
@pytest.mark.parametrize("dtype,atol,rel,min_cos,tiled", [("f32", 1e-5, 1e-5, None, False),
                                                         ("bf16", 1e-4, 2e-4, 0.99999, False),
                                                         ("f32", 1e-5, 1e-5, None, True),
                                                         ("bf16", 1e-4, 2e-4, 0.99999, True)])
def test_syncbn_two_ranks_equal_single_process(dtype, atol, rel, min_cos, tiled):
    """(r06: also the tiled hGRU at 64 x 64 -- BatchNorm over clips x tiles)"""
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    res = _run_ranks(sync_bn=True, dtype=dtype, tiled=tiled)
    x, y = _batch(tiled)
    lo, g = _single(x, y, dtype, tiled)
    for r in (0, 1):
        logits, early, grads = res[r]
        torch.testing.assert_close(torch.from_numpy(logits), lo[2 * r:2 * r + 2], rtol=0, atol=atol)
        assert early > 0                                 # the side-stream part ran
        _close_grads(grads, g, rel, min_cos, tag=f"syncbn_{dtype}{'_tiled' if tiled else ''}_rank{r}")


@pytest.mark.timeout(300)
@pytest.mark.parametrize("three_part", [True, False])
def test_early_gradient_overlap_matches_shard_mean(three_part):
    """Two-part (early cell gradients, then the rest) and r06's three-part
    exchange (early, w_inh under w_exc's weight-gradient launch, the rest)."""
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    res = _run_ranks(sync_bn=False, three_part=three_part)
    x, y = _batch()
    parts = [_single(x[s], y[s]) for s in (slice(0, 2), slice(2, 4))]
    mean = {k: (parts[0][1][k] + parts[1][1][k]) / 2 for k in parts[0][1]}
    for r in (0, 1):
        logits, early, grads = res[r]
        torch.testing.assert_close(torch.from_numpy(logits), parts[r][0], rtol=0, atol=1e-6)
        # every cell param but w_exc / w_inh, and w_inh too in the three-part form
        assert early == (23 if three_part else 22)
        _close_grads(grads, mean, 1e-5)
