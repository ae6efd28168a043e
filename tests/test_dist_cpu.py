"""Data-parallel semantics on CPU with torch.distributed/gloo, world_size 2.

Each rank owns a disjoint shard of clips (no scatter), computes its gradients
with per-replica BatchNorm statistics (the reference's DataParallel semantics,
mainclean.py:132-134) and the ranks average one flat gradient bucket
(ptamd.dist.GradBucket).  The per-rank compute here is the CPU oracle; on GPUs
it is the HIP cell — the exchange code is identical.  Checked: the averaged
gradient equals the single-process mean of the per-shard gradients, and every
rank holds identical parameters after the Adam step.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from goldens import load, params, prepared_input


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard_grads(sd, x, y):
    from oracle import cells
    leaf = {k: v.clone().requires_grad_(k != "unit1.w") for k, v in sd.items()}
    logits, _, _ = cells.recurrent_forward(leaf, x)
    cells.bce_logits(logits, y).backward()
    return leaf


def _worker(rank, world, port, out_q, parts=1):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    sys.path[:0] = [here, repo, os.path.join(repo, "pathtracker-models_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ptamd.dist import GradBucket
    g = load("int_cfg1")                       # B=4, T=32
    sd = params(g)
    x, y = prepared_input(g)
    x, y = x[:, :, :8], y                       # first 8 frames keep the test fast
    shard = slice(rank * 2, rank * 2 + 2)
    leaf = _shard_grads(sd, x[shard], y[shard])
    bucket = GradBucket(list(leaf.values()), "cpu")
    if parts == 3:
        # the three-part exchange in the cell backward's order (ptamd.cell):
        # the early cell gradients, then w_inh, then allreduce_mean the rest
        from ptamd.dist import LATE_KEYS, MID_KEYS
        cell = [k for k in leaf if k.startswith("unit1.") and leaf[k].grad is not None]
        bucket.reduce_early([(id(leaf[k]), leaf[k].grad) for k in cell if k not in LATE_KEYS], None)
        bucket.reduce_early([(id(leaf[k]), leaf[k].grad) for k in cell if k in MID_KEYS], None)
        assert len(bucket._early_done) == len(cell) - 1
    bucket.allreduce_mean()
    assert not bucket._early_done
    opt = torch.optim.Adam([v for v in leaf.values() if v.requires_grad], lr=3e-4)
    opt.step()
    # numpy (pickled by value): torch tensors would travel as fds of a dead process
    out_q.put((rank, {k: v.grad.numpy().copy() for k, v in leaf.items() if v.grad is not None},
               {k: v.detach().numpy().copy() for k, v in leaf.items()}))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("parts", [1, 3])
def test_two_rank_gradient_average_and_identical_params(parts):
    """parts=1: one flat bucket after backward; parts=3: r06's three-part
    exchange (early cell gradients, w_inh, the rest)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, parts)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (gr, pr)) for r, gr, pr in (q.get(timeout=240) for _ in range(2)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single-process reference: mean of the per-shard gradients
    g = load("int_cfg1")
    sd = params(g)
    x, y = prepared_input(g)
    x = x[:, :, :8]
    ref = [_shard_grads(sd, x[s], y[s]) for s in (slice(0, 2), slice(2, 4))]
    for k in res[0][0]:
        mean = (ref[0][k].grad + ref[1][k].grad) / 2
        for r in (0, 1):
            torch.testing.assert_close(torch.from_numpy(res[r][0][k]), mean, rtol=1e-5, atol=1e-7)
    for k in res[0][1]:
        torch.testing.assert_close(torch.from_numpy(res[0][1][k]), torch.from_numpy(res[1][1][k]),
                                   rtol=0, atol=0)


def _lockstep_worker(rank, world, port, out_q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    sys.path[:0] = [here, repo, os.path.join(repo, "pathtracker-models_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ptamd.dist import lockstep
    seen = []
    # uneven shards: rank r holds 3 + 2 r batches; every step also runs a
    # collective, as the gradient all-reduce does -- it must never mismatch
    for item in lockstep(range(3 + 2 * rank), "cpu"):
        t = torch.tensor([float(item)])
        dist.all_reduce(t)
        seen.append((item, float(t)))
    out_q.put((rank, seen))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_lockstep_stops_all_ranks_at_the_smallest_shard():
    """mainclean's train loop over per-rank shards with unequal batch counts."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_lockstep_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=100) for _ in range(3))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    for r in range(3):
        assert res[r] == [(i, 3.0 * i) for i in range(3)]


# ------------------------------------------------------------------ SyncBN
def _syncbn_worker(rank, world, port, out_q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    sys.path[:0] = [here, repo, os.path.join(repo, "pathtracker-models_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import cells
    from ptamd.dist import CellDist, GradBucket
    g = load("int_cfg1")
    sd = params(g)
    x, y = prepared_input(g)
    x = x[:, :, :6]
    shard = slice(rank * 2, rank * 2 + 2)
    leaf = {k: v.clone().requires_grad_(k != "unit1.w") for k, v in sd.items()}
    logits, _, _ = cells.recurrent_forward(leaf, x[shard], bn=cells.sync_batch_norm())
    cells.bce_logits(logits, y[shard]).backward()
    GradBucket(list(leaf.values()), "cpu").allreduce_mean()
    # the product's SyncBN host hook (the ctypes callback the HIP library calls
    # between launches) on a CPU buffer: sums exactly the requested slice
    cd = CellDist(sync_bn=True)
    buf = cd.buffer(10, torch.device("cpu"))
    buf.copy_(torch.arange(10, dtype=torch.float64) * (rank + 1))
    rc = cd._cfn(None, 3, 4)
    out_q.put((rank, logits.detach().numpy().copy(),
               {k: v.grad.numpy().copy() for k, v in leaf.items() if v.grad is not None},
               rc, buf.numpy().copy(), cd.struct(320, torch.device("cpu")).bn_world))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_syncbn_equals_single_process():
    """SyncBN (opt-in): 2 ranks x 2 clips with BatchNorm
    statistics all-reduced over the ranks reproduce the single process on all
    4 clips -- logits per clip and the rank-averaged gradients, to 1e-5.  Also
    drives the product's all-reduce callback (ptamd.dist.CellDist) on gloo."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_syncbn_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: rest for r, *rest in (q.get(timeout=240) for _ in range(2))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from oracle import cells
    g = load("int_cfg1")
    sd = params(g)
    x, y = prepared_input(g)
    x = x[:, :, :6]
    leaf = {k: v.clone().requires_grad_(k != "unit1.w") for k, v in sd.items()}
    lo, _, _ = cells.recurrent_forward(leaf, x)
    cells.bce_logits(lo, y).backward()
    for r in (0, 1):
        logits, grads, rc, buf, world = res[r]
        torch.testing.assert_close(torch.from_numpy(logits), lo[2 * r:2 * r + 2].detach(),
                                   rtol=1e-5, atol=1e-6)
        for k, v in grads.items():
            ref = leaf[k].grad
            err = float((torch.from_numpy(v) - ref).abs().max())
            assert err <= 1e-7 + 1e-5 * float(ref.abs().max()), (k, err)
        assert rc == 0 and world == 2
        expect = torch.arange(10, dtype=torch.float64) * (r + 1)
        expect[3:7] = torch.arange(3, 7, dtype=torch.float64) * 3      # (1 + 2) x
        assert torch.equal(torch.from_numpy(buf), expect)


def test_bucket_skips_early_reduced_params():
    """allreduce_mean averages only what the early (side-stream) all-reduce did
    not (single process: a no-op either way; the pending set is computed)."""
    from ptamd.dist import GradBucket
    ps = [torch.nn.Parameter(torch.ones(3)) for _ in range(3)]
    b = GradBucket(ps, "cpu")
    b._early_done = {id(ps[0])}
    b.allreduce_mean()                 # world 1: returns before touching anything
    assert b._early_done == {id(ps[0])}
