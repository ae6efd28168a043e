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


def _worker(rank, world, port, out_q):
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
    bucket.allreduce_mean()
    opt = torch.optim.Adam([v for v in leaf.values() if v.requires_grad], lr=3e-4)
    opt.step()
    # numpy (pickled by value): torch tensors would travel as fds of a dead process
    out_q.put((rank, {k: v.grad.numpy().copy() for k, v in leaf.items() if v.grad is not None},
               {k: v.detach().numpy().copy() for k, v in leaf.items()}))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_gradient_average_and_identical_params():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
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
