"""Data parallelism for the recurrent trainer: one process per GPU.

The reference scales with single-process ``nn.DataParallel`` (mainclean.py:132-134):
parameters broadcast, input scattered from cuda:0, gradients reduce-added.
Here every rank owns its clips (no scatter), computes its own BatchNorm batch
statistics (exactly DataParallel's per-replica semantics), and the only
exchange is ONE all-reduce per step of a single flat fp32 gradient bucket
(107,190 parameters = 428,760 B for InT), over RCCL/xGMI (backend "nccl") on
GPUs or gloo on CPU.  The bucket is far below any per-link bandwidth concern;
the all-reduce is latency-bound (tens of microseconds).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def env_rank():
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)),
            int(os.environ.get("WORLD_SIZE", 1)))


class GradBucket:
    """Flat fp32 gradient bucket averaged across ranks with one all-reduce."""

    def __init__(self, params, device):
        self.params = [p for p in params if p.requires_grad]
        self.numel = sum(p.numel() for p in self.params)
        self.flat = torch.zeros(self.numel, dtype=torch.float32, device=device)

    def allreduce_mean(self, group=None):
        world = dist.get_world_size(group) if dist.is_initialized() else 1
        if world == 1:
            return
        off = 0
        for p in self.params:
            n = p.numel()
            if p.grad is None:
                self.flat[off:off + n].zero_()
            else:
                self.flat[off:off + n].copy_(p.grad.reshape(-1))
            off += n
        dist.all_reduce(self.flat, group=group)
        self.flat.mul_(1.0 / world)
        off = 0
        for p in self.params:
            n = p.numel()
            if p.grad is not None:          # params no rank differentiates stay None
                p.grad.copy_(self.flat[off:off + n].view_as(p))
            off += n


def lockstep(iterable, device):
    """Yield from a per-rank iterable only while EVERY rank still has an item.

    Each rank reads its own TFRecord shards (file i -> rank i % world), so the
    ranks' batch counts can differ; a rank that ran out first would leave the
    loop and meet the others' gradient all-reduce with a different collective.
    One MIN all-reduce of a has-item flag per step keeps the loop in lockstep:
    all ranks stop at the smallest count.  Single process: plain iteration.
    """
    world = dist.get_world_size() if dist.is_initialized() else 1
    it = iter(iterable)
    flag = torch.zeros(1, dtype=torch.int32, device=device)
    while True:
        item = next(it, None)
        if world > 1:
            flag.fill_(0 if item is None else 1)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN)
            if int(flag.item()) == 0:
                close = getattr(it, "close", None)
                if close is not None:
                    close()
                return
        elif item is None:
            return
        yield item
