"""Data parallelism for the recurrent trainer: one process per GPU.

The reference scales with single-process ``nn.DataParallel`` (mainclean.py:132-134):
parameters broadcast, input scattered from cuda:0, gradients reduce-added.
Here every rank owns its clips (no scatter) and the only exchange of the
default mode is ONE averaging of the fp32 gradients per step (107,190
parameters = 428,760 B for InT) over RCCL/xGMI (backend "nccl") on GPUs or gloo
on CPU.  BatchNorm statistics are per replica by default -- exactly
DataParallel's semantics.

Two opt-in extensions of the HIP cell's C-ABI (``pt_cell_dist``,
include/pt_cell.h), configured through :class:`CellDist`:

* SyncBN: every BatchNorm reduction of the cell (2 per frame forward, 2 per
  frame backward) is summed over the ranks before it is used, so the ranks
  together compute exactly the single-process batch (4 T small all-reduces per
  step, host callbacks between launches, no hipGraph replay);
* gradient overlap: the cell's gradients other than the two k x k weights are
  final before the k x k weight-gradient kernel (~2.1 ms at the headline
  size) starts; :class:`GradBucket` averages them on a side stream while that
  kernel runs.  With the r06 three-part exchange the kernel runs as two
  launches, w_inh's first: w_inh's gradient (50,176 floats) is averaged on the
  side stream while w_exc's launch runs, so 56,896 of the 107,190 floats
  (53 %) are exchanged under the backward; only w_exc and the readout are
  averaged afterwards.
"""
from __future__ import annotations

import os
import traceback

import torch
import torch.distributed as dist

# cell gradients final before the k x k weight-gradient kernel (ptamd.cell.PARAM_KEYS)
LATE_KEYS = ("unit1.w_exc", "unit1.w_inh")
# (r06) the k x k weight final between its own weight-gradient launch and
# w_exc's (pt_cell_dist.grads_mid_event): averaged under w_exc's launch
MID_KEYS = ("unit1.w_inh",)


def env_rank():
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)),
            int(os.environ.get("WORLD_SIZE", 1)))


def _world(group=None):
    return dist.get_world_size(group) if dist.is_initialized() else 1


class GradBucket:
    """fp32 gradients averaged across ranks with one all-reduce of a flat bucket
    (plus, with a :class:`CellDist` overlap, one earlier side-stream all-reduce
    of the cell's early gradients)."""

    def __init__(self, params, device, group=None, three_part=True):
        self.params = [p for p in params if p.requires_grad]
        self.three_part = three_part    # w_inh averaged under w_exc's weight-gradient launch
        self.numel = sum(p.numel() for p in self.params)
        self.flat = torch.zeros(self.numel, dtype=torch.float32, device=device)
        self.group = group
        self._early_done = set()        # ids of params averaged early this step
        self._side = None

    def reduce_early(self, pairs, event):
        """Average the (id(param), grad) pairs on a side stream that waits for
        ``event`` (recorded by the cell's backward once those gradients are
        written), and make the current stream wait for it -- the wait is
        enqueued behind the k x k weight-gradient kernel, which the all-reduce
        therefore overlaps.  Called from the cell's autograd backward."""
        world = _world(self.group)
        if world == 1 or not pairs:
            return
        if not pairs[0][1].is_cuda:       # CPU ranks (gloo): the same exchange, in order
            flat = torch.cat([g.reshape(-1) for _, g in pairs])
            dist.all_reduce(flat, group=self.group)
            flat.mul_(1.0 / world)
            off = 0
            for _, g in pairs:
                g.copy_(flat[off:off + g.numel()].view_as(g))
                off += g.numel()
            self._early_done |= {pid for pid, _ in pairs}
            return
        main = torch.cuda.current_stream()
        if self._side is None:
            self._side = torch.cuda.Stream(device=main.device)
        side = self._side
        side.wait_event(event)
        with torch.cuda.stream(side):
            flat = torch.cat([g.reshape(-1) for _, g in pairs])
            dist.all_reduce(flat, group=self.group)
            flat.mul_(1.0 / world)
            off = 0
            for _, g in pairs:
                n = g.numel()
                g.copy_(flat[off:off + n].view_as(g))
                g.record_stream(side)
                off += n
        main.wait_stream(side)
        self._early_done |= {pid for pid, _ in pairs}       # (early, then mid: both this step)

    def allreduce_mean(self):
        world = _world(self.group)
        if world == 1:
            return
        pend = [p for p in self.params if id(p) not in self._early_done]
        self._early_done = set()
        n_all = sum(p.numel() for p in pend)
        flat = self.flat[:n_all]
        off = 0
        for p in pend:
            n = p.numel()
            if p.grad is None:
                flat[off:off + n].zero_()
            else:
                flat[off:off + n].copy_(p.grad.reshape(-1))
            off += n
        dist.all_reduce(flat, group=self.group)
        flat.mul_(1.0 / world)
        off = 0
        for p in pend:
            n = p.numel()
            if p.grad is not None:          # params no rank differentiates stay None
                p.grad.copy_(flat[off:off + n].view_as(p))
            off += n


class CellDist:
    """Cross-replica options of the HIP cell (``pt_cell_dist``).

    sync_bn: BatchNorm statistics over every rank's clips.  The library writes
      each reduction's per-rank totals into ``bn_buf`` (fp64, on the device) and
      calls back :meth:`allreduce_slice`, which SUMs that slice over ``group``
      on the current stream.
    bucket: a :class:`GradBucket` to average the early cell gradients on a side
      stream while the k x k weight-gradient kernel runs (GPU ranks).
    """

    def __init__(self, group=None, sync_bn=False, bucket=None):
        from . import _lib
        self.group = group
        self.sync_bn = sync_bn
        self.bucket = bucket
        self.bn_buf = None
        self.failed = None
        self._cfn = _lib.ALLREDUCE_FN(self._callback)    # kept alive with self

    def world(self):
        return _world(self.group)

    def buffer(self, n, device):
        if self.bn_buf is None or self.bn_buf.numel() < n or self.bn_buf.device != device:
            self.bn_buf = torch.zeros(n, dtype=torch.float64, device=device)
        return self.bn_buf

    def allreduce_slice(self, offset, count):
        dist.all_reduce(self.bn_buf[offset:offset + count], group=self.group)

    def _callback(self, _user, offset, count):
        try:
            self.allreduce_slice(int(offset), int(count))
            return 0
        except Exception as e:      # the library turns a non-zero return into an error
            self.failed = e
            traceback.print_exc()
            return 1

    def struct(self, bn_doubles, device, early_event=None, mid_event=None):
        """The pt_cell_dist for one call (``bn_doubles`` = pt_cell_bn_sync_doubles)."""
        from . import _lib
        d = _lib.Dist()
        world = self.world()
        d.bn_world = world if self.sync_bn else 1
        if d.bn_world > 1:
            d.bn_buf = self.buffer(bn_doubles, device).data_ptr()
            d.allreduce = self._cfn
        d.user = None
        d.grads_early_event = early_event
        d.grads_mid_event = mid_event
        return d


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
