"""TFRDataset — drop-in for the reference ``utils/TFRDataset.py`` without TensorFlow.

Same functions, arguments and batch contents as the reference:

* ``read_tfrecord(example, timesteps=64)`` (:6-28) — one serialized
  tf.train.Example -> ``(image uint8 [T,32,32,3], label)``;
* ``tfr_data_loader(data_dir, batch_size=32, drop_remainder=True,
  shuffle_buffer=1000, timesteps=64)`` (:31-53) — glob -> GZIP TFRecords ->
  parse -> shuffle(buffer) -> batch(B, drop_remainder).

Decoding runs in the native reader (ptamd/tfrecord.py, libpttfr.so: zlib +
a minimal protobuf wire decoder, CRC-checked, decoder threads).  Batches are
numpy arrays that also answer ``.numpy()`` (what the reference's
``engine.prepare_data`` calls on its TF tensors, utils/engine.py:222-224);
labels are one-byte strings, so ``np.vectorize(ord)`` works on them as on TF's.

Added for one-process-per-GPU training: the files are sharded by rank
(file i -> rank i % world; rank / world from torch.distributed when it is
initialised, else the RANK / WORLD_SIZE environment, else 0 / 1), so every
rank reads disjoint shards with no scatter.
"""
import glob
import os
import queue
import threading

import numpy as np

from ptamd import tfrecord


class _Batch(np.ndarray):
    """numpy array with TF's ``.numpy()`` accessor."""

    def numpy(self):
        return np.asarray(self)


def _as_batch(a):
    return np.asarray(a).view(_Batch)


def _rank_world():
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return dist.get_rank(), dist.get_world_size()
    except ImportError:
        pass
    return int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))


def _labels(codes):
    """uint8 label codes -> the 1-byte strings a TF string tensor yields."""
    return _as_batch(np.array([bytes([v]) for v in codes], dtype=object))


def read_tfrecord(example, timesteps=64):
    """Parse one serialized Example (reference utils/TFRDataset.py:6-28)."""
    if hasattr(example, "numpy"):
        example = example.numpy()
    image, label = tfrecord.parse_example(bytes(example), timesteps)
    return image, label


class _Loader:
    """One pass = one native Reader.  Batches are produced by a background
    thread (the native calls release the GIL) ``prefetch`` batches ahead, so
    decoding overlaps the training step, as tf.data's pipeline does for the
    reference.  The clip arrays live in a ring of ``prefetch + 2`` host
    buffers: a batch stays valid until ``prefetch + 1`` further batches have
    been taken (engine.prepare_data copies it to the device right away)."""

    def __init__(self, files, batch_size, drop_remainder, shuffle_buffer, timesteps, seed,
                 prefetch=2, pin_memory=False):
        self.files, self.batch_size = files, batch_size
        self.drop_remainder, self.shuffle_buffer = drop_remainder, shuffle_buffer
        self.timesteps, self.seed, self.epoch = timesteps, seed, 0
        self.prefetch = prefetch
        self.pin_memory = pin_memory

    def _batches(self, rd):
        # pinned host memory from torch on ROCm is host-coherent: the reader's
        # writes into it ran at 2.2k clips/s on the GPU box vs 20k clips/s into
        # pageable memory (whose H2D copy in prepare_data takes ~3 ms per
        # 50 MB batch), so pinning is opt-in
        if not self.pin_memory:
            if self.prefetch <= 0:
                for clips, labels in rd.batches(self.batch_size):
                    yield _as_batch(clips), labels
                return
            # host ring filled in place: one native call (GIL released) per
            # batch and no 50 MB allocation -- a producer that needs the GIL
            # often waits out the training loop's switch interval each time
            ring = [np.empty((self.batch_size,) + rd.shape, np.uint8) for _ in range(self.prefetch + 2)]
            labs = [np.empty(self.batch_size, np.uint8) for _ in ring]
            k = 0
            while True:
                got = rd.next(self.batch_size, (ring[k], labs[k]))
                if got is None:
                    return
                yield _as_batch(got[0]), got[1]
                k = (k + 1) % len(ring)
        # pinned ring, filled in place by the native reader (pinning per batch
        # costs more than decoding it).  A slot is refilled prefetch + 1 batches
        # after it was handed out; engine.prepare_data copies it to the device
        # synchronously, so the consumer is done with it by then.
        import torch
        ring = [torch.empty((self.batch_size,) + rd.shape, dtype=torch.uint8).pin_memory()
                for _ in range(self.prefetch + 2)]
        labs = [np.empty(self.batch_size, np.uint8) for _ in ring]
        k = 0
        while True:
            got = rd.next(self.batch_size, (ring[k].numpy(), labs[k]))
            if got is None:
                return
            n = len(got[1])
            yield ring[k][:n], labs[k][:n]
            k = (k + 1) % len(ring)

    def __iter__(self):
        # reshuffle_each_iteration=True: a new shuffle seed per pass (:50)
        rank, world = _rank_world()
        rd = tfrecord.Reader(self.files, self.timesteps, rank=rank, world=world,
                             shuffle_buffer=self.shuffle_buffer, seed=self.seed + self.epoch,
                             threads=min(16, os.cpu_count() or 1, max(1, len(self.files))),
                             drop_remainder=self.drop_remainder)
        self.epoch += 1
        if self.prefetch <= 0:
            try:
                for clips, labels in self._batches(rd):
                    yield clips, _labels(labels)
            finally:
                rd.close()
            return
        q = queue.Queue(maxsize=self.prefetch)
        stop = threading.Event()
        end = object()

        def produce():
            try:
                for item in self._batches(rd):
                    while not stop.is_set():
                        try:
                            q.put(item, timeout=0.1)
                            break
                        except queue.Full:
                            continue
                    if stop.is_set():
                        return
                q.put(end)
            except BaseException as e:          # surfaced in the consumer
                q.put(e)

        th = threading.Thread(target=produce, daemon=True)
        th.start()
        try:
            while True:
                item = q.get()
                if item is end:
                    return
                if isinstance(item, BaseException):
                    raise item
                yield item[0], _labels(item[1])
        finally:
            stop.set()
            while th.is_alive():                # unblock a producer waiting on a full queue
                try:
                    q.get(timeout=0.05)
                except queue.Empty:
                    pass
            th.join()
            rd.close()


def tfr_data_loader(data_dir="", batch_size=32, drop_remainder=True, shuffle_buffer=1000,
                    timesteps=64, seed=0, prefetch=2, pin_memory=False):
    """Iterable of ``(images [B,T,32,32,3] uint8, labels [B] 1-byte strings)``
    (reference utils/TFRDataset.py:31-53)."""
    if data_dir is None:
        raise ValueError("Missing path to data directory!")
    files = sorted(glob.glob(data_dir))
    return _Loader(files, batch_size, drop_remainder, shuffle_buffer, timesteps, seed,
                   prefetch=prefetch, pin_memory=pin_memory)
