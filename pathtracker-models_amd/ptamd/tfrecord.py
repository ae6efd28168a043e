"""ctypes binding of ``libpttfr.so`` (include/pt_tfrecord.h): the native GZIP
TFRecord reader / writer that replaces the reference's TensorFlow input
pipeline (utils/TFRDataset.py:6-53).

``Reader`` yields ``(clips uint8 [B,T,H,W,3], labels uint8 [B])`` batches from
this rank's shards (file i -> rank i % world), decoded by native threads;
``write`` / ``write_synthetic_shards`` produce spec-conformant GZIP TFRecord
files of tf.train.Example records (used for synthetic data and tests — there
is no dataset access offline).
"""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libpttfr.so")

EXPORTS = ("pt_tfr_open", "pt_tfr_next", "pt_tfr_count", "pt_tfr_close", "pt_tfr_write",
           "pt_tfr_parse_example", "pt_tfr_crc32c", "pt_tfr_masked_crc32c", "pt_tfr_last_error")


class Options(ctypes.Structure):
    _fields_ = [("timesteps", ctypes.c_int32), ("height", ctypes.c_int32),
                ("width", ctypes.c_int32), ("channels", ctypes.c_int32),
                ("rank", ctypes.c_int32), ("world", ctypes.c_int32),
                ("shuffle_buffer", ctypes.c_int32), ("threads", ctypes.c_int32),
                ("verify_crc", ctypes.c_int32), ("drop_remainder", ctypes.c_int32),
                ("seed", ctypes.c_uint64)]


class TFRecordError(RuntimeError):
    pass


_lock = threading.Lock()
_lib = None
_P = ctypes.c_void_p
_U8P = ctypes.POINTER(ctypes.c_uint8)


def load():
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise TFRecordError(f"{LIB_PATH} is missing: build the native extensions first "
                                "(python __graft_entry__.py build)")
        lib = ctypes.CDLL(LIB_PATH)
        lib.pt_tfr_open.restype = _P
        lib.pt_tfr_open.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.c_int32,
                                    ctypes.POINTER(Options)]
        lib.pt_tfr_next.restype = ctypes.c_int64
        lib.pt_tfr_next.argtypes = [_P, ctypes.c_int32, _U8P, _U8P]
        lib.pt_tfr_count.restype = ctypes.c_int64
        lib.pt_tfr_count.argtypes = [_P]
        lib.pt_tfr_close.restype = ctypes.c_int
        lib.pt_tfr_close.argtypes = [_P]
        lib.pt_tfr_write.restype = ctypes.c_int
        lib.pt_tfr_write.argtypes = [ctypes.c_char_p, _U8P, _U8P, ctypes.c_int64, ctypes.c_int32,
                                     ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]
        lib.pt_tfr_parse_example.restype = ctypes.c_int64
        lib.pt_tfr_parse_example.argtypes = [ctypes.c_char_p, ctypes.c_size_t, _U8P,
                                             ctypes.c_size_t, _U8P]
        lib.pt_tfr_crc32c.restype = ctypes.c_uint32
        lib.pt_tfr_crc32c.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
        lib.pt_tfr_masked_crc32c.restype = ctypes.c_uint32
        lib.pt_tfr_masked_crc32c.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
        lib.pt_tfr_last_error.restype = ctypes.c_char_p
        _lib = lib
        return lib


def _err(rc):
    raise TFRecordError(f"pt_tfrecord error {rc}: {load().pt_tfr_last_error().decode(errors='replace')}")


def _u8(a):
    return a.ctypes.data_as(_U8P)


def crc32c(data: bytes) -> int:
    return load().pt_tfr_crc32c(data, len(data))


def masked_crc32c(data: bytes) -> int:
    return load().pt_tfr_masked_crc32c(data, len(data))


def parse_example(record: bytes, timesteps: int, height: int = 32, width: int = 32,
                  channels: int = 3):
    """One serialized Example -> (image uint8 [T,H,W,C], label byte)."""
    n = timesteps * height * width * channels
    img = np.empty(n, np.uint8)
    lab = np.empty(1, np.uint8)
    got = load().pt_tfr_parse_example(record, len(record), _u8(img), n, _u8(lab))
    if got < 0:
        _err(got)
    if got != n:        # tf.reshape([T, H, W, C]) fails on any other size (TFRDataset.py:20)
        raise TFRecordError(f"image has {got} bytes, cannot reshape to "
                            f"[{timesteps}, {height}, {width}, {channels}]")
    return img.reshape(timesteps, height, width, channels), bytes(lab)


def write(path: str, clips: np.ndarray, labels, gzip: bool = True):
    """clips uint8 [N,T,H,W,C]; labels: N one-byte strings or uint8 codes."""
    clips = np.ascontiguousarray(clips, dtype=np.uint8)
    lab = np.asarray(labels)
    if lab.dtype.kind in "OS":
        lab = np.array([ord(b) for b in lab], np.uint8)
    lab = np.ascontiguousarray(lab, dtype=np.uint8)
    n, t, h, w, c = clips.shape
    rc = load().pt_tfr_write(os.fsencode(path), _u8(clips), _u8(lab), n, t, h, w, c, int(gzip))
    if rc:
        _err(rc)


def write_synthetic_shards(out_dir: str, n_shards: int, clips_per_shard: int, timesteps: int,
                           seed: int = 0, prefix: str = "synthetic"):
    """Seeded synthetic PathTracker shards (ptamd.synth) as GZIP TFRecords."""
    from . import synth
    os.makedirs(out_dir, exist_ok=True)
    paths = []
    for s in range(n_shards):
        clips, labels = synth.make_batch(seed * 100003 + s, clips_per_shard, timesteps)
        p = os.path.join(out_dir, f"{prefix}-{s:05d}-of-{n_shards:05d}.tfrecord.gz")
        write(p, clips, labels)
        paths.append(p)
    return paths


class Reader:
    """Batches of clips from GZIP TFRecord shards, decoded by native threads.

    Semantics of utils/TFRDataset.py:31-53: files in the given order, records in
    file order, optional shuffle buffer (tf.data's sampling scheme; its RNG is
    not TF's), ``batch(B, drop_remainder)``; plus per-rank file sharding.
    """

    def __init__(self, paths, timesteps, height=32, width=32, channels=3, rank=0, world=1,
                 shuffle_buffer=0, seed=0, threads=4, verify_crc=True, drop_remainder=True):
        self._lib = load()
        self.shape = (timesteps, height, width, channels)
        o = Options(timesteps=timesteps, height=height, width=width, channels=channels,
                    rank=rank, world=world, shuffle_buffer=shuffle_buffer, threads=threads,
                    verify_crc=int(verify_crc), drop_remainder=int(drop_remainder), seed=seed)
        enc = [os.fsencode(p) for p in paths]
        arr = (ctypes.c_char_p * max(len(enc), 1))(*enc)
        self._h = self._lib.pt_tfr_open(arr, len(enc), ctypes.byref(o))
        if not self._h:
            _err(-1)

    def next(self, batch, out=None):
        """Next batch, or None at the end.  ``out`` = (clips, labels) buffers to
        fill (reused across calls: no fresh 50 MB allocation per batch)."""
        if out is None:
            clips = np.empty((batch,) + self.shape, np.uint8)
            labels = np.empty(batch, np.uint8)
        else:
            clips, labels = out
            assert clips.shape == (batch,) + self.shape and clips.flags.c_contiguous
            assert labels.shape == (batch,) and clips.dtype == labels.dtype == np.uint8
        n = self._lib.pt_tfr_next(self._h, batch, _u8(clips), _u8(labels))
        if n < 0:
            _err(n)
        if n == 0:
            return None
        return clips[:n], labels[:n]

    def batches(self, batch, reuse=False):
        """Iterate batches; with ``reuse`` every batch is a view of the same two
        buffers (valid until the next one is produced)."""
        out = None
        if reuse:
            out = (np.empty((batch,) + self.shape, np.uint8), np.empty(batch, np.uint8))
        while True:
            b = self.next(batch, out)
            if b is None:
                return
            yield b

    @property
    def count(self):
        return self._lib.pt_tfr_count(self._h)

    def close(self):
        if getattr(self, "_h", None):
            self._lib.pt_tfr_close(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
