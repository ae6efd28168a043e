"""Native TFRecord reader / writer (libpttfr.so, replaces the reference's
tf.data pipeline utils/TFRDataset.py:6-53) against an independent restatement
of the formats (oracle/tfrecord_ref.py: pure-Python CRC32C, Google's protobuf
runtime for tf.train.Example, Python's gzip).

TensorFlow is absent offline and the reference ships no TFRecord files, so
parity with TF-written shards is "unpinned": these tests pin the published
formats (RFC 3720 CRC32C vectors, TFRecord framing, Example wire format).
"""
import gzip
import os

import numpy as np
import pytest

from oracle import tfrecord_ref as ref
from ptamd import synth, tfrecord

T = 4


def _clips(n, seed=0, t=T):
    clips, labels = synth.make_batch(seed, n, t)
    return clips, np.array([ord(b) for b in labels], np.uint8)


def test_crc32c_known_answers():
    # RFC 3720 B.4 / iSCSI test vectors
    for data, want in ((b"123456789", 0xE3069283), (bytes(32), 0x8A9136AA),
                       (bytes([0xFF] * 32), 0x62A8AB43), (bytes(range(32)), 0x46DD794E)):
        assert tfrecord.crc32c(data) == want
        assert ref.crc32c(data) == want
    blob = os.urandom(1000)
    for n in (0, 1, 7, 8, 9, 63, 1000):
        assert tfrecord.crc32c(blob[:n]) == ref.crc32c(blob[:n])
        assert tfrecord.masked_crc32c(blob[:n]) == ref.masked_crc32c(blob[:n])


def test_native_writer_read_by_reference_format(tmp_path):
    clips, labels = _clips(5)
    p = str(tmp_path / "a.tfrecord.gz")
    tfrecord.write(p, clips, labels)
    recs = ref.read_file(p)                       # python gzip + framing + CRCs
    assert len(recs) == 5
    for i, r in enumerate(recs):
        img, lab, h, w = ref.decode_example(r)    # Google's protobuf parser
        assert img == clips[i].tobytes() and lab == bytes([labels[i]]) and (h, w) == (32, 32)


@pytest.mark.parametrize("compress", [True, False])
def test_reference_format_read_natively(tmp_path, compress):
    clips, labels = _clips(7, seed=3)
    p = str(tmp_path / "b.tfrecord")
    ref.write_file(p, [ref.encode_example(c.tobytes(), bytes([l])) for c, l in zip(clips, labels)],
                   compress=compress)
    with tfrecord.Reader([p], T, drop_remainder=False) as rd:
        got = list(rd.batches(3))
    assert [len(b[1]) for b in got] == [3, 3, 1]
    np.testing.assert_array_equal(np.concatenate([b[0] for b in got]), clips)
    np.testing.assert_array_equal(np.concatenate([b[1] for b in got]), labels)


def test_parse_single_example_matches_read_tfrecord():
    from utils.TFRDataset import read_tfrecord
    clips, labels = _clips(1, seed=5)
    rec = ref.encode_example(clips[0].tobytes(), bytes([labels[0]]))
    img, lab = read_tfrecord(rec, timesteps=T)
    assert img.shape == (T, 32, 32, 3) and img.dtype == np.uint8
    np.testing.assert_array_equal(img, clips[0])
    assert lab == bytes([labels[0]])
    with pytest.raises(tfrecord.TFRecordError, match="reshape"):
        read_tfrecord(rec, timesteps=T + 1)


def test_rank_sharding_partitions_files(tmp_path):
    paths = tfrecord.write_synthetic_shards(str(tmp_path), n_shards=5, clips_per_shard=3,
                                            timesteps=T, seed=1)
    seen = []
    for rank in range(3):
        with tfrecord.Reader(paths, T, rank=rank, world=3, drop_remainder=False) as rd:
            for clips, labels in rd.batches(4):
                seen.extend(c.tobytes() for c in clips)
    allrec = [ref.decode_example(r)[0] for p in paths for r in ref.read_file(p)]
    assert sorted(seen) == sorted(allrec) and len(seen) == 15


def test_shuffle_is_a_permutation_and_seeded(tmp_path):
    clips, labels = _clips(40, seed=2)
    p = str(tmp_path / "c.tfrecord.gz")
    tfrecord.write(p, clips, labels)

    def order(buf, seed):
        with tfrecord.Reader([p], T, shuffle_buffer=buf, seed=seed, drop_remainder=False) as rd:
            out = np.concatenate([b[0] for b in rd.batches(16)])
        return [int(np.flatnonzero((clips == c).all(axis=(1, 2, 3, 4)))[0]) for c in out]

    assert order(0, 0) == list(range(40))
    assert order(1, 0) == list(range(40))              # buffer of 1 = file order
    a, b, a2 = order(10, 1), order(10, 2), order(10, 1)
    assert sorted(a) == list(range(40)) and a == a2 and a != b
    # a buffer of N can only emit from the first N + k records at step k
    assert all(idx <= k + 9 for k, idx in enumerate(a))


def test_drop_remainder_and_counts(tmp_path):
    clips, labels = _clips(10, seed=4)
    p = str(tmp_path / "d.tfrecord.gz")
    tfrecord.write(p, clips, labels)
    with tfrecord.Reader([p], T, drop_remainder=True) as rd:
        assert [len(b[0]) for b in rd.batches(4)] == [4, 4]
        assert rd.count == 8
    with tfrecord.Reader([p], T, drop_remainder=False) as rd:
        assert [len(b[0]) for b in rd.batches(4)] == [4, 4, 2]
    with tfrecord.Reader([], T) as rd:                 # empty glob: no batches
        assert rd.next(4) is None
    e = str(tmp_path / "empty.tfrecord.gz")
    tfrecord.write(e, np.zeros((0, T, 32, 32, 3), np.uint8), np.zeros(0, np.uint8))
    with tfrecord.Reader([e, p], T, drop_remainder=False) as rd:
        assert sum(len(b[0]) for b in rd.batches(3)) == 10


def test_corruption_is_detected(tmp_path):
    clips, labels = _clips(3, seed=6)
    raw = b"".join(ref.frame(ref.encode_example(c.tobytes(), bytes([l])))
                   for c, l in zip(clips, labels))
    cases = {
        "data CRC": raw[:100] + bytes([raw[100] ^ 1]) + raw[101:],
        "length CRC": raw[:9] + bytes([raw[9] ^ 1]) + raw[10:],
        "truncated": raw[:-7],
    }
    for what, blob in cases.items():
        p = str(tmp_path / "bad.tfrecord.gz")
        with gzip.open(p, "wb") as fh:
            fh.write(blob)
        with tfrecord.Reader([p], T, drop_remainder=False) as rd:
            with pytest.raises(tfrecord.TFRecordError, match=what.split()[0]):
                list(rd.batches(2))
    # schema errors: wrong image size, multi-byte label
    for rec, msg in ((ref.encode_example(b"\0" * 10, b"\x01"), "image has 10 bytes"),
                     (ref.encode_example(clips[0].tobytes(), b"ab"), "label has 2 bytes")):
        p = str(tmp_path / "schema.tfrecord.gz")
        ref.write_file(p, [rec])
        with tfrecord.Reader([p], T, drop_remainder=False) as rd:
            with pytest.raises(tfrecord.TFRecordError, match=msg):
                rd.next(1)


def test_loader_feeds_prepare_data(tmp_path):
    """tfr_data_loader -> engine.prepare_data, as mainclean.py:183-188 uses them."""
    import types
    from oracle import harness
    from utils import engine
    from utils.TFRDataset import tfr_data_loader
    tfrecord.write_synthetic_shards(str(tmp_path), n_shards=2, clips_per_shard=5, timesteps=T)
    loader = tfr_data_loader(str(tmp_path / "*.tfrecord.gz"), batch_size=4, shuffle_buffer=0,
                             timesteps=T)
    batches = list(loader)
    assert len(batches) == 2                             # 10 clips, drop_remainder
    imgs, target = batches[0]
    assert imgs.numpy().shape == (4, T, 32, 32, 3) and target.numpy().dtype == object
    args = types.SimpleNamespace(model="InT", pretrained=False)
    x, y = engine.prepare_data(imgs.numpy(), target.numpy(), args, "cpu", False)
    xr, yr = harness.prepare_data(imgs.numpy(), target.numpy(), False, False)
    np.testing.assert_array_equal(x.numpy(), xr)
    np.testing.assert_array_equal(y.numpy(), yr)
    assert len(list(loader)) == 2                        # a second epoch re-reads


def test_loader_prefetch_thread(tmp_path):
    """The background producer yields the same batches as the synchronous path,
    stops cleanly when the consumer breaks early, and re-raises reader errors."""
    import threading
    from utils.TFRDataset import tfr_data_loader
    tfrecord.write_synthetic_shards(str(tmp_path), n_shards=3, clips_per_shard=6, timesteps=T)
    pat = str(tmp_path / "*.tfrecord.gz")
    sync = [b[0].copy() for b in tfr_data_loader(pat, 4, shuffle_buffer=0, timesteps=T, prefetch=0)]
    pre = [np.asarray(b[0]).copy() for b in tfr_data_loader(pat, 4, shuffle_buffer=0, timesteps=T,
                                                            prefetch=2, pin_memory=False)]
    assert len(sync) == len(pre) == 4
    for a, b in zip(sync, pre):
        np.testing.assert_array_equal(a, b)
    before = threading.active_count()
    for i, _ in enumerate(tfr_data_loader(pat, 2, shuffle_buffer=0, timesteps=T, prefetch=1)):
        if i == 1:
            break                                          # generator closed mid-epoch
    assert threading.active_count() <= before
    bad = tmp_path / "bad"
    bad.mkdir()
    (bad / "x.tfrecord.gz").write_bytes(gzip.compress(b"\x05\x00\x00\x00\x00\x00\x00\x00junk"))
    with pytest.raises(tfrecord.TFRecordError):
        list(tfr_data_loader(str(bad / "*.gz"), 1, timesteps=T, prefetch=2, pin_memory=False))


@pytest.mark.parametrize("verify", [True, False])
def test_huge_declared_length_is_truncation_not_overread(tmp_path, verify):
    """A header declaring a length within 4 of UINT64_MAX (length CRC valid)
    must be reported as a truncated record: `len + 4` would wrap to a small
    value and let the reader run off the end of the buffer."""
    import struct
    for ln in (2 ** 64 - 1, 2 ** 64 - 4, 2 ** 64 - 2, 2 ** 63):
        hdr = struct.pack("<Q", ln)
        blob = hdr + struct.pack("<I", ref.masked_crc32c(hdr)) + b"\0" * 32
        p = str(tmp_path / "huge.tfrecord.gz")
        with gzip.open(p, "wb") as fh:
            fh.write(blob)
        with tfrecord.Reader([p], T, drop_remainder=False, verify_crc=verify) as rd:
            with pytest.raises(tfrecord.TFRecordError, match="truncated"):
                list(rd.batches(1))
