"""Independent restatement of the TFRecord / tf.train.Example format — TEST
INFRASTRUCTURE ONLY (imported by tests/ alone, as the checker of the native
reader in pathtracker-models_amd/csrc/pt_tfrecord.cpp).

TensorFlow is not installed here and the reference has no TFRecord fixtures,
so parity of the native reader is pinned against the published formats:

* record framing (tensorflow/core/lib/io/record_writer.cc): u64 length LE,
  u32 masked crc32c(length), data, u32 masked crc32c(data);
  masked(c) = ((c >> 15) | (c << 17)) + 0xa282ead8
  (tensorflow/core/lib/hash/crc32c.h) — CRC32C here is a bitwise pure-Python
  loop, independent of the native slicing-by-8 tables;
* tf.train.Example (tensorflow/core/example/{example,feature}.proto) encoded
  and decoded by the ``protobuf`` package from a descriptor built here, i.e. by
  Google's own wire-format implementation, not by ours;
* GZIP (TFRecordDataset(compression_type='GZIP')) by Python's ``gzip``.

The payload schema is the reference's (utils/TFRDataset.py:7-12): 'label'
bytes, 'image' bytes, 'height' / 'width' int64.  Parity is "unpinned" against
TensorFlow itself (no TF-written files exist offline).
"""
from __future__ import annotations

import gzip
import struct

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory


def crc32c(data: bytes) -> int:
    c = 0xFFFFFFFF
    for b in data:
        c ^= b
        for _ in range(8):
            c = (c >> 1) ^ 0x82F63B78 if c & 1 else c >> 1
    return c ^ 0xFFFFFFFF


def masked_crc32c(data: bytes) -> int:
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def _example_class():
    fd = descriptor_pb2.FileDescriptorProto(name="oracle_tf_example.proto",
                                            package="oracle_tf", syntax="proto3")
    L = descriptor_pb2.FieldDescriptorProto

    def msg(name, fields, nested=()):
        m = fd.message_type.add(name=name)
        for fname, num, ftype, label, tname in fields:
            f = m.field.add(name=fname, number=num, type=ftype, label=label)
            if tname:
                f.type_name = tname
        return m

    rep, opt = L.LABEL_REPEATED, L.LABEL_OPTIONAL
    msg("BytesList", [("value", 1, L.TYPE_BYTES, rep, None)])
    msg("FloatList", [("value", 1, L.TYPE_FLOAT, rep, None)])
    msg("Int64List", [("value", 1, L.TYPE_INT64, rep, None)])
    feat = msg("Feature", [("bytes_list", 1, L.TYPE_MESSAGE, opt, ".oracle_tf.BytesList"),
                           ("float_list", 2, L.TYPE_MESSAGE, opt, ".oracle_tf.FloatList"),
                           ("int64_list", 3, L.TYPE_MESSAGE, opt, ".oracle_tf.Int64List")])
    feat.oneof_decl.add(name="kind")
    for f in feat.field:
        f.oneof_index = 0
    feats = msg("Features", [("feature", 1, L.TYPE_MESSAGE, rep, ".oracle_tf.Features.FeatureEntry")])
    entry = feats.nested_type.add(name="FeatureEntry")
    entry.field.add(name="key", number=1, type=L.TYPE_STRING, label=opt)
    entry.field.add(name="value", number=2, type=L.TYPE_MESSAGE, label=opt,
                    type_name=".oracle_tf.Feature")
    entry.options.map_entry = True
    msg("Example", [("features", 1, L.TYPE_MESSAGE, opt, ".oracle_tf.Features")])
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    return message_factory.GetMessageClass(pool.FindMessageTypeByName("oracle_tf.Example"))


Example = _example_class()


def encode_example(image: bytes, label: bytes, height: int = 32, width: int = 32) -> bytes:
    ex = Example()
    f = ex.features.feature
    f["image"].bytes_list.value.append(image)
    f["label"].bytes_list.value.append(label)
    f["height"].int64_list.value.append(height)
    f["width"].int64_list.value.append(width)
    return ex.SerializeToString()


def decode_example(data: bytes):
    ex = Example()
    ex.ParseFromString(data)
    f = ex.features.feature
    return (bytes(f["image"].bytes_list.value[0]), bytes(f["label"].bytes_list.value[0]),
            int(f["height"].int64_list.value[0]), int(f["width"].int64_list.value[0]))


def frame(data: bytes) -> bytes:
    hdr = struct.pack("<Q", len(data))
    return (hdr + struct.pack("<I", masked_crc32c(hdr)) + data
            + struct.pack("<I", masked_crc32c(data)))


def write_file(path: str, records, compress: bool = True):
    blob = b"".join(frame(r) for r in records)
    with (gzip.open(path, "wb") if compress else open(path, "wb")) as fh:
        fh.write(blob)


def read_file(path: str, compress: bool = True, verify: bool = True):
    with (gzip.open(path, "rb") if compress else open(path, "rb")) as fh:
        blob = fh.read()
    out, off = [], 0
    while off < len(blob):
        (n,) = struct.unpack_from("<Q", blob, off)
        (lc,) = struct.unpack_from("<I", blob, off + 8)
        data = blob[off + 12: off + 12 + n]
        (dc,) = struct.unpack_from("<I", blob, off + 12 + n)
        if verify:
            assert lc == masked_crc32c(blob[off:off + 8]), "length crc"
            assert dc == masked_crc32c(data), "data crc"
        out.append(data)
        off += 16 + n
    return out
