"""TensorFlow TensorBundle (V2 checkpoint) writer and reader, implemented from the format.

Reproduces the on-disk layout the reference's MonitoredTrainingSession/Saver produced in
`--log_root`:
  <prefix>.index                    LevelDB-format SSTable: key ""  -> BundleHeaderProto,
                                    key <tensor name> -> BundleEntryProto (sorted keys)
  <prefix>.data-00000-of-00001      raw little-endian tensor bytes, concatenated
Protos (tensorflow/core/protobuf/tensor_bundle.proto):
  BundleHeaderProto { int32 num_shards = 1; Endianness endianness = 2; VersionDef version = 3; }
  BundleEntryProto  { DataType dtype = 1; TensorShapeProto shape = 2; int32 shard_id = 3;
                      int64 offset = 4; int64 size = 5; fixed32 crc32c = 6 (masked); }
  TensorShapeProto  { repeated Dim dim = 2 { int64 size = 1; } }
SSTable: prefix-compressed data blocks with restart points, a block trailer of
{compression type 0, masked crc32c(block + type)}, an empty metaindex block, an index block
(restart interval 1) of BlockHandle{varint offset, varint size}, and a 48-byte footer ending in
the table magic 0xdb4775248b80fb57.
"""
from __future__ import annotations

import os
import struct
from typing import Dict, Iterable, List, Tuple

import numpy as np

from ..utils import crc32c
from ..utils import pbwire as pb

TABLE_MAGIC = 0xDB4775248B80FB57
DTYPES = {np.dtype(np.float32): 1, np.dtype(np.float64): 2, np.dtype(np.int32): 3, np.dtype(np.uint8): 4,
          np.dtype(np.int64): 9, np.dtype(np.float16): 19}
NP_OF = {v: k for k, v in DTYPES.items()}
BLOCK_SIZE = 4096


def _common(a: bytes, b: bytes) -> int:
    n = min(len(a), len(b))
    i = 0
    while i < n and a[i] == b[i]:
        i += 1
    return i


def _build_block(entries: List[Tuple[bytes, bytes]], restart_interval: int) -> bytes:
    buf = bytearray()
    restarts = []
    last = b""
    for i, (k, v) in enumerate(entries):
        if i % restart_interval == 0:
            restarts.append(len(buf))
            shared = 0
        else:
            shared = _common(last, k)
        buf += pb.varint(shared) + pb.varint(len(k) - shared) + pb.varint(len(v)) + k[shared:] + v
        last = k
    if not restarts:
        restarts = [0]
    for r in restarts:
        buf += struct.pack("<I", r)
    buf += struct.pack("<I", len(restarts))
    return bytes(buf)


def _handle(offset: int, size: int) -> bytes:
    return pb.varint(offset) + pb.varint(size)


def write_sstable(path: str, items: Iterable[Tuple[bytes, bytes]]):
    items = sorted(items, key=lambda kv: kv[0])
    out = bytearray()
    index_entries = []

    def emit(block: bytes) -> Tuple[int, int]:
        off = len(out)
        out.extend(block)
        trailer = b"\x00"
        out.extend(trailer + struct.pack("<I", crc32c.mask(crc32c.value(block + trailer))))
        return off, len(block)

    cur: List[Tuple[bytes, bytes]] = []
    cur_size = 0
    for k, v in items:
        cur.append((k, v))
        cur_size += len(k) + len(v) + 8
        if cur_size >= BLOCK_SIZE:
            off, size = emit(_build_block(cur, 16))
            index_entries.append((cur[-1][0], _handle(off, size)))
            cur, cur_size = [], 0
    if cur:
        off, size = emit(_build_block(cur, 16))
        index_entries.append((cur[-1][0], _handle(off, size)))
    meta_off, meta_size = emit(_build_block([], 16))
    idx_off, idx_size = emit(_build_block(index_entries, 1))
    footer = _handle(meta_off, meta_size) + _handle(idx_off, idx_size)
    footer += b"\x00" * (40 - len(footer)) + struct.pack("<Q", TABLE_MAGIC)
    out.extend(footer)
    with open(path, "wb") as f:
        f.write(bytes(out))


def _parse_block(data: bytes) -> List[Tuple[bytes, bytes]]:
    (nr,) = struct.unpack_from("<I", data, len(data) - 4)
    limit = len(data) - 4 - 4 * nr
    pos, last, out = 0, b"", []
    while pos < limit:
        shared, pos = pb.read_varint(data, pos)
        unshared, pos = pb.read_varint(data, pos)
        vlen, pos = pb.read_varint(data, pos)
        key = last[:shared] + data[pos:pos + unshared]
        pos += unshared
        out.append((key, data[pos:pos + vlen]))
        pos += vlen
        last = key
    return out


def read_sstable(path: str, verify: bool = True) -> Dict[bytes, bytes]:
    with open(path, "rb") as f:
        buf = f.read()
    if len(buf) < 48 or struct.unpack_from("<Q", buf, len(buf) - 8)[0] != TABLE_MAGIC:
        raise ValueError(f"{path}: not an SSTable (bad magic)")
    footer = buf[-48:]
    _, p = pb.read_varint(footer, 0)
    _, p = pb.read_varint(footer, p)
    idx_off, p = pb.read_varint(footer, p)
    idx_size, p = pb.read_varint(footer, p)

    def block(off, size):
        data = buf[off:off + size]
        if verify:
            (c,) = struct.unpack_from("<I", buf, off + size + 1)
            if crc32c.mask(crc32c.value(data + buf[off + size:off + size + 1])) != c:
                raise ValueError(f"{path}: block checksum mismatch at {off}")
        return data

    out = {}
    for _, h in _parse_block(block(idx_off, idx_size)):
        off, q = pb.read_varint(h, 0)
        size, _ = pb.read_varint(h, q)
        for k, v in _parse_block(block(off, size)):
            out[k] = v
    return out


def _shape_proto(shape) -> bytes:
    return b"".join(pb.f_bytes(2, pb.f_varint(1, d)) for d in shape)


def write_bundle(prefix: str, tensors: Dict[str, np.ndarray]):
    """Writes <prefix>.index and <prefix>.data-00000-of-00001 (little-endian, 1 shard)."""
    data_path = prefix + ".data-00000-of-00001"
    items = [(b"", pb.f_varint(1, 1) + pb.f_bytes(3, pb.f_varint(1, 1)))]  # num_shards=1, version.producer=1
    offset = 0
    with open(data_path, "wb") as f:
        for name in sorted(tensors):
            arr = np.asarray(tensors[name])
            if not arr.flags["C_CONTIGUOUS"]:
                arr = arr.copy(order="C")  # (np.ascontiguousarray would turn scalars into 1-d)
            if arr.dtype not in DTYPES:
                raise TypeError(f"unsupported dtype {arr.dtype} for {name}")
            raw = arr.astype(arr.dtype.newbyteorder("<"), copy=False).tobytes()
            f.write(raw)
            entry = (pb.f_varint(1, DTYPES[arr.dtype]) + pb.f_bytes(2, _shape_proto(arr.shape)) +
                     (pb.f_varint(4, offset) if offset else b"") + (pb.f_varint(5, len(raw)) if raw else b"") +
                     pb.f_fixed32(6, crc32c.masked_value(raw)))
            items.append((name.encode(), entry))
            offset += len(raw)
    write_sstable(prefix + ".index", items)


def read_bundle(prefix: str, verify: bool = True) -> Dict[str, np.ndarray]:
    table = read_sstable(prefix + ".index", verify)
    hdr = pb.decode(table.get(b"", b""))
    nshards = hdr.get(1, [1])[0]
    if nshards != 1:
        raise NotImplementedError("multi-shard bundles")
    with open(prefix + ".data-00000-of-00001", "rb") as f:
        data = f.read()
    out = {}
    for k, v in table.items():
        if k == b"":
            continue
        e = pb.decode(v)
        dt = NP_OF[e.get(1, [1])[0]]
        shape = []
        if 2 in e:
            for d in pb.decode(e[2][0]).get(2, []):
                shape.append(pb.signed64(pb.decode(d).get(1, [0])[0]))
        off = e.get(4, [0])[0]
        size = e.get(5, [0])[0]
        raw = data[off:off + size]
        if verify and 6 in e and crc32c.masked_value(raw) != pb.as_fixed32(e[6][0]):
            raise ValueError(f"checksum mismatch for tensor {k.decode()}")
        out[k.decode()] = np.frombuffer(raw, dtype=dt).reshape(shape).copy()
    return out
