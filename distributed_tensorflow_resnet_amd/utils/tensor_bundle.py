"""TensorFlow V2 checkpoint ("tensor bundle") reader/writer without TensorFlow.

Keeps the reference's checkpoint layout (SURVEY §2.6, §5 checkpoint row,
Appendix B): ``<prefix>.index`` is a LevelDB-format table whose first entry
(key "") is a BundleHeaderProto and whose remaining entries map the sorted
variable names to BundleEntryProto {dtype, shape, shard_id, offset, size,
crc32c}; ``<prefix>.data-00000-of-00001`` holds the raw little-endian tensor
bytes back to back in key order.  The ``checkpoint`` text file (CheckpointState)
lists the latest and all retained prefixes.

The LevelDB table is built exactly like TF's ``table::TableBuilder`` (restart
interval 16, 256 KiB blocks, no compression, masked-CRC32C block trailers,
shortest-separator index keys, 48-byte footer with magic 0xdb4775248b80fb57),
so an index written from the same entries is byte-identical to TF's
(tests/test_checkpoint.py checks this against the reference's own files).
"""
from __future__ import annotations

import os
import struct
from dataclasses import dataclass, field

import numpy as np

from . import crc32c

MAGIC = 0xDB4775248B80FB57
BLOCK_SIZE = 262144
RESTART_INTERVAL = 16

# tensorflow/core/framework/types.proto
DT = {1: np.float32, 2: np.float64, 3: np.int32, 4: np.uint8, 6: np.int8, 9: np.int64,
      10: np.bool_, 19: np.float16}
DT_BFLOAT16 = 14
NP2DT = {np.dtype(np.float32): 1, np.dtype(np.float64): 2, np.dtype(np.int32): 3,
         np.dtype(np.uint8): 4, np.dtype(np.int8): 6, np.dtype(np.int64): 9,
         np.dtype(np.bool_): 10, np.dtype(np.float16): 19}


# ---------------------------------------------------------------- varint / proto
def put_varint(out: bytearray, v: int) -> None:
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return


def get_varint(buf, pos: int) -> tuple[int, int]:
    shift = 0
    result = 0
    while True:
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, pos
        shift += 7


def _proto_fields(buf: bytes):
    """Yield (field_number, wire_type, value) of a serialized message."""
    pos = 0
    n = len(buf)
    while pos < n:
        tag, pos = get_varint(buf, pos)
        fnum, wt = tag >> 3, tag & 7
        if wt == 0:
            v, pos = get_varint(buf, pos)
        elif wt == 1:
            v = struct.unpack_from("<Q", buf, pos)[0]
            pos += 8
        elif wt == 2:
            ln, pos = get_varint(buf, pos)
            v = bytes(buf[pos:pos + ln])
            pos += ln
        elif wt == 5:
            v = struct.unpack_from("<I", buf, pos)[0]
            pos += 4
        else:
            raise ValueError(f"unsupported wire type {wt}")
        yield fnum, wt, v


def _key(out: bytearray, fnum: int, wt: int):
    put_varint(out, (fnum << 3) | wt)


@dataclass
class BundleEntry:
    dtype: int = 1
    shape: tuple = ()
    shard_id: int = 0
    offset: int = 0
    size: int = 0
    crc32c: int = 0

    def encode(self) -> bytes:
        """proto3 BundleEntryProto (default-valued fields omitted, field order as TF)."""
        out = bytearray()
        if self.dtype:
            _key(out, 1, 0)
            put_varint(out, self.dtype)
        shp = bytearray()
        for d in self.shape:
            dim = bytearray()
            if d:
                _key(dim, 1, 0)
                put_varint(dim, int(d))
            _key(shp, 2, 2)
            put_varint(shp, len(dim))
            shp += dim
        _key(out, 2, 2)
        put_varint(out, len(shp))
        out += shp
        if self.shard_id:
            _key(out, 3, 0)
            put_varint(out, self.shard_id)
        if self.offset:
            _key(out, 4, 0)
            put_varint(out, self.offset)
        if self.size:
            _key(out, 5, 0)
            put_varint(out, self.size)
        if self.crc32c:
            _key(out, 6, 5)
            out += struct.pack("<I", self.crc32c)
        return bytes(out)

    @staticmethod
    def decode(buf: bytes) -> "BundleEntry":
        e = BundleEntry()
        for f, wt, v in _proto_fields(buf):
            if f == 1:
                e.dtype = v
            elif f == 2:
                dims = []
                for f2, _, v2 in _proto_fields(v):
                    if f2 == 2:
                        size = 0
                        for f3, _, v3 in _proto_fields(v2):
                            if f3 == 1:
                                size = v3
                        dims.append(size)
                e.shape = tuple(dims)
            elif f == 3:
                e.shard_id = v
            elif f == 4:
                e.offset = v
            elif f == 5:
                e.size = v
            elif f == 6:
                e.crc32c = v
        return e


def encode_header(num_shards: int = 1, producer: int = 1) -> bytes:
    """BundleHeaderProto {num_shards, endianness=LITTLE (default), version{producer}}."""
    out = bytearray()
    _key(out, 1, 0)
    put_varint(out, num_shards)
    ver = bytearray()
    _key(ver, 1, 0)
    put_varint(ver, producer)
    _key(out, 3, 2)
    put_varint(out, len(ver))
    out += ver
    return bytes(out)


def decode_header(buf: bytes) -> dict:
    h = {"num_shards": 0, "endianness": 0, "producer": 0}
    for f, _, v in _proto_fields(buf):
        if f == 1:
            h["num_shards"] = v
        elif f == 2:
            h["endianness"] = v
        elif f == 3:
            for f2, _, v2 in _proto_fields(v):
                if f2 == 1:
                    h["producer"] = v2
    return h


# ---------------------------------------------------------------- LevelDB table
class _BlockBuilder:
    def __init__(self, restart_interval: int = RESTART_INTERVAL):
        self.buf = bytearray()
        self.restarts = [0]
        self.counter = 0
        self.last_key = b""
        self.interval = restart_interval
        self.n = 0

    def add(self, key: bytes, value: bytes):
        shared = 0
        if self.counter < self.interval:
            m = min(len(self.last_key), len(key))
            while shared < m and self.last_key[shared] == key[shared]:
                shared += 1
        else:
            self.restarts.append(len(self.buf))
            self.counter = 0
        put_varint(self.buf, shared)
        put_varint(self.buf, len(key) - shared)
        put_varint(self.buf, len(value))
        self.buf += key[shared:]
        self.buf += value
        self.last_key = key
        self.counter += 1
        self.n += 1

    def size_estimate(self) -> int:
        return len(self.buf) + 4 * len(self.restarts) + 4

    def finish(self) -> bytes:
        out = bytearray(self.buf)
        for r in self.restarts:
            out += struct.pack("<I", r)
        out += struct.pack("<I", len(self.restarts))
        return bytes(out)

    def empty(self) -> bool:
        return self.n == 0


def _shortest_separator(start: bytes, limit: bytes) -> bytes:
    m = min(len(start), len(limit))
    i = 0
    while i < m and start[i] == limit[i]:
        i += 1
    if i >= m:
        return start
    b = start[i]
    if b < 0xFF and b + 1 < limit[i]:
        return start[:i] + bytes([b + 1])
    return start


def _short_successor(key: bytes) -> bytes:
    for i, b in enumerate(key):
        if b != 0xFF:
            return key[:i] + bytes([b + 1])
    return key


def _handle(offset: int, size: int) -> bytes:
    out = bytearray()
    put_varint(out, offset)
    put_varint(out, size)
    return bytes(out)


def build_table(items: list[tuple[bytes, bytes]], block_size: int = BLOCK_SIZE) -> bytes:
    """LevelDB table of sorted (key, value) pairs, no compression."""
    out = bytearray()
    data = _BlockBuilder()
    index = _BlockBuilder(restart_interval=1)
    pending = None  # handle of the last flushed data block
    last_key = b""

    def write_block(block: bytes) -> tuple[int, int]:
        off = len(out)
        out.extend(block)
        trailer = b"\x00"
        c = crc32c.mask(crc32c.extend(crc32c.value(block), trailer))
        out.extend(trailer + struct.pack("<I", c))
        return off, len(block)

    for key, value in items:
        if pending is not None:
            sep = _shortest_separator(last_key, key)
            index.add(sep, _handle(*pending))
            pending = None
        data.add(key, value)
        last_key = key
        if data.size_estimate() >= block_size:
            pending = write_block(data.finish())
            data = _BlockBuilder()
    if not data.empty():
        pending = write_block(data.finish())
    meta_handle = write_block(_BlockBuilder().finish())
    if pending is not None:
        index.add(_short_successor(last_key), _handle(*pending))
    index_handle = write_block(index.finish())
    footer = bytearray(_handle(*meta_handle) + _handle(*index_handle))
    footer += b"\x00" * (40 - len(footer))
    footer += struct.pack("<Q", MAGIC)
    out += footer
    return bytes(out)


def _read_block(buf: bytes, off: int, size: int, verify: bool = True) -> list[tuple[bytes, bytes]]:
    block = buf[off:off + size]
    if verify:
        ctype = buf[off + size]
        want = struct.unpack_from("<I", buf, off + size + 1)[0]
        got = crc32c.mask(crc32c.extend(crc32c.value(block), bytes([ctype])))
        if want != got:
            raise IOError(f"block checksum mismatch at {off}")
        if ctype != 0:
            raise IOError("compressed tables are not supported")
    nrest = struct.unpack_from("<I", block, len(block) - 4)[0]
    end = len(block) - 4 - 4 * nrest
    pos = 0
    key = b""
    out = []
    while pos < end:
        shared, pos = get_varint(block, pos)
        non_shared, pos = get_varint(block, pos)
        vlen, pos = get_varint(block, pos)
        key = key[:shared] + bytes(block[pos:pos + non_shared])
        pos += non_shared
        out.append((key, bytes(block[pos:pos + vlen])))
        pos += vlen
    return out


def read_table(buf: bytes, verify: bool = True) -> list[tuple[bytes, bytes]]:
    if len(buf) < 48 or struct.unpack_from("<Q", buf, len(buf) - 8)[0] != MAGIC:
        raise IOError("not a LevelDB table (bad magic)")
    foot = buf[len(buf) - 48:]
    _mo, p = get_varint(foot, 0)
    _ms, p = get_varint(foot, p)
    io, p = get_varint(foot, p)
    isz, p = get_varint(foot, p)
    items = []
    for _k, hv in _read_block(buf, io, isz, verify):
        off, q = get_varint(hv, 0)
        sz, _ = get_varint(hv, q)
        items.extend(_read_block(buf, off, sz, verify))
    return items


# ---------------------------------------------------------------- bundle API
def data_path(prefix: str, shard: int = 0, num_shards: int = 1) -> str:
    return f"{prefix}.data-{shard:05d}-of-{num_shards:05d}"


def write_bundle(prefix: str, tensors: dict, atomic: bool = True) -> dict[str, BundleEntry]:
    """Write ``tensors`` (name -> array-like) as a TF V2 checkpoint."""
    names = sorted(tensors)
    entries: dict[str, BundleEntry] = {}
    d_tmp = data_path(prefix) + (".tmp" if atomic else "")
    off = 0
    with open(d_tmp, "wb") as fh:
        for n in names:
            a = np.asarray(tensors[n])
            if not a.flags.c_contiguous:
                a = a.copy()  # (np.ascontiguousarray would turn 0-d into 1-d)
            if a.dtype not in NP2DT:
                a = a.astype(np.float32)
            raw = a.astype(a.dtype.newbyteorder("<"), copy=False).tobytes()
            fh.write(raw)
            entries[n] = BundleEntry(NP2DT[a.dtype], tuple(a.shape), 0, off, len(raw),
                                     crc32c.mask(crc32c.value(raw)))
            off += len(raw)
    items = [(b"", encode_header())]
    items += [(n.encode(), entries[n].encode()) for n in names]
    i_tmp = prefix + ".index" + (".tmp" if atomic else "")
    with open(i_tmp, "wb") as fh:
        fh.write(build_table(items))
    if atomic:
        os.replace(d_tmp, data_path(prefix))
        os.replace(i_tmp, prefix + ".index")
    return entries


def read_index(prefix_or_path: str) -> tuple[dict, dict[str, BundleEntry]]:
    path = prefix_or_path if prefix_or_path.endswith(".index") else prefix_or_path + ".index"
    with open(path, "rb") as fh:
        buf = fh.read()
    items = read_table(buf)
    header = {}
    entries = {}
    for k, v in items:
        if k == b"":
            header = decode_header(v)
        else:
            entries[k.decode()] = BundleEntry.decode(v)
    return header, entries


def read_bundle(prefix: str, names=None, verify: bool = True) -> dict[str, np.ndarray]:
    header, entries = read_index(prefix)
    nshards = max(header.get("num_shards", 1), 1)
    out = {}
    files = {}
    try:
        for n, e in entries.items():
            if names is not None and n not in names:
                continue
            if e.shard_id not in files:
                files[e.shard_id] = open(data_path(prefix, e.shard_id, nshards), "rb")
            fh = files[e.shard_id]
            fh.seek(e.offset)
            raw = fh.read(e.size)
            if verify and e.crc32c and crc32c.mask(crc32c.value(raw)) != e.crc32c:
                raise IOError(f"checksum mismatch for {n}")
            if e.dtype == DT_BFLOAT16:
                u = np.frombuffer(raw, dtype="<u2").astype(np.uint32) << 16
                arr = u.view(np.float32)
            else:
                arr = np.frombuffer(raw, dtype=np.dtype(DT[e.dtype]).newbyteorder("<"))
            out[n] = arr.reshape(e.shape).copy()
    finally:
        for fh in files.values():
            fh.close()
    return out


# ---------------------------------------------------------------- checkpoint state
def write_checkpoint_state(directory: str, latest: str, all_paths: list[str]) -> None:
    """The ``checkpoint`` text file (CheckpointState proto in text format)."""
    lines = [f'model_checkpoint_path: "{latest}"']
    lines += [f'all_model_checkpoint_paths: "{p}"' for p in all_paths]
    tmp = os.path.join(directory, "checkpoint.tmp")
    with open(tmp, "w") as fh:
        fh.write("\n".join(lines) + "\n")
    os.replace(tmp, os.path.join(directory, "checkpoint"))


def read_checkpoint_state(directory: str) -> dict | None:
    path = os.path.join(directory, "checkpoint")
    if not os.path.exists(path):
        return None
    latest, all_paths = None, []
    with open(path) as fh:
        for line in fh:
            line = line.strip()
            if not line or ":" not in line:
                continue
            k, v = line.split(":", 1)
            v = v.strip().strip('"')
            if k == "model_checkpoint_path":
                latest = v
            elif k == "all_model_checkpoint_paths":
                all_paths.append(v)
    return {"model_checkpoint_path": latest, "all_model_checkpoint_paths": all_paths}


def latest_checkpoint(directory: str) -> str | None:
    """tf.train.latest_checkpoint: resolves relative/absolute/foreign prefixes."""
    st = read_checkpoint_state(directory)
    if not st or not st["model_checkpoint_path"]:
        return None
    p = st["model_checkpoint_path"]
    cands = [p, os.path.join(directory, p), os.path.join(directory, os.path.basename(p))]
    for c in cands:
        if os.path.exists(c + ".index"):
            return c
    return None
