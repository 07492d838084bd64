"""TFRecord framing, tf.train.Example parsing and TensorBoard event files.

All three formats share the masked-CRC32C framing:
    uint64 length | uint32 masked_crc(length) | data | uint32 masked_crc(data)

* TFRecord reader/writer: ImageNet shards (resnet_imagenet_main.py:110-163)
  and anything else the reference reads through tf.data.TFRecordDataset.
* tf.train.Example decoder: `image/encoded`, `image/class/label`, ... features
  (hand-decoded protobuf; TensorFlow is not a dependency).
* EventWriter: `events.out.tfevents.*` files with scalar (and image) summaries,
  readable by TensorBoard -- the SummarySaverHook / eval-summary outputs
  (resnet_cifar_main.py:288-293, 405-416).
"""
from __future__ import annotations

import io
import os
import socket
import struct
import time

from . import crc32c
from .tensor_bundle import _proto_fields, put_varint


# ---------------------------------------------------------------- TFRecord
def write_record(fh, data: bytes) -> None:
    hdr = struct.pack("<Q", len(data))
    fh.write(hdr)
    fh.write(struct.pack("<I", crc32c.mask(crc32c.value(hdr))))
    fh.write(data)
    fh.write(struct.pack("<I", crc32c.mask(crc32c.value(data))))


def read_records(path_or_fh, verify: bool = True):
    """Iterate the records of a TFRecord file (uncompressed)."""
    fh = open(path_or_fh, "rb") if isinstance(path_or_fh, (str, os.PathLike)) else path_or_fh
    try:
        while True:
            hdr = fh.read(8)
            if not hdr:
                return
            if len(hdr) < 8:
                raise IOError("truncated record header")
            (n,) = struct.unpack("<Q", hdr)
            (hcrc,) = struct.unpack("<I", fh.read(4))
            if verify and crc32c.mask(crc32c.value(hdr)) != hcrc:
                raise IOError("corrupted record length")
            data = fh.read(n)
            (dcrc,) = struct.unpack("<I", fh.read(4))
            if verify and crc32c.mask(crc32c.value(data)) != dcrc:
                raise IOError("corrupted record data")
            yield data
    finally:
        if fh is not path_or_fh:
            fh.close()


class RecordWriter:
    def __init__(self, path: str):
        self.fh = open(path, "wb")

    def write(self, data: bytes) -> None:
        write_record(self.fh, data)

    def flush(self):
        self.fh.flush()

    def close(self):
        self.fh.close()


# ---------------------------------------------------------------- tf.train.Example
def parse_example(buf: bytes) -> dict:
    """-> {feature name: list of bytes | list of float | list of int}."""
    out = {}
    for f, _, features in _proto_fields(buf):
        if f != 1:
            continue
        for f2, _, entry in _proto_fields(features):
            if f2 != 1:
                continue
            key, feat = None, b""
            for f3, _, v in _proto_fields(entry):
                if f3 == 1:
                    key = v.decode()
                elif f3 == 2:
                    feat = v
            out[key] = _parse_feature(feat)
    return out


def _parse_feature(buf: bytes):
    for kind, _, lst in _proto_fields(buf):
        vals = []
        for f, wt, v in _proto_fields(lst):
            if f != 1:
                continue
            if kind == 1:
                vals.append(v)
            elif kind == 2:
                if wt == 2:  # packed floats
                    vals.extend(struct.unpack(f"<{len(v) // 4}f", v))
                else:
                    vals.append(struct.unpack("<f", struct.pack("<I", v))[0])
            elif kind == 3:
                if wt == 2:  # packed varints
                    pos = 0
                    from .tensor_bundle import get_varint

                    while pos < len(v):
                        x, pos = get_varint(v, pos)
                        vals.append(x - (1 << 64) if x >= 1 << 63 else x)
                else:
                    vals.append(v - (1 << 64) if v >= 1 << 63 else v)
        return vals
    return []


def _len_delim(out: bytearray, field: int, payload: bytes):
    put_varint(out, (field << 3) | 2)
    put_varint(out, len(payload))
    out += payload


def make_example(features: dict) -> bytes:
    """Encode {name: bytes | list[bytes] | int | list[int] | float | list[float]}."""
    feats = bytearray()
    for name, val in features.items():
        vals = val if isinstance(val, (list, tuple)) else [val]
        lst = bytearray()
        if vals and isinstance(vals[0], (bytes, bytearray)):
            for v in vals:
                _len_delim(lst, 1, bytes(v))
            kind = 1
        elif vals and isinstance(vals[0], float):
            _len_delim(lst, 1, struct.pack(f"<{len(vals)}f", *vals))
            kind = 2
        else:
            packed = bytearray()
            for v in vals:
                put_varint(packed, int(v) & ((1 << 64) - 1))
            _len_delim(lst, 1, bytes(packed))
            kind = 3
        feature = bytearray()
        _len_delim(feature, kind, bytes(lst))
        entry = bytearray()
        _len_delim(entry, 1, name.encode())
        _len_delim(entry, 2, bytes(feature))
        _len_delim(feats, 1, bytes(entry))
    ex = bytearray()
    _len_delim(ex, 1, bytes(feats))
    return bytes(ex)


# ---------------------------------------------------------------- event files
def _scalar_value(tag: str, value: float) -> bytes:
    v = bytearray()
    _len_delim(v, 1, tag.encode())
    put_varint(v, (2 << 3) | 5)
    v += struct.pack("<f", float(value))
    return bytes(v)


def _image_value(tag: str, png: bytes, h: int, w: int, c: int) -> bytes:
    img = bytearray()
    put_varint(img, 1 << 3)
    put_varint(img, h)
    put_varint(img, 2 << 3)
    put_varint(img, w)
    put_varint(img, 3 << 3)
    put_varint(img, c)
    _len_delim(img, 4, png)
    v = bytearray()
    _len_delim(v, 1, tag.encode())
    _len_delim(v, 4, bytes(img))
    return bytes(v)


def _event(wall_time: float, step: int, file_version: str | None = None,
           summary_values: list | None = None) -> bytes:
    e = bytearray()
    put_varint(e, (1 << 3) | 1)
    e += struct.pack("<d", wall_time)
    if step:
        put_varint(e, 2 << 3)
        put_varint(e, int(step))
    if file_version is not None:
        _len_delim(e, 3, file_version.encode())
    if summary_values is not None:
        summ = bytearray()
        for sv in summary_values:
            _len_delim(summ, 1, sv)
        _len_delim(e, 5, bytes(summ))
    return bytes(e)


class EventWriter:
    """Minimal tf.summary.FileWriter: scalars (+ optional PNG images)."""

    def __init__(self, logdir: str, filename_suffix: str = ""):
        os.makedirs(logdir, exist_ok=True)
        name = f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}{filename_suffix}"
        self.path = os.path.join(logdir, name)
        self.writer = RecordWriter(self.path)
        self.writer.write(_event(time.time(), 0, file_version="brain.Event:2"))
        self.writer.flush()

    def add_scalars(self, step: int, scalars: dict) -> None:
        vals = [_scalar_value(k, v) for k, v in scalars.items()]
        self.writer.write(_event(time.time(), step, summary_values=vals))

    def add_scalar(self, tag: str, value: float, step: int) -> None:
        self.add_scalars(step, {tag: value})

    def add_image(self, tag: str, hwc_uint8, step: int) -> None:
        """PNG-encode an HWC uint8 array (PIL) as an image summary."""
        from PIL import Image

        arr = hwc_uint8
        buf = io.BytesIO()
        Image.fromarray(arr).save(buf, format="PNG")
        h, w = arr.shape[:2]
        c = arr.shape[2] if arr.ndim == 3 else 1
        self.writer.write(_event(time.time(), step,
                                 summary_values=[_image_value(tag, buf.getvalue(), h, w, c)]))

    def flush(self):
        self.writer.flush()

    def close(self):
        self.writer.close()


def read_events(path: str) -> list[dict]:
    """Decode an event file into [{step, wall_time, scalars:{tag: value}}] (tests/tools)."""
    out = []
    for rec in read_records(path):
        ev = {"step": 0, "wall_time": 0.0, "scalars": {}, "file_version": None}
        for f, wt, v in _proto_fields(rec):
            if f == 1:
                ev["wall_time"] = struct.unpack("<d", struct.pack("<Q", v))[0]
            elif f == 2:
                ev["step"] = v
            elif f == 3:
                ev["file_version"] = v.decode()
            elif f == 5:
                for f2, _, val in _proto_fields(v):
                    if f2 != 1:
                        continue
                    tag, sv = None, None
                    for f3, wt3, x in _proto_fields(val):
                        if f3 == 1:
                            tag = x.decode()
                        elif f3 == 2:
                            sv = struct.unpack("<f", struct.pack("<I", x))[0]
                    if tag is not None and sv is not None:
                        ev["scalars"][tag] = sv
        out.append(ev)
    return out
