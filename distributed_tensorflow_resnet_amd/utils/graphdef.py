"""TensorFlow GraphDef / MetaGraphDef codec without TensorFlow (data only).

The reference freezes its trained CIFAR ResNet-50 into a GraphDef
(`resnet_cifar_frozen_model.py:111-122`, outputs "predictions,precision") and
loads it back for inference (`resnet_cifar_predict_from_pd.py:66-74`).  The
frozen file it ships (`test/resnet50-cifar-ckpt-20190218/
resnet50_cifar_frozen_model_eval.pb`) holds the trained weights as Const nodes.

This module is a hand-rolled protobuf wire-format codec for the subset of
`tensorflow/core/framework/{graph,node_def,attr_value,tensor,tensor_shape,
versions,types}.proto` those files use.  Decoding never executes anything from
the file: it only parses tag/length/value records into plain Python objects
(NodeDef -> `Node`, TensorProto -> numpy array).  Encoding writes the same
schema, so a graph we export (utils/frozen.py) is readable by TF's
`GraphDef.ParseFromString` and by this decoder.

Field numbers (proto3 unless noted):
  GraphDef      node=1 library=2 version=3 versions=4
  NodeDef       name=1 op=2 input=3 device=4 attr=5 (map<string,AttrValue>: key=1 value=2)
  AttrValue     list=1 s=2 i=3 f=4 b=5 type=6 shape=7 tensor=8 placeholder=9 func=10
  ListValue     s=2 i=3 f=4 b=5 type=6 shape=7 tensor=8 func=9
  TensorProto   dtype=1 tensor_shape=2 version_number=3 tensor_content=4 float_val=5
                double_val=6 int_val=7 string_val=8 int64_val=10 bool_val=11 half_val=13
  TensorShapeProto dim=2 (Dim: size=1 name=2) unknown_rank=3
  VersionDef    producer=1 min_consumer=2 bad_consumers=3
  MetaGraphDef  meta_info_def=1 graph_def=2 saver_def=3 collection_def=4
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field

import numpy as np

from .tensor_bundle import _proto_fields, get_varint, put_varint

# tensorflow/core/framework/types.proto
DT_FLOAT, DT_DOUBLE, DT_INT32, DT_UINT8, DT_INT8, DT_STRING = 1, 2, 3, 4, 6, 7
DT_INT64, DT_BOOL, DT_BFLOAT16, DT_HALF = 9, 10, 14, 19
_DT_NP = {DT_FLOAT: np.float32, DT_DOUBLE: np.float64, DT_INT32: np.int32, DT_UINT8: np.uint8,
          DT_INT8: np.int8, DT_INT64: np.int64, DT_BOOL: np.bool_, DT_HALF: np.float16}
_NP_DT = {np.dtype(v): k for k, v in _DT_NP.items()}


@dataclass
class Shape:
    dims: list | None  # None = unknown rank; -1 = unknown dim

    def __repr__(self):
        return "Shape(?)" if self.dims is None else f"Shape({self.dims})"


@dataclass
class Node:
    name: str
    op: str
    inputs: list = field(default_factory=list)
    device: str = ""
    attr: dict = field(default_factory=dict)


@dataclass
class Graph:
    nodes: list
    producer: int = 0
    min_consumer: int = 0

    def by_name(self) -> dict:
        return {n.name: n for n in self.nodes}

    def op_census(self) -> dict:
        c: dict = {}
        for n in self.nodes:
            c[n.op] = c.get(n.op, 0) + 1
        return dict(sorted(c.items()))


# ------------------------------------------------------------------ decoding
def _packed(v, wt, fmt_size, fmt):
    """Repeated scalar field: packed (wt 2) or one unpacked element."""
    if wt == 2:
        if fmt == "varint":
            out, pos = [], 0
            while pos < len(v):
                x, pos = get_varint(v, pos)
                out.append(x)
            return out
        return list(struct.unpack(f"<{len(v) // fmt_size}{fmt}", v))
    if fmt == "f":
        return [struct.unpack("<f", struct.pack("<I", v))[0]]
    if fmt == "d":
        return [struct.unpack("<d", struct.pack("<Q", v))[0]]
    return [v]


def _signed64(x: int) -> int:
    return x - (1 << 64) if x >= (1 << 63) else x


def decode_shape(buf: bytes) -> Shape:
    dims, unknown = [], False
    for f, _, v in _proto_fields(buf):
        if f == 2:
            size = 0
            for f2, _, v2 in _proto_fields(v):
                if f2 == 1:
                    size = _signed64(v2)
            dims.append(size)
        elif f == 3 and v:
            unknown = True
    return Shape(None if unknown else dims)


def decode_tensor(buf: bytes) -> np.ndarray:
    dtype, shape, content = DT_FLOAT, Shape([]), None
    vals: dict = {}
    for f, wt, v in _proto_fields(buf):
        if f == 1:
            dtype = v
        elif f == 2:
            shape = decode_shape(v)
        elif f == 4:
            content = v
        elif f == 5:
            vals.setdefault("f", []).extend(_packed(v, wt, 4, "f"))
        elif f == 6:
            vals.setdefault("d", []).extend(_packed(v, wt, 8, "d"))
        elif f == 7:
            vals.setdefault("i", []).extend(_signed64(x) for x in _packed(v, wt, 0, "varint"))
        elif f == 13:
            vals.setdefault("i", []).extend(_packed(v, wt, 0, "varint"))
        elif f == 10:
            vals.setdefault("i", []).extend(_signed64(x) for x in _packed(v, wt, 0, "varint"))
        elif f == 11:
            vals.setdefault("i", []).extend(_packed(v, wt, 0, "varint"))
        elif f == 8:
            vals.setdefault("s", []).append(v)
    dims = shape.dims or []
    if dtype == DT_STRING:
        arr = np.array(vals.get("s", []), dtype=object)
        return arr.reshape(dims) if arr.size == int(np.prod(dims)) else arr
    if dtype not in _DT_NP:
        raise ValueError(f"unsupported TensorProto dtype {dtype}")
    npd = np.dtype(_DT_NP[dtype])
    n = int(np.prod(dims)) if dims else 1
    if content is not None:
        arr = np.frombuffer(content, dtype=npd.newbyteorder("<")).astype(npd)
    else:
        flat = vals.get("f") or vals.get("d") or vals.get("i") or []
        if dtype == DT_HALF:
            arr = np.array(flat, dtype=np.uint16).view(np.float16)
        else:
            arr = np.array(flat, dtype=npd)
        if arr.size < n:   # TF repeats the last value to fill the shape
            fill = arr[-1] if arr.size else np.zeros((), npd)
            arr = np.concatenate([arr, np.full(n - arr.size, fill, dtype=npd)])
    return arr.reshape(dims)


def _decode_list(buf: bytes) -> list:
    out: list = []
    for f, wt, v in _proto_fields(buf):
        if f == 2:
            out.append(v)
        elif f == 3:
            out.extend(_signed64(x) for x in _packed(v, wt, 0, "varint"))
        elif f == 4:
            out.extend(_packed(v, wt, 4, "f"))
        elif f == 5:
            out.extend(bool(x) for x in _packed(v, wt, 0, "varint"))
        elif f == 6:
            out.extend(("type", x) for x in _packed(v, wt, 0, "varint"))
        elif f == 7:
            out.append(decode_shape(v))
        elif f == 8:
            out.append(decode_tensor(v))
    return out


def decode_attr(buf: bytes):
    """AttrValue -> python value: bytes / int / float / bool / ("type", dt) / Shape /
    ndarray / list.  An empty AttrValue (TF's empty list) decodes to []."""
    for f, wt, v in _proto_fields(buf):
        if f == 1:
            return _decode_list(v)
        if f == 2:
            return v
        if f == 3:
            return _signed64(v)
        if f == 4:
            return struct.unpack("<f", struct.pack("<I", v))[0]
        if f == 5:
            return bool(v)
        if f == 6:
            return ("type", v)
        if f == 7:
            return decode_shape(v)
        if f == 8:
            return decode_tensor(v)
        if f == 9:
            return ("placeholder", v.decode())
        if f == 10:
            return ("func", v)
    return []


def decode_node(buf: bytes) -> Node:
    n = Node(name="", op="")
    for f, _, v in _proto_fields(buf):
        if f == 1:
            n.name = v.decode()
        elif f == 2:
            n.op = v.decode()
        elif f == 3:
            n.inputs.append(v.decode())
        elif f == 4:
            n.device = v.decode()
        elif f == 5:
            key, val = "", b""
            for f2, _, v2 in _proto_fields(v):
                if f2 == 1:
                    key = v2.decode()
                elif f2 == 2:
                    val = v2
            n.attr[key] = decode_attr(val)
    return n


def decode_graph(buf: bytes) -> Graph:
    nodes, producer, min_consumer = [], 0, 0
    for f, _, v in _proto_fields(buf):
        if f == 1:
            nodes.append(decode_node(v))
        elif f == 4:
            for f2, _, v2 in _proto_fields(v):
                if f2 == 1:
                    producer = v2
                elif f2 == 2:
                    min_consumer = v2
    return Graph(nodes, producer, min_consumer)


def read_graph(path: str) -> Graph:
    with open(path, "rb") as fh:
        return decode_graph(fh.read())


def read_meta_graph(path: str) -> Graph:
    """The GraphDef inside a MetaGraphDef (`.meta`, field 2)."""
    with open(path, "rb") as fh:
        buf = fh.read()
    for f, _, v in _proto_fields(buf):
        if f == 2:
            return decode_graph(v)
    raise ValueError(f"{path}: no graph_def in MetaGraphDef")


# ------------------------------------------------------------------ encoding
def _tag(out: bytearray, fnum: int, wt: int) -> None:
    put_varint(out, (fnum << 3) | wt)


def _bytes_field(out: bytearray, fnum: int, data: bytes) -> None:
    _tag(out, fnum, 2)
    put_varint(out, len(data))
    out += data


def _varint_field(out: bytearray, fnum: int, v: int) -> None:
    _tag(out, fnum, 0)
    put_varint(out, v & ((1 << 64) - 1))


def encode_shape(dims) -> bytes:
    out = bytearray()
    if dims is None:
        _varint_field(out, 3, 1)
        return bytes(out)
    for d in dims:
        dim = bytearray()
        if d:
            _varint_field(dim, 1, int(d))
        _bytes_field(out, 2, bytes(dim))
    return bytes(out)


def encode_tensor(arr: np.ndarray) -> bytes:
    arr = np.asarray(arr)
    dt = _NP_DT.get(arr.dtype)
    if dt is None:
        raise ValueError(f"unsupported dtype {arr.dtype}")
    out = bytearray()
    _varint_field(out, 1, dt)
    _bytes_field(out, 2, encode_shape(arr.shape))
    if arr.ndim == 0 and dt in (DT_INT32, DT_INT64, DT_BOOL):
        _varint_field(out, {DT_INT32: 7, DT_INT64: 10, DT_BOOL: 11}[dt], int(arr))
    elif arr.ndim == 0 and dt == DT_FLOAT:
        _tag(out, 5, 2)
        put_varint(out, 4)
        out += struct.pack("<f", float(arr))
    else:
        _bytes_field(out, 4, np.ascontiguousarray(arr).astype(arr.dtype.newbyteorder("<")).tobytes())
    return bytes(out)


def encode_attr(v) -> bytes:
    out = bytearray()
    if isinstance(v, bool):
        _varint_field(out, 5, int(v))
    elif isinstance(v, int):
        _varint_field(out, 3, v)
    elif isinstance(v, float):
        _tag(out, 4, 5)
        out += struct.pack("<f", v)
    elif isinstance(v, bytes):
        _bytes_field(out, 2, v)
    elif isinstance(v, str):
        _bytes_field(out, 2, v.encode())
    elif isinstance(v, tuple) and v and v[0] == "type":
        _varint_field(out, 6, v[1])
    elif isinstance(v, Shape):
        _bytes_field(out, 7, encode_shape(v.dims))
    elif isinstance(v, np.ndarray):
        _bytes_field(out, 8, encode_tensor(v))
    elif isinstance(v, list):
        lst = bytearray()
        if v and isinstance(v[0], int) and not isinstance(v[0], bool):
            packed = bytearray()
            for x in v:
                put_varint(packed, x & ((1 << 64) - 1))
            _bytes_field(lst, 3, bytes(packed))
        elif v and isinstance(v[0], (bytes, str)):
            for x in v:
                _bytes_field(lst, 2, x.encode() if isinstance(x, str) else x)
        elif v and isinstance(v[0], tuple) and v[0][0] == "type":
            packed = bytearray()
            for x in v:
                put_varint(packed, x[1])
            _bytes_field(lst, 6, bytes(packed))
        elif v and isinstance(v[0], Shape):
            for x in v:
                _bytes_field(lst, 7, encode_shape(x.dims))
        _bytes_field(out, 1, bytes(lst))
    else:
        raise TypeError(f"cannot encode attr value {v!r}")
    return bytes(out)


def encode_node(n: Node) -> bytes:
    out = bytearray()
    _bytes_field(out, 1, n.name.encode())
    _bytes_field(out, 2, n.op.encode())
    for i in n.inputs:
        _bytes_field(out, 3, i.encode())
    if n.device:
        _bytes_field(out, 4, n.device.encode())
    for k in sorted(n.attr):   # TF serializes maps in key order
        entry = bytearray()
        _bytes_field(entry, 1, k.encode())
        _bytes_field(entry, 2, encode_attr(n.attr[k]))
        _bytes_field(out, 5, bytes(entry))
    return bytes(out)


def encode_graph(g: Graph) -> bytes:
    out = bytearray()
    for n in g.nodes:
        _bytes_field(out, 1, encode_node(n))
    ver = bytearray()
    if g.producer:
        _varint_field(ver, 1, g.producer)
    if g.min_consumer:
        _varint_field(ver, 2, g.min_consumer)
    _bytes_field(out, 4, bytes(ver))
    return bytes(out)


def encode_meta_graph(g: Graph, variables, tf_version: str = "1.12.0") -> bytes:
    """MetaGraphDef (the `.meta` of tf.train.export_meta_graph): field 1
    MetaInfoDef {meta_graph_version, tensorflow_version}, field 2 the GraphDef,
    field 4 the collections "variables" / "trainable_variables" as serialized
    VariableDef {variable_name "<v>:0", initializer_name "<v>/Assign", snapshot_name
    "<v>/read:0", initial_value_name "<init>:0", trainable} (bytes_list).
    ``variables``: [(name, trainable[, initializer_name, initial_value_name])] in
    creation order."""
    out = bytearray()
    info = bytearray()
    _bytes_field(info, 1, f"v{tf_version}".encode())
    _bytes_field(info, 5, tf_version.encode())
    _bytes_field(out, 1, bytes(info))
    _bytes_field(out, 2, encode_graph(g))
    for key, keep in (("trainable_variables", lambda t: t), ("variables", lambda t: True)):
        blist = bytearray()
        for v in variables:
            name, trainable = v[0], v[1]
            if not keep(trainable):
                continue
            vdef = bytearray()
            _bytes_field(vdef, 1, f"{name}:0".encode())
            if len(v) > 2:
                _bytes_field(vdef, 2, v[2].encode())
            _bytes_field(vdef, 3, f"{name}/read:0".encode())
            if len(v) > 3:
                _bytes_field(vdef, 6, v[3].encode())
            if trainable:
                _varint_field(vdef, 7, 1)
            _bytes_field(blist, 1, bytes(vdef))
        coll = bytearray()
        _bytes_field(coll, 2, bytes(blist))       # CollectionDef.bytes_list
        entry = bytearray()
        _bytes_field(entry, 1, key.encode())
        _bytes_field(entry, 2, bytes(coll))
        _bytes_field(out, 4, bytes(entry))
    return bytes(out)


def read_meta_info(path: str) -> dict:
    """{"tensorflow_version", "collections": {key: [variable names]}} of a `.meta`."""
    with open(path, "rb") as fh:
        buf = fh.read()
    info = {"tensorflow_version": None, "collections": {}}
    for f, _, v in _proto_fields(buf):
        if f == 1:
            for f2, _, v2 in _proto_fields(v):
                if f2 == 5:
                    info["tensorflow_version"] = v2.decode()
        elif f == 4:
            key, names = None, []
            for f2, _, v2 in _proto_fields(v):
                if f2 == 1:
                    key = v2.decode()
                elif f2 == 2:
                    for f3, _, v3 in _proto_fields(v2):
                        if f3 == 2:                   # bytes_list
                            for f4, _, v4 in _proto_fields(v3):
                                if f4 == 1:           # one VariableDef
                                    for f5, _, v5 in _proto_fields(v4):
                                        if f5 == 1:
                                            names.append(v5.decode().rsplit(":", 1)[0])
            info["collections"][key] = names
    return info


def read_variable_defs(path: str) -> dict:
    """{collection: [{field number: value}]} of the VariableDefs in a `.meta`."""
    with open(path, "rb") as fh:
        buf = fh.read()
    out = {}
    for f, _, v in _proto_fields(buf):
        if f != 4:
            continue
        key, defs = None, []
        for f2, _, v2 in _proto_fields(v):
            if f2 == 1:
                key = v2.decode()
            elif f2 == 2:
                for f3, _, v3 in _proto_fields(v2):
                    if f3 == 2:
                        for f4, _, v4 in _proto_fields(v3):
                            if f4 == 1:
                                defs.append({f5: (v5 if isinstance(v5, int) else v5.decode())
                                             for f5, _, v5 in _proto_fields(v4)})
        out[key] = defs
    return out


def write_graph(g: Graph, path: str) -> None:
    import os

    tmp = path + ".tmp"
    with open(tmp, "wb") as fh:
        fh.write(encode_graph(g))
    os.replace(tmp, path)
