"""Frozen inference graphs (reference resnet_cifar_frozen_model.py:81-122,
resnet_cifar_predict_from_pd.py:66-105).

The reference rebuilds its eval graph with placeholders ``X[None,H,W,3]`` and
``Y[None,classes]``, adds ``truth`` / ``predictions`` (argmax) and ``precision``
(mean of equal), and runs TF's freeze_graph so every variable becomes a Const.

`export_graphdef` writes that same GraphDef without TensorFlow: it walks the
ModelSpec in TF's op-creation order (resnet_model_official.py:94-366,
resnet_model.py:69-88) and emits the nodes TF emits -- names (``conv2d_18/
Conv2D``, ``Pad_1``, ``add_7``, ``block_layer1``, ``Relu_16``...), inputs,
attributes (NHWC, SAME/VALID, fused-BN epsilon 1.001e-5, ``_output_shapes``)
and the frozen ``<var>`` Const + ``<var>/read`` Identity pairs.  For CIFAR
ResNet-50 the node list equals the reference's own
``resnet50_cifar_frozen_model_eval.pb`` node for node
(tests/test_graphdef_cpu.py), so a TF consumer can load what we write and we
can load what TF wrote.

`read_frozen` decodes any such GraphDef (data only, utils/graphdef.py), infers
the architecture from its Const set and returns the TF-named tensors that
`FrozenModel` loads into the GPU inference plan or the CPU model.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from ..models.spec import IMAGENET_SIZES, ModelSpec, build_spec, imagenet_spec
from . import graphdef as gd
from . import tensor_bundle as tb

TF_BN_EPS = float(np.float32(1.001e-5))   # what tf.layers' fused BN records
_F = ("type", gd.DT_FLOAT)
_I32 = ("type", gd.DT_INT32)
_I64 = ("type", gd.DT_INT64)


class _GraphBuilder:
    def __init__(self, tensors: dict):
        self.nodes: list = []
        self.tensors = tensors
        self.counts: dict = {}

    def uniq(self, base: str) -> str:
        n = self.counts.get(base, 0)
        self.counts[base] = n + 1
        return base if n == 0 else f"{base}_{n}"

    def add(self, name, op, inputs=(), **attr) -> str:
        self.nodes.append(gd.Node(name, op, list(inputs), "", attr))
        return name

    def var(self, name: str) -> str:
        """A frozen variable: Const + the `/read` Identity tf.get_variable made."""
        v = np.ascontiguousarray(np.asarray(self.tensors[name], dtype=np.float32))
        self.add(name, "Const", dtype=_F, value=v)
        return self.add(f"{name}/read", "Identity", [name], T=_F,
                        _class=[f"loc:@{name}".encode()],
                        _output_shapes=[gd.Shape(list(v.shape))])

    def const_i32(self, name, value, shape) -> str:
        return self.add(name, "Const", dtype=_I32, value=np.asarray(value, dtype=np.int32),
                        _output_shapes=[gd.Shape(list(shape))])


def _shp(h, w, c):
    return [gd.Shape([-1, h, w, c])]


def export_graphdef(spec: ModelSpec, tensors: dict) -> gd.Graph:
    """The reference's frozen eval GraphDef for `spec` with `tensors` (TF names)."""
    b = _GraphBuilder(tensors)
    H, W = spec.image_h, spec.image_w
    b.add("X", "Placeholder", dtype=_F, shape=gd.Shape([-1, H, W, 3]), _output_shapes=_shp(H, W, 3))
    b.add("Y", "Placeholder", dtype=_F, shape=gd.Shape([-1, spec.num_classes]),
          _output_shapes=[gd.Shape([-1, spec.num_classes])])

    def conv(x, c, h, w):
        """conv2d_fixed_padding (official:80-91): explicit Pad + VALID for stride > 1."""
        ho, wo = c.ho, c.wo
        if c.stride > 1:
            beg = (c.kh - 1) // 2
            end = c.kh - 1 - beg
            pn = b.uniq("Pad")
            pads = b.const_i32(f"{pn}/paddings", [[0, 0], [beg, end], [beg, end], [0, 0]], [4, 2])
            x = b.add(pn, "Pad", [x, pads], T=_F, Tpaddings=_I32,
                      _output_shapes=_shp(h + c.kh - 1, w + c.kw - 1, c.cin))
        k = b.var(f"{c.name}/kernel")
        return b.add(f"{c.name}/Conv2D", "Conv2D", [x, k], T=_F, data_format=b"NHWC",
                     strides=[1, c.stride, c.stride, 1], dilations=[1, 1, 1, 1],
                     padding=b"SAME" if c.stride == 1 else b"VALID", use_cudnn_on_gpu=True,
                     _output_shapes=_shp(ho, wo, c.cout))

    def bn_relu(x, bn):
        ins = [x] + [b.var(f"{bn.name}/{p}") for p in ("gamma", "beta", "moving_mean",
                                                       "moving_variance")]
        c = bn.channels
        y = b.add(f"{bn.name}/FusedBatchNorm", "FusedBatchNorm", ins, T=_F, data_format=b"NHWC",
                  epsilon=TF_BN_EPS, is_training=False,
                  _output_shapes=_shp(bn.h, bn.w, c) + [gd.Shape([c])] * 4)
        return b.add(b.uniq("Relu"), "Relu", [y], T=_F, _output_shapes=_shp(bn.h, bn.w, c))

    x = conv("X", spec.stem, H, W)
    h, w = spec.stem.ho, spec.stem.wo
    x = b.add("initial_conv", "Identity", [x], T=_F, _output_shapes=_shp(h, w, spec.stem.cout))
    if spec.maxpool:
        h, w = -(-h // 2), -(-w // 2)
        x = b.add("max_pooling2d/MaxPool", "MaxPool", [x], T=_F, data_format=b"NHWC",
                  ksize=[1, 3, 3, 1], strides=[1, 2, 2, 1], padding=b"SAME",
                  _output_shapes=_shp(h, w, spec.stem.cout))
        x = b.add("initial_max_pool", "Identity", [x], T=_F,
                  _output_shapes=_shp(h, w, spec.stem.cout))
    layer = 0
    for i, blk in enumerate(spec.blocks):
        shortcut = x
        a = bn_relu(x, blk.bns[0])
        if blk.proj is not None:
            shortcut = conv(a, blk.proj, blk.h, blk.w)
        hh = a
        for j, c in enumerate(blk.convs):
            if j > 0:
                hh = bn_relu(hh, blk.bns[j])
            hh = conv(hh, c, c.h, c.w)
        x = b.add(b.uniq("add"), "Add", [hh, shortcut], T=_F,
                  _output_shapes=_shp(blk.ho, blk.wo, blk.cout))
        last_of_layer = i + 1 == len(spec.blocks) or spec.blocks[i + 1].proj is not None
        if last_of_layer:
            layer += 1
            x = b.add(f"block_layer{layer}", "Identity", [x], T=_F,
                      _output_shapes=_shp(blk.ho, blk.wo, blk.cout))
    fb = spec.final_bn
    x = bn_relu(x, fb)
    x = b.add("average_pooling2d/AvgPool", "AvgPool", [x], T=_F, data_format=b"NHWC",
              ksize=[1, fb.h, fb.w, 1], strides=[1, 1, 1, 1], padding=b"VALID",
              _output_shapes=_shp(1, 1, fb.channels))
    x = b.add("final_avg_pool", "Identity", [x], T=_F, _output_shapes=_shp(1, 1, fb.channels))
    rs = b.const_i32("Reshape/shape", [-1, spec.dense_in], [2])
    x = b.add("Reshape", "Reshape", [x, rs], T=_F, Tshape=_I32,
              _output_shapes=[gd.Shape([-1, spec.dense_in])])
    nc = [gd.Shape([-1, spec.num_classes])]
    k = b.var("dense/kernel")          # Dense.build creates kernel and bias first
    bias = b.var("dense/bias")
    x = b.add("dense/MatMul", "MatMul", [x, k], T=_F, transpose_a=False, transpose_b=False,
              _output_shapes=nc)
    x = b.add("dense/BiasAdd", "BiasAdd", [x, bias], T=_F, data_format=b"NHWC", _output_shapes=nc)
    x = b.add("final_dense", "Identity", [x], T=_F, _output_shapes=nc)
    sm = b.add("Softmax", "Softmax", [x], T=_F, _output_shapes=nc)       # resnet_model.py:77
    vec = [gd.Shape([-1])]
    td = b.const_i32("truth/dimension", 1, [])
    b.add("truth", "ArgMax", ["Y", td], T=_F, Tidx=_I32, output_type=_I64, _output_shapes=vec)
    pd_ = b.const_i32("predictions/dimension", 1, [])
    b.add("predictions", "ArgMax", [sm, pd_], T=_F, Tidx=_I32, output_type=_I64,
          _output_shapes=vec)
    b.add("Equal", "Equal", ["predictions", "truth"], T=_I64, _output_shapes=vec)
    b.add("ToFloat", "Cast", ["Equal"], SrcT=("type", gd.DT_BOOL), DstT=_F, Truncate=False,
          _output_shapes=vec)
    c0 = b.const_i32("Const", [0], [1])
    b.add("precision", "Mean", ["ToFloat", c0], T=_F, Tidx=_I32, keep_dims=False,
          _output_shapes=[gd.Shape([])])
    return gd.Graph(b.nodes, producer=27)


# ---------------------------------------------------------------- import
def _candidate_specs(dataset: str, num_classes: int):
    if dataset == "imagenet":
        for size in sorted(IMAGENET_SIZES):
            yield imagenet_spec(size, num_classes)
    else:
        for size in range(8, 1203, 6):
            yield build_spec(dataset, size, num_classes)


def spec_from_graph(graph: gd.Graph) -> ModelSpec:
    """Architecture of a frozen ResNet v2 GraphDef, from its input shape and Const set."""
    nodes = graph.by_name()
    dims = nodes["X"].attr["shape"].dims
    consts = {n.name: tuple(n.attr["value"].shape) for n in graph.nodes if n.op == "Const"}
    num_classes = consts["dense/bias"][0]
    dataset = "imagenet" if dims[1] >= 64 else ("cifar100" if num_classes == 100 else "cifar10")
    n_convs = sum(1 for k in consts if k.endswith("/kernel") and k.startswith("conv2d"))
    for spec in _candidate_specs(dataset, num_classes):
        if len(spec.all_convs()) != n_convs:
            continue
        if all(consts.get(p.name) == tuple(p.shape) for p in spec.params):
            return spec
    raise ValueError(f"no ResNet v2 spec matches this graph ({n_convs} convs, {dataset})")


def read_frozen(path: str):
    """-> (meta, {TF name: fp32 array}) of a frozen GraphDef (ours or TF's)."""
    graph = gd.read_graph(path)
    spec = spec_from_graph(graph)
    consts = {n.name: n.attr["value"] for n in graph.nodes if n.op == "Const"}
    tensors = {p.name: np.asarray(consts[p.name], dtype=np.float32) for p in spec.params}
    meta = {"dataset": spec.dataset, "resnet_size": spec.resnet_size,
            "num_classes": spec.num_classes, "input": [None, spec.image_h, spec.image_w, 3],
            "outputs": ["predictions", "precision"], "nodes": len(graph.nodes)}
    return meta, tensors


def _initializer_nodes(p, dims: list) -> tuple[list, str]:
    """The initializer subgraph TF 1.12 builds in front of a variable (op names as in
    the reference's resnet50_cifar_eval_graph.meta): conv kernels variance-scaling
    truncated normal (resnet_model_official.py:90), the dense kernel glorot uniform,
    gamma / moving_variance ones, the rest zeros.  Returns (nodes, output name)."""
    f32, i32 = ("type", 1), ("type", 3)
    base = f"{p.name}/Initializer"
    shape = np.asarray(dims, dtype=np.int32)
    if p.kind == "conv":
        r = f"{base}/truncated_normal"
        fan_in = int(np.prod(dims[:-1]))
        std = np.asarray(np.sqrt(1.0 / fan_in) / 0.87962566103423978, np.float32)
        return [gd.Node(f"{r}/shape", "Const", [], "", {"dtype": i32, "value": shape}),
                gd.Node(f"{r}/mean", "Const", [], "", {"dtype": f32, "value": np.asarray(0.0, np.float32)}),
                gd.Node(f"{r}/stddev", "Const", [], "", {"dtype": f32, "value": std}),
                gd.Node(f"{r}/TruncatedNormal", "TruncatedNormal", [f"{r}/shape"], "",
                        {"T": i32, "dtype": f32, "seed": 0, "seed2": 0}),
                gd.Node(f"{r}/mul", "Mul", [f"{r}/TruncatedNormal", f"{r}/stddev"], "", {"T": f32}),
                gd.Node(r, "Add", [f"{r}/mul", f"{r}/mean"], "", {"T": f32})], r
    if p.kind == "dense_kernel":
        r = f"{base}/random_uniform"
        lim = np.asarray(np.sqrt(6.0 / (dims[0] + dims[1])), np.float32)
        return [gd.Node(f"{r}/shape", "Const", [], "", {"dtype": i32, "value": shape}),
                gd.Node(f"{r}/min", "Const", [], "", {"dtype": f32, "value": np.asarray(-lim, np.float32)}),
                gd.Node(f"{r}/max", "Const", [], "", {"dtype": f32, "value": lim}),
                gd.Node(f"{r}/RandomUniform", "RandomUniform", [f"{r}/shape"], "",
                        {"T": i32, "dtype": f32, "seed": 0, "seed2": 0}),
                gd.Node(f"{r}/sub", "Sub", [f"{r}/max", f"{r}/min"], "", {"T": f32}),
                gd.Node(f"{r}/mul", "Mul", [f"{r}/RandomUniform", f"{r}/sub"], "", {"T": f32}),
                gd.Node(r, "Add", [f"{r}/mul", f"{r}/min"], "", {"T": f32})], r
    ones = p.kind in ("gamma", "moving_variance")
    r = f"{base}/{'ones' if ones else 'zeros'}"
    return [gd.Node(r, "Const", [], "", {"dtype": f32,
                                         "value": np.full(dims, 1.0 if ones else 0.0,
                                                          dtype=np.float32)})], r


def export_eval_meta_graph(spec: ModelSpec, tensors: dict) -> bytes:
    """The eval graph BEFORE freezing, as a MetaGraphDef (reference
    resnet_cifar_frozen_model.py:91-96, export_meta_graph ->
    resnet50_cifar_eval_graph.meta): the frozen GraphDef's weight Consts are
    VariableV2 nodes again (same names, dtypes and shapes, no values -- those
    live in the checkpoint), each behind its initializer subgraph and followed by
    its `<v>/Assign`, plus `global_step`, and the variables / trainable_variables
    collections whose VariableDefs name the initializer op and initial value
    (so tf.train.import_meta_graph / freeze_graph can rebuild the Variables).
    The other node names are exactly the `.pb`'s."""
    graph = export_graphdef(spec, tensors)
    params = {p.name: p for p in spec.params}
    nodes = []
    inits = {}
    for n in graph.nodes:
        if n.op == "Const" and n.name in params:
            dims = list(np.asarray(n.attr["value"]).shape)
            init_nodes, init = _initializer_nodes(params[n.name], dims)
            nodes += init_nodes
            n = gd.Node(n.name, "VariableV2", [], n.device,
                        {"container": b"", "dtype": ("type", 1), "shape": gd.Shape(dims),
                         "shared_name": b"", "_output_shapes": [gd.Shape(dims)]})
            nodes.append(n)
            nodes.append(gd.Node(f"{n.name}/Assign", "Assign", [n.name, init], "",
                                 {"T": ("type", 1), "use_locking": True,
                                  "validate_shape": True}))
            inits[n.name] = (f"{n.name}/Assign", f"{init}:0")
            continue
        nodes.append(n)
    gs = [gd.Node("global_step/Initializer/zeros", "Const", [], "",
                  {"dtype": ("type", 9), "value": np.asarray(0, np.int64)}),
          gd.Node("global_step", "VariableV2", [], "",
                  {"container": b"", "dtype": ("type", 9), "shape": gd.Shape([]),
                   "shared_name": b"", "_output_shapes": [gd.Shape([])]}),
          gd.Node("global_step/Assign", "Assign", ["global_step", "global_step/Initializer/zeros"],
                  "", {"T": ("type", 9), "use_locking": True, "validate_shape": True})]
    nodes = gs + nodes
    inits["global_step"] = ("global_step/Assign", "global_step/Initializer/zeros:0")
    trainable = {p.name for p in spec.trainables}
    variables = [("global_step", False) + inits["global_step"]] + \
        [(p.name, p.name in trainable) + inits[p.name] for p in spec.params]
    return gd.encode_meta_graph(gd.Graph(nodes, graph.producer, graph.min_consumer), variables)


def freeze(prefix: str, out_path: str, dataset: str, resnet_size: int,
           num_classes: int | None = None, meta_path: str | None = "") -> dict:
    """Checkpoint (tensor bundle) -> frozen eval GraphDef `.pb` (freeze_graph
    equivalent), and the unfrozen eval graph's MetaGraphDef next to it
    (``meta_path``; "" = <dir>/resnet<size>_<cifar|imagenet>_eval_graph.meta,
    None = skip)."""
    spec = build_spec(dataset, resnet_size, num_classes)
    tensors = tb.read_bundle(prefix)
    missing = [p.name for p in spec.params if p.name not in tensors]
    if missing:
        raise KeyError(f"{missing[:3]}... missing from {prefix}")
    graph = export_graphdef(spec, tensors)
    gd.write_graph(graph, out_path)
    if meta_path == "":
        kind = "cifar" if spec.dataset.startswith("cifar") else "imagenet"
        meta_path = os.path.join(os.path.dirname(os.path.abspath(out_path)),
                                 f"resnet{resnet_size}_{kind}_eval_graph.meta")
    if meta_path and os.path.exists(meta_path):
        # like the reference (resnet_cifar_frozen_model.py:92): an existing eval meta
        # graph -- possibly TF's own -- is kept, never overwritten
        pass
    elif meta_path:
        tmp = meta_path + ".tmp"
        with open(tmp, "wb") as fh:
            fh.write(export_eval_meta_graph(spec, tensors))
        os.replace(tmp, meta_path)
    return {"dataset": spec.dataset, "resnet_size": resnet_size, "num_classes": spec.num_classes,
            "nodes": len(graph.nodes), "outputs": ["predictions", "precision"],
            "global_step": int(tensors.get("global_step", 0)), "meta_graph": meta_path}


class FrozenModel:
    """predict(images, labels) -> (class probabilities, precision) from a frozen `.pb`.

    device "gpu"/"cpu"/"auto": the weights run on our GPU inference plan or the
    fp32 CPU model; device "interp": the GraphDef itself through the CPU graph
    interpreter (utils/tf_interp.py), TF's semantics op by op."""

    def __init__(self, path: str, device: str = "auto", batch_size: int = 100):
        self.meta, self.tensors = read_frozen(path)
        self.spec = build_spec(self.meta["dataset"], self.meta["resnet_size"],
                               self.meta["num_classes"])
        self.batch_size = batch_size
        self.device = device
        if device == "interp":
            from .tf_interp import Interpreter

            self.interp = Interpreter(gd.read_graph(path))
            self.model = None
        else:
            from ..train.evaluator import make_inference

            self.model = make_inference(self.spec, batch_size, device)
            self.model.load(self.tensors)

    def predict(self, images, labels=None):
        n = images.shape[0]
        if n != self.batch_size:
            raise ValueError(f"frozen model was loaded for batch {self.batch_size}, got {n}")
        if labels is None:
            labels = torch.zeros(n, dtype=torch.int64)
        if self.model is None:
            from ..data.cifar import augment_cpu

            # uint8 [N,3,H,W] records -> standardized NHWC, as the reference's numpy
            # preprocessing before its feed_dict (resnet_cifar_predict_from_pd.py:86-99)
            x = augment_cpu(images, train=False) if images.dtype == torch.uint8 else images
            y = torch.nn.functional.one_hot(labels.long(), self.spec.num_classes).float()
            probs, prec = self.interp.run(["Softmax", "precision"], {"X": x, "Y": y})
            return probs.float(), float(prec)
        loss, correct, probs = self.model.run(images, labels)
        return probs.detach().float().cpu(), correct / n
