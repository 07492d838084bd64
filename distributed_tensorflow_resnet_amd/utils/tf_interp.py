"""A small CPU interpreter for TensorFlow inference GraphDefs (data-only).

Runs the node set of the reference's frozen CIFAR ResNet-50
(`resnet_cifar_frozen_model.py:111-122` -> `resnet50_cifar_frozen_model_eval.pb`:
Placeholder, Const, Identity, Conv2D, Pad, FusedBatchNorm, Relu, Add, AvgPool,
MaxPool, Reshape, MatMul, BiasAdd, Softmax, ArgMax, Equal, Cast, Mean) with the
TF op semantics written out independently of our model code, so it serves as
a golden forward pass for the network we build from models/spec.py:

  * Conv2D SAME: pad_total = max((ceil(H/s)-1)*s + k - H, 0), pad_top =
    pad_total // 2 (the extra row/column goes bottom/right), NHWC x HWIO;
  * FusedBatchNorm (is_training=False): (x - mean) * rsqrt(var + eps) * gamma
    + beta with the node's own epsilon attribute;
  * AvgPool / MaxPool VALID|SAME windows (SAME max-pool pads with -inf);
  * ArgMax ties resolve to the first index (as TF).

Arithmetic is float64 by default (`dtype=torch.float64`) so the interpreter is
an oracle for fp32 code.  Nothing in the file is executed: only the ops listed
above are understood and anything else raises.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

from .graphdef import DT_BOOL, DT_FLOAT, DT_INT32, DT_INT64, Graph


def _same_pads(size: int, k: int, s: int) -> tuple[int, int]:
    out = math.ceil(size / s)
    total = max((out - 1) * s + k - size, 0)
    return total // 2, total - total // 2


def _s(v) -> str:
    return v.decode() if isinstance(v, bytes) else str(v)


def _np_type(t):
    return {DT_FLOAT: torch.float32, DT_INT32: torch.int32, DT_INT64: torch.int64,
            DT_BOOL: torch.bool}[t[1]]


class Interpreter:
    def __init__(self, graph: Graph, dtype=torch.float64):
        self.graph = graph
        self.nodes = graph.by_name()
        self.dtype = dtype

    def consts(self) -> dict[str, np.ndarray]:
        """Const-node tensors by node name (the frozen variables and shape operands)."""
        return {n.name: n.attr["value"] for n in self.graph.nodes if n.op == "Const"}

    def run(self, fetches, feeds: dict):
        single = isinstance(fetches, str)
        names = [fetches] if single else list(fetches)
        cache: dict = {}
        for k, v in feeds.items():
            t = torch.as_tensor(np.asarray(v))
            cache[k] = t.to(self.dtype) if t.is_floating_point() else t
        out = [self._eval(n, cache) for n in names]
        return out[0] if single else out

    # ----------------------------------------------------------------- eval
    def _input(self, ref: str, cache):
        name, _, idx = ref.partition(":")
        if name.startswith("^"):
            return None
        v = self._eval(name, cache)
        if isinstance(v, tuple):
            return v[int(idx or 0)]
        return v

    def _eval(self, name: str, cache):
        if name in cache:
            return cache[name]
        # iterative DFS so 700-node chains do not hit the recursion limit
        stack = [name]
        while stack:
            cur = stack[-1]
            if cur in cache:
                stack.pop()
                continue
            node = self.nodes[cur]
            pending = [i.partition(":")[0] for i in node.inputs
                       if not i.startswith("^") and i.partition(":")[0] not in cache]
            if pending:
                stack.extend(pending)
                continue
            args = [self._input(i, cache) for i in node.inputs if not i.startswith("^")]
            cache[cur] = self._op(node, args)
            stack.pop()
        return cache[name]

    def _op(self, node, a):
        op, at = node.op, node.attr
        dt = self.dtype
        if op == "Placeholder":
            raise KeyError(f"placeholder {node.name!r} was not fed")
        if op == "Const":
            v = torch.as_tensor(np.array(at["value"]))
            return v.to(dt) if v.is_floating_point() else v
        if op in ("Identity", "StopGradient"):
            return a[0]
        if op == "Conv2D":
            if _s(at.get("data_format", b"NHWC")) != "NHWC":
                raise NotImplementedError("Conv2D NCHW")
            x, w = a
            sh, sw = at["strides"][1], at["strides"][2]
            if list(at.get("dilations", [1, 1, 1, 1])) != [1, 1, 1, 1]:
                raise NotImplementedError("dilated Conv2D")
            kh, kw = w.shape[0], w.shape[1]
            if _s(at["padding"]) == "SAME":
                pt, pb = _same_pads(x.shape[1], kh, sh)
                pl, pr = _same_pads(x.shape[2], kw, sw)
                x = F.pad(x, (0, 0, pl, pr, pt, pb))
            xc = x.permute(0, 3, 1, 2)
            wc = w.permute(3, 2, 0, 1)
            return F.conv2d(xc, wc, stride=(sh, sw)).permute(0, 2, 3, 1)
        if op in ("Pad", "PadV2"):
            x, p = a
            p = p.tolist()
            flat = []
            for lo, hi in reversed(p):
                flat += [int(lo), int(hi)]
            return F.pad(x, flat, value=float(a[2]) if len(a) > 2 else 0.0)
        if op in ("FusedBatchNorm", "FusedBatchNormV3"):
            if at.get("is_training", True):
                raise NotImplementedError("training-mode FusedBatchNorm")
            x, g, b, m, v = a[:5]
            eps = float(at.get("epsilon", 1e-4))
            y = (x - m) * torch.rsqrt(v + eps) * g + b
            return (y, m, v, m, v)
        if op == "Relu":
            return torch.relu(a[0])
        if op in ("Add", "AddV2"):
            return a[0] + a[1]
        if op in ("AvgPool", "MaxPool"):
            x = a[0]
            _, kh, kw, _ = at["ksize"]
            _, sh, sw, _ = at["strides"]
            pad = _s(at["padding"])
            xc = x.permute(0, 3, 1, 2)
            if pad == "SAME":
                pt, pb = _same_pads(x.shape[1], kh, sh)
                pl, pr = _same_pads(x.shape[2], kw, sw)
                if op == "MaxPool":
                    xc = F.pad(xc, (pl, pr, pt, pb), value=-math.inf)
                    return F.max_pool2d(xc, (kh, kw), (sh, sw)).permute(0, 2, 3, 1)
                # TF SAME avg-pool divides by the count of valid taps
                ones = torch.ones_like(xc[:, :1])
                s = F.avg_pool2d(F.pad(xc, (pl, pr, pt, pb)), (kh, kw), (sh, sw),
                                 divisor_override=1)
                c = F.avg_pool2d(F.pad(ones, (pl, pr, pt, pb)), (kh, kw), (sh, sw),
                                 divisor_override=1)
                return (s / c).permute(0, 2, 3, 1)
            fn = F.max_pool2d if op == "MaxPool" else F.avg_pool2d
            return fn(xc, (kh, kw), (sh, sw)).permute(0, 2, 3, 1)
        if op == "Reshape":
            return a[0].reshape([int(d) for d in a[1].tolist()])
        if op == "MatMul":
            x, w = a
            if at.get("transpose_a"):
                x = x.t()
            if at.get("transpose_b"):
                w = w.t()
            return x @ w
        if op == "BiasAdd":
            return a[0] + a[1]
        if op == "Softmax":
            return torch.softmax(a[0], dim=-1)
        if op == "ArgMax":
            axis = int(a[1])
            out_t = _np_type(at.get("output_type", ("type", DT_INT64)))
            # first maximal index, like TF (torch.argmax ties are unspecified)
            x = a[0]
            mx = x.max(dim=axis, keepdim=True).values
            idx = torch.arange(x.shape[axis]).reshape([-1 if d == axis % x.dim() else 1
                                                       for d in range(x.dim())])
            cand = torch.where(x == mx, idx, torch.full_like(idx, x.shape[axis]))
            return cand.min(dim=axis).values.to(out_t)
        if op == "Equal":
            return a[0] == a[1]
        if op == "Cast":
            t = at["DstT"]
            return a[0].to(dt if t[1] == DT_FLOAT else _np_type(t))
        if op == "Mean":
            axes = [int(d) for d in np.atleast_1d(a[1].numpy())]
            return a[0].to(dt).mean(dim=axes, keepdim=bool(at.get("keep_dims", False)))
        raise NotImplementedError(f"op {op} ({node.name})")
