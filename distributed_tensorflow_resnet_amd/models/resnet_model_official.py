"""API-compatible re-statement of the reference's `resnet_model_official.py`.

Same public functions and signatures (resnet_model_official.py:37-366):
  batch_norm_relu, fixed_padding, conv2d_fixed_padding, building_block,
  bottleneck_block, block_layer, cifar10_resnet_v2_generator,
  imagenet_resnet_v2_generator, imagenet_resnet_v2
operating on torch tensors, with TF `tf.layers` variable semantics: each layer
call creates its variables on first use under the TF auto-unique names
(`conv2d`, `conv2d_1`, ..., `batch_normalization_N/gamma`, `dense/kernel`) in
creation order, and later calls of the same model function reuse them (like
a graph built once).  `data_format` 'channels_first' (NCHW) and
'channels_last' (NHWC) both work; inputs to the generated model are NHWC
images as in the reference.

This define-by-run path is the CPU/semantic reference; the MI355X training
path (train/engine.py) executes the same architecture from models/spec.py
with hand-written HIP kernels, and both share the TF variable names, so
`model.variables()` can be loaded into the engine and vice versa.
"""
from __future__ import annotations

import math
import threading
from collections import OrderedDict

import torch
import torch.nn.functional as F

_BATCH_NORM_DECAY = 0.997
# The reference passes 1e-5 (resnet_model_official.py:38), but TF's fused batch norm
# raises any epsilon below 1.001e-5 to that value: the reference's own frozen and
# training graphs carry 1.001e-5 in every FusedBatchNorm(Grad) node
# (tests/test_graphdef_cpu.py), so that is the effective value used here too.
_BATCH_NORM_EPSILON = 1.001e-5
_TRUNC = 0.87962566103423978

_tls = threading.local()


class VariableStore:
    """tf.get_variable + layer auto-naming for one model."""

    def __init__(self, seed: int = 0):
        self.vars: "OrderedDict[str, torch.Tensor]" = OrderedDict()
        self.trainable: list[str] = []
        self.counts: dict[str, int] = {}
        self.gen = torch.Generator().manual_seed(seed)

    def reset_names(self):
        self.counts = {}

    def unique(self, base: str) -> str:
        n = self.counts.get(base, 0)
        self.counts[base] = n + 1
        return base if n == 0 else f"{base}_{n}"

    def get(self, name, shape, init, trainable=True) -> torch.Tensor:
        if name in self.vars:
            v = self.vars[name]
            if tuple(v.shape) != tuple(shape):
                raise ValueError(f"variable {name} shape {tuple(v.shape)} != {tuple(shape)}")
            return v
        v = init(shape, self.gen).float()
        v.requires_grad_(trainable)
        self.vars[name] = v
        if trainable:
            self.trainable.append(name)
        return v


def _store() -> VariableStore:
    s = getattr(_tls, "store", None)
    if s is None:
        s = VariableStore()
        _tls.store = s
    return s


class _Scope:
    def __init__(self, store):
        self.store = store

    def __enter__(self):
        self.prev = getattr(_tls, "store", None)
        _tls.store = self.store
        self.store.reset_names()
        return self.store

    def __exit__(self, *a):
        _tls.store = self.prev


def _variance_scaling(shape, g):
    kh, kw, cin, _ = shape
    std = math.sqrt(1.0 / (kh * kw * cin)) / _TRUNC
    out = torch.randn(shape, generator=g)
    bad = out.abs() > 2
    while bool(bad.any()):
        out[bad] = torch.randn(int(bad.sum()), generator=g)
        bad = out.abs() > 2
    return out * std


def _glorot_uniform(shape, g):
    lim = math.sqrt(6.0 / (shape[0] + shape[1]))
    return torch.rand(shape, generator=g) * 2 * lim - lim


def _const(v):
    return lambda shape, g: torch.full(shape, float(v))


def _channels_axis(data_format):
    return 1 if data_format == "channels_first" else 3


def batch_norm_relu(inputs, is_training, data_format):
    """tf.layers.batch_normalization(fused, momentum 0.997, eps 1e-5 -> TF's effective
    1.001e-5) + ReLU."""
    st = _store()
    name = st.unique("batch_normalization")
    ax = _channels_axis(data_format)
    C = inputs.shape[ax]
    gamma = st.get(f"{name}/gamma", (C,), _const(1.0))
    beta = st.get(f"{name}/beta", (C,), _const(0.0))
    mm = st.get(f"{name}/moving_mean", (C,), _const(0.0), trainable=False)
    mv = st.get(f"{name}/moving_variance", (C,), _const(1.0), trainable=False)
    shape = [1, 1, 1, 1]
    shape[ax] = C
    dims = tuple(d for d in range(4) if d != ax)
    if is_training:
        mean = inputs.mean(dim=dims)
        var = inputs.var(dim=dims, unbiased=False)
        n = inputs.numel() // C
        with torch.no_grad():  # UPDATE_OPS: AssignSub with decay, Bessel-corrected variance
            mm.sub_((1 - _BATCH_NORM_DECAY) * (mm - mean.detach()))
            mv.sub_((1 - _BATCH_NORM_DECAY) * (mv - var.detach() * n / max(n - 1, 1)))
    else:
        mean, var = mm, mv
    y = (inputs - mean.view(shape)) * torch.rsqrt(var.view(shape) + _BATCH_NORM_EPSILON)
    y = y * gamma.view(shape) + beta.view(shape)
    return torch.relu(y)


def fixed_padding(inputs, kernel_size, data_format):
    """Pad H/W by (k-1)//2 before and the rest after, independent of input size."""
    pad_total = kernel_size - 1
    pad_beg = pad_total // 2
    pad_end = pad_total - pad_beg
    if data_format == "channels_first":
        return F.pad(inputs, (pad_beg, pad_end, pad_beg, pad_end))
    return F.pad(inputs, (0, 0, pad_beg, pad_end, pad_beg, pad_end))


def conv2d_fixed_padding(inputs, filters, kernel_size, strides, data_format):
    """Strided 2-D convolution with explicit padding (SAME for stride 1), no bias."""
    st = _store()
    name = st.unique("conv2d")
    ax = _channels_axis(data_format)
    cin = inputs.shape[ax]
    w = st.get(f"{name}/kernel", (kernel_size, kernel_size, cin, filters), _variance_scaling)
    x = inputs if data_format == "channels_first" else inputs.permute(0, 3, 1, 2)
    pad_total = kernel_size - 1
    b, e = pad_total // 2, pad_total - pad_total // 2
    x = F.pad(x, (b, e, b, e))   # SAME (stride 1) == fixed padding for odd kernels
    y = F.conv2d(x, w.permute(3, 2, 0, 1), stride=strides)
    return y if data_format == "channels_first" else y.permute(0, 2, 3, 1)


def _preact_block(x, convs, is_training, projection_shortcut, data_format):
    """Shared pre-activation skeleton: BN-ReLU -> [projection] -> (conv -> BN-ReLU)* -> conv,
    plus the (identity or projected) shortcut.  `convs` = [(filters, k, stride), ...]."""
    pre = batch_norm_relu(x, is_training, data_format)
    residual = projection_shortcut(pre) if projection_shortcut is not None else x
    h = pre
    for i, (f, k, s) in enumerate(convs):
        if i:
            h = batch_norm_relu(h, is_training, data_format)
        h = conv2d_fixed_padding(h, f, k, s, data_format)
    return h + residual


def building_block(inputs, filters, is_training, projection_shortcut, strides, data_format):
    """Two 3x3 convs (official:94-130); the stride sits on the first."""
    return _preact_block(inputs, [(filters, 3, strides), (filters, 3, 1)], is_training,
                         projection_shortcut, data_format)


def bottleneck_block(inputs, filters, is_training, projection_shortcut, strides, data_format):
    """1x1 -> 3x3 (strided) -> 1x1 expanding to 4*filters (official:133-175)."""
    return _preact_block(inputs, [(filters, 1, 1), (filters, 3, strides), (4 * filters, 1, 1)],
                         is_training, projection_shortcut, data_format)


def block_layer(inputs, filters, block_fn, blocks, strides, is_training, name, data_format):
    """`blocks` blocks; only the first projects (1x1, strided) and strides."""
    width = filters * (4 if block_fn is bottleneck_block else 1)

    def project(t):
        return conv2d_fixed_padding(t, width, 1, strides, data_format)

    x = inputs
    for b in range(blocks):
        x = block_fn(x, filters, is_training, project if b == 0 else None,
                     strides if b == 0 else 1, data_format)
    return x


def _dense(inputs, units):
    st = _store()
    k = st.get("dense/kernel", (inputs.shape[1], units), _glorot_uniform)
    b = st.get("dense/bias", (units,), _const(0.0))
    return inputs @ k + b


class _Model:
    """The callable returned by the generators; owns its VariableStore."""

    def __init__(self, body, data_format, seed=0):
        self.body = body
        self.data_format = data_format
        self.store = VariableStore(seed)

    def __call__(self, inputs, is_training):
        with _Scope(self.store):
            if self.data_format == "channels_first":
                inputs = inputs.permute(0, 3, 1, 2)
            return self.body(inputs, is_training, self.data_format)

    def variables(self) -> "OrderedDict[str, torch.Tensor]":
        return self.store.vars

    def trainable_variables(self):
        return [self.store.vars[n] for n in self.store.trainable]


def _resolve_format(data_format):
    return data_format or "channels_last"


def cifar10_resnet_v2_generator(resnet_size, num_classes, data_format=None):
    if resnet_size % 6 != 2:
        raise ValueError("resnet_size must be 6n + 2:", resnet_size)
    num_blocks = (resnet_size - 2) // 6
    data_format = _resolve_format(data_format)

    def body(inputs, is_training, df):
        inputs = conv2d_fixed_padding(inputs, 16, 3, 1, df)
        inputs = block_layer(inputs, 16, building_block, num_blocks, 1, is_training,
                             "block_layer1", df)
        inputs = block_layer(inputs, 32, building_block, num_blocks, 2, is_training,
                             "block_layer2", df)
        inputs = block_layer(inputs, 64, building_block, num_blocks, 2, is_training,
                             "block_layer3", df)
        inputs = batch_norm_relu(inputs, is_training, df)
        sp = (2, 3) if df == "channels_first" else (1, 2)
        inputs = inputs.mean(dim=sp)                   # average_pooling2d(8, VALID) + reshape
        return _dense(inputs, num_classes)

    return _Model(body, data_format)


def imagenet_resnet_v2_generator(block_fn, layers, num_classes, data_format=None):
    data_format = _resolve_format(data_format)

    def body(inputs, is_training, df):
        inputs = conv2d_fixed_padding(inputs, 64, 7, 2, df)
        # max_pooling2d(3, 2, 'SAME'): pad 0 before / the rest after with -inf
        x = inputs if df == "channels_first" else inputs.permute(0, 3, 1, 2)
        H, W = x.shape[2], x.shape[3]
        Ho, Wo = -(-H // 2), -(-W // 2)
        ph, pw = max((Ho - 1) * 2 + 3 - H, 0), max((Wo - 1) * 2 + 3 - W, 0)
        x = F.pad(x, (pw // 2, pw - pw // 2, ph // 2, ph - ph // 2), value=float("-inf"))
        x = F.max_pool2d(x, 3, 2)
        inputs = x if df == "channels_first" else x.permute(0, 2, 3, 1)
        for i, (f, s) in enumerate(((64, 1), (128, 2), (256, 2), (512, 2))):
            inputs = block_layer(inputs, f, block_fn, layers[i], s, is_training,
                                 f"block_layer{i + 1}", df)
        inputs = batch_norm_relu(inputs, is_training, df)
        sp = (2, 3) if df == "channels_first" else (1, 2)
        inputs = inputs.mean(dim=sp)
        return _dense(inputs, num_classes)

    return _Model(body, data_format)


def imagenet_resnet_v2(resnet_size, num_classes, data_format=None):
    model_params = {
        18: {"block": building_block, "layers": [2, 2, 2, 2]},
        34: {"block": building_block, "layers": [3, 4, 6, 3]},
        50: {"block": bottleneck_block, "layers": [3, 4, 6, 3]},
        101: {"block": bottleneck_block, "layers": [3, 4, 23, 3]},
        152: {"block": bottleneck_block, "layers": [3, 8, 36, 3]},
        200: {"block": bottleneck_block, "layers": [3, 24, 36, 3]},
    }
    if resnet_size not in model_params:
        raise ValueError("Not a valid resnet_size:", resnet_size)
    p = model_params[resnet_size]
    return imagenet_resnet_v2_generator(p["block"], p["layers"], num_classes, data_format)
