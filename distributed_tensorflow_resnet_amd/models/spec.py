"""Static architecture description of the pre-activation ResNet v2 family.

One walk over the reference builder (resnet_model_official.py:94-366) produces
everything downstream needs, in TF *creation order*:

* the block structure (stem, building/bottleneck blocks, projection shortcuts,
  final BN, dense) with per-layer shapes -- consumed by the GPU engine's plan
  builder and by the CPU model;
* the TF variable names ``conv2d[_N]/kernel``, ``batch_normalization[_N]/{gamma,
  beta,moving_mean,moving_variance}``, ``dense/{kernel,bias}`` with HWIO shapes --
  consumed by the flat parameter buffers and the tensor-bundle checkpoint.

Creation order matters: the projection conv is created after the block's first
BN and before its first conv (``conv2d_1`` is ``[1,1,16,16]`` in
CIFAR ResNet-50).
"""
from __future__ import annotations

from dataclasses import dataclass, field

# resnet_model_official.py:350-359
IMAGENET_SIZES = {
    18: ("building", [2, 2, 2, 2]),
    34: ("building", [3, 4, 6, 3]),
    50: ("bottleneck", [3, 4, 6, 3]),
    101: ("bottleneck", [3, 4, 23, 3]),
    152: ("bottleneck", [3, 8, 36, 3]),
    200: ("bottleneck", [3, 24, 36, 3]),
}


@dataclass
class ConvSpec:
    name: str          # TF layer name, e.g. "conv2d_3"
    kh: int
    kw: int
    cin: int
    cout: int
    stride: int
    h: int             # input spatial size
    w: int

    @property
    def ho(self) -> int:
        return (self.h - 1) // self.stride + 1

    @property
    def wo(self) -> int:
        return (self.w - 1) // self.stride + 1

    @property
    def shape(self):   # TF kernel variable layout HWIO
        return (self.kh, self.kw, self.cin, self.cout)


@dataclass
class BNSpec:
    name: str          # e.g. "batch_normalization_4"
    channels: int
    h: int
    w: int


@dataclass
class BlockSpec:
    kind: str                    # "building" | "bottleneck"
    stride: int
    cin: int
    cout: int
    bns: list                    # BNSpec per pre-activation (2 or 3)
    convs: list                  # ConvSpec main path (2 or 3)
    proj: ConvSpec | None        # projection shortcut (first block of a layer)
    h: int
    w: int
    ho: int
    wo: int


@dataclass
class ParamSpec:
    name: str          # full variable name, e.g. "conv2d_3/kernel"
    shape: tuple
    kind: str          # conv | gamma | beta | moving_mean | moving_variance | dense_kernel | dense_bias
    trainable: bool
    layer: str         # owning layer name


@dataclass
class ModelSpec:
    dataset: str
    resnet_size: int
    num_classes: int
    image_h: int
    image_w: int
    stem: ConvSpec
    maxpool: bool
    blocks: list
    final_bn: BNSpec
    dense_in: int
    params: list = field(default_factory=list)

    @property
    def trainables(self):
        return [p for p in self.params if p.trainable]

    def num_trainable(self) -> int:
        n = 0
        for p in self.trainables:
            k = 1
            for s in p.shape:
                k *= s
            n += k
        return n

    def all_convs(self):
        out = [self.stem]
        for b in self.blocks:
            if b.proj is not None:
                out.append(b.proj)
            out.extend(b.convs)
        return out


class _Namer:
    def __init__(self):
        self.counts: dict[str, int] = {}

    def __call__(self, base: str) -> str:
        n = self.counts.get(base, 0)
        self.counts[base] = n + 1
        return base if n == 0 else f"{base}_{n}"


def _add_conv(spec_params, namer, kh, cin, cout, stride, h, w) -> ConvSpec:
    c = ConvSpec(namer("conv2d"), kh, kh, cin, cout, stride, h, w)
    spec_params.append(ParamSpec(f"{c.name}/kernel", c.shape, "conv", True, c.name))
    return c


def _add_bn(spec_params, namer, ch, h, w) -> BNSpec:
    b = BNSpec(namer("batch_normalization"), ch, h, w)
    spec_params += [
        ParamSpec(f"{b.name}/gamma", (ch,), "gamma", True, b.name),
        ParamSpec(f"{b.name}/beta", (ch,), "beta", True, b.name),
        ParamSpec(f"{b.name}/moving_mean", (ch,), "moving_mean", False, b.name),
        ParamSpec(f"{b.name}/moving_variance", (ch,), "moving_variance", False, b.name),
    ]
    return b


def _block(params, namer, kind, cin, filters, stride, projection, h, w) -> BlockSpec:
    """building_block (official:94-130) / bottleneck_block (official:133-175)."""
    cout = 4 * filters if kind == "bottleneck" else filters
    ho, wo = (h - 1) // stride + 1, (w - 1) // stride + 1
    bns, convs = [], []
    bns.append(_add_bn(params, namer, cin, h, w))
    proj = _add_conv(params, namer, 1, cin, cout, stride, h, w) if projection else None
    if kind == "building":
        convs.append(_add_conv(params, namer, 3, cin, filters, stride, h, w))
        bns.append(_add_bn(params, namer, filters, ho, wo))
        convs.append(_add_conv(params, namer, 3, filters, filters, 1, ho, wo))
    else:
        convs.append(_add_conv(params, namer, 1, cin, filters, 1, h, w))
        bns.append(_add_bn(params, namer, filters, h, w))
        convs.append(_add_conv(params, namer, 3, filters, filters, stride, h, w))
        bns.append(_add_bn(params, namer, filters, ho, wo))
        convs.append(_add_conv(params, namer, 1, filters, cout, 1, ho, wo))
    return BlockSpec(kind, stride, cin, cout, bns, convs, proj, h, w, ho, wo)


def cifar_spec(resnet_size: int = 50, num_classes: int = 10, image_hw: int = 32) -> ModelSpec:
    """cifar10_resnet_v2_generator (official:217-278): 6n+2, filters 16/32/64."""
    if resnet_size % 6 != 2:
        raise ValueError(f"resnet_size must be 6n + 2: {resnet_size}")
    n = (resnet_size - 2) // 6
    params: list = []
    namer = _Namer()
    H = W = image_hw
    stem = _add_conv(params, namer, 3, 3, 16, 1, H, W)
    blocks = []
    cin = 16
    for filters, stride in ((16, 1), (32, 2), (64, 2)):
        for i in range(n):
            s = stride if i == 0 else 1
            b = _block(params, namer, "building", cin, filters, s, i == 0, H, W)
            blocks.append(b)
            cin, H, W = b.cout, b.ho, b.wo
    final_bn = _add_bn(params, namer, cin, H, W)
    params.append(ParamSpec("dense/kernel", (cin, num_classes), "dense_kernel", True, "dense"))
    params.append(ParamSpec("dense/bias", (num_classes,), "dense_bias", True, "dense"))
    return ModelSpec("cifar10", resnet_size, num_classes, image_hw, image_hw, stem, False, blocks,
                     final_bn, cin, params)


def imagenet_spec(resnet_size: int = 50, num_classes: int = 1000, image_hw: int = 224,
                  block: str | None = None, layers: list | None = None) -> ModelSpec:
    """imagenet_resnet_v2_generator (official:281-347) with the size table (:350-366).

    ``block``/``layers`` override the table (the generator's own arguments,
    official:281) for custom depths, e.g. shallow test networks."""
    if block is not None and layers is not None:
        kind = block
    elif resnet_size not in IMAGENET_SIZES:
        raise ValueError(f"Not a valid resnet_size: {resnet_size}")
    else:
        kind, layers = IMAGENET_SIZES[resnet_size]
    params: list = []
    namer = _Namer()
    stem = _add_conv(params, namer, 7, 3, 64, 2, image_hw, image_hw)
    H = W = -(-stem.ho // 2)   # 3x3/2 SAME max-pool
    blocks = []
    cin = 64
    for li, (filters, stride) in enumerate(((64, 1), (128, 2), (256, 2), (512, 2))):
        for i in range(layers[li]):
            s = stride if i == 0 else 1
            b = _block(params, namer, kind, cin, filters, s, i == 0, H, W)
            blocks.append(b)
            cin, H, W = b.cout, b.ho, b.wo
    final_bn = _add_bn(params, namer, cin, H, W)
    params.append(ParamSpec("dense/kernel", (cin, num_classes), "dense_kernel", True, "dense"))
    params.append(ParamSpec("dense/bias", (num_classes,), "dense_bias", True, "dense"))
    spec = ModelSpec("imagenet", resnet_size, num_classes, image_hw, image_hw, stem, True, blocks,
                     final_bn, cin, params)
    return spec


def build_spec(dataset: str, resnet_size: int, num_classes: int | None = None) -> ModelSpec:
    if dataset in ("cifar10", "cifar100", "cifar"):
        nc = num_classes or (100 if dataset == "cifar100" else 10)
        s = cifar_spec(resnet_size, nc)
        s.dataset = "cifar100" if dataset == "cifar100" else "cifar10"
        return s
    if dataset == "imagenet":
        return imagenet_spec(resnet_size, num_classes or 1000)
    raise ValueError(f"unknown dataset {dataset}")
