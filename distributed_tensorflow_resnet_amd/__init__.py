"""MI355X-native distributed ResNet training (capabilities of
michaelwfc/distributed-tensorflow-resnet, re-designed for gfx950 / CDNA4).

Layers (see README.md / SURVEY.md §1):
  csrc/      hand-written HIP kernels (MFMA implicit-GEMM convs, fused BN-ReLU,
             softmax-xent, SGD-momentum) + native static-plan executor (_C)
  ops/       torch-tensor wrappers of the native ops + fp32 PyTorch references
  models/    resnet_model_official-compatible builders, ResNet/HParams wrapper
  train/     GPU engine (flat buffers, static plan, hipGraph), CPU trainer, hooks
  parallel/  RCCL data parallelism (bucketed all-reduce overlapped with backward)
  data/      CIFAR binary / ImageNet TFRecord readers, VGG preprocessing, synthetic
  utils/     flags, TF tensor-bundle checkpoints, event files, crc32c
"""
from __future__ import annotations

import os

import torch  # noqa: F401  (loads the HIP runtime our extension shares by soname)

__version__ = "0.1.0"

PKG_DIR = os.path.dirname(os.path.abspath(__file__))

_native = None
_native_err: Exception | None = None


def native(required: bool = True):
    """Return the compiled ``_C`` extension.

    On a machine with a GPU the extension is mandatory: a missing or stale build
    raises instead of silently falling back to PyTorch ops.
    """
    global _native, _native_err
    if _native is None and _native_err is None:
        try:
            from . import _C  # type: ignore

            _native = _C
        except Exception as e:  # pragma: no cover - depends on build state
            _native_err = e
    if _native is None and required:
        raise RuntimeError(
            "native extension distributed_tensorflow_resnet_amd._C is not built "
            f"({_native_err}); run `python -m distributed_tensorflow_resnet_amd.build`")
    return _native


def gpu_available() -> bool:
    return torch.cuda.is_available()
