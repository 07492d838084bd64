"""A learnable synthetic CIFAR-10 stand-in, written in the CIFAR-10 binary layout.

There is no network here to fetch CIFAR-10, so the reference's accuracy result
(93.3 % / 93.6 % "Best Precision", README.md:22-28) cannot be reproduced; its
parity stays unpinned.  What CAN be checked offline is that the training stack
learns: this generator makes a 10-class task with real structure -- each class
is a fixed smooth colour template (random 4x4 field, bilinearly upsampled) and
every image is its class template at a random brightness/contrast, shifted by a
few pixels, plus per-pixel noise and a random low-frequency distractor -- so a
ResNet must learn translation-tolerant colour/shape features, the pad-crop-flip
augmentation is exercised, and held-out precision measures generalisation.

  python -m distributed_tensorflow_resnet_amd.data.learnable DIR [--train 10000 --test 2000]

writes DIR/data_batch_{1..5}.bin and DIR/test_batch.bin (3073-byte records:
label byte + 32x32x3 depth-major pixels, cifar_input.py:25-119 layout).
"""
from __future__ import annotations

import argparse
import os

import numpy as np

from .cifar import write_records


def _smooth_fields(rng, n, lo=4):
    """n random 3x32x32 fields, bilinear upsampling of lo x lo noise, in [-1, 1]."""
    import torch

    f = torch.from_numpy(rng.standard_normal((n, 3, lo, lo)).astype(np.float32))
    up = torch.nn.functional.interpolate(f, size=(32, 32), mode="bilinear", align_corners=False)
    up = up / up.abs().amax(dim=(1, 2, 3), keepdim=True).clamp_min(1e-6)
    return up.numpy()


def make_images(rng, templates, labels, noise=45.0, shift=3):
    n = labels.shape[0]
    base = templates[labels]                                   # [n, 3, 32, 32] in [-1, 1]
    dx = rng.integers(-shift, shift + 1, n)
    dy = rng.integers(-shift, shift + 1, n)
    out = np.empty_like(base)
    for i in range(n):
        out[i] = np.roll(base[i], (dy[i], dx[i]), axis=(1, 2))
    contrast = rng.uniform(40, 80, (n, 1, 1, 1))
    bright = rng.uniform(100, 156, (n, 1, 1, 1))
    distract = _smooth_fields(rng, n, lo=3) * rng.uniform(0, 35, (n, 1, 1, 1))
    img = bright + contrast * out + distract + rng.normal(0, noise, out.shape)
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


def make_learnable_cifar(out_dir: str, n_train: int = 10000, n_test: int = 2000, seed: int = 0,
                         num_classes: int = 10, noise: float = 45.0, shift: int = 3,
                         separation: float = 1.0) -> dict:
    """``separation`` < 1 blends every class template with one field common to all
    classes (template = (1 - s) * common + s * own), which with more ``noise`` / ``shift``
    makes the classes confusable: a task a deep network does not solve perfectly."""
    rng = np.random.default_rng(seed)
    templates = _smooth_fields(rng, num_classes)
    if separation != 1.0:
        common = _smooth_fields(rng, 1)
        templates = (1.0 - separation) * common + separation * templates
    os.makedirs(out_dir, exist_ok=True)
    ytr = rng.integers(0, num_classes, n_train)
    yte = rng.integers(0, num_classes, n_test)
    xtr = make_images(rng, templates, ytr, noise, shift)
    xte = make_images(rng, templates, yte, noise, shift)
    parts = np.array_split(np.arange(n_train), 5)
    for i, idx in enumerate(parts, start=1):
        write_records(os.path.join(out_dir, f"data_batch_{i}.bin"), xtr[idx], ytr[idx])
    write_records(os.path.join(out_dir, "test_batch.bin"), xte, yte)
    return {"train": n_train, "test": n_test, "classes": num_classes, "dir": out_dir}


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("out_dir")
    ap.add_argument("--train", type=int, default=10000)
    ap.add_argument("--test", type=int, default=2000)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--noise", type=float, default=45.0, help="per-pixel noise sigma")
    ap.add_argument("--shift", type=int, default=3, help="max template shift (pixels)")
    ap.add_argument("--separation", type=float, default=1.0,
                    help="class-template weight against a common field (1: none common)")
    a = ap.parse_args(argv)
    print(make_learnable_cifar(a.out_dir, a.train, a.test, a.seed, noise=a.noise, shift=a.shift,
                               separation=a.separation))


if __name__ == "__main__":
    main()
