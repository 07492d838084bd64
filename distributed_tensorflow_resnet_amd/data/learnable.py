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


def _imagenet_shard(args):
    """One TFRecord shard of the learnable ImageNet-format task (worker of
    make_learnable_imagenet): JPEG-encoded class templates under random shift,
    brightness / contrast, a low-frequency distractor and per-pixel noise."""
    import io

    from PIL import Image

    from ..utils import records

    path, labels, templates, distract, seed, size, noise, shift = args
    rng = np.random.default_rng(seed)
    w = records.RecordWriter(path)
    for lab in labels:
        t = np.roll(templates[lab], tuple(rng.integers(-shift, shift + 1, 2)), axis=(1, 2))
        d = distract[rng.integers(0, len(distract))]
        img = (rng.uniform(100, 156) + rng.uniform(40, 80) * t + rng.uniform(0, 30) * d
               + noise * rng.standard_normal(t.shape, dtype=np.float32))
        arr = np.clip(np.rint(img), 0, 255).astype(np.uint8).transpose(1, 2, 0)
        buf = io.BytesIO()
        Image.fromarray(arr).save(buf, format="JPEG", quality=90)
        w.write(records.make_example({"image/encoded": buf.getvalue(), "image/format": b"JPEG",
                                      "image/class/label": int(lab) + 1}))
    w.close()
    return len(labels)


def make_learnable_imagenet(out_dir: str, n_train: int = 25600, n_test: int = 5000,
                            classes: int = 100, seed: int = 0, size: int = 256,
                            noise: float = 30.0, shift: int = 32, separation: float = 0.5,
                            shards: int = 16, workers: int = 8) -> dict:
    """The ImageNet input format (train-%05d-of-01024 / validation-%05d-of-00128
    TFRecord shards of tf.train.Example with JPEG `image/encoded` and a 1-based
    `image/class/label`, data/imagenet.py) holding a learnable task: `classes` smooth
    colour templates (6x6 noise upsampled to `size`), each (1 - separation) a field
    common to all classes, under random shift, brightness / contrast, a distractor and
    per-pixel noise.  The reference's VGG preprocessing then adds scale (shorter side
    256-512) and crop jitter."""
    import multiprocessing as mp

    import torch

    rng = np.random.default_rng(seed)
    f = torch.from_numpy(rng.standard_normal((classes + 1, 3, 6, 6)).astype(np.float32))
    up = torch.nn.functional.interpolate(f, size=(size, size), mode="bilinear",
                                         align_corners=False)
    up = (up / up.abs().amax(dim=(1, 2, 3), keepdim=True).clamp_min(1e-6)).numpy()
    templates = ((1.0 - separation) * up[classes:] + separation * up[:classes]).astype(np.float32)
    d = torch.nn.functional.interpolate(torch.from_numpy(rng.standard_normal((64, 3, 3, 3))
                                                         .astype(np.float32)),
                                        size=(size, size), mode="bilinear", align_corners=False)
    distract = d.numpy()   # a bank of low-frequency distractors, one drawn per image
    os.makedirs(out_dir, exist_ok=True)
    jobs = []
    for split, n, nsh, fmt in (("train", n_train, shards, "train-%05d-of-01024"),
                               ("validation", n_test, max(1, shards // 4),
                                "validation-%05d-of-00128")):
        labels = rng.integers(0, classes, n)
        for k, part in enumerate(np.array_split(labels, nsh)):
            jobs.append((os.path.join(out_dir, fmt % k), part, templates, distract,
                         seed * 100003 + len(jobs), size, noise, shift))
    with mp.get_context("spawn").Pool(max(1, workers)) as pool:
        done = sum(pool.map(_imagenet_shard, jobs))
    return {"images": done, "classes": classes, "dir": out_dir}


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
    ap.add_argument("--imagenet", action="store_true",
                    help="the ImageNet TFRecord/JPEG format (make_learnable_imagenet; --classes, "
                         "--workers; noise / shift / separation default 30 / 32 / 0.5)")
    ap.add_argument("--classes", type=int, default=100)
    ap.add_argument("--workers", type=int, default=8)
    a = ap.parse_args(argv)
    if a.imagenet:
        kw = {k: v for k, v in (("noise", a.noise), ("shift", a.shift),
                                ("separation", a.separation))
              if v != ap.get_default(k)}
        print(make_learnable_imagenet(a.out_dir, a.train, a.test, a.classes, a.seed,
                                      workers=a.workers, **kw))
        return
    print(make_learnable_cifar(a.out_dir, a.train, a.test, a.seed, noise=a.noise, shift=a.shift,
                               separation=a.separation))


if __name__ == "__main__":
    main()
