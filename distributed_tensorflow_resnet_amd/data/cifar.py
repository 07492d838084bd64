"""CIFAR-10 / CIFAR-100 binary input pipeline.

Record layouts (resnet_cifar_main.py:150-198, cifar_input.py:25-119):
  CIFAR-10   <1 x label><3072 x pixel>               3073 bytes, files
             cifar-10-batches-bin/data_batch_{1..5}.bin, test_batch.bin
  CIFAR-100  <1 x coarse><1 x fine label><3072 x pixel>  3074 bytes (fine label
             used, label_offset=1), files cifar-100-binary/{train,test}.bin
Pixels are depth-major [3][32][32] -- exactly what the device augmentation
kernel (csrc/data.hip cifar_augment) consumes, so the GPU path ships raw uint8
records to the device and pads/crops/flips/standardizes there.  The CPU path
(augment_cpu) implements the same transform with torch ops.

Fixes reference defect #7 (CIFAR-100 training hard-coded to CIFAR-10 records).
"""
from __future__ import annotations

import glob
import os

import numpy as np
import torch

HEIGHT = WIDTH = 32
DEPTH = 3
IMAGE_BYTES = HEIGHT * WIDTH * DEPTH
NUM_IMAGES = {"train": 50000, "validation": 10000}


def record_layout(dataset: str) -> tuple[int, int, int]:
    """(label_offset, label_bytes, num_classes)."""
    if dataset == "cifar10":
        return 0, 1, 10
    if dataset == "cifar100":
        return 1, 1, 100
    raise ValueError(f"Not supported dataset {dataset}")


def get_filenames(is_training: bool, data_dir: str, dataset: str = "cifar10") -> list[str]:
    """Directory (reference layout), explicit file, or glob pattern."""
    if any(ch in data_dir for ch in "*?["):
        files = sorted(glob.glob(data_dir))
    elif os.path.isfile(data_dir):
        files = [data_dir]
    else:
        if dataset == "cifar10":
            sub = os.path.join(data_dir, "cifar-10-batches-bin")
            base = sub if os.path.isdir(sub) else data_dir
            names = ([f"data_batch_{i}.bin" for i in range(1, 6)] if is_training
                     else ["test_batch.bin"])
        else:
            sub = os.path.join(data_dir, "cifar-100-binary")
            base = sub if os.path.isdir(sub) else data_dir
            names = ["train.bin"] if is_training else ["test.bin"]
        files = [os.path.join(base, n) for n in names]
    missing = [f for f in files if not os.path.exists(f)]
    if not files or missing:
        raise FileNotFoundError(f"CIFAR data not found: {missing or data_dir}")
    return files


def load_records(files: list[str], dataset: str = "cifar10") -> tuple[np.ndarray, np.ndarray]:
    """-> images uint8 [N, 3, 32, 32] (depth-major, as stored), labels int64 [N]."""
    off, lb, _ = record_layout(dataset)
    rec = off + lb + IMAGE_BYTES
    imgs, labels = [], []
    for f in files:
        raw = np.fromfile(f, dtype=np.uint8)
        if raw.size % rec:
            raise IOError(f"{f}: size {raw.size} is not a multiple of record size {rec}")
        raw = raw.reshape(-1, rec)
        labels.append(raw[:, off].astype(np.int64))
        imgs.append(raw[:, off + lb:].reshape(-1, DEPTH, HEIGHT, WIDTH))
    return np.concatenate(imgs), np.concatenate(labels)


def write_records(path: str, images: np.ndarray, labels: np.ndarray, dataset: str = "cifar10"):
    """Write images [N,3,32,32] uint8 + labels in the binary layout (fixtures/tools)."""
    off, _, _ = record_layout(dataset)
    n = images.shape[0]
    out = np.zeros((n, off + 1 + IMAGE_BYTES), dtype=np.uint8)
    if off:
        out[:, 0] = (labels // 5).astype(np.uint8)  # coarse label placeholder
    out[:, off] = labels.astype(np.uint8)
    out[:, off + 1:] = images.reshape(n, -1)
    out.tofile(path)


def augment_cpu(img_u8: torch.Tensor, train: bool, generator: torch.Generator | None = None,
                pad: int = 4) -> torch.Tensor:
    """[N,3,H,W] uint8 -> standardized float NHWC (pad/crop/flip/standardize)."""
    x = img_u8.float().permute(0, 2, 3, 1)  # NHWC
    N, H, W, C = x.shape
    if train:
        xp = torch.zeros(N, H + 2 * pad, W + 2 * pad, C)
        xp[:, pad:pad + H, pad:pad + W] = x
        oy = torch.randint(0, 2 * pad + 1, (N,), generator=generator)
        ox = torch.randint(0, 2 * pad + 1, (N,), generator=generator)
        flip = torch.randint(0, 2, (N,), generator=generator).bool()
        out = torch.empty_like(x)
        for i in range(N):
            c = xp[i, oy[i]:oy[i] + H, ox[i]:ox[i] + W]
            out[i] = c.flip(1) if flip[i] else c
        x = out
    flat = x.reshape(N, -1)
    mean = flat.mean(1, keepdim=True)
    std = flat.std(1, unbiased=False, keepdim=True)
    adj = torch.clamp(std, min=1.0 / (flat.shape[1] ** 0.5))
    return ((flat - mean) / adj).reshape(N, H, W, C)


class CifarData:
    """In-memory CIFAR split with rank-sharded, epoch-shuffled batching."""

    def __init__(self, data_path: str, dataset: str = "cifar10", train: bool = True):
        self.dataset = dataset
        self.train = train
        self.files = get_filenames(train, data_path, dataset)
        self.images, self.labels = load_records(self.files, dataset)
        self.num_classes = record_layout(dataset)[2]

    def __len__(self):
        return self.images.shape[0]

    def batches(self, batch_size: int, *, shuffle: bool | None = None, num_epochs: int | None = None,
                seed: int = 0, rank: int = 0, world: int = 1):
        """Yield (uint8 [B,3,32,32], int64 [B]) for this rank: each epoch a fresh
        permutation (same on every rank) is split into disjoint rank shards, like
        tf.data shuffle(50000) per worker; the tail that does not fill a batch on
        every rank is dropped."""
        shuffle = self.train if shuffle is None else shuffle
        n = len(self)
        epoch = 0
        rng = np.random.default_rng(seed)
        while num_epochs is None or epoch < num_epochs:
            perm = rng.permutation(n) if shuffle else np.arange(n)
            per_rank = (n // world) // batch_size * batch_size
            mine = perm[rank * per_rank:(rank + 1) * per_rank] if world > 1 else perm
            for s in range(0, len(mine) - batch_size + 1, batch_size):
                idx = np.sort(mine[s:s + batch_size]) if not shuffle else mine[s:s + batch_size]
                yield torch.from_numpy(self.images[idx]), torch.from_numpy(self.labels[idx])
            epoch += 1


def synthetic_batches(batch_size: int, num_classes: int = 10, seed: int = 0):
    """Endless random uint8 CIFAR-shaped records (for --synthetic)."""
    g = torch.Generator().manual_seed(seed)
    imgs = torch.randint(0, 256, (batch_size, DEPTH, HEIGHT, WIDTH), generator=g, dtype=torch.uint8)
    labels = torch.randint(0, num_classes, (batch_size,), generator=g)
    while True:
        yield imgs, labels
