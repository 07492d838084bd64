"""ImageNet TFRecord input pipeline (resnet_imagenet_main.py:110-192).

Shards: train-00000-of-01024 ... / validation-00000-of-00128 (tf.train.Example
records with `image/encoded` JPEG bytes and a 1-based `image/class/label`).
Records are read with our TFRecord codec, decoded with PIL and VGG-preprocessed
in CPU worker processes (torch DataLoader), batched as float NHWC.

Label fix (reference defect #6): the TFRecord labels are 1-based and the
reference feeds them straight into one_hot(label, 1000), mapping class 1000 to
an all-zero target.  We subtract 1 (``label_offset=1``); pass 0 to reproduce
the reference.
"""
from __future__ import annotations

import io
import os

import numpy as np
import torch

from ..utils.records import parse_example, read_records
from . import vgg

NUM_TRAIN_FILES = 1024
NUM_VAL_FILES = 128
NUM_IMAGES = {"train": 1281167, "validation": 50000}


def filenames(is_training: bool, data_dir: str) -> list[str]:
    if is_training:
        return [os.path.join(data_dir, "train-%05d-of-01024" % i) for i in range(NUM_TRAIN_FILES)]
    return [os.path.join(data_dir, "validation-%05d-of-00128" % i) for i in range(NUM_VAL_FILES)]


def record_parser(raw: bytes, is_training: bool, rng=None, label_offset: int = 1,
                  image_size: int = 224, u8: bool = False):
    """-> (float32 HWC image, int label); u8=True: the uint8 HWC crop for the GPU feed
    (flip + mean subtraction left to imagenet_u8_pack on the device)."""
    from PIL import Image

    ex = parse_example(raw)
    jpeg = ex["image/encoded"][0]
    label = int(ex["image/class/label"][0]) - label_offset
    img = Image.open(io.BytesIO(jpeg))
    # JPEG DCT-domain downscale of large images, never below the preprocessing's
    # resize target (train: shorter side up to 512, eval: 256): PIL's draft keeps both
    # sides >= the request, so the aspect-preserving resize still only downsamples,
    # as vgg_preprocessing.py does from the full decode
    side = vgg._RESIZE_SIDE_MAX if is_training else vgg._RESIZE_SIDE_MIN
    img.draft("RGB", (side, side))
    img = img.convert("RGB")
    if u8:
        return vgg.crop_u8(img, image_size, image_size, is_training, rng=rng), label
    x = vgg.preprocess_image(img, image_size, image_size, is_training, rng=rng)
    return x.astype(np.float32), label


class TFRecordImages(torch.utils.data.IterableDataset):
    """Streams records of the shards assigned to (rank, dataloader worker)."""

    def __init__(self, files, is_training, rank=0, world=1, seed=0, label_offset=1,
                 image_size=224, shuffle_buffer=1024, u8=False):
        self.files = [f for f in files if os.path.exists(f)]
        if not self.files:
            raise FileNotFoundError(f"no TFRecord shards found (e.g. {files[:1]})")
        self.is_training = is_training
        self.rank, self.world = rank, world
        self.seed = seed
        self.label_offset = label_offset
        self.image_size = image_size
        self.shuffle_buffer = shuffle_buffer
        self.u8 = u8

    def __iter__(self):
        wi = torch.utils.data.get_worker_info()
        nw, wid = (wi.num_workers, wi.id) if wi else (1, 0)
        rng = np.random.default_rng(self.seed + 1000 * self.rank + wid)
        files = list(self.files)
        if self.is_training:
            rng.shuffle(files)  # _FILE_SHUFFLE_BUFFER over filenames
        mine = files[self.rank * nw + wid::self.world * nw] or files[wid::nw]
        buf = []
        for f in mine:
            for raw in read_records(f):
                item = record_parser(raw, self.is_training, rng, self.label_offset,
                                     self.image_size, self.u8)
                if not self.is_training:
                    yield item
                    continue
                buf.append(item)
                if len(buf) >= self.shuffle_buffer:
                    yield buf.pop(int(rng.integers(0, len(buf))))
        while buf:
            yield buf.pop(int(rng.integers(0, len(buf))))


def input_fn(is_training, data_dir, batch_size, num_epochs=1, rank=0, world=1, workers=5, seed=0,
             label_offset=1, image_size=224, u8=False, pin_memory=False):
    """Yields (NHWC [B,224,224,3], int64 [B]) for num_epochs passes: float32 VGG-
    preprocessed, or (u8=True) uint8 crops for the device-side flip/mean/pack."""
    ds = TFRecordImages(filenames(is_training, data_dir), is_training, rank, world, seed,
                        label_offset, image_size, u8=u8)
    for ep in range(num_epochs):
        ds.seed = seed + ep
        dl = torch.utils.data.DataLoader(ds, batch_size=batch_size, num_workers=workers,
                                         drop_last=is_training, pin_memory=pin_memory,
                                         collate_fn=_collate, persistent_workers=False,
                                         prefetch_factor=4 if workers else None)
        yield from dl


def _collate(items):
    x = torch.from_numpy(np.stack([i[0] for i in items]))
    y = torch.tensor([i[1] for i in items], dtype=torch.int64)
    return x, y


def synthetic_batches(batch_size, num_classes=1000, image_size=224, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(batch_size, image_size, image_size, 3, generator=g)
    y = torch.randint(0, num_classes, (batch_size,), generator=g)
    while True:
        yield x, y
