"""Real-data ImageNet feed, host half (data/vgg.py crop_u8, data/imagenet.py u8
loader): the uint8 crops are the reference's VGG train/eval crops
(vgg_preprocessing.py:284-333) minus the flip and mean subtraction, which run
on the device (tests/test_imagenet_feed_gpu.py)."""
import io

import numpy as np
import pytest
import torch
from PIL import Image

from distributed_tensorflow_resnet_amd.data import imagenet, vgg
from distributed_tensorflow_resnet_amd.utils import records


@pytest.mark.parametrize("train", [True, False])
@pytest.mark.parametrize("hw", [(375, 500), (500, 333), (256, 256)])
def test_crop_u8_equals_resize_then_crop(train, hw):
    rng0 = np.random.default_rng(1)
    img = Image.fromarray(rng0.integers(0, 256, hw + (3,)).astype(np.uint8))
    for seed in range(4):
        got = vgg.crop_u8(img, 224, 224, train, rng=np.random.default_rng(seed))
        r = np.random.default_rng(seed)
        side = int(r.integers(256, 513)) if train else 256
        full = vgg.aspect_preserving_resize(img, side)
        want = vgg.random_crop(full, 224, 224, r) if train else vgg.central_crop(full, 224, 224)
        assert got.dtype == np.uint8 and got.shape == (224, 224, 3)
        d = np.abs(got.astype(int) - want.astype(int))
        assert d.max() <= 2 and d.mean() < 0.05     # PIL fixed-point rounding of the box



def test_u8_loader_batches(tmp_path):
    rng = np.random.default_rng(0)
    w = records.RecordWriter(str(tmp_path / "train-00000-of-01024"))
    for i in range(6):
        buf = io.BytesIO()
        Image.fromarray(rng.integers(0, 256, (300, 400, 3)).astype(np.uint8)).save(buf, "JPEG")
        w.write(records.make_example({"image/encoded": buf.getvalue(), "image/format": b"JPEG",
                                      "image/class/label": 1 + i}))
    w.close()
    (x, y), = list(imagenet.input_fn(True, str(tmp_path), 6, workers=0, u8=True))
    assert x.dtype == torch.uint8 and x.shape == (6, 224, 224, 3)
    assert sorted(y.tolist()) == list(range(6))     # 1-based labels -> 0-based
