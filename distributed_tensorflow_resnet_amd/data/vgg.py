"""VGG-style ImageNet preprocessing (vgg_preprocessing.py:37-363 semantics).

train: aspect-preserving resize so the smaller side is a random integer in
       [256, 512], random 224x224 crop, random left-right flip, per-channel
       mean subtraction (R,G,B = 123.68, 116.78, 103.94);
eval:  aspect-preserving resize to smaller side 256, central 224x224 crop,
       mean subtraction.
Operates on HWC uint8 numpy arrays / PIL images on CPU worker processes (the
real-data path is kept off the benchmark path, SURVEY §7.4 risk 8).
"""
from __future__ import annotations

import numpy as np

_R_MEAN, _G_MEAN, _B_MEAN = 123.68, 116.78, 103.94
_RESIZE_SIDE_MIN = 256
_RESIZE_SIDE_MAX = 512


def smallest_size_at_least(height: int, width: int, smallest_side: int) -> tuple[int, int]:
    """_smallest_size_at_least: scale so min(h, w) == smallest_side (rounded)."""
    scale = smallest_side / min(height, width)
    return int(round(height * scale)), int(round(width * scale))


def aspect_preserving_resize(img, smallest_side: int):
    """Bilinear resize (PIL) preserving aspect ratio; returns HWC float32."""
    from PIL import Image

    pil = img if isinstance(img, Image.Image) else Image.fromarray(np.asarray(img, dtype=np.uint8))
    w, h = pil.size
    nh, nw = smallest_size_at_least(h, w, smallest_side)
    return np.asarray(pil.convert("RGB").resize((nw, nh), Image.BILINEAR), dtype=np.float32)


def central_crop(img: np.ndarray, ch: int, cw: int) -> np.ndarray:
    h, w = img.shape[:2]
    oy, ox = (h - ch) // 2, (w - cw) // 2
    return img[oy:oy + ch, ox:ox + cw]


def random_crop(img: np.ndarray, ch: int, cw: int, rng: np.random.Generator) -> np.ndarray:
    h, w = img.shape[:2]
    if h < ch or w < cw:
        raise ValueError("Crop size greater than the image size.")
    oy = int(rng.integers(0, h - ch + 1))
    ox = int(rng.integers(0, w - cw + 1))
    return img[oy:oy + ch, ox:ox + cw]


def mean_image_subtraction(img: np.ndarray, means=(_R_MEAN, _G_MEAN, _B_MEAN)) -> np.ndarray:
    if img.ndim != 3 or img.shape[-1] != len(means):
        raise ValueError("len(means) must match the number of channels")
    return img - np.asarray(means, dtype=np.float32)


def preprocess_for_train(img, out_h=224, out_w=224, resize_side_min=_RESIZE_SIDE_MIN,
                         resize_side_max=_RESIZE_SIDE_MAX, rng=None) -> np.ndarray:
    rng = rng or np.random.default_rng()
    side = int(rng.integers(resize_side_min, resize_side_max + 1))
    x = aspect_preserving_resize(img, side)
    x = random_crop(x, out_h, out_w, rng)
    if rng.integers(0, 2):
        x = x[:, ::-1]
    return mean_image_subtraction(np.ascontiguousarray(x))


def preprocess_for_eval(img, out_h=224, out_w=224, resize_side=_RESIZE_SIDE_MIN) -> np.ndarray:
    x = aspect_preserving_resize(img, resize_side)
    x = central_crop(x, out_h, out_w)
    return mean_image_subtraction(np.ascontiguousarray(x))


def crop_u8(img, out_h=224, out_w=224, is_training=False, resize_side_min=_RESIZE_SIDE_MIN,
            resize_side_max=_RESIZE_SIDE_MAX, rng=None) -> np.ndarray:
    """The CPU half of preprocess_image for the GPU feed: aspect-preserving resize +
    random (train) / central (eval) crop, returned as uint8 HWC.  The random flip
    and the mean subtraction run on the device (imagenet_u8_pack, csrc/data.hip),
    so the host ships 1 byte per value instead of 4."""
    from PIL import Image

    pil = img if isinstance(img, Image.Image) else Image.fromarray(np.asarray(img, dtype=np.uint8))
    pil = pil.convert("RGB")
    w, h = pil.size
    if is_training:
        rng = rng or np.random.default_rng()
        side = int(rng.integers(resize_side_min, resize_side_max + 1))
    else:
        side = resize_side_min
    nh, nw = smallest_size_at_least(h, w, side)
    if nh < out_h or nw < out_w:
        raise ValueError("Crop size greater than the image size.")
    if is_training:   # the same draws as random_crop on the resized image
        oy = int(rng.integers(0, nh - out_h + 1))
        ox = int(rng.integers(0, nw - out_w + 1))
    else:
        oy, ox = (nh - out_h) // 2, (nw - out_w) // 2
    # resize only the crop's source window: PIL samples output pixel i of the box at
    # box0 + (i + 0.5) * scale - 0.5 with the full-image filter support, i.e. exactly
    # pixel ox + i of the resized image (tests/test_framework_cpu.py), at a fraction
    # of the work (224x224 instead of up to 512x683 resized pixels)
    sx, sy = w / nw, h / nh
    box = (ox * sx, oy * sy, (ox + out_w) * sx, (oy + out_h) * sy)
    x = np.asarray(pil.resize((out_w, out_h), Image.BILINEAR, box=box), dtype=np.uint8)
    return np.ascontiguousarray(x)


def preprocess_image(image, output_height, output_width, is_training=False,
                     resize_side_min=_RESIZE_SIDE_MIN, resize_side_max=_RESIZE_SIDE_MAX, rng=None):
    """vgg_preprocessing.preprocess_image (vgg_preprocessing.py:336-363)."""
    if is_training:
        return preprocess_for_train(image, output_height, output_width, resize_side_min,
                                    resize_side_max, rng)
    return preprocess_for_eval(image, output_height, output_width, resize_side_min)
