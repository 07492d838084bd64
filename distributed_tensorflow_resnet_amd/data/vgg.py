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


def preprocess_image(image, output_height, output_width, is_training=False,
                     resize_side_min=_RESIZE_SIDE_MIN, resize_side_max=_RESIZE_SIDE_MAX, rng=None):
    """vgg_preprocessing.preprocess_image (vgg_preprocessing.py:336-363)."""
    if is_training:
        return preprocess_for_train(image, output_height, output_width, resize_side_min,
                                    resize_side_max, rng)
    return preprocess_for_eval(image, output_height, output_width, resize_side_min)
