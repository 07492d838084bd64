"""`cifar_input` API of the reference (cifar_input.py:25-204).

build_input(dataset, data_path, batch_size, mode)  -> iterator of
    (images float NHWC standardized [B,32,32,3], labels one-hot [B,num_classes])
    train: pad to 36 (this pipeline's reference value; resnet_cifar_main pads to
    40 -- defect #11, both offered via `pad`), random crop, flip, standardize.
eval_data_input(data_path, num, dataset) -> numpy (images standardized NHWC, labels int)
show_eval_images / display_eval_images / save_image_grid -> PNG grids (PIL; the
    reference used matplotlib windows).
"""
import numpy as np
import torch

from distributed_tensorflow_resnet_amd.data.cifar import CifarData, augment_cpu


def build_input(dataset, data_path, batch_size, mode, pad=2, seed=0):
    data = CifarData(data_path, dataset, train=(mode == "train"))
    nc = data.num_classes
    g = torch.Generator().manual_seed(seed)
    for x, y in data.batches(batch_size, shuffle=(mode == "train"),
                             num_epochs=None if mode == "train" else 1, seed=seed):
        imgs = augment_cpu(x, train=(mode == "train"), generator=g, pad=pad)
        onehot = torch.nn.functional.one_hot(y, nc).float()
        yield imgs, onehot


def eval_data_input(data_path, num=100, dataset="cifar10"):
    data = CifarData(data_path, dataset, train=False)
    x = torch.from_numpy(data.images[:num])
    return augment_cpu(x, train=False).numpy(), data.labels[:num].copy()


def save_image_grid(images_u8_chw, pred, truth, path, class_names=None, cols=10):
    """Write a labelled grid of [N,3,32,32] uint8 images (PIL)."""
    from PIL import Image, ImageDraw

    x = images_u8_chw
    if isinstance(x, torch.Tensor):
        x = x.cpu().numpy()
    if x.dtype != np.uint8:  # standardized NHWC float -> displayable
        x = np.asarray(x, dtype=np.float32)
        x = ((x - x.min()) / max(x.max() - x.min(), 1e-6) * 255).astype(np.uint8)
        x = x.transpose(0, 3, 1, 2)
    n = x.shape[0]
    rows = (n + cols - 1) // cols
    cell = 48
    grid = Image.new("RGB", (cols * cell, rows * cell), "white")
    d = ImageDraw.Draw(grid)
    for i in range(n):
        img = Image.fromarray(x[i].transpose(1, 2, 0))
        r, c = divmod(i, cols)
        grid.paste(img, (c * cell + 8, r * cell))
        p, t = int(pred[i]), int(truth[i])
        lab = class_names[p][:6] if class_names else str(p)
        d.text((c * cell + 2, r * cell + 33), lab, fill=(0, 128, 0) if p == t else (200, 0, 0))
    grid.save(path)
    return path


def show_eval_images(images, pred, truth, path="eval_images.png", class_names=None):
    return save_image_grid(images, pred, truth, path, class_names)


def display_eval_images(images, labels, path="eval_images.png"):
    return save_image_grid(images, labels, labels, path)
