"""Plain-PyTorch fp32 statements of every op, with TF 1.12 semantics.

These are the numerical oracles for the HIP kernels (tests compare against
them) and the compute path of the CPU trainer (BASELINE config 1, the
``resnet_single.py`` plumbing run).  All tensors are NHWC; conv weights HWIO
(``[kh, kw, Cin, Cout]``, the TF variable layout).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

BN_DECAY = 0.997   # _BATCH_NORM_DECAY, resnet_model_official.py:37
# _BATCH_NORM_EPSILON = 1e-5 (resnet_model_official.py:38), but tf.layers' fused batch
# norm raises any epsilon below 1.001e-5 to 1.001e-5 (cuDNN's minimum): every
# FusedBatchNorm/FusedBatchNormGrad node in the reference's graphs carries
# epsilon = float32(1.001e-5) (model.ckpt-107738.meta, resnet50_cifar_frozen_model_eval.pb;
# tests/test_graphdef_cpu.py pins it).  This is the value the math uses.
BN_EPS = 1.001e-5


def fixed_pads(kernel_size: int) -> tuple[int, int]:
    """fixed_padding (resnet_model_official.py:53-77): (pad_beg, pad_end)."""
    total = kernel_size - 1
    beg = total // 2
    return beg, total - beg


def conv2d(x: torch.Tensor, w_hwio: torch.Tensor, stride: int) -> torch.Tensor:
    """conv2d_fixed_padding on NHWC: SAME for stride 1, explicit pad + VALID otherwise.

    For odd kernels both cases pad (k-1)//2 before and the rest after, so one
    formula covers them (TF SAME at stride 1 pads total k-1, top = total//2).
    """
    kh, kw = w_hwio.shape[0], w_hwio.shape[1]
    bh, eh = fixed_pads(kh)
    bw, ew = fixed_pads(kw)
    xn = x.permute(0, 3, 1, 2)
    xn = F.pad(xn, (bw, ew, bh, eh))
    w = w_hwio.permute(3, 2, 0, 1)  # OIHW
    y = F.conv2d(xn, w, stride=stride)
    return y.permute(0, 2, 3, 1)


def batch_norm_train(x: torch.Tensor, gamma, beta, eps: float = BN_EPS):
    """TF fused batch norm, training mode.  Returns y, batch mean, biased var,
    Bessel-corrected var (the value fed to the moving variance)."""
    dims = tuple(range(x.dim() - 1))
    mean = x.mean(dim=dims)
    var = x.var(dim=dims, unbiased=False)
    n = x.numel() // x.shape[-1]
    uvar = var * n / max(n - 1, 1)
    y = (x - mean) * torch.rsqrt(var + eps) * gamma + beta
    return y, mean, var, uvar


def batch_norm_eval(x, gamma, beta, moving_mean, moving_var, eps: float = BN_EPS):
    return (x - moving_mean) * torch.rsqrt(moving_var + eps) * gamma + beta


def moving_update(moving, batch_value, decay: float = BN_DECAY):
    """AssignSub: moving -= (1 - decay) * (moving - value)."""
    return moving - (1.0 - decay) * (moving - batch_value)


def max_pool_same(x: torch.Tensor, k: int = 3, stride: int = 2) -> torch.Tensor:
    """tf.layers.max_pooling2d(padding='SAME') on NHWC (pads with -inf,
    pad_top = total//2 -> 0 before / 1 after for 112->56)."""
    N, H, W, C = x.shape
    Ho, Wo = -(-H // stride), -(-W // stride)
    ph = max((Ho - 1) * stride + k - H, 0)
    pw = max((Wo - 1) * stride + k - W, 0)
    xn = x.permute(0, 3, 1, 2)
    xn = F.pad(xn, (pw // 2, pw - pw // 2, ph // 2, ph - ph // 2), value=float("-inf"))
    y = F.max_pool2d(xn, k, stride)
    return y.permute(0, 2, 3, 1)


def softmax_cross_entropy(logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    """tf.losses.softmax_cross_entropy(onehot, logits): mean over the batch."""
    return F.cross_entropy(logits, labels.long(), reduction="mean")


def l2_loss(v: torch.Tensor) -> torch.Tensor:
    """tf.nn.l2_loss = sum(v**2) / 2."""
    return (v * v).sum() * 0.5


def momentum_step(w, accum, g, lr: float, momentum: float = 0.9):
    """tf.train.MomentumOptimizer (use_nesterov=False): accum = m*accum + g; w -= lr*accum."""
    accum.mul_(momentum).add_(g)
    w.sub_(lr * accum)
    return w, accum


def per_image_standardization(img: torch.Tensor) -> torch.Tensor:
    """tf.image.per_image_standardization on one HWC image."""
    x = img.float()
    n = x.numel()
    mean = x.mean()
    std = x.std(unbiased=False)
    adj = torch.clamp(std, min=1.0 / (n ** 0.5))
    return (x - mean) / adj
