"""Torch-tensor front end of the native gfx950 kernels.

Every function here validates shapes/dtypes/devices on the host, allocates the
outputs with torch's caching allocator and launches the HIP kernel on the
current stream.  There is deliberately NO fallback: on a GPU box a missing
extension or a bad argument raises.  CPU code paths use ``ops.reference``.

Layout conventions: activations NHWC bf16; conv weights bf16 in
``ohwi`` = [K][kh][kw][C] (forward B operand) and ``hwio`` = [kh][kw][C][K]
(TF layout; dgrad B operand); BN statistics and all optimizer state fp32.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from .. import native
from .reference import BN_EPS

BF16 = torch.bfloat16


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _ptr(t: torch.Tensor | None) -> int:
    return 0 if t is None else t.data_ptr()


def _check(t: torch.Tensor, dtype, ndim: int | None = None, name: str = "tensor"):
    if not t.is_cuda:
        raise ValueError(f"{name} must be a GPU tensor")
    if t.dtype != dtype:
        raise ValueError(f"{name} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if ndim is not None and t.dim() != ndim:
        raise ValueError(f"{name} must be {ndim}-D, got {tuple(t.shape)}")


@dataclass(frozen=True)
class ConvGeom:
    """TF ``conv2d_fixed_padding`` geometry (resnet_model_official.py:80-91)."""
    N: int
    H: int
    W: int
    C: int
    K: int
    kh: int
    kw: int
    stride: int

    @property
    def pad(self) -> int:
        return (self.kh - 1) // 2

    @property
    def Ho(self) -> int:
        return (self.H - 1) // self.stride + 1

    @property
    def Wo(self) -> int:
        return (self.W - 1) // self.stride + 1

    def as_list(self):
        return [self.N, self.H, self.W, self.C, self.Ho, self.Wo, self.K, self.kh, self.kw,
                self.stride, self.pad]


def stat_tiles(M: int, ncol: int) -> tuple[int, int]:
    """(tiles, rows per tile) of the conv epilogue's BN-stat partials."""
    bm = native().conv_gemm_bm(M, ncol)
    return (M + bm - 1) // bm, bm


def conv2d_fwd(x, w_ohwi, stride: int, *, pre_scale=None, pre_shift=None, residual=None,
               stat_part=None, bias=None, out=None, out_f32: bool = False, accumulate=False,
               fin=None, pfin=None):
    """y = conv(relu(x*pre_scale+pre_shift) if pre else x, W) [+bias] [+residual].

    ``fin=[counters, gamma, beta, mmean, mvar, mean, rstd, scale, shift, gpart, group,
    groups_only]`` (tensors or ints) finalizes the output's BN statistics inside the
    kernel (last arriver); ``pfin=[part, cnt, rows_per, M, gamma, beta, mean, rstd,
    scale, shift, mmean, mvar]`` finalizes the PRE BatchNorm in the prologue (the
    kernel is that BN's first consumer; pre_scale/pre_shift are then outputs)."""
    _check(x, BF16, 4, "x")
    _check(w_ohwi, BF16, 4, "w_ohwi")
    N, H, W, C = x.shape
    K, kh, kw, C2 = w_ohwi.shape
    if C2 != C:
        raise ValueError(f"channel mismatch x C={C} vs w C={C2}")
    g = ConvGeom(N, H, W, C, K, kh, kw, stride)
    if out is None:
        out = torch.empty((N, g.Ho, g.Wo, K), device=x.device,
                          dtype=torch.float32 if out_f32 else BF16)
    if residual is not None:
        _check(residual, BF16, 4, "residual")
        if tuple(residual.shape) != tuple(out.shape):
            raise ValueError("residual shape mismatch")
    if pre_scale is not None:
        _check(pre_scale, torch.float32, 1, "pre_scale")
        _check(pre_shift, torch.float32, 1, "pre_shift")
    if stat_part is not None:
        tiles, _ = stat_tiles(N * g.Ho * g.Wo, K)
        if stat_part.numel() < tiles * 2 * K:
            raise ValueError("stat_part too small")
    native().conv_gemm(0, x.data_ptr(), w_ohwi.data_ptr(),
                       0 if out_f32 else out.data_ptr(), out.data_ptr() if out_f32 else 0,
                       _ptr(residual), _ptr(pre_scale), _ptr(pre_shift), _ptr(bias),
                       0 if bias is None else bias.numel(), _ptr(stat_part), int(accumulate),
                       g.as_list(), [], _ptrs(fin), [], _ptrs(pfin), [], 0.997, BN_EPS, 1, _stream())
    return out


def _ptrs(lst):
    return [] if lst is None else [t.data_ptr() if torch.is_tensor(t) else int(t) for t in lst]


def conv2d_dgrad(dy, w_hwio, x_shape, stride: int, *, out=None, accumulate=False, bnb=None,
                 bfin=None, abwd=None):
    """dx = conv2d_transpose(dy, W) with TF fixed padding; w_hwio [kh][kw][C][K].

    ``bnb=(x, mean, rstd, scale, shift, part)`` additionally emits the
    BN+ReLU backward partials of dx (per tile: sum g, sum g*xhat, g = dx*[relu]).
    ``abwd=[x, add, mean, rstd, scale, shift, gamma, part, cnt, a_out, dgamma, dbeta,
    coef]``: ``dy`` is the gradient BEFORE its BatchNorm+ReLU backward, which the kernel
    applies while staging (writing the result to a_out) -- direct 3x3 kernel only."""
    _check(dy, BF16, 4, "dy")
    _check(w_hwio, BF16, 4, "w_hwio")
    N, H, W, C = x_shape
    kh, kw, C2, K = w_hwio.shape
    g = ConvGeom(N, H, W, C, K, kh, kw, stride)
    if tuple(dy.shape) != (N, g.Ho, g.Wo, K) or C2 != C:
        raise ValueError(f"dgrad shape mismatch dy={tuple(dy.shape)} geom={g}")
    if out is None:
        out = torch.empty((N, H, W, C), device=dy.device, dtype=BF16)
    bl = [] if bnb is None else [t.data_ptr() for t in bnb]
    native().conv_gemm(1, dy.data_ptr(), w_hwio.data_ptr(), out.data_ptr(), 0, 0, 0, 0, 0, 0, 0,
                       int(accumulate), g.as_list(), bl, [], _ptrs(bfin), [], _ptrs(abwd), 0.997, BN_EPS, 1,
                       _stream())
    return out


def conv2d_wgrad(dy, x, kh: int, kw: int, stride: int, *, pre_scale=None, pre_shift=None,
                 grad_hwio=None, scale: float = 1.0, accumulate=False, k_valid=None):
    """dW (fp32, TF HWIO) = sum_pixels dy (x) im2col(x); deterministic split-K."""
    _check(dy, BF16, 4, "dy")
    _check(x, BF16, 4, "x")
    N, H, W, C = x.shape
    K = dy.shape[3]
    g = ConvGeom(N, H, W, C, K, kh, kw, stride)
    if tuple(dy.shape) != (N, g.Ho, g.Wo, K):
        raise ValueError("wgrad shape mismatch")
    kv = K if k_valid is None else k_valid
    nat = native()
    splits, pps = nat.wgrad_pick_splits(g.as_list())
    part = torch.empty(splits * K * kh * kw * C, device=dy.device, dtype=torch.float32)
    if grad_hwio is None:
        grad_hwio = torch.empty((kh, kw, C, kv), device=dy.device, dtype=torch.float32)
    nat.conv_wgrad(dy.data_ptr(), x.data_ptr(), _ptr(pre_scale), _ptr(pre_shift),
                   part.data_ptr(), g.as_list(), splits, pps, _stream())
    nat.wgrad_reduce(part.data_ptr(), grad_hwio.data_ptr(), splits, K, kv, kh * kw, C, C,
                     float(scale), int(accumulate), _stream())
    return grad_hwio


def bn_finalize(stat_part, tiles, tile_rows, M, gamma, beta, moving_mean, moving_var,
                momentum=0.997, eps=BN_EPS, update_moving=True):
    C = gamma.numel()
    dev = gamma.device
    mean, rstd, scale, shift = (torch.empty(C, device=dev) for _ in range(4))
    native().bn_finalize(stat_part.data_ptr(), tiles, tile_rows, M, C, gamma.data_ptr(),
                         beta.data_ptr(), moving_mean.data_ptr(), moving_var.data_ptr(),
                         momentum, eps, int(update_moving), mean.data_ptr(), rstd.data_ptr(),
                         scale.data_ptr(), shift.data_ptr(), _stream())
    return mean, rstd, scale, shift


def bn_stats(x2d):
    """Welford partials (tiles x 2 x C) of a [M][C] bf16 tensor."""
    _check(x2d, BF16, 2, "x")
    M, C = x2d.shape
    nat = native()
    tiles = nat.bn_bwd_tiles(M, C)
    part = torch.empty(tiles * 2 * C, device=x2d.device)
    nat.bn_stats(x2d.data_ptr(), M, C, part.data_ptr(), _stream())
    return part, tiles, nat.bn_stats_tile_rows()


def bn_relu_backward(dy2d, x2d, mean, rstd, scale, shift, gamma, add=None):
    """Returns (dx, dgamma, dbeta) of y = relu(bn(x)) given dL/dy (training stats)."""
    _check(dy2d, BF16, 2, "dy")
    _check(x2d, BF16, 2, "x")
    M, C = x2d.shape
    nat = native()
    tiles = nat.bn_bwd_tiles(M, C)
    dev = x2d.device
    part = torch.empty(tiles * 2 * C, device=dev)
    dgamma = torch.empty(C, device=dev)
    dbeta = torch.empty(C, device=dev)
    coef = torch.empty(3 * C, device=dev)
    dx = torch.empty_like(x2d)
    st = _stream()
    nat.bn_bwd_reduce(dy2d.data_ptr(), x2d.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                      scale.data_ptr(), shift.data_ptr(), M, C, part.data_ptr(), st)
    nat.bn_bwd_finalize(part.data_ptr(), tiles, M, C, gamma.data_ptr(), rstd.data_ptr(),
                        dgamma.data_ptr(), dbeta.data_ptr(), coef.data_ptr(), st)
    nat.bn_bwd_apply(dy2d.data_ptr(), x2d.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                     scale.data_ptr(), shift.data_ptr(), coef.data_ptr(), _ptr(add),
                     dx.data_ptr(), M, C, st)
    return dx, dgamma, dbeta


def bn_relu_apply(x2d, scale, shift):
    _check(x2d, BF16, 2, "x")
    M, C = x2d.shape
    y = torch.empty_like(x2d)
    native().bn_relu_apply(x2d.data_ptr(), scale.data_ptr(), shift.data_ptr(), y.data_ptr(), M,
                           C, _stream())
    return y


def bnrelu_avgpool(x, scale, shift):
    _check(x, BF16, 4, "x")
    N, H, W, C = x.shape
    pooled = torch.empty((N, C), device=x.device, dtype=BF16)
    native().bnrelu_avgpool(x.data_ptr(), scale.data_ptr(), shift.data_ptr(), pooled.data_ptr(),
                            N, H * W, C, _stream())
    return pooled


def avgpool_bwd(dpooled, H, W):
    _check(dpooled, BF16, 2, "dpooled")
    N, C = dpooled.shape
    dx = torch.empty((N, H, W, C), device=dpooled.device, dtype=BF16)
    native().avgpool_bwd(dpooled.data_ptr(), dx.data_ptr(), N, H * W, C, _stream())
    return dx


def softmax_xent(logits, labels, classes, grad_scale, want_probs=False):
    """Returns (loss_sum, correct, dlogits bf16 [N][ld], dbias fp32 [classes], probs)."""
    _check(logits, torch.float32, 2, "logits")
    N, ld = logits.shape
    dev = logits.device
    loss = torch.zeros(1, device=dev)
    corr = torch.zeros(1, device=dev)
    dl = torch.empty((N, ld), device=dev, dtype=BF16)
    db = torch.empty(classes, device=dev)
    probs = torch.zeros((N, ld), device=dev) if want_probs else None
    labels = labels.to(device=dev, dtype=torch.int32).contiguous()
    ws = torch.empty(native().softmax_xent_ws_floats(N, ld), device=dev)
    native().softmax_xent(logits.data_ptr(), ld, labels.data_ptr(), N, classes, loss.data_ptr(),
                          corr.data_ptr(), dl.data_ptr(), db.data_ptr(), float(grad_scale),
                          _ptr(probs), ws.data_ptr(), _stream())
    return loss, corr, dl, db, probs


def maxpool_fwd(x, k=3, stride=2):
    """TF max_pooling2d(pool k, stride, padding='SAME') on NHWC.
    Returns (y, argmax) where argmax holds the window position of the first max."""
    _check(x, BF16, 4, "x")
    N, H, W, C = x.shape
    Ho, Wo = -(-H // stride), -(-W // stride)
    pad = max((Ho - 1) * stride + k - H, 0) // 2
    y = torch.empty((N, Ho, Wo, C), device=x.device, dtype=BF16)
    am = torch.empty((N, Ho, Wo, C), device=x.device, dtype=torch.uint8)
    native().maxpool_fwd(x.data_ptr(), y.data_ptr(), am.data_ptr(),
                         [N, H, W, C, Ho, Wo, C, k, k, stride, pad], k, _stream())
    return y, am


def maxpool_bwd(argmax, dy, x_shape, k=3, stride=2):
    N, H, W, C = x_shape
    Ho, Wo = dy.shape[1], dy.shape[2]
    pad = max((Ho - 1) * stride + k - H, 0) // 2
    dx = torch.empty(x_shape, device=dy.device, dtype=BF16)
    native().maxpool_bwd(argmax.data_ptr(), dy.data_ptr(), dx.data_ptr(),
                         [N, H, W, C, Ho, Wo, C, k, k, stride, pad], k, _stream())
    return dx


def cifar_augment(img_u8, cpad=8, pad=4, seed=0, gstep=None, train=True, log_crops=False):
    """Raw CIFAR records [N,3,H,W] uint8 -> standardized bf16 NHWC (Cpad channels)."""
    if img_u8.dtype != torch.uint8 or not img_u8.is_cuda:
        raise ValueError("img must be a uint8 GPU tensor [N,3,H,W]")
    N, _, H, W = img_u8.shape
    out = torch.empty((N, H, W, cpad), device=img_u8.device, dtype=BF16)
    log = torch.zeros((N, 3), device=img_u8.device, dtype=torch.int32) if log_crops else None
    native().cifar_augment(img_u8.data_ptr(), out.data_ptr(), N, H, W, cpad, pad, seed,
                           _ptr(gstep), int(train), _ptr(log), 0, 0, _stream())
    return (out, log) if log_crops else out
