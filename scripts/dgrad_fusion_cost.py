#!/usr/bin/env python3
"""Implicit-GEMM dgrad: device time per launch plain vs with the BN-backward sums
epilogue (BNB: reads the BN input rows, masks the ReLU, sums g and g*xhat into the
fp64 accumulators), on the ImageNet ResNet-50 dgrad shapes.
python scripts/dgrad_fusion_cost.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_tensorflow_resnet_amd.ops import functional as fn  # noqa: E402

BF = torch.bfloat16
# (H, C = dgrad output channels, K = dy channels, k, stride)
SHAPES = [(56, 256, 64, 1, 1), (56, 64, 64, 3, 1), (56, 64, 256, 1, 1), (28, 512, 128, 1, 1),
          (28, 128, 128, 3, 1), (28, 128, 512, 1, 1), (14, 1024, 256, 1, 1), (14, 256, 256, 3, 1),
          (14, 256, 1024, 1, 1), (7, 2048, 512, 1, 1), (7, 512, 512, 3, 1), (7, 512, 2048, 1, 1)]


def timeit(f, iters=20):
    for _ in range(3):
        f()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        f()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    dev = torch.device("cuda")
    N = 128
    nat = fn.native()
    for H, C, K, k, s in SHAPES:
        g = fn.ConvGeom(N, H, H, C, K, k, k, s)
        dy = torch.randn(N, g.Ho, g.Wo, K, device=dev).to(BF)
        w = (torch.randn(k, k, C, K, device=dev) * 0.05).to(BF)
        x = torch.randn(N, H, H, C, device=dev).to(BF)
        dx = torch.empty_like(x)
        mean, rstd = torch.randn(C, device=dev) * 0.1, torch.rand(C, device=dev) + 0.5
        sc, sh = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
        M = N * H * H
        part = torch.zeros(nat.conv_gemm_bm(M, C) and (M // 64 + 1) * 2 * C, device=dev)
        acc = torch.zeros(8 * 2 * C, device=dev, dtype=torch.float64)
        t0 = timeit(lambda: fn.conv2d_dgrad(dy, w, tuple(x.shape), s, out=dx))
        bnb = (x, mean, rstd, sc, sh, part)
        t1 = timeit(lambda: fn.conv2d_dgrad(dy, w, tuple(x.shape), s, out=dx, bnb=bnb))
        t2 = timeit(lambda: fn.conv2d_dgrad(dy, w, tuple(x.shape), s, out=dx, bnb=bnb, bfin=[acc]))
        print(f"H {H:2d} C {C:4d} K {K:4d} k{k}: plain {t0:7.1f} | +bnb partials {t1:7.1f} | "
              f"+bnb fp64 acc {t2:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
