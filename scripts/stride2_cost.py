#!/usr/bin/env python3
"""Device time of the stride-2 convs' data gradients (the implicit GEMM masks 3/4 of
the tap x pixel pairs by output parity) vs their forward, CIFAR and ImageNet shapes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_tensorflow_resnet_amd.ops import functional as fn  # noqa: E402

SHAPES = [(128, 32, 16, 32, 3), (128, 32, 16, 32, 1), (128, 16, 32, 64, 3), (128, 16, 32, 64, 1),
          (128, 56, 128, 128, 3), (128, 56, 256, 512, 1), (128, 28, 256, 256, 3),
          (128, 28, 512, 1024, 1), (128, 14, 512, 512, 3), (128, 14, 1024, 2048, 1)]


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
    for N, H, C, K, k in SHAPES:
        g = fn.ConvGeom(N, H, H, C, K, k, k, 2)
        x = torch.randn(N, H, H, C, device=dev).to(torch.bfloat16)
        w = (torch.randn(K, k, k, C, device=dev) * 0.05).to(torch.bfloat16)
        whwio = w.permute(1, 2, 3, 0).contiguous()
        dy = torch.randn(N, g.Ho, g.Wo, K, device=dev).to(torch.bfloat16)
        dx = torch.empty_like(x)
        out = torch.empty(N, g.Ho, g.Wo, K, device=dev, dtype=torch.bfloat16)
        t_f = timeit(lambda: fn.conv2d_fwd(x, w, 2, out=out))
        t_d = timeit(lambda: fn.conv2d_dgrad(dy, whwio, tuple(x.shape), 2, out=dx))
        fl = 2.0 * N * g.Ho * g.Wo * K * k * k * C
        print(f"N{N} H{H:3d} C{C:5d} K{K:5d} k{k} s2: fwd {t_f:7.1f} us ({fl / t_f / 1e6:5.0f} TF) | "
              f"dgrad {t_d:7.1f} us ({fl / t_d / 1e6:5.0f} TF)", flush=True)


if __name__ == "__main__":
    main()
