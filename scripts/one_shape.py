#!/usr/bin/env python3
"""Run one conv shape's fwd / dgrad / wgrad kernels a few times (for rocprofv3 --pmc
passes on a single kernel).  usage: one_shape.py N H C K k s [reps] [passes]
passes: comma list of fwd (pre+stats), fwd_plain, fwd_stats, dgrad, dgrad_bnb, wgrad
(default fwd,dgrad,wgrad)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_tensorflow_resnet_amd.ops import functional as fn  # noqa: E402


def main():
    N, H, C, K, k, s = (int(v) for v in sys.argv[1:7])
    reps = int(sys.argv[7]) if len(sys.argv) > 7 else 5
    passes = (sys.argv[8] if len(sys.argv) > 8 else "fwd,dgrad,wgrad").split(",")
    dev = torch.device("cuda")
    g = fn.ConvGeom(N, H, H, C, K, k, k, s)
    x = torch.randn(N, H, H, C, device=dev).to(torch.bfloat16)
    w = (torch.randn(K, k, k, C, device=dev) * 0.05).to(torch.bfloat16)
    whwio = w.permute(1, 2, 3, 0).contiguous()
    sc = torch.rand(C, device=dev) + 0.5
    sh = torch.randn(C, device=dev) * 0.1
    dy = torch.randn(N, g.Ho, g.Wo, K, device=dev).to(torch.bfloat16)
    tiles, _ = fn.stat_tiles(N * g.Ho * g.Wo, K)
    part = torch.empty(tiles * 2 * K, device=dev)
    out = torch.empty(N, g.Ho, g.Wo, K, device=dev, dtype=torch.bfloat16)
    dx = torch.empty_like(x)
    gw = torch.empty(k, k, C, K, device=dev)
    M = N * H * H
    bnb = (x, torch.randn(C, device=dev) * 0.1, torch.rand(C, device=dev) + 0.5, sc, sh,
           torch.zeros((M // 64 + 1) * 2 * C, device=dev))
    bacc = torch.zeros(8 * 2 * C, device=dev, dtype=torch.float64)
    for _ in range(reps):
        if "fwd" in passes:
            fn.conv2d_fwd(x, w, s, stat_part=part, out=out, pre_scale=sc, pre_shift=sh)
        if "fwd_plain" in passes:
            fn.conv2d_fwd(x, w, s, out=out)
        if "fwd_stats" in passes:
            fn.conv2d_fwd(x, w, s, stat_part=part, out=out)
        if "dgrad" in passes:
            fn.conv2d_dgrad(dy, whwio, tuple(x.shape), s, out=dx)
        if "dgrad_bnb" in passes:
            fn.conv2d_dgrad(dy, whwio, tuple(x.shape), s, out=dx, bnb=bnb, bfin=[bacc])
        if "wgrad" in passes:
            fn.conv2d_wgrad(dy, x, k, k, s, grad_hwio=gw, pre_scale=sc, pre_shift=sh)
    torch.cuda.synchronize()
    print("ok", flush=True)


if __name__ == "__main__":
    main()
