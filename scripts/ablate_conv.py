#!/usr/bin/env python3
"""Ablation timing of the conv kernels on the CIFAR shapes: mainloop alone vs
with the fused BN prologue (PRE), the Welford epilogue (STATS), the residual
add, and dgrad with the fused BN-backward sums (BNB).  One process, interleaved
repeats, median of 5 (cdna_hip_programming.md §5.4 rule 24)."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_tensorflow_resnet_amd.ops import functional as fn  # noqa: E402

SHAPES = [("c16_3x3", 128, 32, 16, 16, 3, 1), ("c16_1x1", 128, 32, 16, 16, 1, 1),
          ("c32_3x3", 128, 16, 32, 32, 3, 1), ("c64_3x3", 128, 8, 64, 64, 3, 1),
          ("c16_3x3_b32", 32, 32, 16, 16, 3, 1), ("c64_3x3_b32", 32, 8, 64, 64, 3, 1)]


ITERS = int(os.environ.get("ABL_ITERS", "50"))
REPS = int(os.environ.get("ABL_REPS", "5"))


def t_us(f, iters=None):
    iters = iters or ITERS
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    f()
    s.record()
    for _ in range(iters):
        f()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    dev = torch.device("cuda")
    for name, N, H, C, K, k, s in SHAPES:
        g = fn.ConvGeom(N, H, H, C, K, k, k, s)
        x = torch.randn(N, H, H, C, device=dev).to(torch.bfloat16)
        w = (torch.randn(K, k, k, C, device=dev) * 0.05).to(torch.bfloat16)
        wh = w.permute(1, 2, 3, 0).contiguous()
        sc = torch.rand(C, device=dev) + 0.5
        sh = torch.randn(C, device=dev) * 0.1
        out = torch.empty(N, g.Ho, g.Wo, K, device=dev, dtype=torch.bfloat16)
        res = torch.randn_like(out)
        tiles, _ = fn.stat_tiles(N * g.Ho * g.Wo, K)
        part = torch.empty(tiles * 2 * K, device=dev)
        dy = torch.randn_like(out)
        dx = torch.empty_like(x)
        mean = torch.zeros(C, device=dev)
        rstd = torch.ones(C, device=dev)
        tiles_b, _ = fn.stat_tiles(N * H * H, C)
        bpart = torch.empty(tiles_b * 2 * C, device=dev)
        gw = torch.empty(k, k, C, K, device=dev)
        var = {
            "fwd": lambda: fn.conv2d_fwd(x, w, s, out=out),
            "fwd+pre": lambda: fn.conv2d_fwd(x, w, s, out=out, pre_scale=sc, pre_shift=sh),
            "fwd+stats": lambda: fn.conv2d_fwd(x, w, s, out=out, stat_part=part),
            "fwd+pre+stats": lambda: fn.conv2d_fwd(x, w, s, out=out, pre_scale=sc, pre_shift=sh,
                                                   stat_part=part),
            "fwd+pre+res+stats": lambda: fn.conv2d_fwd(x, w, s, out=out, pre_scale=sc,
                                                       pre_shift=sh, residual=res, stat_part=part),
            "dgrad": lambda: fn.conv2d_dgrad(dy, wh, tuple(x.shape), s, out=dx),
            "dgrad+bnb": lambda: fn.conv2d_dgrad(dy, wh, tuple(x.shape), s, out=dx,
                                                 bnb=(x, mean, rstd, sc, sh, bpart)),
            "wgrad": lambda: fn.conv2d_wgrad(dy, x, k, k, s, grad_hwio=gw),
            "wgrad+pre": lambda: fn.conv2d_wgrad(dy, x, k, k, s, grad_hwio=gw, pre_scale=sc,
                                                 pre_shift=sh),
            "empty": lambda: torch.cuda._sleep(0),
        }
        samples = {kk: [] for kk in var}
        for _ in range(REPS):
            for kk, f in var.items():
                samples[kk].append(t_us(f))
        line = " | ".join(f"{kk} {statistics.median(v):6.1f}" for kk, v in samples.items())
        print(f"{name:12s} M={N*g.Ho*g.Wo:6d}: {line}", flush=True)


if __name__ == "__main__":
    main()
