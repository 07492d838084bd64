#!/usr/bin/env python3
"""Calibration: what the vendor library GEMM (torch.matmul -> hipBLASLt, bf16) reaches
on the plain-GEMM shapes of ImageNet ResNet-50's 1x1 convolutions (NHWC: M = N*H*W
pixels, K = Cin, N = Cout) against our fused implicit-GEMM conv kernel on the same
shapes (conv_gemm via ops/functional.py, no fusions).  TF/s = 2*M*N*K / time."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_tensorflow_resnet_amd.ops import functional as fn  # noqa: E402

SHAPES = [  # (batch, H, Cin, Cout) 1x1 stride-1 convs of RN50 at batch 128
    (128, 56, 64, 256), (128, 56, 256, 64), (128, 28, 128, 512), (128, 28, 512, 128),
    (128, 14, 256, 1024), (128, 14, 1024, 256), (128, 7, 512, 2048), (128, 7, 2048, 512)]


def timeit(fn_, reps=20):
    for _ in range(3):
        fn_()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn_()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    dev = torch.device("cuda", 0)
    print("| N,H,Cin,Cout | M | hipBLASLt us | TF/s | ours fwd us | TF/s | ours dgrad us | TF/s |")
    print("|---|---|---|---|---|---|---|---|")
    for N, H, C, K in SHAPES:
        M = N * H * H
        a = torch.randn(M, C, device=dev, dtype=torch.bfloat16)
        b = torch.randn(C, K, device=dev, dtype=torch.bfloat16)
        t_lib = timeit(lambda: torch.matmul(a, b))
        x = a.view(N, H, H, C)
        w = (torch.randn(K, 1, 1, C, device=dev) * 0.05).to(torch.bfloat16)     # OHWI
        t_fwd = timeit(lambda: fn.conv2d_fwd(x, w, 1))
        dy = torch.randn(N, H, H, K, device=dev, dtype=torch.bfloat16)
        wh = w.permute(1, 2, 3, 0).contiguous()                                  # HWIO
        t_dg = timeit(lambda: fn.conv2d_dgrad(dy, wh, (N, H, H, C), 1))
        fl = 2.0 * M * C * K
        print(f"| {N},{H},{C},{K} | {M} | {t_lib:.1f} | {fl / t_lib / 1e6:.0f} | {t_fwd:.1f} | "
              f"{fl / t_fwd / 1e6:.0f} | {t_dg:.1f} | {fl / t_dg / 1e6:.0f} |", flush=True)


if __name__ == "__main__":
    main()
