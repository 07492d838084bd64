#!/usr/bin/env python3
"""Calibration of the deep-K convolutions: what the vendor GEMM
(torch.matmul -> hipBLASLt, bf16) reaches on the plain GEMM of the same M, N, K as
ImageNet ResNet-50's 3x3 convolutions at batch 128, against our kernels on the real
conv (ops/functional.py: conv_gemm / conv_ring forward and dgrad, split-K weight
gradient + its deterministic reduce).  The library numbers are a ceiling for a GEMM
of that shape, not a conv: an im2col conv would add the 9x gather bytes on top.

  fwd / dgrad: M = N*Ho*Wo, N = Cout (dgrad: Cin), K = 9*Cin (dgrad: 9*Cout)
  wgrad:       M = Cout, N = 9*Cin, K = N*Ho*Wo   (dW = dy^T . im2col(x))

TF/s = 2*M*N*K / time (HIP events, median of 5 x 20 reps)."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_tensorflow_resnet_amd.ops import functional as fn  # noqa: E402

SHAPES = [  # (batch, H in, Cin, Cout, stride) 3x3 convs of RN50 at batch 128
    (128, 56, 64, 64, 1), (128, 28, 128, 128, 1), (128, 14, 256, 256, 1), (128, 7, 512, 512, 1),
    (128, 56, 128, 128, 2), (128, 28, 256, 256, 2), (128, 14, 512, 512, 2)]


def timeit(fn_, reps=20, rounds=5):
    for _ in range(3):
        fn_()
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn_()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / reps * 1e3)
    return statistics.median(ts)


def main():
    dev = torch.device("cuda", 0)
    rows = []
    if os.environ.get("CALIB_ONLY") == "wgrad":   # our weight gradients only (A/B sweeps)
        for N, H, C, K, s in SHAPES:
            Ho = H // s
            x = torch.randn(N, H, H, C, device=dev, dtype=torch.bfloat16)
            dy = torch.randn(N, Ho, Ho, K, device=dev, dtype=torch.bfloat16)
            t = timeit(lambda: fn.conv2d_wgrad(dy, x, 3, 3, s))
            fl = 2.0 * N * Ho * Ho * K * 9 * C
            print(f"| {N},{H},{C}->{K},/{s} | wgrad {t:.1f} us ({fl / t / 1e6:.0f} TF/s) |", flush=True)
        return
    for N, H, C, K, s in SHAPES:
        Ho = H // s
        M = N * Ho * Ho
        fl = 2.0 * M * K * 9 * C
        # vendor GEMMs of the same shapes
        a = torch.randn(M, 9 * C, device=dev, dtype=torch.bfloat16)
        b = torch.randn(9 * C, K, device=dev, dtype=torch.bfloat16)
        t_lib_f = timeit(lambda: torch.matmul(a, b))
        dyf = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        t_lib_w = timeit(lambda: torch.matmul(dyf.t(), a))
        # ours on the conv
        x = torch.randn(N, H, H, C, device=dev, dtype=torch.bfloat16)
        w = (torch.randn(K, 3, 3, C, device=dev) * 0.05).to(torch.bfloat16)       # OHWI
        t_fwd = timeit(lambda: fn.conv2d_fwd(x, w, s))
        dy = torch.randn(N, Ho, Ho, K, device=dev, dtype=torch.bfloat16)
        wh = w.permute(1, 2, 3, 0).contiguous()                                    # HWIO
        t_dg = timeit(lambda: fn.conv2d_dgrad(dy, wh, (N, H, H, C), s))
        t_wg = timeit(lambda: fn.conv2d_wgrad(dy, x, 3, 3, s))
        tf = lambda t: fl / t / 1e6  # noqa: E731
        rows.append(f"| {N},{H},{C}->{K},/{s} | {M} | {9 * C} | {t_lib_f:.1f} ({tf(t_lib_f):.0f}) | "
                    f"{t_fwd:.1f} ({tf(t_fwd):.0f}) | {t_dg:.1f} ({tf(t_dg):.0f}) | "
                    f"{t_lib_w:.1f} ({tf(t_lib_w):.0f}) | {t_wg:.1f} ({tf(t_wg):.0f}) |")
        print(rows[-1], flush=True)
    print("\n| N,H,Cin->Cout,/s | M | K (9Cin) | hipBLASLt fwd-shape us (TF/s) | ours fwd | ours dgrad "
          "| hipBLASLt wgrad-shape | ours wgrad (+reduce) |")
    print("|---|---|---|---|---|---|---|---|")
    print("\n".join(rows))


if __name__ == "__main__":
    main()
