#!/usr/bin/env python3
"""The 1x1 forward convs of the ImageNet RN50 bottlenecks the streaming kernel covers (the
expanding K narrow -> C wide, the narrowing 256 -> 64 / 512 -> 128; BN+ReLU prologue, residual,
BN statistics into fp64 accumulators): the implicit-GEMM kernel vs the
streaming kernel (bn_fwd1x1.hip), HIP events, median of reps, 128 images.

    python3 scripts/fwd1x1_probe.py [reps]
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_tensorflow_resnet_amd.ops import functional as fn  # noqa: E402
from distributed_tensorflow_resnet_amd.ops import reference as ref  # noqa: E402

BF = torch.bfloat16


def timed(f, reps):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        f()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return statistics.median(ts)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    nat = fn.native()
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream().cuda_stream
    print("| N,H,K->C | PRE | MB moved | implicit GEMM us | TB/s | streaming us | TB/s |")
    print("|---|---|---|---|---|---|---|")
    for (H, K, C) in [(56, 64, 256), (28, 128, 512), (14, 256, 1024), (56, 256, 64), (28, 512, 128),
                      (56, 64, 64), (28, 256, 128)]:
        for pre in (True, False):
            N = 128
            M = N * H * H
            g = fn.ConvGeom(N, H, H, K, C, 1, 1, 1).as_list()
            x = torch.randn(N, H, H, K, device=dev).to(BF)
            w = (torch.randn(C, 1, 1, K, device=dev) / K ** 0.5).to(BF)
            res = torch.randn(N, H, H, C, device=dev).to(BF)
            out = torch.empty_like(res)
            sc, sh = torch.rand(K, device=dev) + 0.5, torch.randn(K, device=dev) * 0.2
            sacc = torch.zeros(nat.bn_acc_rep() * 2 * C, device=dev, dtype=torch.float64)
            dummy = torch.zeros(16, device=dev)
            ps, psh = (sc.data_ptr(), sh.data_ptr()) if pre else (0, 0)
            t0 = timed(lambda: nat.conv_gemm(0, x.data_ptr(), w.data_ptr(), out.data_ptr(), 0,
                                             res.data_ptr(), ps, psh, 0, 0, dummy.data_ptr(), 0, g,
                                             [], [sacc.data_ptr()], [], [], [], 0.997, ref.BN_EPS,
                                             1, st), reps)
            t1 = timed(lambda: nat.bnf1x1([x.data_ptr(), w.data_ptr(), res.data_ptr(),
                                           out.data_ptr(), ps, psh, sacc.data_ptr()], [], M, C, K,
                                          0.997, ref.BN_EPS, 1, st), reps)
            mb = (M * K + 2 * M * C) * 2 / 1e6 if C > K else (M * K + M * C) * 2 / 1e6
            print(f"| {N},{H},{K}->{C} | {pre} | {mb:.0f} | {t0:.1f} | {mb / t0:.2f} | "
                  f"{t1:.1f} | {mb / t1:.2f} |", flush=True)


if __name__ == "__main__":
    main()
