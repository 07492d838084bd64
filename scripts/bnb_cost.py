#!/usr/bin/env python3
"""What the BN-backward sums epilogue (BNB: read the BN input x, relu mask, two column sums,
fp64 accumulator atomics) costs each ImageNet RN50 dgrad that carries it: the dgrad alone
vs with BNB, HIP events, median of reps (1x MI355X, 128 images).

    python3 scripts/bnb_cost.py [reps]
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_tensorflow_resnet_amd.ops import functional as fn  # noqa: E402
from distributed_tensorflow_resnet_amd.ops import reference as ref  # noqa: E402

BF = torch.bfloat16
# dgrads that emit BN-backward sums: (H_in, Cin = dgrad output channels, Cout, k, s, per step)
SHAPES = [(56, 64, 256, 1, 1, 3), (56, 64, 64, 3, 1, 3), (56, 256, 64, 1, 1, 1),
          (56, 128, 128, 3, 2, 1), (28, 128, 512, 1, 1, 4), (28, 128, 128, 3, 1, 3),
          (28, 256, 256, 3, 2, 1), (14, 256, 1024, 1, 1, 6), (14, 256, 256, 3, 1, 5),
          (14, 1024, 256, 1, 1, 5), (14, 512, 512, 3, 2, 1), (7, 512, 2048, 1, 1, 3),
          (7, 512, 512, 3, 1, 2), (7, 2048, 512, 1, 1, 2)]


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
    N = 128
    print("| H,Cin<-Cout,k,s | x/step | ring | dgrad us | +BNB us | BNB cost us | x MB | step ms "
          "| streaming +BNB us |")
    print("|---|---|---|---|---|---|---|---|---|")
    tot = 0.0
    for (H, C, K, k, s, n) in SHAPES:
        g = fn.ConvGeom(N, H, H, C, K, k, k, s)
        M = N * H * H
        dy = torch.randn(N, g.Ho, g.Wo, K, device=dev).to(BF)
        w = (torch.randn(k, k, C, K, device=dev) / (k * k * K) ** 0.5).to(BF)
        x = torch.randn(N, H, H, C, device=dev).to(BF)
        out = torch.empty_like(x)
        mean, rstd = torch.randn(C, device=dev) * 0.1, torch.rand(C, device=dev) + 0.5
        sc, sh = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.2
        part = torch.zeros((M // 64 + 1) * 2 * C, device=dev)
        bacc = torch.zeros(nat.bn_acc_rep() * 2 * C, device=dev, dtype=torch.float64)
        bl = [x.data_ptr(), mean.data_ptr(), rstd.data_ptr(), sc.data_ptr(), sh.data_ptr(),
              part.data_ptr()]

        def dg(bnb, bfin):
            nat.conv_gemm(1, dy.data_ptr(), w.data_ptr(), out.data_ptr(), 0, 0, 0, 0, 0, 0, 0, 0,
                          g.as_list(), bnb, [], bfin, [], [], 0.997, ref.BN_EPS, 1, st)
        t0 = timed(lambda: dg([], []), reps)
        t1 = timed(lambda: dg(bl, [bacc.data_ptr()]), reps)
        ring = nat.conv_ring_covers(1, g.as_list())
        t2 = float("nan")
        if k == 1 and s == 1 and nat.bnd1x1_covers(M, C, K):
            t2 = timed(lambda: nat.bnd1x1(2, [dy.data_ptr(), w.data_ptr(), x.data_ptr(), 0,
                                              out.data_ptr()] + bl[1:5] + [0, bacc.data_ptr()],
                                          M, C, K, st), reps)
        tot += n * (t1 - t0)
        print(f"| {H},{C}<-{K},{k},{s} | {n} | {ring} | {t0:.1f} | {t1:.1f} | {t1 - t0:.1f} | "
              f"{M * C * 2 / 1e6:.0f} | {n * (t1 - t0) / 1e3:.3f} | {t2:.1f} |", flush=True)
    print(f"\nBNB epilogue cost over the step's dgrads: {tot / 1e3:.3f} ms")


if __name__ == "__main__":
    main()
