#!/usr/bin/env python3
"""Where the time of the narrow-K 1x1 dgrads goes (ImageNet RN50 bottleneck conv1 dgrads,
128 images, 1x MI355X): the implicit-GEMM dgrad alone, + BN-backward sums (fp64 accumulators
or per-tile partials), the separate streaming apply, and the streaming kernel's sums and
apply passes, each timed with HIP events (median of reps).  (The implicit-GEMM sums-only
and apply-epilogue passes of profiles/imagenet_bn_backward_fusion.md were removed.)

    python3 scripts/bap_probe.py [reps]
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
    print("| N,H,C(wide),K | MB wide | dgrad | +BNB acc | +BNB part | separate apply "
          "| dgrad+BNB+apply | stream sums | stream apply | stream 2-pass |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for (N, H, C, K) in [(128, 56, 256, 64), (128, 28, 512, 128), (128, 14, 1024, 256),
                         (128, 7, 2048, 512)]:
        M = N * H * H
        g = fn.ConvGeom(N, H, H, C, K, 1, 1, 1).as_list()
        dy = torch.randn(N, H, H, K, device=dev).to(BF)
        w = (torch.randn(1, 1, C, K, device=dev) / K ** 0.5).to(BF)
        x = torch.randn(N, H, H, C, device=dev).to(BF)
        add = torch.randn(N, H, H, C, device=dev).to(BF)
        out = torch.empty_like(x)
        dx = torch.empty_like(x)
        mean = torch.randn(C, device=dev) * 0.1
        rstd = torch.rand(C, device=dev) + 0.5
        gamma = torch.rand(C, device=dev) + 0.5
        sc, sh = gamma * rstd, torch.randn(C, device=dev) * 0.2
        bl = [x.data_ptr(), mean.data_ptr(), rstd.data_ptr(), sc.data_ptr(), sh.data_ptr()]
        part = torch.zeros((M // 64 + 1) * 2 * C, device=dev)
        bacc = torch.zeros(nat.bn_acc_rep() * 2 * C, device=dev, dtype=torch.float64)
        dgb, coef = torch.empty(2 * C, device=dev), torch.empty(3 * C, device=dev)
        nat.bn_bwd_finalize(bacc.data_ptr(), -1, M, C, gamma.data_ptr(), rstd.data_ptr(),
                            dgb.data_ptr(), dgb.data_ptr() + 4 * C, coef.data_ptr(), st)

        def dg(o, bnb, bfin, resid=0):
            nat.conv_gemm(1, dy.data_ptr(), w.data_ptr(), o, 0, resid, 0, 0, 0, 0, 0, 0, g,
                          bnb, [], bfin, [], [], 0.997, ref.BN_EPS, 1, st)

        t = {}
        t["dgrad"] = timed(lambda: dg(out.data_ptr(), [], []), reps)
        t["acc"] = timed(lambda: dg(out.data_ptr(), bl + [part.data_ptr()], [bacc.data_ptr()]), reps)
        t["part"] = timed(lambda: dg(out.data_ptr(), bl + [part.data_ptr()], []), reps)
        t["apply"] = timed(lambda: nat.bn_bwd_apply(
            out.data_ptr(), x.data_ptr(), mean.data_ptr(), rstd.data_ptr(), sc.data_ptr(),
            sh.data_ptr(), coef.data_ptr(), add.data_ptr(), dx.data_ptr(), M, C, st), reps)
        t["ss"] = t["sa"] = float("nan")
        if nat.bnd1x1_covers(M, C, K):
            base = [dy.data_ptr(), w.data_ptr(), x.data_ptr()]
            bnp = [mean.data_ptr(), rstd.data_ptr(), sc.data_ptr(), sh.data_ptr()]
            t["ss"] = timed(lambda: nat.bnd1x1(0, base + [0, 0] + bnp + [0, bacc.data_ptr()], M, C,
                                               K, st), reps)
            t["sa"] = timed(lambda: nat.bnd1x1(1, base + [add.data_ptr(), dx.data_ptr()] + bnp +
                                               [coef.data_ptr(), 0], M, C, K, st), reps)
        mb = M * C * 2 / 1e6
        print(f"| {N},{H},{C},{K} | {mb:.0f} | {t['dgrad']:.1f} | {t['acc']:.1f} | {t['part']:.1f} | "
              f"{t['apply']:.1f} | {t['acc'] + t['apply']:.1f} | {t['ss']:.1f} | "
              f"{t['sa']:.1f} | {t['ss'] + t['sa']:.1f} |", flush=True)


if __name__ == "__main__":
    main()
