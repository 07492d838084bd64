#!/usr/bin/env python3
"""Forward implicit-GEMM conv: device time per launch with each epilogue/prologue
fusion switched on separately (plain, +BN-ReLU prologue, +BN statistics,
+residual, all), on the ImageNet ResNet-50 shapes.  Shows where a fused forward
conv's time goes.   python scripts/fwd_fusion_cost.py [batch]"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import distributed_tensorflow_resnet_amd as dtr  # noqa: E402
from distributed_tensorflow_resnet_amd.ops import functional as fn  # noqa: E402

BF = torch.bfloat16
SHAPES = [(56, 64, 256, 1, 1), (56, 64, 64, 3, 1), (56, 256, 64, 1, 1), (28, 128, 128, 3, 1),
          (28, 128, 512, 1, 1), (28, 512, 128, 1, 1), (14, 256, 256, 3, 1),
          (14, 256, 1024, 1, 1), (14, 1024, 256, 1, 1), (7, 512, 512, 3, 1), (7, 512, 2048, 1, 1)]


def dev_time(plan):
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    plan.run(0, plan.size(), st.cuda_stream, st.cuda_stream)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / plan.size()


def main():
    nat = dtr.native()
    dev = torch.device("cuda", 0)
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    variants = {"plain": (0, 0, 0), "+pre": (1, 0, 0), "+stats": (0, 1, 0), "+res": (0, 0, 1),
                "pre+stats": (1, 1, 0), "all": (1, 1, 1)}
    for H, C, K, k, s in SHAPES:
        g = fn.ConvGeom(N, H, H, C, K, k, k, s)
        gl = g.as_list()
        M = N * g.Ho * g.Wo
        x = torch.randn(N, H, H, C, device=dev).to(BF)
        w = torch.randn(K, k, k, C, device=dev).to(BF)
        y = torch.empty(N, g.Ho, g.Wo, K, device=dev, dtype=BF)
        res = torch.randn_like(y)
        sc, sh = torch.rand(C, device=dev), torch.rand(C, device=dev)
        part = torch.empty(-(-M // nat.conv_gemm_bm(M, K)) * 2 * K, device=dev)
        plans = {}
        for name, (p, st, r) in variants.items():
            pl = nat.Plan()
            for _ in range(10):
                pl.conv_gemm(0, x.data_ptr(), w.data_ptr(), y.data_ptr(), 0,
                             res.data_ptr() if r else 0, sc.data_ptr() if p else 0,
                             sh.data_ptr() if p else 0, 0, 0, part.data_ptr() if st else 0, 0, gl,
                             [], [], [], [], [], 0.997, 1e-5, 1)
            plans[name] = pl
        ts = {n: [] for n in plans}
        for _ in range(5):
            for n, pl in plans.items():
                ts[n].append(dev_time(pl))
        mb = 2 * (x.numel() + y.numel()) / 1e6
        print(f"H{H:3d} C{C:5d} K{K:5d} k{k} ({mb:6.1f} MB): " +
              " | ".join(f"{n} {statistics.median(v):6.1f}" for n, v in ts.items()), flush=True)


if __name__ == "__main__":
    main()
