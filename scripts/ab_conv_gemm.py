#!/usr/bin/env python3
"""In-process A/B of implicit-GEMM conv variants on the ImageNet ResNet-50 shapes.

Each (shape, pass) is timed with the pipelined FAST loop on and off
(`set_conv_pipeline`), interleaved over several rounds in ONE process (median
reported), from native Plans of back-to-back launches (device time per launch,
kernel boundary included).  Passes use the step's fusions: forward with the
BN+ReLU prologue, BN statistics and residual; dgrad with the BN-backward sums.

  python scripts/ab_conv_gemm.py [batch] [rounds]
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import distributed_tensorflow_resnet_amd as dtr  # noqa: E402
from distributed_tensorflow_resnet_amd.ops import functional as fn  # noqa: E402

BF = torch.bfloat16
SHAPES = [  # (H, C, K, k, s)
    (56, 64, 256, 1, 1), (56, 64, 64, 3, 1), (56, 256, 64, 1, 1), (56, 256, 128, 1, 1),
    (56, 128, 128, 3, 2), (28, 128, 128, 3, 1), (28, 128, 512, 1, 1), (28, 512, 128, 1, 1),
    (14, 256, 256, 3, 1), (14, 1024, 256, 1, 1), (14, 256, 1024, 1, 1),
    (7, 512, 512, 3, 1), (7, 2048, 512, 1, 1), (7, 512, 2048, 1, 1),
]


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
    batch = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    n = 10
    tot = {"fwd": [0.0, 0.0], "dgrad": [0.0, 0.0], "wgrad": [0.0, 0.0]}
    knob = os.environ.get("AB_KNOB", "pipe")   # pipe: FAST loop off/on; fuse: epilogue fusions
    only = os.environ.get("AB_SHAPES")   # e.g. "56,256,64,1,1;28,128,128,3,1"
    shapes = [tuple(int(v) for v in t.split(",")) for t in only.split(";")] if only else SHAPES
    for H, C, K, k, s in shapes:
        N = batch
        g = fn.ConvGeom(N, H, H, C, K, k, k, s)
        gl = g.as_list()
        Mf, Md = N * g.Ho * g.Wo, N * H * H
        x = torch.randn(N, H, H, C, device=dev).to(BF)
        w = torch.randn(K, k, k, C, device=dev).to(BF)
        wh = w.permute(1, 2, 3, 0).contiguous()
        y = torch.empty(N, g.Ho, g.Wo, K, device=dev, dtype=BF)
        res = torch.randn_like(y)
        dx = torch.empty_like(x)
        sc, sh = torch.rand(max(C, K), device=dev), torch.rand(max(C, K), device=dev)
        part = torch.empty(-(-Mf // nat.conv_gemm_bm(Mf, K)) * 2 * K, device=dev)
        bpart = torch.empty(-(-Md // nat.conv_gemm_bm(Md, C)) * 2 * C, device=dev)
        sp, pps = nat.wgrad_pick_splits(gl)
        wpart = torch.empty(sp * k * k * C * K, device=dev)
        pf, pd, pw = nat.Plan(), nat.Plan(), nat.Plan()
        pf0, pd0 = nat.Plan(), nat.Plan()   # AB_KNOB=fuse: no stats/residual/pre, no BNB
        for _ in range(n):
            pf0.conv_gemm(0, x.data_ptr(), w.data_ptr(), y.data_ptr(), 0, 0, 0, 0, 0, 0, 0, 0, gl,
                          [], [], [], [], [], 0.997, 1e-5, 1)
            pd0.conv_gemm(1, res.data_ptr(), wh.data_ptr(), dx.data_ptr(), 0, 0, 0, 0, 0, 0, 0, 0,
                          gl, [], [], [], [], [], 0.997, 1e-5, 1)
            pw.conv_wgrad(res.data_ptr(), x.data_ptr(), sc.data_ptr(), sh.data_ptr(),
                          wpart.data_ptr(), gl, sp, pps)
            pf.conv_gemm(0, x.data_ptr(), w.data_ptr(), y.data_ptr(), 0, res.data_ptr(),
                         sc.data_ptr(), sh.data_ptr(), 0, 0, part.data_ptr(), 0, gl, [], [], [],
                         [], [], 0.997, 1e-5, 1)
            pd.conv_gemm(1, res.data_ptr(), wh.data_ptr(), dx.data_ptr(), 0, 0, 0, 0, 0, 0, 0, 0,
                         gl, [x.data_ptr(), sc.data_ptr(), sh.data_ptr(), sc.data_ptr(),
                              sh.data_ptr(), bpart.data_ptr()], [], [], [], [], 0.997, 1e-5, 1)
        passes = (("fwd", pf), ("dgrad", pd), ("wgrad", pw))
        ts = {(p, v): [] for p, _ in passes for v in (0, 1)}
        for _ in range(rounds):
            for v in (0, 1):
                if knob == "fuse":   # 0 = plain GEMM epilogue, 1 = the step's fusions
                    for p, plan in (("fwd", pf if v else pf0), ("dgrad", pd if v else pd0),
                                    ("wgrad", pw)):
                        ts[(p, v)].append(dev_time(plan))
                    continue
                nat.set_conv_pipeline(v)
                for p, plan in passes:
                    ts[(p, v)].append(dev_time(plan))
        nat.set_conv_pipeline(1)
        line = []
        for p, _ in passes:
            a, b = statistics.median(ts[(p, 0)]), statistics.median(ts[(p, 1)])
            tot[p][0] += a
            tot[p][1] += b
            line.append(f"{p} {a:7.1f} -> {b:7.1f} us ({a / b:4.2f}x)")
        print(f"H{H:3d} C{C:5d} K{K:5d} k{k} s{s}: " + " | ".join(line), flush=True)
    for p, (a, b) in tot.items():
        print(f"total {p}: {a:.1f} -> {b:.1f} us ({a / b:.2f}x)")


if __name__ == "__main__":
    main()
