#!/usr/bin/env python3
"""Device-time ablation of the direct 3x3 conv (conv_direct.hip) on the CIFAR
ResNet-50 shapes, from native Plans of back-to-back launches (no Python per
launch; kernel boundary included).  Variants add the step's fusions one at a
time: BN+ReLU prologue (PRE), consumer-side BN finalize of the producer's
partials (PFIN), output BN statistics (STATS), residual; dgrad with BN-backward
sums (BNB) and the pending BN backward applied while staging (ABWD).  A one-
element fill gives the launch floor; the HBM floor is bytes / 5 TB/s.

  python scripts/ablate_direct.py [batch] [rounds]
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import distributed_tensorflow_resnet_amd as dtr  # noqa: E402
from distributed_tensorflow_resnet_amd.ops import functional as fn  # noqa: E402

BF = torch.bfloat16
SHAPES = [(32, 16), (16, 32), (8, 64)]   # (H = W, C = K)


def dev_time(plan):
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    plan.run(0, plan.size(), st.cuda_stream, st.cuda_stream)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / plan.size()


def main():
    nat = dtr.native(required=True)
    dev = torch.device("cuda", 0)
    batch = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    n = 20
    f1 = torch.zeros(1, device=dev)
    pfill = nat.Plan()
    for _ in range(n):
        pfill.fill(f1.data_ptr(), 1, 0.0)
    for H, C in SHAPES:
        N, K = batch, C
        g = fn.ConvGeom(N, H, H, C, K, 3, 3, 1)
        gl = g.as_list()
        M = N * H * H
        assert nat.conv_direct_covers(0, gl) if hasattr(nat, "conv_direct_covers") else True
        x = torch.randn(N, H, H, C, device=dev).to(BF)
        w = (torch.randn(K, 3, 3, C, device=dev) * 0.05).to(BF)
        wh = w.permute(1, 2, 3, 0).contiguous()
        y = torch.empty(N, H, H, K, device=dev, dtype=BF)
        res = torch.randn_like(y)
        dx = torch.empty_like(x)
        aout = torch.empty_like(x)
        vec = [torch.rand(C, device=dev) + 0.5 for _ in range(16)]
        T = -(-M // nat.conv_gemm_bm(M, K))
        part = torch.empty(T * 2 * K, device=dev)
        ppart = torch.rand(T * 2 * C, device=dev)   # the producer's partials (mean, M2)
        bpart = torch.empty(T * 2 * C, device=dev)
        p = {k: nat.Plan() for k in ("fwd", "pre", "pre+st", "pre+st+res", "pfin+st+res",
                                     "ACC:pre+st+res", "ACC:pfin+st+res", "dgrad", "bnb",
                                     "bnb+abwd", "ACC:bnb", "ACC:bnb+abwd")}
        rep = nat.bn_acc_rep()
        acc = torch.zeros(rep * 2 * max(C, K), dtype=torch.float64, device=dev)
        pacc = torch.rand(rep * 2 * C, dtype=torch.float64, device=dev) + M
        V = [v.data_ptr() for v in vec]
        pfin = [ppart.data_ptr(), T, M // T, M, V[0], V[1], V[2], V[3], V[4], V[5], V[6], V[7]]
        abwd = [x.data_ptr(), res.data_ptr(), V[8], V[9], V[10], V[11], V[12], ppart.data_ptr(),
                T, aout.data_ptr(), V[13], V[14], torch.empty(3 * C, device=dev).data_ptr()]
        bnb = [x.data_ptr(), V[2], V[3], V[4], V[5], bpart.data_ptr()]
        pfin_acc = [pacc.data_ptr(), 0xFFFFFFFF] + pfin[2:]
        abwd_acc = abwd[:7] + [pacc.data_ptr(), 0xFFFFFFFF] + abwd[9:]
        xs, ws, ys = x.data_ptr(), w.data_ptr(), y.data_ptr()
        sc, sh = V[4], V[5]
        for _ in range(n):
            p["fwd"].conv_gemm(0, xs, ws, ys, 0, 0, 0, 0, 0, 0, 0, 0, gl, [], [], [], [], [],
                               0.997, 1e-5, 1)
            p["pre"].conv_gemm(0, xs, ws, ys, 0, 0, sc, sh, 0, 0, 0, 0, gl, [], [], [], [], [],
                               0.997, 1e-5, 1)
            p["pre+st"].conv_gemm(0, xs, ws, ys, 0, 0, sc, sh, 0, 0, part.data_ptr(), 0, gl, [],
                                  [], [], [], [], 0.997, 1e-5, 1)
            p["pre+st+res"].conv_gemm(0, xs, ws, ys, 0, res.data_ptr(), sc, sh, 0, 0,
                                      part.data_ptr(), 0, gl, [], [], [], [], [], 0.997, 1e-5, 1)
            p["pfin+st+res"].conv_gemm(0, xs, ws, ys, 0, res.data_ptr(), sc, sh, 0, 0,
                                       part.data_ptr(), 0, gl, [], [], [], pfin, [], 0.997, 1e-5,
                                       1)
            p["ACC:pre+st+res"].conv_gemm(0, xs, ws, ys, 0, res.data_ptr(), sc, sh, 0, 0,
                                          part.data_ptr(), 0, gl, [], [acc.data_ptr()], [], [],
                                          [], 0.997, 1e-5, 1)
            p["ACC:pfin+st+res"].conv_gemm(0, xs, ws, ys, 0, res.data_ptr(), sc, sh, 0, 0,
                                           part.data_ptr(), 0, gl, [], [acc.data_ptr()], [],
                                           pfin_acc, [], 0.997, 1e-5, 1)
            p["ACC:bnb"].conv_gemm(1, res.data_ptr(), wh.data_ptr(), dx.data_ptr(), 0, 0, 0, 0, 0,
                                   0, 0, 0, gl, bnb, [], [acc.data_ptr()], [], [], 0.997, 1e-5, 1)
            p["ACC:bnb+abwd"].conv_gemm(1, res.data_ptr(), wh.data_ptr(), dx.data_ptr(), 0, 0, 0,
                                        0, 0, 0, 0, 0, gl, bnb, [], [acc.data_ptr()], [],
                                        abwd_acc, 0.997, 1e-5, 1)
            p["dgrad"].conv_gemm(1, res.data_ptr(), wh.data_ptr(), dx.data_ptr(), 0, 0, 0, 0, 0,
                                 0, 0, 0, gl, [], [], [], [], [], 0.997, 1e-5, 1)
            p["bnb"].conv_gemm(1, res.data_ptr(), wh.data_ptr(), dx.data_ptr(), 0, 0, 0, 0, 0, 0,
                               0, 0, gl, bnb, [], [], [], [], 0.997, 1e-5, 1)
            p["bnb+abwd"].conv_gemm(1, res.data_ptr(), wh.data_ptr(), dx.data_ptr(), 0, 0, 0, 0,
                                    0, 0, 0, 0, gl, bnb, [], [], [], abwd, 0.997, 1e-5, 1)
        ts = {k: [] for k in p}
        tf = []
        for _ in range(rounds):
            tf.append(dev_time(pfill))
            for k, plan in p.items():
                ts[k].append(dev_time(plan))
        hbm = 2.0 * M * C * 2 / 5e12 * 1e6
        line = " | ".join(f"{k} {statistics.median(v):5.1f}" for k, v in ts.items())
        print(f"N{N} H{H:2d} C{C:2d} T{T}: fill {statistics.median(tf):4.1f} | hbm-floor "
              f"{hbm:4.1f} | {line}  (us)", flush=True)


if __name__ == "__main__":
    main()
