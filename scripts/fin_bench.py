#!/usr/bin/env python3
"""Device time per launch of the BN finalize kernels (forward Welford combine and
backward sums) for the CIFAR / ImageNet partial counts, per kernel variant."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import distributed_tensorflow_resnet_amd as dtr  # noqa: E402
from conv_device_time import dev_time  # noqa: E402


def main():
    nat = dtr.native()
    dev = torch.device("cuda", 0)
    n = 200
    shapes = [(512, 16), (512, 32), (128, 64), (2048, 16), (1568, 64), (392, 128), (98, 256),
              (392, 512), (98, 1024), (25, 2048)]
    bufs = [torch.rand(64, device=dev) for _ in range(8)]
    for T, C in shapes:
        part = torch.rand(T * 2 * C, device=dev) + 0.1
        g = torch.rand(C, device=dev)
        outs = [torch.zeros(max(3 * C, 64), device=dev) for _ in range(8)]
        line = []
        # fp64 reference (Chan over the tiles): mean, rstd
        pm = part.view(T, 2, C).double()
        ref_mean = pm[:, 0].mean(0)
        ref_var = (pm[:, 1].sum(0) + 256 * ((pm[:, 0] - ref_mean) ** 2).sum(0)) / (T * 256)
        ref_rstd = (ref_var + 1e-5).rsqrt()
        ref_sg = pm[:, 0].sum(0)
        for v in (0, 2, 1):   # LDS tree, per-channel, auto
            nat.set_fin_version(v)
            p = nat.Plan()
            for _ in range(n):
                p.bn_finalize(part.data_ptr(), T, 256, T * 256, C, g.data_ptr(), g.data_ptr(),
                              outs[0].data_ptr(), outs[1].data_ptr(), 0.997, 1e-5, 1,
                              outs[2].data_ptr(), outs[3].data_ptr(), outs[4].data_ptr(),
                              outs[5].data_ptr())
            line.append(f"fwd v{v} {dev_time(p):.2f}")
            ref = [o.clone() for o in outs[2:6]]
            em = (ref[0][:C].double() - ref_mean).abs().max().item()
            er = ((ref[1][:C].double() - ref_rstd) / ref_rstd).abs().max().item()
            p = nat.Plan()
            for _ in range(n):
                p.bn_bwd_finalize(part.data_ptr(), T, T * 256, C, g.data_ptr(), g.data_ptr(),
                                  outs[6].data_ptr(), outs[7].data_ptr(), outs[2].data_ptr())
            line.append(f"bwd v{v} {dev_time(p):.2f}")
            eb = ((outs[7][:C].double() - ref_sg) / ref_sg).abs().max().item()
            line.append(f"(err mean {em:.1e} rstd {er:.1e} dbeta {eb:.1e})")
        p = nat.Plan()
        for _ in range(n):
            p.fill(bufs[0].data_ptr(), 64, 1.0)
        line.append(f"fill {dev_time(p):.2f}")
        print(f"T={T} C={C}: " + " | ".join(line), flush=True)
    nat.set_fin_version(1)


if __name__ == "__main__":
    main()
