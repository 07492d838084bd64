#!/usr/bin/env python3
"""BN+ReLU backward apply with the finalize fused in (bn_bwd_apply_acc): device time and
streamed bandwidth over the ImageNet ResNet-50 bs128 BN shapes.  Round 3 swept the grid
cap (256-2048 workgroups, then a tune key): 256 was never beaten, the key was removed
(profiles/bn_bwd_apply_bandwidth.md).   python3 scripts/bn_bwd_grid.py"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_tensorflow_resnet_amd.ops import functional as fn  # noqa: E402

BF = torch.bfloat16
# (rows M, channels C, residual-gradient add): the RN50 v2 BN backward applies at 128 images
SHAPES = [(401408, 64, False), (401408, 256, True), (100352, 128, False), (100352, 512, True),
          (25088, 256, False), (25088, 1024, True), (6272, 512, False), (6272, 2048, True)]


def main():
    caps = [256]
    nat = fn.native()
    dev = torch.device("cuda")
    st = torch.cuda.current_stream().cuda_stream
    print("| M | C | add | " + " | ".join(f"cap {c} us (TB/s)" for c in caps) + " |")
    print("|---|---|---|" + "---|" * len(caps))
    for M, C, add in SHAPES:
        dy = torch.randn(M, C, device=dev).to(BF)
        x = torch.randn(M, C, device=dev).to(BF)
        ad = torch.randn(M, C, device=dev).to(BF) if add else None
        dx = torch.empty(M, C, device=dev, dtype=BF)
        mean, rstd = torch.randn(C, device=dev) * 0.1, torch.rand(C, device=dev) + 0.5
        sc, sh = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
        acc = torch.randn(8 * 2 * C, device=dev, dtype=torch.float64)
        gamma = torch.rand(C, device=dev) + 0.5
        dg, db, coef = (torch.empty(C, device=dev), torch.empty(C, device=dev),
                        torch.empty(3 * C, device=dev))
        byts = M * C * 2 * (4 if add else 3)
        res = {c: [] for c in caps}
        for _ in range(3):
            for c in caps:
                if not nat.bn_bwd_apply_acc_fits(M, C):
                    continue
                f = lambda: nat.bn_bwd_apply_acc(  # noqa: E731
                    dy.data_ptr(), x.data_ptr(), mean.data_ptr(), rstd.data_ptr(), sc.data_ptr(),
                    sh.data_ptr(), [acc.data_ptr(), gamma.data_ptr(), dg.data_ptr(),
                                    db.data_ptr(), coef.data_ptr()],
                    ad.data_ptr() if add else 0, dx.data_ptr(), M, C, st)
                for _ in range(3):
                    f()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(20):
                    f()
                b.record()
                b.synchronize()
                res[c].append(a.elapsed_time(b) * 1e3 / 20)
        cells = []
        for c in caps:
            if res[c]:
                us = statistics.median(res[c])
                cells.append(f"{us:.1f} ({byts / us / 1e6:.2f})")
            else:
                cells.append("(not fused)")
        print(f"| {M} | {C} | {int(add)} | " + " | ".join(cells) + " |", flush=True)


if __name__ == "__main__":
    main()
