#!/usr/bin/env python3
"""Achieved HBM bandwidth of the streaming BN kernels on ImageNet-sized tensors
(bn_bwd_apply with / without the residual-gradient add), vs a torch copy."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import distributed_tensorflow_resnet_amd as dtr  # noqa: E402

BF = torch.bfloat16


def timeit(f, iters=20):
    for _ in range(3):
        f()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        f()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    nat = dtr.native()
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream().cuda_stream
    for M, C, add in ((401408, 256, True), (401408, 256, False), (401408, 64, False),
                      (100352, 512, True), (6272, 2048, True)):
        dy = torch.randn(M, C, device=dev).to(BF)
        x = torch.randn(M, C, device=dev).to(BF)
        a = torch.randn(M, C, device=dev).to(BF) if add else None
        dx = torch.empty_like(x)
        p = [torch.rand(C, device=dev) for _ in range(4)]
        coef = torch.rand(3 * C, device=dev)

        def run():
            nat.bn_bwd_apply(dy.data_ptr(), x.data_ptr(), p[0].data_ptr(), p[1].data_ptr(),
                             p[2].data_ptr(), p[3].data_ptr(), coef.data_ptr(),
                             a.data_ptr() if add else 0, dx.data_ptr(), M, C, st)
        t = timeit(run)
        nbytes = M * C * 2 * (4 if add else 3)
        tc = timeit(lambda: dx.copy_(x))
        print(f"apply M={M} C={C} add={add}: {t:7.1f} us  {nbytes / t / 1e6:5.2f} TB/s | "
              f"torch copy {tc:6.1f} us {M * C * 4 / tc / 1e6:5.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
