#!/usr/bin/env python3
"""Sweep the split-K factor of conv_wgrad on CIFAR shapes: kernel vs reduce time."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_tensorflow_resnet_amd import native  # noqa: E402
from distributed_tensorflow_resnet_amd.ops import functional as fn  # noqa: E402


def t(f, it=30):
    for _ in range(3):
        f()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        f()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


nat = native()
dev = torch.device("cuda")
for (N, H, C, K, k, s) in [(128, 32, 16, 16, 3, 1), (128, 16, 32, 32, 3, 1), (128, 8, 64, 64, 3, 1),
                           (128, 56, 64, 64, 3, 1), (128, 14, 256, 1024, 1, 1)]:
    g = fn.ConvGeom(N, H, H, C, K, k, k, s)
    x = torch.randn(N, H, H, C, device=dev).to(torch.bfloat16)
    dy = torch.randn(N, g.Ho, g.Wo, K, device=dev).to(torch.bfloat16)
    P = N * g.Ho * g.Wo
    NT = k * k * C
    grad = torch.empty(k, k, C, K, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    d_sp, d_pps = nat.wgrad_pick_splits(g.as_list())
    line = f"N{N} H{H} C{C} K{K} k{k} (default splits {d_sp}):"
    for splits in (32, 64, 128, 256, 512, 1024, 2048):
        pps = -(-P // splits)
        pps = -(-pps // 64) * 64
        sp = -(-P // pps)
        part = torch.empty(sp * K * NT, device=dev)
        tw = t(lambda: nat.conv_wgrad(dy.data_ptr(), x.data_ptr(), 0, 0, part.data_ptr(),
                                      g.as_list(), sp, pps, st))
        tr = t(lambda: nat.wgrad_reduce(part.data_ptr(), grad.data_ptr(), sp, K, K, k * k, C, C,
                                        1.0, 0, st))
        line += f" | sp{sp}: {tw:.1f}+{tr:.1f}"
    print(line, flush=True)
