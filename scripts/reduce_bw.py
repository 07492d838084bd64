#!/usr/bin/env python3
"""Bandwidth of the grouped split-K wgrad reduce (wgrad_reduce_grouped) on
ImageNet-like slab shapes vs torch.sum over the split axis (a streaming-read
reference of the same bytes)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import distributed_tensorflow_resnet_amd as dtr  # noqa: E402
from distributed_tensorflow_resnet_amd.train.engine import WGD_DTYPE, _ceil  # noqa: E402

SHAPES = [  # (splits, K, taps, C)
    (96, 64, 1, 256), (24, 64, 9, 64), (12, 128, 9, 128), (3, 512, 9, 512), (6, 1024, 1, 256),
    (12, 256, 1, 1024), (4, 2048, 1, 512),
]


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
    nat = dtr.native(required=True)
    dev = torch.device("cuda")
    st = torch.cuda.current_stream().cuda_stream
    for sp, K, taps, C in SHAPES:
        part = torch.randn(sp, K, taps * C, device=dev)
        grad = torch.empty(taps, C, K, device=dev)
        arr = np.zeros(1, dtype=WGD_DTYPE)
        arr[0] = (part.data_ptr(), grad.data_ptr(), sp, K, K, taps, C, C, 0)
        chunks = nat.wgrad_reduce_chunks(sp, K, taps, C) if hasattr(nat, "wgrad_reduce_chunks") \
            else _ceil(K * taps * C, 256)
        t = torch.from_numpy(arr.view(np.uint8).copy()).to(dev)
        us = timeit(lambda: nat.wgrad_reduce_grouped(t.data_ptr(), 1, chunks, 1.0, st))
        ref = part.sum(0).view(K, taps, C).permute(1, 2, 0)
        err = (grad - ref).abs().max().item()
        out = torch.empty(K, taps * C, device=dev)
        us_t = timeit(lambda: torch.sum(part, 0, out=out))
        gb = part.numel() * 4 / 1e9
        print(f"splits {sp:3d} K {K:4d} taps {taps} C {C:4d}: {gb*1e3:7.1f} MB | ours {us:7.1f} us "
              f"{gb/us*1e3:5.2f} TB/s | torch.sum {us_t:7.1f} us {gb/us_t*1e3:5.2f} TB/s | "
              f"max err {err:.1e}", flush=True)


if __name__ == "__main__":
    main()
