#!/usr/bin/env python3
"""Host cost of one plan op: tiny fill kernels, CIFAR-sized conv launches, and
cross-stream event record/wait pairs (what the forked wgrad stream costs)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import distributed_tensorflow_resnet_amd as dtr  # noqa: E402
from distributed_tensorflow_resnet_amd.ops import functional as fn  # noqa: E402


def host_time(plan, reps=5):
    st = torch.cuda.current_stream().cuda_stream
    side = torch.cuda.Stream().cuda_stream
    best = 1e9
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        plan.run(0, plan.size(), st, side)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        best = min(best, t1 - t0)
    return best, t2 - t0


def main():
    nat = dtr.native()
    dev = torch.device("cuda", 0)
    n = 1000
    buf = torch.empty(256, device=dev)
    p = nat.Plan()
    for _ in range(n):
        p.fill(buf.data_ptr(), 256, 1.0)
    h, tot = host_time(p)
    print(f"fill kernel: host {h / n * 1e6:.2f} us/launch (device+host {tot / n * 1e6:.2f})")
    # conv launch, CIFAR stage-3 shape at N=2 (tiny device work)
    g = fn.ConvGeom(2, 8, 8, 64, 64, 3, 3, 1)
    x = torch.randn(2, 8, 8, 64, device=dev).to(torch.bfloat16)
    w = torch.randn(64, 3, 3, 64, device=dev).to(torch.bfloat16)
    y = torch.empty(2, 8, 8, 64, device=dev, dtype=torch.bfloat16)
    p = nat.Plan()
    for _ in range(n):
        p.conv_gemm(0, x.data_ptr(), w.data_ptr(), y.data_ptr(), 0, 0, 0, 0, 0, 0, 0, 0,
                    g.as_list(), [], [], [], [], [], 0.997, 1e-5, 1)
    h, tot = host_time(p)
    print(f"conv launch: host {h / n * 1e6:.2f} us/launch (device+host {tot / n * 1e6:.2f})")
    # event record (main) + wait (side) pairs
    p = nat.Plan()
    for _ in range(n):
        e = p.new_event()
        p.record(e)
        p.use_stream(1)
        p.wait(e)
        p.use_stream(0)
    h, tot = host_time(p)
    print(f"event record+wait pair: host {h / n * 1e6:.2f} us/pair")
    # fork pattern: record, side wait, side kernel, main kernel
    p = nat.Plan()
    for _ in range(n // 2):
        e = p.new_event()
        p.record(e)
        p.use_stream(1)
        p.wait(e)
        p.fill(buf.data_ptr(), 256, 1.0)
        p.use_stream(0)
        p.fill(buf.data_ptr(), 256, 2.0)
    h, tot = host_time(p)
    print(f"fork pattern (record, wait, 2 kernels): host {h / (n // 2) * 1e6:.2f} us/iter")


if __name__ == "__main__":
    main()
