#!/usr/bin/env python3
"""Is the device ever waiting for the host?  Steady-state per-step host issue times
(perf_counter around eng.step()) of a bench-like loop, and the device step time
from HIP events.  If host issue per step << device time, the host runs ahead and
blocks only on queue/kernarg back-pressure; a host step time spread that matches
device gaps points at runtime pacing.  usage: host_pacing.py [batch] [steps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from distributed_tensorflow_resnet_amd.models.spec import build_spec  # noqa: E402
from distributed_tensorflow_resnet_amd.train.engine import Engine, cifar_lr_schedule  # noqa: E402


def main():
    batch = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    dev = torch.device("cuda", 0)
    eng = Engine(build_spec("cifar10", 50), batch, weight_decay=2e-4,
                 lr_schedule=cifar_lr_schedule(), device=dev)
    eng.fill_synthetic(0)
    for _ in range(30):
        eng.step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    host = np.zeros(steps)
    e0.record()
    t00 = time.perf_counter()
    for k in range(steps):
        t0 = time.perf_counter()
        eng.step()
        host[k] = time.perf_counter() - t0
    t_issue = time.perf_counter() - t00
    e1.record()
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t00
    dev_ms = e0.elapsed_time(e1) / steps
    q = np.percentile(host * 1e3, [10, 50, 90, 99])
    env = {k: v for k, v in os.environ.items() if k.startswith(("HSA_", "ROC_", "DEBUG_CLR", "GPU_"))}
    print(f"batch {batch}: device {dev_ms:.4f} ms/step | host issue total {t_issue * 1e3 / steps:.4f} "
          f"ms/step, p10/50/90/99 {q[0]:.3f}/{q[1]:.3f}/{q[2]:.3f}/{q[3]:.3f} ms | wall "
          f"{t_all * 1e3 / steps:.4f} ms/step | env {env}", flush=True)


if __name__ == "__main__":
    main()
