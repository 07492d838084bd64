#!/usr/bin/env python3
"""Is the step CPU-launch-bound?  Host issue time vs device time per step, eager
(two streams) vs hipGraph replay, for the CIFAR bench config."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_tensorflow_resnet_amd.models.spec import build_spec  # noqa: E402
from distributed_tensorflow_resnet_amd.train.engine import Engine, cifar_lr_schedule  # noqa: E402


def measure(eng, steps=200):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return (t1 - t0) / steps * 1e3, (t2 - t0) / steps * 1e3


def main():
    batch = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    dev = torch.device("cuda", 0)
    for graph, fork in ((False, True), (False, False), (True, False), (True, True)):
        os.environ["DTR_TUNE"] = f"fork_wgrad={int(bool(fork))}"
        eng = Engine(build_spec("cifar10", 50), batch, weight_decay=2e-4,
                     lr_schedule=cifar_lr_schedule(), device=dev, use_graph=graph)
        eng.fill_synthetic(0)
        if graph:
            eng.capture(warmup=2)
        for _ in range(10):
            eng.step()
        host, total = measure(eng)
        print(f"batch {batch} graph={graph} fork={eng.fork_wgrad}: host issue {host:.3f} ms/step, "
              f"total {total:.3f} ms/step, plan ops {eng.plan.size()}", flush=True)
        del eng
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
