"""Step time of the persistent CIFAR step with the native RCCL communicator at world 1
(the world > 1 plan shape on one GPU: grouped slab reduce, bf16 casts, all-reduce,
optimizer) against the same engine without a communicator.  Usage:
    python scripts/comm_step_time.py [batch] [steps]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_resnet_amd.models.spec import cifar_spec  # noqa: E402
from distributed_tensorflow_resnet_amd.train.engine import Engine, cifar_lr_schedule  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    dev = torch.device("cuda", 0)
    for comm in (False, True):
        kw = dict(native_comm=True, allreduce_dtype="bf16") if comm else {}
        eng = Engine(cifar_spec(50), N, weight_decay=2e-4, lr_schedule=cifar_lr_schedule(),
                     device=dev, use_graph=False, **kw)
        eng.fill_synthetic(0)
        for _ in range(30):
            eng.step()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(steps):
            eng.step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) * 1e3 / steps
        ops = eng.plan.names()
        print(f"bs{N} persistent={eng.persist} comm={comm}: {ms:.4f} ms/step, "
              f"{sum(1 for n in ops if n == 'all_reduce')} all-reduce op(s)", flush=True)
        assert not eng.persist_error()


if __name__ == "__main__":
    main()
