"""Step time of the persistent CIFAR step with the native RCCL communicator at world 1
(the world > 1 plan shape on one GPU: slab reduces, bf16 casts, all-reduces, optimizer)
against the same engine without a communicator, with the buckets overlapping the backward
(tune persist_overlap=1) and after it (0).  Variants interleaved in one process, best of
`rounds`.  Usage:
    python scripts/comm_step_time.py [batch,...] [steps] [rounds]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_resnet_amd.models.spec import cifar_spec  # noqa: E402
from distributed_tensorflow_resnet_amd.train.engine import Engine, cifar_lr_schedule  # noqa: E402


def build(N, comm, overlap):
    os.environ["DTR_TUNE"] = f"persist_overlap={overlap}"
    kw = dict(native_comm=True, allreduce_dtype=os.environ.get("COMM_DTYPE", "bf16")) if comm else {}
    eng = Engine(cifar_spec(50), N, weight_decay=2e-4, lr_schedule=cifar_lr_schedule(),
                 device=torch.device("cuda", 0), use_graph=False, **kw)
    del os.environ["DTR_TUNE"]
    eng.fill_synthetic(0)
    for _ in range(20):
        eng.step()
    torch.cuda.synchronize()
    return eng


def main():
    batches = [int(b) for b in (sys.argv[1] if len(sys.argv) > 1 else "16,32").split(",")]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    for N in batches:
        engs = {"no comm": build(N, False, 1), "comm, buckets after the backward": build(N, True, 0),
                "comm, buckets overlapping the backward": build(N, True, 1)}
        best = {k: 1e9 for k in engs}
        for _ in range(rounds):
            for k, eng in engs.items():
                torch.cuda.synchronize()
                t = time.perf_counter()
                for _ in range(steps):
                    eng.step()
                torch.cuda.synchronize()
                best[k] = min(best[k], (time.perf_counter() - t) * 1e3 / steps)
        for k, eng in engs.items():
            assert not eng.persist_error(), k
            ops = eng.plan.names()
            print(f"bs{N} {k}: {best[k]:.4f} ms/step (persistent={eng.persist}, overlap="
                  f"{eng.persist_overlap}, {sum(1 for n in ops if n == 'all_reduce')} all-reduce "
                  f"op(s))", flush=True)
        del engs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
