"""Same-process A/B of ENGINE tune settings on the persistent CIFAR step: one engine per
(batch, setting), built under DTR_TUNE=<setting>, timed interleaved (rounds x settings),
best and median reported.

    python scripts/persist_engine_ab.py "setA;setB[;...]" [batch,...] [steps] [rounds]
e.g.  python scripts/persist_engine_ab.py "persist_head_in_bwd=0;persist_head_in_bwd=1" 128,16
"""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import distributed_tensorflow_resnet_amd.train.engine as E  # noqa: E402
from distributed_tensorflow_resnet_amd.models.spec import cifar_spec  # noqa: E402


def build(N, setting):
    old = os.environ.get("DTR_TUNE")
    os.environ["DTR_TUNE"] = setting
    try:
        eng = E.Engine(cifar_spec(50), N, weight_decay=2e-4, lr_schedule=E.cifar_lr_schedule(),
                       device=torch.device("cuda", 0), use_graph=False, input_mode="cifar_u8")
    finally:
        if old is None:
            del os.environ["DTR_TUNE"]
        else:
            os.environ["DTR_TUNE"] = old
    assert eng.persist, eng.persist_reason
    eng.fill_synthetic(0)
    for _ in range(20):
        eng.step()
    torch.cuda.synchronize()
    return eng


def main():
    settings = sys.argv[1].split(";")
    batches = [int(b) for b in (sys.argv[2] if len(sys.argv) > 2 else "128,16").split(",")]
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    for N in batches:
        engs = {s: build(N, s) for s in settings}
        res = {s: [] for s in settings}
        for _ in range(rounds):
            for s, eng in engs.items():
                eng.step()
                torch.cuda.synchronize()
                t = time.perf_counter()
                for _ in range(steps):
                    eng.step()
                torch.cuda.synchronize()
                res[s].append((time.perf_counter() - t) * 1e3 / steps)
        for s, eng in engs.items():
            assert not eng.persist_error(), s
            print(f"bs{N} [{s}]: best {min(res[s]):.4f} median {statistics.median(res[s]):.4f} "
                  f"ms/step ({len(eng.plan.names())} plan ops)", flush=True)
        del engs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
