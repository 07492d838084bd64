"""Same-process A/B of a native tune key on the persistent CIFAR step: one engine per
batch, the key flipped between timed windows with _C.tune_set (values interleaved, rounds
x values, best and median reported).

    python scripts/persist_tune_ab.py KEY v1,v2[,...] [batch,...] [steps] [rounds]
"""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import distributed_tensorflow_resnet_amd.train.engine as E  # noqa: E402
from distributed_tensorflow_resnet_amd.models.spec import cifar_spec  # noqa: E402


def main():
    key = sys.argv[1]
    vals = [int(v) for v in sys.argv[2].split(",")]
    batches = [int(b) for b in (sys.argv[3] if len(sys.argv) > 3 else "128,64,32,16").split(",")]
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 200
    rounds = int(sys.argv[5]) if len(sys.argv) > 5 else 3
    nat = E.native(required=True)
    dflt = {k: cur for k, _, _, cur in nat.tune_table()}[key]
    for N in batches:
        eng = E.Engine(cifar_spec(50), N, weight_decay=2e-4, lr_schedule=E.cifar_lr_schedule(),
                       device=torch.device("cuda", 0), use_graph=False, input_mode="cifar_u8")
        assert eng.persist, eng.persist_reason
        eng.fill_synthetic(0)
        res = {v: [] for v in vals}
        for v in vals:   # warm every variant
            nat.tune_set(key, v)
            for _ in range(10):
                eng.step()
        for _ in range(rounds):
            for v in vals:
                nat.tune_set(key, v)
                eng.step()
                torch.cuda.synchronize()
                t = time.perf_counter()
                for _ in range(steps):
                    eng.step()
                torch.cuda.synchronize()
                res[v].append((time.perf_counter() - t) * 1e3 / steps)
        nat.tune_set(key, dflt)
        assert not eng.persist_error()
        P = eng.prn
        for v in vals:
            print(f"bs{N} (P fwd/bwd {P.P_fwd}/{P.P}) {key}={v}: best {min(res[v]):.4f} "
                  f"median {statistics.median(res[v]):.4f} ms/step", flush=True)
        del eng
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
