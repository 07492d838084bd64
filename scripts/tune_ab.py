#!/usr/bin/env python3
"""Same-process A/B of one native tuning entry on the CIFAR RN50 step (MI355X discipline:
the variants interleaved in one process on one box; best and median of `rounds` x `steps`
per variant).  The entry is flipped with _C.tune_set between timed runs, so it must be read
at launch time (the persistent step's launchers read prn_shards / prn_poll2 per launch).

    python scripts/tune_ab.py KEY v1,v2[,...] [batch,...] [steps] [rounds]
"""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_resnet_amd.models.spec import cifar_spec  # noqa: E402
from distributed_tensorflow_resnet_amd.train.engine import Engine, cifar_lr_schedule  # noqa: E402


def main():
    key = sys.argv[1]
    vals = [int(v) for v in sys.argv[2].split(",")]
    batches = [int(b) for b in (sys.argv[3] if len(sys.argv) > 3 else "16,32,128").split(",")]
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 200
    rounds = int(sys.argv[5]) if len(sys.argv) > 5 else 5
    for N in batches:
        eng = Engine(cifar_spec(50), N, weight_decay=2e-4, lr_schedule=cifar_lr_schedule(),
                     device=torch.device("cuda", 0), use_graph=False, input_mode="cifar_u8")
        nat = eng.nat
        dflt = {t[0]: t[1] for t in nat.tune_table()}[key]
        eng.fill_synthetic(0)
        for _ in range(20):
            eng.step()
        torch.cuda.synchronize()
        times = {v: [] for v in vals}
        for _ in range(rounds):
            for v in vals:
                nat.tune_set(key, v)
                for _ in range(10):
                    eng.step()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(steps):
                    eng.step()
                torch.cuda.synchronize()
                times[v].append((time.perf_counter() - t0) / steps * 1e3)
        nat.tune_set(key, dflt)
        if eng.persist_error():
            raise SystemExit("a persistent barrier timed out")
        print(f"bs{N} {key}: " + "  ".join(
            f"{v}: best {min(t):.4f} med {statistics.median(t):.4f}" for v, t in times.items()),
            flush=True)


if __name__ == "__main__":
    main()
