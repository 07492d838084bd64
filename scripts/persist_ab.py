"""Same-process A/B of the persistent CIFAR step's barrier / slicing choices (MI355X
discipline: variants interleaved in one process on one box, rounds x variants, best and
median reported).  Variants: the arrival-counter shards (native tune prn_shards, flipped
between steps with _C.tune_set) x the forward's slices per image (default vs the
alternative, patched into train/persist.fwd_slices_for before each engine is built).

    python scripts/persist_ab.py [batch,...] [steps] [rounds]
"""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import distributed_tensorflow_resnet_amd.train.engine as E  # noqa: E402
import distributed_tensorflow_resnet_amd.train.persist as PS  # noqa: E402
from distributed_tensorflow_resnet_amd.models.spec import cifar_spec  # noqa: E402


def build(N, p_fwd=None):
    orig = PS.fwd_slices_for
    if p_fwd is not None:
        PS.fwd_slices_for = lambda n, cus, override=-1: p_fwd
    try:
        eng = E.Engine(cifar_spec(50), N, weight_decay=2e-4, lr_schedule=E.cifar_lr_schedule(),
                       device=torch.device("cuda", 0), use_graph=False, input_mode="cifar_u8")
    finally:
        PS.fwd_slices_for = orig
    assert eng.persist, eng.persist_reason
    eng.fill_synthetic(0)
    for _ in range(20):
        eng.step()
    torch.cuda.synchronize()
    return eng


def timed(eng, steps):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        eng.step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) * 1e3 / steps


def main():
    batches = [int(b) for b in (sys.argv[1] if len(sys.argv) > 1 else "128,64,32,16").split(",")]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    nat = E.native(required=True)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    for N in batches:
        engs = {"fwd P auto": build(N)}
        pa = engs["fwd P auto"].prn.P_fwd
        alt = 2 if pa == 1 else 1
        if N * alt <= cus:
            engs[f"fwd P {alt}"] = build(N, alt)
        res = {}
        for _ in range(rounds):
            for shards in (1, 8):
                nat.tune_set("prn_shards", shards)
                for name, eng in engs.items():
                    eng.step()
                    res.setdefault((shards, name), []).append(timed(eng, steps))
        nat.tune_set("prn_shards", 8)
        for name, eng in engs.items():
            assert not eng.persist_error(), name
        for (shards, name), v in sorted(res.items()):
            P = engs[name].prn
            print(f"bs{N} shards {shards} {name} (P fwd/bwd {P.P_fwd}/{P.P}): "
                  f"best {min(v):.4f} median {statistics.median(v):.4f} ms/step", flush=True)
        del engs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
