"""A/B of persistent-step choices that have no tune key, by patching the selection
functions before the engine is built (diagnostics): the forward's slices per image at
a given batch and the one-launch optimizer's tile budget.  Usage:
    python scripts/persist_variants.py [batch] [steps]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import distributed_tensorflow_resnet_amd.train.engine as E  # noqa: E402
import distributed_tensorflow_resnet_amd.train.persist as PS  # noqa: E402
from distributed_tensorflow_resnet_amd.models.spec import cifar_spec  # noqa: E402


def run(N, steps, label):
    eng = E.Engine(cifar_spec(50), N, weight_decay=2e-4, lr_schedule=E.cifar_lr_schedule(),
                   device=torch.device("cuda", 0), use_graph=False, input_mode="cifar_u8")
    eng.fill_synthetic(0)
    for _ in range(30):
        eng.step()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        t = time.perf_counter()
        for _ in range(steps):
            eng.step()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t) * 1e3 / steps)
    assert not eng.persist_error()
    print(f"bs{N} {label}: P fwd/bwd {eng.prn.P_fwd}/{eng.prn.P}: {best:.4f} ms/step", flush=True)
    del eng
    torch.cuda.empty_cache()


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    run(N, steps, "default")
    orig = PS.fwd_slices_for
    for p in (1, 2):
        PS.fwd_slices_for = lambda n, cus, override=-1, p=p: p
        run(N, steps, f"forward slices {p}")
    PS.fwd_slices_for = orig
    for loads in (1024, 4096, 8192):
        E.OPT_TILE_LOADS = loads
        run(N, steps, f"OPT_TILE_LOADS {loads}")
    E.OPT_TILE_LOADS = 2048


if __name__ == "__main__":
    main()
