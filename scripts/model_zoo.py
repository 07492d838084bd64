#!/usr/bin/env python3
"""Every supported network of the reference (pre-activation ResNet v2: CIFAR 6n+2 depths
and the bottleneck CIFAR-50 of the headline, ImageNet ResNet-18 ... 200;
resnet_model_official.py:_get_block_sizes, resnet_model.py) trained on one GPU with the
bench's step (synthetic uint8 batch packed / augmented on the device every step,
random-init weights, SGD-momentum + weight decay, BN moving averages): ms/step, images/s,
peak device memory and the step path the engine chose.  One JSON line per model.

    python scripts/model_zoo.py [--steps 50] [--warmup 10] [--only imagenet_resnet50,...]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_tensorflow_resnet_amd.models.spec import build_spec  # noqa: E402
from distributed_tensorflow_resnet_amd.train.engine import (Engine, cifar_lr_schedule,  # noqa: E402
                                                            imagenet_lr_schedule)

ZOO = [("cifar10", 20, 128), ("cifar10", 32, 128), ("cifar10", 56, 128), ("cifar10", 110, 128),
       ("cifar10", 50, 128), ("imagenet", 18, 128), ("imagenet", 34, 128),
       ("imagenet", 50, 128), ("imagenet", 101, 128), ("imagenet", 152, 128),
       ("imagenet", 200, 128)]


def run(dataset, size, batch, steps, warmup, dev):
    cifar = dataset.startswith("cifar")
    spec = build_spec(dataset, size)
    eng = Engine(spec, batch, weight_decay=2e-4 if cifar else 1e-4,
                 lr_schedule=cifar_lr_schedule() if cifar else imagenet_lr_schedule(),
                 device=dev, seed=0, data_seed=1234,
                 input_mode="cifar_u8" if cifar else "imagenet_u8")
    eng.fill_synthetic(seed=0)
    torch.cuda.reset_peak_memory_stats(dev)
    for _ in range(warmup):
        eng.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    m = eng.metrics()
    path = ("persistent (P fwd/bwd = %d/%d)" % (eng.prn.P_fwd, eng.prn.P) if eng.persist
            else "per-layer plan")
    params = sum(s.numel for s in eng.params.train_slots)
    out = {"model": f"{dataset}_resnet{size}_v2", "batch": batch, "params_M": round(params / 1e6, 3),
           "ms_per_step": round(ms, 4), "images_per_sec": round(batch / ms * 1e3, 1),
           "peak_mem_gb": round(torch.cuda.max_memory_allocated(dev) / 2 ** 30, 2),
           "step_path": path, "loss": round(m["cross_entropy"], 4),
           "persist_error": eng.persist_error()}
    del eng
    torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    only = set(filter(None, a.only.split(",")))
    for dataset, size, batch in ZOO:
        name = f"{dataset.rstrip('10')}_resnet{size}"
        if only and name not in only:
            continue
        print(json.dumps(run(dataset, size, batch, a.steps, a.warmup, dev)), flush=True)


if __name__ == "__main__":
    main()
