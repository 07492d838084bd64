#!/usr/bin/env python3
"""Headline benchmark: steps/sec of the reference's flagship training step.

BASELINE.json metric: "steps/sec (global_batch=128 CIFAR-10 / 1024 ImageNet)
ResNet-50 at 1/2/4/8 MI355X".  Default config = CIFAR-10 ResNet-50 v2 (6n+2,
n=8; 758,618 params), global batch 128 split over the N ranks (strong scaling),
bf16 compute / fp32 master weights, synthetic data (random uint8 CIFAR records
augmented on the device every step: pad-4/crop/flip/standardize), random-init
weights.  One full training step is timed: forward, backward, RCCL gradient
all-reduce (N>1), SGD-momentum + weight-decay update, BN moving averages.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--model cifar_resnet50]
  torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Rank 0 prints ONE JSON line.  `--model imagenet_resnet50` measures BASELINE
config 4 (128 images per GPU, weak scaling, baseline 0.93 stp/s).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

MODELS = {
    # name: (dataset, size, batch, batch_is_global, baseline stp/s, baseline source)
    "cifar_resnet50": ("cifar10", 50, 128, True, 21.82, "README.md:16-22 (4x Titan Xp, Horovod)"),
    "cifar_resnet20": ("cifar10", 20, 128, True, None, None),
    "imagenet_resnet50": ("imagenet", 50, 128, False, 0.93, "README.md:39-44 (8 P100, 8ps-8wk)"),
    "imagenet_resnet101": ("imagenet", 101, 256, False, None, None),
}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--model", default="cifar_resnet50", choices=sorted(MODELS))
    ap.add_argument("--batch", type=int, default=None,
                    help="global batch (cifar) or per-GPU batch (imagenet)")
    ap.add_argument("--graph", action="store_true",
                    help="capture the step in a hipGraph (single stream); default: eager native "
                         "plan with weight gradients on a second stream (measured faster)")
    ap.add_argument("--no-graph", action="store_true", help="(default; kept for compatibility)")
    ap.add_argument("--bucket-mb", type=float, default=0.0,
                    help="all-reduce bucket size (MiB); 0 = auto (~4 buckets, <= 25 MiB)")
    ap.add_argument("--allreduce-dtype", default="fp32", choices=("fp32", "bf16"),
                    help="gradient all-reduce precision (bf16 halves the xGMI bytes)")
    ap.add_argument("--roctx", action="store_true",
                    help="wrap each step's phases in roctx ranges (rocprofv3 --marker-trace)")
    args = ap.parse_args(argv)
    if args.roctx:
        os.environ["DTR_ROCTX"] = "1"

    import torch

    from distributed_tensorflow_resnet_amd.models.spec import build_spec
    from distributed_tensorflow_resnet_amd.parallel.dist import DistContext, local_device_index
    from distributed_tensorflow_resnet_amd.train.engine import (Engine, cifar_lr_schedule,
                                                                imagenet_lr_schedule)

    dataset, size, batch, is_global, baseline, _src = MODELS[args.model]
    if args.batch:
        batch = args.batch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            print("bench.py: --gpus > 1 must be launched with torchrun", file=sys.stderr)
            return 2
    local_rank = local_device_index()
    torch.cuda.set_device(local_rank)
    device = torch.device("cuda", local_rank)
    ctx = DistContext(device=device)
    if is_global:
        if batch % world:
            raise SystemExit(f"global batch {batch} not divisible by {world}")
        per_rank, global_batch = batch // world, batch
    else:
        per_rank, global_batch = batch, batch * world

    spec = build_spec(dataset, size)
    sched = cifar_lr_schedule() if dataset.startswith("cifar") else imagenet_lr_schedule()
    wd = 2e-4 if dataset.startswith("cifar") else 1e-4
    use_graph = bool(args.graph) and not args.no_graph
    eng = Engine(spec, per_rank, weight_decay=wd, lr_schedule=sched, device=device,
                 dist_ctx=ctx, global_batch=global_batch, bucket_mb=args.bucket_mb,
                 seed=0, data_seed=1234 + ctx.rank, use_graph=use_graph,
                 allreduce_dtype=args.allreduce_dtype)
    eng.broadcast_parameters(0)
    eng.fill_synthetic(seed=ctx.rank)

    done = 0
    if use_graph:
        done = eng.capture(warmup=min(2, max(args.warmup, 1)))
    for _ in range(max(args.warmup - done, 0)):
        eng.step()
    torch.cuda.synchronize()
    ctx.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.step()
    torch.cuda.synchronize()
    ctx.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    ctx.all_reduce_max(t)
    elapsed = float(t.item())
    m = eng.metrics()
    sps = args.steps / elapsed
    if ctx.is_chief:
        out = {
            "metric": "steps/sec (global_batch=128 CIFAR-10 / 1024 ImageNet) ResNet-50 at 1/2/4/8 MI355X",
            "value": round(sps, 3),
            "unit": "steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * elapsed / args.steps, 4),
            "higher_is_better": True,
            "scaling": "strong" if is_global else "weak",
            "vs_baseline": round(sps / baseline, 3) if baseline else None,
            "dtype": "bf16",
            "data": "synthetic (random uint8 images, on-device augmentation each step), random-init weights",
            "config": {
                "model": f"resnet{size}_v2_{dataset}",
                "global_batch": global_batch,
                "per_gpu_batch": per_rank,
                "seq_len": None,
                "image_size": spec.image_h,
                "parallelism": f"dp{world}",
                "graph": use_graph,
                "wgrad_stream": eng.fork_wgrad,
                "allreduce_dtype": args.allreduce_dtype,
            },
            "images_per_sec": round(sps * global_batch, 1),
            "final_loss": round(m["cross_entropy"], 4),
        }
        print(json.dumps(out), flush=True)
    ctx.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
