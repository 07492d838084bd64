#!/usr/bin/env python3
"""Soak run of the GPU training step: the bench configuration (synthetic uint8 batch,
random init, per-step augmentation / packing on the device) trained for a wall-clock
budget instead of a step count, checked every chunk:

* the persistent step's barrier-timeout flag and the logged metrics (Engine.metrics ->
  check_health raises PersistentStepError on a timed-out grid barrier);
* loss finite; per-chunk ms/step (min / max over the run: no drift, no stalls);
* world > 1: every rank's fp32 master weights and momentum bit-identical at the end
  (CRC32 of the bytes, compared through a max all-reduce of (crc, -crc)).

The batch is fixed (fill_synthetic), so the training loss falls as the model memorises
it under the random crops / flips -- a long-run learning signal, not an accuracy claim.

    python scripts/soak.py --seconds 300 --batch 128           # CIFAR RN50, 1 GPU
    DTR_DIST_BACKEND=gloo DTR_COMM_TRANSPORT=shm DTR_CU_PARTITION=2 \\
      python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
      scripts/soak.py --seconds 120 --batch 16                 # two ranks on CU halves
"""
import argparse
import json
import math
import os
import sys
import time
import zlib

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_tensorflow_resnet_amd.models.spec import build_spec  # noqa: E402
from distributed_tensorflow_resnet_amd.parallel.dist import (DistContext,  # noqa: E402
                                                             apply_cu_partition,
                                                             local_device_index)
from distributed_tensorflow_resnet_amd.train.engine import (Engine,  # noqa: E402
                                                            cifar_lr_schedule,
                                                            imagenet_lr_schedule)
from distributed_tensorflow_resnet_amd.train.persist import OVERLAP_RESERVE_CUS  # noqa: E402


def _crc(t: torch.Tensor) -> int:
    return zlib.crc32(t.detach().contiguous().view(torch.uint8).cpu().numpy().tobytes())


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="cifar10_resnet50")
    ap.add_argument("--batch", type=int, default=128, help="per-rank batch")
    ap.add_argument("--seconds", type=float, default=120.0)
    ap.add_argument("--chunk", type=int, default=2000, help="steps between checks")
    ap.add_argument("--out", default="gpurun_out/soak.jsonl")
    a = ap.parse_args()
    dataset, _, size = a.model.rpartition("_resnet")
    cifar = dataset.startswith("cifar")
    cu_mask = apply_cu_partition()
    torch.cuda.set_device(local_device_index())
    dev = torch.device("cuda", local_device_index())
    ctx = DistContext(device=dev, rccl_max_channels=OVERLAP_RESERVE_CUS if cifar else None)
    world, rank = ctx.world_size, ctx.rank
    spec = build_spec(dataset, int(size))
    eng = Engine(spec, a.batch, weight_decay=2e-4 if cifar else 1e-4,
                 lr_schedule=cifar_lr_schedule() if cifar else imagenet_lr_schedule(),
                 device=dev, dist_ctx=ctx, global_batch=a.batch * world, seed=0,
                 data_seed=1234 + rank, input_mode="cifar_u8" if cifar else "imagenet_u8")
    eng.broadcast_parameters(0)
    eng.fill_synthetic(seed=rank)
    path = "persistent" if eng.persist else f"per-layer ({eng.persist_reason})"
    out = open(a.out, "w") if rank == 0 else None
    if rank == 0:
        print(f"soak: {a.model} batch {a.batch}/rank x {world}, {path}, cu mask {cu_mask}",
              flush=True)
    eng.step()                       # the first step's loss: the untrained model
    loss0 = eng.metrics()["cross_entropy"]
    t_start = time.perf_counter()
    steps, chunks, rates, losses = 1, 0, [], []
    while True:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.chunk):
            eng.step()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        m = eng.metrics()            # raises PersistentStepError on a barrier timeout
        steps += a.chunk
        chunks += 1
        rates.append(dt / a.chunk * 1e3)
        losses.append(m["cross_entropy"])
        if not math.isfinite(m["cross_entropy"]):
            raise SystemExit(f"soak: non-finite loss at step {m['global_step']}")
        rec = {"step": m["global_step"], "ms_per_step": round(rates[-1], 4),
               "cross_entropy": round(m["cross_entropy"], 5), "precision": m["precision"],
               "lr": m["lr"]}
        if rank == 0:
            out.write(json.dumps(rec) + "\n")
            out.flush()
            if chunks % 10 == 1:
                print("soak:", json.dumps(rec), flush=True)
        # every rank stops after the same chunk: the slowest rank's clock decides
        el = torch.tensor([time.perf_counter() - t_start], dtype=torch.float64, device=dev)
        ctx.all_reduce_max(el)
        if float(el.item()) >= a.seconds:
            break
    same = True
    if world > 1:
        h = float(_crc(eng.params.master) ^ (_crc(eng.mom) << 1))
        t = torch.tensor([h, -h], dtype=torch.float64, device=dev)
        ctx.all_reduce_max(t)
        same = t[0].item() == -t[1].item()
    summary = {"soak": a.model, "batch_per_rank": a.batch, "world": world, "step_path": path,
               "steps": steps, "seconds": round(time.perf_counter() - t_start, 1),
               "ms_per_step_min": round(min(rates), 4), "ms_per_step_max": round(max(rates), 4),
               "ms_per_step_median": round(sorted(rates)[len(rates) // 2], 4),
               "loss_step1": round(loss0, 4),
               "loss_first_chunk": round(losses[0], 5), "loss_last": round(losses[-1], 5),
               "persist_error": eng.persist_error(), "replicas_identical": same}
    if rank == 0:
        out.write(json.dumps(summary) + "\n")
        out.close()
        print(json.dumps(summary), flush=True)
    return 0 if same and not summary["persist_error"] else 1


if __name__ == "__main__":
    sys.exit(main())
