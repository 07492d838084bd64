#!/usr/bin/env python3
"""Gradient all-reduce vs backward overlap on ONE GPU, at the queue level.

The training plan's bucket all-reduces run on the comm stream (stream 2) while the
main and side streams continue the backward (train/engine.py _emit_allreduce).  On a
single GPU there is no peer, so the all-reduce itself is stood in for by the native
loopback transport (csrc/comm.h: the bucket scaled in place on the comm stream),
with the bf16 exchange's cast kernels around it -- the same comm-stream ops, events
and issue thread as RCCL.  Run under rocprofv3 --kernel-trace, the trace shows which
hardware queue each stream's kernels land on (GPU_MAX_HW_QUEUES = 4 on the box) and
whether comm-stream kernels overlap compute kernels in time; scripts/overlap_summary.py
reads it.  Prints one JSON line with phase_ms (allreduce_exposed) and the comm info.

    rocprofv3 --kernel-trace -d gpurun_out/prof_overlap -- \\
        python3 scripts/comm_overlap.py --model imagenet_resnet50 --batch 128
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import distributed_tensorflow_resnet_amd as dtr  # noqa: E402
from distributed_tensorflow_resnet_amd.models.spec import build_spec  # noqa: E402
from distributed_tensorflow_resnet_amd.train.engine import (Engine, cifar_lr_schedule,  # noqa: E402
                                                            imagenet_lr_schedule)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="imagenet_resnet50")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--allreduce-dtype", default="bf16")
    ap.add_argument("--bucket-mb", type=float, default=0.0)
    a = ap.parse_args()
    ds = "cifar10" if a.model.startswith("cifar") else "imagenet"
    size = int(a.model.rsplit("resnet", 1)[1])
    spec = build_spec(ds, size)
    dev = torch.device("cuda", 0)
    sched = cifar_lr_schedule() if ds == "cifar10" else imagenet_lr_schedule()
    eng = Engine(spec, a.batch, weight_decay=1e-4, lr_schedule=sched, device=dev,
                 comm=dtr.native().Comm.loopback(1.0), allreduce_dtype=a.allreduce_dtype,
                 bucket_mb=a.bucket_mb or None)
    eng.fill_synthetic(0)
    for _ in range(a.warmup):
        eng.step()
    torch.cuda.synchronize()
    for _ in range(a.steps):
        eng.step()
    torch.cuda.synchronize()
    ph = [eng.step_timed() for _ in range(5)]
    out = {k: round(sum(p[k] for p in ph) / len(ph), 4) for k in ph[0]}
    print(json.dumps({"model": a.model, "batch": a.batch, "phase_ms": out,
                      "comm": eng.comm_info(), "streams": {
                          "main": torch.cuda.current_stream().cuda_stream,
                          "side": eng.side.cuda_stream, "comm": eng.comm_stream.cuda_stream}}),
          flush=True)


if __name__ == "__main__":
    main()
