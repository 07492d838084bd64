#!/usr/bin/env python3
"""Headline benchmark: steps/sec of the reference's flagship training step.

BASELINE.json metric: "steps/sec (global_batch=128 CIFAR-10 / 1024 ImageNet)
ResNet-50 at 1/2/4/8 MI355X".  Default config = CIFAR-10 ResNet-50 v2 (6n+2,
n=8; 758,618 params), global batch 128 split over the N ranks (strong scaling),
bf16 compute / fp32 master weights, synthetic data (random uint8 CIFAR records
augmented on the device every step: pad-4/crop/flip/standardize), random-init
weights.  One full training step is timed: forward, backward, RCCL gradient
all-reduce (N>1, native communicator on a comm stream overlapping backward),
SGD-momentum + weight-decay update, BN moving averages.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--model cifar_resnet50]
  torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Without torchrun, `--gpus N` (N > 1) spawns the N rank processes itself before
anything touches the GPU (env RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR /
MASTER_PORT, as torchrun sets them) and relays rank 0's line; it fails if any
rank fails.  Rank 0 prints ONE JSON line.  `--model imagenet_resnet50` measures
BASELINE config 4 (128 images per GPU, weak scaling, baseline 0.93 stp/s),
`--model imagenet_resnet101` config 5 (256 per GPU).

`--device cpu` runs the fp32 PyTorch CPU trainer (gloo for N > 1): a plumbing
check of this contract for hosts without a GPU, never a headline number.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

MODELS = {
    # name: (dataset, size, batch, batch_is_global, headline baseline stp/s, its source)
    "cifar_resnet50": ("cifar10", 50, 128, True, 21.82, "README.md:16-22 (4x Titan Xp, Horovod)"),
    "cifar_resnet20": ("cifar10", 20, 128, True, None, None),
    "imagenet_resnet50": ("imagenet", 50, 128, False, 0.93, "README.md:39-44 (8 P100, 8ps-8wk)"),
    "imagenet_resnet101": ("imagenet", 101, 256, False, None, None),
}
# vs_baseline compares like with like: the reference row run on the same number of
# GPUs when it published one (BASELINE.md rows 3 / 1 / 7 for CIFAR, 12 / 8 for
# ImageNet), else the model's headline row above; the JSON names the row used.
BASELINE_BY_GPUS = {
    "cifar_resnet50": {1: (13.94, "BASELINE.md row 3: README.md:24-28 (1x P100, local)"),
                       4: (21.82, "BASELINE.md row 1: README.md:16-22 (4x Titan Xp, Horovod)"),
                       8: (28.66, "BASELINE.md row 7: README.md:31 (8x P100, Horovod)")},
    "imagenet_resnet50": {1: (0.96, "BASELINE.md row 12: README.md:48 (1x P100, batch 128)"),
                          8: (0.93, "BASELINE.md row 8: README.md:39-44 (8x P100, 8ps-8wk)")},
}


def baseline_for(model: str, n_gpus: int):
    """(stp/s, source) of the reference number this run is compared with."""
    row = BASELINE_BY_GPUS.get(model, {}).get(n_gpus)
    if row is not None:
        return row
    b, src = MODELS[model][4], MODELS[model][5]
    return (b, f"headline row (no {n_gpus}-GPU row published): {src}") if b else (None, None)
DATA = {
    True: "synthetic: random uint8 32x32 CIFAR records, on-device pad-4/crop/flip/standardize "
          "every step; random-init weights",
    False: "synthetic: random uint8 224x224 crops, on-device flip/mean-subtract/bf16 pack "
           "every step (imagenet_u8_pack); random-init weights",
}
METRIC = "steps/sec (global_batch=128 CIFAR-10 / 1024 ImageNet) ResNet-50 at 1/2/4/8 MI355X"


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--model", default="cifar_resnet50", choices=sorted(MODELS))
    ap.add_argument("--batch", type=int, default=None,
                    help="global batch (cifar) or per-GPU batch (imagenet)")
    ap.add_argument("--device", default="cuda", choices=("cuda", "cpu"),
                    help="cpu: fp32 PyTorch trainer (contract check only, not a headline)")
    ap.add_argument("--graph", action="store_true",
                    help="capture the step in a hipGraph (single stream, 1 GPU only); default: "
                         "eager native plan with weight gradients on a second stream (measured faster)")
    ap.add_argument("--no-graph", action="store_true", help="(default; kept for compatibility)")
    ap.add_argument("--bucket-mb", type=float, default=0.0,
                    help="all-reduce bucket size (MiB); 0 = auto (~4 buckets, <= 25 MiB)")
    ap.add_argument("--allreduce-dtype", default="fp32", choices=("fp32", "bf16"),
                    help="gradient all-reduce precision (bf16 halves the xGMI bytes)")
    ap.add_argument("--phase-steps", type=int, default=5,
                    help="extra steps after the timed region with per-phase HIP-event timing "
                         "(forward / backward / exposed all-reduce / optimizer); 0 = skip")
    ap.add_argument("--step-timeout", type=float, default=300.0,
                    help="watchdog: abort the communicator and exit 3 when no step completes for "
                         "this many seconds (first step: 3x), or on a communicator async error")
    ap.add_argument("--roctx", action="store_true",
                    help="wrap each step's phases in roctx ranges (rocprofv3 --marker-trace); "
                         "adds host overhead, recorded in the JSON")
    return ap.parse_args(argv)


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, argv: list[str]) -> int:
    """Run this script as n rank processes (torchrun's env contract) and relay rank
    0's stdout.  The parent never imports torch, so it never touches the GPU.
    Rank 0 writes into a temp file, not a pipe, so a chatty rank (NCCL_DEBUG=INFO)
    can never block on a full pipe while the others wait in a collective."""
    import tempfile

    port = _free_port()
    procs = []
    out0 = tempfile.TemporaryFile(mode="w+")
    for r in range(n):
        # HSA_ENABLE_IPC_MODE_LEGACY=0 selects ROCm's dmabuf IPC: the hosts of the MI355X
        # pool only support dmabuf IPC, and under the legacy mode RCCL's intra-node P2P
        # (xGMI) buffer exchange fails with "hipIpcGetMemHandle: invalid argument".  An
        # explicit user value is kept.
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
        out = out0 if r == 0 else subprocess.DEVNULL
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv,
                                      env=env, stdout=out, text=True))
    rc = 0
    failed = None
    while True:
        alive = False
        for r, p in enumerate(procs):
            c = p.poll()
            if c is None:
                alive = True
            elif c != 0 and failed is None:
                failed = (r, c)
        if failed is not None or not alive:
            break
        time.sleep(0.2)
    if failed is not None:
        print(f"bench.py: rank {failed[0]} exited with {failed[1]}; stopping the others",
              file=sys.stderr)
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        rc = 1
    out0.seek(0)
    for line in out0.read().splitlines():
        print(line, flush=True)
    out0.close()
    return rc or max(p.returncode or 0 for p in procs)


def dtr_env() -> dict:
    """Every DTR_* knob of this run (fusion modes, diagnostics): echoed into the JSON."""
    return {k: v for k, v in sorted(os.environ.items()) if k.startswith("DTR_")}


def run_cpu(args, dataset, size, per_rank, global_batch, world):
    import torch

    from distributed_tensorflow_resnet_amd.models.spec import build_spec
    from distributed_tensorflow_resnet_amd.parallel.dist import DistContext
    from distributed_tensorflow_resnet_amd.train.backends import CPUBackend
    from distributed_tensorflow_resnet_amd.train.engine import cifar_lr_schedule, imagenet_lr_schedule

    ctx = DistContext(backend="gloo")
    spec = build_spec(dataset, size)
    sched = cifar_lr_schedule() if dataset.startswith("cifar") else imagenet_lr_schedule()
    be = CPUBackend(spec, per_rank, weight_decay=2e-4, lr_schedule=sched, seed=0, dist_ctx=ctx,
                    global_batch=global_batch)
    be.broadcast_parameters(0)
    g = torch.Generator().manual_seed(ctx.rank)
    x = torch.randint(0, 256, (per_rank, 3, spec.image_h, spec.image_w), generator=g,
                      dtype=torch.uint8)
    y = torch.randint(0, spec.num_classes, (per_rank,), generator=g)
    for _ in range(args.warmup):
        be.set_batch(x, y)
        be.step()
    ctx.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        be.set_batch(x, y)
        be.step()
    ctx.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    ctx.all_reduce_max(el)
    m = be.metrics()
    return ctx, float(el.item()), m, {"dtype": "fp32", "device": "cpu"}, None


def run_gpu(args, dataset, size, per_rank, global_batch, world):
    import torch

    from distributed_tensorflow_resnet_amd.models.spec import build_spec
    from distributed_tensorflow_resnet_amd.parallel.dist import (DistContext, apply_cu_partition,
                                                                 local_device_index)
    from distributed_tensorflow_resnet_amd.parallel.watchdog import CommWatchdog
    from distributed_tensorflow_resnet_amd.train.engine import (Engine, cifar_lr_schedule,
                                                                imagenet_lr_schedule)

    # DTR_CU_PARTITION (rehearsals of several ranks on one GPU): this rank's CU mask, in
    # the environment before the first HIP call
    cu_mask = apply_cu_partition()
    local_rank = local_device_index()
    torch.cuda.set_device(local_rank)
    device = torch.device("cuda", local_rank)
    # CIFAR: the persistent step's overlap plan runs RCCL beside its backward grid on the
    # CUs it reserves -- at most one channel (one all-reduce workgroup) per reserved CU
    from distributed_tensorflow_resnet_amd.train.persist import OVERLAP_RESERVE_CUS
    ctx = DistContext(device=device, rccl_max_channels=(OVERLAP_RESERVE_CUS
                                                        if dataset.startswith("cifar") else None))
    spec = build_spec(dataset, size)
    sched = cifar_lr_schedule() if dataset.startswith("cifar") else imagenet_lr_schedule()
    wd = 2e-4 if dataset.startswith("cifar") else 1e-4
    use_graph = bool(args.graph) and not args.no_graph
    # per-step input work for both datasets: CIFAR augments random uint8 records
    # (pad/crop/flip/standardize), ImageNet flips / mean-subtracts / packs random
    # uint8 224x224 crops into the stem's bf16 layout (imagenet_u8_pack)
    input_mode = "cifar_u8" if dataset.startswith("cifar") else "imagenet_u8"
    # A persistent-step grid barrier that times out (workgroups not co-resident beside
    # the job's other kernels) flags the step instead of hanging, and its numbers are
    # garbage.  World > 1 then measures again, all ranks together, on the next plan down
    # -- the persistent step without the comm-stream overlap, then the per-layer plan --
    # and records why (`fallback`); one GPU reports the failure.
    base_tune = os.environ.get("DTR_TUNE")
    plans = [""] + (["persist_overlap=0", "persist=0"] if world > 1 else [])
    fallback = []
    for plan_i, plan_tune in enumerate(plans):
        os.environ["DTR_TUNE"] = ",".join(filter(None, [base_tune or "", plan_tune]))
        eng = Engine(spec, per_rank, weight_decay=wd, lr_schedule=sched, device=device,
                     dist_ctx=ctx, global_batch=global_batch, bucket_mb=args.bucket_mb,
                     seed=0, data_seed=1234 + ctx.rank, use_graph=use_graph,
                     allreduce_dtype=args.allreduce_dtype, input_mode=input_mode)
        dog = CommWatchdog(eng.comm, args.step_timeout, 3 * args.step_timeout).start()
        eng.broadcast_parameters(0)
        eng.fill_synthetic(seed=ctx.rank)

        done = 0
        if use_graph:
            done = eng.capture(warmup=min(2, max(args.warmup, 1)))
        for _ in range(max(args.warmup - done, 0)):
            eng.step()
            dog.beat()
        torch.cuda.synchronize()
        ctx.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            eng.step()
            dog.beat()
        torch.cuda.synchronize()
        ctx.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        dog.beat()
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        ctx.all_reduce_max(t)
        elapsed = float(t.item())
        if ctx._agree(not eng.persist_error()) or plan_i == len(plans) - 1:
            break
        dog.stop()
        fallback.append(f"{plans[plan_i] or 'default plan'}: persistent barrier timeout "
                        f"on some rank")
        print(f"bench.py: rank {ctx.rank}: {fallback[-1]}; measuring again with "
              f"DTR_TUNE={plans[plan_i + 1]}", file=sys.stderr, flush=True)
        del eng
    if base_tune is None:
        os.environ.pop("DTR_TUNE", None)
    else:
        os.environ["DTR_TUNE"] = base_tune
    m = eng.metrics()
    # per-phase timing, outside the timed region (not part of `value`)
    phases = None
    if args.phase_steps > 0 and not use_graph:
        acc = {}
        for _ in range(args.phase_steps):
            for k, v in eng.step_timed().items():
                acc[k] = acc.get(k, 0.0) + v
        phases = {k: round(v / args.phase_steps, 4) for k, v in acc.items()}
    dog.stop()
    # the persistent CIFAR step bounds every grid-barrier wait (2 s) and flags a timeout
    # instead of hanging: a flagged run computed garbage, so its timing is not reported
    if eng.persist_error():
        raise SystemExit(f"bench.py: rank {ctx.rank}: a persistent-step barrier wait timed "
                         "out (workgroups not co-resident?) -- the measurement is invalid")
    # (the persistent step has no side stream: its weight gradients run inside the
    # backward launch)
    extra = {"dtype": "bf16", "device": torch.cuda.get_device_name(device),
             "graph": use_graph, "wgrad_stream": bool(eng.fork_wgrad and not eng.persist),
             "comm": eng.comm_info(),
             "step_path": ("persistent (P fwd/bwd = %d/%d)" % (eng.prn.P_fwd, eng.prn.P)
                           if eng.persist else "per-layer plan"),
             "persist_off_reason": eng.persist_reason or None,
             "persist_overlap": bool(eng.persist_overlap),
             "fallback": fallback or None,
             "cus": int(eng.nat.cu_count()), "cu_mask": cu_mask,
             "peak_mem_gb": round(torch.cuda.max_memory_allocated(device) / 2 ** 30, 2)}
    return ctx, elapsed, m, extra, phases


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse(argv)
    if os.environ.get("DTR_DIAG_SKIP"):
        print("bench.py: refusing to benchmark with DTR_DIAG_SKIP set (it drops launches: "
              "wrong math, timing only)", file=sys.stderr)
        return 2
    under_launcher = "WORLD_SIZE" in os.environ
    if args.gpus > 1 and not under_launcher:
        return spawn_ranks(args.gpus, argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 2
    if args.graph and world > 1:
        print("bench.py: --graph is single-GPU only (no test covers RCCL inside a captured "
              "multi-stream step)", file=sys.stderr)
        return 2
    if args.roctx:
        os.environ["DTR_ROCTX"] = "1"

    dataset, size, batch, is_global, _b, _src = MODELS[args.model]
    if args.batch:
        batch = args.batch
    if is_global:
        if batch % world:
            raise SystemExit(f"global batch {batch} not divisible by {world}")
        per_rank, global_batch = batch // world, batch
    else:
        per_rank, global_batch = batch, batch * world

    runner = run_cpu if args.device == "cpu" else run_gpu
    ctx, elapsed, m, extra, phases = runner(args, dataset, size, per_rank, global_batch, world)
    import torch.distributed as dist

    pg_world = dist.get_world_size() if dist.is_initialized() else 1
    backend = dist.get_backend() if dist.is_initialized() else None
    sps = args.steps / elapsed
    baseline, baseline_src = baseline_for(args.model, world)
    if ctx.is_chief:
        out = {
            "metric": METRIC,
            "value": round(sps, 3),
            "unit": "steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * elapsed / args.steps, 4),
            "higher_is_better": True,
            "scaling": "strong" if is_global else "weak",
            "vs_baseline": round(sps / baseline, 3) if baseline else None,
            "baseline": {"value": baseline, "source": baseline_src},
            "dtype": extra["dtype"],
            "data": DATA[dataset.startswith("cifar")] if args.device == "cuda" else
                    "synthetic uint8 batch (CPU fp32 trainer), random-init weights",
            "config": {
                "model": f"resnet{size}_v2_{dataset}",
                "global_batch": global_batch,
                "per_gpu_batch": per_rank,
                "seq_len": None,
                "image_size": 32 if dataset.startswith("cifar") else 224,
                "parallelism": f"dp{world}",
                "allreduce_dtype": args.allreduce_dtype,
                "roctx": bool(args.roctx),
                "env": dtr_env(),
                **{k: v for k, v in extra.items() if k != "dtype"},
            },
            "dist_backend": backend,
            "pg_world_size": pg_world,
            "phase_ms": phases,
            "images_per_sec": round(sps * global_batch, 1),
            "final_loss": round(m["cross_entropy"], 4),
        }
        print(json.dumps(out), flush=True)
    ctx.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
