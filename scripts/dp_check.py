#!/usr/bin/env python3
"""Data-parallel correctness check for the GPU engine (run under torchrun).

Every rank trains the same random-init model on its own synthetic shard.  After
one step the all-reduced gradient of the DP engine must equal, bit for bit, the
rank-order sum of a second, non-distributed engine's local gradients on the same
shards (fp32; with a bf16 exchange: the rank-order fp32 sum of the bf16-rounded
local gradients, rounded to bf16 once -- what the shm transport computes; the
c10d/gloo bf16 path is checked to 1e-2 relative), and after further steps every
rank must hold identical fp32 master weights and momentum (BN moving statistics
stay per-replica, as with Horovod).

    DTR_DIST_BACKEND=gloo torchrun --nproc-per-node 2 --master-addr 127.0.0.1 \
        scripts/dp_check.py            # 2 ranks rehearsed on one GPU, c10d transport
    DTR_DIST_BACKEND=gloo DTR_COMM_TRANSPORT=shm torchrun ... scripts/dp_check.py
                                       # the native plan-op path (comm stream, issue
                                       # threads, bf16 casts) over the shm transport
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_tensorflow_resnet_amd.models.spec import build_spec  # noqa: E402
from distributed_tensorflow_resnet_amd.parallel.dist import (DistContext,  # noqa: E402
                                                             apply_cu_partition,
                                                             local_device_index)
from distributed_tensorflow_resnet_amd.train.engine import Engine, cifar_lr_schedule  # noqa: E402


def main() -> int:
    size = int(os.environ.get("DP_CHECK_SIZE", "14"))
    per_rank = int(os.environ.get("DP_CHECK_BATCH", "8"))
    bucket_mb = float(os.environ.get("DP_CHECK_BUCKET_MB", "0.25"))
    cu_mask = apply_cu_partition()   # DTR_CU_PARTITION: before the first HIP call
    torch.cuda.set_device(local_device_index())
    dev = torch.device("cuda", local_device_index())
    ctx = DistContext(device=dev)
    world, rank = ctx.world_size, ctx.rank
    # DP_CHECK_DATASET=imagenet: the ImageNet per-layer plan (side stream + comm-stream
    # buckets), e.g. ResNet-50 at 16 images per rank with DP_CHECK_BUCKET_MB=25
    spec = build_spec(os.environ.get("DP_CHECK_DATASET", "cifar10"), size)
    ar_dtype = os.environ.get("DP_CHECK_ALLREDUCE", "fp32")
    kw = dict(weight_decay=2e-4, lr_schedule=cifar_lr_schedule(), device=dev,
              global_batch=per_rank * world, seed=0, data_seed=1234 + rank)
    eng = Engine(spec, per_rank, dist_ctx=ctx, bucket_mb=bucket_mb, allreduce_dtype=ar_dtype,
                 **kw)
    ref = Engine(spec, per_rank, dist_ctx=None, **kw)
    eng.broadcast_parameters(0)
    for e in (eng, ref):
        e.fill_synthetic(seed=rank)
    if eng.persist != ref.persist:
        raise SystemExit(f"dp_check: persistent step on the DP engine {eng.persist} "
                         f"({eng.persist_reason}) but {ref.persist} on the local one ({ref.persist_reason})")
    eng.step()
    # the local gradient without an update (the one-GPU persistent step leaves its
    # weight-gradient slabs to the optimizer launch; forward_backward sums them into grad)
    ref.forward_backward()
    torch.cuda.synchronize()
    if eng.persist_error() or ref.persist_error():
        raise SystemExit("dp_check: a persistent-step grid barrier timed out")
    info = eng.comm_info()
    if ctx.backend == "gloo":
        local = ref.grad.cpu()
        parts = [torch.empty_like(local) for _ in range(world)]
        torch.distributed.all_gather(parts, local)
    else:   # nccl: gather through the device
        dparts = [torch.empty_like(ref.grad) for _ in range(world)]
        torch.distributed.all_gather(dparts, ref.grad)
        parts = [p.cpu() for p in dparts]
    got = eng.grad.cpu()
    if ar_dtype == "bf16":
        acc = parts[0].to(torch.bfloat16).float()
        for p in parts[1:]:
            acc = acc + p.to(torch.bfloat16).float()
        want = acc.to(torch.bfloat16).float()
        if info["native"]:   # exact: the native transports' rank-order bf16 sum
            grad_ok = torch.equal(want, got)
        else:                # c10d: the backend's own bf16 summation
            grad_ok = bool(((want - got).norm() / want.norm()) < 1e-2)
    else:
        want = parts[0].clone()
        for p in parts[1:]:
            want = want + p
        grad_ok = torch.equal(want, got)
    maxdiff = float((want - got).abs().max())
    for _ in range(int(os.environ.get("DP_CHECK_STEPS", "3"))):
        eng.step()
    torch.cuda.synchronize()
    state = torch.cat([eng.params.master, eng.mom])
    r0 = state.clone()
    ctx.broadcast(r0, 0)
    sync_ok = torch.equal(r0, state)
    flags = torch.tensor([0 if grad_ok else 1, 0 if sync_ok else 1], device=dev)
    ctx.all_reduce_sum(flags)
    err = torch.tensor([int(eng.persist_error())], device=dev)
    ctx.all_reduce_sum(err)
    m = eng.metrics()
    if ctx.is_chief:
        path = (f"persistent(P={eng.prn.P_fwd}/{eng.prn.P},overlap={int(eng.persist_overlap)},"
                f"wgrad_wgs={eng.prn.wgrad_wgs})" if eng.persist else "per-layer")
        print(f"dp_check world={world} transport={info['transport']} "
              f"native={info['native']} allreduce_ops={info['allreduce_ops']} "
              f"fallback={info['fallback_reason']} step_path={path} cus={eng.nat.cu_count()} "
              f"cu_mask={cu_mask} grad_equal_ranks_failing="
              f"{int(flags[0])} (max|diff|={maxdiff:.3g}) replicas_diverged={int(flags[1])} "
              f"persist_errors={int(err)} "
              f"loss={m['cross_entropy']:.4f} step={m['global_step']}", flush=True)
        ok = int(flags.sum()) == 0 and int(err) == 0
        print("DP_CHECK_OK" if ok else "DP_CHECK_FAIL", flush=True)
    ctx.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
