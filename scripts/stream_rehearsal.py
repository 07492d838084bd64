"""One-GPU rehearsal of the world > 1 stream set.

One process builds exactly what a rank of the 8-GPU job builds: a c10d NCCL (RCCL)
process group initialised eagerly with ``device_id`` (its internal stream), the
engine's main / side / comm streams, a native RCCL ``Comm`` forced at world 1 with
the bf16 gradient exchange (cast kernels + all-reduce on the comm stream), and a c10d
all-reduce per step like the metrics / timing reductions of bench.py.  Run it under
``rocprofv3 --kernel-trace --hip-runtime-trace`` and summarise the trace with
``scripts/queue_table.py``: every stream's hardware queue id.

usage: python scripts/stream_rehearsal.py MODEL BATCH STEPS [late]
(late: the round-3 order -- engine streams created and first used after the process
group -- for the A/B in profiles/stream_queues.md)"""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_resnet_amd.models.spec import build_spec  # noqa: E402
from distributed_tensorflow_resnet_amd.parallel.dist import DistContext  # noqa: E402
from distributed_tensorflow_resnet_amd.train.engine import (Engine, cifar_lr_schedule,  # noqa: E402
                                                            imagenet_lr_schedule)


def main():
    model, batch, steps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    dataset, size = ("cifar10", int(model.split("resnet")[1])) if model.startswith("cifar") else \
        ("imagenet", int(model.split("resnet")[1]))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29561")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    late = len(sys.argv) > 4 and sys.argv[4] == "late"
    if not late:
        ctx0 = DistContext(device=dev)   # (world 1: creates the engine streams, like a rank does)
        del ctx0
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    if late:
        from distributed_tensorflow_resnet_amd.parallel import dist as dmod
        dmod._STREAMS[(dev.type, dev.index)] = (torch.cuda.Stream(device=dev),
                                               torch.cuda.Stream(device=dev))
    ctx = DistContext(device=dev)
    spec = build_spec(dataset, size)
    cifar = dataset.startswith("cifar")
    eng = Engine(spec, batch, weight_decay=2e-4 if cifar else 1e-4,
                 lr_schedule=cifar_lr_schedule() if cifar else imagenet_lr_schedule(),
                 device=dev, dist_ctx=ctx, native_comm=True, allreduce_dtype="bf16",
                 input_mode="cifar_u8" if cifar else "imagenet_u8")
    info = eng.comm_info()
    assert info["native_rccl"] and info["allreduce_ops"] >= 1, info
    eng.fill_synthetic(0)
    handles = {"torch current (main)": torch.cuda.current_stream().cuda_stream,
               "engine side": eng.side.cuda_stream, "engine comm": eng.comm_stream.cuda_stream}
    t = torch.ones(4, device=dev)
    for _ in range(steps):
        eng.step()
        dist.all_reduce(t)   # the c10d control-plane collective (metrics, timing max)
    torch.cuda.synchronize()
    print("STREAMS", {k: hex(v) for k, v in handles.items()})
    print("COMM", {k: info[k] for k in ("transport", "allreduce_ops", "allreduce_bytes", "buckets")
                   if k in info}, "persist", eng.persist)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
