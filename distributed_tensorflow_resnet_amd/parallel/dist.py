"""Process-group context: one process per GPU, torch.distributed over RCCL.

Replaces the reference's two distribution runtimes:
  * Horovod (`hvd.init()`, `hvd.DistributedOptimizer`, BroadcastGlobalVariablesHook)
  * TF parameter servers (`tf.train.Server`, `replica_device_setter`,
    `SyncReplicasOptimizer`, gRPC)
with synchronous data parallelism: backend "nccl" (= RCCL on ROCm, ring /
tree collectives over the xGMI links) for GPU ranks, "gloo" for CPU ranks.
Rendezvous is the standard env:// contract (RANK, WORLD_SIZE, LOCAL_RANK,
MASTER_ADDR, MASTER_PORT) set by torchrun or parallel/launch.py.
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist


def env_world() -> tuple[int, int, int]:
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def local_device_index() -> int:
    """GPU for this rank: LOCAL_RANK, folded onto the visible devices.  Folding
    only matters for rehearsals that put several ranks on one GPU (with
    DTR_DIST_BACKEND=gloo, since RCCL refuses duplicate devices);
    `torch.cuda.device_count()` does not initialise the GPU."""
    local = int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0")))
    n = torch.cuda.device_count()
    return local % n if n > 0 else local


class DistContext:
    """Thin, explicit wrapper so the engine never touches global state."""

    def __init__(self, backend: str | None = None, device: torch.device | None = None,
                 timeout_s: float = 600.0):
        self.rank, self.world_size, self.local_rank = env_world()
        self.backend = backend
        self.device = device
        self.initialized_here = False
        if self.world_size > 1 and not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29500")
            if backend is None:
                backend = os.environ.get("DTR_DIST_BACKEND") or (
                    "nccl" if torch.cuda.is_available() else "gloo")
            self.backend = backend
            kw = {}
            if backend == "nccl" and device is not None:
                kw["device_id"] = device
            dist.init_process_group(backend=backend, init_method="env://", rank=self.rank,
                                    world_size=self.world_size,
                                    timeout=datetime.timedelta(seconds=timeout_s), **kw)
            self.initialized_here = True
        elif dist.is_initialized():
            self.backend = dist.get_backend()

    def native_comm(self, device_index: int, force: bool = False):
        """The native RCCL communicator of this job (`_C.Comm`, csrc/comm.h) or None.

        Built when the job runs on RCCL ("nccl" backend) with more than one rank,
        or when ``force`` (single-rank tests of the comm path).  Rank 0's
        ncclUniqueId travels through the c10d TCP store, the same rendezvous the
        process group used; each call makes a fresh communicator (the ranks must
        call in the same order, as they build their engines in the same order).
        DTR_NATIVE_COMM=0 keeps the gradient all-reduce on c10d instead."""
        if os.environ.get("DTR_NATIVE_COMM", "1") == "0" and not force:
            return None
        if not force and not (self.active and self.backend == "nccl"):
            return None
        from .. import native

        nat = native(required=True)
        self._comm_seq = getattr(self, "_comm_seq", 0) + 1
        if self.active:
            store = dist.distributed_c10d._get_default_store()
            key = f"dtr/rccl_uid/{self._comm_seq}"
            if self.rank == 0:
                uid = nat.Comm.unique_id()
                store.set(key, uid)
            else:
                uid = bytes(store.get(key))
            world, rank = self.world_size, self.rank
        else:
            uid, world, rank = nat.Comm.unique_id(), 1, 0
        return nat.Comm(uid, world, rank, device_index)

    @property
    def is_chief(self) -> bool:
        return self.rank == 0

    @property
    def active(self) -> bool:
        return self.world_size > 1 and dist.is_initialized()

    def all_reduce_async(self, t: torch.Tensor):
        return dist.all_reduce(t, op=dist.ReduceOp.SUM, async_op=True)

    def all_reduce_sum(self, t: torch.Tensor) -> torch.Tensor:
        if self.active:
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return t

    def all_reduce_max(self, t: torch.Tensor) -> torch.Tensor:
        if self.active:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return t

    def broadcast(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        if self.active:
            dist.broadcast(t, src)
        return t

    def barrier(self):
        if self.active:
            if self.backend == "nccl" and self.device is not None:
                dist.barrier(device_ids=[self.device.index])
            else:
                dist.barrier()

    def shutdown(self):
        if self.initialized_here and dist.is_initialized():
            dist.destroy_process_group()
