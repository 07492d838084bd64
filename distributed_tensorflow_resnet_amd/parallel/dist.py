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

import contextlib
import datetime
import faulthandler
import os
import socket
import sys
import threading
import time
import uuid

import torch
import torch.distributed as dist

INIT_HANG_EXIT = 3   # same code as the step watchdog: the launcher restarts the job


@contextlib.contextmanager
def _deadline(seconds: float, what: str):
    """End the process (exit 3) if the body has not returned within `seconds`:
    a collective init that never completes (a rank that never joined) cannot be
    aborted from Python, and a hung job is worse than a restartable one."""
    def fire():
        print(f"[dist] {what} did not complete within {seconds:.0f}s: exiting for restart",
              file=sys.stderr, flush=True)
        faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
        os._exit(INIT_HANG_EXIT)
    t = threading.Timer(seconds, fire)
    t.daemon = True
    t.start()
    try:
        yield
    finally:
        t.cancel()


def _canary(nat, comm, world: int, device_index: int, timeout_s: float):
    """One small all-reduce through a fresh communicator: None if every element
    came back as 1 + 2 + ... + world, else the reason."""
    try:
        dev = torch.device("cuda", device_index)
        x = torch.full((256,), float(comm.rank + 1), dtype=torch.float32, device=dev)
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        comm.all_reduce(x.data_ptr(), x.numel(), nat.COMM_F32, s.cuda_stream)
        ev = torch.cuda.Event()
        ev.record(s)
        t0 = time.monotonic()
        while not ev.query():
            if comm.async_error():
                return f"canary: async error {comm.async_error()}"
            if time.monotonic() - t0 > timeout_s:
                comm.abort()
                return f"canary all-reduce did not complete within {timeout_s:.0f}s"
            time.sleep(0.001)
        want = world * (world + 1) / 2
        if not bool((x == want).all()):
            return f"canary all-reduce returned {float(x[0])}, expected {want}"
    except Exception as e:   # noqa: BLE001 - reported as the fallback reason
        return f"canary raised: {e}"
    return None


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


_STREAMS: dict = {}


def engine_streams(device: torch.device):
    """The engine's side (weight-gradient) and comm (all-reduce) streams of `device`,
    created once per process.

    Created BEFORE the c10d NCCL group and RCCL set up their own streams: a stream's
    hardware queue is assigned at creation (GPU_MAX_HW_QUEUES = 4), and created after
    RCCL's eight internal streams the side stream landed on the main stream's queue and
    the comm stream on a queue shared with RCCL's proxy copies (rocprofv3 queue ids,
    profiles/stream_queues.md).  DistContext calls this before init_process_group; the
    engine takes the same pair."""
    key = (device.type, device.index)
    if key not in _STREAMS and device.type == "cuda":
        pair = (torch.cuda.Stream(device=device), torch.cuda.Stream(device=device))
        # a stream is bound to its hardware queue at its first dispatch: dispatch on the
        # default stream and on both engine streams now, before RCCL's streams do
        torch.zeros(1, device=device)
        for s in pair:
            with torch.cuda.stream(s):
                torch.zeros(1, device=device)
        torch.cuda.synchronize(device)
        _STREAMS[key] = pair
    if key not in _STREAMS:
        return torch.cuda.Stream(device=device), torch.cuda.Stream(device=device)
    return _STREAMS[key]


def device_identity(index: int) -> str:
    """Physical identity of visible device `index` on this host: its PCI location, else
    its UUID, else (neither exposed) the visible-device masks plus the ordinal -- so ranks
    that each see one GPU through HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES (ordinal 0
    everywhere) still differ."""
    props = torch.cuda.get_device_properties(index)
    pci = tuple(getattr(props, k, None) for k in ("pci_domain_id", "pci_bus_id", "pci_device_id"))
    if all(v is not None for v in pci) and any(pci):
        return "pci:%x:%x:%x" % pci
    uid = str(getattr(props, "uuid", "") or "")
    if uid.strip("0-") and uid.lower() not in ("none",):
        return f"uuid:{uid}"
    vis = "|".join(os.environ.get(k, "") for k in
                   ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"))
    return f"ord:{vis}|{index}"


def ranks_on_device(store, rank: int, world: int, ident: str, tag: str = "dev") -> int:
    """How many ranks of this job (this one included) run on the physical device `ident`
    of this host: every rank publishes (hostname, identity) through the c10d store and
    reads the others' (blocking until each rank has published -- every rank calls this
    at the same point, the engine build)."""
    return len(peers_on_device(store, rank, world, ident, tag))


def peers_on_device(store, rank: int, world: int, ident: str, tag: str = "dev") -> list:
    """The ranks (this one included) on the physical device `ident` of this host
    (ranks_on_device)."""
    mine = f"{socket.gethostname()}|{ident}"
    store.set(f"dtr/{tag}/{rank}", mine)
    return [r for r in range(world)
            if (mine if r == rank else bytes(store.get(f"dtr/{tag}/{r}")).decode()) == mine]


def _kfd_cu_count() -> int:
    """CUs of this host's GPUs from the KFD topology (no HIP call: the CU mask must be in
    the environment before the runtime starts); 256 (MI355X) when it is not readable."""
    root = "/sys/class/kfd/kfd/topology/nodes"
    try:
        for node in sorted(os.listdir(root)):
            props = {}
            with open(os.path.join(root, node, "properties")) as f:
                for line in f:
                    k, _, v = line.partition(" ")
                    props[k] = v.strip()
            simds, per = int(props.get("simd_count", 0)), int(props.get("simd_per_cu", 0))
            if simds > 0 and per > 0:
                return simds // per
    except (OSError, ValueError):
        pass
    return 256


def cu_partition_mask(index: int, parts: int, total: int) -> int:
    """CU mask (bit i = CU i) of partition `index` of `parts` contiguous equal ranges."""
    if not 0 <= index < parts or parts < 1 or total < parts:
        raise ValueError(f"CU partition {index}/{parts} of {total} CUs")
    lo, hi = index * total // parts, (index + 1) * total // parts
    return ((1 << (hi - lo)) - 1) << lo


def apply_cu_partition() -> str | None:
    """Split one GPU's CUs between the ranks that share it (DTR_CU_PARTITION): ``n`` =
    this process takes partition LOCAL_RANK % n of n contiguous CU ranges, ``i/n`` =
    partition i.  Sets ROC_GLOBAL_CU_MASK, the HIP runtime's process-wide CU mask that
    every queue of the process (the null stream, the engine's streams, the transport's
    copies) inherits, so it must run before the first HIP call (entrypoints call it
    before touching the GPU).  With disjoint masks two ranks on one GPU can each run
    the persistent step's co-resident grids (gpu_shared_by_ranks compares the masks;
    the grids are sized by the masked CU count, _C.cu_count).  Returns the mask (hex)
    or None when no partition is asked for."""
    env = os.environ
    spec = os.environ.get("DTR_CU_PARTITION", "").strip()
    if not spec or spec == "0":
        return None
    if "/" in spec:
        i, n = (int(v) for v in spec.split("/", 1))
    else:
        n = int(spec)
        i = int(env.get("LOCAL_RANK", env.get("RANK", "0"))) % n
    mask = hex(cu_partition_mask(i, n, _kfd_cu_count()))
    env["ROC_GLOBAL_CU_MASK"] = mask
    return mask


def _cu_mask_int() -> int:
    """This process's CU mask on the current device as an int (0: unknown = all CUs)."""
    try:
        from .. import native
        words = native(required=True).cu_mask()
    except Exception:   # noqa: BLE001 - no extension: treat as the whole device
        return 0
    return sum(int(w) << (32 * i) for i, w in enumerate(words))


def gpu_shared_by_ranks(ctx=None, device_index: int | None = None) -> bool:
    """Whether another rank of this job runs on this rank's physical GPU (the one-GPU
    rehearsals that fold ranks onto one device) on CUs this rank also uses.  Kernels that
    need every workgroup co-resident (the persistent CIFAR step) must not run then: two
    processes' grids interleaved on one device could each hold part of the CUs and wait
    for the rest forever.  Decided from the devices' physical identities (device_identity)
    and the processes' CU masks (apply_cu_partition) exchanged through the c10d store,
    not from rank / device counts: launchers that hand every rank one GPU by
    visible-device masks see one device per process; ranks whose CU masks are disjoint
    do not share."""
    if torch.cuda.device_count() == 0:
        return False
    if ctx is not None and getattr(ctx, "active", False):
        rank, world = ctx.rank, ctx.world_size
    elif dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        # an engine built without a context (a single-process reference beside the
        # distributed one, as the DP rehearsals build) shares the device all the same
        rank, world = dist.get_rank(), dist.get_world_size()
    else:
        return False
    idx = torch.cuda.current_device() if device_index is None else device_index
    store = dist.distributed_c10d._get_default_store()
    peers = [r for r in peers_on_device(store, rank, world, device_identity(idx)) if r != rank]
    if not peers:
        return False
    # several ranks on this GPU: shared unless every other one's CU mask is disjoint
    mine = _cu_mask_int()
    store.set(f"dtr/cumask/{rank}", f"{mine:x}")
    for r in peers:
        other = int(bytes(store.get(f"dtr/cumask/{r}")).decode(), 16)
        if mine == 0 or other == 0 or (mine & other):
            return True
    return False


def rccl_channels_reported(path: str | None) -> int | None:
    """RCCL's channel count from its INIT debug log (``Channel 00/NN`` lines: the largest
    NN of this process's communicators), None when there is no log."""
    if not path or not os.path.exists(path):
        return None
    import re

    best = None
    with open(path, errors="replace") as fh:
        for line in fh:
            for m in re.finditer(r"Channel \d+/(\d+)", line):
                best = max(best or 0, int(m.group(1)))
    return best


class DistContext:
    """Thin, explicit wrapper so the engine never touches global state.

    ``rccl_max_channels``: cap RCCL's channels (NCCL_MAX_NCHANNELS, set before the first
    communicator of the process unless the user set it): each channel is one workgroup of
    an all-reduce kernel, and the persistent CIFAR step's overlap plan runs the all-reduces
    beside its backward grid on the OVERLAP_RESERVE_CUS it leaves free -- at one channel
    per reserved CU they fit (train/persist.py).  RCCL's own INIT log (NCCL_DEBUG=INFO,
    NCCL_DEBUG_SUBSYS=INIT into a per-process file, unless the user set NCCL_DEBUG) is kept
    so comm_info can report the channel count RCCL actually built."""

    def __init__(self, backend: str | None = None, device: torch.device | None = None,
                 timeout_s: float = 600.0, rccl_max_channels: int | None = None):
        self.rank, self.world_size, self.local_rank = env_world()
        self.backend = backend
        self.device = device
        self.timeout_s = float(timeout_s)
        self.comm_fallback_reason = None
        self.initialized_here = False
        self.rccl_log = None
        if device is not None and device.type == "cuda":
            engine_streams(device)   # before RCCL's streams: distinct hardware queues
        if self.world_size > 1 and not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29500")
            if backend is None:
                backend = os.environ.get("DTR_DIST_BACKEND") or (
                    "nccl" if torch.cuda.is_available() else "gloo")
            self.backend = backend
            if backend == "nccl":
                if rccl_max_channels and "NCCL_MAX_NCHANNELS" not in os.environ:
                    os.environ["NCCL_MAX_NCHANNELS"] = str(int(rccl_max_channels))
                if "NCCL_DEBUG" not in os.environ:
                    import tempfile

                    self.rccl_log = os.path.join(tempfile.gettempdir(),
                                                 f"dtr-rccl-init-{os.getpid()}.log")
                    os.environ.update(NCCL_DEBUG="INFO", NCCL_DEBUG_SUBSYS="INIT",
                                      NCCL_DEBUG_FILE=self.rccl_log)
            kw = {}
            if backend == "nccl" and device is not None:
                kw["device_id"] = device
            dist.init_process_group(backend=backend, init_method="env://", rank=self.rank,
                                    world_size=self.world_size,
                                    timeout=datetime.timedelta(seconds=timeout_s), **kw)
            self.initialized_here = True
        elif dist.is_initialized():
            self.backend = dist.get_backend()

    def comm_transport(self) -> str:
        """Gradient-exchange transport of this job (env DTR_COMM_TRANSPORT):
        ``auto`` (default) = ``rccl`` on the nccl backend, ``c10d`` otherwise;
        ``rccl`` native RCCL communicator (plan ops on the comm stream);
        ``shm`` native host-staged shared-memory rehearsal transport, the same
        plan ops with several ranks folded onto one GPU (csrc/comm_shm.cpp);
        ``c10d`` host-issued torch.distributed all-reduces between plan segments."""
        t = os.environ.get("DTR_COMM_TRANSPORT", "auto")
        if t not in ("auto", "rccl", "shm", "c10d"):
            raise ValueError(f"DTR_COMM_TRANSPORT must be auto|rccl|shm|c10d, got {t!r}")
        if t == "auto":
            return "rccl" if self.backend == "nccl" else "c10d"
        return t

    def _agree(self, ok: bool) -> bool:
        """True iff every rank passed `ok` (a c10d MAX of the failure flags)."""
        if not self.active:
            return ok
        dev = self.device if (self.backend == "nccl" and self.device is not None) else "cpu"
        t = torch.tensor([0 if ok else 1], dtype=torch.int32, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return int(t.item()) == 0

    def native_comm(self, device_index: int, force: bool = False, transport: str | None = None):
        """The native communicator of this job (`_C.Comm`, csrc/comm.h) or None
        (then the engine issues c10d all-reduces from the host instead).

        Built for world > 1 when the transport (``comm_transport``) is rccl or
        shm, or when ``force`` (a single-rank RCCL communicator: tests of the comm
        path).  Fail-safe and collective -- every rank takes the same decision:
          1. preflight (the extension loads, RCCL's symbols resolve), agreed
             over c10d;
          2. rendezvous: rank 0's ncclUniqueId / shm segment name travels through
             the c10d store; construction runs under a timer that ends the
             process (exit 3, launcher restart) if the collective init hangs;
          3. a canary all-reduce of (rank + 1) must return world(world+1)/2
             within the timeout, agreed over c10d.
        Any failure falls back to c10d on EVERY rank, with the reason in
        ``self.comm_fallback_reason`` (bench.py JSON `comm.fallback_reason`)."""
        self.comm_fallback_reason = None
        kind = transport or ("rccl" if force and not self.active else self.comm_transport())
        if kind == "c10d":
            return None
        if not force and not self.active:
            return None
        from .. import native

        nat = native(required=True)
        ok = kind != "rccl" or bool(nat.Comm.rccl_available())
        if not self._agree(ok):
            self.comm_fallback_reason = f"{kind} preflight failed on some rank"
            return None
        self._comm_seq = getattr(self, "_comm_seq", 0) + 1
        world, rank = (self.world_size, self.rank) if self.active else (1, 0)
        key = f"dtr/comm_id/{self._comm_seq}"
        if kind == "rccl":
            ident = nat.Comm.unique_id() if rank == 0 else None
        else:
            ident = (f"/dtr-{os.getpid()}-{uuid.uuid4().hex[:16]}".encode()
                     if rank == 0 else None)
        if self.active:
            store = dist.distributed_c10d._get_default_store()
            if rank == 0:
                store.set(key, ident)
            else:
                ident = bytes(store.get(key))
        comm, err = None, None
        with _deadline(self.timeout_s, f"{kind} communicator init"):
            try:
                if kind == "rccl":
                    comm = nat.Comm(ident, world, rank, device_index)
                else:
                    # the transport's own attach timeout fires well inside the
                    # deadline, so a missing peer reaches the agreed c10d fallback
                    # below instead of the deadline's exit
                    comm = nat.Comm.shm(ident.decode(), world, rank, device_index,
                                        timeout_s=self.timeout_s,
                                        init_timeout_s=max(1.0, 0.8 * self.timeout_s))
            except Exception as e:   # noqa: BLE001 - reported as the fallback reason
                err = f"{kind} init failed on rank {rank}: {e}"
        if not self._agree(comm is not None):
            self.comm_fallback_reason = err or f"{kind} init failed on another rank"
            if comm is not None:
                comm.abort()
            return None
        err = _canary(nat, comm, world, device_index, min(self.timeout_s, 120.0))
        if not self._agree(err is None):
            comm.abort()
            self.comm_fallback_reason = err or f"{kind} canary failed on another rank"
            return None
        return comm

    def rccl_channel_info(self) -> dict:
        """The channel cap in force and the count RCCL reported (bench JSON, comm_info)."""
        return {"rccl_max_nchannels": os.environ.get("NCCL_MAX_NCHANNELS"),
                "rccl_channels": rccl_channels_reported(self.rccl_log)}

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
