"""Execution backends behind TrainingSession.

GPUBackend  the MI355X engine (native plan + HIP kernels + RCCL all-reduce)
CPUBackend  fp32 PyTorch autograd with TF semantics (BASELINE config 1,
            `resnet_single.py`; also runs multi-process data parallel over
            gloo for CPU tests of the distributed logic)
Both expose the same small interface (set_batch / step / metrics /
state_tensors / load_state / broadcast_parameters) and the same TF-named
checkpoint layout, so a run can be resumed on either.
"""
from __future__ import annotations

import math
import os

import torch

from ..data.cifar import augment_cpu
from ..models.params import ParamStore
from ..models.resnet_torch import TorchResNet
from ..models.spec import ModelSpec
from ..parallel.dist import local_device_index
from ..utils.checkpoint import state_to_tf, tf_to_state


class GPUBackend:
    def __init__(self, engine, use_graph: bool = False):
        self.engine = engine
        self.use_graph = use_graph
        self._host_step = int(engine.gstep.item())
        self.profile_phases = False
        self.last_phase_ms = None
        self._captured = False
        self._eager_done = False

    @property
    def global_step(self) -> int:
        return self._host_step

    def set_batch(self, images, labels):
        self.engine.set_batch(images, labels)

    def step(self, need_cost: bool = False):
        eng = self.engine
        if self.profile_phases:
            self.last_phase_ms = eng.step_timed(need_cost)
        elif self.use_graph:
            # first step eager (initialises RCCL communicators), second step
            # captures the hipGraph (capture executes nothing) and replays it:
            # exactly one training step per call either way.
            if self._eager_done and not self._captured:
                eng.capture(warmup=0)
                self._captured = True
            eng.step(need_cost)
            self._eager_done = True
        else:
            eng.step(need_cost)
        self._host_step += 1

    def metrics(self):
        # rank-local (the session's hooks read metrics on their own schedules, chief-only
        # hooks on the chief only, so a collective here would be joined by nobody -- or,
        # with the c10d transport, by another rank's gradient all-reduce).  Like the
        # reference's per-worker LoggingTensorHook, each rank logs its own batch.
        return self.engine.metrics(reduce=False)

    def synchronize(self):
        torch.cuda.synchronize()

    def check_health(self):
        """Raise (engine.PersistentStepError) if a persistent launch failed: called before
        every checkpoint save, so a half-computed step never reaches a checkpoint."""
        self.engine.check_health()

    def state_tensors(self):
        self.check_health()
        return state_to_tf(self.engine.params, self.engine.mom, self.global_step)

    def load_state(self, tensors):
        eng = self.engine
        gs = tf_to_state(tensors, eng.params, eng.mom, strict=True)
        eng.sync_from_params()
        self._host_step = gs

    def broadcast_parameters(self, src: int = 0):
        self.engine.broadcast_parameters(src)
        self._host_step = int(self.engine.gstep.item())


class CPUBackend:
    """fp32 autograd trainer; DP over torch.distributed (gloo) when dist_ctx given."""

    def __init__(self, spec: ModelSpec, batch_size: int, *, weight_decay: float, lr_schedule,
                 optimizer: str = "mom", momentum: float = 0.9, seed: int = 0, dist_ctx=None,
                 global_batch: int | None = None, threads: int = 0,
                 allreduce_dtype: str = "fp32"):
        # intra-op threads: DTR_CPU_THREADS, default 1 -- on small containers the
        # OpenMP pool's spin-waits oversubscribe the CPU quota (measured here: one
        # 8x32x32x16 conv fwd+bwd 1.2 ms on 1 thread, 612 ms on 8)
        threads = threads or int(os.environ.get("DTR_CPU_THREADS", "1"))
        if threads > 0:
            torch.set_num_threads(threads)
        self.spec = spec
        self.N = batch_size
        self.dist = dist_ctx
        self.world = dist_ctx.world_size if dist_ctx is not None else 1
        self.global_batch = global_batch or batch_size * self.world
        self.store = ParamStore(spec)
        self.store.initialize(seed)
        self.model = TorchResNet(spec, self.store)
        self.mom = torch.zeros(self.store.n_train)
        self.wd = weight_decay
        self.momentum = momentum
        self.use_momentum = optimizer == "mom"
        self.sched = lr_schedule
        self.step_count = 0
        self.gen = torch.Generator().manual_seed(seed + 97 * (dist_ctx.rank if dist_ctx else 0))
        self._x = None
        self._y = None
        self._last = {}
        self.profile_phases = False
        self.last_phase_ms = None
        if allreduce_dtype not in ("fp32", "bf16"):
            raise ValueError(f"allreduce_dtype must be fp32 or bf16, got {allreduce_dtype!r}")
        self.allreduce_bf16 = allreduce_dtype == "bf16"

    @property
    def global_step(self) -> int:
        return self.step_count

    def set_batch(self, images, labels):
        if images.dtype == torch.uint8:
            images = augment_cpu(images, train=True, generator=self.gen)
        self._x = images.float()
        self._y = labels.long()

    def step(self, need_cost: bool = False):   # the CPU loss always includes the l2 term
        m = self.model
        master = self.store.master
        if master.grad is not None:
            master.grad = None
        logits = m(self._x, True)
        xent, _ = m.loss(logits, self._y, self.wd)
        # mean over the GLOBAL batch: local mean * (local/global), then sum-allreduce
        (xent * (self.N / self.global_batch)).backward()
        g = master.grad
        if self.dist is not None and self.world > 1:
            if self.allreduce_bf16:   # compressed exchange, fp32 accumulate of the result
                gb = g.to(torch.bfloat16)
                self.dist.all_reduce_sum(gb)
                g = gb.float()
            else:
                self.dist.all_reduce_sum(g)
        lr = self.sched.at(self.step_count)
        with torch.no_grad():
            gp = g + self.wd * master
            if self.use_momentum:
                self.mom.mul_(self.momentum).add_(gp)
                master.sub_(lr * self.mom)
            else:
                master.sub_(lr * gp)
            l2 = 0.5 * float((master * master).sum())
            correct = float((logits.argmax(1) == self._y).float().sum())
        loss_sum = float(xent) * self.N
        if self.dist is not None and self.world > 1:
            t = torch.tensor([loss_sum, correct])
            self.dist.all_reduce_sum(t)
            loss_sum, correct = t.tolist()
        n = self.global_batch
        self.step_count += 1
        self._last = {"global_step": self.step_count, "cross_entropy": loss_sum / n,
                      "cost": loss_sum / n + self.wd * l2, "precision": correct / n, "lr": lr,
                      "l2": l2}

    def metrics(self):
        return dict(self._last)

    def synchronize(self):
        pass

    def check_health(self):
        pass

    def state_tensors(self):
        return state_to_tf(self.store, self.mom, self.step_count)

    def load_state(self, tensors):
        with torch.no_grad():
            self.step_count = tf_to_state(tensors, self.store, self.mom)

    def broadcast_parameters(self, src: int = 0):
        if self.dist is not None and self.world > 1:
            with torch.no_grad():
                for t in (self.store.master, self.store.stats, self.mom):
                    self.dist.broadcast(t.data, src)
                s = torch.tensor([self.step_count])
                self.dist.broadcast(s, src)
                self.step_count = int(s.item())

    # -------------------------------------------------------------- eval
    def evaluate_batch(self, images, labels):
        """(loss_sum, correct, probs) in inference mode (moving BN statistics)."""
        if images.dtype == torch.uint8:
            images = augment_cpu(images, train=False)
        with torch.no_grad():
            logits = self.model(images.float(), False)
            probs = torch.softmax(logits, 1)
            loss = torch.nn.functional.cross_entropy(logits, labels.long(), reduction="sum")
            correct = (logits.argmax(1) == labels.long()).float().sum()
        return float(loss), float(correct), probs


def make_backend(spec: ModelSpec, batch_size: int, *, device: str, weight_decay: float,
                 lr_schedule, optimizer: str = "mom", seed: int = 0, dist_ctx=None,
                 bucket_mb: float | None = None, use_graph: bool = False, global_batch=None,
                 input_mode: str = "auto", data_seed: int = 1234,
                 allreduce_dtype: str = "fp32"):
    """device: gpu | cpu | auto."""
    if device == "auto":
        device = "gpu" if torch.cuda.is_available() else "cpu"
    if device == "gpu":
        from .engine import Engine

        local = local_device_index()
        torch.cuda.set_device(local)
        eng = Engine(spec, batch_size, weight_decay=weight_decay, lr_schedule=lr_schedule,
                     optimizer=optimizer, device=torch.device("cuda", local), dist_ctx=dist_ctx,
                     bucket_mb=bucket_mb, seed=seed, input_mode=input_mode,
                     global_batch=global_batch, use_graph=use_graph, data_seed=data_seed,
                     allreduce_dtype=allreduce_dtype)
        return GPUBackend(eng, use_graph=use_graph)
    return CPUBackend(spec, batch_size, weight_decay=weight_decay, lr_schedule=lr_schedule,
                      optimizer=optimizer, seed=seed, dist_ctx=dist_ctx,
                      global_batch=global_batch, allreduce_dtype=allreduce_dtype)
