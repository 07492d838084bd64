"""Entrypoint logic shared by resnet_cifar_main.py / resnet_imagenet_main.py
(and the legacy trainer names).  Mirrors the reference's main() (resnet_cifar_
main.py:424-494, resnet_imagenet_main.py:460-531):

  mode=train           synchronous data-parallel training (one process per GPU,
                       RCCL all-reduce) with the LR / logging / summary /
                       step-counter / checkpoint / stop-at-step hooks
  mode=eval            the side-car evaluator polling --train_dir
  mode=train_and_eval  train, then evaluate the final checkpoint

Multi-GPU: launch with `python -m distributed_tensorflow_resnet_amd.parallel.launch
--nproc N resnet_cifar_main.py ...` or torchrun; rank/world come from the env.
"""
from __future__ import annotations

import os
import queue
import threading
import time

import torch

from ..models.spec import build_spec
from ..parallel.dist import DistContext, apply_cu_partition, local_device_index
from ..utils.checkpoint import Saver
from ..utils.flags import build_parser, warn_unsupported
from ..utils.records import EventWriter
from . import hooks as H
from .backends import make_backend
from .engine import (PersistentStepError, cifar_lr_schedule, imagenet_lr_schedule,
                     lr_values_scaled, scaled)
from .evaluator import SidecarEvaluator, make_inference
from .session import TrainingSession, run_training


# written into --train_dir when a persistent CIFAR launch failed: restarts use the per-layer plan
PERSIST_FAULT_MARKER = "persist_fault"


class Prefetcher:
    """Background thread that keeps `depth` host batches ready (pinned when a GPU exists)."""

    def __init__(self, it, depth: int = 2):
        self.q: queue.Queue = queue.Queue(maxsize=depth)
        self.pin = torch.cuda.is_available()
        self.t = threading.Thread(target=self._run, args=(it,), daemon=True)
        self.t.start()

    def _run(self, it):
        try:
            for x, y in it:
                if self.pin:
                    x, y = x.pin_memory(), y.pin_memory()
                self.q.put((x, y))
        except Exception as e:  # surface loader errors in the training thread
            self.q.put(e)
        self.q.put(None)

    def __iter__(self):
        return self

    def __next__(self):
        item = self.q.get()
        if item is None:
            raise StopIteration
        if isinstance(item, Exception):
            raise item
        return item


def _train_batches(flags, spec, rank, world, u8=False):
    if flags.synthetic:
        return None
    if spec.dataset.startswith("cifar"):
        from ..data.cifar import CifarData

        data = CifarData(flags.train_data_path, spec.dataset, train=True)
        return data.batches(flags.batch_size, num_epochs=flags.num_epochs, seed=flags.seed,
                            rank=rank, world=world)
    from ..data import imagenet

    return imagenet.input_fn(True, flags.train_data_path, flags.batch_size,
                             num_epochs=flags.num_epochs, rank=rank, world=world,
                             workers=flags.num_parallel_calls, seed=flags.seed, u8=u8)


def _eval_batches_factory(flags, spec):
    bs = flags.eval_batch_size
    if flags.synthetic or not flags.eval_data_path:
        if spec.dataset.startswith("cifar"):
            from ..data.cifar import synthetic_batches
        else:
            from ..data.imagenet import synthetic_batches
        return lambda: synthetic_batches(bs, spec.num_classes, seed=123)
    if spec.dataset.startswith("cifar"):
        from ..data.cifar import CifarData

        data = CifarData(flags.eval_data_path, spec.dataset, train=False)
        return lambda: data.batches(bs, shuffle=False, num_epochs=1)
    from ..data import imagenet

    return lambda: imagenet.input_fn(False, flags.eval_data_path, bs, num_epochs=1,
                                     workers=flags.num_parallel_calls)


def run_eval(flags, spec, device: str):
    model = make_inference(spec, flags.eval_batch_size, device)
    ev = SidecarEvaluator(model, _eval_batches_factory(flags, spec), flags.train_dir,
                          flags.eval_dir or None, flags.eval_batch_count, flags.eval_once,
                          flags.eval_interval_secs,
                          exit_if_no_checkpoint=not spec.dataset.startswith("cifar"))
    return ev.run()


def persist_fault_policy(flags) -> str:
    """The persist_fault marker's lifecycle at start-up: '' when this attempt may select
    the persistent CIFAR step, else why not (the marker left by an attempt whose grid
    barrier timed out: DTR_TUNE gets persist=0 for this process and its children, and
    the reason is logged and written into metrics.jsonl through the engine's
    persist_reason).  --reset_persist_fault deletes the marker first."""
    if not flags.train_dir:
        return ""
    path = os.path.join(flags.train_dir, PERSIST_FAULT_MARKER)
    if flags.reset_persist_fault and os.path.exists(path):
        try:
            os.remove(path)
        except FileNotFoundError:   # another rank removed it first
            pass
        H.log(f"--reset_persist_fault: removed {path}; the persistent step may be selected again")
    if not os.path.exists(path):
        return ""
    try:
        with open(path) as fh:
            why = fh.read().strip().splitlines()[0]
    except (OSError, IndexError):
        why = "(unreadable)"
    os.environ["DTR_TUNE"] = ",".join(filter(None, [os.environ.get("DTR_TUNE", ""), "persist=0"]))
    reason = f"{PERSIST_FAULT_MARKER} in {flags.train_dir}: {why}"
    H.log(f"persistent step disabled: {reason} (a previous attempt's grid barrier timed out; "
          "--reset_persist_fault to retry it)")
    return reason


def main(argv=None, kind: str = "cifar") -> int:
    flags = build_parser(kind).parse_args(argv)
    # DTR_CU_PARTITION (several ranks on one GPU): the CU mask before the first HIP call
    apply_cu_partition()
    warn_unsupported(flags, H.log)
    if flags.job_name == "ps":
        return 0
    spec = build_spec(flags.dataset, flags.resnet_size, flags.num_classes)
    device = flags.device
    if device == "auto":
        device = "gpu" if torch.cuda.is_available() else "cpu"
    if flags.mode == "eval":
        run_eval(flags, spec, device)
        return 0

    # ---------------------------------------------------------------- train
    # a previous attempt's persistent CIFAR step failed (a grid barrier timed out): this
    # attempt runs the launch-per-layer plan (every rank reads the same marker, and the
    # engine agrees the choice over c10d anyway)
    fault_reason = persist_fault_policy(flags)
    dev = None
    if device == "gpu":
        local = local_device_index()
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    from .persist import OVERLAP_RESERVE_CUS
    # CIFAR: RCCL's channels capped at the persistent overlap plan's CU reserve (DistContext)
    ctx = DistContext(device=dev, timeout_s=flags.comm_timeout_secs,
                      rccl_max_channels=(OVERLAP_RESERVE_CUS if spec.dataset.startswith("cifar")
                                         else None))
    dp_ctx = None if flags.variable_update == "independent" else ctx
    rank, world = ctx.rank, ctx.world_size
    sched = cifar_lr_schedule() if spec.dataset.startswith("cifar") else imagenet_lr_schedule()
    sched = lr_values_scaled(scaled(sched, flags.lr_schedule_scale), flags.lr_value_scale)
    # real ImageNet on the GPU: uint8 crops from the workers, flip/mean/bf16 pack on device
    u8 = device == "gpu" and spec.dataset == "imagenet" and not flags.synthetic
    backend = make_backend(spec, flags.batch_size, device=device, weight_decay=flags.weight_decay,
                           lr_schedule=sched, optimizer=flags.optimizer, seed=flags.seed,
                           dist_ctx=dp_ctx, bucket_mb=flags.bucket_mb, use_graph=flags.use_graph,
                           data_seed=1234 + rank, allreduce_dtype=flags.allreduce_dtype,
                           input_mode="imagenet_u8" if u8 else "auto")
    eng = getattr(backend, "engine", None)
    if fault_reason and eng is not None and not eng.persist:
        eng.persist_reason = fault_reason
    it = _train_batches(flags, spec, rank, world, u8=u8)
    feeder = None
    if it is None:
        if device == "gpu":
            backend.engine.fill_synthetic(seed=flags.seed + rank)
        else:
            if spec.dataset.startswith("cifar"):
                from ..data.cifar import synthetic_batches
            else:
                from ..data.imagenet import synthetic_batches
            feeder = synthetic_batches(flags.batch_size, spec.num_classes, seed=flags.seed + rank)
    else:
        feeder = Prefetcher(it)

    is_chief = rank == 0
    writer = EventWriter(flags.log_dir) if (flags.log_dir and is_chief) else None
    gb = flags.batch_size * world
    prec_key = "precision" if spec.dataset.startswith("cifar") else "training precision"
    hooks = [H.LearningRateSetterHook(sched),
             H.LoggingTensorHook(flags.log_every, prec_key),
             H.StepCounterHook(100, gb, writer),
             H.StopAtStepHook(flags.train_steps)]
    chief_hooks = []
    if writer is not None:
        chief_hooks.append(H.SummarySaverHook(writer, flags.summary_every,
                                              "Precision" if spec.dataset.startswith("cifar")
                                              else "Training Precision"))
        chief_hooks.append(H.JsonlMetricsHook(os.path.join(flags.log_dir, "metrics.jsonl"),
                                              flags.summary_every))
    if flags.train_dir:
        saver = Saver(flags.train_dir, flags.max_to_keep)
        chief_hooks.append(H.CheckpointSaverHook(saver, flags.save_checkpoint_steps,
                                                 flags.save_checkpoint_secs))
    if eng is not None and eng.persist and world > 1 and dp_ctx is not None:
        # every rank agrees the persistent launches' health before saves (and at the end)
        hooks.append(H.PersistHealthHook(ctx, flags.save_checkpoint_steps or flags.log_every))
    if flags.check_numerics:
        hooks.append(H.NanGuardHook())
    ks = int(os.environ.get("DTR_FAULT_KILL_STEP", flags.fault_kill_step))
    if ks >= 0:
        hooks.append(H.FaultInjectionHook(ks, int(os.environ.get("DTR_FAULT_KILL_RANK",
                                                                 flags.fault_kill_rank))))
    if flags.profile_steps:
        hooks.append(H.ProfilerHook(flags.profile_steps))
    # multi-rank jobs always watch the step and the communicator's async error
    wd_secs = flags.step_watchdog_secs or (flags.comm_timeout_secs if world > 1 else 0.0)
    if wd_secs > 0:
        hooks.append(H.StepWatchdogHook(wd_secs, comm=getattr(getattr(backend, "engine", None),
                                                              "comm", None)))
    sess = TrainingSession(backend, hooks, chief_hooks, checkpoint_dir=flags.train_dir or None,
                           is_chief=is_chief, rank=rank, feeder=feeder)
    t0 = time.time()
    steps0 = sess.global_step
    try:
        final = run_training(sess)
    except PersistentStepError as e:
        # fail the job, not the model: no checkpoint of this state is written (the session
        # skips the hooks' end() on an exception); the launcher (--max_restarts) restarts
        # from the last good checkpoint and the marker puts the restart on the per-layer plan
        H.log(f"FATAL: {e}; exiting with code {H.StepWatchdogHook.EXIT_CODE} for a restart")
        if flags.train_dir:   # whichever rank faulted (every rank, once agreed)
            os.makedirs(flags.train_dir, exist_ok=True)
            tmp = os.path.join(flags.train_dir, f".{PERSIST_FAULT_MARKER}.{rank}")
            with open(tmp, "w") as fh:
                fh.write(f"rank {rank} at step {sess.global_step}: {e}\n")
            os.replace(tmp, os.path.join(flags.train_dir, PERSIST_FAULT_MARKER))
        return H.StepWatchdogHook.EXIT_CODE
    dt = time.time() - t0
    if is_chief:
        H.log(f"training done: global_step={final}, {final - steps0} steps in {dt:.1f}s")
    if writer is not None:
        writer.close()
    if flags.mode == "train_and_eval" and is_chief and flags.train_dir:
        flags.eval_once = True
        run_eval(flags, spec, device)
    ctx.shutdown()
    return 0
