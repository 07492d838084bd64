"""Session hooks with the reference's cadence and keys (SURVEY §5 metrics row).

resnet_cifar_main.py:288-324 / resnet_imagenet_main.py:292-329 install:
  SummarySaverHook(save_steps=100, output_dir=log_dir)   cross_entropy, cost,
                                                         learning_rate, Precision
  LoggingTensorHook(every_n_iter=20 | 40)                step, loss, precision, lr
  StopAtStepHook(last_step=train_steps)
  _LearningRateSetterHook                                piecewise schedule
and MonitoredTrainingSession adds StepCounterHook (global_step/sec every 100
steps, the README's "stp/sec") and CheckpointSaverHook (every 60 s on the
Horovod path, every 1000 steps on the PS path).

Hooks only read device metrics when they are due (a read synchronises).
"""
from __future__ import annotations

import json
import math
import os
import sys
import time


class Hook:
    def begin(self, session):
        pass

    def before_run(self, session):
        pass

    def after_run(self, session, step: int):
        """`step` = global_step after this run."""

    def wants_metrics(self, session, step: int) -> bool:
        """Will after_run(step) read session.metrics()?  The session then asks the
        backend for the exact `cost` of that step (its weight-decay term is only
        computed on such steps)."""
        return False

    def end(self, session):
        pass


def _every(n: int, step: int) -> bool:
    return n > 0 and step % n == 0


def log(msg: str):
    print(msg, flush=True)


class LearningRateSetterHook(Hook):
    """The LR itself is evaluated on the device from global_step (engine
    LRSchedule); this hook mirrors it on the host for logs/summaries."""

    def __init__(self, schedule):
        self.schedule = schedule
        self.lr = schedule.init

    def before_run(self, session):
        self.lr = self.schedule.at(session.global_step)


class LoggingTensorHook(Hook):
    def __init__(self, every_n_iter: int = 20, precision_key: str = "precision"):
        self.n = every_n_iter
        self.key = precision_key

    def wants_metrics(self, session, step):
        return _every(self.n, step) and session.is_chief

    def after_run(self, session, step):
        if self.n > 0 and step % self.n == 0 and session.is_chief:
            m = session.metrics()
            log(f"INFO:tensorflow:step = {m['global_step']}, loss = {m['cost']:.6f}, "
                f"{self.key} = {m['precision']:.4f}, lr = {m['lr']:.6g}")


class StepCounterHook(Hook):
    """global_step/sec + examples/sec every `every_n_steps` (tf StepCounterHook)."""

    def __init__(self, every_n_steps: int = 100, batch_size: int = 1, writer=None):
        self.n = every_n_steps
        self.batch = batch_size
        self.writer = writer
        self.t0 = None
        self.s0 = None
        self.last_rate = None

    def begin(self, session):
        self.t0, self.s0 = time.perf_counter(), session.global_step

    def after_run(self, session, step):
        if self.n > 0 and step - self.s0 >= self.n:
            session.synchronize()
            t = time.perf_counter()
            rate = (step - self.s0) / (t - self.t0)
            self.last_rate = rate
            if session.is_chief:
                log(f"INFO:tensorflow:global_step/sec: {rate:.4f}  "
                    f"(examples/sec: {rate * self.batch:.1f})")
                if self.writer is not None:
                    self.writer.add_scalars(step, {"global_step/sec": rate,
                                                   "examples/sec": rate * self.batch})
            self.t0, self.s0 = t, step


class SummarySaverHook(Hook):
    def __init__(self, writer, save_steps: int = 100, precision_tag: str = "Precision"):
        self.writer = writer
        self.n = save_steps
        self.tag = precision_tag

    def wants_metrics(self, session, step):
        return self.writer is not None and _every(self.n, step) and session.is_chief

    def after_run(self, session, step):
        if self.writer is not None and self.n > 0 and step % self.n == 0 and session.is_chief:
            m = session.metrics()
            self.writer.add_scalars(step, {"cross_entropy": m["cross_entropy"], "cost": m["cost"],
                                           "learning_rate": m["lr"], self.tag: m["precision"]})
            self.writer.flush()

    def end(self, session):
        if self.writer is not None:
            self.writer.flush()


class JsonlMetricsHook(Hook):
    """Scalars to <dir>/metrics.jsonl (machine-readable twin of the event file)."""

    def __init__(self, path: str, every: int = 100):
        self.path = path
        self.n = every

    def wants_metrics(self, session, step):
        return _every(self.n, step) and session.is_chief

    def after_run(self, session, step):
        if self.n > 0 and step % self.n == 0 and session.is_chief:
            m = dict(session.metrics())
            m["time"] = time.time()
            eng = getattr(session.backend, "engine", None)
            if eng is not None:   # which step ran, and why the persistent one did not
                m["step_path"] = "persistent" if getattr(eng, "persist", False) else "per-layer"
                m["persist_disabled_reason"] = getattr(eng, "persist_reason", "") or None
            os.makedirs(os.path.dirname(self.path) or ".", exist_ok=True)
            with open(self.path, "a") as fh:
                fh.write(json.dumps(m) + "\n")


class StopAtStepHook(Hook):
    def __init__(self, last_step: int):
        self.last_step = last_step

    def begin(self, session):
        if session.global_step >= self.last_step:
            session.request_stop()

    def after_run(self, session, step):
        if step >= self.last_step:
            session.request_stop()


class CheckpointSaverHook(Hook):
    """Chief-only, every `save_steps` steps and/or `save_secs` seconds, and at end."""

    def __init__(self, saver, save_steps: int = 0, save_secs: float = 0.0):
        self.saver = saver
        self.steps = save_steps
        self.secs = save_secs
        self.last_t = time.time()
        self.last_step = None

    def begin(self, session):
        self.last_step = session.global_step

    def _save(self, session, step):
        if session.is_chief:
            p = self.saver.save(session.state_tensors(), step)
            log(f"INFO:tensorflow:Saving checkpoints for {step} into {p}.")
        self.last_t = time.time()
        self.last_step = step

    def after_run(self, session, step):
        due = (self.steps > 0 and step % self.steps == 0) or \
              (self.secs > 0 and time.time() - self.last_t >= self.secs)
        # with a PersistHealthHook (multi-rank persistent step) only steps whose health
        # every rank has agreed are saved: a due time-based save waits for the next one
        if due and step != self.last_step and getattr(session, "health_step", step) == step:
            self._save(session, step)

    def end(self, session):
        if session.global_step != self.last_step:
            self._save(session, session.global_step)


class PersistHealthHook(Hook):
    """Every rank, multi-rank jobs on the persistent CIFAR step: every `every` steps and at
    the end, agree over the process group whether ANY rank's persistent launch failed a
    grid barrier (its error flag).  A failing rank's gradients still reach the all-reduce,
    so every replica holds garbage after it, while the checkpoint is written by the chief,
    whose own flag is clean: the agreement raises PersistentStepError on every rank (each
    writes the persist_fault marker, driver.py), and the checkpoint hook saves only agreed
    steps (session.health_step).  A collective, so every rank runs it at the same steps."""

    def __init__(self, ctx, every: int):
        self.ctx, self.every = ctx, max(1, int(every))

    def begin(self, session):
        session.health_step = -1

    def _agree(self, session, step):
        from .engine import PersistentStepError

        eng = session.backend.engine
        bad = eng.persist_error()
        if not self.ctx._agree(not bad):
            raise PersistentStepError(
                f"a persistent-step grid barrier timed out on {'this' if bad else 'another'} "
                f"rank by step {step}; every replica's state is invalid")
        session.health_step = step

    def after_run(self, session, step):
        if step % self.every == 0:
            self._agree(session, step)

    def end(self, session):
        self._agree(session, session.global_step)


class NanGuardHook(Hook):
    """tf.check_numerics analogue on the loss (opt-in: reads metrics every step)."""

    def __init__(self, every: int = 1):
        self.n = every

    def wants_metrics(self, session, step):
        return _every(self.n, step)

    def after_run(self, session, step):
        if step % self.n == 0:
            c = session.metrics()["cost"]
            if not math.isfinite(c):
                raise FloatingPointError(f"loss is {c} at step {step}")


class StepWatchdogHook(Hook):
    """Failure detection for hung steps and communicator errors (SURVEY §5
    failure-detection row), parallel/watchdog.py's CommWatchdog driven by the
    session: a daemon thread polls the native communicator's async error
    (ncclCommGetAsyncError, or the shm transport's dead-peer state) and the time
    since the last completed step (a dead peer leaves the others blocked inside a
    collective; a faulting kernel can leave the host blocked in a
    synchronisation).  On either it dumps every thread's stack, aborts the
    communicator (ncclCommAbort) and exits with code 3 so the launcher
    (parallel/launch.py --max_restarts) restarts the job from the latest
    checkpoint.  The first step gets `first_timeout_s` (plan build, kernel
    loading, rendezvous)."""

    EXIT_CODE = 3

    def __init__(self, timeout_s: float, first_timeout_s: float | None = None,
                 _exit=os._exit, poll_s: float | None = None, comm=None):
        from ..parallel.watchdog import CommWatchdog

        self.wd = CommWatchdog(comm, timeout_s, first_timeout_s,
                               poll_s or min(5.0, max(float(timeout_s) / 10, 0.01)),
                               self.EXIT_CODE, _exit, log)
        self.timeout_s = self.wd.timeout_s
        self.first_timeout_s = self.wd.first_timeout_s

    @property
    def fired(self) -> bool:
        return self.wd.fired is not None

    def begin(self, session):
        if self.wd.comm is None and session is not None:
            eng = getattr(getattr(session, "backend", None), "engine", None)
            self.wd.comm = getattr(eng, "comm", None)
        self.wd.start()

    def after_run(self, session, step):
        self.wd.beat()

    def end(self, session):
        self.wd.stop()


class FaultInjectionHook(Hook):
    """Kills this rank at a given step (tests of checkpoint/resume and of the
    launcher's failure handling).  Env DTR_FAULT_KILL_STEP / DTR_FAULT_KILL_RANK
    or flags --fault_kill_step / --fault_kill_rank."""

    def __init__(self, step: int, rank: int):
        self.step, self.rank = step, rank

    def after_run(self, session, step):
        if step == self.step and session.rank == self.rank:
            log(f"[fault-injection] rank {self.rank} exiting at step {step}")
            sys.stdout.flush()
            os._exit(17)


class ProfilerHook(Hook):
    """Per-phase device timing (forward / backward+allreduce / optimizer) over a
    step window, using the backend's phase timer (HIP events); `profile_steps`
    'a:b' measures steps a..b-1 and prints a table."""

    def __init__(self, spec: str):
        a, b = spec.split(":")
        self.a, self.b = int(a), int(b)
        self.acc = {}
        self.n = 0

    def before_run(self, session):
        s = session.global_step
        session.backend.profile_phases = self.a <= s < self.b

    def after_run(self, session, step):
        t = getattr(session.backend, "last_phase_ms", None)
        if t and self.a < step <= self.b:
            for k, v in t.items():
                self.acc[k] = self.acc.get(k, 0.0) + v
            self.n += 1
        if step == self.b and self.n and session.is_chief:
            log("phase timing (ms/step): " + ", ".join(
                f"{k}={v / self.n:.3f}" for k, v in self.acc.items()))
