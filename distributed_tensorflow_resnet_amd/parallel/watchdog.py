"""Communicator watchdog: failure detection for the data-parallel step.

SURVEY §5 (failure detection): "RCCL async-error polling + ncclCommAbort with a
watchdog timeout; the launcher restarts the job".  The reference has no such
code of its own; it leans on MonitoredTrainingSession's session recovery and
`stop_grace_period_secs` (/root/reference/resnet_imagenet_main.py:363) and on
`srun --no-kill` (/root/reference/mkl-scripts/run_dist_train_eval_daint.sh:203-205).

A dead peer leaves the surviving ranks blocked inside a collective -- on the
device for RCCL (the host then blocks in the next synchronisation), on the
comm stream's issue thread for the shm transport.  A daemon thread here:
  * polls ``comm.async_error()`` (ncclCommGetAsyncError; the shm transport's
    dead-peer / timeout state) every ``poll_s``;
  * tracks a heartbeat (``beat()`` after every completed step);
and on an async error, or when no step completed for ``timeout_s``
(``first_timeout_s`` before the first one: plan build, kernel load, rendezvous),
dumps every thread's stack, calls ``comm.abort()`` (ncclCommAbort: releases the
stuck collective kernels so the process can exit cleanly) and exits with
``EXIT_CODE`` -- parallel/launch.py --max_restarts then restarts the job, which
resumes from the latest checkpoint.
"""
from __future__ import annotations

import faulthandler
import os
import sys
import threading
import time

EXIT_CODE = 3


class CommWatchdog:
    def __init__(self, comm=None, timeout_s: float = 600.0, first_timeout_s: float | None = None,
                 poll_s: float | None = None, exit_code: int = EXIT_CODE, _exit=os._exit,
                 log=None):
        self.comm = comm
        self.timeout_s = float(timeout_s)
        self.first_timeout_s = float(first_timeout_s or max(600.0, 4 * self.timeout_s))
        self.poll_s = poll_s or min(1.0, max(self.timeout_s / 20, 0.01))
        self.exit_code = exit_code
        self._exit = _exit
        self._log = log or (lambda m: print(m, file=sys.stderr, flush=True))
        self._last = time.monotonic()
        self._beats = 0
        self._stop = threading.Event()
        self._thread = None
        self.fired = None   # the reason, once fired

    def start(self):
        self._last = time.monotonic()
        self._thread = threading.Thread(target=self._watch, name="dtr-comm-watchdog", daemon=True)
        self._thread.start()
        return self

    def beat(self):
        self._beats += 1
        self._last = time.monotonic()

    def stop(self):
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()
        return False

    def check(self) -> str | None:
        """One poll: the reason to fire, or None."""
        if self.comm is not None:
            try:
                err = int(self.comm.async_error())
            except Exception as e:   # noqa: BLE001
                return f"communicator async_error() raised: {e}"
            if err != 0:
                return f"communicator async error {err} ({self.comm.transport})"
        limit = self.timeout_s if self._beats else self.first_timeout_s
        idle = time.monotonic() - self._last
        if idle > limit:
            return f"no step completed for {idle:.0f}s (limit {limit:.0f}s)"
        return None

    def _watch(self):
        while not self._stop.wait(self.poll_s):
            why = self.check()
            if why is None:
                continue
            self.fired = why
            self._log(f"[watchdog] {why}: aborting the communicator and exiting "
                      f"({self.exit_code}) for a restart")
            faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
            sys.stderr.flush()
            if self.comm is not None:
                try:
                    self.comm.abort()
                except Exception:   # noqa: BLE001
                    pass
            self._exit(self.exit_code)
            return
