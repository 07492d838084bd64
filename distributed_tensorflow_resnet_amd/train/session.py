"""MonitoredTrainingSession analogue (resnet_cifar_main.py:326-358).

    with TrainingSession(backend, hooks, checkpoint_dir=..., is_chief=...) as sess:
        while not sess.should_stop():
            sess.run()

On entry: restore the latest checkpoint of `checkpoint_dir` if any (every rank
reads it, then rank 0's state is broadcast so all replicas start identical --
BroadcastGlobalVariablesHook(0)); hooks' begin().  Each run(): fetch the next
batch from the feeder (copied into the backend's static input buffers),
one training step (graph replay on GPU), hooks' after_run().
"""
from __future__ import annotations

import time

from ..utils import tensor_bundle as tb
from ..utils.checkpoint import Saver
from .hooks import log


class TrainingSession:
    def __init__(self, backend, hooks=(), chief_only_hooks=(), checkpoint_dir: str | None = None,
                 is_chief: bool = True, rank: int = 0, feeder=None, restore: bool = True):
        self.backend = backend
        self.is_chief = is_chief
        self.rank = rank
        self.hooks = list(hooks) + (list(chief_only_hooks) if is_chief else [])
        self.checkpoint_dir = checkpoint_dir
        self.feeder = feeder
        self._stop = False
        self._metrics_cache = None
        self._metrics_step = -1
        if restore and checkpoint_dir:
            self._maybe_restore()
        backend.broadcast_parameters(0)

    # ------------------------------------------------------------ state
    @property
    def global_step(self) -> int:
        return self.backend.global_step

    def _maybe_restore(self):
        prefix = tb.latest_checkpoint(self.checkpoint_dir)
        if prefix:
            tensors = Saver.restore(prefix)
            self.backend.load_state(tensors)
            log(f"INFO:tensorflow:Restoring parameters from {prefix} "
                f"(global_step={self.backend.global_step})")

    def state_tensors(self):
        return self.backend.state_tensors()

    def metrics(self) -> dict:
        if self._metrics_step != self.global_step:
            self._metrics_cache = self.backend.metrics()
            self._metrics_step = self.global_step
        return self._metrics_cache

    def synchronize(self):
        self.backend.synchronize()

    def request_stop(self):
        self._stop = True

    def should_stop(self) -> bool:
        return self._stop

    # ------------------------------------------------------------ loop
    def __enter__(self):
        for h in self.hooks:
            h.begin(self)
        return self

    def run(self):
        for h in self.hooks:
            h.before_run(self)
        if self.feeder is not None:
            try:
                images, labels = next(self.feeder)
            except StopIteration:
                self.request_stop()
                return
            self.backend.set_batch(images, labels)
        nxt = self.global_step + 1
        self.backend.step(need_cost=any(h.wants_metrics(self, nxt) for h in self.hooks))
        step = self.global_step
        for h in self.hooks:
            h.after_run(self, step)

    def __exit__(self, exc_type, exc, tb_):
        if exc_type is None:
            for h in self.hooks:
                h.end(self)
        self.backend.synchronize()
        return False


def run_training(session: TrainingSession, max_wall_s: float | None = None) -> int:
    t0 = time.time()
    with session:
        while not session.should_stop():
            session.run()
            if max_wall_s is not None and time.time() - t0 > max_wall_s:
                session.request_stop()
    return session.global_step
