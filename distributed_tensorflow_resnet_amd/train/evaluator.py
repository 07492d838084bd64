"""Side-car evaluator (resnet_cifar_main.py:361-421, resnet_cifar_eval.py,
resnet_imagenet_eval.py).

Polls `train_dir` for the newest checkpoint, restores it into an inference
model (GPU: the engine's forward-only plan with moving-average BN; CPU: the
fp32 model), scores `eval_batch_count` batches, logs

    precision: 0.933, best precision: 0.936

and writes `Precision` / `Best_Precision` scalar summaries at the checkpoint's
global_step into `eval_dir`.  `eval_once` evaluates a single checkpoint and
returns; otherwise it sleeps `eval_interval_secs` (60 s in the reference)
between polls and skips checkpoints it has already scored.
"""
from __future__ import annotations

import time

import torch

from ..utils import tensor_bundle as tb
from ..utils.checkpoint import tf_to_state
from ..utils.records import EventWriter
from .hooks import log


class GPUInference:
    def __init__(self, spec, batch_size: int, device=None):
        from .engine import Engine, constant_lr

        self.engine = Engine(spec, batch_size, weight_decay=0.0, lr_schedule=constant_lr(0.0),
                             device=device, use_graph=False)
        self.plan = self.engine.build_eval_plan(batch_size)

    def load(self, tensors):
        tf_to_state(tensors, self.engine.params, None, strict=True)
        self.engine.repack()

    def run(self, images, labels):
        raw = images.dtype == torch.uint8
        n, full = images.shape[0], self.engine.N
        if n < full:
            # a short last batch (an eval pipeline's remainder, e.g. several loader
            # workers over 390-image ImageNet validation shards): the static plan runs
            # the full batch with the first image repeated, and the loss / correct count
            # are taken from the valid rows' probabilities
            pad = full - n
            images = torch.cat([images, images[:1].expand(pad, *images.shape[1:])])
            labels_p = torch.cat([labels, labels[:1].expand(pad)])
            _, _, probs = self.plan.run(images.to(self.engine.device),
                                        labels_p.to(self.engine.device), raw_u8=raw)
            p = probs[:n].float()
            y = labels.to(p.device).long()
            loss = float(-torch.log(p.gather(1, y[:, None]).clamp_min(1e-30)).sum())
            correct = float((p.argmax(1) == y).sum())
            return loss, correct, probs[:n]
        loss, correct, probs = self.plan.run(images.to(self.engine.device),
                                             labels.to(self.engine.device), raw_u8=raw)
        return loss, correct, probs


class CPUInference:
    def __init__(self, spec, batch_size: int):
        from .backends import CPUBackend
        from .engine import constant_lr

        self.backend = CPUBackend(spec, batch_size, weight_decay=0.0, lr_schedule=constant_lr(0.0))

    def load(self, tensors):
        tf_to_state(tensors, self.backend.store, None, strict=True)

    def run(self, images, labels):
        return self.backend.evaluate_batch(images, labels)


def make_inference(spec, batch_size: int, device: str = "auto"):
    if device == "auto":
        device = "gpu" if torch.cuda.is_available() else "cpu"
    return GPUInference(spec, batch_size) if device == "gpu" else CPUInference(spec, batch_size)


def evaluate_checkpoint(model, prefix: str, batches, eval_batch_count: int):
    """Restore `prefix`, score up to eval_batch_count batches -> (precision, loss, step)."""
    tensors = tb.read_bundle(prefix)
    model.load(tensors)
    step = int(tensors.get("global_step", 0))
    total = correct = loss = 0.0
    for i, (x, y) in enumerate(batches()):
        if i >= eval_batch_count:
            break
        l, c, _ = model.run(x, y)
        loss += l
        correct += c
        total += y.shape[0]
    return (correct / max(total, 1.0)), (loss / max(total, 1.0)), step


class SidecarEvaluator:
    def __init__(self, model, batches, train_dir: str, eval_dir: str | None,
                 eval_batch_count: int = 50, eval_once: bool = False,
                 interval_s: float = 60.0, exit_if_no_checkpoint: bool = False):
        self.model = model
        self.batches = batches
        self.train_dir = train_dir
        self.writer = EventWriter(eval_dir) if eval_dir else None
        self.count = eval_batch_count
        self.once = eval_once
        self.interval = interval_s
        self.exit_if_none = exit_if_no_checkpoint
        self.best = 0.0
        self.last_prefix = None
        self.history = []

    def run(self, max_polls: int | None = None):
        polls = 0
        while True:
            polls += 1
            prefix = tb.latest_checkpoint(self.train_dir)
            if prefix is None:
                log(f"INFO:tensorflow:No model to eval yet at {self.train_dir}")
                if self.exit_if_none or self.once:
                    return self.history
            elif prefix != self.last_prefix:
                prec, loss, step = evaluate_checkpoint(self.model, prefix, self.batches, self.count)
                self.best = max(self.best, prec)
                self.last_prefix = prefix
                self.history.append((step, prec, loss))
                log(f"INFO:tensorflow:loss: {loss:.3f}, precision: {prec:.3f}, "
                    f"best precision: {self.best:.3f}")
                if self.writer is not None:
                    self.writer.add_scalars(step, {"Precision": prec, "Best_Precision": self.best})
                    self.writer.flush()
                if self.once:
                    return self.history
            if max_polls is not None and polls >= max_polls:
                return self.history
            time.sleep(self.interval)
