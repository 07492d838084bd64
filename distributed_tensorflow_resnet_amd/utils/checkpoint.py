"""tf.train.Saver / CheckpointSaverHook equivalent over the tensor-bundle codec.

Variables saved exactly as the reference's MonitoredTrainingSession did
(403 entries for CIFAR ResNet-50): every trainable
under its TF name (HWIO conv kernels, BN gamma/beta, dense kernel/bias), its
``<name>/Momentum`` optimizer slot, the BN moving statistics and the int64
``global_step``.  ``max_to_keep`` = 5, the ``checkpoint`` state file lists the
retained prefixes, files are written to temporaries and renamed (a killed
writer never leaves a half checkpoint that restore would pick up).
"""
from __future__ import annotations

import glob
import os

import numpy as np
import torch

from . import tensor_bundle as tb


def state_to_tf(store, momentum: torch.Tensor | None, global_step: int) -> dict[str, np.ndarray]:
    """ParamStore (+flat momentum in the same layout) -> {TF name: array}."""
    out: dict[str, np.ndarray] = {}
    master = store.master.detach().float().cpu().numpy()
    stats = store.stats.detach().float().cpu().numpy()
    mom = momentum.detach().float().cpu().numpy() if momentum is not None else None
    for s in store.train_slots:
        out[s.name] = master[s.offset:s.offset + s.numel].reshape(s.shape).copy()
        if mom is not None:
            out[f"{s.name}/Momentum"] = mom[s.offset:s.offset + s.numel].reshape(s.shape).copy()
    for s in store.stat_slots:
        out[s.name] = stats[s.offset:s.offset + s.numel].reshape(s.shape).copy()
    out["global_step"] = np.array(int(global_step), dtype=np.int64)
    return out


def tf_to_state(tensors: dict, store, momentum: torch.Tensor | None = None,
                strict: bool = True) -> int:
    """Load {TF name: array} into the ParamStore (+momentum); returns global_step."""
    missing = []
    for s in store.train_slots + store.stat_slots:
        if s.name not in tensors:
            missing.append(s.name)
            continue
        a = np.asarray(tensors[s.name], dtype=np.float32).reshape(s.shape)
        buf = store.master if s in store.train_slots else store.stats
        buf.data[s.offset:s.offset + s.numel].copy_(torch.from_numpy(a.reshape(-1)))
    if momentum is not None:
        for s in store.train_slots:
            k = f"{s.name}/Momentum"
            if k in tensors:
                a = np.asarray(tensors[k], dtype=np.float32).reshape(-1)
                momentum.data[s.offset:s.offset + s.numel].copy_(torch.from_numpy(a))
    if strict and missing:
        raise KeyError(f"checkpoint lacks {len(missing)} variables, e.g. {missing[:3]}")
    gs = int(np.asarray(tensors.get("global_step", 0)))
    store.global_step = gs
    return gs


class Saver:
    def __init__(self, directory: str, max_to_keep: int = 5, basename: str = "model.ckpt"):
        self.dir = directory
        self.max_to_keep = max_to_keep
        self.basename = basename
        os.makedirs(directory, exist_ok=True)
        st = tb.read_checkpoint_state(directory)
        self.kept: list[str] = []
        if st:
            for p in st["all_model_checkpoint_paths"]:
                q = p if os.path.exists(p + ".index") else os.path.join(directory, os.path.basename(p))
                if os.path.exists(q + ".index"):
                    self.kept.append(q)

    def save(self, tensors: dict, global_step: int) -> str:
        prefix = os.path.join(self.dir, f"{self.basename}-{int(global_step)}")
        tb.write_bundle(prefix, tensors)
        if prefix in self.kept:
            self.kept.remove(prefix)
        self.kept.append(prefix)
        while len(self.kept) > self.max_to_keep:
            old = self.kept.pop(0)
            for f in glob.glob(old + ".*"):
                try:
                    os.remove(f)
                except OSError:
                    pass
        tb.write_checkpoint_state(self.dir, prefix, self.kept)
        return prefix

    def latest(self) -> str | None:
        return tb.latest_checkpoint(self.dir)

    @staticmethod
    def restore(prefix: str) -> dict[str, np.ndarray]:
        return tb.read_bundle(prefix)
