"""Flat parameter storage with TF variable names.

All trainables live in ONE contiguous fp32 buffer in TF creation order (so the
data-parallel gradient all-reduce works on contiguous bucket slices of one
buffer and the optimizer is a single launch); BN moving statistics live in a
second buffer.  ``views()`` exposes per-variable tensors under the reference's
names for checkpointing (utils/tensor_bundle.py) and for the CPU model.

Initialisers follow the reference graph:
  conv kernels  tf.variance_scaling_initializer() = truncated normal, fan_in,
                stddev = sqrt(1/fan_in)/0.87962566103423978, cut at 2 sigma
  dense kernel  glorot uniform, limit sqrt(6/(fan_in+fan_out)); bias 0
  BN            gamma 1, beta 0, moving_mean 0, moving_variance 1
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch

from .spec import ModelSpec

_TRUNC_NORMAL_STD_CORR = 0.87962566103423978


@dataclass
class Slot:
    name: str
    shape: tuple
    kind: str
    offset: int
    numel: int


class ParamStore:
    def __init__(self, spec: ModelSpec, device="cpu"):
        self.spec = spec
        self.train_slots: list[Slot] = []
        self.stat_slots: list[Slot] = []
        t_off = s_off = 0
        for p in spec.params:
            n = math.prod(p.shape)
            if p.trainable:
                self.train_slots.append(Slot(p.name, tuple(p.shape), p.kind, t_off, n))
                t_off += n
            else:
                self.stat_slots.append(Slot(p.name, tuple(p.shape), p.kind, s_off, n))
                s_off += n
        self.n_train = t_off
        self.n_stats = s_off
        self.by_name = {s.name: ("t", s) for s in self.train_slots}
        self.by_name.update({s.name: ("s", s) for s in self.stat_slots})
        self.master = torch.zeros(self.n_train, dtype=torch.float32, device=device)
        self.stats = torch.zeros(self.n_stats, dtype=torch.float32, device=device)
        self.global_step = 0

    # ------------------------------------------------------------ access
    def view(self, name: str) -> torch.Tensor:
        which, s = self.by_name[name]
        buf = self.master if which == "t" else self.stats
        return buf[s.offset:s.offset + s.numel].view(s.shape)

    def slot(self, name: str) -> Slot:
        return self.by_name[name][1]

    def views(self) -> dict[str, torch.Tensor]:
        return {name: self.view(name) for name in self.by_name}

    # ------------------------------------------------------------ init
    def initialize(self, seed: int = 0) -> None:
        """Deterministic TF-style init computed on the CPU (identical on every
        rank for the same seed; rank 0 broadcasts anyway)."""
        g = torch.Generator().manual_seed(seed)
        cpu_master = torch.zeros(self.n_train)
        cpu_stats = torch.zeros(self.n_stats)
        for s in self.train_slots:
            v = cpu_master[s.offset:s.offset + s.numel].view(s.shape)
            if s.kind == "conv":
                kh, kw, cin, _ = s.shape
                std = math.sqrt(1.0 / (kh * kw * cin)) / _TRUNC_NORMAL_STD_CORR
                v.copy_(_truncated_normal(s.shape, std, g))
            elif s.kind == "dense_kernel":
                fi, fo = s.shape
                lim = math.sqrt(6.0 / (fi + fo))
                v.copy_(torch.rand(s.shape, generator=g) * 2 * lim - lim)
            elif s.kind == "gamma":
                v.fill_(1.0)
            else:  # beta, dense_bias
                v.zero_()
        for s in self.stat_slots:
            v = cpu_stats[s.offset:s.offset + s.numel]
            v.fill_(1.0 if s.kind == "moving_variance" else 0.0)
        self.master.copy_(cpu_master)
        self.stats.copy_(cpu_stats)
        self.global_step = 0

    def state_dict(self) -> dict[str, torch.Tensor]:
        """name -> CPU fp32 tensor (TF layouts); plus 'global_step'."""
        d = {n: t.detach().cpu().clone() for n, t in self.views().items()}
        d["global_step"] = torch.tensor(self.global_step, dtype=torch.int64)
        return d

    def load_state_dict(self, d: dict[str, torch.Tensor], strict: bool = True) -> list[str]:
        missing = []
        for name in self.by_name:
            if name in d:
                self.view(name).copy_(torch.as_tensor(d[name]).reshape(self.slot(name).shape))
            else:
                missing.append(name)
        if strict and missing:
            raise KeyError(f"missing variables in checkpoint: {missing[:5]}...")
        if "global_step" in d:
            self.global_step = int(torch.as_tensor(d["global_step"]).item())
        return missing


def _truncated_normal(shape, std, g):
    """Rejection-resampled N(0, std) truncated at +-2 std (tf.truncated_normal)."""
    out = torch.randn(shape, generator=g)
    bad = out.abs() > 2.0
    while bool(bad.any()):
        out[bad] = torch.randn(int(bad.sum()), generator=g)
        bad = out.abs() > 2.0
    return out * std
