"""fp32 PyTorch (autograd) execution of a ModelSpec with TF semantics.

This is the CPU compute path (BASELINE config 1, `resnet_single.py`) and the
end-to-end oracle the GPU engine is tested against.  Parameters are views into
a ParamStore's flat buffers, so the same TF-named checkpoint serves both paths.
NHWC throughout; conv kernels HWIO.
"""
from __future__ import annotations

import torch

from ..ops import reference as ref
from .params import ParamStore
from .spec import ModelSpec


class _Q(torch.autograd.Function):
    """Round to bf16 in forward (optional) and the gradient in backward."""

    @staticmethod
    def forward(ctx, x, fwd: bool):
        return x.to(torch.bfloat16).float() if fwd else x.clone()

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).float(), None


class _W(torch.autograd.Function):
    """Round a weight to bf16 in forward; straight-through gradient."""

    @staticmethod
    def forward(ctx, w):
        return w.to(torch.bfloat16).float()

    @staticmethod
    def backward(ctx, g):
        return g


class TorchResNet:
    """``emulate_bf16=True`` rounds values and gradients to bf16 exactly where
    the GPU engine stores them (conv outputs, BN-ReLU outputs feeding MFMA,
    pooled features, logits' gradient, weights), keeping fp32 arithmetic --
    the like-for-like oracle for the engine's end-to-end test."""

    def __init__(self, spec: ModelSpec, store: ParamStore, emulate_bf16: bool = False):
        self.spec = spec
        self.store = store
        self.emu = emulate_bf16
        self.master = store.master  # flat leaf for autograd
        self.master.requires_grad_(True)

    def _q(self, x, fwd=True):
        return _Q.apply(x, fwd) if self.emu else x

    def _p(self, name):
        s = self.store.slot(name)
        return self.master[s.offset:s.offset + s.numel].view(s.shape)

    def _bn_relu(self, x, bn_name, training):
        g = self._p(f"{bn_name}/gamma")
        b = self._p(f"{bn_name}/beta")
        mm = self.store.view(f"{bn_name}/moving_mean")
        mv = self.store.view(f"{bn_name}/moving_variance")
        if training:
            y, mean, _, uvar = ref.batch_norm_train(x, g, b)
            with torch.no_grad():
                mm.copy_(ref.moving_update(mm, mean.detach()))
                mv.copy_(ref.moving_update(mv, uvar.detach()))
        else:
            y = ref.batch_norm_eval(x, g, b, mm, mv)
        return torch.relu(y)

    def _conv(self, x, c):
        w = self._p(f"{c.name}/kernel")
        if self.emu:
            w = _W.apply(w)
        return ref.conv2d(x, w, c.stride)

    def __call__(self, images_nhwc: torch.Tensor, is_training: bool) -> torch.Tensor:
        """Logits for NHWC float images (3 channels)."""
        spec = self.spec
        q = self._q
        x = q(self._conv(q(images_nhwc), spec.stem))
        if spec.maxpool:
            x = q(ref.max_pool_same(x, 3, 2))
        for b in spec.blocks:
            shortcut = x
            a = q(self._bn_relu(x, b.bns[0].name, is_training))
            if b.proj is not None:
                shortcut = q(self._conv(a, b.proj))
            h = a
            for j, c in enumerate(b.convs):
                if j > 0:
                    h = q(self._bn_relu(h, b.bns[j].name, is_training))
                h = self._conv(h, c)
                if j < len(b.convs) - 1:
                    h = q(h)
            x = q(h + shortcut)
        x = q(self._bn_relu(x, spec.final_bn.name, is_training), False)
        x = q(x.mean(dim=(1, 2)))
        wd = self._p("dense/kernel")
        if self.emu:
            wd = _W.apply(wd)
        return q(x @ wd + self._p("dense/bias"), False)

    def loss(self, logits, labels, weight_decay: float):
        """cost = xent + wd * sum(l2_loss(v) for v in trainables) (resnet_model.py:78-86)."""
        xent = ref.softmax_cross_entropy(logits, labels)
        l2 = (self.master * self.master).sum() * 0.5
        return xent, xent + weight_decay * l2
