"""`resnet_model.py` API: HParams + ResNet wrapper (resnet_model.py:36-140).

    hps = HParams(num_classes=10, lrn_rate=0.1, weight_decay_rate=2e-4, optimizer='mom')
    model = ResNet(hps, images, labels, 'train', dataset='cifar10', resnet_size=50)
    model.build_graph()            # forward: logits, predictions, cross_entropy, cost
    model.train_op()               # backward + MomentumOptimizer(lr, 0.9) step, global_step += 1

Eager (define-by-run) re-statement for the CPU/fp32 path and for API users:
cost = softmax_cross_entropy(onehot, logits) + wd * sum(l2_loss(v) for all
trainables) -- including BN gamma/beta and the dense bias (resnet_model.py:78-86);
'mom' = tf.train.MomentumOptimizer(lr, 0.9) (accum = 0.9*accum + g; v -= lr*accum),
'sgd' = GradientDescent.  Labels may be one-hot (reference) or class indices.
`resnet_size` is a real argument here (the reference hard-codes 50, defect #8).
The MI355X training path is train/engine.py (same math, HIP kernels).
"""
from __future__ import annotations

from collections import namedtuple

import torch
import torch.nn.functional as F

from . import resnet_model_official

HParams = namedtuple("HParams", "num_classes, lrn_rate, weight_decay_rate, optimizer")


class ResNet:
    """ResNet model (images NHWC float, labels one-hot [N, classes] or int [N])."""

    def __init__(self, hps: HParams, images, labels, mode: str, dataset: str = "cifar10",
                 resnet_size: int = 50, data_format: str = "channels_last", network=None):
        self.hps = hps
        self._images = images
        self.labels = labels
        self.mode = mode
        self.dataset = dataset
        self.resnet_size = resnet_size
        self.data_format = data_format
        self.network = network
        self.global_step = 0
        self.lrn_rate = hps.lrn_rate
        self._slots: dict[int, torch.Tensor] = {}
        self.summaries = {}

    def _make_network(self):
        if self.dataset in ("cifar10", "cifar100"):
            return resnet_model_official.cifar10_resnet_v2_generator(
                self.resnet_size, self.hps.num_classes, self.data_format)
        return resnet_model_official.imagenet_resnet_v2(self.resnet_size, self.hps.num_classes,
                                                        self.data_format)

    def build_graph(self, istrain: bool = True):
        if self.network is None:
            self.network = self._make_network()
        self._build_model(istrain)
        self.summaries = {"cross_entropy": float(self.cross_entropy.detach()),
                          "cost": float(self.cost.detach()),
                          "learning_rate": self.lrn_rate}
        return self

    def _build_model(self, istrain: bool):
        logits = self.network(self._images, istrain)
        self.logits = logits
        self.predictions = torch.softmax(logits, dim=1)
        labels = self.labels
        if labels.dim() == 2:
            self.cross_entropy = -(labels * F.log_softmax(logits, 1)).sum(1).mean()
        else:
            self.cross_entropy = F.cross_entropy(logits, labels.long())
        l2 = sum((v * v).sum() * 0.5 for v in self.network.trainable_variables())
        self.cost = self.cross_entropy + self.hps.weight_decay_rate * l2

    def train_op(self, lrn_rate: float | None = None):
        """minimize(cost, global_step) with the configured optimizer."""
        if lrn_rate is not None:
            self.lrn_rate = lrn_rate
        vs = self.network.trainable_variables()
        for v in vs:
            v.grad = None
        self.cost.backward()
        with torch.no_grad():
            for v in vs:
                g = v.grad
                if self.hps.optimizer == "mom":
                    acc = self._slots.get(id(v))
                    if acc is None:
                        acc = torch.zeros_like(v)
                        self._slots[id(v)] = acc
                    acc.mul_(0.9).add_(g)
                    v.sub_(self.lrn_rate * acc)
                else:
                    v.sub_(self.lrn_rate * g)
        self.global_step += 1
        return self.global_step

    def precision(self) -> float:
        y = self.labels.argmax(1) if self.labels.dim() == 2 else self.labels
        return float((self.predictions.argmax(1) == y).float().mean())
