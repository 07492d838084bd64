"""Frozen inference artifacts (reference resnet_cifar_frozen_model.py:81-200,
resnet_cifar_predict_from_pd.py).

TF's freeze_graph folds the checkpoint's variables into a GraphDef with outputs
`predictions` and `precision`.  Our equivalent is one self-contained
safetensors file: the inference variables (trainables + BN moving statistics,
TF names and HWIO layouts) plus metadata naming the architecture (dataset,
resnet_size, num_classes, input shape, output names).  `load_frozen` rebuilds
the network from models/spec.py and runs it on the GPU engine's inference plan
or on the CPU fp32 model.
"""
from __future__ import annotations

import json

import numpy as np
import torch
from safetensors.numpy import load_file, save_file

from ..models.spec import build_spec
from . import tensor_bundle as tb


def freeze(prefix: str, out_path: str, dataset: str, resnet_size: int,
           num_classes: int | None = None) -> dict:
    spec = build_spec(dataset, resnet_size, num_classes)
    tensors = tb.read_bundle(prefix)
    keep = {}
    for p in spec.params:
        if p.name not in tensors:
            raise KeyError(f"{p.name} missing from {prefix}")
        keep[p.name] = np.ascontiguousarray(tensors[p.name].astype(np.float32))
    meta = {"format": "dtr-frozen-v1", "dataset": spec.dataset, "resnet_size": resnet_size,
            "num_classes": spec.num_classes, "input": [None, spec.image_h, spec.image_w, 3],
            "outputs": ["predictions", "precision"],
            "global_step": str(int(tensors.get("global_step", 0)))}
    save_file(keep, out_path, metadata={"dtr": json.dumps(meta)})
    return meta


def read_frozen(path: str):
    from safetensors import safe_open

    with safe_open(path, framework="numpy") as f:
        meta = json.loads(f.metadata()["dtr"])
    return meta, load_file(path)


class FrozenModel:
    """predict(images) -> class probabilities; precision(images, labels)."""

    def __init__(self, path: str, device: str = "auto", batch_size: int = 100):
        from ..train.evaluator import make_inference

        self.meta, tensors = read_frozen(path)
        self.spec = build_spec(self.meta["dataset"], self.meta["resnet_size"],
                               self.meta["num_classes"])
        self.model = make_inference(self.spec, batch_size, device)
        self.model.load(tensors)
        self.batch_size = batch_size

    def predict(self, images, labels=None):
        n = images.shape[0]
        if n != self.batch_size:
            raise ValueError(f"frozen model was loaded for batch {self.batch_size}, got {n}")
        if labels is None:
            labels = torch.zeros(n, dtype=torch.int64)
        loss, correct, probs = self.model.run(images, labels)
        return probs.detach().float().cpu(), correct / n
