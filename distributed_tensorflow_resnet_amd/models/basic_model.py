"""A working version of the reference's generic model template and registry
(`models/basic_model.py` `BasicAgent`, `models/__init__.py` `make_model` /
`get_model_class`; SURVEY §2.1 "broken model-registry template": the reference
imports a nonexistent `agents.other_model`).

    model = make_model({"model_name": "ResNetModel", "dataset": "cifar10",
                        "resnet_size": 20, "batch_size": 32, "max_iter": 2,
                        "result_dir": "/tmp/run", "device": "cpu"})
    model.train(save_every=1)        # learn_from_epoch() x max_iter, checkpoint each epoch
    logits = model.infer(images)

The lifecycle is the reference's: the config is deep-copied, optionally updated
from get_best_config(), set_agent_props() adds subclass fields, build() creates
the model, init() restores the latest checkpoint in result_dir (TF tensor-bundle
format) or keeps the fresh initialization, save() writes a checkpoint plus
config.json.  Subclasses here run on this framework's backends (MI355X engine or
the CPU path) instead of a tf.Session.
"""
from __future__ import annotations

import copy
import json
import os

import torch

from ..utils.checkpoint import Saver
from .spec import build_spec

DEFAULTS = {"best": False, "debug": False, "random_seed": 0, "result_dir": "", "max_iter": 1,
            "lr": None, "batch_size": 32, "steps_per_epoch": 10, "device": "auto"}


class BasicModel:
    """Config-driven model base (reference: BasicAgent)."""

    def __init__(self, config: dict):
        cfg = dict(DEFAULTS)
        cfg.update(config)
        if cfg["best"]:
            cfg.update(self.get_best_config())
        self.config = copy.deepcopy(cfg)
        if cfg["debug"]:
            print("config", self.config)
        self.random_seed = self.config["random_seed"]
        self.result_dir = self.config["result_dir"]
        self.max_iter = self.config["max_iter"]
        self.lr = self.config["lr"]
        torch.manual_seed(self.random_seed)
        self.set_agent_props()
        self.build()
        self.saver = Saver(self.result_dir, max_to_keep=50) if self.result_dir else None
        self.init()

    # ---- to override
    def set_agent_props(self):
        pass

    def get_best_config(self) -> dict:
        return {}

    @staticmethod
    def get_random_config(fixed_params=None) -> dict:
        raise NotImplementedError("get_random_config must be overridden by the model")

    def build(self):
        raise NotImplementedError("build must be overridden by the model")

    def infer(self, *args):
        raise NotImplementedError("infer must be overridden by the model")

    def learn_from_epoch(self):
        raise NotImplementedError("learn_from_epoch must be overridden by the model")

    def state_tensors(self) -> dict:
        raise NotImplementedError

    def load_state(self, tensors: dict):
        raise NotImplementedError

    def global_step(self) -> int:
        return 0

    # ---- common
    def train(self, save_every: int = 1):
        for epoch_id in range(self.max_iter):
            self.learn_from_epoch()
            if save_every > 0 and epoch_id % save_every == 0:
                self.save()

    def save(self):
        if self.saver is None:
            return None
        prefix = self.saver.save(self.state_tensors(), self.global_step())
        if self.config["debug"]:
            print(f"Saving to {self.result_dir} with global_step {self.global_step()}")
        path = os.path.join(self.result_dir, "config.json")
        if not os.path.isfile(path):
            with open(path, "w") as fh:
                json.dump({k: v for k, v in self.config.items() if k != "phi"}, fh, default=str)
        return prefix

    def init(self):
        if self.saver is None:
            return
        latest = self.saver.latest()
        if latest is not None:
            if self.config["debug"]:
                print(f"Loading the model from folder: {self.result_dir}")
            self.load_state(Saver.restore(latest))


class ResNetModel(BasicModel):
    """ResNet v2 on this framework's training backends (engine on MI355X, fp32 on CPU)."""

    def set_agent_props(self):
        c = self.config
        c.setdefault("dataset", "cifar10")
        c.setdefault("resnet_size", 50 if c["dataset"] == "imagenet" else 20)

    def build(self):
        from ..train.backends import make_backend
        from ..train.engine import cifar_lr_schedule, constant_lr, imagenet_lr_schedule

        c = self.config
        self.spec = build_spec(c["dataset"], c["resnet_size"])
        cifar = c["dataset"].startswith("cifar")
        sched = (constant_lr(c["lr"]) if c["lr"] is not None else
                 cifar_lr_schedule() if cifar else imagenet_lr_schedule())
        self.backend = make_backend(self.spec, c["batch_size"], device=c["device"],
                                    weight_decay=2e-4 if cifar else 1e-4, lr_schedule=sched,
                                    seed=self.random_seed)

    def _batches(self):
        """Synthetic batches of the dataset's shape (uint8 CIFAR records / NHWC floats)."""
        from ..data.cifar import synthetic_batches

        n, seed = self.config["batch_size"], self.random_seed + self.global_step()
        if self.spec.dataset.startswith("cifar"):
            yield from synthetic_batches(n, self.spec.num_classes, seed=seed)
        g = torch.Generator().manual_seed(seed)
        while True:
            yield (torch.randn(n, self.spec.image_h, self.spec.image_w, 3, generator=g),
                   torch.randint(0, self.spec.num_classes, (n,), generator=g))

    def learn_from_epoch(self):
        it = self._batches()
        for _ in range(self.config["steps_per_epoch"]):
            images, labels = next(it)
            self.backend.set_batch(images, labels)
            self.backend.step()
        self.backend.synchronize()
        return self.backend.metrics()

    def infer(self, images):
        """Class probabilities of a batch (eval-mode BatchNorm, current weights)."""
        from ..train.evaluator import make_inference

        inf = make_inference(self.spec, images.shape[0], device=self.config["device"])
        inf.load(self.state_tensors())
        labels = torch.zeros(images.shape[0], dtype=torch.long)
        return inf.run(images, labels)[2]

    def state_tensors(self):
        return self.backend.state_tensors()

    def load_state(self, tensors):
        self.backend.load_state(tensors)

    def global_step(self):
        return int(self.backend.global_step)


class MLPModel(BasicModel):
    """The reference's 1-hidden-layer MLP debug model (logist_model.py) on CPU."""

    def build(self):
        h = self.config.get("hidden_units", 100)
        self.net = torch.nn.Sequential(torch.nn.Linear(784, h), torch.nn.ReLU(),
                                       torch.nn.Linear(h, 10))
        self.opt = torch.optim.Adam(self.net.parameters(), lr=self.lr or 1e-3)
        self.step_ = 0

    def learn_from_epoch(self):
        g = torch.Generator().manual_seed(self.random_seed + self.step_)
        for _ in range(self.config["steps_per_epoch"]):
            x = torch.rand(self.config["batch_size"], 784, generator=g)
            y = torch.randint(0, 10, (self.config["batch_size"],), generator=g)
            loss = torch.nn.functional.cross_entropy(self.net(x), y)
            self.opt.zero_grad()
            loss.backward()
            self.opt.step()
            self.step_ += 1
        return {"loss": float(loss)}

    def infer(self, x):
        with torch.no_grad():
            return self.net(x)

    def state_tensors(self):
        out = {k: v.detach().numpy() for k, v in self.net.state_dict().items()}
        out["global_step"] = torch.tensor(self.step_).numpy()
        return out

    def load_state(self, tensors):
        self.step_ = int(tensors.pop("global_step", 0))
        self.net.load_state_dict({k: torch.from_numpy(v.copy()) for k, v in tensors.items()})

    def global_step(self):
        return self.step_


__all__ = ["BasicModel", "ResNetModel", "MLPModel"]
_REGISTRY = {"BasicModel": BasicModel, "ResNetModel": ResNetModel, "MLPModel": MLPModel}


def get_model_class(config: dict):
    name = config["model_name"]
    if name not in _REGISTRY:
        raise KeyError(f"The model name {name} does not exist")
    return _REGISTRY[name]


def make_model(config: dict, env=None):
    return get_model_class(config)(config)
