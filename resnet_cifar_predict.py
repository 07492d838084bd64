#!/usr/bin/env python3
"""Predict CIFAR test images from the latest checkpoint (reference
resnet_cifar_predict.py; EVAL_NUM = 100).  Prints truth / predictions /
precision and optionally writes a labelled image grid (PIL instead of
matplotlib).  Fixes the reference's empty-graph session bug (defect: the model
was built in the default graph but run in a fresh graph).

    python resnet_cifar_predict.py --train_dir /tmp/ckpt --eval_data_path /data/cifar10
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

from distributed_tensorflow_resnet_amd.data.cifar import CifarData, synthetic_batches  # noqa: E402
from distributed_tensorflow_resnet_amd.models.spec import build_spec  # noqa: E402
from distributed_tensorflow_resnet_amd.train.evaluator import make_inference  # noqa: E402
from distributed_tensorflow_resnet_amd.utils import tensor_bundle as tb  # noqa: E402

EVAL_NUM = 100
CLASSES = ("airplane", "automobile", "bird", "cat", "deer", "dog", "frog", "horse", "ship", "truck")


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--train_dir", default="")
    ap.add_argument("--checkpoint_path", default="")
    ap.add_argument("--eval_data_path", default="")
    ap.add_argument("--dataset", default="cifar10")
    ap.add_argument("--resnet_size", type=int, default=50)
    ap.add_argument("--device", default="auto")
    ap.add_argument("--save_grid", default="", help="write a PNG grid of the predictions")
    a = ap.parse_args(argv)
    prefix = a.checkpoint_path or tb.latest_checkpoint(a.train_dir)
    if not prefix:
        print("no checkpoint found", file=sys.stderr)
        return 1
    spec = build_spec(a.dataset, a.resnet_size)
    if a.eval_data_path:
        data = CifarData(a.eval_data_path, a.dataset, train=False)
        n = min(EVAL_NUM, len(data))
        x, y = next(data.batches(n, shuffle=False, num_epochs=1))
    else:
        n = EVAL_NUM
        x, y = next(synthetic_batches(n, spec.num_classes, seed=7))
    model = make_inference(spec, n, a.device)
    model.load(tb.read_bundle(prefix))
    _, correct, probs = model.run(x, y)
    pred = probs.argmax(1).cpu()
    print("truth:      ", y.tolist())
    print("predictions:", pred.tolist())
    print(f"precision: {correct / n:.3f}")
    if a.save_grid:
        from cifar_input import save_image_grid

        names = CLASSES if spec.num_classes == 10 else None
        save_image_grid(x, pred, y, a.save_grid, names)
        print(f"wrote {a.save_grid}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
