#!/usr/bin/env python3
"""Predict ImageNet images from the latest checkpoint and print the top-5 classes
(reference: resnet_imagenet_predict.ipynb, which restored a checkpoint and looked
classes up in data/imagenet1000_clsidx_to_labels.txt).  The labels file is
optional (`--labels_file`, one `idx: 'name'` or plain name per line, 0-based);
without validation TFRecords the images are synthetic.

    python resnet_imagenet_predict.py --train_dir /tmp/in_ckpt --eval_data_path /data/val \
        --labels_file imagenet1000_clsidx_to_labels.txt
"""
import argparse
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

from distributed_tensorflow_resnet_amd.data import imagenet  # noqa: E402
from distributed_tensorflow_resnet_amd.models.spec import build_spec  # noqa: E402
from distributed_tensorflow_resnet_amd.train.evaluator import make_inference  # noqa: E402
from distributed_tensorflow_resnet_amd.utils import tensor_bundle as tb  # noqa: E402


def read_labels(path):
    """`{0: 'tench, Tinca tinca',` dict-literal lines (the reference's file) or plain lines."""
    names = []
    with open(path) as fh:
        for line in fh:
            m = re.match(r"\s*\{?\s*(\d+)\s*:\s*['\"](.*)['\"]\s*,?\s*\}?\s*$", line)
            if m:
                names.append(m.group(2))
            elif line.strip():
                names.append(line.strip())
    return names


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--train_dir", default="")
    ap.add_argument("--checkpoint_path", default="")
    ap.add_argument("--eval_data_path", default="")
    ap.add_argument("--labels_file", default="")
    ap.add_argument("--resnet_size", type=int, default=50)
    ap.add_argument("--num_images", type=int, default=16)
    ap.add_argument("--device", default="auto")
    a = ap.parse_args(argv)
    prefix = a.checkpoint_path or tb.latest_checkpoint(a.train_dir)
    if not prefix:
        print("no checkpoint found", file=sys.stderr)
        return 1
    spec = build_spec("imagenet", a.resnet_size)
    n = a.num_images
    if a.eval_data_path:
        x, y = next(iter(imagenet.input_fn(False, a.eval_data_path, n, num_epochs=1, workers=0)))
    else:
        x, y = next(imagenet.synthetic_batches(n, spec.num_classes, spec.image_h, seed=7))
    names = read_labels(a.labels_file) if a.labels_file else None
    model = make_inference(spec, n, a.device)
    model.load(tb.read_bundle(prefix))
    _, correct, probs = model.run(x, y)
    top = torch.topk(probs.float().cpu(), 5, dim=1)
    for i in range(n):
        cls = top.indices[i].tolist()
        desc = ", ".join(f"{c}{'=' + names[c] if names and c < len(names) else ''} "
                         f"({p:.3f})" for c, p in zip(cls, top.values[i].tolist()))
        print(f"image {i}: truth {int(y[i])} | top-5 {desc}")
    print(f"top-1 precision: {correct / n:.3f}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
