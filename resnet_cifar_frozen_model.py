#!/usr/bin/env python3
"""Freeze a checkpoint into a self-contained inference artifact and run it
(reference resnet_cifar_frozen_model.py: export_meta_graph + freeze_graph ->
.pb with outputs `predictions,precision`, then feed-dict inference on 100
test images).  utils/frozen.py writes the same TensorFlow GraphDef (node for
node the reference's resnet50_cifar_frozen_model_eval.pb), without TensorFlow.

    python resnet_cifar_frozen_model.py --checkpoint_path /tmp/ckpt/model.ckpt-1000 \
        --output resnet50_cifar_frozen_model_eval.pb [--eval_data_path DIR]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from distributed_tensorflow_resnet_amd.utils import tensor_bundle as tb  # noqa: E402
from distributed_tensorflow_resnet_amd.utils.frozen import freeze  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--checkpoint_path", default="")
    ap.add_argument("--train_dir", default="")
    ap.add_argument("--output", default="resnet50_cifar_frozen_model_eval.pb")
    ap.add_argument("--dataset", default="cifar10")
    ap.add_argument("--resnet_size", type=int, default=50)
    ap.add_argument("--eval_data_path", default="")
    ap.add_argument("--device", default="auto", choices=("auto", "gpu", "cpu", "interp"))
    a = ap.parse_args(argv)
    prefix = a.checkpoint_path or tb.latest_checkpoint(a.train_dir)
    if not prefix:
        print("no checkpoint found", file=sys.stderr)
        return 1
    meta = freeze(prefix, a.output, a.dataset, a.resnet_size)
    print(f"froze {prefix} -> {a.output}: {meta}")
    from resnet_cifar_predict_from_pd import main as predict

    return predict(["--frozen", a.output, "--device", a.device] +
                   (["--eval_data_path", a.eval_data_path] if a.eval_data_path else []))


if __name__ == "__main__":
    sys.exit(main())
