#!/usr/bin/env python3
"""Predict from a frozen inference artifact (reference
resnet_cifar_predict_from_pd.py: load_graph(.pb) + feed-dict run of
`predictions` on 100 standardized test images).

    python resnet_cifar_predict_from_pd.py --frozen resnet50_cifar_frozen_model_eval.pb \
        [--eval_data_path DIR] [--device auto|gpu|cpu|interp]

Any frozen ResNet v2 GraphDef works -- ours (resnet_cifar_frozen_model.py) or
TensorFlow's, e.g. the reference's test/resnet50-cifar-ckpt-20190218/
resnet50_cifar_frozen_model_eval.pb.  `--device interp` runs the graph itself
op by op (utils/tf_interp.py); the other devices load its weights into our
GPU inference plan or CPU model.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from distributed_tensorflow_resnet_amd.data.cifar import CifarData, synthetic_batches  # noqa: E402
from distributed_tensorflow_resnet_amd.utils.frozen import FrozenModel  # noqa: E402

EVAL_NUM = 100


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--frozen", required=True)
    ap.add_argument("--eval_data_path", default="")
    ap.add_argument("--device", default="auto", choices=("auto", "gpu", "cpu", "interp"))
    a = ap.parse_args(argv)
    from distributed_tensorflow_resnet_amd.utils.frozen import read_frozen

    meta, _ = read_frozen(a.frozen)
    if a.eval_data_path:
        data = CifarData(a.eval_data_path, meta["dataset"], train=False)
        n = min(EVAL_NUM, len(data))
        x, y = next(data.batches(n, shuffle=False, num_epochs=1))
    else:
        n = EVAL_NUM
        x, y = next(synthetic_batches(n, meta["num_classes"], seed=7))
    m = FrozenModel(a.frozen, a.device, n)
    probs, precision = m.predict(x, y)
    print("predictions:", probs.argmax(1).tolist())
    print(f"precision: {precision:.3f}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
