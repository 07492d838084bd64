#!/usr/bin/env python3
"""Predict from a frozen inference artifact (reference
resnet_cifar_predict_from_pd.py: load_graph(.pb) + feed-dict run of
`predictions` on 100 standardized test images).

    python resnet_cifar_predict_from_pd.py --frozen model.safetensors [--eval_data_path DIR]
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
    ap.add_argument("--device", default="auto")
    a = ap.parse_args(argv)
    m = FrozenModel(a.frozen, a.device, EVAL_NUM)
    if a.eval_data_path:
        x, y = next(CifarData(a.eval_data_path, m.spec.dataset, train=False).batches(
            EVAL_NUM, shuffle=False, num_epochs=1))
    else:
        x, y = next(synthetic_batches(EVAL_NUM, m.spec.num_classes, seed=7))
    probs, precision = m.predict(x, y)
    print("predictions:", probs.argmax(1).tolist())
    print(f"precision: {precision:.3f}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
