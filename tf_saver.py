#!/usr/bin/env python3
"""Checkpoint inspector (reference tf_saver.py:56-135).

Lists every variable of a TF V2 checkpoint (name, dtype, shape) like
`tf.train.NewCheckpointReader(...).get_variable_to_shape_map()`, and can
restore it into a rebuilt model and print one tensor (the reference prints
`dense/bias`).  Works on the reference's own `.index` files (layout only, the
`.data` blobs were withheld upstream) and on checkpoints written here.

    python tf_saver.py --checkpoint_path /root/reference/test/resnet50-cifar-ckpt-20190218/model.ckpt-107738
    python tf_saver.py --checkpoint_dir /tmp/ckpt --tensor dense/bias --restore
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import numpy as np  # noqa: E402

from distributed_tensorflow_resnet_amd.utils import tensor_bundle as tb  # noqa: E402

DT_NAMES = {1: "float32", 2: "float64", 3: "int32", 4: "uint8", 6: "int8", 9: "int64",
            10: "bool", 14: "bfloat16", 19: "float16"}


def list_variables(prefix: str):
    _, entries = tb.read_index(prefix)
    return [(k, DT_NAMES.get(e.dtype, str(e.dtype)), list(e.shape)) for k, e in sorted(entries.items())]


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--checkpoint_path", default="")
    ap.add_argument("--checkpoint_dir", default="")
    ap.add_argument("--tensor", default="dense/bias")
    ap.add_argument("--restore", action="store_true",
                    help="restore into a rebuilt model (needs the .data file)")
    ap.add_argument("--dataset", default="cifar10")
    ap.add_argument("--resnet_size", type=int, default=50)
    a = ap.parse_args(argv)
    prefix = a.checkpoint_path or tb.latest_checkpoint(a.checkpoint_dir)
    if not prefix:
        print("no checkpoint found", file=sys.stderr)
        return 1
    vs = list_variables(prefix)
    total = 0
    for name, dt, shape in vs:
        print(f"{name} ({dt}) {shape}")
        if dt.startswith("float") and not name.endswith("/Momentum"):
            total += int(np.prod(shape)) if shape else 1
    print(f"{len(vs)} tensors; {total:,} non-slot float values")
    if os.path.exists(tb.data_path(prefix)):
        t = tb.read_bundle(prefix, names={a.tensor})
        if a.tensor in t:
            print(f"{a.tensor} = {t[a.tensor]}")
        if a.restore:
            from distributed_tensorflow_resnet_amd.models.params import ParamStore
            from distributed_tensorflow_resnet_amd.models.spec import build_spec
            from distributed_tensorflow_resnet_amd.utils.checkpoint import tf_to_state

            store = ParamStore(build_spec(a.dataset, a.resnet_size))
            step = tf_to_state(tb.read_bundle(prefix), store, None)
            print(f"restored {store.n_train:,} trainables into a ResNet-{a.resnet_size} "
                  f"({a.dataset}) at global_step {step}")
    else:
        print(f"(data file {tb.data_path(prefix)} absent: layout only)")
    return 0


if __name__ == "__main__":
    sys.exit(main())
