#!/usr/bin/env python3
"""Legacy PS-era ImageNet trainer name (resnet_imagenet_train.py) -> same driver.

Usage (1 GPU):   python resnet_imagenet_train.py --train_dir /tmp/ckpt --log_dir /tmp/logs ...
Multi-GPU:       python -m distributed_tensorflow_resnet_amd.parallel.launch --nproc 8 resnet_imagenet_train.py ...
Flags keep the reference's names/defaults; see distributed_tensorflow_resnet_amd/utils/flags.py.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from distributed_tensorflow_resnet_amd.train.driver import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main(kind="imagenet"))
