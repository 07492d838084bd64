#!/usr/bin/env python3
"""CIFAR-10/100 training + side-car evaluation (resnet_cifar_main.py:424-494).

Usage (1 GPU):   python resnet_cifar_main.py --train_dir /tmp/ckpt --log_dir /tmp/logs ...
Multi-GPU:       python -m distributed_tensorflow_resnet_amd.parallel.launch --nproc 8 resnet_cifar_main.py ...
Flags keep the reference's names/defaults; see distributed_tensorflow_resnet_amd/utils/flags.py.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from distributed_tensorflow_resnet_amd.train.driver import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main(kind="cifar"))
