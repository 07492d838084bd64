"""`resnet_model` API of the reference (HParams, ResNet; resnet_model.py:36-140).
Implementation: distributed_tensorflow_resnet_amd/models/resnet_model.py"""
from distributed_tensorflow_resnet_amd.models.resnet_model import HParams, ResNet  # noqa: F401
