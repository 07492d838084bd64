"""Top-level alias of the reference module name (`import resnet_model_official`).

Implementation: distributed_tensorflow_resnet_amd/models/resnet_model_official.py
"""
from distributed_tensorflow_resnet_amd.models.resnet_model_official import *  # noqa: F401,F403
from distributed_tensorflow_resnet_amd.models.resnet_model_official import (  # noqa: F401
    _BATCH_NORM_DECAY, _BATCH_NORM_EPSILON)
