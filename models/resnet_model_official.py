"""Reference duplicate path `models/resnet_model_official.py`."""
from distributed_tensorflow_resnet_amd.models.resnet_model_official import *  # noqa: F401,F403
