"""Reference duplicate path `models/resnet_model.py`."""
from distributed_tensorflow_resnet_amd.models.resnet_model import *  # noqa: F401,F403
