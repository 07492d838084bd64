"""Reference path `models/basic_model.py` (BasicAgent template) -> working template."""
from distributed_tensorflow_resnet_amd.models.basic_model import *  # noqa: F401,F403
from distributed_tensorflow_resnet_amd.models.basic_model import BasicModel as BasicAgent  # noqa: F401
