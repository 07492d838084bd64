"""`vgg_preprocessing` API of the reference (vgg_preprocessing.py:284-363):
preprocess_image / preprocess_for_train / preprocess_for_eval on HWC images.
Implementation: distributed_tensorflow_resnet_amd/data/vgg.py"""
from distributed_tensorflow_resnet_amd.data.vgg import *  # noqa: F401,F403
