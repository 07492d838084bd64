"""Reference-compatible `models` package (reference: models/__init__.py).

`make_model(config)` / `get_model_class(config)` over the working template in
distributed_tensorflow_resnet_amd.models.basic_model; `models.resnet_model` and
`models.resnet_model_official` are the reference's duplicate module paths."""
from distributed_tensorflow_resnet_amd.models.basic_model import (  # noqa: F401
    BasicModel, MLPModel, ResNetModel, get_model_class, make_model)

__all__ = ["BasicModel", "ResNetModel", "MLPModel", "make_model", "get_model_class"]
