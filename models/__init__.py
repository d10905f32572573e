"""Drop-in for the reference's `models` package (`models/__init__.py:1` star-exports
`models/resnet.py`): ResNet18/34/50/101/152, BasicBlock, Bottleneck, ResNet with the same
module names and state_dict keys, backed by data_diet_distributed_amd.resnet."""
from data_diet_distributed_amd.resnet import *  # noqa: F401,F403
from data_diet_distributed_amd.resnet import (BasicBlock, Bottleneck, ResNet, ResNet18,  # noqa: F401
                                              ResNet34, ResNet50, ResNet101, ResNet152)
