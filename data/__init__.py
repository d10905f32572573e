"""Drop-in for the reference's `data` package (`data/__init__.py:1` star-exports
`data/loader.py`): transform, MyDataset, load_data, get_dataloader, without torchvision
(CIFAR-10 read from torchvision's own download layout, or synthetic sets)."""
from data_diet_distributed_amd.loader import *  # noqa: F401,F403
from data_diet_distributed_amd.loader import (MyDataset, get_dataloader, load_data,  # noqa: F401
                                              transform)
