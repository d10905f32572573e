"""Drop-in for the reference's `trainer` package (`trainer/__init__.py:1` star-exports
`trainer/trainer.py`): `train(epoch, net, optimizer, trainloader, device, criterion)` and
`test(epoch, net, testloader, device, criterion, save_path)`, which saves
`{'net', 'acc', 'epoch'}` to save_path/ckpt_{epoch}.pth (trainer/trainer.py:64-71)."""
import os  # noqa: F401  (train_sparse.py uses os through this star import)

import torch  # noqa: F401

from data_diet_distributed_amd.sparse_train import test, train  # noqa: F401
