"""Drop-in for the reference's top-level `get_scores_and_prune.py`.

The reference scripts star-import it (`train.py:7`, `train_sparse.py:1`, `ddp.py:14`,
`ddp_new.py:18`) and call `sparse_loader(train_loader, train_samples, net, device, sparsity,
batch_size, num_workers)` (`train_sparse.py:28`, `train.py:64`, `ddp.py:75`).  With this
file in place of theirs (or this repository's root first on `sys.path`), those scripts run
unedited on the MI355X kernels.  Like the reference module (its line 6, `from data import *`)
it re-exports the data helpers, so star-importers keep seeing `load_data`, `get_dataloader`
and `MyDataset`.
"""
import torch  # noqa: F401  (the reference module's namespace: torch, Dataset, DataLoader)
from torch.utils.data import DataLoader, Dataset  # noqa: F401

from data import *  # noqa: F401,F403  (reference get_scores_and_prune.py:6)
from data_diet_distributed_amd.get_scores_and_prune import sparse_loader  # noqa: F401
