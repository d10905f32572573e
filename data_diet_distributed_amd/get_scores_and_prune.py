"""Drop-in for reference get_scores_and_prune.py: `sparse_loader` with the same signature,
return value and selection semantics, running on the MI355X kernels of libdd.so.

Reference: get_scores_and_prune.py:8-34.
  :11-20  per batch: forward, softmax - one_hot, L2, per-example .item() into a Python list
          -> here: forward (PyTorch-ROCm), dd_el2n writes the batch's scores into a device
             vector in visit order; no per-example host sync
  :22     samples = int((1-sparsity)*train_samples)            -> dd_keep_count
  :23-24  stable sorted(..., reverse=True)[:samples]            -> dd_select_topk over the
          visit-ordered scores (ties keep visit order), mapped back to dataset indices
  :26-34  Subset(load_data('cifar10') train, indices), assert, shuffled DataLoader
          -> Subset over the CALLER's training set (`train_loader.dataset`: the same
             MyDataset the reference re-loads at :26, without decoding it a second time),
             assert, shuffled DataLoader
Extension keywords (all optional) re-load a named dataset like :26, or write the index file;
with none given the behaviour is the reference's.
"""
from __future__ import annotations

import torch
from torch.utils.data import DataLoader, Subset

from . import _capi
from .loader import load_data
from .subset_index import write_subset_index
from .synthetic import state_digest


def el2n_scores_from_loader(train_loader, net, device, num_classes=None):
    """Scores of every example the loader yields, in visit order, plus the visited indices.

    Runs `net(input)` exactly as the reference does (:15), so BN follows `net.training`
    (train mode for a freshly built net, as in train.py:59-63)."""
    scores, visit = [], []
    with torch.no_grad():
        for _batch_idx, (idx, inp, target) in enumerate(train_loader):
            inp = inp.to(device, non_blocking=True)
            target = torch.as_tensor(target).to(device, non_blocking=True).to(torch.int64)
            out = net(inp).float().contiguous()
            if num_classes is not None and out.shape[1] != num_classes:
                raise ValueError(f"net produces {out.shape[1]} classes, expected {num_classes}")
            s = torch.empty(out.shape[0], dtype=torch.float32, device=out.device)
            _capi.el2n(out, target.contiguous(), score=s)
            scores.append(s)
            visit.append(torch.as_tensor(idx).to(out.device, non_blocking=True))
    if not scores:
        return (torch.empty(0, dtype=torch.float32, device=device),
                torch.empty(0, dtype=torch.int64, device=device))
    return torch.cat(scores), torch.cat(visit).to(torch.int64)


def select_keep_indices(scores_visit: torch.Tensor, visit_idx: torch.Tensor, samples: int):
    """Reference :23-24 on device: positions of the top `samples` scores (descending, ties in
    visit order) mapped to dataset indices."""
    pos, _thr, _nan = _capi.select_topk(scores_visit.contiguous(), samples)
    return visit_idx[pos]


def _training_set(train_loader, dataset):
    """The dataset the Subset is built over: the caller's loader's dataset (the reference
    re-loads the same training set by name at :26), or load_data(dataset) when asked."""
    if dataset is not None:
        return load_data(dataset)[0]
    ds = getattr(train_loader, "dataset", None)
    if ds is None:
        raise ValueError("train_loader has no .dataset: pass dataset=<name> to re-load it")
    return ds


def sparse_loader(train_loader, train_samples, net, device, sparsity, batch_size, num_workers,
                  *, dataset=None, subset_index_path=None, return_indices=False):
    """Reference-compatible: returns (DataLoader over the kept Subset, samples)."""
    if torch.device(device).type != "cuda":
        raise ValueError("sparse_loader runs its kernels on a GPU device (libdd.so)")
    module = net.module if hasattr(net, "module") else net
    # digest of the checkpoint as handed in: a train-mode forward (reference semantics)
    # updates the BN running statistics while scoring
    digest = state_digest(module.state_dict()) if subset_index_path else None
    scores, visit = el2n_scores_from_loader(train_loader, net, device)
    samples = _capi.keep_count(train_samples, sparsity)
    if samples < 0 or samples > scores.numel():
        raise ValueError(f"keep count {samples} outside [0, {scores.numel()}]")
    kept = select_keep_indices(scores, visit, samples)
    indices = kept.cpu().tolist()  # one device->host copy for the whole keep-set

    train_dense = _training_set(train_loader, dataset)
    train_subset = Subset(train_dense, indices)
    assert len(train_subset) == samples
    print(len(train_subset))
    if subset_index_path:
        write_subset_index(subset_index_path, indices,
                           {"n": int(train_samples), "sparsity": float(sparsity),
                            "score_methods": ["el2n"], "select_by": "el2n", "K": 1,
                            "arch": type(module).__name__,
                            "num_classes": int(getattr(getattr(module, "linear", None),
                                                       "out_features", 0)) or None,
                            "bn_mode": "train" if module.training else "eval",
                            "order": "loader visit order (reference semantics)",
                            "checkpoint_digests": [digest]})
    sparse_train_loader = DataLoader(train_subset, batch_size=batch_size, shuffle=True,
                                     num_workers=num_workers)
    if return_indices:
        return sparse_train_loader, samples, indices
    return sparse_train_loader, samples
