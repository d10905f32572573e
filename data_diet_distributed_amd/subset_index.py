"""Pruned-index artefact.

The reference hands the keep-set over only as an in-memory
`DataLoader(Subset(MyDataset(train), indices))` (get_scores_and_prune.py:26-34), consumed by
train.py:64-65 and train_sparse.py:28.  The build also writes it to disk so sparse training
can run in another process / job:

  <path>.npy   int64 [k] kept indices in the reference's order (score descending, ties by
               ascending index)
  <path>.json  metadata: n, k, sparsity, score method(s), K, checkpoint digests, ...
"""
from __future__ import annotations

import json
import os

import numpy as np
import torch


def _stem(path: str) -> str:
    return path[:-4] if path.endswith(".npy") else path


def write_subset_index(path: str, indices, meta: dict | None = None) -> str:
    stem = _stem(path)
    os.makedirs(os.path.dirname(os.path.abspath(stem)) or ".", exist_ok=True)
    idx = np.asarray(indices.cpu() if isinstance(indices, torch.Tensor) else indices,
                     dtype=np.int64)
    np.save(stem + ".npy", idx, allow_pickle=False)
    m = dict(meta or {})
    m.setdefault("k", int(idx.size))
    m["format"] = "data_diet_subset_index/v1"
    with open(stem + ".json", "w") as f:
        json.dump(m, f, indent=1, sort_keys=True)
    return stem + ".npy"


def read_subset_index(path: str):
    stem = _stem(path)
    idx = np.load(stem + ".npy", allow_pickle=False)
    meta = {}
    if os.path.exists(stem + ".json"):
        with open(stem + ".json") as f:
            meta = json.load(f)
    if idx.dtype != np.int64 or idx.ndim != 1:
        raise ValueError("subset index must be a 1-D int64 array")
    if "k" in meta and meta["k"] != idx.size:
        raise ValueError("subset index length disagrees with its metadata")
    return idx, meta


def subset_loader(dataset, path: str, batch_size: int, num_workers: int = 0, shuffle=True):
    """DataLoader(Subset(dataset, indices)) from an index file — the reference's return
    value (get_scores_and_prune.py:27,32) rebuilt in another process."""
    idx, meta = read_subset_index(path)
    if "n" in meta and meta["n"] != len(dataset):
        raise ValueError(f"index file was made for n={meta['n']}, dataset has {len(dataset)}")
    sub = torch.utils.data.Subset(dataset, idx.tolist())
    return torch.utils.data.DataLoader(sub, batch_size=batch_size, shuffle=shuffle,
                                       num_workers=num_workers)
