"""ORACLE (test infrastructure): EL2N rows and keep-set selection in NumPy.

Restates reference get_scores_and_prune.py:16-24.
"""
from __future__ import annotations

import numpy as np


def el2n_rows(logits: np.ndarray, labels: np.ndarray, with_e: bool = False):
    """softmax(dim=1) - one_hot(y) -> L2 over classes (get_scores_and_prune.py:16-18).

    Computed in float64 from the float32 logits (the reference rounds to float32 at each
    torch op; the difference is ~1e-7 relative, far inside the 1e-3 tolerance).
    """
    x = np.asarray(logits, dtype=np.float64)
    m = x.max(axis=1, keepdims=True)
    ex = np.exp(x - m)
    p = ex / ex.sum(axis=1, keepdims=True)
    e = p.copy()
    e[np.arange(x.shape[0]), np.asarray(labels, dtype=np.int64)] -= 1.0
    s = np.sqrt((e * e).sum(axis=1))
    return (s, e) if with_e else s


def keep_count(train_samples: int, sparsity: float) -> int:
    """samples = int((1-sparsity)*train_samples)  (get_scores_and_prune.py:22)."""
    return int((1 - sparsity) * train_samples)


def stable_topk_python(indices, scores, k: int):
    """Literal restatement of get_scores_and_prune.py:23-24 on (index, score) pairs in
    loader-visit order (pure Python; small cases)."""
    pairs = [(int(i), float(s)) for i, s in zip(indices, scores)]
    top = sorted(pairs, key=lambda x: x[1], reverse=True)[:k]
    return [i for i, _ in top]


def stable_topk(scores: np.ndarray, k: int, visit_order: np.ndarray | None = None) -> np.ndarray:
    """NumPy form of the same: order by score descending, ties in visit order.

    `scores[j]` is the score of the example visited j-th; returned values are visit
    positions (== global indices under the unshuffled protocol) unless `visit_order`
    maps positions to indices.  +0.0 and -0.0 compare equal (as Python floats do).
    """
    s = np.asarray(scores, dtype=np.float64)
    if np.isnan(s).any():
        raise ValueError("NaN score: the reference's sort is undefined")
    order = np.argsort(-s, kind="stable")[:k]
    if visit_order is not None:
        order = np.asarray(visit_order)[order]
    return order.astype(np.int64)
