"""config.yaml handling: the reference's 14 keys stay accepted, new keys get defaults.

Reference keys (config.yaml:1-14), read by train.py:36-49 / ddp.py:54-62.  `sparsity` (:3)
and `batch_size_scores` (:4) are never read by the reference (the CLI `--sparsity` wins and
scoring uses `batch_size`); they are kept and ignored the same way.
"""
from __future__ import annotations

import yaml

REFERENCE_KEYS = ("device", "sparse", "sparsity", "batch_size_scores", "num_workers", "dataset",
                  "batch_size", "start_epoch", "num_epochs", "lr", "momentum", "weight_decay",
                  "checkpoint_path", "sparse_checkpoint_path")

# build extensions (defaults reproduce the reference: EL2N, one checkpoint ckpt_19, train BN)
DEFAULTS = {
    "score_methods": ["el2n"],        # el2n and/or grand
    "select_by": "el2n",
    "score_checkpoints": 1,           # K (seed{k}/ckpt_{epoch}.pth when K > 1)
    "score_epoch": 19,
    "bn_mode": "batch",               # EL2N BN: batch (reference) | running (eval)
    "grand_batch": 1024,
    "pegrad_method": "auto",          # auto | direct | ghost
    "score_precision": "split",       # split (exact keep-set) | split_fast | bf16x3[_fast] | fp32
    "score_lanes": 3,                 # HIP streams the launch chunks are dealt to
    "refine_max_frac": 0.08,          # bf16x3: most of the set the fp32 re-scoring may take
    "score_gpus": 1,
    "subset_index_path": None,        # write the keep-set here when set
    "arch": "resnet18",
    "num_classes": 10,
}


def load_config(path: str) -> dict:
    with open(path) as f:
        cfg = yaml.safe_load(f) or {}
    out = dict(DEFAULTS)
    out.update(cfg)
    return out
