"""K-checkpoint discovery and loading.

The reference scores one hard-coded checkpoint, `checkpoint_path/ckpt_19.pth`
(train.py:61, train_sparse.py:23, ddp.py:72), in the trainer's format
`{'net', 'acc', 'epoch'}` (trainer/trainer.py:64-71).  Its DDP trainer writes a different
format, `{'model_state_dict', ...}` with a `module.` prefix (ddp.py:116-123).  Both load here.
K seed checkpoints live at `checkpoint_path/seed{k}/ckpt_{epoch}.pth`.

Files are loaded with `torch.load(..., weights_only=True)` only (nothing executes).
"""
from __future__ import annotations

import os
from typing import List

import torch

from .resnet import build


def extract_state_dict(obj) -> dict:
    if isinstance(obj, dict) and "net" in obj:
        sd = obj["net"]
    elif isinstance(obj, dict) and "model_state_dict" in obj:
        sd = obj["model_state_dict"]
    elif isinstance(obj, dict) and all(isinstance(v, torch.Tensor) for v in obj.values()):
        sd = obj
    else:
        raise ValueError("unrecognised checkpoint format (want {'net': ...} or "
                         "{'model_state_dict': ...})")
    return {(k[len("module."):] if k.startswith("module.") else k): v for k, v in sd.items()}


def load_state_dict(path: str) -> dict:
    return extract_state_dict(torch.load(path, map_location="cpu", weights_only=True))


def discover(checkpoint_path: str, epoch: int = 19, k: int = 1) -> List[str]:
    """Paths of K checkpoints: seed{i}/ckpt_{epoch}.pth, or ckpt_{epoch}.pth when K == 1."""
    single = os.path.join(checkpoint_path, f"ckpt_{epoch}.pth")
    if k == 1 and os.path.exists(single):
        return [single]
    paths = [os.path.join(checkpoint_path, f"seed{i}", f"ckpt_{epoch}.pth") for i in range(k)]
    missing = [p for p in paths if not os.path.exists(p)]
    if missing:
        raise FileNotFoundError(f"missing checkpoints: {missing}")
    return paths


def build_models(state_dicts, arch="resnet18", num_classes=10, stem="cifar", device="cuda"):
    """One resident model per checkpoint (ResNet-18: 45 MB each; K=10 fits trivially)."""
    models = []
    for sd in state_dicts:
        if isinstance(sd, str):
            sd = load_state_dict(sd)
        m = build(arch, num_classes, stem)
        m.load_state_dict(sd)
        models.append(m.to(device))
    return models
