"""Deterministic synthetic CIFAR-shape data and ResNet checkpoints (NumPy PCG64).

There is no network and no real CIFAR-10 in this environment, so every benchmark and parity
case runs on synthetic inputs.  Generation uses NumPy's PCG64 only (never torch's RNG), so
the same (seed, shape) yields byte-identical images, labels and checkpoints on any x86 host:
the golden fixtures made in the build container pin results the GPU box reproduces.

Images are class-structured (a low-frequency per-class prototype plus pixel noise) so a
network's logits spread and the EL2N ranking has few near-ties.
"""
from __future__ import annotations

import hashlib

import numpy as np
import torch

from .resnet import build


def _rng(seed: int, stream: int) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64([int(seed), int(stream)]))


def make_images(n: int, num_classes: int = 10, seed: int = 0, hw: int = 32, chunk: int = 8192,
                lo: int = 0, hi: int = None):
    """uint8 images [n, 3, hw, hw] (CHW, like ToTensor's output layout) and int64 labels [n].

    With lo/hi: only examples [lo, hi) of that same n-example set (byte-identical to
    `make_images(n, ...)[lo:hi]`; only the noise chunks overlapping the range are drawn), so
    a rank builds just its shard."""
    hi = n if hi is None else hi
    if not 0 <= lo <= hi <= n:
        raise ValueError(f"range [{lo}, {hi}) outside [0, {n}]")
    lab_rng = _rng(seed, 1)
    labels = lab_rng.integers(0, num_classes, size=n, dtype=np.int64)
    proto_rng = _rng(seed, 2)
    cell = max(hw // 8, 1)
    protos = proto_rng.uniform(0.0, 255.0, size=(num_classes, 3, hw // cell, hw // cell))
    protos = np.repeat(np.repeat(protos, cell, axis=2), cell, axis=3).astype(np.float32)
    images = np.empty((hi - lo, 3, hw, hw), dtype=np.uint8)
    for c0 in range((lo // chunk) * chunk, hi, chunk):
        c1 = min(n, c0 + chunk)
        noise = _rng(seed, 1000 + c0 // chunk).normal(0.0, 48.0, size=(c1 - c0, 3, hw, hw))
        x = 0.55 * protos[labels[c0:c1]] + 57.0 + noise.astype(np.float32)
        a, b = max(lo, c0), min(hi, c1)
        images[a - lo:b - lo] = np.clip(np.rint(x[a - c0:b - c0]), 0, 255).astype(np.uint8)
    return images, labels[lo:hi].copy()


def device_shard(seed: int, lo: int, hi: int, num_classes: int, hw: int = 32, device="cuda"):
    """Examples [lo, hi) of the hash-defined synthetic set `seed`, generated directly in HBM by
    dd_synth_images_u8 (no host copy; the ImageNet-shape set of BASELINE config 5 is 193 GB of
    uint8, so each rank generates only its shard).  A different family from `make_images`
    (counter-based hash, not PCG64), pinned bit-exactly by oracle/synth.py."""
    from . import _capi
    return _capi.synth_images_u8(seed, lo, hi - lo, num_classes, hw, 3, device)


def make_checkpoint(arch: str = "resnet18", num_classes: int = 10, seed: int = 0,
                    stem: str = "cifar", logit_scale: float = 6.0) -> dict:
    """A `{'net': state_dict}` checkpoint (reference trainer/trainer.py:64-71 format).

    Conv weights He-uniform, BN affine/statistics randomised around identity, final Linear
    scaled by `logit_scale` so softmax outputs are far from uniform.
    """
    model = build(arch, num_classes, stem)
    sd = model.state_dict()
    rng = _rng(seed, 7)
    out = {}
    for name, t in sd.items():
        shape = tuple(t.shape)
        if name.endswith("num_batches_tracked"):
            out[name] = torch.tensor(100, dtype=torch.int64)
            continue
        if t.dim() == 4:  # conv weight
            fan_in = shape[1] * shape[2] * shape[3]
            bound = np.sqrt(6.0 / fan_in)
            a = rng.uniform(-bound, bound, size=shape)
        elif name.startswith("linear.") and name.endswith("weight"):
            bound = 1.0 / np.sqrt(shape[1])
            a = rng.uniform(-bound, bound, size=shape) * logit_scale
        elif name.startswith("linear.") and name.endswith("bias"):
            a = rng.uniform(-0.1, 0.1, size=shape)
        elif name.endswith("running_mean"):
            a = rng.normal(0.0, 0.2, size=shape)
        elif name.endswith("running_var"):
            a = rng.uniform(0.5, 2.0, size=shape)
        elif name.endswith("weight"):  # BN gamma
            a = rng.uniform(0.6, 1.4, size=shape)
        elif name.endswith("bias"):  # BN beta
            a = rng.normal(0.0, 0.1, size=shape)
        else:
            raise KeyError(f"unexpected state_dict entry {name}")
        out[name] = torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32))
    return {"net": out, "acc": 0.0, "epoch": 19}


def digest(*arrays) -> str:
    """sha256 over raw bytes of numpy arrays / torch tensors (fixture input pinning)."""
    h = hashlib.sha256()
    for a in arrays:
        if isinstance(a, torch.Tensor):
            a = a.detach().cpu().numpy()
        a = np.ascontiguousarray(a)
        h.update(str(a.dtype).encode())
        h.update(str(a.shape).encode())
        h.update(a.tobytes())
    return h.hexdigest()


def state_digest(state_dict: dict) -> str:
    return digest(*[state_dict[k] for k in sorted(state_dict)])
