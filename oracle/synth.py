"""ORACLE (test infrastructure only; never imported by the product path): NumPy restatement
of the on-device synthetic set generator (data_diet_distributed_amd/csrc/dd_synth.hip,
include/dd_capi.h `dd_synth_images_u8`).

Not in the reference: it replaces the dataset source of reference data/loader.py:27-33
(torchvision CIFAR10 download) for offline and ImageNet-shape (BASELINE config 5) runs, so it
is pinned to its own definition — the integer hash written out in dd_synth.hip — and the GPU
test demands bit-exact bytes.  All arithmetic is uint32 with wrap-around.
"""
from __future__ import annotations

import numpy as np

U32 = np.uint32


def mix(h):
    """murmur3 fmix32 on uint32 arrays."""
    h = np.asarray(h, dtype=U32).copy()
    with np.errstate(over="ignore"):
        h ^= h >> U32(16)
        h *= U32(0x85EBCA6B)
        h ^= h >> U32(13)
        h *= U32(0xC2B2AE35)
        h ^= h >> U32(16)
    return h


def example_keys(seed: int, idx: np.ndarray) -> np.ndarray:
    idx = np.asarray(idx, dtype=np.uint64)
    s0, s1 = U32(seed & 0xFFFFFFFF), U32((seed >> 32) & 0xFFFFFFFF)
    i0 = (idx & np.uint64(0xFFFFFFFF)).astype(U32)
    i1 = (idx >> np.uint64(32)).astype(U32)
    with np.errstate(over="ignore"):
        a = mix(i0 ^ mix(np.array([s0 + U32(0x9E3779B9)], dtype=U32))[0])
        return mix(a ^ (i1 * U32(0x85EBCA77) + s1))


def synth_images_u8(seed: int, idx0: int, n: int, num_classes: int, hw: int = 32,
                    channels: int = 3):
    """(uint8 [n, C, hw, hw], int64 [n]) — examples idx0 .. idx0+n-1 of set `seed`."""
    H = W = hw
    key = example_keys(seed, np.arange(idx0, idx0 + n, dtype=np.uint64))       # [n]
    label = mix(key ^ U32(0xA511E9B3)) % U32(num_classes)
    with np.errstate(over="ignore"):
        hc = mix(label * U32(0x9E3779B1) + U32(0x6A09E667))                     # [n]
        fx = U32(1) + (hc & U32(7))
        fy = U32(1) + ((hc >> U32(3)) & U32(7))
        ch = np.arange(channels, dtype=U32)
        base = U32(32) + ((mix(hc[:, None] + ch[None, :]) >> U32(25)) & U32(127))  # [n, C]
        base = base + ((key >> U32(8)) & U32(31))[:, None]
        y = np.arange(H, dtype=U32)[:, None]
        x = np.arange(W, dtype=U32)[None, :]
        stripe = (((x[None] * fx[:, None, None] + y[None] * fy[:, None, None]) * U32(16))
                  // U32(W)) & U32(1)                                           # [n, H, W]
        r = np.arange(channels * H * W, dtype=U32).reshape(channels, H, W)
        noise = mix(key[:, None, None, None] ^ (r[None] * U32(0x27D4EB2F))) & U32(63)
        v = base[:, :, None, None] + U32(48) * stripe[:, None] + noise
    img = np.minimum(v, U32(255)).astype(np.uint8)
    return img, label.astype(np.int64)
