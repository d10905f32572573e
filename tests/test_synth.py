"""Hash-defined synthetic set (dd_synth_images_u8; SURVEY §8 row f3, BASELINE config 5).

CPU: the NumPy restatement (oracle/synth.py) is shard-invariant, class-structured and has
uniform-ish labels.  GPU: the kernel is bit-exact against it, at CIFAR and ImageNet shape,
at 64-bit indices and on the scalar (W % 16 != 0) path.
"""
import numpy as np
import pytest
import torch

from oracle import synth as o_synth


def test_oracle_shard_invariant():
    a, la = o_synth.synth_images_u8(7, 0, 40, 10)
    b, lb = o_synth.synth_images_u8(7, 0, 17, 10)
    c, lc = o_synth.synth_images_u8(7, 17, 23, 10)
    assert np.array_equal(a, np.concatenate([b, c])) and np.array_equal(la, np.concatenate([lb, lc]))
    d, _ = o_synth.synth_images_u8(8, 0, 40, 10)
    assert not np.array_equal(a, d)


def test_oracle_labels_and_class_structure():
    img, lab = o_synth.synth_images_u8(0, 0, 2000, 10)
    assert img.dtype == np.uint8 and img.shape == (2000, 3, 32, 32)
    counts = np.bincount(lab, minlength=10)
    assert counts.min() > 140 and counts.max() < 260
    means = np.stack([img[lab == c].mean(axis=0) for c in range(10)])  # class prototypes
    spread = np.abs(means[:, None] - means[None]).mean(axis=(2, 3, 4))
    assert spread[~np.eye(10, dtype=bool)].min() > 2.0


@pytest.mark.gpu
@pytest.mark.parametrize("seed,idx0,n,classes,hw", [
    (0, 0, 300, 10, 32), (12345, 4999, 77, 100, 32), (2**40 + 3, 2**33 + 5, 3, 1000, 224),
    (1, 1281160, 7, 1000, 224), (5, 10, 9, 10, 20)])
def test_kernel_bit_exact(cuda, seed, idx0, n, classes, hw):
    from data_diet_distributed_amd import synthetic
    img, lab = synthetic.device_shard(seed, idx0, idx0 + n, classes, hw, cuda)
    want_img, want_lab = o_synth.synth_images_u8(seed, idx0, n, classes, hw)
    assert np.array_equal(lab.cpu().numpy(), want_lab)
    assert np.array_equal(img.cpu().numpy(), want_img)


@pytest.mark.gpu
def test_kernel_shards_equal_whole(cuda):
    from data_diet_distributed_amd import _capi
    whole, wl = _capi.synth_images_u8(3, 0, 1000, 10, device=cuda)
    parts = [_capi.synth_images_u8(3, lo, hi - lo, 10, device=cuda)
             for lo, hi in [(0, 333), (333, 334), (334, 1000)]]
    assert torch.equal(whole, torch.cat([p[0] for p in parts]))
    assert torch.equal(wl, torch.cat([p[1] for p in parts]))
