"""Minimal in-process stand-in for the `torchvision` pieces the reference imports.

torchvision is not installed in the build container and nothing may be downloaded, so the
golden-vector script injects this module as `sys.modules['torchvision']` before importing
the reference.  It provides exactly what reference data/loader.py:1-11,27-33 and
get_scores_and_prune.py:3-4 touch:
  transforms.Compose / ToTensor / Normalize  — same arithmetic as torchvision 0.20.1
      (ToTensor: uint8 -> float32 / 255; Normalize: sub_(mean).div_(std) per channel)
  datasets.CIFAR10(root, train, download, transform) — serves the synthetic arrays placed in
      `SOURCE` (no file or network access)
  utils — empty namespace
"""
import types

import numpy as np
import torch

SOURCE = {"train": None, "test": None}  # (images uint8 [N,3,H,W], labels int64 [N])


class Compose:
    def __init__(self, transforms):
        self.transforms = transforms

    def __call__(self, x):
        for t in self.transforms:
            x = t(x)
        return x


class ToTensor:
    def __call__(self, img):
        # images are already CHW uint8 (torchvision permutes HWC PIL data to CHW first)
        return torch.from_numpy(np.ascontiguousarray(img)).to(torch.float32).div(255)


class Normalize:
    def __init__(self, mean, std):
        self.mean, self.std = mean, std

    def __call__(self, t):
        mean = torch.as_tensor(self.mean, dtype=t.dtype)[:, None, None]
        std = torch.as_tensor(self.std, dtype=t.dtype)[:, None, None]
        return t.sub_(mean).div_(std)


class CIFAR10(torch.utils.data.Dataset):
    def __init__(self, root=None, train=True, download=False, transform=None):
        src = SOURCE["train" if train else "test"]
        if src is None:
            raise RuntimeError("standin CIFAR10: no synthetic source installed")
        self.images, self.labels = src
        self.transform = transform

    def __len__(self):
        return len(self.labels)

    def __getitem__(self, i):
        img = self.images[i]
        if self.transform is not None:
            img = self.transform(img)
        return img, int(self.labels[i])


def install():
    import sys
    tv = types.ModuleType("torchvision")
    tv.transforms = types.SimpleNamespace(Compose=Compose, ToTensor=ToTensor, Normalize=Normalize)
    tv.datasets = types.SimpleNamespace(CIFAR10=CIFAR10)
    tv.utils = types.SimpleNamespace()
    sys.modules["torchvision"] = tv
    sys.modules["torchvision.transforms"] = tv.transforms
    sys.modules["torchvision.datasets"] = tv.datasets
    sys.modules["torchvision.utils"] = tv.utils
    return tv
