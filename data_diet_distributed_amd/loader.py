"""Data feed mirroring reference data/loader.py, without torchvision and without downloads.

Reference interface kept: `transform` (:8-11), `MyDataset` returning (idx, image, label)
(:13-25), `load_data(dataset)` -> (train MyDataset, test) (:27-33),
`get_dataloader(dataset, batch_size, num_workers)` -> (train_loader shuffle=True,
test_loader batch 100, train_samples) (:35-43).

Datasets:
  "cifar10"            CIFAR-10 under `root` in the layout the reference's torchvision loader
                       downloads (`cifar-10-batches-py/`, data/loader.py:29,31), read with a
                       restricted unpickler that can only rebuild dicts, lists and uint8
                       NumPy arrays (nothing in the file can execute code); or the binary
                       batches (`cifar-10-batches-bin/*.bin`).  Downloads are not possible
                       offline, so a missing directory raises with instructions.
  "synthetic-cifar10"  / "synthetic-cifar100"   class-structured NumPy-PCG64 images
                       (data_diet_distributed_amd.synthetic), size from DD_SYNTHETIC_N
                       (default 50000).
Every dataset keeps its uint8 CHW array and labels (`.images`, `.labels`) so the scoring
engine can move the whole set to HBM once (150 MB at CIFAR scale) instead of re-decoding.
"""
from __future__ import annotations

import os

import numpy as np
import torch
from torch.utils.data import DataLoader, Dataset

MEAN = (0.4914, 0.4822, 0.4465)
STD = (0.2023, 0.1994, 0.2010)


class _Normalize:
    """ToTensor + Normalize of the reference transform (data/loader.py:8-11)."""

    def __init__(self, mean=MEAN, std=STD):
        self.mean = torch.tensor(mean, dtype=torch.float32)[:, None, None]
        self.std = torch.tensor(std, dtype=torch.float32)[:, None, None]

    def __call__(self, img_chw_u8):
        x = torch.from_numpy(np.ascontiguousarray(img_chw_u8)).to(torch.float32).div(255)
        return x.sub_(self.mean).div_(self.std)


transform = _Normalize()


class ArrayImageDataset(Dataset):
    """(image, label) pairs over uint8 CHW arrays, like torchvision's CIFAR10 with a transform."""

    def __init__(self, images: np.ndarray, labels: np.ndarray, transform=transform):
        if images.dtype != np.uint8 or images.ndim != 4:
            raise ValueError("images must be uint8 [N, C, H, W]")
        self.images = images
        self.labels = np.asarray(labels, dtype=np.int64)
        self.transform = transform

    def __len__(self):
        return len(self.labels)

    def __getitem__(self, i):
        img = self.images[i]
        return (self.transform(img) if self.transform else img), int(self.labels[i])


class MyDataset(Dataset):
    """Index-carrying wrapper: returns (idx, image, label) (reference data/loader.py:13-25)."""

    def __init__(self, data):
        self.data = data

    def __getitem__(self, idx):
        image, label = self.data[idx]
        return idx, image, label

    def __len__(self):
        return len(self.data)

    # raw arrays for the device-resident engine path
    @property
    def images(self):
        return self.data.images

    @property
    def labels(self):
        return self.data.labels


class _CifarUnpickler:
    """pickle.Unpickler restricted to what a CIFAR python batch holds (a dict of bytes keys,
    a label list and one uint8 ndarray): any other global raises."""

    ALLOWED = {("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
               ("numpy", "ndarray"), ("numpy", "dtype"), ("_codecs", "encode")}

    @classmethod
    def load(cls, f):
        import pickle

        class U(pickle.Unpickler):
            def find_class(self, module, name):
                if (module, name) not in cls.ALLOWED:
                    raise pickle.UnpicklingError(f"CIFAR batch: global {module}.{name} refused")
                return super().find_class(module, name)

        return U(f, encoding="latin1").load()


def read_cifar10_py(root: str):
    """CIFAR-10 python batches, the layout torchvision.datasets.CIFAR10 downloads
    (cifar-10-batches-py/data_batch_1..5, test_batch): dict with 'data' uint8 [n, 3072]
    (CHW rows) and 'labels'."""
    d = os.path.join(root, "cifar-10-batches-py")
    if not os.path.isdir(d):
        raise FileNotFoundError(d)

    def read(names):
        xs, ys = [], []
        for nm in names:
            with open(os.path.join(d, nm), "rb") as f:
                ent = _CifarUnpickler.load(f)
            ent = {(k.decode() if isinstance(k, bytes) else k): v for k, v in ent.items()}
            x = np.asarray(ent["data"], dtype=np.uint8)
            xs.append(x.reshape(-1, 3, 32, 32))
            ys.append(np.asarray(ent.get("labels", ent.get("fine_labels")), dtype=np.int64))
        return np.ascontiguousarray(np.concatenate(xs)), np.concatenate(ys)

    return read([f"data_batch_{i}" for i in range(1, 6)]), read(["test_batch"])


def read_cifar10(root: str):
    """Either CIFAR-10 layout under `root` (torchvision's python batches first)."""
    if os.path.isdir(os.path.join(root, "cifar-10-batches-py")):
        return read_cifar10_py(root)
    return read_cifar10_bin(root)


def read_cifar10_bin(root: str):
    """CIFAR-10 binary format: records of 1 label byte + 3072 pixel bytes (CHW)."""
    d = os.path.join(root, "cifar-10-batches-bin")
    if not os.path.isdir(d):
        raise FileNotFoundError(
            f"neither {os.path.join(root, 'cifar-10-batches-py')} (torchvision's layout) nor {d} "
            f"found: place CIFAR-10 there (no downloads offline), or use dataset "
            f"'synthetic-cifar10'")

    def read(names):
        raw = b"".join(open(os.path.join(d, nm), "rb").read() for nm in names)
        a = np.frombuffer(raw, dtype=np.uint8).reshape(-1, 3073)
        return a[:, 1:].reshape(-1, 3, 32, 32).copy(), a[:, 0].astype(np.int64)

    train = read([f"data_batch_{i}.bin" for i in range(1, 6)])
    test = read(["test_batch.bin"])
    return train, test


def _synthetic(num_classes):
    from . import synthetic
    n = int(os.environ.get("DD_SYNTHETIC_N", "50000"))
    seed = int(os.environ.get("DD_SYNTHETIC_SEED", "0"))
    train = synthetic.make_images(n, num_classes, seed=seed)
    test = synthetic.make_images(max(n // 5, 1), num_classes, seed=seed + 100)
    return train, test


def load_data(dataset, root="./"):
    """(train MyDataset, test dataset) (reference data/loader.py:27-33)."""
    if dataset == "cifar10":
        (xtr, ytr), (xte, yte) = read_cifar10(root)
    elif dataset == "synthetic-cifar10":
        (xtr, ytr), (xte, yte) = _synthetic(10)
    elif dataset == "synthetic-cifar100":
        (xtr, ytr), (xte, yte) = _synthetic(100)
    else:
        raise ValueError(f"unknown dataset {dataset!r}")
    return MyDataset(ArrayImageDataset(xtr, ytr)), ArrayImageDataset(xte, yte)


def get_dataloader(dataset, batch_size, num_workers):
    """(train_loader, test_loader, train_samples) (reference data/loader.py:35-43)."""
    train, test = load_data(dataset)
    train_samples = len(train)
    train_loader = DataLoader(train, batch_size=batch_size, shuffle=True, num_workers=num_workers)
    test_loader = DataLoader(test, batch_size=100, shuffle=False, num_workers=num_workers)
    return train_loader, test_loader, train_samples


def to_device(ds, device):
    """uint8 images and int64 labels of a dataset on `device` (one H2D copy)."""
    images = torch.from_numpy(np.ascontiguousarray(ds.images)).to(device)
    labels = torch.from_numpy(np.ascontiguousarray(ds.labels)).to(device)
    return images, labels
