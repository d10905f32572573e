"""Timing of the drop-in `sparse_loader` (reference get_scores_and_prune.py:8-34) at the
headline size, against the engine's EL2N pass on data already in HBM.

    python tools/bench_dropin.py [--n 50000] [--json-out PATH]

Cases (ResNet-18 / CIFAR-10 shape, one checkpoint, train-mode BN, batch 128, sparsity 0.5):
  engine_el2n      ScoringEngine(methods=el2n).run on resident uint8 (what bench.py times)
  sparse_loader    the reference call on a shuffled DataLoader over MyDataset(CIFAR10-like
                   with torchvision's `.data` uint8 NHWC + Compose(ToTensor, Normalize)):
                   fast path = batch-sampler visit order, one H2D of the raw set, grouped
                   train-BN forward on the hand kernels, select, Subset + DataLoader
  sparse_loader_general   the same call with fast=False (net(input) per decoded host batch),
                   on the first --general-n examples only (host decode dominates)
Each is run once cold and timed warm (median of --reps).
"""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from data_diet_distributed_amd import checkpoints, loader, synthetic  # noqa: E402
from data_diet_distributed_amd.get_scores_and_prune import sparse_loader  # noqa: E402
from data_diet_distributed_amd.resnet import ResNet18  # noqa: E402
from data_diet_distributed_amd.scoring import ScoreConfig, ScoringEngine  # noqa: E402


class _ToTensor:
    def __call__(self, a):
        return torch.from_numpy(np.ascontiguousarray(a.transpose(2, 0, 1))).float().div(255)


class _Normalize:
    def __init__(self, mean, std):
        self.mean, self.std = mean, std

    def __call__(self, t):
        return (t - torch.tensor(self.mean)[:, None, None]) / torch.tensor(self.std)[:, None, None]


_ToTensor.__name__, _Normalize.__name__ = "ToTensor", "Normalize"


class Compose:
    def __init__(self, ts):
        self.transforms = ts

    def __call__(self, x):
        for t in self.transforms:
            x = t(x)
        return x


class CIFAR10Like(torch.utils.data.Dataset):
    """torchvision.datasets.CIFAR10's attributes: .data uint8 NHWC, .targets, .transform."""

    def __init__(self, images_nchw, labels):
        self.data = np.ascontiguousarray(images_nchw.transpose(0, 2, 3, 1))
        self.targets = [int(v) for v in labels]
        self.transform = Compose([_ToTensor(), _Normalize(loader.MEAN, loader.STD)])
        self.target_transform = None

    def __len__(self):
        return len(self.targets)

    def __getitem__(self, i):
        return self.transform(self.data[i]), self.targets[i]


def timed(fn, reps):
    torch.cuda.synchronize()
    t = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    cold = time.perf_counter() - t
    warm = []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        warm.append(time.perf_counter() - t)
    return cold, statistics.median(warm)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=50000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--general-n", type=int, default=2048)
    ap.add_argument("--json-out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    images, labels = synthetic.make_images(a.n, 10, seed=0)
    sd = synthetic.make_checkpoint("resnet18", 10, seed=0)["net"]
    out = {"n": a.n, "batch_size": 128, "sparsity": 0.5}

    eng = ScoringEngine(checkpoints.build_models([sd], device=dev), ScoreConfig(methods=("el2n",)),
                        dev)
    img_d, lab_d = torch.from_numpy(images).to(dev), torch.from_numpy(labels).to(dev)
    c, w = timed(lambda: eng.run(img_d, lab_d, 0.5), a.reps)
    out["engine_el2n"] = {"cold_s": c, "warm_s": w, "examples_per_s": a.n / w}

    ds = loader.MyDataset(CIFAR10Like(images, labels))
    net = ResNet18().to(dev)
    net.load_state_dict(sd)
    gen = torch.Generator().manual_seed(0)
    ld = torch.utils.data.DataLoader(ds, batch_size=128, shuffle=True, generator=gen)
    c, w = timed(lambda: sparse_loader(ld, a.n, net, dev, 0.5, 125, 0), a.reps)
    assert sparse_loader.last_path == "fast"
    out["sparse_loader"] = {"path": "fast", "cold_s": c, "warm_s": w,
                            "examples_per_s": a.n / w, "vs_engine_el2n": w / out["engine_el2n"]["warm_s"]}

    ng = min(a.general_n, a.n)
    dsg = loader.MyDataset(CIFAR10Like(images[:ng], labels[:ng]))
    ldg = torch.utils.data.DataLoader(dsg, batch_size=128, shuffle=True, generator=gen)
    c, w = timed(lambda: sparse_loader(ldg, ng, net, dev, 0.5, 125, 0, fast=False), 1)
    out["sparse_loader_general"] = {"path": "general", "n": ng, "cold_s": c, "warm_s": w,
                                    "examples_per_s": ng / w}
    text = json.dumps(out)
    print(text)
    if a.json_out:
        with open(a.json_out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
