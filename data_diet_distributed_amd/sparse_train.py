"""Sparse training on the kept set, one process per GPU.

Consumer side of the keep-set: the reference trains on the pruned subset single-device in
`train_sparse.py:28-43` (via `trainer/trainer.py:5-35` `train` and `:39-71` `test`) and with
DDP in `ddp.py:127-164`.  Kept here:

* `train(epoch, net, optimizer, trainloader, device, criterion)` and
  `test(epoch, net, testloader, device, criterion, save_path)` with the trainer's meaning
  (`trainer/trainer.py:5,39`); `test` saves `{'net', 'acc', 'epoch'}` to
  `save_path/ckpt_{epoch}.pth` (`:64-71`), the format `checkpoints.load_state_dict` reads
  back as a scoring checkpoint.
* `ddp_train(...)`: DDP over RCCL (`nccl`) on GPUs or gloo on CPU, SGD(lr, momentum,
  weight_decay) + CosineAnnealingLR(T_max=num_epochs) from config.yaml (`ddp.py:135-137`).

Two deliberate differences from `ddp.py`:
* `ddp.py:80,139` hands the DataLoader returned by `sparse_loader` to
  `DistributedSampler`/`DataLoader` again, so each rank samples *batches of a loader*
  (a DataLoader-in-DataLoader: `len()` is the batch count and items are whole batches).
  Here the sampler shards the kept **examples**: rank r of W takes positions r, r+W, … of
  the epoch's permutation of the keep list, padded by wrap-around to a multiple of W
  (the `torch.utils.data.DistributedSampler` rule, `seed + epoch` permutation).
* `ddp.py:116-123` saves `model_state_dict` with the DDP `module.` prefix; here the
  unwrapped module is saved in the trainer format (both load via `checkpoints`).

Feeds.  `DeviceSubsetFeed` keeps the whole uint8 training set and labels resident in HBM
and builds each batch with one `dd_normalize_u8_gather` launch (gather by kept index +
ToTensor/Normalize of `data/loader.py:8-11`), so no host worker or H2D copy sits in the
step.  It needs libdd.so and a GPU and raises otherwise.  `loader_feed` is the reference's
host path (`Subset` + `DistributedSampler` + `DataLoader`) for CPU/gloo runs.
"""
from __future__ import annotations

import argparse
import math
import os
import time

import numpy as np
import torch
import torch.distributed as dist
import torch.nn as nn
from torch.utils.data import DataLoader, Subset

from .loader import MEAN, STD


def epoch_positions(n_keep: int, world: int, rank: int, epoch: int, seed: int = 0,
                    shuffle: bool = True) -> torch.Tensor:
    """Positions into the keep list that rank `rank` visits in `epoch`.

    Same rule as torch's DistributedSampler (drop_last=False): permutation from a generator
    seeded with seed + epoch, padded by wrap-around to ceil(n/W)·W, then every W-th entry."""
    if n_keep <= 0:
        return torch.empty(0, dtype=torch.int64)
    if shuffle:
        g = torch.Generator()
        g.manual_seed(seed + epoch)
        order = torch.randperm(n_keep, generator=g)
    else:
        order = torch.arange(n_keep)
    per_rank = math.ceil(n_keep / world)
    total = per_rank * world
    if total > n_keep:
        reps = math.ceil((total - n_keep) / n_keep)
        order = torch.cat([order] + [order] * reps)[:total]
    return order[rank:total:world]


class DeviceSubsetFeed:
    """Batches of the kept subset gathered and normalised on device.

    images uint8 [N,3,H,W] and labels int64 [N] on the GPU (the whole set, loaded once);
    keep int64 [k] global indices.  Iterating yields (idx, x fp32 [b,3,H,W], y) like the
    reference's MyDataset loader (`data/loader.py:19-23`)."""

    def __init__(self, images: torch.Tensor, labels: torch.Tensor, keep, batch_size: int,
                 world: int = 1, rank: int = 0, seed: int = 0, shuffle: bool = True):
        from . import _capi
        if images.device.type != "cuda":
            raise RuntimeError("DeviceSubsetFeed needs the dataset resident on a GPU "
                               "(use loader_feed for host/CPU training)")
        _capi.lib()  # fail loudly now if libdd.so is missing
        self._capi = _capi
        self.images, self.labels = images, labels
        self.keep = torch.as_tensor(np.asarray(keep, dtype=np.int64)).to(images.device)
        if self.keep.numel() and (int(self.keep.min()) < 0 or
                                  int(self.keep.max()) >= images.shape[0]):
            raise ValueError("keep indices out of range of the dataset")
        self.batch_size, self.world, self.rank = batch_size, world, rank
        self.seed, self.shuffle = seed, shuffle
        self.epoch = 0
        self._out = torch.empty((batch_size,) + tuple(images.shape[1:]),
                                dtype=torch.float32, device=images.device)

    def set_epoch(self, epoch: int):
        self.epoch = epoch

    def __len__(self):
        per_rank = math.ceil(self.keep.numel() / self.world) if self.keep.numel() else 0
        return math.ceil(per_rank / self.batch_size)

    def __iter__(self):
        pos = epoch_positions(self.keep.numel(), self.world, self.rank, self.epoch, self.seed,
                              self.shuffle).to(self.images.device)
        gidx_all = self.keep[pos]
        for s in range(0, gidx_all.numel(), self.batch_size):
            gidx = gidx_all[s:s + self.batch_size]
            # fresh output per batch: the previous one may still be read by autograd
            out = torch.empty((gidx.numel(),) + tuple(self.images.shape[1:]),
                              dtype=torch.float32, device=self.images.device)
            self._capi.normalize_u8(self.images, MEAN, STD, out, index=gidx)
            yield gidx, out, self.labels[gidx]


class _ShardSampler(torch.utils.data.Sampler):
    def __init__(self, n, world, rank, seed, shuffle):
        self.n, self.world, self.rank, self.seed, self.shuffle = n, world, rank, seed, shuffle
        self.epoch = 0

    def set_epoch(self, epoch):
        self.epoch = epoch

    def __iter__(self):
        return iter(epoch_positions(self.n, self.world, self.rank, self.epoch, self.seed,
                                    self.shuffle).tolist())

    def __len__(self):
        return math.ceil(self.n / self.world) if self.n else 0


def loader_feed(train_dataset, keep, batch_size: int, num_workers: int = 0, world: int = 1,
                rank: int = 0, seed: int = 0, shuffle: bool = True) -> DataLoader:
    """The host path: Subset of MyDataset over the kept examples, sharded per rank with the
    same permutation rule as DeviceSubsetFeed (fixes the loader-in-loader of ddp.py:80,139)."""
    sub = Subset(train_dataset, [int(i) for i in np.asarray(keep, dtype=np.int64)])
    sampler = _ShardSampler(len(sub), world, rank, seed, shuffle)
    return DataLoader(sub, batch_size=batch_size, sampler=sampler, num_workers=num_workers)


def train(epoch, net, optimizer, trainloader, device, criterion):
    """One epoch (reference trainer/trainer.py:5-35).  Returns (mean loss, accuracy %) of
    this rank's batches; loss/accuracy are accumulated on device (one sync per epoch, not
    two per batch as in the reference's `.item()` calls)."""
    net.train()
    loss_sum = torch.zeros((), dtype=torch.float64, device=device)
    correct = torch.zeros((), dtype=torch.int64, device=device)
    total = 0
    nb = 0
    for _, inputs, targets in trainloader:
        inputs = inputs.to(device, non_blocking=True)
        targets = targets.to(device, non_blocking=True)
        optimizer.zero_grad(set_to_none=True)
        outputs = net(inputs)
        loss = criterion(outputs, targets)
        loss.backward()
        optimizer.step()
        loss_sum += loss.detach().double()
        correct += (outputs.detach().argmax(1) == targets).sum()
        total += targets.numel()
        nb += 1
    return (float(loss_sum) / max(nb, 1)), (100.0 * int(correct) / max(total, 1))


@torch.no_grad()
def evaluate(net, testloader, device, criterion, world: int = 1):
    """(mean loss per example, accuracy %) over `testloader`; with world > 1 the example-
    weighted loss sum, correct count and example count are all-reduced before dividing, so
    the loss is the mean over the whole (sharded) test set."""
    net.eval()
    acc = torch.zeros(3, dtype=torch.float64, device=device)  # loss sum, correct, total
    for batch in testloader:
        inputs, targets = batch[-2], batch[-1]
        inputs = inputs.to(device, non_blocking=True)
        targets = targets.to(device, non_blocking=True)
        out = net(inputs)
        # criterion is a batch mean: weight it by the batch's example count
        acc[0] += criterion(out, targets).double() * targets.numel()
        acc[1] += (out.argmax(1) == targets).sum().double()
        acc[2] += targets.numel()
    if world > 1:
        dist.all_reduce(acc)
    total = max(float(acc[2]), 1.0)
    return float(acc[0]) / total, 100.0 * float(acc[1]) / total


def save_checkpoint(net, acc, epoch, save_path):
    """{'net', 'acc', 'epoch'} -> save_path/ckpt_{epoch}.pth (trainer/trainer.py:64-71);
    a DDP wrapper is unwrapped so the keys carry no `module.` prefix."""
    module = net.module if hasattr(net, "module") else net
    os.makedirs(save_path, exist_ok=True)
    path = os.path.join(save_path, f"ckpt_{epoch}.pth")
    torch.save({"net": module.state_dict(), "acc": acc, "epoch": epoch}, path)
    return path


def test(epoch, net, testloader, device, criterion, save_path):
    """Evaluate and save the checkpoint (reference trainer/trainer.py:39-71).  Returns acc."""
    _, acc = evaluate(net, testloader, device, criterion)
    save_checkpoint(net, acc, epoch, save_path)
    return acc


def ddp_train(net, feed, config: dict, save_path: str, num_epochs: int, test_loader=None,
              device="cpu", log=print):
    """DDP training of `net` on `feed` (DeviceSubsetFeed or loader_feed), ddp.py:127-164.

    The process group must already be initialised (torchrun env; `nccl` = RCCL on GPUs,
    `gloo` on CPU) or world == 1.  Rank 0 saves a trainer-format checkpoint per epoch.
    Returns the per-epoch history [(epoch, train loss, train acc, test acc)]."""
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    net = net.to(device)
    if world > 1:
        ids = [torch.device(device).index] if torch.device(device).type == "cuda" else None
        model = nn.parallel.DistributedDataParallel(net, device_ids=ids)
    else:
        model = net
    criterion = nn.CrossEntropyLoss()
    optimizer = torch.optim.SGD(net.parameters(), lr=config["lr"], momentum=config["momentum"],
                                weight_decay=config["weight_decay"])
    scheduler = torch.optim.lr_scheduler.CosineAnnealingLR(optimizer, T_max=num_epochs)
    start = int(config.get("start_epoch", 0))
    hist = []
    for epoch in range(start, start + num_epochs):
        sampler = getattr(feed, "sampler", feed)
        if hasattr(sampler, "set_epoch"):
            sampler.set_epoch(epoch)
        t0 = time.time()
        loss, tr_acc = train(epoch, model, optimizer, feed, device, criterion)
        te_acc = None
        if test_loader is not None:
            _, te_acc = evaluate(model, test_loader, device, criterion, world)
        if rank == 0:
            save_checkpoint(model, te_acc, epoch, save_path)
            log(f"epoch {epoch}: loss {loss:.4f} train acc {tr_acc:.2f}% "
                f"test acc {te_acc if te_acc is None else round(te_acc, 2)} "
                f"({time.time() - t0:.1f}s)")
        scheduler.step()
        hist.append((epoch, loss, tr_acc, te_acc))
    return hist


def main(argv=None):
    """torchrun entry: train on a written keep-set (subset_index.write_subset_index).

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \\
        -m data_diet_distributed_amd.sparse_train --subset-index keep.npy --epochs 20
    """
    from .config import load_config
    from .loader import load_data, to_device
    from .resnet import build
    from .subset_index import read_subset_index

    ap = argparse.ArgumentParser(description="DDP sparse training on a Data Diet keep-set")
    ap.add_argument("--config", default="config.yaml")
    ap.add_argument("--subset-index", required=True)
    ap.add_argument("--epochs", type=int, default=None)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--feed", choices=("device", "loader"), default=None)
    args = ap.parse_args(argv)
    cfg = load_config(args.config)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    gpu = torch.cuda.is_available()
    device = torch.device("cuda", local) if gpu else torch.device("cpu")
    if gpu:
        torch.cuda.set_device(device)
    if world > 1:
        dist.init_process_group("nccl" if gpu else "gloo")
    torch.manual_seed(args.seed)
    keep, meta = read_subset_index(args.subset_index)
    train_set, test_set = load_data(cfg["dataset"])
    feed_kind = args.feed or ("device" if gpu else "loader")
    if feed_kind == "device":
        images, labels = to_device(train_set, device)
        feed = DeviceSubsetFeed(images, labels, keep, cfg["batch_size"], world, rank, args.seed)
    else:
        feed = loader_feed(train_set, keep, cfg["batch_size"], cfg["num_workers"], world, rank,
                           args.seed)
    tl = DataLoader(Subset(test_set, list(range(rank, len(test_set), world))), batch_size=100)
    net = build(cfg.get("arch", "resnet18"), cfg.get("num_classes", 10))
    save = cfg["sparse_checkpoint_path"]
    ddp_train(net, feed, cfg, save, args.epochs or cfg["num_epochs"], tl, device)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
