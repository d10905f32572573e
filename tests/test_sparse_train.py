"""Sparse training on the kept set (reference ddp.py:127-164,
trainer/trainer.py, train_sparse.py).

CPU: the per-rank shard rule equals torch's DistributedSampler; shards cover the keep-set;
a gloo world-2 DDP run over `loader_feed` keeps both ranks' weights identical and writes a
trainer-format checkpoint the scoring side loads back.  GPU: `DeviceSubsetFeed` (one
dd_normalize_u8_gather launch per batch) yields exactly the host loader's batches, and a
DDP-free training epoch on it runs.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
from torch.utils.data import DistributedSampler

from data_diet_distributed_amd import checkpoints, synthetic
from data_diet_distributed_amd.loader import ArrayImageDataset, MyDataset
from data_diet_distributed_amd.resnet import ResNet18
from data_diet_distributed_amd.sparse_train import (DeviceSubsetFeed, ddp_train,
                                                    epoch_positions, loader_feed)

CFG = {"lr": 0.01, "momentum": 0.9, "weight_decay": 5e-4, "start_epoch": 0}


@pytest.mark.parametrize("n,world", [(10, 1), (10, 3), (25, 4), (7, 8), (128, 2)])
@pytest.mark.parametrize("epoch", [0, 3])
def test_shard_rule_equals_distributed_sampler(n, world, epoch):
    for rank in range(world):
        s = DistributedSampler(list(range(n)), num_replicas=world, rank=rank, shuffle=True,
                               seed=5)
        s.set_epoch(epoch)
        assert epoch_positions(n, world, rank, epoch, seed=5).tolist() == list(iter(s))


def test_shards_cover_keep_set():
    n, world = 1001, 4
    got = torch.cat([epoch_positions(n, world, r, 2) for r in range(world)])
    assert set(got.tolist()) == set(range(n))
    assert got.numel() == 1004  # padded by wrap-around to a multiple of W


def test_loader_feed_yields_examples_not_batches():
    images, labels = synthetic.make_images(40, 10, seed=1)
    ds = MyDataset(ArrayImageDataset(images, labels))
    keep = np.array([3, 17, 5, 30, 9, 11], dtype=np.int64)
    fl = loader_feed(ds, keep, batch_size=4, world=1, rank=0)
    seen = []
    for idx, x, y in fl:
        assert x.shape[1:] == (3, 32, 32) and x.dtype == torch.float32
        assert torch.equal(y, torch.from_numpy(labels[idx.numpy()]))
        seen += idx.tolist()
    assert sorted(seen) == sorted(keep.tolist())


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(0)  # identical init on every rank (DDP also broadcasts rank 0's)
        images, labels = synthetic.make_images(48, 10, seed=2)
        ds = MyDataset(ArrayImageDataset(images, labels))
        keep = np.arange(0, 48, 2, dtype=np.int64)[::-1].copy()  # 24 kept examples
        feed = loader_feed(ds, keep, batch_size=6, world=world, rank=rank, seed=1)
        test = torch.utils.data.DataLoader(ArrayImageDataset(images[:8], labels[:8]),
                                           batch_size=4)
        hist = ddp_train(ResNet18(), feed, CFG, os.path.join(out_dir, "ck"), 2, test,
                         log=lambda *_: None)
        assert len(hist) == 2
        net_sd = torch.load(os.path.join(out_dir, "ck", "ckpt_1.pth"), weights_only=True) \
            if rank == 0 else None
        del net_sd
        # DDP keeps replicas identical: save each rank's flat parameters
        dist.barrier()
        ck = checkpoints.load_state_dict(os.path.join(out_dir, "ck", "ckpt_1.pth"))
        flat = torch.cat([v.flatten().double() for k, v in sorted(ck.items())
                          if v.is_floating_point()])
        np.save(os.path.join(out_dir, f"r{rank}.npy"), flat.numpy())
    finally:
        dist.destroy_process_group()


def test_gloo_ddp_sparse_train(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    r0, r1 = (np.load(tmp_path / f"r{r}.npy") for r in range(world))
    assert np.array_equal(r0, r1)
    ck = torch.load(tmp_path / "ck" / "ckpt_1.pth", weights_only=True)
    assert set(ck) == {"net", "acc", "epoch"} and ck["epoch"] == 1
    assert not any(k.startswith("module.") for k in ck["net"])
    m = checkpoints.build_models([str(tmp_path / "ck" / "ckpt_1.pth")], device="cpu")[0]
    assert isinstance(m, torch.nn.Module)


def test_device_feed_requires_gpu():
    images, labels = synthetic.make_images(8, 10, seed=0)
    with pytest.raises(RuntimeError):
        DeviceSubsetFeed(torch.from_numpy(images), torch.from_numpy(labels), [0, 1], 2)


@pytest.mark.gpu
def test_device_feed_matches_host_loader(cuda):
    images, labels = synthetic.make_images(300, 10, seed=3)
    ds = MyDataset(ArrayImageDataset(images, labels))
    keep = np.random.default_rng(0).permutation(300)[:150].astype(np.int64)
    for world, rank in [(1, 0), (3, 2)]:
        host = loader_feed(ds, keep, 32, world=world, rank=rank, seed=4)
        dev = DeviceSubsetFeed(torch.from_numpy(images).to(cuda),
                               torch.from_numpy(labels).to(cuda), keep, 32, world, rank, seed=4)
        for epoch in (0, 1):
            host.sampler.set_epoch(epoch)
            dev.set_epoch(epoch)
            nb = 0
            for (hi, hx, hy), (di, dx, dy) in zip(host, dev):
                assert torch.equal(hi, di.cpu()) and torch.equal(hy, dy.cpu())
                torch.testing.assert_close(dx.cpu(), hx, rtol=0, atol=2e-6)
                nb += 1
            assert nb == len(dev) == len(host)


@pytest.mark.gpu
def test_device_feed_training_epoch(cuda, tmp_path):
    images, labels = synthetic.make_images(256, 10, seed=4)
    keep = np.arange(0, 256, 2, dtype=np.int64)
    feed = DeviceSubsetFeed(torch.from_numpy(images).to(cuda),
                            torch.from_numpy(labels).to(cuda), keep, 64)
    torch.manual_seed(0)
    hist = ddp_train(ResNet18(), feed, CFG, str(tmp_path), 2, device=cuda, log=lambda *_: None)
    assert len(hist) == 2 and all(np.isfinite(h[1]) for h in hist)
    assert os.path.exists(tmp_path / "ckpt_1.pth")


def test_evaluate_loss_is_mean_over_examples():
    """Ragged test batches: the loss is the mean over every example, not a mean of batch
    means."""
    from data_diet_distributed_amd.sparse_train import evaluate
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Flatten(), torch.nn.Linear(12, 4))
    x = torch.randn(10, 3, 2, 2)
    y = torch.randint(0, 4, (10,))
    loader = torch.utils.data.DataLoader(torch.utils.data.TensorDataset(x, y), batch_size=4)
    crit = torch.nn.CrossEntropyLoss()
    loss, acc = evaluate(net, loader, "cpu", crit)
    with torch.no_grad():
        out = net(x)
        want = float(crit(out, y))
        want_acc = 100.0 * float((out.argmax(1) == y).sum()) / 10
    assert abs(loss - want) < 1e-6 and abs(acc - want_acc) < 1e-9
