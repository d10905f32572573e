"""The drop-in boundary for the reference's callers (train.py:7, train_sparse.py:1, ddp.py:14
star-import `get_scores_and_prune`, `data`, `models`, `trainer`) and the config-driven
scoring entry (reference config -> scoring flow, train.py:36-64, ddp.py:54-77).

CPU: the root shims expose every name the reference scripts use; the CIFAR reader accepts
torchvision's download layout and refuses anything but arrays in it; config keys map onto
the engine.  GPU: sparse_loader called the reference way with a torchvision-style dataset
(no raw arrays, tensors from a transform), and the config entry at K = 3 read back through
subset_loader.
"""
import os
import pickle

import numpy as np
import pytest
import torch

from data_diet_distributed_amd import checkpoints, config, loader, score, subset_index, synthetic

# the import lines of the reference scripts (train_sparse.py:1-4, train.py:4-7)
REF_IMPORTS = ("from get_scores_and_prune import *\nfrom data import *\n"
               "from models import *\nfrom trainer import *\n")


def test_root_shims_expose_the_reference_namespace():
    ns = {}
    exec(REF_IMPORTS, ns)  # noqa: S102 - fixed text above
    for name in ("sparse_loader", "get_dataloader", "load_data", "MyDataset", "transform",
                 "ResNet18", "ResNet50", "BasicBlock", "Bottleneck", "train", "test", "os",
                 "torch", "DataLoader"):
        assert name in ns, name
    from data_diet_distributed_amd.get_scores_and_prune import sparse_loader
    assert ns["sparse_loader"] is sparse_loader
    net = ns["ResNet18"]()
    assert len(net.state_dict()) == 122  # reference key set


def _write_py_batches(root, n_per=6, seed=0):
    d = os.path.join(root, "cifar-10-batches-py")
    os.makedirs(d)
    rng = np.random.default_rng(seed)
    allx, ally = [], []
    for nm in [f"data_batch_{i}" for i in range(1, 6)] + ["test_batch"]:
        x = rng.integers(0, 256, (n_per, 3072), dtype=np.uint8)
        y = [int(v) for v in rng.integers(0, 10, n_per)]
        with open(os.path.join(d, nm), "wb") as f:  # the python-2 era protocol of the archive
            pickle.dump({b"batch_label": b"b", b"labels": y, b"data": x,
                         b"filenames": [b"f"] * n_per}, f, protocol=2)
        allx.append(x)
        ally.append(y)
    return allx, ally


def test_cifar10_torchvision_layout(tmp_path):
    xs, ys = _write_py_batches(str(tmp_path))
    train, test = loader.load_data("cifar10", root=str(tmp_path))
    assert len(train) == 30 and len(test) == 6
    np.testing.assert_array_equal(train.images, np.concatenate(xs[:5]).reshape(-1, 3, 32, 32))
    np.testing.assert_array_equal(train.labels, np.concatenate(ys[:5]))
    idx, img, lab = train[7]
    assert idx == 7 and img.shape == (3, 32, 32) and lab == ys[1][1]
    # ToTensor + Normalize of the reference transform (data/loader.py:8-11)
    want = (torch.from_numpy(train.images[7]).float() / 255 -
            torch.tensor(loader.MEAN)[:, None, None]) / torch.tensor(loader.STD)[:, None, None]
    torch.testing.assert_close(img, want)


def test_cifar_reader_refuses_code(tmp_path):
    class Evil:
        def __reduce__(self):
            return (os.system, ("true",))
    d = tmp_path / "cifar-10-batches-py"
    d.mkdir()
    for nm in [f"data_batch_{i}" for i in range(1, 6)] + ["test_batch"]:
        with open(d / nm, "wb") as f:
            pickle.dump({b"data": Evil(), b"labels": [0]}, f, protocol=2)
    with pytest.raises(pickle.UnpicklingError, match="refused"):
        loader.load_data("cifar10", root=str(tmp_path))


def test_config_keys_map_onto_the_engine(tmp_path):
    p = tmp_path / "c.yaml"
    p.write_text("dataset: synthetic-cifar10\nbatch_size: 128\nscore_methods: [el2n, grand]\n"
                 "select_by: grand\nbn_mode: train\npegrad_method: direct\ngrand_batch: 512\n"
                 "score_checkpoints: 3\nscore_gpus: 2\nsubset_index_path: out/keep\n")
    cfg = config.load_config(str(p))
    e = score.engine_config(cfg)
    assert e.methods == ("el2n", "grand") and e.select_by == "grand"
    assert e.el2n_bn == "batch" and e.pegrad_method == "direct" and e.grand_batch == 512
    cfg["bn_mode"] = "eval"
    assert score.engine_config(cfg).el2n_bn == "running"
    cfg["bn_mode"] = "bogus"
    with pytest.raises(ValueError):
        score.engine_config(cfg)
    args = score.parse(["--config", str(p), "--sparsity", "0.3", "--gpus", "1"])
    assert args.sparsity == 0.3 and args.gpus == 1


def test_repo_config_yaml_has_every_reference_key():
    cfg = config.load_config(os.path.join(os.path.dirname(__file__), "..", "config.yaml"))
    assert all(k in cfg for k in config.REFERENCE_KEYS)


class _TorchvisionLikeCIFAR(torch.utils.data.Dataset):
    """What torchvision.datasets.CIFAR10(transform=transform) yields: (fp32 CHW tensor,
    int label); no raw arrays exposed."""

    def __init__(self, images, labels):
        self._x, self._y = images, labels

    def __len__(self):
        return len(self._y)

    def __getitem__(self, i):
        return loader.transform(self._x[i]), int(self._y[i])


@pytest.mark.gpu
def test_sparse_loader_reference_call_with_torchvision_style_dataset(cuda, tmp_path):
    """train_sparse.py:15-28 shape of call: ResNet18 in train mode, MyDataset over a
    torchvision-style CIFAR10, the reference's own shuffled loader; the returned loader
    iterates the caller's dataset (reference :26-34) and the index file records digests."""
    from oracle import el2n as o_el2n
    from oracle import pipeline as o_pipe
    ns = {}
    exec(REF_IMPORTS, ns)  # noqa: S102
    n = 384
    images, labels = synthetic.make_images(n, 10, seed=12)
    sd = synthetic.make_checkpoint("resnet18", 10, seed=4)["net"]
    train = ns["MyDataset"](_TorchvisionLikeCIFAR(images, labels))
    g = torch.Generator().manual_seed(3)
    train_loader = torch.utils.data.DataLoader(train, batch_size=128, shuffle=True, generator=g)
    model = ns["ResNet18"]().to(cuda)
    model.load_state_dict(sd)
    out_loader, samples, idx = ns["sparse_loader"](train_loader, n, model, cuda, 0.5, 125, 0,
                                                   subset_index_path=str(tmp_path / "keep"),
                                                   return_indices=True)
    assert samples == o_el2n.keep_count(n, 0.5) == len(idx) == len(out_loader.dataset)
    assert out_loader.dataset.dataset is train  # the caller's dataset, not a re-load
    # reference semantics: the batches are the shuffled loader's; re-score them on the CPU
    visit = [int(i) for (bi, _, _) in torch.utils.data.DataLoader(
        train, batch_size=128, shuffle=True, generator=torch.Generator().manual_seed(3))
        for i in bi]
    want = np.empty(n, np.float32)
    for b in range(0, n, 128):
        sel = np.array(visit[b:b + 128])
        want[sel] = o_pipe.el2n_scores(sd, images[sel], labels[sel], 128)
    kept_ref = [visit[i] for i in o_el2n.stable_topk(want[visit], samples)]
    thr = np.sort(want)[::-1][samples - 1]
    diff = np.setxor1d(idx, kept_ref)
    assert np.all(np.abs(want[diff] - thr) <= 1e-5 * thr), diff
    meta = subset_index.read_subset_index(str(tmp_path / "keep"))[1]
    assert meta["arch"] == "ResNet" and meta["bn_mode"] == "train"
    assert meta["checkpoint_digests"] == [synthetic.state_digest(sd)]
    i0, x0, y0 = next(iter(torch.utils.data.DataLoader(out_loader.dataset, batch_size=1)))
    assert int(i0) in set(idx)


@pytest.mark.gpu
def test_config_entry_k3_roundtrip(cuda, tmp_path):
    """`python -m data_diet_distributed_amd.score --config` at K = 3 (EL2N + GraNd), read back
    through subset_loader; scores equal the oracle's ensemble."""
    from oracle import pipeline as o_pipe
    n = 320
    ck = tmp_path / "checkpoint"
    sds = []
    for s in range(3):
        c = synthetic.make_checkpoint("resnet18", 10, seed=20 + s)
        os.makedirs(ck / f"seed{s}")
        torch.save(c, ck / f"seed{s}" / "ckpt_19.pth")
        sds.append(c["net"])
    cfgp = tmp_path / "config.yaml"
    cfgp.write_text(f"dataset: synthetic-cifar10\nsynthetic_n: {n}\nsynthetic_seed: 6\n"
                    f"batch_size: 128\nsparsity: 0.7\ncheckpoint_path: {ck}\n"
                    f"score_methods: [el2n, grand]\nselect_by: el2n\nscore_checkpoints: 3\n"
                    f"grand_batch: 128\nsubset_index_path: {tmp_path / 'idx' / 'keep'}\n")
    assert score.main(["--config", str(cfgp)]) == 0
    idx, meta = subset_index.read_subset_index(str(tmp_path / "idx" / "keep"))
    assert meta["K"] == 3 and meta["k"] == 96 and meta["score_methods"] == ["el2n", "grand"]
    assert meta["checkpoint_digests"] == [synthetic.state_digest(s) for s in sds]
    images, labels = synthetic.make_images(n, 10, seed=6)
    want = sum(o_pipe.el2n_scores(sd, images, labels, 128) for sd in sds) / np.float32(3)
    got = np.load(str(tmp_path / "idx" / "keep") + ".scores.npz")
    np.testing.assert_allclose(got["el2n"], want, rtol=1e-3)
    ds = loader.MyDataset(loader.ArrayImageDataset(images, labels))
    sub = subset_index.subset_loader(ds, str(tmp_path / "idx" / "keep"), batch_size=32)
    seen = sorted(int(i) for b in sub for i in b[0])
    assert seen == sorted(idx.tolist()) and len(seen) == 96
