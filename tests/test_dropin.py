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

# keep-set tie band (relative to the threshold score), fixed: see tests/test_gpu_pipeline.py
KEEP_BAND = 6e-4
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
    cfg["bn_mode"] = "batch"
    # score_precision: the default ("split") runs the EL2N forward on fp16 halves
    # and refines the keep-set in fp32 only where the ranking pass has bf16-halves arithmetic
    # (refine "auto"); split_refined forces the refinement, split_fast skips it; bf16x3 keeps
    # every split conv on bf16 halves and refines; fp32 runs the plain fp32 path throughout
    assert e.refine == "auto" and e.fast_convs and e.pegrad_precision == "bf16x3"
    assert e.el2n_operands == "f16x3"
    cfg["score_precision"] = "split_fast"
    assert score.engine_config(cfg).refine is False
    cfg["score_precision"] = "split_refined"
    assert score.engine_config(cfg).refine is True
    assert e.grand_operands == "f16x3"
    cfg["score_precision"] = "bf16x3"
    assert score.engine_config(cfg).el2n_operands == "bf16x3"
    assert score.engine_config(cfg).grand_operands == "bf16x3"
    assert score.engine_config(cfg).refine is True
    cfg["score_precision"] = "bf16x3_fast"
    eb = score.engine_config(cfg)
    assert eb.refine is False and eb.el2n_operands == "bf16x3"
    cfg["score_precision"] = "fp32"
    e32 = score.engine_config(cfg)
    assert (not e32.fast_convs and not e32.fast_el2n and not e32.fused_grand
            and e32.pegrad_precision == "fp32")
    cfg["score_precision"] = "fp16"
    with pytest.raises(ValueError):
        score.engine_config(cfg)
    cfg["score_precision"] = "split"
    assert e.refine_max_frac == 0.08
    cfg["refine_max_frac"] = 0.5
    assert score.engine_config(cfg).refine_max_frac == 0.5
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
@pytest.mark.parametrize("kind", ["torchvision_raw", "tensor_only"])
def test_sparse_loader_reference_call_with_torchvision_style_dataset(cuda, tmp_path, kind):
    """train_sparse.py:15-28 shape of call: ResNet18 in train mode, MyDataset over a
    torchvision-style CIFAR10, the reference's own shuffled loader; the returned loader
    iterates the caller's dataset (reference :26-34) and the index file records digests.
    A set exposing torchvision's raw `.data`/`.targets` takes the fast path (hand-written
    grouped train-BN forward over the loader's own visit batches); one that only yields
    tensors takes the general `net(input)` path.  Both keep the reference's set."""
    from data_diet_distributed_amd import get_scores_and_prune as gsp
    from oracle import el2n as o_el2n
    from oracle import pipeline as o_pipe
    ns = {}
    exec(REF_IMPORTS, ns)  # noqa: S102
    n = 384 + 40  # a ragged last visit batch
    images, labels = synthetic.make_images(n, 10, seed=12)
    sd = synthetic.make_checkpoint("resnet18", 10, seed=4)["net"]
    inner = (TorchvisionCIFAR10Like(images, labels) if kind == "torchvision_raw"
             else _TorchvisionLikeCIFAR(images, labels))
    train = ns["MyDataset"](inner)
    g = torch.Generator().manual_seed(3)
    train_loader = torch.utils.data.DataLoader(train, batch_size=128, shuffle=True, generator=g)
    model = ns["ResNet18"]().to(cuda)
    model.load_state_dict(sd)
    out_loader, samples, idx = ns["sparse_loader"](train_loader, n, model, cuda, 0.5, 125, 0,
                                                   subset_index_path=str(tmp_path / "keep"),
                                                   return_indices=True)
    assert gsp.sparse_loader.last_path == ("fast" if kind == "torchvision_raw" else "general")
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
    assert np.all(np.abs(want[diff] - thr) <= KEEP_BAND * thr), diff
    meta = subset_index.read_subset_index(str(tmp_path / "keep"))[1]
    assert meta["arch"] == "ResNet" and meta["bn_mode"] == "train"
    assert meta["checkpoint_digests"] == [synthetic.state_digest(sd)]
    i0, x0, y0 = next(iter(torch.utils.data.DataLoader(out_loader.dataset, batch_size=1)))
    assert int(i0) in set(idx)
    if kind == "torchvision_raw":
        # the general path on an identically seeded loader: the same keep-set
        g2 = torch.Generator().manual_seed(3)
        loader2 = torch.utils.data.DataLoader(train, batch_size=128, shuffle=True, generator=g2)
        _, _, idx2 = ns["sparse_loader"](loader2, n, model, cuda, 0.5, 125, 0,
                                         return_indices=True, fast=False)
        assert gsp.sparse_loader.last_path == "general"
        diff = np.setxor1d(idx, idx2)
        assert np.all(np.abs(want[diff] - thr) <= KEEP_BAND * thr), diff


@pytest.mark.gpu
def test_sparse_loader_fast_path_over_a_subset_loader(cuda):
    """Re-pruning: a loader over Subset(MyDataset) scores the subset's examples and the new
    Subset is built over the underlying dataset with MyDataset indices (fast path)."""
    from data_diet_distributed_amd import get_scores_and_prune as gsp
    from oracle import el2n as o_el2n
    from oracle import pipeline as o_pipe
    n = 512
    images, labels = synthetic.make_images(n, 10, seed=15)
    sd = synthetic.make_checkpoint("resnet18", 10, seed=2)["net"]
    base = loader.MyDataset(TorchvisionCIFAR10Like(images, labels))
    keep = np.arange(n - 1, -1, -2)  # 256 odd indices, reversed
    ld = torch.utils.data.DataLoader(torch.utils.data.Subset(base, keep.tolist()), batch_size=128)
    from data_diet_distributed_amd.resnet import ResNet18
    net = ResNet18().to(cuda)
    net.load_state_dict(sd)
    out, samples, idx = gsp.sparse_loader(ld, 256, net, cuda, 0.5, 64, 0, return_indices=True)
    assert gsp.sparse_loader.last_path == "fast"
    assert out.dataset.dataset is base and set(idx) <= set(keep.tolist())
    want = o_pipe.el2n_scores(sd, images[keep], labels[keep], 128)
    kept_ref = keep[o_el2n.stable_topk(want, samples)]
    thr = np.sort(want)[::-1][samples - 1]
    diff = np.setxor1d(idx, kept_ref)
    full = np.zeros(n, np.float32)
    full[keep] = want
    assert np.all(np.abs(full[diff] - thr) <= KEEP_BAND * thr), diff
    assert all(out.dataset[j][0] == idx[j] for j in range(3))


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


# ---- sparse_loader fast path: detection and visit order (CPU) --------------------------------
class _TVToTensor:
    """torchvision.transforms.ToTensor on an HWC uint8 ndarray: CHW float32 / 255."""

    def __call__(self, a):
        return torch.from_numpy(np.ascontiguousarray(a.transpose(2, 0, 1))).float().div(255)


class _TVNormalize:
    def __init__(self, mean, std):
        self.mean, self.std, self.inplace = mean, std, False

    def __call__(self, t):
        return (t - torch.tensor(self.mean)[:, None, None]) / torch.tensor(self.std)[:, None, None]


_TVToTensor.__name__ = "ToTensor"
_TVNormalize.__name__ = "Normalize"


class Compose:
    def __init__(self, ts):
        self.transforms = ts

    def __call__(self, x):
        for t in self.transforms:
            x = t(x)
        return x


class TorchvisionCIFAR10Like(torch.utils.data.Dataset):
    """The attributes torchvision.datasets.CIFAR10 has: `.data` uint8 [N, 32, 32, 3] (HWC),
    `.targets` list of int, `.transform`, `.target_transform`."""

    def __init__(self, images_nchw, labels, mean=loader.MEAN, std=loader.STD):
        self.data = np.ascontiguousarray(images_nchw.transpose(0, 2, 3, 1))
        self.targets = [int(v) for v in labels]
        self.transform = Compose([_TVToTensor(), _TVNormalize(mean, std)])
        self.target_transform = None

    def __len__(self):
        return len(self.targets)

    def __getitem__(self, i):
        return self.transform(self.data[i]), self.targets[i]


def test_raw_source_recognises_torchvision_and_array_sets():
    from data_diet_distributed_amd import get_scores_and_prune as g
    images, labels = synthetic.make_images(20, 10, seed=3)
    src = g.raw_source(loader.MyDataset(TorchvisionCIFAR10Like(images, labels)))
    assert src is not None and src[1] == "NHWC" and src[0].shape == (20, 32, 32, 3)
    np.testing.assert_array_equal(src[2], labels)
    src = g.raw_source(loader.MyDataset(loader.ArrayImageDataset(images, labels)))
    assert src is not None and src[1] == "NCHW"
    assert np.allclose(src[3], loader.MEAN) and np.allclose(src[4], loader.STD)
    # no raw arrays, a transform that is not ToTensor + Normalize, or arrays that do not
    # match what __getitem__ returns -> general path
    assert g.raw_source(loader.MyDataset(_TorchvisionLikeCIFAR(images, labels))) is None
    tv = TorchvisionCIFAR10Like(images, labels)
    tv.transform = Compose([_TVToTensor()])
    assert g.raw_source(loader.MyDataset(tv)) is None
    tv = TorchvisionCIFAR10Like(images, labels)
    tv.data = tv.data[::-1].copy()  # arrays disagree with the examples
    tv.__class__ = type("Lying", (TorchvisionCIFAR10Like,), {
        "__getitem__": lambda self, i: (self.transform(np.ascontiguousarray(
            self.data[len(self.data) - 1 - i])), self.targets[i])})
    assert g.raw_source(loader.MyDataset(tv)) is None


def test_unwrap_subsets_composes_indices():
    from data_diet_distributed_amd import get_scores_and_prune as g
    base = loader.MyDataset(loader.ArrayImageDataset(*synthetic.make_images(30, 10, seed=1)))
    inner = torch.utils.data.Subset(base, list(range(29, -1, -2)))  # 29, 27, ..., 1
    outer = torch.utils.data.Subset(inner, [3, 0, 7])
    ds, pos = g._unwrap_subsets(outer)
    assert ds is base and pos.tolist() == [23, 29, 15]
    assert [outer[j][0] for j in range(3)] == pos.tolist()
    loader_ = torch.utils.data.DataLoader(outer, batch_size=2)
    assert g._training_set(loader_, None) is base


@pytest.mark.parametrize("seeded", [True, False])
def test_visit_batches_follow_the_loaders_shuffle(seeded):
    """The fast path's index batches are the ones `enumerate(train_loader)` yields, and it
    consumes the same RNG draws (so later shuffles are unchanged too)."""
    from data_diet_distributed_amd import get_scores_and_prune as g
    ds = loader.MyDataset(loader.ArrayImageDataset(*synthetic.make_images(50, 10, seed=2)))

    def make():
        gen = torch.Generator().manual_seed(5) if seeded else None
        return torch.utils.data.DataLoader(ds, batch_size=16, shuffle=True, generator=gen)

    torch.manual_seed(11)
    ref_loader = make()
    ref = [b[0].tolist() for b in ref_loader]
    ref_next = torch.rand(3) if not seeded else torch.rand(3, generator=ref_loader.generator)
    torch.manual_seed(11)
    got_loader = make()
    got = g._visit_batches(got_loader)
    got_next = torch.rand(3) if not seeded else torch.rand(3, generator=got_loader.generator)
    assert got == ref and [len(b) for b in got] == [16, 16, 16, 2]
    assert torch.equal(ref_next, got_next)


def test_dataset_size_defaults_without_synthetic_n(monkeypatch):
    """A synthetic config without `synthetic_n` (and no $DD_SYNTHETIC_N) gets the size of the
    set it stands for, like loader._synthetic; a non-positive size raises."""
    monkeypatch.delenv("DD_SYNTHETIC_N", raising=False)
    assert score.dataset_size({"dataset": "synthetic-cifar10"}) == 50000
    assert score.dataset_size({"dataset": "synthetic-imagenet"}) == 1281167
    monkeypatch.setenv("DD_SYNTHETIC_N", "640")
    assert score.dataset_size({"dataset": "synthetic-cifar100"}) == 640
    assert score.dataset_size({"dataset": "synthetic-cifar10", "synthetic_n": 96}) == 96
    monkeypatch.setenv("DD_SYNTHETIC_N", "0")
    with pytest.raises(ValueError):
        score.dataset_size({"dataset": "synthetic-cifar10"})
    assert score.dataset_size({"dataset": "cifar10"}) is None


def test_fast_path_refuses_what_it_cannot_replay_or_load():
    """(1) a persistent-workers loader that has been iterated draws no base seed
    on its next enumerate, so the fast path's RNG replay would visit other batches: general
    path; (2) a BasicBlock ResNet with non-standard widths cannot be rebuilt by block counts:
    _el2n_model returns None instead of raising in load_state_dict."""
    from data_diet_distributed_amd import get_scores_and_prune as gsp
    from data_diet_distributed_amd.resnet import ResNet18
    ds = loader.MyDataset(loader.ArrayImageDataset(*synthetic.make_images(8, 10, seed=1)))
    assert gsp._replayable(torch.utils.data.DataLoader(ds, batch_size=4))
    ld = torch.utils.data.DataLoader(ds, batch_size=4, num_workers=1, persistent_workers=True)
    assert gsp._replayable(ld)          # never iterated: its first enumerate draws as usual
    ld._iterator = object()
    assert not gsp._replayable(ld)
    net = ResNet18()
    net.layer1[0].conv1 = torch.nn.Conv2d(64, 32, 3, padding=1, bias=False)
    net.layer1[0].bn1 = torch.nn.BatchNorm2d(32)
    net.layer1[0].conv2 = torch.nn.Conv2d(32, 64, 3, padding=1, bias=False)
    net.train()
    assert gsp._el2n_model(net, "cpu") is None


@pytest.mark.gpu
def test_sparse_loader_fast_path_bottleneck_resnet50(cuda):
    """The reference's ResNet50() (Bottleneck, models/resnet.py:35-63,108-109) through the
    reference entry point takes the fast path (grouped train-BN forward on the 1x1 / 3x3 /
    stride-2 kernels); its keep-set equals the general net(input) path's and the CPU
    oracle's outside the tie band, ragged last batch included."""
    from data_diet_distributed_amd import get_scores_and_prune as gsp
    from data_diet_distributed_amd.resnet import ResNet50
    from oracle import el2n as o_el2n
    from oracle import pipeline as o_pipe
    n = 256 + 40
    images, labels = synthetic.make_images(n, 10, seed=19)
    sd = synthetic.make_checkpoint("resnet50", 10, seed=6)["net"]
    ds = loader.MyDataset(TorchvisionCIFAR10Like(images, labels))
    net = ResNet50().to(cuda)
    net.load_state_dict(sd)
    got = {}
    for fast in (True, False):
        ld = torch.utils.data.DataLoader(ds, batch_size=128, shuffle=False)
        _, samples, idx = gsp.sparse_loader(ld, n, net, cuda, 0.5, 64, 0, return_indices=True,
                                            fast=fast)
        assert gsp.sparse_loader.last_path == ("fast" if fast else "general")
        got[fast] = np.array(idx)
    want = o_pipe.el2n_scores(sd, images, labels, 128)
    thr = np.sort(want)[::-1][samples - 1]
    for fast in (True, False):
        diff = np.setxor1d(got[fast], o_el2n.stable_topk(want, samples))
        assert np.all(np.abs(want[diff] - thr) <= KEEP_BAND * thr), (fast, diff)
