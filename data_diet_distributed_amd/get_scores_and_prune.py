"""Drop-in for reference get_scores_and_prune.py: `sparse_loader` with the same signature,
return value and selection semantics, running on the MI355X kernels of libdd.so.

Reference: get_scores_and_prune.py:8-34.
  :11-20  per batch: forward, softmax - one_hot, L2, per-example .item() into a Python list
          -> here: forward (PyTorch-ROCm), dd_el2n writes the batch's scores into a device
             vector in visit order; no per-example host sync
  :22     samples = int((1-sparsity)*train_samples)            -> dd_keep_count
  :23-24  stable sorted(..., reverse=True)[:samples]            -> dd_select_topk over the
          visit-ordered scores (ties keep visit order), mapped back to dataset indices
  :26-34  Subset(load_data('cifar10') train, indices), assert, shuffled DataLoader
          -> Subset over the CALLER's training set (`train_loader.dataset`: the same
             MyDataset the reference re-loads at :26, without decoding it a second time),
             assert, shuffled DataLoader
Extension keywords (all optional) re-load a named dataset like :26, or write the index file;
with none given the behaviour is the reference's.

Two scoring paths, same batches, same selection:
  fast     (the default whenever it applies, `fast_path()`): the loader's dataset exposes its
           raw uint8 images (torchvision CIFAR10 `.data`/`.targets`, or `.images`/`.labels`)
           behind ToTensor + Normalize, and `net` is a train-mode CIFAR ResNet (BasicBlock or
           Bottleneck).
           The visit batches come from the loader's own batch sampler, drawn with exactly the
           RNG calls `enumerate(train_loader)` makes (so the same shuffle, without decoding a
           single image on the host); the raw set goes to HBM once; each chunk of whole visit
           batches is gathered + normalised on device (dd_normalize_u8_gather) and scored by
           the hand-written grouped train-BN forward (el2n_fast: one BN group per visit
           batch, the reference's per-batch statistics) -> dd_el2n.
  fallback `net(input)` per loader batch (any dataset, any module) -> dd_el2n.
The fast path leaves the scoring net's BN running statistics as they were (the reference's
train-mode forward updates them as a side effect; every reference call site deletes that
net right after: train.py:65, train_sparse.py:30-33, ddp.py:75-80).
"""
from __future__ import annotations

import numpy as np
import torch
from torch.utils.data import DataLoader, Subset

from . import _capi
from .loader import load_data
from .subset_index import write_subset_index
from .synthetic import state_digest


def el2n_scores_from_loader(train_loader, net, device, num_classes=None):
    """Scores of every example the loader yields, in visit order, plus the visited indices.

    Runs `net(input)` exactly as the reference does (:15), so BN follows `net.training`
    (train mode for a freshly built net, as in train.py:59-63).  A label outside [0, C)
    raises LabelError, as the reference's one_hot does (:17)."""
    scores, visit = [], []
    bad = _capi.label_counter(device)
    C = None
    with torch.no_grad():
        for _batch_idx, (idx, inp, target) in enumerate(train_loader):
            inp = inp.to(device, non_blocking=True)
            target = torch.as_tensor(target).to(device, non_blocking=True).to(torch.int64)
            out = net(inp).float().contiguous()
            if num_classes is not None and out.shape[1] != num_classes:
                raise ValueError(f"net produces {out.shape[1]} classes, expected {num_classes}")
            s = torch.empty(out.shape[0], dtype=torch.float32, device=out.device)
            C = out.shape[1]
            _capi.el2n(out, target.contiguous(), score=s, bad_labels=bad)
            scores.append(s)
            visit.append(torch.as_tensor(idx).to(out.device, non_blocking=True))
    if not scores:
        return (torch.empty(0, dtype=torch.float32, device=device),
                torch.empty(0, dtype=torch.int64, device=device))
    _capi.check_labels(bad, C, "sparse_loader")
    return torch.cat(scores), torch.cat(visit).to(torch.int64)


def select_keep_indices(scores_visit: torch.Tensor, visit_idx: torch.Tensor, samples: int):
    """Reference :23-24 on device: positions of the top `samples` scores (descending, ties in
    visit order) mapped to dataset indices."""
    pos, _thr, _nan = _capi.select_topk(scores_visit.contiguous(), samples)
    return visit_idx[pos]


def _unwrap_subsets(ds):
    """(innermost non-Subset dataset, positions into it or None): torch Subset layers peeled
    with their indices composed (Subset(Subset(d, a), b)[j] = d[a[b[j]]])."""
    pos = None
    while isinstance(ds, Subset):
        ind = np.asarray(ds.indices, dtype=np.int64)
        pos = ind if pos is None else ind[pos]
        ds = ds.dataset
    return ds, pos


def _training_set(train_loader, dataset):
    """The dataset the Subset is built over: the training set the loader draws from (the
    reference re-loads the same training set by name at :26), or load_data(dataset) when
    asked.  The scored indices are the `idx` values the index-carrying dataset yields, i.e.
    positions in it, so a loader over a Subset (e.g. re-pruning a loader this function
    returned) builds the new Subset over the underlying dataset, not over the Subset."""
    if dataset is not None:
        return load_data(dataset)[0]
    ds = getattr(train_loader, "dataset", None)
    if ds is None:
        raise ValueError("train_loader has no .dataset: pass dataset=<name> to re-load it")
    return _unwrap_subsets(ds)[0]


# ---- fast path ------------------------------------------------------------------------------
def _mean_std(transform):
    """(mean, std) of ToTensor + Normalize (torchvision Compose, or loader._Normalize), else
    None."""
    from .loader import _Normalize
    if isinstance(transform, _Normalize):
        return ([float(v) for v in transform.mean.flatten()],
                [float(v) for v in transform.std.flatten()])
    ts = getattr(transform, "transforms", None)
    if (type(transform).__name__ != "Compose" or not isinstance(ts, (list, tuple))
            or len(ts) != 2 or type(ts[0]).__name__ != "ToTensor"
            or type(ts[1]).__name__ != "Normalize"
            or getattr(ts[1], "inplace", False) not in (False, True)):
        return None
    try:
        return ([float(v) for v in torch.as_tensor(ts[1].mean).flatten()],
                [float(v) for v in torch.as_tensor(ts[1].std).flatten()])
    except (TypeError, ValueError):
        return None


def raw_source(ds):
    """The raw uint8 set behind an index-carrying dataset, or None.

    `ds` must yield (idx, image, label) with (image, label) = ds.data[idx] (reference
    MyDataset, data/loader.py:13-25) over either a torchvision-CIFAR10-like set (`.data`
    uint8 [N, H, W, C], `.targets`) or an array set (`.images` uint8 [N, C, H, W],
    `.labels`), transformed by ToTensor + Normalize and no target transform.  Returns
    (images uint8 ndarray, layout "NHWC" | "NCHW", labels int64 ndarray, mean, std).  The
    claim is checked on three examples against the dataset's own __getitem__, so an
    unrecognised layout or transform falls back instead of scoring the wrong pixels."""
    inner = getattr(ds, "data", None)
    if type(ds).__name__ != "MyDataset" or inner is None:
        return None
    if getattr(inner, "target_transform", None) is not None:
        return None
    ms = _mean_std(getattr(inner, "transform", None))
    if ms is None:
        return None
    imgs = getattr(inner, "images", None)
    labs = getattr(inner, "labels", None)
    layout = "NCHW"
    if not (isinstance(imgs, np.ndarray) and labs is not None):
        imgs, labs, layout = getattr(inner, "data", None), getattr(inner, "targets", None), "NHWC"
    if not (isinstance(imgs, np.ndarray) and imgs.dtype == np.uint8 and imgs.ndim == 4
            and labs is not None and len(labs) == len(imgs) == len(ds) > 0):
        return None
    C = imgs.shape[3] if layout == "NHWC" else imgs.shape[1]
    if len(ms[0]) != C or len(ms[1]) != C:
        return None
    labs = np.asarray(labs, dtype=np.int64)
    mean = torch.tensor(ms[0])[:, None, None]
    std = torch.tensor(ms[1])[:, None, None]
    for i in sorted({0, len(imgs) // 2, len(imgs) - 1}):
        item = ds[i]
        if not (isinstance(item, (tuple, list)) and len(item) == 3 and int(item[0]) == i
                and int(item[2]) == int(labs[i]) and isinstance(item[1], torch.Tensor)):
            return None
        raw = imgs[i] if layout == "NCHW" else np.transpose(imgs[i], (2, 0, 1))
        want = (torch.from_numpy(np.ascontiguousarray(raw)).float() / 255 - mean) / std
        if item[1].shape != want.shape or not torch.allclose(item[1].float(), want, atol=1e-5):
            return None
    return imgs, layout, labs, ms[0], ms[1]


def _el2n_model(net, device):
    """The engine's copy of a train-mode CIFAR ResNet of BasicBlocks (ResNet-18/34) or
    Bottlenecks (ResNet-50/101/152, reference models/resnet.py:35-63,108-117): its weights and
    the hand kernels' packs, or None when the fast path does not apply to `net` (including a
    net whose widths differ from the standard ones, which the rebuilt copy cannot load)."""
    from .resnet import BasicBlock, Bottleneck, ResNet
    module = net.module if hasattr(net, "module") else net
    if not isinstance(module, ResNet) or module.stem != "cifar":
        return None
    kinds = {type(b) for b in module.blocks()}
    if len(kinds) != 1 or kinds.pop() not in (BasicBlock, Bottleneck):
        return None
    block = type(next(module.blocks()))
    bns = [m for m in module.modules() if isinstance(m, torch.nn.BatchNorm2d)]
    if not module.training or not all(b.training and b.track_running_stats for b in bns):
        return None  # eval-mode scoring: the per-batch forward is exact as it is
    try:
        if next(module.parameters()).device != torch.device(device):
            return None
    except StopIteration:
        return None
    nb = [len(layer) for layer in (module.layer1, module.layer2, module.layer3, module.layer4)]
    sd = module.state_dict()
    eng = ResNet(block, nb, module.linear.out_features, "cifar")
    ref = eng.state_dict()
    if set(sd) != set(ref) or any(sd[k].shape != ref[k].shape for k in ref):
        return None  # non-standard widths: the general path scores it as it is
    eng = eng.to(device)
    eng.load_state_dict(sd)
    eng.eval()
    for p in eng.parameters():
        p.requires_grad_(False)
    eng.prepare_fast_convs()
    return eng


def _replayable(train_loader) -> bool:
    """Whether _visit_batches reproduces the RNG draws of the loader's next enumerate: not for
    a persistent-workers loader that has already been iterated, whose live iterator only
    _reset()s (no base-seed draw); such a loader takes the general path."""
    return not (getattr(train_loader, "persistent_workers", False)
                and getattr(train_loader, "_iterator", None) is not None)


def _visit_batches(train_loader):
    """The index batches `enumerate(train_loader)` would visit, with the same RNG draws
    (torch DataLoader: _BaseDataLoaderIter.__init__ creates the sampler iterator, then draws
    the workers' base seed from loader.generator; the sampler's own draws happen on its first
    batch), without fetching any example."""
    it = iter(train_loader.batch_sampler)
    torch.empty((), dtype=torch.int64).random_(generator=train_loader.generator)
    return [list(b) for b in it]


def _group_size_ok(hw: int, B: int) -> bool:
    """The grouped train-BN kernels have a tile geometry for BN groups of B examples at every
    map of a CIFAR ResNet (hw, hw/2, hw/4, hw/8; stride-2 heads at the last three; a
    Bottleneck's 1x1 convs fall back per conv where their kernel has no tile for it)."""
    lib = _capi.lib()
    if hw % 8:
        return False
    return (all(lib.dd_conv3x3_tiles_per_group(hw >> s, hw >> s, B) > 0 for s in range(4))
            and all(lib.dd_down_tiles_per_group(hw >> s, hw >> s, B) > 0 for s in (1, 2, 3)))


def fast_path(train_loader, net, device):
    """(raw source, engine model) when sparse_loader can score on the hand-written grouped
    train-BN forward, else None (see the module docstring for the conditions).  Decided
    before any RNG draw, so the general path sees the loader exactly as the caller made it."""
    if torch.device(device).type != "cuda":
        return None
    ds = getattr(train_loader, "dataset", None)
    bs = getattr(train_loader, "batch_sampler", None)
    if (ds is None or isinstance(ds, torch.utils.data.IterableDataset)
            or type(bs) is not torch.utils.data.BatchSampler or bs.batch_size <= 0):
        return None  # custom batch samplers may yield any batch shapes: general path
    if not _replayable(train_loader):
        return None
    base, _pos = _unwrap_subsets(ds)
    src = raw_source(base)
    if src is None:
        return None
    imgs, layout = src[0], src[1]
    H, W = imgs.shape[1:3] if layout == "NHWC" else imgs.shape[2:4]
    if H != W or not _group_size_ok(H, bs.batch_size):
        return None
    model = _el2n_model(net, device)
    if model is None:
        return None
    return src, model


def el2n_scores_fast(train_loader, src, model, device, chunk_rows: int = 1024):
    """Scores in visit order + visited indices, like el2n_scores_from_loader, on the hand
    kernels: every visit batch of the loader's BatchSampler (all of size B but a ragged last
    one) is one BN group; chunks of whole batches are gathered + normalised on device."""
    from . import el2n_fast
    imgs, layout, labs, mean, std = src
    B = train_loader.batch_sampler.batch_size
    batches = _visit_batches(train_loader)
    dev = torch.device(device)
    if not batches:
        return (torch.empty(0, dtype=torch.float32, device=dev),
                torch.empty(0, dtype=torch.int64, device=dev))
    _, pos = _unwrap_subsets(train_loader.dataset)
    visit = torch.tensor([i for b in batches for i in b], dtype=torch.int64)
    if pos is not None:  # positions in the loader's Subset -> the index-carrying dataset's idx
        visit = torch.from_numpy(pos)[visit]
    img_d = torch.from_numpy(imgs).to(dev)
    if layout == "NHWC":
        img_d = img_d.permute(0, 3, 1, 2).contiguous()
    lab_d = torch.from_numpy(labs).to(dev)
    visit_d = visit.to(dev)
    n = visit.numel()
    CH = max(B, (chunk_rows // B) * B)
    x = torch.zeros((min(CH, -(-n // B) * B),) + tuple(img_d.shape[1:]), dtype=torch.float32,
                    device=dev)
    scores = torch.empty(n, dtype=torch.float32, device=dev)
    bad = _capi.label_counter(dev)
    with torch.inference_mode():
        for c0 in range(0, n, CH):
            c1 = min(n, c0 + CH)
            rows = c1 - c0
            xb = x[:-(-rows // B) * B]
            if rows < xb.shape[0]:
                xb[rows:].zero_()
            idx = visit_d[c0:c1]
            _capi.normalize_u8(img_d, mean, std, xb[:rows], index=idx)
            logits = el2n_fast.forward_logits(model, xb, B, rows)[:rows]
            _capi.el2n(logits.contiguous(), lab_d[idx], score=scores[c0:c1], bad_labels=bad)
    # a label outside [0, C): the reference's one_hot raises (:17), so does this path
    _capi.check_labels(bad, model.linear.out_features, "sparse_loader")
    return scores, visit_d


def refine_fast_keep_set(train_loader, src, model, device, scores, visit, samples, cfg=None):
    """The exact keep-set of the fast path (reference :18-24 ranks exact fp32 scores): the
    visit batches nearest the threshold are re-scored on the plain-fp32 forward
    (el2n_fast.forward_logits_fp32: fp32 convs, the same per-batch train-mode BN) until the
    expected number of examples on the wrong side is under `refine_tol`
    (scoring.refine_keep_set, the engine's refinement; the unit is one visit batch, whose BN
    couples its rows, and ties keep visit order).  Returns (keep positions in visit order,
    the refinement record)."""
    from . import el2n_fast
    from .scoring import ScoreConfig, refine_keep_set
    cfg = cfg or ScoreConfig()
    imgs, layout, labs, mean, std = src
    B = train_loader.batch_sampler.batch_size
    dev = torch.device(device)
    img_d = torch.from_numpy(imgs).to(dev)
    if layout == "NHWC":
        img_d = img_d.permute(0, 3, 1, 2).contiguous()
    lab_d = torch.from_numpy(labs).to(dev)

    def rescore(rows):
        """fp32 scores of the visit-position ranges `rows` (whole visit batches; only the
        last visit batch can be ragged, and it comes last), `refine_groups` batches per
        launch, each its own BN group."""
        outs = []
        step = cfg.refine_groups
        with torch.inference_mode():
            for c in range(0, len(rows), step):
                part = rows[c:c + step]
                G = 1 << (len(part) - 1).bit_length()  # few distinct MIOpen batch sizes
                x = torch.zeros((G * B,) + tuple(img_d.shape[1:]), dtype=torch.float32,
                                device=dev)
                sel, idx = [], []
                for gi, (r0, r1) in enumerate(part):
                    ix = visit[r0:r1]
                    _capi.normalize_u8(img_d, mean, std, x[gi * B:gi * B + (r1 - r0)], index=ix)
                    sel.append(torch.arange(gi * B, gi * B + (r1 - r0), device=dev))
                    idx.append(ix)
                sel, idx = torch.cat(sel), torch.cat(idx)
                n_valid = (len(part) - 1) * B + (part[-1][1] - part[-1][0])
                logits = el2n_fast.forward_logits_fp32(model, x, B, n_valid)
                out = torch.empty(sel.numel(), dtype=torch.float32, device=dev)
                _capi.el2n(logits[sel].float().contiguous(), lab_d[idx].contiguous(), score=out)
                outs.append(out)
        return torch.cat(outs)

    _, kept_pos, info = refine_keep_set(scores, samples, B, rescore, cfg)
    return kept_pos, dict(method="el2n", **info)


def sparse_loader(train_loader, train_samples, net, device, sparsity, batch_size, num_workers,
                  *, dataset=None, subset_index_path=None, return_indices=False,
                  fast: bool = True, refine="auto"):
    """Reference-compatible: returns (DataLoader over the kept Subset, samples).

    fast=False forces the general `net(input)` path (same batches, same selection).
    refine=True re-scores the fast path's near-threshold visit batches in plain fp32
    (refine_fast_keep_set; `sparse_loader.last_refine` records what it did); "auto" (default)
    and False keep the fast path's keep-set as it is: its forward runs on fp16 halves, whose
    scores are fp32-grade (ScoreConfig.refine)."""
    from .scoring import normalize_refine
    refine = normalize_refine(refine)
    if torch.device(device).type != "cuda":
        raise ValueError("sparse_loader runs its kernels on a GPU device (libdd.so)")
    module = net.module if hasattr(net, "module") else net
    # digest of the checkpoint as handed in: a train-mode forward (reference semantics)
    # updates the BN running statistics while scoring
    digest = state_digest(module.state_dict()) if subset_index_path else None
    fp = fast_path(train_loader, net, device) if fast else None
    sparse_loader.last_path = "fast" if fp is not None else "general"
    if fp is not None:
        scores, visit = el2n_scores_fast(train_loader, fp[0], fp[1], device)
    else:
        scores, visit = el2n_scores_from_loader(train_loader, net, device)
    samples = _capi.keep_count(train_samples, sparsity)
    if samples < 0 or samples > scores.numel():
        raise ValueError(f"keep count {samples} outside [0, {scores.numel()}]")
    sparse_loader.last_refine = None
    if fp is not None and refine is True and 0 < samples < scores.numel():
        pos, sparse_loader.last_refine = refine_fast_keep_set(
            train_loader, fp[0], fp[1], device, scores, visit, samples)
        kept = visit[pos]
    else:
        kept = select_keep_indices(scores, visit, samples)
    indices = kept.cpu().tolist()  # one device->host copy for the whole keep-set

    train_dense = _training_set(train_loader, dataset)
    train_subset = Subset(train_dense, indices)
    assert len(train_subset) == samples
    print(len(train_subset))
    if subset_index_path:
        write_subset_index(subset_index_path, indices,
                           {"n": int(train_samples), "sparsity": float(sparsity),
                            "score_methods": ["el2n"], "select_by": "el2n", "K": 1,
                            "arch": type(module).__name__,
                            "num_classes": int(getattr(getattr(module, "linear", None),
                                                       "out_features", 0)) or None,
                            "bn_mode": "train" if module.training else "eval",
                            "order": "loader visit order (reference semantics)",
                            "checkpoint_digests": [digest]})
    sparse_train_loader = DataLoader(train_subset, batch_size=batch_size, shuffle=True,
                                     num_workers=num_workers)
    if return_indices:
        return sparse_train_loader, samples, indices
    return sparse_train_loader, samples
