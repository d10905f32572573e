"""End-to-end parity on the GPU: scoring engine and `sparse_loader` drop-in vs the golden
vectors of the reference (EL2N) and the CPU oracle (GraNd, ResNet-50/CIFAR-100).

Tolerance (north star): scores within 1e-3 relative (fp32); kept-index sets equal except for
indices whose score lies within a tie band of the threshold (1e-5 relative; the count of
such swaps is asserted small).
"""
import glob
import json
import os

import numpy as np
import pytest
import torch

from data_diet_distributed_amd import _capi, checkpoints, synthetic
from data_diet_distributed_amd.get_scores_and_prune import sparse_loader
from data_diet_distributed_amd.loader import ArrayImageDataset, MyDataset
from data_diet_distributed_amd.scoring import ScoreConfig, ScoringEngine, shard_bounds
from oracle import el2n as o_el2n
from oracle import pipeline as o_pipe

pytestmark = pytest.mark.gpu
RTOL = 1e-3  # north star: scores within 1e-3 relative
# The EL2N forward's split MFMA on fp16 operand halves (hi*hi + hi*lo + lo*hi, fp32 accumulate:
# ~2^-22 relative per product) carried through 17 BN-normalised layers: measured max relative
# EL2N error 2.4e-5 over the 50 000 reference scores (profiles/r05_s2/keepset_swaps.json; plain
# fp32 MIOpen: 2.0e-5; on bf16 halves it was 2.2e-4).  SCORE_REL is the fixed bound the EL2N
# engine is held to; KEEP_BAND = 2 x SCORE_REL is the tie band of the tests that check the
# unrefined keep-set (two scores each within SCORE_REL of the reference can trade places only
# if the reference scores lie that close to the threshold).
SCORE_REL = 1e-4
KEEP_BAND = 2 * SCORE_REL
# ... plus an absolute term for softmax-saturated scores (the trained-regime golden, whose
# thresholds sit at EL2N 0.01-0.4): both sides compute e_y = p_y - 1 in fp32 with p_y within
# a few 1e-4 of 1, so each carries the rounding of p_y (~ulp(1) = 2^-23) as an ABSOLUTE error
# whatever the score; 8 ulps of 1.0 bounds it (the softmax's exp / division order differs)
SCORE_ATOL = 8 * 2.0 ** -24
# The shipped EL2N path (fp16 halves; ScoreConfig.refine "auto" leaves it unrefined), and any
# path with the near-threshold fp32 re-scoring, must keep the reference's kept set except for
# indices whose reference score is within EXACT_ULPS fp32 ulps of the threshold (a tie up to
# the last bits of CPU-vs-GPU fp32 rounding).
EXACT_ULPS = 16
# GraNd has no reference output: its oracle runs in float64 (the fp32 CPU restatement is
# itself off by up to 35 % on near-zero scores and 0.2 % on chaotic large ones; see
# oracle/pipeline.grand_scores)
F64 = torch.float64
# A ReLU gate whose float64 pre-activation lies within GATE_REL of zero (relative to that
# example's RMS of the tensor) can fall either way under fp32 rounding of the conv that feeds
# it (fp32 pre-activations carry ~1e-6 of the layer scale; MIOpen's solvers differ per run).
# The GraNd cross-checks against the MIOpen paths exempt an example from RTOL only when it has
# such a gate AND its score equals the float64 oracle with those gates flipped
# (oracle.resnet_fn.gate_flip) to RTOL: the deviation is then the gate, not the arithmetic.
GATE_REL = 1e-5
GOLDEN = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "el2n_*.npz")))


def _case(path):
    d = dict(np.load(path))
    n, dseed = int(d["n"]), int(d["data_seed"])
    images, labels = synthetic.make_images(n, 10, seed=dseed)
    assert synthetic.digest(images, labels) == str(d["images_digest"])
    sds = []
    for s in d["ckpt_seeds"].tolist():
        sd = synthetic.make_checkpoint("resnet18", 10, seed=s)["net"]
        if f"ckpt{s}_linear_weight" in d:  # the trained-regime case: the fitted classifier
            sd["linear.weight"] = torch.from_numpy(d[f"ckpt{s}_linear_weight"])
            sd["linear.bias"] = torch.from_numpy(d[f"ckpt{s}_linear_bias"])
        assert synthetic.state_digest(sd) == str(d[f"ckpt{s}_digest"])
        sds.append(sd)
    return d, images, labels, sds


def _outside_band(scores, a, b, k, rel=1e-5):
    diff = np.setxor1d(a, b)
    if k == 0 or diff.size == 0:
        return diff
    thr = np.sort(scores)[::-1][k - 1]
    return diff[np.abs(scores[diff] - thr) > rel * abs(thr)]


def _ulp_band(scores, k, ulps=EXACT_ULPS):
    """`ulps` fp32 ulps of the k-th largest score, relative to it."""
    thr = np.float32(np.sort(scores)[::-1][k - 1])
    return ulps * float(np.spacing(np.abs(thr))) / float(abs(thr))


def _swap_record(want, got, kept, ref_kept, k):
    """How a kept set differs from the reference's: swapped indices, the worst distance of a
    swapped index's reference score from the threshold (relative, and in fp32 ulps of the
    threshold), and the band the test allows."""
    diff = np.setxor1d(kept, ref_kept)
    thr = np.float32(np.sort(want)[::-1][k - 1]) if k else np.float32(0)
    ulp = float(np.spacing(np.abs(thr))) if k else 0.0
    worst = float(np.max(np.abs(want[diff] - thr))) if diff.size else 0.0
    return {"k": int(k), "swaps": int(diff.size), "threshold": float(thr),
            "worst_swap_rel": worst / float(abs(thr)) if k else 0.0,
            "worst_swap_ulps": worst / ulp if ulp else 0.0,
            "band_rel": KEEP_BAND, "band_ulps": KEEP_BAND * float(abs(thr)) / ulp if ulp else 0.0,
            "max_score_rel_err": float(np.max(np.abs(got / want - 1.0))),
            "max_score_abs_err": float(np.max(np.abs(got - want))),
            "median_score": float(np.median(want))}


@pytest.mark.parametrize("refine", ["auto", True], ids=["default", "refined"])
@pytest.mark.parametrize("path", GOLDEN, ids=os.path.basename)
def test_engine_el2n_matches_reference_golden(cuda, path, refine):
    """Scores within SCORE_REL of the reference's own outputs, and the kept set EQUAL to the
    reference's except for indices whose reference score lies within EXACT_ULPS (16) fp32 ulps
    of the threshold: the default ScoreConfig (fp16-halves forward, refine "auto" = no
    re-scoring) and with the near-threshold fp32 re-scoring forced on.  The swap counts, the
    band in ulps and what the refinement re-scored are recorded
    (profiles/r05_*/keepset_swaps.json via $DD_PARITY_OUT)."""
    d, images, labels, sds = _case(path)
    n = int(d["n"])
    models = checkpoints.build_models(sds, device=cuda)
    eng = ScoringEngine(models, ScoreConfig(methods=("el2n",), refine=refine), cuda)
    img = torch.from_numpy(images).to(cuda)
    lab = torch.from_numpy(labels).to(cuda)
    want = d["ensemble_scores"] if len(sds) > 1 else d[f"ckpt{d['ckpt_seeds'][0]}_scores"]
    records = {}
    for key in [k for k in d if "_kept_" in k and k.startswith(f"ckpt{d['ckpt_seeds'][0]}")]:
        sp = float(key.split("_kept_")[1])
        full, kept, k = eng.run(img, lab, sp)
        got = full["el2n"].cpu().numpy()
        np.testing.assert_allclose(got, want, rtol=SCORE_REL, atol=SCORE_ATOL)
        assert k == o_el2n.keep_count(n, sp)
        ref_kept = d[key] if len(sds) == 1 else o_el2n.stable_topk(want, k)
        kept = kept.cpu().numpy()
        rec = _swap_record(want, got, kept, ref_kept, k)
        rec["refine"] = eng.last_refine
        if k:
            rec["band_ulps"], rec["band_rel"] = EXACT_ULPS, _ulp_band(want, k)
        records[sp] = rec
        if k and k < n:
            assert len(_outside_band(want, kept, ref_kept, k, _ulp_band(want, k))) == 0, rec
        else:
            assert np.array_equal(np.sort(kept), np.sort(ref_kept))
    _record(os.path.basename(path) + ("" if refine == "auto" else "@refined"), records)


def _record(name, records):
    out = os.environ.get("DD_PARITY_OUT")
    if not out:
        return
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    try:
        with open(out) as f:
            allrec = json.load(f)
    except (OSError, ValueError):
        allrec = {}
    allrec[name] = {str(k): v for k, v in records.items()}
    with open(out, "w") as f:
        json.dump(allrec, f, indent=1, sort_keys=True)


def test_el2n_full_size_swaps_split_bf16_vs_fp32_miopen(cuda):
    """At N = 50 000 (the headline size) the keep-set of the split-bf16 engine is compared
    with that of a plain-fp32 GPU path (MIOpen convs + torch BN, per 128-example batch):
    both are within the fixed band of the reference; their swap counts against the
    reference are recorded side by side, so the split-bf16 error is judged against what
    fp32 on a GPU already does."""
    path = [p for p in GOLDEN if "n50000" in p]
    if not path:
        pytest.skip("no full-size golden")
    d, images, labels, sds = _case(path[0])
    n = int(d["n"])
    img = torch.from_numpy(images).to(cuda)
    lab = torch.from_numpy(labels).to(cuda)
    want = d["ckpt0_scores"]
    records = {}
    for name, cfg in (("split_engine", ScoreConfig(methods=("el2n",), refine=False)),
                      ("split_refined", ScoreConfig(methods=("el2n",), refine=True)),
                      ("split_bf16_engine", ScoreConfig(methods=("el2n",), refine=False,
                                                        el2n_operands="bf16x3")),
                      ("fp32_miopen", ScoreConfig(methods=("el2n",), fast_convs=False,
                                                  fast_el2n=False))):
        eng = ScoringEngine(checkpoints.build_models(sds, device=cuda), cfg, cuda)
        for sp in (0.5, 0.7, 0.9):
            full, kept, k = eng.run(img, lab, sp)
            got = full["el2n"].cpu().numpy()
            ref_kept = d[f"ckpt0_kept_{sp}"]
            kept = kept.cpu().numpy()
            assert len(_outside_band(want, kept, ref_kept, k, KEEP_BAND)) == 0, (name, sp)
            records[f"{name}@{sp}"] = _swap_record(want, got, kept, ref_kept, k)
            records[f"{name}@{sp}"]["refine"] = eng.last_refine
    _record("n50000_split_bf16_vs_fp32_miopen", records)


def test_engine_shards_are_rank_invariant(cuda):
    """Train-mode BN scores do not depend on the world size (batch-aligned shards): every
    shard scores exactly the batches the single-rank run does, on kernels that compute a BN
    group's statistics from that group's tiles in a fixed order and a classifier that reduces
    each row alone (dd_linear_forward), so the shard scores are bitwise the full run's."""
    d, images, labels, sds = _case(GOLDEN[1])  # ragged N=2000
    n = int(d["n"])
    eng = ScoringEngine(checkpoints.build_models(sds, device=cuda), ScoreConfig(), cuda)
    img, lab = torch.from_numpy(images).to(cuda), torch.from_numpy(labels).to(cuda)
    full = eng.score_shard(img, lab, 0, n)["el2n"].cpu().numpy()
    for W in (2, 3, 4, 8):
        parts = [eng.score_shard(img, lab, *shard_bounds(n, 128, W, r))["el2n"].cpu().numpy()
                 for r in range(W)]
        got = np.concatenate(parts)
        assert np.array_equal(got, full), (W, float(np.max(np.abs(got / full - 1))))


def test_engine_grand_matches_oracle(cuda):
    images, labels = synthetic.make_images(96, 10, seed=21)
    sds = [synthetic.make_checkpoint("resnet18", 10, seed=s)["net"] for s in (3, 4)]
    ref = np.zeros(96, np.float32)
    for sd in sds:
        ref += o_pipe.grand_scores(sd, images, labels, batch_size=48, dtype=F64)
    ref /= np.float32(2)
    eng = ScoringEngine(checkpoints.build_models(sds, device=cuda),
                        ScoreConfig(methods=("el2n", "grand"), select_by="grand", grand_batch=40),
                        cuda)
    full, kept, k = eng.run(torch.from_numpy(images).to(cuda), torch.from_numpy(labels).to(cuda), 0.5)
    np.testing.assert_allclose(full["grand"].cpu().numpy(), ref, rtol=RTOL)
    assert len(_outside_band(ref, kept.cpu().numpy(), o_el2n.stable_topk(ref, k), k, 1e-4)) == 0


def test_engine_concurrent_passes_match_sequential(cuda):
    """EL2N and GraNd on two HIP streams (ScoreConfig.concurrent_passes) produce the scores
    of the one-stream schedule: the passes share only read-only inputs and packs.  All the
    hand-written kernels are deterministic, so the bar is bit equality."""
    images, labels = synthetic.make_images(1024 + 96, 10, seed=23)
    sds = [synthetic.make_checkpoint("resnet18", 10, seed=s)["net"] for s in (5, 6)]
    img, lab = torch.from_numpy(images).to(cuda), torch.from_numpy(labels).to(cuda)
    out = {}
    for conc in (False, True):
        eng = ScoringEngine(checkpoints.build_models(sds, device=cuda),
                            ScoreConfig(methods=("el2n", "grand"), grand_batch=512,
                                        el2n_chunk=512, concurrent_passes=conc), cuda)
        out[conc] = {m: v.cpu() for m, v in eng.score_shard(img, lab, 0, len(labels)).items()}
    for m in ("el2n", "grand"):
        assert torch.equal(out[False][m], out[True][m]), m


@pytest.mark.parametrize("method", ["direct", "ghost"])
def test_engine_grand_methods_agree(cuda, method):
    images, labels = synthetic.make_images(24, 10, seed=2)
    sds = [synthetic.make_checkpoint("resnet18", 10, seed=9)["net"]]
    ref = o_pipe.grand_scores(sds[0], images, labels, batch_size=24, dtype=F64)
    eng = ScoringEngine(checkpoints.build_models(sds, device=cuda),
                        ScoreConfig(methods=("grand",), select_by="grand", pegrad_method=method),
                        cuda)
    sc = eng.score_shard(torch.from_numpy(images).to(cuda), torch.from_numpy(labels).to(cuda), 0, 24)
    np.testing.assert_allclose(sc["grand"].cpu().numpy(), ref, rtol=RTOL)


def test_engine_resnet50_cifar100(cuda):
    """Config 4 family: ResNet-50, 100 classes (beyond the reference's one_hot(10))."""
    images, labels = synthetic.make_images(40, 100, seed=8)
    sd = synthetic.make_checkpoint("resnet50", 100, seed=1)["net"]
    el2n_ref = o_pipe.el2n_scores(sd, images, labels, batch_size=16)
    grand_ref = o_pipe.grand_scores(sd, images, labels, batch_size=20, dtype=F64)
    models = checkpoints.build_models([sd], "resnet50", 100, device=cuda)
    eng = ScoringEngine(models, ScoreConfig(methods=("el2n", "grand"), batch_size=16,
                                            grand_batch=20), cuda)
    sc = eng.score_shard(torch.from_numpy(images).to(cuda), torch.from_numpy(labels).to(cuda), 0, 40)
    np.testing.assert_allclose(sc["el2n"].cpu().numpy(), el2n_ref, rtol=RTOL)
    np.testing.assert_allclose(sc["grand"].cpu().numpy(), grand_ref, rtol=RTOL)


def test_engine_imagenet_stem_el2n(cuda):
    """Config 5 family at reduced size: ResNet-50 ImageNet stem, 1000 classes, 224x224."""
    images, labels = synthetic.make_images(8, 1000, seed=3, hw=224)
    sd = synthetic.make_checkpoint("resnet50", 1000, seed=2, stem="imagenet")["net"]
    ref = o_pipe.el2n_scores(sd, images, labels, batch_size=4, stem="imagenet")
    models = checkpoints.build_models([sd], "resnet50", 1000, "imagenet", device=cuda)
    eng = ScoringEngine(models, ScoreConfig(batch_size=4), cuda)
    sc = eng.score_shard(torch.from_numpy(images).to(cuda), torch.from_numpy(labels).to(cuda), 0, 8)
    np.testing.assert_allclose(sc["el2n"].cpu().numpy(), ref, rtol=RTOL)


@pytest.mark.parametrize("padded", [True, False])
def test_engine_imagenet_stem_hand_kernels(cuda, monkeypatch, padded):
    """Config 5 network on the hand-written kernels at the reference's batch of 128 (BN groups
    of 128 x 49 positions tile exactly): the 7x7 stem on dd_stem7_forward, the stride-1 3x3s
    at 56 / 28 / 14 / 7 on dd_conv3x3_forward's padded-width tiles and the stride-2 ones on
    dd_down_forward's (padded=False: DD_CONV_PW=0 DD_DOWN_PW=0 DD_STEM7=0, the stem and every
    3x3 on the implicit GEMM), the 1x1s
    on dd_conv1x1_forward; EL2N equals the MIOpen module path (train-mode BN per 128-row
    batch) to fp32 rounding, and a ragged second group of 2 rows is scored too."""
    if not padded:
        monkeypatch.setenv("DD_CONV_PW", "0")
        monkeypatch.setenv("DD_DOWN_PW", "0")
        monkeypatch.setenv("DD_STEM7", "0")
    n = 130
    images, labels = synthetic.make_images(n, 1000, seed=4, hw=224)
    sd = synthetic.make_checkpoint("resnet50", 1000, seed=5, stem="imagenet")["net"]
    x, y = torch.from_numpy(images).to(cuda), torch.from_numpy(labels).to(cuda)
    calls = {"gemm": 0, "c1": 0, "c1u": 0, "c3": 0, "dn": 0, "s7": 0}
    real_gemm, real_c1, real_c1u = _capi.conv_gemm, _capi.conv1x1, _capi.conv1x1_unit_input
    real_c3, real_dn, real_s7 = _capi.conv3x3, _capi.conv_down_unit_input, _capi.stem7

    def count(name, fn):
        def f(*a, **k):
            calls[name] += 1
            return fn(*a, **k)
        return f
    monkeypatch.setattr(_capi, "conv_gemm", count("gemm", real_gemm))
    monkeypatch.setattr(_capi, "conv1x1", count("c1", real_c1))
    monkeypatch.setattr(_capi, "conv1x1_unit_input", count("c1u", real_c1u))
    monkeypatch.setattr(_capi, "conv3x3", count("c3", real_c3))
    monkeypatch.setattr(_capi, "conv_down_unit_input", count("dn", real_dn))
    monkeypatch.setattr(_capi, "stem7", count("s7", real_s7))
    models = checkpoints.build_models([sd], "resnet50", 1000, "imagenet", device=cuda)
    fast = ScoringEngine(models, ScoreConfig(batch_size=128), cuda).score_shard(x, y, 0, n)
    # per launch chunk: the stem + 16 3x3 convs (13 of them stride 1 at 56 / 28 / 14 / 7 and
    # the 3 stride-2 ones: the padded-width tiles and heads), 32 Bottleneck 1x1s + 4 projections; 13 of the conv1s take the
    # previous unit's output fused (every unit input on a 56 / 28 / 14 map but the first,
    # which follows the stem's max-pool; the 7x7 maps keep the separate pass)
    # (padded: the stem on dd_stem7_forward, no implicit GEMM left)
    n_chunks = calls["s7"] if padded else calls["gemm"] // 17
    assert n_chunks > 0 and calls["gemm"] == (0 if padded else 17 * n_chunks)
    assert calls["s7"] == (n_chunks if padded else 0)
    assert calls["c3"] == (13 if padded else 0) * n_chunks
    assert calls["dn"] == (3 if padded else 0) * n_chunks
    assert calls["c1"] + calls["c1u"] == 36 * n_chunks and calls["c1u"] == 13 * n_chunks
    models = checkpoints.build_models([sd], "resnet50", 1000, "imagenet", device=cuda)
    ref = ScoringEngine(models, ScoreConfig(batch_size=128, fast_convs=False, fast_el2n=False),
                        cuda).score_shard(x, y, 0, n)
    got = fast["el2n"].cpu().numpy()
    np.testing.assert_allclose(got, ref["el2n"].cpu().numpy(), rtol=RTOL)
    # and directly against the CPU oracle (reference models/resnet.py:35-63 Bottleneck, the
    # ImageNet stem restated in oracle/resnet_fn.py) on the same pinned partition: batch 128
    # and the ragged 2-row second group, each with its own train-mode BN statistics
    want = o_pipe.el2n_scores(sd, images, labels, batch_size=128, stem="imagenet")
    np.testing.assert_allclose(got, want, rtol=RTOL)
    _record("imagenet_stem_hand_kernels_vs_oracle" + ("" if padded else "_gemm_only"),
            {"n130": {"max_rel": float(np.max(np.abs(got / want - 1))),
                      "miopen_max_rel": float(np.max(np.abs(ref["el2n"].cpu().numpy() / want
                                                            - 1)))}})


def test_sparse_loader_dropin_matches_reference(cuda, monkeypatch, tmp_path):
    """The reference entry point, reference semantics (net(input) in train mode), unshuffled
    loader: kept indices equal the reference's (outside the tie band), index file written."""
    d, images, labels, sds = _case(GOLDEN[0])
    n = int(d["n"])
    monkeypatch.setenv("DD_SYNTHETIC_N", str(n))
    monkeypatch.setenv("DD_SYNTHETIC_SEED", str(int(d["data_seed"])))
    from data_diet_distributed_amd.resnet import ResNet18
    net = ResNet18().to(cuda)
    net.load_state_dict(sds[0])  # train mode, as train.py:59-63
    ds = MyDataset(ArrayImageDataset(images, labels))
    loader = torch.utils.data.DataLoader(ds, batch_size=128, shuffle=False)
    out_loader, samples, idx = sparse_loader(loader, n, net, cuda, 0.5, 125, 0,
                                             dataset="synthetic-cifar10",
                                             subset_index_path=str(tmp_path / "keep"),
                                             return_indices=True)
    assert samples == 512 and len(out_loader.dataset) == 512
    assert sparse_loader.last_path == "fast"  # MyDataset over raw arrays, train-mode ResNet18
    # the fast path's keep-set is the exact one (16 ulps, as the engine's) without re-scoring
    assert len(_outside_band(d["ckpt0_scores"], np.array(idx), d["ckpt0_kept_0.5"], samples,
                             _ulp_band(d["ckpt0_scores"], samples))) == 0
    assert sparse_loader.last_refine is None
    saved = np.load(tmp_path / "keep.npy")
    assert saved.tolist() == idx
    i0, img0, y0 = out_loader.dataset[0]
    assert i0 == idx[0] and y0 == labels[idx[0]]


def test_sparse_loader_shuffled_ties_follow_visit_order(cuda):
    """With a shuffled loader the reference keeps ties in visit order; so do we."""
    images, labels = synthetic.make_images(300, 10, seed=1)
    net = torch.nn.Sequential(torch.nn.Flatten(), torch.nn.Linear(3 * 32 * 32, 10)).to(cuda)
    torch.nn.init.zeros_(net[1].weight)
    torch.nn.init.zeros_(net[1].bias)  # every score identical -> all ties
    ds = MyDataset(ArrayImageDataset(images, labels))
    g = torch.Generator().manual_seed(0)
    loader = torch.utils.data.DataLoader(ds, batch_size=64, shuffle=True, generator=g)
    visit = [int(i) for (idx, _, _) in torch.utils.data.DataLoader(
        ds, batch_size=64, shuffle=True, generator=torch.Generator().manual_seed(0)) for i in idx]
    from data_diet_distributed_amd.get_scores_and_prune import (el2n_scores_from_loader,
                                                                select_keep_indices)
    s, v = el2n_scores_from_loader(loader, net, cuda)
    kept = select_keep_indices(s, v, 100).cpu().tolist()
    assert kept == visit[:100]


def test_fused_grand_path_equals_autograd_tape_path(cuda):
    """The hand-scheduled GraNd fwd/bwd (fused epilogues) == the autograd tape path."""
    images, labels = synthetic.make_images(100, 10, seed=31)
    sd = synthetic.make_checkpoint("resnet18", 10, seed=6)["net"]
    img, lab = torch.from_numpy(images).to(cuda), torch.from_numpy(labels).to(cuda)
    out = {}
    for fused in (True, False):
        eng = ScoringEngine(checkpoints.build_models([sd], device=cuda),
                            ScoreConfig(methods=("grand",), select_by="grand", grand_batch=64,
                                        fused_grand=fused), cuda)
        out[fused] = eng.score_shard(img, lab, 0, 100)["grand"].cpu().numpy()
    # The tape path's MIOpen stride-2 convs are not run-to-run deterministic, and example 10 has
    # a ReLU pre-activation within fp32 rounding of zero. Its tape score takes one of two values
    # from run to run, 3487.957 (the fused path's and the float64 oracle's side of the gate) or
    # 3494.676 (+1.9e-3; tools/grand_repeat.py, profiles/r05_s7/grand_tape_nondeterminism.txt).
    # So the tape path is held to the float64 oracle at RTOL on every example except those
    # with a gate within GATE_REL whose score is the flipped-gate oracle's (named, recorded);
    # the fused path is held to the float64 oracle on every example, no exemption.
    ref = o_pipe.grand_scores(sd, images, labels, batch_size=50, dtype=F64)
    np.testing.assert_allclose(out[True], ref, rtol=RTOL)
    exempt = _gate_exemptions(out[False], ref, lambda near: o_pipe.grand_scores(
        sd, images, labels, batch_size=50, dtype=F64, flip_rel=GATE_REL, near_gates=near),
        "fused_vs_tape_grand_gate_exemptions")
    rel = np.abs(out[True] / out[False] - 1)
    keep = np.setdiff1d(np.arange(rel.size), exempt)
    assert np.all(rel[keep] <= 2 * RTOL), (rel[keep].max(), keep[rel[keep].argmax()])


def _gate_exemptions(got, ref, flipped_oracle, record_name):
    """Indices of `got` (a MIOpen-path GraNd vector) exempt from RTOL against the float64
    oracle `ref`: each has a ReLU gate within GATE_REL of zero and matches the oracle with
    those gates flipped (`flipped_oracle(near_gates_out) -> scores`) to RTOL.  Every other
    index must be within RTOL of `ref` (asserted here); the exemptions are recorded."""
    err = np.abs(got / ref - 1)
    if not (err > RTOL).any():
        return np.zeros(0, dtype=np.int64)
    near = np.zeros(got.size, dtype=np.int64)
    flip = flipped_oracle(near)
    err_flip = np.abs(got / flip - 1)
    bad = np.nonzero(err > RTOL)[0]
    exempt = bad[(near[bad] > 0) & (err_flip[bad] <= RTOL)]
    _record(record_name, {"exempt": {
        "rows": exempt.tolist(), "err_vs_float64": err[exempt].tolist(),
        "err_vs_flipped_gates": err_flip[exempt].tolist(),
        "gates_within_gate_rel": near[exempt].tolist(), "gate_rel": GATE_REL}})
    left = np.setdiff1d(bad, exempt)
    assert left.size == 0, {"rows": left.tolist(), "err": err[left].tolist(),
                            "err_flipped": err_flip[left].tolist(), "near": near[left].tolist()}
    return exempt


def test_engine_grand_all_params_matches_oracle(cuda):
    """grand_params = all (every BN gamma / beta too) vs the float64 hook oracle pinned to
    torch.func per-sample gradients over all parameters; the BN part (s_all^2 - s_cl^2) is
    checked on its own against the oracle's BN terms."""
    images, labels = synthetic.make_images(64, 10, seed=17)
    sd = synthetic.make_checkpoint("resnet18", 10, seed=8)["net"]
    ref_all = o_pipe.grand_scores(sd, images, labels, batch_size=32, params="all", dtype=F64)
    ref_cl = o_pipe.grand_scores(sd, images, labels, batch_size=32, dtype=F64)
    img, lab = torch.from_numpy(images).to(cuda), torch.from_numpy(labels).to(cuda)
    got = {}
    for gp in ("all", "conv_linear"):
        eng = ScoringEngine(checkpoints.build_models([sd], device=cuda),
                            ScoreConfig(methods=("grand",), select_by="grand", grand_batch=64,
                                        grand_params=gp), cuda)
        got[gp] = eng.score_shard(img, lab, 0, 64)["grand"].cpu().numpy().astype(np.float64)
    np.testing.assert_allclose(got["all"], ref_all, rtol=RTOL)
    bn_got = got["all"] ** 2 - got["conv_linear"] ** 2
    bn_ref = ref_all ** 2 - ref_cl ** 2
    np.testing.assert_allclose(bn_got, bn_ref, rtol=0.05, atol=1e-3 * ref_cl.max() ** 2 * 1e-2)


def test_engine_resnet50_cifar100_config4_parity(cuda):
    """BASELINE config 4 model (ResNet-50, CIFAR-100) on the hand-written kernels: the EL2N
    grouped train-BN forward (1x1 convs on dd_conv1x1_forward, stride-2 3x3 on
    dd_down_forward) at N = 512 (four pinned batches) vs the CPU oracle, and the fused
    Bottleneck GraNd schedule vs the float64 oracle; keep-sets equal outside the tie band."""
    n = 512
    images, labels = synthetic.make_images(n, 100, seed=41)
    sd = synthetic.make_checkpoint("resnet50", 100, seed=5)["net"]
    models = checkpoints.build_models([sd], "resnet50", 100, device=cuda)
    eng = ScoringEngine(models, ScoreConfig(methods=("el2n", "grand"), grand_batch=128), cuda)
    img, lab = torch.from_numpy(images).to(cuda), torch.from_numpy(labels).to(cuda)
    full, kept, k = eng.run(img, lab, 0.5)
    el2n_ref = o_pipe.el2n_scores(sd, images, labels, batch_size=128)
    got = full["el2n"].cpu().numpy()
    # The north star's 1e-3 on the hand kernels: the EL2N forward runs on fp16 operand halves
    # (~2^-22 relative per product).  On bf16 halves (~2^-17) ResNet-50's 53 convs had carried
    # the rounding to 1.0005e-3 on one row of these 512 (profiles/r04_parity/
    # diag_r50_layers.json); tools/emulate_split.py puts fp16 halves at 3.3e-5 on the CPU.
    np.testing.assert_allclose(got, el2n_ref, rtol=RTOL)
    _record("r50_c100_config4_el2n", {"split": {"max_rel": float(np.max(np.abs(got / el2n_ref
                                                                             - 1)))}})
    assert len(_outside_band(el2n_ref, kept.cpu().numpy(), o_el2n.stable_topk(el2n_ref, k), k,
                             KEEP_BAND)) == 0
    from data_diet_distributed_amd.score import SCORE_PRECISIONS
    eng32 = ScoringEngine(checkpoints.build_models([sd], "resnet50", 100, device=cuda),
                          ScoreConfig(methods=("el2n",), **SCORE_PRECISIONS["fp32"]), cuda)
    got32 = eng32.score_shard(img, lab, 0, n)["el2n"].cpu().numpy()
    np.testing.assert_allclose(got32, el2n_ref, rtol=RTOL)
    m = 96
    grand_ref = o_pipe.grand_scores(sd, images[:m], labels[:m], batch_size=48, dtype=F64)
    np.testing.assert_allclose(full["grand"].cpu().numpy()[:m], grand_ref, rtol=RTOL)


def test_fused_bottleneck_grand_equals_autograd(cuda):
    """The hand-scheduled Bottleneck GraNd (1x1 / stride-2 kernels, up2-scattered projection
    backward) == the autograd tape path on MIOpen, every example."""
    images, labels = synthetic.make_images(64, 100, seed=33)
    sd = synthetic.make_checkpoint("resnet50", 100, seed=7)["net"]
    img, lab = torch.from_numpy(images).to(cuda), torch.from_numpy(labels).to(cuda)
    out = {}
    for fused in (True, False):
        eng = ScoringEngine(checkpoints.build_models([sd], "resnet50", 100, device=cuda),
                            ScoreConfig(methods=("grand",), select_by="grand", grand_batch=64,
                                        fused_grand=fused), cuda)
        out[fused] = eng.score_shard(img, lab, 0, 64)["grand"].cpu().numpy()
    np.testing.assert_allclose(out[True], out[False], rtol=RTOL)


def test_sparse_loader_fast_path_shuffled_ties_follow_visit_order(cuda):
    """Fast path, shuffled loader, every score tied (zero classifier): the kept indices are
    the first `samples` of the loader's visit order, exactly as the reference's stable sort
    of its visit-ordered list gives."""
    from data_diet_distributed_amd.resnet import ResNet18
    images, labels = synthetic.make_images(300, 10, seed=1)
    net = ResNet18().to(cuda)
    torch.nn.init.zeros_(net.linear.weight)
    torch.nn.init.zeros_(net.linear.bias)
    ds = MyDataset(ArrayImageDataset(images, labels))
    loader = torch.utils.data.DataLoader(ds, batch_size=128, shuffle=True,
                                         generator=torch.Generator().manual_seed(0))
    visit = [int(i) for (idx, _, _) in torch.utils.data.DataLoader(
        ds, batch_size=128, shuffle=True, generator=torch.Generator().manual_seed(0)) for i in idx]
    _, samples, kept = sparse_loader(loader, 300, net, cuda, 0.5, 64, 0, return_indices=True)
    assert sparse_loader.last_path == "fast" and samples == 150
    assert kept == visit[:150]


# ---- GraNd at the benched configuration ------------------------------------------------------
def test_grand_at_bench_config_matches_float64_oracle(cuda):
    """The bench's exact ScoreConfig (EL2N + GraNd, grand_batch = el2n_chunk = 1024,
    pegrad_method auto, split-bf16) at K = 2 on N = 3032: three 1024-row chunks (chunk_plan
    keeps G = 1024 here, as at N = 50 000), the last one ragged (984 valid rows), so every
    persistent kernel (direct3x3p over 4096 layer-2 tiles = 16 rounds of 256 workgroups, the
    conv3x3 / r2 tiles' next-tile prefetch, the GraNd epilogues' bias / ReLU / fragment-mask
    writes and reads on later tiles) runs its multi-round form.  Eval BN makes every
    example independent, so GraNd on 128 rows spread over all three chunks (every tile round)
    is an exact check against the float64 oracle; EL2N is checked on all rows."""
    n = 3 * 1024 - 40
    images, labels = synthetic.make_images(n, 10, seed=51)
    sds = [synthetic.make_checkpoint("resnet18", 10, seed=s)["net"] for s in (11, 12)]
    cfg = ScoreConfig(methods=("el2n", "grand"), select_by="el2n", batch_size=128,
                      grand_batch=1024, el2n_chunk=1024, pegrad_method="auto")
    from data_diet_distributed_amd.scoring import chunk_plan
    plan, G = chunk_plan(0, n, 128, 1024)
    assert G == 1024 and len(plan) == 3 and plan[-1][1] - plan[-1][0] == 984
    eng = ScoringEngine(checkpoints.build_models(sds, device=cuda), cfg, cuda)
    img, lab = torch.from_numpy(images).to(cuda), torch.from_numpy(labels).to(cuda)
    full, kept, k = eng.run(img, lab, 0.5)
    rows = np.unique(np.concatenate([np.arange(5, n, 24), [0, 1023, 1024, 2047, 2048, n - 1]]))
    assert rows.size >= 128
    ref = np.zeros(rows.size, np.float64)
    for sd in sds:
        ref += o_pipe.grand_scores(sd, images[rows], labels[rows], batch_size=64, dtype=F64)
    ref /= 2
    got = full["grand"].cpu().numpy()[rows]
    # GraNd vs float64 at the north star's 1e-3.  Measured on these 133 rows (profiles/
    # r05_s3/keepset_swaps.json): 9.9e-5 with the GraNd forward on fp16 halves (its weights
    # scaled by a power of two), 8.8e-4 with it on bf16 halves (round 4), 4.2e-5 on the
    # plain-fp32 path
    # the same rows on the plain-fp32 GraNd path (MIOpen convs with folded BN, autograd to the
    # conv outputs, fp32-MFMA norms): if it shows the same worst rows and error, the deviation
    # is the fp32-vs-float64 ReLU flip, not the split-bf16 arithmetic (recorded side by side)
    eng32 = ScoringEngine(checkpoints.build_models(sds, device=cuda),
                          ScoreConfig(methods=("grand",), select_by="grand", grand_batch=1024,
                                      pegrad_precision="fp32", fast_convs=False,
                                      fused_grand=False, refine=False), cuda)
    idx = torch.from_numpy(rows).to(cuda)
    got32 = eng32.score_shard(img[idx].contiguous(), lab[idx].contiguous(), 0,
                              rows.size)["grand"].cpu().numpy()
    err = np.abs(got / ref - 1)
    err32 = np.abs(got32 / ref - 1)
    worst = np.argsort(err)[::-1][:4]
    _record("grand_bench_config_vs_float64", {
        "split": {"max_rel_err": float(err.max()), "worst_rows": rows[worst].tolist(),
                       "worst_errs": err[worst].tolist()},
        "fp32_path": {"max_rel_err": float(err32.max()),
                      "worst_rows": rows[np.argsort(err32)[::-1][:4]].tolist(),
                      "errs_on_split_worst_rows": err32[worst].tolist()},
        "rows": int(rows.size)})
    np.testing.assert_allclose(got, ref, rtol=RTOL)
    # (the plain-fp32 path runs every conv on MIOpen, which is not run-to-run deterministic: as in
    # test_fused_grand_path_equals_autograd_tape_path, a row with a ReLU gate within GATE_REL of
    # zero is exempt when its score is the flipped-gate float64 oracle's)

    def flipped(near):
        acc = np.zeros(rows.size, np.float64)
        for sd in sds:
            nk = np.zeros(rows.size, dtype=np.int64)
            acc += o_pipe.grand_scores(sd, images[rows], labels[rows], batch_size=64, dtype=F64,
                                       flip_rel=GATE_REL, near_gates=nk)
            near += nk
        return acc / 2
    _gate_exemptions(got32, ref, flipped, "grand_bench_config_fp32_path_gate_exemptions")
    el2n_ref = sum(o_pipe.el2n_scores(sd, images, labels, batch_size=128) for sd in sds) / 2
    np.testing.assert_allclose(full["el2n"].cpu().numpy(), el2n_ref, rtol=SCORE_REL)
    assert len(_outside_band(el2n_ref, kept.cpu().numpy(), o_el2n.stable_topk(el2n_ref, k), k,
                             KEEP_BAND)) == 0


def test_grand_scores_independent_of_chunk_and_world(cuda):
    """GraNd chunk size follows the shard length (chunk_plan), so it changes with the world
    size; the fused schedule's kernels make each example's score independent of it (chunk
    1024 vs 256 vs 4-rank shards), the classifier included (dd_linear_forward reduces each
    row alone; a library GEMM picked its kernel per batch size and moved the last ulp of the
    logits, which saturated-softmax examples turn into their whole ~1e-20 norm): bitwise."""
    n = 1000
    images, labels = synthetic.make_images(n, 10, seed=52)
    sd = synthetic.make_checkpoint("resnet18", 10, seed=13)["net"]
    img, lab = torch.from_numpy(images).to(cuda), torch.from_numpy(labels).to(cuda)
    out = {}
    for G in (1024, 256):
        eng = ScoringEngine(checkpoints.build_models([sd], device=cuda),
                            ScoreConfig(methods=("grand",), select_by="grand", grand_batch=G),
                            cuda)
        out[G] = eng.score_shard(img, lab, 0, n)["grand"].cpu()
        if G == 1024:
            out["w4"] = torch.cat([eng.score_shard(img, lab, *shard_bounds(n, 128, 4, r))["grand"]
                                   .cpu() for r in range(4)])
    for key in (256, "w4"):
        assert torch.equal(out[key], out[1024]), key


def test_rccl_world1_gather_branch(cuda):
    """The RCCL branch of gather_scores (all_gather_into_tensor, scoring.gather_scores) runs:
    a child process initialises a world-1 "nccl" group before any other GPU call (as a
    launched rank does), runs ScoringEngine.run with EL2N + GraNd through it, and matches the
    group-less run bit for bit (tests/helpers/rank_child.py nccl_engine)."""
    import subprocess
    import sys
    from data_diet_distributed_amd import launch
    child = os.path.join(os.path.dirname(os.path.abspath(__file__)), "helpers", "rank_child.py")
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", LOCAL_WORLD_SIZE="1",
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(launch.free_port()),
               HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, child, "nccl_engine"], env=env, capture_output=True,
                       text=True, timeout=300)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")]
    assert r.returncode == 0 and lines, r.stdout[-2000:] + r.stderr[-2000:]
    res = json.loads(lines[-1][7:])
    assert res["backend"] == "nccl" and res["calls"] == 2


# ---- more than one rank on the GPU box -------------------------------------------------------
def test_two_ranks_engine_equals_world1_bitwise(cuda, tmp_path):
    """The real multi-rank job: launch_ranks starts two rank processes (no GPU call before),
    both on cuda:0 (the one-GPU box; RCCL refuses two ranks on a device, so the gather runs
    over gloo through host memory), each holding ONLY its batch-aligned shard and running
    ScoringEngine.run(n_total=N) with EL2N + GraNd at the bench's chunk sizes.  The gathered
    scores and the keep-set equal the single-process world-1 run bit for bit: every
    hand-written kernel computes an example from its own rows (or its own BN group) in a fixed
    order, and the classifier is dd_linear_forward, so nothing depends on the shard size."""
    from data_diet_distributed_amd import launch
    ENGINE_SHARDS_SEED = 71  # tests/helpers/rank_child.py
    n = 2 * 1024 + 3 * 128 + 40  # shards [0, 1280), [1280, 2472): chunk plans differ per rank
    child = os.path.join(os.path.dirname(os.path.abspath(__file__)), "helpers", "rank_child.py")
    out = str(tmp_path / "w2.npz")
    rc = launch.launch_ranks(2, [child, "engine_shards", out, str(n)])
    assert rc == 0
    w2 = np.load(out)
    assert int(w2["world"]) == 2 and str(w2["backend"]) == "gloo"
    assert w2["shard"].tolist() == list(shard_bounds(n, 128, 2, 0))
    images, labels = synthetic.make_images(n, 10, seed=ENGINE_SHARDS_SEED)
    sds = [synthetic.make_checkpoint("resnet18", 10, seed=s)["net"] for s in (14, 15)]
    models = checkpoints.build_models(sds, device=cuda)
    img, lab = torch.from_numpy(images).to(cuda), torch.from_numpy(labels).to(cuda)
    eng = ScoringEngine(models, ScoreConfig(methods=("el2n", "grand"), refine=False), cuda)
    full, kept, k = eng.run(img, lab, 0.5)
    for m in ("el2n", "grand"):
        got, want = w2[m], full[m].cpu().numpy()
        assert np.array_equal(got, want), (m, float(np.max(np.abs(got / want - 1))))
    assert int(w2["k"]) == k and np.array_equal(w2["kept"], kept.cpu().numpy())
    # with the near-threshold fp32 re-scoring forced on: the same keep-set, up to ties within
    # EXACT_ULPS of the threshold (its MIOpen convs are not bitwise reproducible)
    eng_r = ScoringEngine(models, ScoreConfig(methods=("el2n", "grand"), refine=True), cuda)
    full_r, kept_r, _ = eng_r.run(img, lab, 0.5)
    s = full_r["el2n"].cpu().numpy()
    assert len(_outside_band(s, w2["kept_refined"], kept_r.cpu().numpy(), k,
                             _ulp_band(s, k))) == 0


def test_bench_two_ranks_share_device_prints_one_line(cuda):
    """bench.py --gpus 2 past its launcher: two self-launched ranks (shared cuda:0, gloo
    gather), per-rank shard generation, n_total scoring, the MAX-reduced timing and exactly
    one JSON line from rank 0 reporting world size 2."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2",
                        "--share-device", "--n", "2472", "--ckpts", "2", "--steps", "1",
                        "--warmup", "1"], env=env, cwd=root, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["ranks"]["world_size"] == 2 and d["ranks"]["backend"] == "gloo"
    assert d["value"] > 0 and d["config"]["kept"] == 1236 and d["cpu_baseline"] is None
    assert d["config"]["shard_examples_rank0"] == 1280


def test_lanes_are_bitwise_equal_to_one_stream(cuda):
    """ScoreConfig.lanes = 2 / 3 deals the launch chunks of every pass round-robin to that many
    HIP streams, issued interleaved: every chunk is computed exactly as on one stream and every
    example belongs to one lane, so the scores are bit-identical to lanes = 1 (EL2N + GraNd,
    K = 2, five chunks of 640 with a ragged tail)."""
    n = 5 * 640 - 70
    images, labels = synthetic.make_images(n, 10, seed=57)
    sds = [synthetic.make_checkpoint("resnet18", 10, seed=s)["net"] for s in (16, 17)]
    img, lab = torch.from_numpy(images).to(cuda), torch.from_numpy(labels).to(cuda)
    out = {}
    for lanes in (1, 2, 3):
        eng = ScoringEngine(checkpoints.build_models(sds, device=cuda),
                            ScoreConfig(methods=("el2n", "grand"), el2n_chunk=640,
                                        grand_batch=640, lanes=lanes), cuda)
        out[lanes] = {m: v.cpu() for m, v in eng.score_shard(img, lab, 0, n).items()}
    for lanes in (2, 3):
        for m in ("el2n", "grand"):
            assert torch.equal(out[lanes][m], out[1][m]), (lanes, m)


@pytest.mark.parametrize("path", [p for p in GOLDEN if "n50000" in p], ids=os.path.basename)
@pytest.mark.parametrize("general,refine", [(False, "auto"), (False, True), (True, "auto")],
                         ids=["fast", "fast_refined", "general"])
def test_sparse_loader_full_size_keep_set_is_exact(cuda, general, refine, path):
    """The reference's own entry point at the headline size (N = 50 000 golden, the reference's
    outputs), unshuffled loader, sparsity 0.5 / 0.7 / 0.9: the kept set equals the reference's
    except for indices within EXACT_ULPS (16) fp32 ulps of the threshold.  The fast path as it
    ships (forward on fp16 halves, no re-scoring: refine "auto"), the same with the visit-batch
    fp32 refinement forced on (round 4's bf16 halves swapped 2 at 0.5 without it), and the
    general path (net(input) on MIOpen fp32) are checked the same way.  Two goldens: the
    random-init checkpoint (thresholds among EL2N ~1.27) and the trained-regime one (a
    classifier fitted to the set, reference train.py:61-64 scores a trained ckpt_19: median
    EL2N 0.033, thresholds at 0.011 / 0.033 / 0.097 / 0.36 for sparsity 0.3 / 0.5 / 0.7 / 0.9,
    among softmax-saturated scores)."""
    d, images, labels, sds = _case(path)
    n = int(d["n"])
    want = d["ckpt0_scores"]
    from data_diet_distributed_amd.resnet import ResNet18
    ds = MyDataset(ArrayImageDataset(images, labels))
    records = {}
    sps = sorted(float(k.split("_kept_")[1]) for k in d if k.startswith("ckpt0_kept_"))
    for sp in sps:
        net = ResNet18().to(cuda)
        net.load_state_dict(sds[0])  # train mode, as train.py:59-63
        loader = torch.utils.data.DataLoader(ds, batch_size=128, shuffle=False)
        _, samples, idx = sparse_loader(loader, n, net, cuda, sp, 128, 0, return_indices=True,
                                        fast=not general, refine=refine)
        assert sparse_loader.last_path == ("general" if general else "fast")
        ref_kept = d[f"ckpt0_kept_{sp}"]
        assert samples == o_el2n.keep_count(n, sp) == ref_kept.size
        kept = np.array(idx)
        rec = _swap_record(want, want, kept, ref_kept, samples)
        rec["refine"] = sparse_loader.last_refine
        rec["band_ulps"], rec["band_rel"] = EXACT_ULPS, _ulp_band(want, samples)
        records[sp] = rec
        assert len(_outside_band(want, kept, ref_kept, samples,
                                 _ulp_band(want, samples))) == 0, rec
        if not general and refine is True:
            assert sparse_loader.last_refine["converged"], rec
        else:
            assert sparse_loader.last_refine is None
    name = "general" if general else ("fast_refined" if refine is True else "fast")
    _record(f"sparse_loader_{os.path.basename(path)[:-4]}_{name}", records)


def test_short_tail_plan_equals_even_plan_bitwise(cuda):
    """chunk_plan's full chunks + a short tail (the default) and the round-4 even plan (equal
    chunks, the tail padded to the buffer) give bitwise equal EL2N and GraNd scores on a
    W = 2 shard-like length (every pinned batch is its own BN group; GraNd rows are
    independent): the launch plan changes only speed."""
    n = 2 * 1024 + 3 * 128 + 40  # two full chunks, a 3-batch tail, a ragged last batch
    images, labels = synthetic.make_images(n, 10, seed=61)
    sd = synthetic.make_checkpoint("resnet18", 10, seed=21)["net"]
    img, lab = torch.from_numpy(images).to(cuda), torch.from_numpy(labels).to(cuda)
    out = {}
    for even in (False, True):
        eng = ScoringEngine(checkpoints.build_models([sd], device=cuda),
                            ScoreConfig(methods=("el2n", "grand"), even_chunks=even), cuda)
        out[even] = eng.score_shard(img, lab, 0, n)
    for m in ("el2n", "grand"):
        assert torch.equal(out[False][m], out[True][m]), m


def test_refine_auto_skips_fp32_rescoring_for_el2n_and_keeps_it_for_grand(cuda, monkeypatch):
    """ScoreConfig.refine = "auto" (the default): the EL2N-selected job (fp16-halves forward,
    fp32-grade) never reaches the plain-fp32 re-scoring (no MIOpen on the default path; the
    re-scoring entry point is made to fail here), while a GraNd-selected job (bf16-halves
    backward) does re-score near its threshold."""
    from data_diet_distributed_amd import scoring
    n = 1024 + 128 * 3
    images, labels = synthetic.make_images(n, 10, seed=83)
    sds = [synthetic.make_checkpoint("resnet18", 10, seed=s)["net"] for s in (31, 32)]
    img, lab = torch.from_numpy(images).to(cuda), torch.from_numpy(labels).to(cuda)
    real = scoring.ScoringEngine._rescore_fp32
    calls = []

    def guard(self, method, *a, **k):
        calls.append(method)
        if method == "el2n":
            raise AssertionError("EL2N fp32 re-scoring under refine='auto'")
        return real(self, method, *a, **k)
    monkeypatch.setattr(scoring.ScoringEngine, "_rescore_fp32", guard)
    eng = ScoringEngine(checkpoints.build_models(sds, device=cuda),
                        ScoreConfig(methods=("el2n", "grand"), grand_batch=512), cuda)
    assert eng.cfg.refine == "auto"
    eng.run(img, lab, 0.5)
    assert eng.last_refine is None and calls == []
    eng_g = ScoringEngine(checkpoints.build_models(sds, device=cuda),
                          ScoreConfig(methods=("el2n", "grand"), select_by="grand",
                                      grand_batch=512), cuda)
    eng_g.run(img, lab, 0.5)
    assert eng_g.last_refine is not None and eng_g.last_refine["method"] == "grand"
    assert calls and set(calls) == {"grand"}


def test_out_of_range_labels_raise_like_the_reference(cuda):
    """A label of 10 for a 10-class net: the reference's one_hot(target, num_classes=10) raises
    (get_scores_and_prune.py:17).  dd_el2n counts it on the device and the host raises
    LabelError (a ValueError and a RuntimeError) once per job: through the engine (EL2N and
    GraNd, run() and score_shard) and through sparse_loader on both paths."""
    n = 300
    images, labels = synthetic.make_images(n, 10, seed=5)
    labels[137] = 10
    sd = synthetic.make_checkpoint("resnet18", 10, seed=1)["net"]
    img, lab = torch.from_numpy(images).to(cuda), torch.from_numpy(labels).to(cuda)
    for methods in (("el2n",), ("grand",), ("el2n", "grand")):
        eng = ScoringEngine(checkpoints.build_models([sd], device=cuda),
                            ScoreConfig(methods=methods, select_by=methods[0], grand_batch=256),
                            cuda)
        with pytest.raises(_capi.LabelError, match="1 label"):
            eng.run(img, lab, 0.5)
        with pytest.raises(ValueError, match="outside"):
            eng.score_shard(img, lab, 0, n)
        eng.score_shard(img, lab, 0, 128)  # the bad row is not in [0, 128)
    from data_diet_distributed_amd.resnet import ResNet18
    ds = MyDataset(ArrayImageDataset(images, labels))
    for fast in (True, False):
        net = ResNet18().to(cuda)
        net.load_state_dict(sd)
        loader = torch.utils.data.DataLoader(ds, batch_size=128, shuffle=False)
        with pytest.raises(RuntimeError, match="outside"):
            sparse_loader(loader, n, net, cuda, 0.5, 128, 0, fast=fast)
        assert sparse_loader.last_path == ("fast" if fast else "general")


def test_bad_label_on_one_rank_raises_on_every_rank(cuda, tmp_path):
    """Two ranks (shared cuda:0, gloo), the bad label only in rank 1's shard: both ranks raise
    LabelError after the score all-gather (ScoringEngine._validate), neither waits in a
    collective for the other (a raise before the gather on one rank only hung the
    others until the process-group timeout)."""
    from data_diet_distributed_amd import launch
    child = os.path.join(os.path.dirname(os.path.abspath(__file__)), "helpers", "rank_child.py")
    out = str(tmp_path / "bad")
    rc = launch.launch_ranks(2, [child, "bad_label_shard", out, "600"])
    assert rc == 0
    for r in range(2):
        with open(f"{out}.{r}") as f:
            res = json.load(f)
        assert res["error"] == "LabelError" and res["seconds"] < 60, res


@pytest.mark.parametrize("methods", [("grand",), ("el2n", "grand")], ids=["grand", "both"])
def test_fp16_overflow_falls_back_to_bf16_halves(cuda, methods):
    """a checkpoint whose activations leave fp16's range (a BN gamma of 1e5 in
    layer1.0.bn1: the GraNd forward folds it into conv1, the EL2N forward applies it after the
    batch statistics) overflows the forward on fp16 operand halves.  The kernels' ReLUs
    propagate the resulting NaN (nmax), so the scores are non-finite instead of silently wrong:
    score_shard raises ValueError; run() re-scores the affected methods on bf16 halves on every
    rank (after the gather) and returns finite scores bitwise equal to an engine built on bf16
    packs, and records the fallback."""
    n = 256
    images, labels = synthetic.make_images(n, 10, seed=9)
    sd = synthetic.make_checkpoint("resnet18", 10, seed=4)["net"]
    sd["layer1.0.bn1.weight"] = sd["layer1.0.bn1.weight"] * 1e5
    img, lab = torch.from_numpy(images).to(cuda), torch.from_numpy(labels).to(cuda)
    cfg = dict(methods=methods, select_by="grand", grand_batch=256, refine=False)
    eng = ScoringEngine(checkpoints.build_models([sd], device=cuda), ScoreConfig(**cfg), cuda)
    with pytest.raises(ValueError, match="non-finite"):
        eng.score_shard(img, lab, 0, n)
    full, kept, k = eng.run(img, lab, 0.5)
    assert set(eng.fallback) == set(methods) and eng.grand_fallback
    assert eng.cfg.grand_operands == "bf16x3"
    assert eng.cfg.el2n_operands == ("bf16x3" if "el2n" in methods else "f16x3")
    ops = {"grand_operands": "bf16x3"}
    if "el2n" in methods:
        ops["el2n_operands"] = "bf16x3"
    ref = ScoringEngine(checkpoints.build_models([sd], device=cuda), ScoreConfig(**ops, **cfg),
                        cuda)
    full_r, kept_r, _ = ref.run(img, lab, 0.5)
    assert ref.fallback == {}
    for m in methods:
        got = full[m].cpu()
        assert bool(torch.isfinite(got).all()) and torch.equal(got, full_r[m].cpu()), m
    assert torch.equal(kept, kept_r)


def test_engine_empty_shard(cuda):
    """A rank whose batch-aligned shard is empty (W > number of batches: shard_bounds gives
    lo == hi) scores nothing and returns empty score vectors for every method, lanes or not."""
    images, labels = synthetic.make_images(256, 10, seed=3)
    sd = synthetic.make_checkpoint("resnet18", 10, seed=2)["net"]
    img, lab = torch.from_numpy(images).to(cuda), torch.from_numpy(labels).to(cuda)
    assert shard_bounds(200, 128, 3, 0) == (0, 0)
    for lanes in (1, 3):
        eng = ScoringEngine(checkpoints.build_models([sd], device=cuda),
                            ScoreConfig(methods=("el2n", "grand"), lanes=lanes), cuda)
        out = eng.score_shard(img, lab, 128, 128)
        assert set(out) == {"el2n", "grand"}
        assert all(v.numel() == 0 and v.device.type == "cuda" for v in out.values())
