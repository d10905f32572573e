"""Host-side logic on CPU: shard partition, config keys, checkpoint formats, index files,
data feed, model state_dict compatibility."""
import dataclasses
import os

import numpy as np
import pytest
import torch

from data_diet_distributed_amd import checkpoints, config, loader, subset_index, synthetic
from data_diet_distributed_amd.resnet import ResNet18, ResNet50, build
from data_diet_distributed_amd.scoring import ScoreConfig, all_shards, shard_bounds
from oracle import resnet_fn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("n", [0, 1, 127, 128, 2000, 50000, 1281167])
@pytest.mark.parametrize("W", [1, 2, 3, 4, 7, 8])
def test_shards_partition_batch_aligned(n, W):
    b = all_shards(n, 128, W)
    assert b[0][0] == 0 and b[-1][1] == n
    for (lo, hi), (lo2, _) in zip(b, b[1:]):
        assert hi == lo2
    for lo, hi in b:
        assert lo % 128 == 0 and lo <= hi
    sizes = [hi - lo for lo, hi in b]
    assert max(sizes) - min(sizes) <= 128 + (n % 128 == 0) * 0 + 128


def test_shard_bounds_validation():
    with pytest.raises(ValueError):
        shard_bounds(10, 4, 2, 2)


def test_score_config_validation():
    with pytest.raises(ValueError):
        ScoreConfig(methods=("foo",))
    with pytest.raises(ValueError):
        ScoreConfig(methods=("el2n",), select_by="grand")
    ScoreConfig(methods=("el2n", "grand"), select_by="grand")


def test_config_keeps_reference_keys():
    cfg = config.load_config(os.path.join(ROOT, "config.yaml"))
    for k in config.REFERENCE_KEYS:
        assert k in cfg
    assert cfg["batch_size"] == 128 and cfg["score_methods"] == ["el2n"]
    assert cfg["score_checkpoints"] == 1 and cfg["bn_mode"] == "batch"


def test_checkpoint_formats(tmp_path):
    sd = synthetic.make_checkpoint("resnet18", 10, seed=0)["net"]
    p1 = tmp_path / "ckpt_19.pth"
    torch.save({"net": sd, "acc": 1.0, "epoch": 19}, p1)  # trainer/trainer.py:64-71
    p2 = tmp_path / "ddp.pth"
    torch.save({"epoch": 3, "model_state_dict": {"module." + k: v for k, v in sd.items()},
                "optimizer_state_dict": {}, "accuracy": 1.0}, p2)  # ddp.py:116-123
    for p in (p1, p2):
        got = checkpoints.load_state_dict(str(p))
        assert list(got) == list(sd) and all(torch.equal(got[k], sd[k]) for k in sd)
    assert checkpoints.discover(str(tmp_path), 19, 1) == [str(p1)]
    for i in range(3):
        os.makedirs(tmp_path / f"seed{i}")
        torch.save({"net": sd}, tmp_path / f"seed{i}" / "ckpt_19.pth")
    assert len(checkpoints.discover(str(tmp_path), 19, 3)) == 3
    with pytest.raises(FileNotFoundError):
        checkpoints.discover(str(tmp_path), 19, 4)


def test_subset_index_roundtrip(tmp_path):
    idx = np.array([5, 3, 9, 0], dtype=np.int64)
    subset_index.write_subset_index(str(tmp_path / "k"), idx, {"n": 10, "sparsity": 0.6})
    got, meta = subset_index.read_subset_index(str(tmp_path / "k.npy"))
    assert got.tolist() == idx.tolist() and meta["k"] == 4 and meta["n"] == 10
    images, labels = synthetic.make_images(10, 10, seed=0)
    ds = loader.MyDataset(loader.ArrayImageDataset(images, labels))
    dl = subset_index.subset_loader(ds, str(tmp_path / "k"), batch_size=2, shuffle=False)
    seen = [int(i) for (ib, _, _) in dl for i in ib]
    assert seen == idx.tolist()
    with pytest.raises(ValueError):
        subset_index.subset_loader(loader.MyDataset(loader.ArrayImageDataset(images[:5], labels[:5])),
                                   str(tmp_path / "k"), 2)


def test_mydataset_and_transform_match_reference_arithmetic():
    images, labels = synthetic.make_images(4, 10, seed=0)
    ds = loader.MyDataset(loader.ArrayImageDataset(images, labels))
    i, x, y = ds[2]
    ref = torch.from_numpy(images[2]).float().div(255)
    ref = ref.sub(torch.tensor(loader.MEAN)[:, None, None]).div(torch.tensor(loader.STD)[:, None, None])
    assert i == 2 and y == labels[2] and torch.equal(x, ref)


def test_synthetic_is_deterministic():
    a = synthetic.make_images(100, 10, seed=3)
    b = synthetic.make_images(100, 10, seed=3)
    assert synthetic.digest(*a) == synthetic.digest(*b)
    c1 = synthetic.make_checkpoint("resnet18", 10, seed=1)["net"]
    c2 = synthetic.make_checkpoint("resnet18", 10, seed=1)["net"]
    assert synthetic.state_digest(c1) == synthetic.state_digest(c2)


@pytest.mark.parametrize("arch,nc,stem,hw", [("resnet18", 10, "cifar", 32),
                                             ("resnet50", 100, "cifar", 32),
                                             ("resnet34", 10, "cifar", 32),
                                             ("resnet50", 1000, "imagenet", 64)])
def test_product_model_equals_oracle_forward(arch, nc, stem, hw):
    """Product nn.Module forward == the oracle's functional restatement on the same weights,
    both BN modes; state_dict keys as the reference (122 for ResNet-18)."""
    sd = synthetic.make_checkpoint(arch, nc, seed=0, stem=stem)["net"]
    m = build(arch, nc, stem)
    m.load_state_dict(sd)
    x = torch.randn(4, 3, hw, hw, generator=torch.Generator().manual_seed(0))
    with torch.no_grad():
        for bn in ("batch", "running"):
            torch.testing.assert_close(m.run(x, bn=bn), resnet_fn.forward(sd, x, bn, stem),
                                       rtol=1e-5, atol=1e-5)
    if arch == "resnet18":
        assert len(ResNet18().state_dict()) == 122
    if arch == "resnet50" and stem == "cifar":
        assert len(ResNet50().state_dict()) == 320


def test_masked_batch_bn_equals_unpadded_batch():
    """A ragged batch padded to B rows with stats over the valid rows gives exactly the
    unpadded batch's outputs on those rows (EL2N tail batch, scoring.el2n_pass)."""
    sd = synthetic.make_checkpoint("resnet18", 10, seed=0)["net"]
    m = build("resnet18")
    m.load_state_dict(sd)
    x = torch.randn(80, 3, 32, 32, generator=torch.Generator().manual_seed(1))
    xp = torch.cat([x, torch.zeros(48, 3, 32, 32)])
    with torch.no_grad():
        want = m.run(x, bn="batch")
        got = m.run(xp, bn="batch", n_valid=80)[:80]
    torch.testing.assert_close(got, want, rtol=1e-5, atol=1e-5)


def test_folded_bn_equals_running_bn_and_tape_scales():
    sd = synthetic.make_checkpoint("resnet18", 10, seed=2)["net"]
    m = build("resnet18")
    m.load_state_dict(sd)
    m.fold_bn()
    x = torch.randn(4, 3, 32, 32, generator=torch.Generator().manual_seed(2))
    tape_f, tape_r = [], []
    with torch.no_grad():
        yf = m.run(x, bn="folded", tape=tape_f)
        yr = m.run(x, bn="running", tape=tape_r)
    torch.testing.assert_close(yf, yr, rtol=1e-4, atol=1e-4)
    assert len(tape_f) == len(tape_r) == 21  # 20 convs + linear (ResNet-18)
    for (cf, _, _, s), (cr, _, _, s_r) in zip(tape_f[:-1], tape_r[:-1]):
        assert cf is cr and s is not None and s_r is None and s.numel() == cf.out_channels


@pytest.mark.parametrize("lo,hi,gran,chunk", [(0, 50000, 128, 1024), (0, 6272, 128, 1024),
                                               (6272, 12416, 128, 1024), (0, 80, 128, 1024),
                                               (0, 1000, 64, 64), (128, 129, 128, 1024),
                                               (0, 0, 128, 1024), (0, 50000, 128, 100),
                                               (0, 24960, 128, 1024)])
@pytest.mark.parametrize("even", [False, True])
def test_chunk_plan_covers_balanced(lo, hi, gran, chunk, even):
    from data_diet_distributed_amd.scoring import chunk_plan, run_rows
    plan, rows = chunk_plan(lo, hi, gran, chunk, even)
    if hi == lo:
        assert plan == []
        return
    g = min(gran, chunk)
    assert plan[0][0] == lo and plan[-1][1] == hi
    assert all(a[1] == b[0] for a, b in zip(plan, plan[1:]))      # contiguous
    assert all((c1 - c0) == rows for c0, c1 in plan[:-1])          # equal except the tail
    assert 0 < plan[-1][1] - plan[-1][0] <= rows <= max(chunk, g)
    assert rows % g == 0 and all((c0 - lo) % g == 0 for c0, _ in plan)  # whole batches
    nb = -(-(hi - lo) // g)
    naive = -(-nb // max(1, chunk // g))
    if even:
        # at most 4 launches more than the naive fixed-size split, never more padded work
        assert naive <= len(plan) <= naive + 4
        naive_rows = -(-nb // naive)
        assert len(plan) * rows <= naive * naive_rows * g
    else:
        # full chunks (the whole set's launch size) and a tail run at whole granules only
        assert len(plan) == naive
        assert rows == min(max(g, chunk // g * g), run_rows(hi - lo, g))
        work = sum(run_rows(c1 - c0, g) for c0, c1 in plan)
        assert work == nb * g


def test_chunk_plan_shard_sizes():
    """W = 2 / 4 / 8 rank-0 shards of the 50k set: full 1024-row launches and one short tail
    (the even plan ran 896-row launches there: fewer tiles per persistent grid)."""
    from data_diet_distributed_amd.scoring import chunk_plan
    plan, rows = chunk_plan(0, 24960, 128, 1024)
    assert rows == 1024 and len(plan) == 25 and plan[-1] == (24576, 24960)
    plan, rows = chunk_plan(0, 12416, 128, 1024)
    assert rows == 1024 and len(plan) == 13 and plan[-1][1] - plan[-1][0] == 128
    plan, rows = chunk_plan(0, 49 * 128, 128, 1024, even=True)
    assert rows == 896 and len(plan) == 7
    plan, rows = chunk_plan(0, 12500, 128, 1024, even=True)
    assert rows == 896 and len(plan) == 14 and plan[-1][1] == 12500


def test_grand_params_all_refuses_zero_bn_gamma():
    """A zero BN gamma (zero-init residual BNs) would make dd_bn_pegrad_sqnorm divide 0/0:
    the engine refuses it by name."""
    from data_diet_distributed_amd.resnet import ResNet18
    from data_diet_distributed_amd.scoring import check_bn_gammas
    net = ResNet18()
    check_bn_gammas(net)  # default gamma = 1
    with torch.no_grad():
        net.layer2[0].bn2.weight[5] = 0.0
    with pytest.raises(ValueError, match=r"layer2\.0\.bn2\.weight is exactly 0 in channel\(s\) \[5\]"):
        check_bn_gammas(net)


def _fake_engine(monkeypatch, cfg, true_scores):
    """A ScoringEngine shell on the CPU for the refinement's host logic: the select is the
    oracle's stable sort, and the fp32 re-scoring returns the true scores of the rows asked."""
    from data_diet_distributed_amd import _capi
    from data_diet_distributed_amd import scoring
    from oracle import el2n as o_el2n

    def select_topk(keys, k, check_nan=True):
        idx = o_el2n.stable_topk(keys.numpy(), k)
        return (torch.from_numpy(np.asarray(idx, dtype=np.int64)),
                keys[int(idx[-1])].reshape(1).clone(), torch.zeros(1, dtype=torch.int32))
    monkeypatch.setattr(_capi, "select_topk", select_topk)
    monkeypatch.setattr(torch.cuda, "synchronize", lambda *a, **k: None)
    eng = scoring.ScoringEngine.__new__(scoring.ScoringEngine)
    eng.cfg, eng.device, eng.models, eng.last_refine = cfg, torch.device("cpu"), [None], None
    asked = []

    def rescore(method, images_u8, labels, rows, off, N):
        asked.extend(rows)
        return torch.cat([true_scores[r0:r1] for r0, r1 in rows])
    eng._rescore_fp32 = rescore
    return eng, asked


@pytest.mark.parametrize("method", ["el2n", "grand"])
def test_refine_makes_the_keep_set_exact(monkeypatch, method):
    """ScoringEngine._refine (ScoreConfig.refine): fast-path scores off by up to 2e-4 relative
    (with a few 10x outliers), the true ones known to the fake fp32 re-scoring.  The band
    widens until the expected number of examples left on the wrong side (from the differences
    seen on everything re-scored) is <= refine_tol, and the final keep-set equals the stable
    top-k of the true scores; EL2N re-scores whole pinned batches, GraNd single examples, and
    fewer rows than N."""
    from oracle import el2n as o_el2n
    rng = np.random.default_rng(0)
    N, B, k = 20000, 128, 10000
    true = torch.from_numpy(rng.uniform(0.5, 1.5, N).astype(np.float32))
    err = rng.uniform(-2e-4, 2e-4, N)
    err[rng.integers(0, N, 20)] *= 10
    split = (true.double() * torch.from_numpy(1 + err)).float()
    cfg = ScoreConfig(methods=("el2n", "grand"), select_by=method, batch_size=B,
                      refine_max_frac=0.5)
    eng, asked = _fake_engine(monkeypatch, cfg, true)
    full, kept = eng._refine({method: split}, k, None, None, 0, N, 0, N, None, True)
    # the keep-SET is exact (the order inside it follows the fast-path scores away from the
    # threshold, which no consumer reads: the Subset is shuffled by its loader)
    assert np.array_equal(np.sort(kept.numpy()), np.sort(o_el2n.stable_topk(true.numpy(), k)))
    info = eng.last_refine
    assert info["expected_wrong_side"] <= cfg.refine_tol and info["max_rel_diff"] > 0
    # (EL2N's batch granularity: each near row brings its whole batch; at this density the
    # 10x outliers take about a third of the rows, hence the raised budget)
    assert 0 < info["examples_rescored"] < N // 2, info
    if method == "el2n":
        assert all(r0 % B == 0 and (r1 - r0 == B or r1 == N) for r0, r1 in asked)
    else:
        assert all(r1 - r0 == 1 for r0, r1 in asked)
    # the split-bf16 keep-set alone is NOT exact here (that is what the refinement is for)
    assert not np.array_equal(np.sort(o_el2n.stable_topk(split.numpy(), k)),
                              np.sort(o_el2n.stable_topk(true.numpy(), k)))


def test_refine_is_skipped_where_the_path_is_already_fp32():
    from data_diet_distributed_amd import scoring
    eng = scoring.ScoringEngine.__new__(scoring.ScoringEngine)
    eng.cfg = ScoreConfig(methods=("el2n",), fast_convs=False)
    assert not eng._refines("el2n")
    eng.cfg = ScoreConfig(methods=("el2n",), refine=False)
    assert not eng._refines("el2n")
    # "auto": the default EL2N pass runs on fp16 halves (fp32-grade), no refinement; on bf16
    # halves, or forced, it refines; GraNd's backward is bf16 halves, so it refines
    eng.cfg = ScoreConfig(methods=("el2n",))
    assert eng.cfg.refine == "auto" and not eng._refines("el2n")
    eng.cfg = ScoreConfig(methods=("el2n",), el2n_operands="bf16x3")
    assert eng._refines("el2n")
    eng.cfg = ScoreConfig(methods=("el2n",), refine=True)
    assert eng._refines("el2n")
    eng.cfg = ScoreConfig(methods=("grand",), select_by="grand")
    assert eng._refines("grand")
    eng.cfg = ScoreConfig(methods=("grand",), select_by="grand", fast_convs=False,
                          pegrad_precision="fp32")
    assert not eng._refines("grand")
    with pytest.raises(ValueError):
        ScoreConfig(methods=("el2n",), refine="yes")


def test_refine_budget_cap(monkeypatch):
    """refine_max_frac bounds the fp32 re-scoring: with a 0.5 % budget on a fast path whose
    errors need more, the refinement stops after its first sample (512 rows) instead of
    spending the budget on a partial band, and last_refine says the tolerance was not met."""
    rng = np.random.default_rng(1)
    N, B, k = 20000, 128, 10000
    true = torch.from_numpy(rng.uniform(0.5, 1.5, N).astype(np.float32))
    split = (true.double() * torch.from_numpy(1 + rng.uniform(-1e-3, 1e-3, N))).float()
    cfg = ScoreConfig(methods=("el2n",), batch_size=B, refine_max_frac=0.005)
    eng, asked = _fake_engine(monkeypatch, cfg, true)
    eng._refine({"el2n": split}, k, None, None, 0, N, 0, N, None, True)
    info = eng.last_refine
    assert info["budget_capped"] and not info["converged"]
    assert info["examples_rescored"] <= 640 and info["expected_wrong_side"] > cfg.refine_tol
    assert sum(r1 - r0 for r0, r1 in asked) == info["examples_rescored"]
    # what the band would have needed is reported (whole batches, more than the budget)
    assert info["rows_needed"] > cfg.refine_max_frac * N and info["rows_needed"] % B == 0
    assert info["max_frac_needed"] == info["rows_needed"] / N


@pytest.mark.parametrize("method", ["el2n", "grand"])
def test_refine_first_sample_is_bounded_on_a_dense_set(monkeypatch, method):
    """The first sample is the units within refine_rel of the threshold, or those of the
    refine_min_sample (512) nearest rows where that band holds more: EL2N the batches of the
    4 nearest rows (4 x 128 rows), GraNd the 512 nearest examples.  A band narrower than
    that distance is used as is."""
    rng = np.random.default_rng(2)
    N, B, k = 1 << 20, 128, 1 << 19
    true = torch.from_numpy(rng.uniform(0.5, 1.5, N).astype(np.float32))
    cfg = ScoreConfig(methods=("el2n", "grand"), select_by=method, batch_size=B,
                      refine_max_iter=1, refine_rel=1e-3)
    eng, asked = _fake_engine(monkeypatch, cfg, true)
    eng._refine({method: true.clone()}, k, None, None, 0, N, 0, N, None, True)
    rows = sum(r1 - r0 for r0, r1 in asked)
    if method == "el2n":
        assert len(asked) == 4 and rows == 4 * B     # the batches of the 4 nearest rows
    else:
        assert rows == 512                            # the 512 nearest examples
    eng.cfg = dataclasses.replace(cfg, refine_rel=1e-9)
    asked.clear()
    eng._refine({method: true.clone()}, k, None, None, 0, N, 0, N, None, True)
    assert 0 < sum(r1 - r0 for r0, r1 in asked) <= B


def test_refine_estimate_is_fresh_when_iterations_run_out(monkeypatch):
    """refine_max_iter = 1: the one round re-scores its first sample and the loop ends. The
    reported expected_wrong_side / converged must describe the state AFTER that round (ADVICE
    r04: it was left at None / the previous round's value)."""
    rng = np.random.default_rng(3)
    N, B, k = 20000, 128, 10000
    true = torch.from_numpy(rng.uniform(0.5, 1.5, N).astype(np.float32))
    split = (true.double() * torch.from_numpy(1 + rng.uniform(-2e-4, 2e-4, N))).float()
    for iters in (1, 2):
        cfg = ScoreConfig(methods=("el2n",), batch_size=B, refine_max_iter=iters,
                          refine_max_frac=0.5)
        eng, asked = _fake_engine(monkeypatch, cfg, true)
        full, _ = eng._refine({"el2n": split}, k, None, None, 0, N, 0, N, None, True)
        info = eng.last_refine
        assert info["iterations"] == iters and info["examples_rescored"] > 0
        # recompute the estimate independently from the final state
        s = full["el2n"].double().numpy()
        thr = np.sort(s)[::-1][k - 1]
        done = np.zeros(N, bool)
        for r0, r1 in asked:
            done[r0:r1] = True
        err = np.sort(np.abs(split.double().numpy()[done] - s[done]) / thr)
        d = np.abs(s[~done] - thr) / thr
        want = float((1.0 - np.searchsorted(err, d, side="right") / err.size).sum())
        assert info["expected_wrong_side"] == pytest.approx(want, rel=1e-9, abs=1e-12)
        assert info["converged"] == (want <= cfg.refine_tol)


def test_refine_setting_is_normalised():
    """refine = 0 / 1 (an int from a CLI or env override) must mean False / True
    everywhere (the checks use identity); other values are rejected."""
    from data_diet_distributed_amd.scoring import ScoreConfig, normalize_refine
    assert ScoreConfig(refine=0).refine is False and ScoreConfig(refine=1).refine is True
    assert ScoreConfig(refine=np.int64(1)).refine is True
    assert ScoreConfig().refine == "auto" and normalize_refine(True) is True
    for bad in (2, "yes", None, 0.5, "Auto"):
        with pytest.raises(ValueError):
            ScoreConfig(refine=bad)
