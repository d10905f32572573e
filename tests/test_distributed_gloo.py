"""Multi-rank path on CPU with gloo: shard -> all-gather -> global select == single process.

The GPU run uses the same code with backend "nccl" (RCCL over xGMI); here every rank scores
its batch-aligned shard with a deterministic stand-in score (a function of the global index,
so the gathered vector is known exactly), gathers with `gather_scores`, and selects with the
oracle's stable top-k.
"""
import os
import socket
import time

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from data_diet_distributed_amd.scoring import gather_scores, shard_bounds
from oracle import el2n as o_el2n


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _score(idx):
    # many exact ties on purpose
    return (np.sin(idx * 0.37) * 7).round(1).astype(np.float32)


def _worker(rank, world, port, n, batch, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = shard_bounds(n, batch, world, rank)
        local = torch.from_numpy(_score(np.arange(lo, hi)))
        full = gather_scores(local, n, batch)
        k = o_el2n.keep_count(n, 0.5)
        kept = o_el2n.stable_topk(full.numpy(), k)
        np.save(os.path.join(out_dir, f"r{rank}.npy"), np.concatenate([full.numpy(), kept]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 1000), (2, 128), (3, 2000), (4, 777)])
def test_gloo_gather_select_equals_single_process(tmp_path, world, n):
    mp.spawn(_worker, args=(world, _free_port(), n, 128, str(tmp_path)), nprocs=world, join=True)
    want_full = _score(np.arange(n))
    want_kept = o_el2n.stable_topk(want_full, o_el2n.keep_count(n, 0.5))
    outs = [np.load(tmp_path / f"r{r}.npy") for r in range(world)]
    for o in outs:
        assert np.array_equal(o[:n], want_full)
        assert np.array_equal(o[n:].astype(np.int64), want_kept)


def _job_worker(rank, world, port, n, out_dir):
    """One rank of the real orchestration (`scoring.sharded_job`, the body of
    ScoringEngine.run): builds ONLY its shard of the synthetic set, scores it with the CPU
    oracle in place of the HIP passes, gathers with gather_scores, selects globally."""
    from data_diet_distributed_amd import synthetic
    from data_diet_distributed_amd.scoring import sharded_job
    from oracle import pipeline as o_pipe
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sd = synthetic.make_checkpoint("resnet18", 10, seed=3)["net"]

        def score(lo, hi):
            img, lab = synthetic.make_images(n, 10, seed=5, lo=lo, hi=hi)
            return {"el2n": torch.from_numpy(o_pipe.el2n_scores(sd, img, lab, 128))}

        full, kept, k = sharded_job(
            score, n, 128, 0.5, "el2n",
            lambda keys, kk: torch.from_numpy(o_el2n.stable_topk(keys.numpy(), kk)),
            o_el2n.keep_count)
        np.save(os.path.join(out_dir, f"job{rank}.npy"),
                np.concatenate([full["el2n"].numpy(), kept.numpy().astype(np.float32), [k]]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 400), (3, 300)])
def test_gloo_sharded_job_equals_single_process(tmp_path, world, n):
    from data_diet_distributed_amd import synthetic
    from oracle import pipeline as o_pipe
    mp.spawn(_job_worker, args=(world, _free_port(), n, str(tmp_path)), nprocs=world, join=True)
    nt = torch.get_num_threads()
    torch.set_num_threads(1)
    try:
        img, lab = synthetic.make_images(n, 10, seed=5)
        sd = synthetic.make_checkpoint("resnet18", 10, seed=3)["net"]
        want = o_pipe.el2n_scores(sd, img, lab, 128)
    finally:
        torch.set_num_threads(nt)
    k = o_el2n.keep_count(n, 0.5)
    want_kept = o_el2n.stable_topk(want, k)
    for r in range(world):
        o = np.load(tmp_path / f"job{r}.npy")
        np.testing.assert_array_equal(o[:n], want)
        assert int(o[-1]) == k
        np.testing.assert_array_equal(o[n:n + k].astype(np.int64), want_kept)


def _validate_worker(rank, world, port, n, out_dir):
    """sharded_job's `validate` hook sees the GATHERED vectors, identical on every rank: a
    NaN scored on the last rank's shard only makes every rank raise (the engine's label /
    overflow checks sit there, ScoringEngine._validate), and nobody reaches the select."""
    from data_diet_distributed_amd.scoring import sharded_job
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    seen = []
    try:
        def score(lo, hi):
            s = torch.from_numpy(_score(np.arange(lo, hi)))
            if rank == world - 1:
                s[-1] = float("nan")
            return {"el2n": s}

        def validate(full):
            seen.append(full["el2n"].clone())
            if bool(torch.isnan(full["el2n"]).any()):
                raise ValueError("nan")
            return full

        def select(keys, kk):
            raise AssertionError("select reached")
        try:
            sharded_job(score, n, 128, 0.5, "el2n", select, o_el2n.keep_count,
                        validate=validate)
            res = "no raise"
        except ValueError:
            res = "raised"
        np.save(os.path.join(out_dir, f"v{rank}.npy"), seen[0].numpy())
        with open(os.path.join(out_dir, f"v{rank}.txt"), "w") as f:
            f.write(res)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 300), (3, 700)])
def test_gloo_validate_sees_gathered_vector_on_every_rank(tmp_path, world, n):
    mp.spawn(_validate_worker, args=(world, _free_port(), n, str(tmp_path)), nprocs=world,
             join=True)
    v0 = np.load(tmp_path / "v0.npy")
    assert v0.size == n and np.isnan(v0[-1]) and not np.isnan(v0[:-1]).any()
    for r in range(world):
        assert (tmp_path / f"v{r}.txt").read_text() == "raised"
        np.testing.assert_array_equal(np.load(tmp_path / f"v{r}.npy"), v0)


# ---- launcher fail-fast ----------------------------------------------------------------------
def _child():
    return os.path.join(os.path.dirname(os.path.abspath(__file__)), "helpers", "rank_child.py")


def test_launcher_stops_siblings_when_a_rank_dies():
    """Rank 1 exits 3 before joining; rank 0 would block in the gloo rendezvous for its
    600 s timeout.  launch_ranks returns 3 within seconds and leaves no rank running."""
    from data_diet_distributed_amd import launch
    t0 = time.monotonic()
    rc = launch.launch_ranks(2, [_child(), "die_rank1"], grace_s=5.0)
    assert rc == 3
    assert time.monotonic() - t0 < 60


def test_launcher_all_ranks_ok():
    from data_diet_distributed_amd import launch
    assert launch.launch_ranks(3, [_child(), "ok"]) == 0


def _refine_worker(rank, world, port, n, K, out_dir):
    """One rank of ScoringEngine._refine with the checkpoint-split re-scoring (W > 1): a
    CPU stand-in for the fp32 path whose per-checkpoint value is a function of the global
    row index decoded from the row's (gathered) image bytes, so a wrong gather shows."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from data_diet_distributed_amd import _capi, scoring
        from data_diet_distributed_amd.scoring import ScoreConfig
        B = 128
        lo, hi = shard_bounds(n, B, world, rank)
        rng = np.random.default_rng(0)
        true = rng.uniform(0.5, 1.5, n).astype(np.float32)
        err = rng.uniform(-2e-4, 2e-4, n)
        split = torch.from_numpy((true.astype(np.float64) * (1 + err)).astype(np.float32))
        gidx = np.arange(lo, hi, dtype=np.int64)
        img = torch.from_numpy(np.stack([gidx & 255, (gidx >> 8) & 255, (gidx >> 16) & 255],
                                        axis=1).astype(np.uint8))
        lab = torch.zeros(hi - lo, dtype=torch.int64)
        asked = []

        def rescore(method, images_u8, labels, rows, off, N, models=None, per_ckpt=False):
            models = list(range(K)) if models is None else models
            outs = []
            for r0, r1 in rows:
                im = images_u8[r0 - off:r1 - off].to(torch.int64)
                i = (im[:, 0] + 256 * im[:, 1] + 65536 * im[:, 2]).numpy()
                # checkpoint m: true * (1 + 0.01 (m - (K - 1) / 2)) plus an ulp-sized per-row
                # wobble, so the fp32 sum order shows in the result bits
                per = np.stack([true[i] * np.float32(1 + 0.01 * (m - (K - 1) / 2))
                                * np.float32(1 + 1e-7 * np.sin(i * (m + 1)))
                                for m in models]).astype(np.float32)
                if per_ckpt:
                    outs.append(per)
                else:
                    acc = np.zeros(r1 - r0, np.float32)
                    for v in per:  # checkpoint order (the kernel's accum += s_k)
                        acc += v
                    outs.append(acc / np.float32(K))
                asked.append((r0, r1, tuple(models)))
            return torch.from_numpy(np.concatenate(outs, axis=-1))

        _capi.select_topk = lambda keys, k, check_nan=True: (
            torch.from_numpy(np.asarray(o_el2n.stable_topk(keys.numpy(), k), dtype=np.int64)),
            keys[int(o_el2n.stable_topk(keys.numpy(), k)[-1])].reshape(1).clone(),
            torch.zeros(1, dtype=torch.int32))
        _capi.ensemble_finalize = lambda acc, K_, out: out.copy_(acc / np.float32(K_))
        torch.cuda.synchronize = lambda *a, **kw: None
        eng = scoring.ScoringEngine.__new__(scoring.ScoringEngine)
        eng.cfg = ScoreConfig(methods=("el2n",), batch_size=B, refine_max_frac=0.5)
        eng.device, eng.models, eng.last_refine = torch.device("cpu"), list(range(K)), None
        eng._rescore_fp32 = rescore
        if os.environ.get("DD_TEST_REFINE_GATHER_BYTES"):
            eng.refine_gather_bytes = int(os.environ["DD_TEST_REFINE_GATHER_BYTES"])
        k = o_el2n.keep_count(n, 0.5)
        full, kept = eng._refine({"el2n": split}, k, img, lab, lo, hi, lo, n, None, True)
        # every rank ran only its own checkpoints, on rows of every shard
        mine = {m for _, _, ms in asked for m in ms}
        assert mine == {m for m in range(K) if m % world == rank}, mine
        np.save(os.path.join(out_dir, f"k{rank}.npy"), kept.numpy())
        np.save(os.path.join(out_dir, f"s{rank}.npy"), full["el2n"].numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n,K", [(2, 20000, 4), (3, 9000, 2), (2, 9000, 5)])
def test_gloo_refine_checkpoint_split(tmp_path, world, n, K):
    """The W > 1 refinement re-scores near-threshold rows split by checkpoint (images
    all-gathered, per-checkpoint vectors all-reduced and accumulated in checkpoint order):
    every rank ends with the same scores, bitwise the one-rank refinement's, and a keep-set
    equal to the stable top-k of the true scores.  (K = 5 over 2 ranks: uneven checkpoint
    counts per rank.)"""
    one = tmp_path / "w1"
    one.mkdir()
    mp.spawn(_refine_worker, args=(1, _free_port(), n, K, str(one)), nprocs=1, join=True)
    mp.spawn(_refine_worker, args=(world, _free_port(), n, K, str(tmp_path)), nprocs=world,
             join=True)
    rng = np.random.default_rng(0)
    true = rng.uniform(0.5, 1.5, n).astype(np.float32)
    want = np.sort(o_el2n.stable_topk(true, o_el2n.keep_count(n, 0.5)))
    s0 = np.load(tmp_path / "s0.npy")
    assert np.array_equal(np.load(one / "s0.npy"), s0)  # bitwise world-size independent
    for r in range(world):
        assert np.array_equal(np.load(tmp_path / f"s{r}.npy"), s0)
        assert np.array_equal(np.sort(np.load(tmp_path / f"k{r}.npy")), want)


def test_gloo_refine_checkpoint_split_slices_the_gather(tmp_path, monkeypatch):
    """With a tiny refine_gather_bytes the rows go through many gathers (one pinned batch
    each) and the result is the same bitwise."""
    one = tmp_path / "w1"
    one.mkdir()
    mp.spawn(_refine_worker, args=(1, _free_port(), 9000, 3, str(one)), nprocs=1, join=True)
    os.environ["DD_TEST_REFINE_GATHER_BYTES"] = "64"
    try:
        mp.spawn(_refine_worker, args=(2, _free_port(), 9000, 3, str(tmp_path)), nprocs=2,
                 join=True)
    finally:
        del os.environ["DD_TEST_REFINE_GATHER_BYTES"]
    assert np.array_equal(np.load(one / "s0.npy"), np.load(tmp_path / "s0.npy"))
    assert np.array_equal(np.load(one / "k0.npy"), np.load(tmp_path / "k1.npy"))
