"""Keep-set selection (dd_select_topk) vs the reference's stable descending sort.

Reference get_scores_and_prune.py:22-24; the oracle restates it in oracle/el2n.py.  Integer
/index work: results must be bit-exact (same indices, same order).
"""
import numpy as np
import pytest
import torch

from data_diet_distributed_amd import _capi
from oracle import el2n as o_el2n

pytestmark = pytest.mark.gpu


def _run(cuda, keys, k):
    t = torch.from_numpy(np.asarray(keys, dtype=np.float32)).to(cuda)
    idx, thr, nan = _capi.select_topk(t, k)
    return idx.cpu().numpy(), float(thr.item()) if k else None


@pytest.mark.parametrize("n,k", [(1, 1), (10, 3), (1000, 500), (50000, 25000), (50000, 4999),
                                 (50000, 0), (50000, 50000), (4097, 1), (300000, 123457)])
def test_select_random(cuda, n, k):
    keys = np.random.default_rng(n + k).random(n, dtype=np.float32)
    idx, thr = _run(cuda, keys, k)
    ref = o_el2n.stable_topk(keys, k)
    assert np.array_equal(idx, ref)
    if k:
        assert thr == keys[ref[-1]]


@pytest.mark.parametrize("dist", ["lognormal", "signed", "narrow", "pow8"])
def test_select_key_ranges(cuda, dist):
    # the survivors' key range sets the LSD digit width (ceil(R / 3) bits, R = 21..32): keys
    # within one top bin (7-bit digits), over a few octaves (8), many octaves and both signs
    # (10-11)
    rng = np.random.default_rng(7)
    n = 200003
    if dist == "lognormal":
        keys = rng.lognormal(0.0, 12.0, n).astype(np.float32)
    elif dist == "signed":
        keys = (rng.standard_normal(n) * 10.0 ** rng.integers(-30, 30, n)).astype(np.float32)
    elif dist == "narrow":
        keys = (0.95 + 1e-4 * rng.random(n)).astype(np.float32)
    else:
        keys = (rng.random(n) ** 8).astype(np.float32)
    for k in (1, n // 3, n // 2, n - 1, n):
        idx, thr = _run(cuda, keys, k)
        ref = o_el2n.stable_topk(keys, k)
        assert np.array_equal(idx, ref), (dist, k)
        assert thr == keys[ref[-1]]


def test_select_ties_keep_visit_order(cuda):
    # heavy ties: 7 distinct values over 10k keys, including +0.0 and -0.0 (equal in Python)
    rng = np.random.default_rng(0)
    vals = np.array([0.5, 0.25, 0.0, -0.0, 1.0, 3.0, -2.0], dtype=np.float32)
    keys = vals[rng.integers(0, len(vals), 10000)]
    for k in (0, 1, 17, 5000, 9999, 10000):
        idx, _ = _run(cuda, keys, k)
        assert np.array_equal(idx, o_el2n.stable_topk(keys, k)), k
    # the literal Python statement of the reference on a small case
    small = keys[:300]
    idx, _ = _run(cuda, small, 150)
    assert list(idx) == o_el2n.stable_topk_python(range(300), small, 150)


def test_select_all_equal(cuda):
    keys = np.full(5000, 0.7, np.float32)
    idx, thr = _run(cuda, keys, 1234)
    assert np.array_equal(idx, np.arange(1234)) and thr == np.float32(0.7)


def test_select_special_values(cuda):
    keys = np.array([np.inf, -np.inf, 1e-45, -1e-45, 3.4e38, -3.4e38, 0.0, 1.0, 1.0, 2.0],
                    dtype=np.float32)
    for k in range(len(keys) + 1):
        idx, _ = _run(cuda, keys, k)
        assert np.array_equal(idx, o_el2n.stable_topk(keys, k))


def test_select_nan_rejected(cuda):
    keys = torch.tensor([1.0, float("nan"), 0.5], device=cuda)
    with pytest.raises(ValueError, match="NaN"):
        _capi.select_topk(keys, 2)
    # unchecked: NaN ranks last
    idx, _, nan = _capi.select_topk(keys, 3, check_nan=False)
    assert int(nan.item()) == 1 and idx.cpu().tolist() == [0, 2, 1]


def test_select_empty(cuda):
    idx, _, _ = _capi.select_topk(torch.empty(0, device=cuda), 0)
    assert idx.numel() == 0


def test_select_large_properties(cuda):
    # size-independent properties at 2^24 keys: exact count, sorted descending, ties ascending,
    # everything kept >= everything dropped
    n = 1 << 24
    g = torch.Generator(device=cuda).manual_seed(0)
    keys = torch.rand(n, device=cuda, generator=g)
    keys = torch.round(keys * 4096) / 4096  # force ties
    k = n // 2
    idx, thr, _ = _capi.select_topk(keys, k)
    assert idx.numel() == k
    kept = keys[idx]
    assert bool((kept[:-1] >= kept[1:]).all())
    same = kept[:-1] == kept[1:]
    assert bool((idx[:-1][same] < idx[1:][same]).all())
    mask = torch.ones(n, dtype=torch.bool, device=cuda)
    mask[idx] = False
    assert int(mask.sum()) == n - k
    assert float(keys[mask].max()) <= float(kept.min()) == float(thr.item())
    # dropped ties at the threshold have larger indices than the kept ones
    t = float(thr.item())
    eq_kept = idx[kept == t]
    eq_drop = torch.nonzero(mask & (keys == t)).flatten()
    if eq_drop.numel():
        assert int(eq_kept.max()) < int(eq_drop.min())


def test_keep_count_matches_reference():
    # get_scores_and_prune.py:22 float truncation: 0.9 -> 4999, 0.8 -> 9999 at N=50k
    for sp, want in [(0.9, 4999), (0.8, 9999), (0.5, 25000), (0.7, 15000), (0.0, 50000),
                     (1.0, 0)]:
        assert o_el2n.keep_count(50000, sp) == want
        assert _capi.keep_count(50000, sp) == want


def test_select_ballot_match_rank_path(tmp_path):
    # the fallback rank (ballot digit matching, used when the lane-order probe of the LDS
    # atomics fails) on the same cases, in a child process started with DD_SELECT_RANK=match
    import os
    import subprocess
    import sys
    code = (
        "import numpy as np, torch\n"
        "from data_diet_distributed_amd import _capi\n"
        "from oracle import el2n as o\n"
        "rng = np.random.default_rng(3)\n"
        "cases = [rng.random(50000, dtype=np.float32),\n"
        "         np.array([0.5, 0.25, 0.0, -0.0, 1.0], np.float32)[rng.integers(0, 5, 10000)],\n"
        "         (rng.standard_normal(70001) * 10.0 ** rng.integers(-20, 20, 70001)).astype(np.float32)]\n"
        "for keys in cases:\n"
        "    for k in (1, len(keys) // 2, len(keys)):\n"
        "        idx, _, _ = _capi.select_topk(torch.from_numpy(keys).cuda(), k)\n"
        "        assert np.array_equal(idx.cpu().numpy(), o.stable_topk(keys, k)), k\n"
        "print('match path ok')\n")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, DD_SELECT_RANK="match", PYTHONPATH=root)
    r = subprocess.run([sys.executable, "-c", code], env=env, cwd=root, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0 and "match path ok" in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("n", [1281167, (1 << 20) + 4099])
def test_select_sizes_with_empty_blocks(cuda, n):
    # sizes whose 4096-entry tiles leave hist_top / split blocks empty (313 tiles over 256
    # blocks: blocks 157..255 hold nothing) with n % 4 != 0: an empty block must not count the
    # last n % 4 keys again (it did, inflating the histogram and the NaN count).
    # The ImageNet-shape keep-set (config 5) is this size.
    rng = np.random.default_rng(n)
    keys = rng.random(n, dtype=np.float32)
    for k in (1, n // 10, n // 2, n - 1):
        idx, thr = _run(cuda, keys, k)
        ref = o_el2n.stable_topk(keys, k)
        assert np.array_equal(idx, ref), k
        assert thr == keys[ref[-1]]
    # a NaN among the tail keys is counted exactly once
    keys[-1] = np.nan
    idx, _, nan = _capi.select_topk(torch.from_numpy(keys).to(cuda), n // 2, check_nan=False)
    assert int(nan.item()) == 1
    assert np.array_equal(idx.cpu().numpy(), o_el2n.stable_topk(keys[:-1], n // 2))


def test_select_first_call_is_graph_capturable(tmp_path):
    # include/dd_capi.h: no entry point allocates or synchronises, so the FIRST dd_select_topk
    # of a fresh process can be captured into a HIP graph (the once-per-process lane-order
    # probe of the LDS atomics is enqueued on the call's stream, so the graph holds and replays
    # it; its verdict lives in a device global); replays are bit-exact
    import os
    import subprocess
    import sys
    code = (
        "import numpy as np, torch\n"
        "from data_diet_distributed_amd import _capi\n"
        "from oracle import el2n as o\n"
        "n, k = 300001, 123456\n"
        "keys = np.random.default_rng(5).random(n, dtype=np.float32)\n"
        "t = torch.from_numpy(keys).cuda()\n"
        "ws = torch.empty(_capi.select_workspace_bytes(n), dtype=torch.uint8, device='cuda')\n"
        "idx = torch.empty(k, dtype=torch.int64, device='cuda')\n"
        "torch.cuda.synchronize()\n"
        "ref = o.stable_topk(keys, k)\n"
        "s = torch.cuda.Stream()\n"
        "g = torch.cuda.CUDAGraph()\n"
        "with torch.cuda.graph(g, stream=s):\n"
        "    _capi.select_topk(t, k, idx_out=idx, workspace=ws, check_nan=False)\n"
        "for r in range(3):\n"
        "    idx.fill_(-1)\n"
        "    g.replay()\n"
        "    torch.cuda.synchronize()\n"
        "    got = idx.cpu().numpy()\n"
        "    assert np.array_equal(got, ref), (r, int((got != ref).sum()), int((got == -1).sum()))\n"
        "# the same workspace reused by eager calls (after the graph's)\n"
        "for r in range(2):\n"
        "    _capi.select_topk(t, k, idx_out=idx, workspace=ws, check_nan=False)\n"
        "    torch.cuda.synchronize()\n"
        "    assert np.array_equal(idx.cpu().numpy(), ref), ('eager', r)\n"
        "t.copy_(torch.from_numpy(keys[::-1].copy()))\n"
        "g.replay()\n"
        "torch.cuda.synchronize()\n"
        "assert np.array_equal(idx.cpu().numpy(), o.stable_topk(keys[::-1].copy(), k))\n"
        "print('graph ok')\n")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root)
    r = subprocess.run([sys.executable, "-c", code], env=env, cwd=root, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0 and "graph ok" in r.stdout, r.stdout + r.stderr
