"""Multi-rank path on CPU with gloo: shard -> all-gather -> global select == single process.

The GPU run uses the same code with backend "nccl" (RCCL over xGMI); here every rank scores
its batch-aligned shard with a deterministic stand-in score (a function of the global index,
so the gathered vector is known exactly), gathers with `gather_scores`, and selects with the
oracle's stable top-k.
"""
import os
import socket

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
