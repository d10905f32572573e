"""Child-process programs for the launcher / process-group tests (run as `python -m
tests.helpers.rank_child MODE` or by path).  Not collected by pytest.

  die_rank1  : rank 1 exits 3 at once; rank 0 blocks in gloo rendezvous (it would wait for
               the process-group timeout without the launcher's fail-fast)
  ok         : every rank joins a gloo group, barriers, exits 0
  nccl_engine: world-1 RCCL group initialised BEFORE any other GPU call, then the scoring
               engine's run() through gather_scores' all_gather_into_tensor branch; prints a
               JSON verdict (scores equal the group-less run bit for bit)
  engine_shards OUT N: every rank on cuda:0 in a gloo group (RCCL refuses two ranks on one
               device); each holds ONLY its batch-aligned shard of the N synthetic examples,
               runs ScoringEngine.run(n_total=N) (EL2N + GraNd, two checkpoints, the bench's
               chunk sizes), the scores are gathered through host memory and every rank
               selects; rank 0 writes the gathered scores and keep-set to OUT (.npz), every
               rank checks its keep-set equals rank 0's
  bad_label_shard OUT N: as engine_shards (one checkpoint, EL2N + GraNd), but one label of
               rank 1's shard is out of range; every rank must raise LabelError from run()
               (after the gather, ScoringEngine._validate) instead of leaving the others
               blocked in a collective; each rank writes {"error", "seconds"} to OUT.<rank>
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main(mode):
    from data_diet_distributed_amd import launch
    world, rank, local = launch.rank_env()
    if mode == "die_rank1":
        if rank == 1:
            sys.exit(3)
        launch.init_process_group("gloo", rank, world, timeout_s=600)
        import torch.distributed as dist
        dist.barrier()
        time.sleep(600)
        return 0
    if mode == "ok":
        launch.init_process_group("gloo", rank, world, timeout_s=60)
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()
        return 0
    if mode == "nccl_engine":
        return nccl_engine(local)
    if mode == "engine_shards":
        return engine_shards(rank, world, sys.argv[2], int(sys.argv[3]))
    if mode == "bad_label_shard":
        return bad_label_shard(rank, world, sys.argv[2], int(sys.argv[3]))
    raise SystemExit(f"unknown mode {mode}")


def nccl_engine(local):
    import torch
    import torch.distributed as dist
    from data_diet_distributed_amd import checkpoints, launch, synthetic
    from data_diet_distributed_amd.scoring import ScoreConfig, ScoringEngine
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    launch.init_process_group("nccl", 0, 1, dev, timeout_s=120)  # first GPU call of the process
    calls = {"all_gather_into_tensor": 0}
    real = dist.all_gather_into_tensor

    def counted(*a, **k):
        calls["all_gather_into_tensor"] += 1
        return real(*a, **k)
    dist.all_gather_into_tensor = counted
    n = 384 + 56
    images, labels = synthetic.make_images(n, 10, seed=61)
    sd = synthetic.make_checkpoint("resnet18", 10, seed=3)["net"]
    eng = ScoringEngine(checkpoints.build_models([sd], device=dev),
                        ScoreConfig(methods=("el2n", "grand"), grand_batch=256, refine=False), dev)
    img, lab = torch.from_numpy(images).to(dev), torch.from_numpy(labels).to(dev)
    full, kept, k = eng.run(img, lab, 0.5)
    torch.cuda.synchronize()
    backend = dist.get_backend()
    dist.destroy_process_group()
    full0, kept0, k0 = eng.run(img, lab, 0.5)
    res = {"backend": backend, "calls": calls["all_gather_into_tensor"],
           "el2n_equal": bool(torch.equal(full["el2n"], full0["el2n"])),
           "grand_equal": bool(torch.equal(full["grand"], full0["grand"])),
           "kept_equal": bool(torch.equal(kept, kept0)), "k": int(k)}
    print("RESULT " + json.dumps(res), flush=True)
    ok = (backend == "nccl" and res["calls"] == 2 and res["el2n_equal"] and res["grand_equal"]
          and res["kept_equal"])
    return 0 if ok else 1


ENGINE_SHARDS_SEED = 71


def engine_shards(rank, world, out, n):
    import numpy as np
    import torch
    import torch.distributed as dist
    from data_diet_distributed_amd import checkpoints, launch, synthetic
    from data_diet_distributed_amd.scoring import ScoreConfig, ScoringEngine, shard_bounds
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    launch.init_process_group("gloo", rank, world, timeout_s=300)
    lo, hi = shard_bounds(n, 128, world, rank)
    images, labels = synthetic.make_images(n, 10, seed=ENGINE_SHARDS_SEED, lo=lo, hi=hi)
    sds = [synthetic.make_checkpoint("resnet18", 10, seed=s)["net"] for s in (14, 15)]
    models = checkpoints.build_models(sds, device=dev)
    img, lab = torch.from_numpy(images).to(dev), torch.from_numpy(labels).to(dev)
    # the fast-path scores (bitwise comparable); then with the near-threshold fp32 re-scoring
    # forced on (its MIOpen convs are not bitwise reproducible between processes)
    eng = ScoringEngine(models, ScoreConfig(methods=("el2n", "grand"), refine=False), dev)
    full, kept, k = eng.run(img, lab, 0.5, n_total=n)
    kept = kept.cpu()
    eng_r = ScoringEngine(models, ScoreConfig(methods=("el2n", "grand"), refine=True), dev)
    kept_r = eng_r.run(img, lab, 0.5, n_total=n)[1].cpu()
    k0 = kept.clone()
    dist.broadcast(k0, 0)
    same = bool(torch.equal(kept, k0))
    if rank == 0:
        np.savez(out, el2n=full["el2n"].cpu().numpy(), grand=full["grand"].cpu().numpy(),
                 kept=kept.numpy(), kept_refined=kept_r.numpy(), k=k, world=dist.get_world_size(), backend=dist.get_backend(),
                 shard=np.array([lo, hi]))
    dist.barrier()
    dist.destroy_process_group()
    print(f"RANK {rank} shard [{lo}, {hi}) keep-set equal to rank 0's: {same}", flush=True)
    return 0 if same else 1


def bad_label_shard(rank, world, out, n):
    import torch
    import torch.distributed as dist
    from data_diet_distributed_amd import _capi, checkpoints, launch, synthetic
    from data_diet_distributed_amd.scoring import ScoreConfig, ScoringEngine, shard_bounds
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    launch.init_process_group("gloo", rank, world, timeout_s=120)
    lo, hi = shard_bounds(n, 128, world, rank)
    images, labels = synthetic.make_images(n, 10, seed=ENGINE_SHARDS_SEED, lo=lo, hi=hi)
    if rank == 1:
        labels[(hi - lo) // 2] = 10
    sd = synthetic.make_checkpoint("resnet18", 10, seed=14)["net"]
    eng = ScoringEngine(checkpoints.build_models([sd], device=dev),
                        ScoreConfig(methods=("el2n", "grand"), grand_batch=256, refine=False), dev)
    img, lab = torch.from_numpy(images).to(dev), torch.from_numpy(labels).to(dev)
    t = time.perf_counter()
    err = None
    try:
        eng.run(img, lab, 0.5, n_total=n)
    except _capi.LabelError:
        err = "LabelError"
    except Exception as ex:  # noqa: BLE001 - recorded for the test's message
        err = f"{type(ex).__name__}: {ex}"
    res = {"error": err, "seconds": time.perf_counter() - t}
    with open(f"{out}.{rank}", "w") as f:
        json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()
    print(f"RANK {rank} {res}", flush=True)
    return 0 if err == "LabelError" else 1


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
