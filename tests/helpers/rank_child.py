"""Child-process programs for the launcher / process-group tests (run as `python -m
tests.helpers.rank_child MODE` or by path).  Not collected by pytest.

  die_rank1  : rank 1 exits 3 at once; rank 0 blocks in gloo rendezvous (it would wait for
               the process-group timeout without the launcher's fail-fast)
  ok         : every rank joins a gloo group, barriers, exits 0
  nccl_engine: world-1 RCCL group initialised BEFORE any other GPU call, then the scoring
               engine's run() through gather_scores' all_gather_into_tensor branch; prints a
               JSON verdict (scores equal the group-less run bit for bit)
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
                        ScoreConfig(methods=("el2n", "grand"), grand_batch=256), dev)
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


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
