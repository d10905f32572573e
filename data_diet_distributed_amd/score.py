"""Config-driven scoring entry: the K-checkpoint engine run from config.yaml.

    python -m data_diet_distributed_amd.score --config config.yaml [--sparsity P]
        [--out PATH] [--gpus N]

Reference anchor: the config -> scoring flow of train.py:36-64 and ddp.py:54-77
(load_config, get_dataloader, ResNet18 + checkpoint_path/ckpt_19.pth, sparse_loader,
`--sparsity` from the command line).  The reference keys keep their meaning (`dataset`,
`batch_size` = the EL2N batch partition, `checkpoint_path`); the engine keys select the
rest (config.DEFAULTS):

  score_methods      el2n and/or grand               select_by     ranking score
  score_checkpoints  K: checkpoint_path/seed{k}/ckpt_{score_epoch}.pth (K = 1: ckpt_E.pth)
  bn_mode            EL2N BatchNorm: batch|train (reference) or running|eval
  pegrad_method      auto | direct | ghost             grand_batch   GraNd chunk
  score_gpus         ranks (one per GPU; self-launched here, or run under torchrun)
  subset_index_path  where the keep-set (.npy) + metadata (.json) + scores (.scores.npz) go
  arch, num_classes, stem                             the backbone of the checkpoints

Each rank loads or generates ONLY its batch-aligned shard of the training set into HBM
(`synthetic-imagenet`: generated on device by dd_synth_images_u8), scores it against all K
checkpoints, and the engine all-gathers the score vectors (RCCL) before the global select.
Rank 0 writes the artefact; its metadata records the checkpoints' sha256 digests, the
architecture, methods and BN mode, so a later sparse-training job can check what it reads.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

from . import config as config_mod
from . import launch

BN_MODES = {"batch": "batch", "train": "batch", "running": "running", "eval": "running"}


def _methods(cfg):
    m = cfg.get("score_methods", ["el2n"])
    return (m,) if isinstance(m, str) else tuple(m)


def dataset_size(cfg) -> int:
    """Examples in a synthetic dataset: `synthetic_n`, else $DD_SYNTHETIC_N, else the size of
    the real set it stands for (1,281,167 ImageNet / 50,000 CIFAR, like loader._synthetic).
    None for a real dataset (known after loading)."""
    ds = cfg["dataset"]
    if not ds.startswith("synthetic"):
        return None
    raw = cfg.get("synthetic_n")
    if raw is None:
        raw = os.environ.get("DD_SYNTHETIC_N")
    n = int(raw) if raw is not None else (1281167 if ds == "synthetic-imagenet" else 50000)
    if n <= 0:
        raise ValueError(f"{ds}: dataset size must be positive (got {n})")
    return n


def load_shard(cfg, world, rank, device):
    """(n_total, images uint8 [hi-lo, 3, H, W], labels int64 [hi-lo]) of this rank's shard,
    on `device`."""
    import torch

    from . import loader, synthetic
    from .scoring import shard_bounds
    ds = cfg["dataset"]
    B = int(cfg["batch_size"])
    seed = int(cfg.get("synthetic_seed", os.environ.get("DD_SYNTHETIC_SEED", "0")))
    if ds == "synthetic-imagenet":
        n = dataset_size(cfg)
        lo, hi = shard_bounds(n, B, world, rank)
        img, lab = synthetic.device_shard(seed, lo, hi, int(cfg["num_classes"]), hw=224,
                                          device=device)
        return n, img, lab
    if ds in ("synthetic-cifar10", "synthetic-cifar100"):
        n = dataset_size(cfg)
        lo, hi = shard_bounds(n, B, world, rank)
        ncls = 10 if ds == "synthetic-cifar10" else 100
        img, lab = synthetic.make_images(n, ncls, seed=seed, lo=lo, hi=hi)
    else:
        train, _ = loader.load_data(ds, root=cfg.get("data_root", "./"))
        n = len(train)
        lo, hi = shard_bounds(n, B, world, rank)
        img, lab = train.images[lo:hi], train.labels[lo:hi]
    return (n, torch.from_numpy(np.ascontiguousarray(img)).to(device),
            torch.from_numpy(np.ascontiguousarray(lab, dtype=np.int64)).to(device))


# config.yaml `score_precision`:
#   split          split MFMA (the default): the EL2N and GraNd forwards on fp16 halves
#                  (fp32-grade scores), the GraNd backward on bf16 halves; scores near the
#                  threshold re-computed in plain fp32 where the ranking pass carries bf16-halves
#                  arithmetic (ScoreConfig.refine "auto": select_by grand)
#   split_refined  the same, the near-threshold fp32 re-scoring forced on for either method
#   split_fast     the split scores alone, never re-scored
#   bf16x3         every split conv on bf16 halves (the round-4 arithmetic, ~2e-4 relative),
#                  near-threshold fp32 re-scoring on
#   bf16x3_fast    the bf16-halves scores alone
#   fp32           the plain fp32 path throughout (MIOpen convs, autograd, fp32-MFMA norms)
SCORE_PRECISIONS = {
    "split": {},
    "split_refined": {"refine": True},
    "split_fast": {"refine": False},
    "bf16x3": {"el2n_operands": "bf16x3", "grand_operands": "bf16x3", "refine": True},
    "bf16x3_fast": {"el2n_operands": "bf16x3", "grand_operands": "bf16x3", "refine": False},
    "fp32": {"fast_convs": False, "fast_el2n": False, "fused_grand": False,
             "pegrad_precision": "fp32", "refine": False},
}


def engine_config(cfg):
    from .scoring import ScoreConfig
    methods = _methods(cfg)
    bn = str(cfg.get("bn_mode", "batch"))
    if bn not in BN_MODES:
        raise ValueError(f"bn_mode must be one of {sorted(BN_MODES)} (got {bn!r})")
    prec = str(cfg.get("score_precision", "split"))
    if prec not in SCORE_PRECISIONS:
        raise ValueError(f"score_precision must be one of {sorted(SCORE_PRECISIONS)} "
                         f"(got {prec!r})")
    return ScoreConfig(methods=methods, select_by=cfg.get("select_by", methods[0]),
                       batch_size=int(cfg["batch_size"]), el2n_bn=BN_MODES[bn],
                       grand_batch=int(cfg.get("grand_batch", 1024)),
                       pegrad_method=cfg.get("pegrad_method", "auto"),
                       lanes=int(cfg.get("score_lanes", 3)),
                       refine_max_frac=float(cfg.get("refine_max_frac", 0.08)),
                       **SCORE_PRECISIONS[prec])


def score_from_config(cfg: dict, sparsity: float, out_path=None, log=print):
    """Run the job as this rank (call under launch_ranks/torchrun for >1 rank).  Returns
    (kept indices np.int64, {method: np.float32 scores}, meta) on rank 0, None elsewhere."""
    import torch
    import torch.distributed as dist

    from . import checkpoints, synthetic
    from .scoring import ScoringEngine
    from .subset_index import write_subset_index

    world, rank, local = launch.rank_env()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if launch.under_launcher() and not dist.is_initialized():
        launch.init_process_group("nccl", rank, world, dev)
    try:
        ecfg = engine_config(cfg)
        arch, ncls = cfg.get("arch", "resnet18"), int(cfg.get("num_classes", 10))
        stem = cfg.get("stem") or ("imagenet" if cfg["dataset"] == "synthetic-imagenet"
                                   else "cifar")
        K = int(cfg.get("score_checkpoints", 1))
        paths = checkpoints.discover(cfg["checkpoint_path"], int(cfg.get("score_epoch", 19)), K)
        sds = [checkpoints.load_state_dict(p) for p in paths]
        digests = [synthetic.state_digest(sd) for sd in sds]
        models = checkpoints.build_models(sds, arch, ncls, stem, device=dev)
        n, img, lab = load_shard(cfg, world, rank, dev)
        eng = ScoringEngine(models, ecfg, dev)
        t0 = time.perf_counter()
        full, kept, k = eng.run(img, lab, sparsity, n_total=n)
        torch.cuda.synchronize()
        secs = time.perf_counter() - t0
        if rank != 0:
            return None
        kept_np = kept.cpu().numpy().astype(np.int64)
        scores = {m: v.cpu().numpy() for m, v in full.items()}
        meta = {"n": int(n), "k": int(k), "sparsity": float(sparsity),
                "score_methods": list(ecfg.methods), "select_by": ecfg.select_by, "K": K,
                "checkpoints": [os.path.abspath(p) for p in paths],
                "checkpoint_digests": digests, "arch": arch, "num_classes": ncls,
                "stem": stem, "dataset": cfg["dataset"], "batch_size": ecfg.batch_size,
                "bn_mode": ecfg.el2n_bn, "pegrad_method": ecfg.pegrad_method,
                "grand_batch": ecfg.grand_batch, "world_size": world,
                "order": "score descending, ties by ascending index (pinned batch partition)",
                "seconds": secs, "examples_per_s": n / secs if secs > 0 else None}
        out_path = out_path or cfg.get("subset_index_path")
        if out_path:
            path = write_subset_index(out_path, kept_np, meta)
            stem_p = path[:-4]
            np.savez(stem_p + ".scores.npz", **scores)
            log(f"kept {k} of {n} examples -> {path} ({secs:.2f} s, {world} rank(s))")
        return kept_np, scores, meta
    finally:
        if launch.under_launcher() and dist.is_initialized():
            dist.destroy_process_group()


def parse(argv=None):
    ap = argparse.ArgumentParser(description="Data Diet scoring from config.yaml (MI355X)")
    ap.add_argument("--config", default="config.yaml")
    ap.add_argument("--sparsity", type=float, default=None,
                    help="fraction pruned (the reference's --sparsity; default: config key)")
    ap.add_argument("--out", default=None, help="index artefact path (default: "
                                                 "subset_index_path of the config)")
    ap.add_argument("--gpus", type=int, default=None, help="ranks (default: score_gpus)")
    return ap.parse_args(argv)


def main(argv=None):
    args = parse(argv)
    cfg = config_mod.load_config(args.config)
    gpus = args.gpus or int(cfg.get("score_gpus", 1))
    if gpus > 1 and not launch.under_launcher():
        rest = list(sys.argv[1:] if argv is None else argv)
        return launch.launch_ranks(gpus, ["-m", "data_diet_distributed_amd.score"] + rest)
    sparsity = args.sparsity if args.sparsity is not None else float(cfg["sparsity"])
    if not (args.out or cfg.get("subset_index_path")):
        raise SystemExit("no output: set subset_index_path in the config or pass --out")
    score_from_config(cfg, sparsity, args.out)
    return 0


if __name__ == "__main__":
    sys.exit(main())
