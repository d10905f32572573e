"""Benchmark: examples scored/sec for ResNet-18 / CIFAR-10 EL2N + GraNd over K=10 checkpoints
(BASELINE.json metric, configs[1]), 50% keep-set, on 1..8 MI355X (one process per GPU).

    python bench.py [--gpus N] [--steps K] [--warmup W]        (starts N ranks itself)
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

With --gpus N > 1 and no torchrun environment, this process is only a launcher: it starts N
rank processes (python bench.py ... with RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set) BEFORE
touching the GPU, waits for them and exits with the worst exit code (reference ddp.py:179-181
spawns its own ranks the same way).  `--spawn` forces that path at N = 1.

One step = the whole job on the fixed dataset: every rank scores its batch-aligned shard of
the N=50,000 synthetic examples against all K checkpoints (EL2N with batch-stat BN over the
pinned 128-batch partition; GraNd with eval BN), RCCL all-gathers the score vectors, and
selects the global keep-set (dd_select_topk).  Each rank holds ONLY its shard in HBM (built
from the same synthetic set, byte-identical to a slice of it), plus the K models.  Inputs
are resident in HBM before timing.  Total work is fixed as N grows -> "scaling": "strong".

Rank 0 prints ONE JSON line.  `roofline` is measured live with HIP events around the
dominant hand-written kernel over the timed steps; `cpu_baseline` times the oracle's CPU
restatement of the reference path (config 1: EL2N, one checkpoint) on a bounded sample.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "examples scored/sec (whole node), EL2N+GraNd ResNet-18 CIFAR-10, 1/2/4/8 GPU"
SPLIT = ("split MFMA (fp16 halves in the EL2N forward, bf16 in GraNd): the dense 16-bit peak "
         "(2.5 PF, fp16 = bf16) / 3 MFMAs per fp32-equivalent product")
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)
# kind -> (bound, unit, peak, kernel description[, peak basis]); work units per _capi.kernel_log
KINDS = {
    "conv3x3": ("mfma", "TFLOP/s", 2500.0 / 3, "conv3x3_r2_kernel (16x16 and below) + "
                "conv3x3_kernel (32x32): backbone 3x3/1 conv, fwd + bwd-data, fused "
                "BN/ReLU/residual/mask epilogues (rocprof lists the two names; their "
                "launch-weighted mean is this kind's average)", SPLIT),
    "conv3x3_unit": ("mfma", "TFLOP/s", 2500.0 / 3, "conv3x3_kernel / conv3x3_r2_kernel with "
                     "the fused residual-unit input (EL2N: the staging reads the previous "
                     "unit's conv output and shortcut, applies BN + add + ReLU and writes the "
                     "unit output once -- a dd_bn_apply pass folded in; same MFMA work as "
                     "conv3x3)", SPLIT),
    "conv1x1": ("mfma", "TFLOP/s", 2500.0 / 3, "conv1x1_kernel: Bottleneck / projection 1x1 "
                "conv GEMM, fwd + bwd-data, fused BN/ReLU/residual/mask epilogues", SPLIT),
    "conv1x1_unit": ("mfma", "TFLOP/s", 2500.0 / 3, "conv1x1_kernel with the fused "
                     "residual-unit input (EL2N, configs 4-5: the previous Bottleneck's BN + "
                     "shortcut + ReLU computed while staging, the unit output written once -- a "
                     "dd_bn_apply pass folded in)", SPLIT),
    "conv_gemm": ("mfma", "TFLOP/s", 2500.0 / 3, "conv1x1_kernel (implicit-GEMM mode): kh x kw "
                  "conv where no staged-row kernel applies, fused BN staging/stats", SPLIT),
    "stem7": ("mfma", "TFLOP/s", 2500.0 / 3, "stem7_kernel: the ImageNet 7x7/2 stem conv, "
              "input rows staged once per output-row pair, BN statistics epilogue", SPLIT),
    "down_fwd": ("mfma", "TFLOP/s", 2500.0 / 3, "down_fwd_kernel: 3x3/2 conv + fused 1x1/2 "
                 "shortcut", SPLIT),
    "down_fwd_unit": ("mfma", "TFLOP/s", 2500.0 / 3, "down_fwd_kernel with the staging "
                      "transform (EL2N: the previous unit's BN + shortcut + ReLU computed while "
                      "staging -- a dd_bn_apply pass folded in)", SPLIT),
    "down_bwd": ("mfma", "TFLOP/s", 2500.0 / 3, "down_bwd2_kernel (down_bwd_kernel at 32x32): "
                 "transposed 3x3/2 + 1x1/2, ReLU mask", SPLIT),
    "direct3x3": ("mfma", "TFLOP/s", 2500.0 / 3, "pegrad_direct3x3_kernel: per-example weight "
                  "gradient norm, all taps", SPLIT),
    "pgram": ("mfma", "TFLOP/s", 2500.0 / 3, "pgram_kernel: shifted-Gram ghost norm "
              "(HBM/latency bound in practice)", SPLIT),
    "pgram_q": ("mfma", "TFLOP/s", 2500.0 / 3, "pgram_q_kernel: shifted-Gram ghost norm at "
                "16x16 (T = 256), tiled by quarters of the output positions; work = the "
                "identity's 2 (Ti^2 cin + To^2 cout)", SPLIT),
    "stem": ("hbm", "GB/s", 8000.0, "stem_kernel: input-conv per-example weight-gradient norm "
             "(reads act + gout once)"),
    "direct": ("mfma", "TFLOP/s", 157.3, "pegrad_direct_kernel (fp32 MFMA)"),
    "direct1x1": ("mfma", "TFLOP/s", 2500.0 / 3, "pegrad_direct1x1_kernel: per-example 1x1 "
                  "weight-gradient norm, split-bf16 GEMM over positions", SPLIT),
    "ghost": ("mfma", "TFLOP/s", 157.3, "pegrad_ghost64/16_kernel (fp32 MFMA)"),
    "el2n": ("hbm", "GB/s", 8000.0, "el2n_rows_kernel (latency-bound at these row counts)"),
    "linear": ("hbm", "GB/s", 8000.0, "linear_rows_kernel: classifier logits, one fixed-order "
               "wave reduction per row (latency-bound at these row counts)"),
    "bn_apply": ("hbm", "GB/s", 8000.0, "bn apply_kernel: grouped BN + residual + ReLU (+pool)"),
    "bn_pegrad": ("hbm", "GB/s", 8000.0, "bn_pegrad_kernel: per-example BN-affine gradient norm "
                  "(grand_params all)"),
    "select": ("hbm", "GB/s", 8000.0, "dd_select_topk: radix select + stable compaction + sort "
               "(latency-bound at 50k keys; 4N + 8k algorithmic bytes)"),
    "synth": ("hbm", "GB/s", 8000.0, "dd_synth_images_u8: on-device synthetic images"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n", type=int, default=50000, help="examples (config: 50k CIFAR-10)")
    ap.add_argument("--ckpts", type=int, default=10, help="K seed checkpoints")
    ap.add_argument("--sparsity", type=float, default=0.5)
    ap.add_argument("--grand-batch", type=int, default=1024)
    ap.add_argument("--el2n-chunk", type=int, default=1024)
    ap.add_argument("--pegrad", default="auto")
    ap.add_argument("--grand-params", default="conv_linear", help="conv_linear | all")
    ap.add_argument("--select-by", default="el2n")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-el2n-sample", type=int, default=5120)
    ap.add_argument("--cpu-1t-sample", type=int, default=384)
    ap.add_argument("--cpu-grand-sample", type=int, default=256)
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--no-kernel-log", action="store_true",
                    help="diagnostic: time the steps without per-launch events (no roofline)")
    ap.add_argument("--arch", default="resnet18", help="resnet18 (configs 1-3) | resnet50")
    ap.add_argument("--classes", type=int, default=10, help="10 | 100 (config 4) | 1000")
    ap.add_argument("--imagenet", action="store_true",
                    help="config 5 shape: 224x224 ImageNet-stem images generated on device per "
                         "rank (dd_synth_images_u8), EL2N only unless --methods says otherwise")
    ap.add_argument("--methods", default=None, help="comma list (default el2n,grand; "
                                                    "el2n with --imagenet)")
    ap.add_argument("--lanes", type=int, default=3,
                    help="HIP streams the launch chunks are dealt to (ScoreConfig.lanes)")
    ap.add_argument("--even-chunks", action="store_true",
                    help="A/B: the round-4 launch plan (equal chunks, tail padded to the buffer)")
    ap.add_argument("--el2n-operands", default="f16x3",
                    help="A/B: operand halves of the EL2N forward (f16x3 | bf16x3)")
    ap.add_argument("--grand-operands", default="f16x3",
                    help="A/B: operand halves of the GraNd forward (f16x3 | bf16x3)")
    ap.add_argument("--refine", default="auto", choices=("auto", "on", "off"),
                    help="near-threshold fp32 re-scoring (ScoreConfig.refine): auto = where the "
                         "selecting pass carries bf16-halves arithmetic")
    ap.add_argument("--no-refine", action="store_true", help="= --refine off")
    ap.add_argument("--concurrent-passes", action="store_true",
                    help="run the EL2N and GraNd passes on two HIP streams")
    ap.add_argument("--spawn", action="store_true",
                    help="start the rank process(es) from this launcher even at --gpus 1")
    ap.add_argument("--share-device", action="store_true",
                    help="rehearsal on a one-GPU box: every rank on cuda:0, scores gathered over "
                         "gloo through host memory (RCCL refuses two ranks on one device); the "
                         "ranks share the GPU, so the line measures the code path, not scaling")
    return ap.parse_args()


def setup_dist(args):
    """Join the job's RCCL process group whenever a launcher started this process (torchrun
    or launch_ranks, also at world 1: `--spawn` then runs the score all-gather through RCCL's
    all_gather_into_tensor), with a bounded timeout (launch.init_process_group)."""
    from data_diet_distributed_amd import launch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.share_device:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if launch.under_launcher():
        launch.init_process_group("gloo" if args.share_device else "nccl", rank, world, dev)
    return world, rank, dev


def workload_name(args, methods):
    if args.arch == "resnet18" and args.classes == 10 and not args.imagenet:
        return "R18/C10 EL2N+GraNd, K checkpoints, global keep-set"  # configs 1-3
    if args.arch == "resnet50" and args.classes == 100 and not args.imagenet:
        return "R50/C100 " + "+".join(m.upper() if m == "el2n" else "GraNd" for m in methods) + \
            ", K checkpoints, global keep-set (BASELINE config 4)"
    if args.imagenet:
        return (f"{args.arch} ImageNet-shape 224x224 synthetic, "
                + "+".join(methods) + ", global top-k (BASELINE config 5)")
    return f"{args.arch}/C{args.classes} " + "+".join(methods)


def _rccl_version():
    try:
        v = torch.cuda.nccl.version()
        return ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
    except Exception:  # noqa: BLE001 - informational only
        return None


def barrier(world):
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize()


def usable_cores():
    """(cores this process may run on, host logical CPUs).  The first is the affinity set
    capped by a cgroup CPU quota if one is set (the GPU box gives a job a share of a larger
    host); it is the thread count the CPU baseline uses."""
    host = os.cpu_count() or 1
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = host
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(float(q) / float(per))))
    except (OSError, ValueError):
        pass
    return n, host


def cpu_baseline(args, images, labels, sd0, methods, stem):
    """The reference's CPU scoring path (oracle.pipeline = its restatement, pinned to the
    reference's own outputs by tests/golden) on a bounded sample, on this host's cores.

    R18/C10 (configs 1-3) `value`: BASELINE config 1 = EL2N, ONE checkpoint, train-mode BN,
    batch 128, examples/s on all usable cores; also the same on one thread, and EL2N + GraNd
    over K checkpoints (the GPU workload; GraNd has no reference CPU path: the restatement's
    hook formulation).  Configs 4-5 (ResNet-50; the reference itself cannot run them:
    get_scores_and_prune.py:17 hard-codes one_hot(..., 10)): `value` is the bench's own
    workload (its methods x K checkpoints) on the oracle port, from a bounded sample."""
    from oracle import pipeline as o_pipe
    cores, host = usable_cores()
    r18 = args.arch == "resnet18" and args.classes == 10 and stem == "cifar"
    if r18:
        ne, ng = args.cpu_el2n_sample, args.cpu_grand_sample
    elif stem == "imagenet":
        ne, ng = min(args.cpu_el2n_sample, 128), 8
    else:
        ne, ng = min(args.cpu_el2n_sample, 768), 32
    n1 = args.cpu_1t_sample
    ne, ng, n1 = (min(v, len(labels)) for v in (ne, ng, n1))

    def rate(fn, n, threads):
        torch.set_num_threads(threads)
        fn(min(n, 16 if stem == "imagenet" else 128))  # warm the allocator / oneDNN, untimed
        t0 = time.perf_counter()
        fn(n)
        return n / (time.perf_counter() - t0)

    bs_e = 128 if stem == "cifar" else 32
    el2n = lambda n: o_pipe.el2n_scores(sd0, images[:n], labels[:n], batch_size=bs_e,  # noqa: E731
                                        stem=stem)
    grand = lambda n: o_pipe.grand_scores(sd0, images[:n], labels[:n], batch_size=min(n, 64),  # noqa: E731
                                          stem=stem)
    K = args.ckpts
    r_el2n = rate(el2n, ne, cores)
    r_grand = rate(grand, ng, cores) if "grand" in methods else None
    work = 1.0 / (K / r_el2n + (K / r_grand if r_grand else 0.0))
    desc = (f"EL2N {ne}" + (f" + GraNd {ng}" if r_grand else "") + f" examples, 1 checkpoint, "
            f"{cores} threads, scaled x{K} checkpoints")
    if r18:
        r_1t = rate(el2n, n1, 1)
        torch.set_num_threads(cores)
        return {"value": r_el2n, "unit": "examples/s", "cores": cores, "kind": "port",
                "sample": f"config 1 (reference CPU path: EL2N, 1 checkpoint, train-mode BN, "
                          f"batch 128) = oracle.pipeline.el2n_scores on the first {ne} examples, "
                          f"torch CPU fp32, {cores} threads",
                "host_logical_cpus": host,
                "el2n_1ckpt_1thread": {"value": r_1t, "sample": f"first {n1} examples, 1 thread"},
                "el2n_grand_kckpt": {"value": work, "checkpoints": K,
                                     "sample": desc + " (eval-BN GraNd by hook/unfold norms)"}}
    torch.set_num_threads(cores)
    return {"value": work, "unit": "examples/s", "cores": cores, "kind": "port",
            "sample": f"this line's workload ({'+'.join(methods)} x {K} checkpoints, "
                      f"{args.arch}/{args.classes} classes, {stem} stem) on the oracle port "
                      f"(torch CPU fp32): {desc}; the reference's own path cannot run it "
                      f"(get_scores_and_prune.py:17 one_hot(..., 10))",
            "host_logical_cpus": host,
            "el2n_1ckpt": {"value": r_el2n, "sample": f"first {ne} examples"},
            "grand_1ckpt": None if r_grand is None else {"value": r_grand,
                                                         "sample": f"first {ng} examples"}}


def kernel_report(log, steps):
    """Per-kind rooflines from a kernel log (`_capi.kernel_log` entries of `steps` steps):
    (dominant kind's line, other kinds' lines, kernel seconds per step, top launch shapes)."""
    # per (kind, shape, tag) key: exact launch count, mean duration of its sampled launches,
    # algorithmic HBM bytes per launch (matrix kernels; 0 = not logged)
    # (shapes with equal flop can differ in bytes: the bytes are part of the key)
    keys = {}
    for kind, work, e0, e1, tag, nb in log:
        ent = keys.setdefault((kind, work, tag, nb), [0, 0.0, 0])
        ent[0] += 1
        if e0 is not None:
            ent[1] += e0.elapsed_time(e1) * 1e-3
            ent[2] += 1
    kind_mean = {}  # fallback for a key with no sampled launch: its kind's seconds per work
    for (kind, work, _tag, _nb), (n, secs, ns) in keys.items():
        a = kind_mean.setdefault(kind, [0.0, 0.0])
        a[0] += secs
        a[1] += work * ns
    agg = {}  # kind -> [work, estimated seconds, launches, sampled launches, HBM bytes]
    by_shape = {}  # (kind:tag, work per launch) -> [seconds, launches]: which layers dominate
    for (kind, work, tag, nb), (n, secs, ns) in keys.items():
        est = secs / ns * n if ns else work * n * kind_mean[kind][0] / max(kind_mean[kind][1], 1e-30)
        a = agg.setdefault(kind, [0.0, 0.0, 0, 0, 0.0])
        a[0] += work * n
        a[1] += est
        a[2] += n
        a[3] += ns
        a[4] += nb * n
        b = by_shape.setdefault((kind + (":" + tag if tag else ""), work), [0.0, 0])
        b[0] += est
        b[1] += n
    kernel_s = sum(v[1] for v in agg.values())
    top = sorted(by_shape.items(), key=lambda kv: -kv[1][0])[:12]

    def line(kind):
        work, secs, cnt, sampled, nbytes = agg[kind]
        bound, unit, peak, desc = KINDS[kind][:4]
        if sampled == 0:  # a short run can leave a rare kind with no timed launch
            return {"kernel": desc, "bound": bound, "achieved": None, "peak": peak,
                    "unit": unit, "frac": None, "launches": cnt, "timed_launches": 0}
        ach = work / secs / (1e12 if unit == "TFLOP/s" else 1e9)
        d = {"kernel": desc, "bound": bound, "achieved": ach, "peak": peak, "unit": unit,
             "frac": ach / peak, "launches": cnt, "timed_launches": sampled,
             "avg_launch_us": secs / cnt * 1e6,
             ("flop_per_launch" if unit == "TFLOP/s" else "bytes_per_launch"): work / cnt,
             "total_s": secs, "share_of_kernel_time": secs / kernel_s}
        if len(KINDS[kind]) > 4:
            d["peak_basis"] = KINDS[kind][4]
        if unit == "TFLOP/s" and nbytes > 0:
            # the binding roofline: flop per algorithmic HBM byte against the ridge point
            intensity = work / nbytes
            ridge = peak * 1e12 / (HBM_PEAK_GBS * 1e9)
            d["flop_per_byte"] = intensity
            d["ridge_flop_per_byte"] = ridge
            d["mfma"] = {"achieved": ach, "peak": peak, "unit": unit, "frac": ach / peak}
            hbm = nbytes / secs / 1e9
            d["hbm"] = {"achieved": hbm, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": hbm / HBM_PEAK_GBS, "bytes_per_launch": nbytes / cnt}
            if intensity < ridge:  # below the ridge: HBM binds; report against it
                d.update({"bound": "hbm", "achieved": hbm, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": hbm / HBM_PEAK_GBS})
        return d

    # the dominant hand-written kernel = the kind with the most GPU time in the logged steps
    dom = max(agg, key=lambda k: agg[k][1])
    roofline = line(dom)
    roofline["traffic"] = None
    pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc):
        with open(pmc) as f:
            tr = json.load(f).get(dom)
        if tr:
            roofline["traffic"] = tr.get("hbm_bytes_per_launch")
            roofline["traffic_source"] = tr.get("source")
    extra = {k: line(k) for k in agg if k != dom}
    top_shapes = [{"kind": k, "work_per_launch": w, "s_per_step": t / steps,
                   "launches_per_step": n / steps,
                   "rate": w * n / t / (1e12 if KINDS[k.split(":")[0]][1] == "TFLOP/s" else 1e9)}
                  for (k, w), (t, n) in top]
    return roofline, extra, kernel_s / steps, top_shapes

def refine_setting(args):
    """ScoreConfig.refine from --refine / --no-refine."""
    if args.no_refine or args.refine == "off":
        return False
    return True if args.refine == "on" else "auto"


def full_record(args, methods, *, world, rank, elapsed, kept, shard, launcher, roofline, extra,
                kernel_step_s, top_shapes, roofline_timed, extra_timed, kernel_step_overlapped,
                refine, setup_s, phases, first_step_s):
    """Everything one bench run measured (written whole to --json-out; the printed line is
    compact_line() of it)."""
    return {
        "metric": METRIC if workload_name(args, methods).startswith("R18/C10") and
        set(methods) == {"el2n", "grand"} else
        f"examples scored/sec (whole node), {workload_name(args, methods)}",
        "value": args.n * args.steps / elapsed, "unit": "examples/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
        "dtype": "fp32 (split MFMA: hi*hi + hi*lo + lo*hi with fp32 accumulation; EL2N forward "
                 f"on {args.el2n_operands} halves, GraNd forward on {args.grand_operands}, "
                 "GraNd backward on bf16x3" + ("; near-threshold scores re-computed in plain "
                 "fp32" if (refine or {}).get("examples_rescored") else "") + ")",
        "data": ("synthetic (hash-defined 3x224x224 uint8 generated on device per rank, seed 0"
                 if args.imagenet else "synthetic (NumPy PCG64 class-structured 3x32x32 uint8, "
                 "seed 0") + f"; random-init {args.arch} checkpoints seeds 0..K-1)",
        "config": {"workload": workload_name(args, methods),
                   "arch": args.arch, "input": "3x224x224 imagenet stem" if args.imagenet
                   else "3x32x32 cifar stem",
                   "methods": list(methods),
                   "n_examples": args.n, "checkpoints": args.ckpts, "classes": args.classes,
                   "score_batch": 128, "grand_batch": args.grand_batch,
                   "el2n_chunk": args.el2n_chunk,
                   "sparsity": args.sparsity, "kept": kept, "select_by": args.select_by,
                   "pegrad_method": args.pegrad, "grand_params": args.grand_params,
                   "passes": "EL2N and GraNd on two HIP streams"
                   if args.concurrent_passes and len(methods) > 1 else "sequential",
                   "lanes": args.lanes, "launch_plan": "even" if args.even_chunks
                   else "full chunks + short tail", "el2n_operands": args.el2n_operands,
                   "grand_operands": args.grand_operands,
                   "parallelism": f"{world} rank(s): batch-aligned shards + " +
                   ("gloo all-gather, every rank on cuda:0 (shared-device rehearsal)"
                    if args.share_device else "RCCL all-gather"),
                   "shard_examples_rank0": shard if rank == 0 else None},
        "ranks": {"world_size": dist.get_world_size() if dist.is_initialized() else 1,
                  "backend": dist.get_backend() if dist.is_initialized() else None,
                  "rccl_version": _rccl_version(), "launcher": launcher},
        "roofline": roofline,
        "rooflines_other": extra,
        "roofline_timed_region": roofline_timed,
        "rooflines_other_timed_region": extra_timed,
        # summed kernel durations of one step on a single lane (the isolated step when
        # lanes > 1); the overlapped lanes' sum counts co-scheduled time once per launch
        "kernel_time_per_step_s": kernel_step_s,
        "kernel_time_per_step_s_overlapped": kernel_step_overlapped,
        # exact keep-set (ScoreConfig.refine): what the last timed step re-scored in fp32 near
        # the threshold, and its wall time (inside the timed step)
        "refine": refine,
        "top_launch_shapes": top_shapes,
        "setup_s": setup_s,
        "setup_breakdown_s": phases,
        # what a one-shot user pays from checkpoints in host memory to the keep-set: setup
        # without the synthetic generators (a real job reads files instead) + the first,
        # cold step (module loads, first-touch allocations)
        "one_shot": None if first_step_s is None else {
            "setup_s": setup_s - phases.get("data_synth_host_s", 0.0)
            - phases.get("ckpt_synth_host_s", 0.0),
            "first_step_s": first_step_s,
            "wall_s": setup_s - phases.get("data_synth_host_s", 0.0)
            - phases.get("ckpt_synth_host_s", 0.0) + first_step_s,
            "steady_step_s": elapsed / args.steps},
        "cpu_baseline": None,
    }


LINE_MAX_BYTES = 8000  # the driver parses the printed line; round 4's 22.6 KB line did not


def _sig(x, n=4):
    """Round floats to n significant digits (recursively) for the printed line."""
    if isinstance(x, float):
        return float(f"{x:.{n}g}")
    if isinstance(x, dict):
        return {k: _sig(v, n) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_sig(v, n) for v in x]
    return x


def compact_line(full: dict, side_file=None) -> dict:
    """The ONE printed JSON line: the bench contract's fields, the dominant kernel's roofline,
    one short entry per other kernel kind, the CPU baseline and the refinement record.  The
    overlapped timed-region rooflines, the per-shape split and the setup breakdown stay in the
    --json-out side file (`side_file`)."""
    keep = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
            "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config", "ranks")
    line = {k: full[k] for k in keep}
    r = full.get("roofline") or {}
    rl = {k: r[k] for k in ("bound", "achieved", "peak", "unit", "frac", "traffic",
                            "avg_launch_us", "launches", "timed_launches",
                            "share_of_kernel_time", "flop_per_launch", "bytes_per_launch",
                            "measured_on") if k in r}
    rl["kernel"] = r.get("kernel", "").split(":")[0]
    if "hbm" in r:
        rl["hbm_frac"] = r["hbm"]["frac"]
        rl["algorithmic_bytes_per_launch"] = r["hbm"]["bytes_per_launch"]
        if r.get("traffic"):
            rl["traffic_over_algorithmic"] = r["traffic"] / r["hbm"]["bytes_per_launch"]
    line["roofline"] = rl
    others = {}
    for kind, d in sorted((full.get("rooflines_other") or {}).items(),
                          key=lambda kv: -(kv[1].get("total_s") or 0.0)):
        others[kind] = {"bound": d["bound"], "frac": d.get("frac"),
                        "avg_us": d.get("avg_launch_us"), "share": d.get("share_of_kernel_time")}
    line["rooflines_other"] = others
    line["kernel_time_per_step_s"] = full.get("kernel_time_per_step_s")
    line["refine"] = full.get("refine")
    line["one_shot_wall_s"] = (full.get("one_shot") or {}).get("wall_s")
    line["cpu_baseline"] = full.get("cpu_baseline")
    if side_file:
        line["side_file"] = side_file
    line = _sig(line)
    line["value"] = full["value"]
    line["ms_per_step"] = full["ms_per_step"]
    while len(json.dumps(line)) > LINE_MAX_BYTES and line["rooflines_other"]:
        # drop the smallest kinds first (the side file keeps them all)
        last = list(line["rooflines_other"])[-1]
        del line["rooflines_other"][last]
    return line


def main():
    args = parse()
    from data_diet_distributed_amd import launch
    if not launch.under_launcher() and (args.gpus > 1 or args.spawn):
        argv = [os.path.abspath(__file__)] + [a for a in sys.argv[1:] if a != "--spawn"]
        sys.exit(launch.launch_ranks(args.gpus, argv))
    torch.backends.cudnn.benchmark = False  # MIOpen immediate mode: seconds, not minutes, to start
    world, rank, dev = setup_dist(args)
    launcher = launch.launcher_name(world)
    from data_diet_distributed_amd import _capi, checkpoints, synthetic
    from data_diet_distributed_amd.scoring import ScoreConfig, ScoringEngine, shard_bounds

    t_setup = time.time()
    phases = {}  # setup breakdown (outside the timed steps; a one-shot user pays all of it)

    def phase(name, t):
        torch.cuda.synchronize()
        phases[name] = phases.get(name, 0.0) + time.perf_counter() - t

    B = 128
    lo, hi = shard_bounds(args.n, B, world, rank)
    stem = "imagenet" if args.imagenet else "cifar"
    methods = tuple((args.methods or ("el2n" if args.imagenet else "el2n,grand")).split(","))
    t = time.perf_counter()
    if args.imagenet:
        # BASELINE config 5: each rank generates ONLY its shard in HBM (the whole set is
        # 193 GB of uint8); hash-defined, pinned by oracle/synth.py
        img_d, lab_d = synthetic.device_shard(0, lo, hi, args.classes, hw=224, device=dev)
        images = labels = None
        phase("data_s", t)
    else:
        # this rank's shard only (byte-identical to the slice of the whole synthetic set)
        images, labels = synthetic.make_images(args.n, args.classes, seed=0, lo=lo, hi=hi)
        phase("data_synth_host_s", t)
        t = time.perf_counter()
        img_d = torch.from_numpy(images).to(dev)
        lab_d = torch.from_numpy(labels).to(dev)
        phase("data_h2d_s", t)
    t = time.perf_counter()
    sds = [synthetic.make_checkpoint(args.arch, args.classes, seed=s, stem=stem)["net"]
           for s in range(args.ckpts)]
    phase("ckpt_synth_host_s", t)  # stands in for reading K checkpoint files
    t = time.perf_counter()
    models = checkpoints.build_models(sds, args.arch, args.classes, stem, device=dev)
    phase("ckpt_load_h2d_s", t)
    cfg = ScoreConfig(methods=methods, select_by=args.select_by if args.select_by in methods
                      else methods[0], batch_size=B, grand_batch=args.grand_batch,
                      el2n_chunk=args.el2n_chunk, pegrad_method=args.pegrad,
                      grand_params=args.grand_params,
                      concurrent_passes=args.concurrent_passes, refine=refine_setting(args),
                      lanes=args.lanes, even_chunks=args.even_chunks,
                      el2n_operands=args.el2n_operands, grand_operands=args.grand_operands)
    t = time.perf_counter()
    eng = ScoringEngine(models, cfg, dev)
    phase("fold_pack_s", t)
    for kname, v in eng.setup_times.items():
        phases[kname] = v
    setup_s = time.time() - t_setup

    def step():
        return eng.run(img_d, lab_d, args.sparsity, n_total=args.n)

    def progress(msg):
        if rank == 0:  # a heartbeat on stderr (long config-5 steps)
            print(f"[bench] {msg} at {time.time() - t_setup:.1f}s", file=sys.stderr, flush=True)

    if args.n > 200000:  # config 5: a pass runs for minutes; keep a heartbeat going
        eng.progress = progress
    progress(f"setup done ({setup_s:.1f}s)")
    first_step_s = None
    for i in range(args.warmup):
        t = time.perf_counter()
        step()
        torch.cuda.synchronize()
        if i == 0:
            first_step_s = time.perf_counter() - t
        progress(f"warmup step {i + 1}/{args.warmup}")
    barrier(world)
    # live per-launch HIP events on the launch stream (timed steps only)
    _capi.kernel_log = None if args.no_kernel_log else []
    t0 = time.perf_counter()
    for i in range(args.steps):
        full, kept, k = step()
        if args.steps > 1 and args.n > 200000:
            progress(f"timed step {i + 1}/{args.steps} issued")
    barrier(world)
    elapsed = time.perf_counter() - t0
    if dist.is_initialized():
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    log, _capi.kernel_log = _capi.kernel_log, None
    if log is None:
        print(json.dumps({"value": args.n * args.steps / elapsed,
                          "ms_per_step": elapsed / args.steps * 1e3, "kernel_log": False}))
        return

    roofline, extra, kernel_step_s, top_shapes = kernel_report(log, args.steps)
    roofline_timed, extra_timed, kernel_step_overlapped = None, None, None
    if args.lanes > 1:
        # With lanes > 1 the timed steps' launches overlap, so a launch's duration includes
        # the co-scheduled kernels: the per-kernel rooflines come from one more step on a
        # single lane (same kernels, same shapes, timed alone), the overlapped figures are
        # kept beside them
        roofline_timed, extra_timed = roofline, extra
        kernel_step_overlapped = kernel_step_s
        eng.cfg.lanes = 1
        _capi.kernel_log = []
        barrier(world)
        step()
        barrier(world)
        log1, _capi.kernel_log = _capi.kernel_log, None
        eng.cfg.lanes = args.lanes
        roofline, extra, kernel_step_s, top_shapes = kernel_report(log1, 1)
        roofline["measured_on"] = ("one extra single-lane step after the timed region (the "
                                   f"timed steps run {args.lanes} lanes whose launches overlap)")
    else:
        roofline["measured_on"] = "the timed steps (HIP events around sampled launches)"

    value = args.n * args.steps / elapsed
    out = full_record(args, methods, world=world, rank=rank, elapsed=elapsed, kept=int(k),
                      shard=hi - lo, launcher=launcher, roofline=roofline, extra=extra,
                      kernel_step_s=kernel_step_s, top_shapes=top_shapes,
                      roofline_timed=roofline_timed, extra_timed=extra_timed,
                      kernel_step_overlapped=kernel_step_overlapped,
                      refine=eng.last_refine if eng.last_refine is not None else {
                          "ran": False, "setting": cfg.refine,
                          "why": "selecting pass fp32-grade (f16x3 halves)"
                          if cfg.refine == "auto" else "off"},
                      setup_s=setup_s, phases=phases, first_step_s=first_step_s)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        if images is None:  # config 5: the sample comes back from the device-generated shard
            ns = min(args.cpu_el2n_sample, 128, hi - lo)
            images, labels = img_d[:ns].cpu().numpy(), lab_d[:ns].cpu().numpy()
        cb = cpu_baseline(args, images, labels, sds[0], methods, stem)
        kk = cb.get("el2n_grand_kckpt", {}).get("value", cb["value"])
        cb["gpu_vs_cpu"] = value / kk
        out["cpu_baseline"] = cb
    else:
        # the CPU baseline is timed on rank 0 of a one-GPU run only (bench contract): with N
        # ranks the host cores are shared by N GPU processes
        out["cpu_baseline"] = None
    if rank == 0:
        line = compact_line(out, side_file=args.json_out)
        print(json.dumps(line), flush=True)
        if args.json_out:  # the full record (every kernel kind, timed-region lanes, shapes)
            with open(args.json_out, "w") as f:
                f.write(json.dumps(out) + "\n")
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
