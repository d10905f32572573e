"""bench.py's printed line stays driver-readable: kernel_report + full_record + compact_line on a
synthetic kernel log holding every kernel kind, with the long side-file blocks present.
(Round 4's 22.6 KB line was not parsed by the driver.)"""
import argparse
import json

import bench


class _Ev:
    def __init__(self, t):
        self.t = t

    def elapsed_time(self, other):
        return (other.t - self.t) * 1e3  # ms, like torch.cuda.Event


def _log(n_shapes=6, per_shape=40):
    log = []
    t = 0.0
    for kind, spec in bench.KINDS.items():
        for s in range(n_shapes):
            work = 1e9 * (s + 1) if spec[1] == "TFLOP/s" else 1e7 * (s + 1)
            nbytes = 3e8 if spec[1] == "TFLOP/s" else 0
            for i in range(per_shape):
                if i % 8 == 0:
                    e0, e1 = _Ev(t), _Ev(t + 1e-4 * (s + 1))
                else:
                    e0 = e1 = None
                t += 1e-3
                log.append((kind, work, e0, e1, f"epi{s % 3}", nbytes))
    return log


def _args(**kw):
    a = dict(gpus=1, steps=20, warmup=5, n=50000, ckpts=10, sparsity=0.5, grand_batch=1024,
             el2n_chunk=1024, pegrad="auto", grand_params="conv_linear", select_by="el2n",
             json_out="profiles/r05_x/bench.json", arch="resnet18", classes=10, imagenet=False,
             methods=None, lanes=3, concurrent_passes=False, share_device=False,
             even_chunks=False, el2n_operands="f16x3", grand_operands="f16x3")
    a.update(kw)
    return argparse.Namespace(**a)


def _full(args, methods=("el2n", "grand")):
    log = _log()
    roof, extra, ks, top = bench.kernel_report(log, 1)
    roof_t, extra_t, _, _ = bench.kernel_report(log, 20)
    full = bench.full_record(
        args, methods, world=1, rank=0, elapsed=119.0, kept=25000, shard=50000,
        launcher="torchrun", roofline=roof, extra=extra, kernel_step_s=ks, top_shapes=top,
        roofline_timed=roof_t, extra_timed=extra_t, kernel_step_overlapped=ks * 0.7,
        refine={"method": "el2n", "iterations": 3, "band_rel": 6e-6, "max_rel_diff": 8e-6,
                "expected_wrong_side": 0.0, "converged": True, "budget_capped": False,
                "examples_rescored": 640, "seconds": 0.094},
        setup_s=40.0, phases={f"phase_{i}_s": 1.0 for i in range(12)}, first_step_s=9.0)
    full["cpu_baseline"] = {
        "value": 552.6, "unit": "examples/s", "cores": 16, "kind": "port",
        "sample": "config 1 (reference CPU path: EL2N, 1 checkpoint, train-mode BN, batch 128) "
                  "= oracle.pipeline.el2n_scores on the first 5120 examples, 16 threads",
        "host_logical_cpus": 256,
        "el2n_1ckpt_1thread": {"value": 200.5, "sample": "first 384 examples, 1 thread"},
        "el2n_grand_kckpt": {"value": 3.2, "checkpoints": 10, "sample": "x" * 150},
        "gpu_vs_cpu": 2730.9}
    return full


def test_printed_line_under_10kb_with_required_fields():
    args = _args()
    full = _full(args)
    assert len(json.dumps(full)) > 10000  # the side file keeps the long blocks
    line = bench.compact_line(full, side_file=args.json_out)
    text = json.dumps(line)
    assert len(text) <= 10 * 1024, len(text)
    back = json.loads(text)
    for key in ("metric", "value", "unit", "ms_per_step", "steps", "warmup", "n_gpus", "config",
                "dtype", "ranks", "roofline", "rooflines_other", "cpu_baseline", "refine",
                "higher_is_better", "scaling", "vs_baseline"):
        assert key in back, key
    for key in ("roofline_timed_region", "rooflines_other_timed_region", "top_launch_shapes",
                "setup_breakdown_s"):
        assert key not in back, key
    r = back["roofline"]
    for key in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert key in r, key
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3 * r["frac"]
    assert back["value"] == full["value"]  # not rounded
    assert back["steps"] == 20 and back["warmup"] == 5 and back["n_gpus"] == 1
    assert len(back["rooflines_other"]) == len(bench.KINDS) - 1
    assert back["cpu_baseline"]["cores"] == 16


def test_line_drops_small_kinds_before_exceeding_cap(monkeypatch):
    args = _args()
    full = _full(args)
    monkeypatch.setattr(bench, "LINE_MAX_BYTES", 3500)
    line = bench.compact_line(full)
    assert len(json.dumps(line)) <= 3500
    assert 0 < len(line["rooflines_other"]) < len(bench.KINDS) - 1
