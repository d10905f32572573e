"""HBM roofline sweep for the byte-bound kernels: dd_el2n, dd_normalize_u8, dd_select_topk.

At the bench configuration these run on 1024-row chunks / a 50k-key vector and are bound by
launch latency, so their HBM roofline is shown on a size sweep.  Algorithmic
bytes (read once + written once):
  el2n (score + accum)    4C (logits) + 8 (label) + 4 (score) + 8 (accum RMW) per row
  el2n (score + e row)    4C + 8 + 4 + 4C per row
  normalize               3*HW (u8 in) + 12*HW (fp32 out) per image
  select_topk             4N (keys, read once) + 8k (int64 idx out): the minimum; the
                          implementation reads the keys once per radix pass
Every configuration is timed two ways: HIP events on the launch stream around `iters` calls
(this script's own JSON), and — when run under `rocprofv3 --kernel-trace` — by the trace:
one-image dd_synth_images_u8 launches bracket each configuration's timed calls,
and tools/hbm_trace_table.py sums the dispatches between markers (all kernels of a
select_topk call included).

    python tools/bench_hbm_kernels.py OUT.json
    rocprofv3 --kernel-trace --output-format csv -d D -o hbm -- python3 tools/bench_hbm_kernels.py OUT.json
    python tools/hbm_trace_table.py D/.../hbm_kernel_trace.csv OUT.json > table.txt
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from data_diet_distributed_amd import _capi  # noqa: E402

HBM_PEAK = 8000.0


def marker():
    _capi.synth_images_u8(0, 0, 1, 10, hw=32, device="cuda")


def timed(fn, iters):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    marker()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    marker()
    return e0.elapsed_time(e1) / iters * 1e-3


def main():
    dev = torch.device("cuda:0")
    only = os.environ.get("DD_HBM_ONLY", "")  # e.g. "select": run one kernel family
    rows = []

    def add(kernel, byts, t, iters, **shape):
        rows.append(dict(kernel=kernel, bytes=byts, iters=iters, us=t * 1e6,
                         GBps=byts / t / 1e9, frac=byts / t / 1e9 / HBM_PEAK, **shape))
        print(json.dumps(rows[-1]), flush=True)

    for C in (10, 100, 1000) if only in ("", "el2n") else ():
        for B in (1024, 1 << 16, 1 << 20, 1 << 23):
            if B * C > (1 << 30):
                continue
            it = 20 if B * C <= (1 << 24) else 5
            lg = torch.randn(B, C, device=dev)
            y = torch.randint(0, C, (B,), device=dev)
            sc = torch.empty(B, device=dev)
            acc = torch.zeros(B, device=dev)
            t = timed(lambda: _capi.el2n(lg, y, score=sc, accum=acc), it)
            add("el2n", B * (4 * C + 8 + 4 + 8), t, it, C=C, rows=B)
            e = torch.empty(B, C, device=dev)
            t = timed(lambda: _capi.el2n(lg, y, score=sc, e=e), it)
            add("el2n+e", B * (8 * C + 8 + 4), t, it, C=C, rows=B)
            del lg, e
    for n in (1024, 1 << 14, 1 << 17) if only in ("", "normalize") else ():
        img = torch.randint(0, 256, (n, 3, 32, 32), dtype=torch.uint8, device=dev)
        out = torch.empty(n, 3, 32, 32, device=dev)
        t = timed(lambda: _capi.normalize_u8(img, (0.4914, 0.4822, 0.4465),
                                             (0.2023, 0.1994, 0.2010), out), 10)
        add("normalize", n * 3 * 1024 * 5, t, 10, images=n)
    for n in (50000, 1 << 20, 1281167, 1 << 24, 1 << 26) if only in ("", "select") else ():
        keys = torch.rand(n, device=dev)
        k = n // 2
        idx = torch.empty(k, dtype=torch.int64, device=dev)
        ws = torch.empty(_capi.select_workspace_bytes(n), dtype=torch.uint8, device=dev)
        t = timed(lambda: _capi.select_topk(keys, k, idx_out=idx, workspace=ws,
                                            check_nan=False), 5)
        add("select_topk", 4 * n + 8 * k, t, 5, n=n, k=k)
    # a wider key range (survivors over many octaves: 4 LSD passes instead of 3)
    for n in (1 << 24,) if only in ("", "select") else ():
        keys = torch.rand(n, device=dev) ** 8
        k = n // 2
        idx = torch.empty(k, dtype=torch.int64, device=dev)
        ws = torch.empty(_capi.select_workspace_bytes(n), dtype=torch.uint8, device=dev)
        t = timed(lambda: _capi.select_topk(keys, k, idx_out=idx, workspace=ws,
                                            check_nan=False), 5)
        add("select_topk", 4 * n + 8 * k, t, 5, n=n, k=k, dist="rand^8")
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
