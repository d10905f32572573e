"""Micro-benchmark of dd_conv_pegrad_sqnorm per ResNet layer shape (GPU; not product code).

Times each (shape, method, precision) with HIP events on the launch stream and prints the
algorithmic TFLOP/s (SURVEY §8(d) flop model) and the algorithmic HBM bytes/s (act + gout
read once)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from data_diet_distributed_amd import _capi  # noqa: E402
from data_diet_distributed_amd._capi import pegrad_flop  # noqa: E402

# (name, cin, h, cout, k, stride, pad) — ResNet-18 at 32x32
R18 = [("stem", 3, 32, 64, 3, 1, 1), ("l1", 64, 32, 64, 3, 1, 1),
       ("l2.0.c1", 64, 32, 128, 3, 2, 1), ("l2", 128, 16, 128, 3, 1, 1),
       ("l2.sc", 64, 32, 128, 1, 2, 0), ("l3.0.c1", 128, 16, 256, 3, 2, 1),
       ("l3", 256, 8, 256, 3, 1, 1), ("l3.sc", 128, 16, 256, 1, 2, 0),
       ("l4.0.c1", 256, 8, 512, 3, 2, 1), ("l4", 512, 4, 512, 3, 1, 1),
       ("l4.sc", 256, 8, 512, 1, 2, 0)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--json", default=None)
    ap.add_argument("--auto-only", action="store_true", help="only the production dispatch")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    B = args.batch
    rows = []
    for name, cin, h, cout, k, s, p in R18:
        ho = (h + 2 * p - k) // s + 1
        act = torch.relu(torch.randn(B, cin, h, h, device=dev))
        gout = torch.randn(B, cout, ho, ho, device=dev) * 1e-2
        geom = _capi.conv_geom(act, gout, (k, k), s, p)
        combos = (("direct", "fp32"), ("ghost", "fp32"), ("direct", "bf16x3"),
                  ("auto", "bf16x3"))
        for method, prec in combos[3:] if args.auto_only else combos:
            kind = _capi.conv_method(geom, method, prec)
            if method == "direct" and prec == "bf16x3" and kind != "direct3x3":
                continue
            ws = torch.empty(_capi.conv_workspace_bytes(geom, method, prec), dtype=torch.uint8,
                             device=dev)
            sq = torch.zeros(B, device=dev)
            for _ in range(3):
                _capi.conv_pegrad_sqnorm(act, gout, (k, k), s, p, sq, ws, method, precision=prec)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                _capi.conv_pegrad_sqnorm(act, gout, (k, k), s, p, sq, ws, method, precision=prec)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / args.iters * 1e3
            fl = pegrad_flop(geom, kind)
            byts = 4.0 * (act.numel() + gout.numel())
            row = {"layer": name, "method": method, "prec": prec, "kernel": kind, "us": us,
                   "tflops": fl / us / 1e6, "gbs": byts / us / 1e3, "us_per_example": us / B}
            rows.append(row)
            print(f"{name:8s} {method:6s} {prec:6s} -> {kind:9s} {us:9.1f} us  "
                  f"{row['tflops']:7.1f} TF/s  {row['gbs']:7.0f} GB/s  "
                  f"{row['us_per_example']:.3f} us/ex", flush=True)
    for prec in ("fp32", "bf16x3"):
        tot = sum(r["us"] for r in rows if r["method"] == "auto" and r["prec"] == prec) \
            if prec == "bf16x3" else None
    auto = [r for r in rows if r["method"] == "auto"]
    print("auto total per example (all 11 shapes once): %.3f us" %
          sum(r["us_per_example"] for r in auto))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
