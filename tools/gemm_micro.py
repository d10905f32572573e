"""Micro-benchmark of the implicit-GEMM conv (dd_conv_gemm_forward) on the ResNet-50 ImageNet
shapes of BASELINE config 5, launched as the EL2N pass launches them (the producer's grouped
train-BN + ReLU staged, BN statistics epilogue, fp16 operand halves, 128-example BN groups).

    python tools/gemm_micro.py [--iters N] [--batch B]
Prints per shape: time per launch, achieved fp32-equivalent TF/s and the fraction of the split
peak (833 TF/s)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from data_diet_distributed_amd import _capi  # noqa: E402

SHAPES = (  # cin, cout, H (input), k, stride, pad
    (3, 64, 224, 7, 2, 3),
    (64, 64, 56, 3, 1, 1), (128, 128, 28, 3, 1, 1), (256, 256, 14, 3, 1, 1),
    (512, 512, 7, 3, 1, 1),
    (128, 128, 56, 3, 2, 1), (256, 256, 28, 3, 2, 1), (512, 512, 14, 3, 2, 1),
)


def timed(fn, iters):
    for _ in range(2):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--only", default=None, help="indices into SHAPES, comma-separated")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    B, gs = a.batch, 128
    g = torch.Generator(device=dev).manual_seed(0)
    sel = range(len(SHAPES)) if a.only is None else [int(v) for v in a.only.split(",")]
    for i in sel:
        cin, cout, H, k, s, p = SHAPES[i]
        x = torch.randn(B, cin, H, H, device=dev, generator=g)
        w = torch.randn(cout, cin, k, k, device=dev, generator=g) / (k * cin ** 0.5)
        pk = _capi.conv_gemm_pack(w, operands="f16x3")
        G = B // gs
        aff = None
        if cin > 3:
            aff = (torch.rand(G, cin, device=dev, generator=g) + 0.5,
                   torch.randn(G, cin, device=dev, generator=g) * 0.1)
        Ho = (H + 2 * p - k) // s + 1
        fn = (lambda: _capi.conv_gemm(x, pk, cout, k, s, p, in_affine=aff, group_size=gs,
                                      stats=True))
        t = timed(fn, a.iters)
        fl = 2.0 * B * Ho * Ho * cin * cout * k * k
        print(f"conv_gemm {k}x{k}/{s} {cin:4d}->{cout:4d} {H:3d}->{Ho:<3d} {t:9.1f} us "
              f"{fl / t / 1e6:6.1f} TF/s {fl / t / 1e6 / 833.3:.3f}", flush=True)
        if k == 3 and s == 1 and _capi.conv3x3_padded_supported(H, H, cin, cout, gs):
            # the same launch on dd_conv3x3_forward's padded-width tiles (ABI 10)
            p3 = _capi.conv3x3_pack(w, operands="f16x3")
            fn3 = (lambda: _capi.conv3x3(x, p3, cout, in_affine=aff, group_size=gs, stats=True))
            t3 = timed(fn3, a.iters)
            print(f"conv3x3pw {k}x{k}/{s} {cin:4d}->{cout:4d} {H:3d}->{Ho:<3d} {t3:9.1f} us "
                  f"{fl / t3 / 1e6:6.1f} TF/s {fl / t3 / 1e6 / 833.3:.3f}", flush=True)
        if k == 3 and s == 2 and _capi.down_padded_supported(Ho, Ho, cin, cout, gs):
            # the same launch on dd_down_forward's padded-width heads (ABI 10)
            p3 = _capi.conv3x3_pack(w, operands="f16x3")
            fnd = (lambda: _capi.conv_down_unit_input(x, aff, p3, cout, gs))
            td = timed(fnd, a.iters)
            print(f"downpw    {k}x{k}/{s} {cin:4d}->{cout:4d} {H:3d}->{Ho:<3d} {td:9.1f} us "
                  f"{fl / td / 1e6:6.1f} TF/s {fl / td / 1e6 / 833.3:.3f}", flush=True)


if __name__ == "__main__":
    main()
