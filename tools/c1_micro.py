"""Micro-benchmark of the 1x1 conv GEMM (dd_conv1x1_forward) on the ResNet-50 ImageNet shapes
of BASELINE config 5, launched as the EL2N pass launches them (fp16 operand halves, BN
statistics epilogue over 128-example groups; the producer's BN + ReLU staged where the pass
stages it), plus a write-bandwidth reference: a plain copy of the output size.

    python tools/c1_micro.py [--iters N] [--batch B] [--no-stats]
Prints per shape: time per launch, algorithmic bytes (input read + output written) per
second and its fraction of 8 TB/s, and fp32-equivalent TF/s."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from data_diet_distributed_amd import _capi  # noqa: E402

SHAPES = (  # cin, cout, H (input), stride, staged BN (the pass's conv3s; conv1s / projections raw)
    (64, 64, 56, 1, False), (64, 256, 56, 1, True), (64, 256, 56, 1, False),
    (256, 512, 56, 2, False), (128, 512, 28, 1, True), (512, 1024, 28, 2, False),
    (256, 1024, 14, 1, True), (1024, 2048, 14, 2, False), (512, 2048, 7, 1, True),
    (2048, 512, 7, 1, False),
)


# the fused unit-input launches (a Bottleneck's conv1 reading the previous unit's output,
# identity residual): (cin, cout, H, 1, False) -- `--epi unit`
UNIT = ((256, 64, 56, 1, False), (256, 128, 56, 1, False), (512, 128, 28, 1, False),
        (512, 256, 28, 1, False), (1024, 256, 14, 1, False), (1024, 512, 14, 1, False))
UNIT_CIFAR = ((256, 64, 32, 1, False), (256, 128, 32, 1, False), (512, 128, 16, 1, False),
              (512, 256, 16, 1, False), (1024, 256, 8, 1, False), (1024, 512, 8, 1, False))

# config 4's GraNd backward-data GEMMs (bf16 halves; `--epi bwd`): (cin', cout', H, kind, -)
# with kind 0 = conv3^T (ReLU mask), 1 = conv1^T (residual + mask), 2 = projection^T (plain)
BWD_CIFAR = ((256, 64, 32, 0), (512, 128, 16, 0), (1024, 256, 8, 0), (2048, 512, 4, 0),
             (64, 256, 32, 1), (128, 512, 16, 1), (256, 1024, 8, 1), (512, 2048, 4, 1),
             (256, 64, 32, 2), (512, 256, 16, 2), (1024, 512, 8, 2), (2048, 1024, 4, 2))

# config 4 (ResNet-50 CIFAR-100, 32x32 input): the same launches at the CIFAR maps
CIFAR = (
    (64, 64, 32, 1, False), (64, 256, 32, 1, True), (64, 256, 32, 1, False),
    (256, 512, 32, 2, False), (128, 512, 16, 1, True), (512, 1024, 16, 2, False),
    (256, 1024, 8, 1, True), (1024, 2048, 8, 2, False), (512, 2048, 4, 1, True),
    (2048, 512, 4, 1, False),
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
    ap.add_argument("--no-stats", action="store_true")
    ap.add_argument("--cifar", action="store_true", help="config 4's shapes")
    ap.add_argument("--epi", default="el2n",
                    choices=("el2n", "grandf", "grandb", "unit", "bwd"),
                    help="el2n: BN statistics, fp16 (default); grandf: the GraNd forward's "
                         "folded-BN epilogues, fp16 (bias + residual + ReLU on the staged-BN "
                         "rows' shapes, bias + ReLU or, at stride 2, bias on the others); "
                         "grandb: the backward-data GEMM W^T dy with the ReLU mask, bf16")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    B, gs = a.batch, 128
    g = torch.Generator(device=dev).manual_seed(0)
    if a.epi == "bwd":
        for cin, cout, H, kind in BWD_CIFAR:
            dy = torch.randn(B, cin, H, H, device=dev, generator=g)
            w = torch.randn(cin, cout, 1, 1, device=dev, generator=g) / cin ** 0.5
            pt = _capi.conv1x1_pack(w, transpose=True)  # dx = w^T dy, bf16 halves
            msk = torch.randn(B, cout, H, H, device=dev, generator=g)
            res = torch.randn(B, cout, H, H, device=dev, generator=g)
            dx = torch.empty(B, cout, H, H, device=dev)
            kw = ({"mask_src": msk}, {"mask_src": msk, "residual": res}, {})[kind]
            t = timed(lambda: _capi.conv1x1(dy, pt, cout, out=dx, **kw), a.iters)
            print(f"bwd{kind} {cin:4d}->{cout:4d} {H:3d}/1    {t:8.1f} us", flush=True)
        return
    shapes = (UNIT_CIFAR if a.cifar else UNIT) if a.epi == "unit" else (CIFAR if a.cifar else SHAPES)
    for cin, cout, H, s, xf in shapes:
        Ho = H // s
        x = torch.randn(B, cin, H, H, device=dev, generator=g)
        w = torch.randn(cout, cin, 1, 1, device=dev, generator=g) / cin ** 0.5
        pk = _capi.conv1x1_pack(w, operands="f16x3")
        aff = None
        if xf:
            aff = (torch.rand(B // gs, cin, device=dev, generator=g) + 0.5,
                   torch.randn(B // gs, cin, device=dev, generator=g) * 0.1)
        y = torch.empty(B, cout, Ho, Ho, device=dev)
        st = not a.no_stats
        if a.epi == "el2n":
            t = timed(lambda: _capi.conv1x1(x, pk, cout, stride=s, out=y, in_affine=aff,
                                            group_size=gs, stats=st), a.iters)
        elif a.epi == "unit":
            G = B // gs
            paff = (torch.rand(G, cin, device=dev, generator=g) + 0.5,
                    torch.randn(G, cin, device=dev, generator=g) * 0.1)
            res = torch.randn(B, cin, H, H, device=dev, generator=g)
            t = timed(lambda: _capi.conv1x1_unit_input(x, paff, pk, cout, gs, residual=res),
                      a.iters)
        elif a.epi == "grandf":
            bias = torch.randn(cout, device=dev, generator=g)
            res = torch.randn(B, cout, Ho, Ho, device=dev, generator=g) if xf else None
            t = timed(lambda: _capi.conv1x1(x, pk, cout, stride=s, out=y, bias=bias,
                                            residual=res, relu=s == 1), a.iters)
        else:
            pt = _capi.conv1x1_pack(w, transpose=True)  # bf16 halves
            dy = torch.randn(B, cout, Ho, Ho, device=dev, generator=g)
            msk = torch.randn(B, cin, Ho, Ho, device=dev, generator=g)
            dx = torch.empty(B, cin, Ho, Ho, device=dev)
            t = timed(lambda: _capi.conv1x1(dy, pt, cin, out=dx, mask_src=msk), a.iters)
        src = torch.empty(B * cout * Ho * Ho // 2, device=dev)
        dst = torch.empty_like(src)
        tc = timed(lambda: dst.copy_(src), a.iters)  # same bytes moved: half read, half written
        nb = 4.0 * B * (cin * Ho * Ho * (1 if s == 1 else 1) + cout * Ho * Ho)
        fl = 2.0 * B * Ho * Ho * cin * cout
        print(f"conv1x1 {cin:4d}->{cout:4d} {H:3d}/{s}{' xf' if xf else '   '} {t:8.1f} us "
              f"{nb / t / 1e3:7.1f} GB/s {nb / t / 1e3 / 8000:.3f} {fl / t / 1e6:6.1f} TF/s"
              f" | copy of the output bytes {tc:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
