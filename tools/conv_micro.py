"""Micro-benchmark of the hand-written backbone kernels on the ResNet-18 CIFAR shapes (for
profiling: every launch is one kernel at the bench's chunk sizes).

    python tools/conv_micro.py [--iters N] [--only conv|down|bwd|pegrad] [--batch B]
Prints achieved TF/s (algorithmic fp32-equivalent flop) per shape."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from data_diet_distributed_amd import _capi  # noqa: E402


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
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--only", default="conv,down,bwd,pegrad")
    ap.add_argument("--shapes", default=None,
                    help="conv3x3 shapes 'cin:cout:H,...' instead of the ResNet-18 ones")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    B = a.batch
    only = a.only.split(",")
    g = torch.Generator(device=dev).manual_seed(0)
    if "conv" in only:
        shapes = ((64, 64, 32), (128, 128, 16), (256, 256, 8), (512, 512, 4), (3, 64, 32))
        if a.shapes:
            shapes = [tuple(int(v) for v in sh.split(":")) for sh in a.shapes.split(",")]
        for cin, cout, H in shapes:
            x = torch.randn(B, cin, H, H, device=dev, generator=g)
            w = torch.randn(cout, cin, 3, 3, device=dev, generator=g) / (3 * cin ** 0.5)
            pk = _capi.conv3x3_pack(w)
            y = torch.empty(B, cout, H, H, device=dev)
            t = timed(lambda: _capi.conv3x3(x, pk, cout, out=y), a.iters)
            fl = 2.0 * B * H * H * cin * cout * 9
            print(f"conv3x3 {cin:4d}->{cout:4d} {H:2d}x{H:<2d} {t:8.1f} us {fl / t / 1e6:6.1f} TF/s",
                  flush=True)
    if "down" in only or "bwd" in only:
        for cin, cout, HI in ((64, 128, 32), (128, 256, 16), (256, 512, 8)):
            HO = HI // 2
            x = torch.randn(B, cin, HI, HI, device=dev, generator=g)
            w3 = torch.randn(cout, cin, 3, 3, device=dev, generator=g) / (3 * cin ** 0.5)
            w1 = torch.randn(cout, cin, 1, 1, device=dev, generator=g) / cin ** 0.5
            fl = 2.0 * B * HO * HO * cin * cout * 10
            if "down" in only:
                p3, p1 = _capi.conv3x3_pack(w3), _capi.conv1x1_pack(w1)
                t = timed(lambda: _capi.conv_down(x, p3, cout, p1), a.iters)
                print(f"down_fwd {cin:4d}->{cout:4d} {HI:2d}->{HO:<2d} {t:8.1f} us "
                      f"{fl / t / 1e6:6.1f} TF/s", flush=True)
            if "bwd" in only:
                p3t = _capi.conv3x3_pack(w3, transpose_flip=True)
                p1t = _capi.conv1x1_pack(w1, transpose=True)
                dh = torch.randn(B, cout, HO, HO, device=dev, generator=g)
                dz = torch.randn(B, cout, HO, HO, device=dev, generator=g)
                t = timed(lambda: _capi.down_backward(dh, p3t, cin, dz=dz, packed1x1_t=p1t,
                                                      mask_src=x), a.iters)
                print(f"down_bwd {cout:4d}->{cin:4d} {HO:2d}->{HI:<2d} {t:8.1f} us "
                      f"{fl / t / 1e6:6.1f} TF/s", flush=True)
    if "c1x1" in only:
        # ResNet-50 CIFAR 1x1 convs (Bottleneck conv1/conv3, projections), against MIOpen fp32
        import torch.nn.functional as F
        for cin, cout, H, st in ((64, 64, 32, 1), (256, 64, 32, 1), (64, 256, 32, 1),
                                 (256, 512, 32, 2), (512, 128, 16, 1), (128, 512, 16, 1),
                                 (1024, 256, 8, 1), (256, 1024, 8, 1), (2048, 512, 4, 1),
                                 (512, 2048, 4, 1)):
            Ho = H // st
            x = torch.randn(B, cin, H, H, device=dev, generator=g)
            w = torch.randn(cout, cin, 1, 1, device=dev, generator=g) / cin ** 0.5
            pk = _capi.conv1x1_pack(w)
            y = torch.empty(B, cout, Ho, Ho, device=dev)
            t = timed(lambda: _capi.conv1x1(x, pk, cout, stride=st, out=y), a.iters)
            tm = timed(lambda: F.conv2d(x, w, stride=st), a.iters)
            fl = 2.0 * B * Ho * Ho * cin * cout
            print(f"conv1x1 {cin:4d}->{cout:4d} {H:2d}/{st} {t:8.1f} us {fl / t / 1e6:6.1f} TF/s"
                  f" | MIOpen fp32 {tm:8.1f} us {fl / tm / 1e6:6.1f} TF/s", flush=True)
    if "pegrad" in only:
        for cin, cout, H, st in ((3, 64, 32, 1), (64, 64, 32, 1), (128, 128, 16, 1),
                                 (256, 256, 8, 1), (512, 512, 4, 1), (64, 128, 32, 2),
                                 (128, 256, 16, 2), (256, 512, 8, 2)):
            Ho = H // st
            act = torch.relu(torch.randn(B, cin, H, H, device=dev, generator=g))
            gout = torch.randn(B, cout, Ho, Ho, device=dev, generator=g) * 1e-2
            geom = _capi.conv_geom(act, gout, (3, 3), st, 1)
            kind = _capi.conv_method(geom, "auto")
            ws = torch.empty(max(_capi.conv_workspace_bytes(geom, "auto"), 4), dtype=torch.uint8,
                             device=dev)
            sq = torch.zeros(B, device=dev)
            t = timed(lambda: _capi.conv_pegrad_sqnorm(act, gout, (3, 3), st, 1, sq, ws), a.iters)
            T = Ho * Ho
            fl = (2.0 * B * T * cin * 9 * cout if kind.startswith("direct")
                  else 2.0 * B * T * T * (cin * 9 + cout))
            print(f"pegrad[{kind:9s}] {cin:4d}->{cout:4d} {H:2d}/{st} {t:8.1f} us "
                  f"{fl / t / 1e6:6.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
