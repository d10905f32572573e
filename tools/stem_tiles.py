"""Time the stem conv (3 -> 64, 32x32, 1024 examples) through libdd under the current
DD_CONV_TILE family: plain, GraNd-forward (bias + ReLU + mask_out) and EL2N (stats) epilogues.
    DD_CONV_TILE=wide python tools/stem_tiles.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from data_diet_distributed_amd import _capi  # noqa: E402


def timed(fn, iters=30):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    B, cin, cout, H = 1024, 3, 64, 32
    x = torch.randn(B, cin, H, H, device=dev, generator=g)
    w = torch.randn(cout, cin, 3, 3, device=dev, generator=g) / 5
    pk = _capi.conv3x3_pack(w)
    bias = torch.randn(cout, device=dev, generator=g)
    mo = _capi.conv3x3_mask(B, cout, H, H, dev)
    fl = 2.0 * B * H * H * cin * cout * 9
    tag = os.environ.get("DD_CONV_TILE", "default")
    for name, fn in (
            ("plain", lambda: _capi.conv3x3(x, pk, cout)),
            ("bias+relu+mask_out", lambda: _capi.conv3x3(x, pk, cout, bias=bias, relu=True,
                                                        mask_out=mo)),
            ("stats", lambda: _capi.conv3x3(x, pk, cout, group_size=128, stats=True))):
        us = timed(fn)
        print(f"stem {tag:8s} {name:20s} {us:7.1f} us  {fl / us / 1e6:6.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
