"""Micro-benchmark: split-bf16 3x3 conv kernel vs MIOpen fp32 (F.conv2d) on ResNet shapes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from data_diet_distributed_amd import _capi  # noqa: E402


def timed(fn, iters=20):
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
    torch.backends.cudnn.benchmark = False
    dev = torch.device("cuda:0")
    for B in (512, 128):
        for cin, cout, H in ((64, 64, 32), (128, 128, 16), (256, 256, 8), (512, 512, 4)):
            W = H
            x = torch.randn(B, cin, H, W, device=dev)
            w = torch.randn(cout, cin, 3, 3, device=dev) / (3 * cin ** 0.5)
            flop = 2.0 * B * H * W * cout * cin * 9
            t_m = timed(lambda: F.conv2d(x, w, padding=1))
            line = f"B={B:4d} {cin:4d}->{cout:4d} {H:2d}x{W:2d}  MIOpen {t_m:8.1f} us {flop/t_m/1e6:6.1f} TF/s"
            if W in (4, 8, 16, 32):
                packed = _capi.conv3x3_pack(w)
                y = torch.empty(B, cout, H, W, device=dev)
                t_o = timed(lambda: _capi.conv3x3(x, packed, cout, out=y))
                line += f" | ours {t_o:8.1f} us {flop/t_o/1e6:6.1f} TF/s  x{t_m/t_o:.2f}"
            print(line, flush=True)


if __name__ == "__main__":
    main()
