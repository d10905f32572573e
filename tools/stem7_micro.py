"""The ImageNet stem's EL2N launch (B = 512, 128-example BN groups, fp16 halves): dd_stem7_forward
against the implicit GEMM (dd_conv_gemm_forward dense mode) on the same input."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from data_diet_distributed_amd import _capi  # noqa: E402


def timed(fn, iters=10):
    for _ in range(2):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


dev = torch.device("cuda:0")
B, gs = 512, 128
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(B, 3, 224, 224, device=dev, generator=g)
w = torch.randn(64, 3, 7, 7, device=dev, generator=g) / 12
fl = 2.0 * B * 112 * 112 * 147 * 64
pg = _capi.conv_gemm_pack(w, operands="f16x3")
t = timed(lambda: _capi.conv_gemm(x, pg, 64, 7, 2, 3, group_size=gs, stats=True))
print(f"conv_gemm 7x7/2 {t:8.1f} us {fl / t / 1e6:6.1f} TF/s {fl / t / 1e6 / 833.3:.3f}")
p7 = _capi.stem7_pack(w, operands="f16x3")
t7 = timed(lambda: _capi.stem7(x, p7, 64, gs))
print(f"stem7     7x7/2 {t7:8.1f} us {fl / t7 / 1e6:6.1f} TF/s {fl / t7 / 1e6 / 833.3:.3f}")
y1, _ = _capi.conv_gemm(x, pg, 64, 7, 2, 3, group_size=gs, stats=True)
y2, _ = _capi.stem7(x, p7, 64, gs)
print("max |stem7 - conv_gemm| / max|y|", ((y1 - y2).abs().max() / y1.abs().max()).item())
