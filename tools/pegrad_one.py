"""One GraNd 3x3 norm shape in its own process (the library named by DD_LIB), for per-kernel
PMC / trace passes: python tools/pegrad_one.py [cin H cout stride] [iters]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from data_diet_distributed_amd import _capi  # noqa: E402


def main():
    a = [int(v) for v in sys.argv[1:]] or [64, 32, 64, 1]
    cin, H, cout, s = a[:4]
    iters = a[4] if len(a) > 4 else 30
    B = 1024
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    act = torch.relu(torch.randn(B, cin, H, H, device=dev, generator=g))
    gout = torch.randn(B, cout, H // s, H // s, device=dev, generator=g) * 1e-2
    geom = _capi.conv_geom(act, gout, (3, 3), s, 1)
    ws = torch.empty(max(_capi.conv_workspace_bytes(geom, "auto", "bf16x3"), 4),
                     dtype=torch.uint8, device=dev)
    sq = torch.zeros(B, device=dev)
    for _ in range(iters):
        _capi.conv_pegrad_sqnorm(act, gout, (3, 3), s, 1, sq, ws, method="auto",
                                 precision="bf16x3")
    torch.cuda.synchronize()
    print("sq[0]", sq[0].item(), flush=True)


if __name__ == "__main__":
    main()
