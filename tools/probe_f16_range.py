"""Probe: what the fp16-halves split does with activations past fp16's range (65504).

Runs dd_conv3x3_forward with an f16x3 pack on inputs holding a few large values (1e5, 2e5,
1e6, 1e7, -3e5) and compares with a float64 conv: prints, per magnitude, whether the outputs
that read it are finite and their relative error."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from data_diet_distributed_amd import _capi  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(0)
w = torch.randn(64, 64, 3, 3, generator=g) / 24
pk = _capi.conv3x3_pack(w.to(dev), operands="f16x3")
for big in (6e4, 1e5, 1.3e5, 2e5, 1e6, 1e7, -3e5):
    x = torch.randn(2, 64, 16, 16, generator=g)
    x[0, 5, 7, 7] = big
    want = F.conv2d(x.double(), w.double(), padding=1)
    got = _capi.conv3x3(x.to(dev), pk, 64).double().cpu()
    near = (slice(0, 1), slice(None), slice(6, 9), slice(6, 9))
    fin = bool(torch.isfinite(got[near]).all())
    err = float(((got[near] - want[near]).abs() / want[near].abs().clamp_min(1e-3)).max())
    print(f"input {big:10.3g}: outputs finite {fin}, max rel err {err:.3g}", flush=True)
