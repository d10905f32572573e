"""CPU emulation of the split-precision conv arithmetic on the ResNet-50 / CIFAR-100 config-4
parity case: which operand split keeps EL2N within 1e-3 of exact?

Every conv of the oracle forward (train-mode BN) is replaced by an emulation of the MFMA form:
operands split into two 16-bit halves v = hi + lo, products hi*hi + hi*lo + lo*hi (each exact
in fp32) accumulated in fp32.  Modes:
  fp32        plain fp32 conv (the reference's arithmetic)
  bf16x3      the kernels' current split (bf16 hi/lo)
  bf16x4      + lo*lo
  f16x3       fp16 hi/lo, no scaling (lo of small weights is subnormal)
  f16x3s      fp16 hi/lo with each layer's weights scaled by a power of two so max|w| ~ 2^13
              (exact; undone on the fp32 result)
Errors are relative to a float64 forward of the same network.

    python tools/emulate_split.py [n] [json_out]
"""
import json
import math
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from data_diet_distributed_amd import synthetic  # noqa: E402
from oracle import pipeline as o_pipe  # noqa: E402
from oracle import resnet_fn  # noqa: E402

_conv = F.conv2d


def _split(x, dt):
    h = x.to(dt).float()
    return h, (x - h).to(dt).float()


def make_conv(mode):
    def conv(inp, w, b=None, stride=1, padding=0, *a, **kw):
        if mode == "fp32" or inp.dtype == torch.float64:
            return _conv(inp, w, b, stride, padding)
        scale = 1.0
        if mode == "f16x3s":
            scale = 2.0 ** (13 - math.ceil(math.log2(float(w.abs().max()))))
        dt = torch.bfloat16 if mode.startswith("bf16") else torch.float16
        ah, al = _split(inp, dt)
        wh, wl = _split(w * scale, dt)
        y = _conv(ah, wh, None, stride, padding) + _conv(ah, wl, None, stride, padding) \
            + _conv(al, wh, None, stride, padding)
        if mode == "bf16x4":
            y = y + _conv(al, wl, None, stride, padding)
        return y / scale if scale != 1.0 else y
    return conv


def el2n(sd, x, y, dtype=torch.float32):
    if dtype == torch.float64:
        sd = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
        x = x.double()
    logits = resnet_fn.forward(sd, x, bn="batch")
    e = F.softmax(logits, dim=1) - F.one_hot(y, logits.shape[1])
    return e.norm(dim=1).double().numpy()


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    torch.set_num_threads(os.cpu_count())
    images, labels = synthetic.make_images(512, 100, seed=41)
    sd = synthetic.make_checkpoint("resnet50", 100, seed=5)["net"]
    x = o_pipe.normalize(images[:n])
    y = torch.from_numpy(labels[:n].astype(np.int64))
    with torch.no_grad():
        ref = el2n(sd, x, y, torch.float64)
        rep = {}
        for mode in ("fp32", "bf16x3", "bf16x4", "f16x3", "f16x3s"):
            F.conv2d = make_conv(mode)
            try:
                got = el2n(sd, x, y)
            finally:
                F.conv2d = _conv
            err = np.abs(got / ref - 1)
            rep[mode] = {"max_rel": float(err.max()), "argmax": int(err.argmax()),
                         "p99": float(np.percentile(err, 99)), "median": float(np.median(err))}
            print(mode, json.dumps(rep[mode]), flush=True)
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            json.dump(rep, f, indent=1)


if __name__ == "__main__":
    main()
