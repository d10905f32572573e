"""CPU emulation of the split-precision arithmetic on GraNd (ResNet-18 / CIFAR-10, eval BN):
forward convs, backward-data convs and the per-example weight-gradient products all in the
split form (hi*hi + hi*lo + lo*hi, each exact in fp32, fp32 sums), against the float64
oracle.  Modes as tools/emulate_split.py; "+ls" scales the backward seed e by 2^10 (a power
of two: exact) and the squared norms back by 2^-20, so small gradients stay clear of fp16's
subnormal range.

    python tools/emulate_split_grand.py [n] [arch] [json_out]
"""
import json
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
# operand halves per stage: forward convs, backward-data convs, per-example weight-gradient
# products (None: plain fp32)
MODE = {"dt": None, "fwd": None, "bwd": None, "pw": None}


def _split(x, dt=None):
    dt = dt or MODE["dt"]
    h = x.to(dt).float()
    return h, (x - h).to(dt).float()


def _sconv(a, w, stride, pad):
    if MODE["fwd"] is None:
        return _conv(a, w, None, stride, pad)
    ah, al = _split(a, MODE["fwd"])
    sc = 1.0
    if MODE.get("wscale"):  # the weights scaled by a power of two to max |w| ~ 2^13 (exact)
        import math
        sc = 2.0 ** (13 - math.ceil(math.log2(float(w.abs().max()))))
    wh, wl = _split(w * sc, MODE["fwd"])
    if sc != 1.0:
        return (_conv(ah, wh, None, stride, pad) + _conv(ah, wl, None, stride, pad)
                + _conv(al, wh, None, stride, pad)) / sc
    return (_conv(ah, wh, None, stride, pad) + _conv(ah, wl, None, stride, pad)
            + _conv(al, wh, None, stride, pad))


class SplitConv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, inp, w, stride, pad):
        ctx.save_for_backward(w)
        ctx.cfg = (inp.shape, stride, pad)
        return _sconv(inp, w, stride, pad)

    @staticmethod
    def backward(ctx, g):
        (w,) = ctx.saved_tensors
        shape, stride, pad = ctx.cfg
        ci = torch.nn.grad.conv2d_input
        if MODE["bwd"] is None:
            return ci(shape, w, g, stride, pad), None, None, None
        gh, gl = _split(g, MODE["bwd"])
        wh, wl = _split(w, MODE["bwd"])
        gi = (ci(shape, wh, gh, stride, pad) + ci(shape, wl, gh, stride, pad)
              + ci(shape, wh, gl, stride, pad))
        return gi, None, None, None


def conv(inp, w, b=None, stride=1, padding=0, *a, **kw):
    return SplitConv.apply(inp, w, stride, padding)


def grand(sd, images, labels, ls):
    x = o_pipe.normalize(images).requires_grad_(True)
    y = torch.from_numpy(np.asarray(labels, dtype=np.int64))
    tape = []
    logits = resnet_fn.forward(sd, x, bn="running", tape=tape)
    # e without the p_y - 1 cancellation (as dd_el2n emits it: e_y = -sum_{j != y} p_j)
    e = (F.softmax(logits.double(), dim=1) - F.one_hot(y, logits.shape[1])).float().detach()
    if ls == "pe":  # per example: max |e_i| scaled to 2^8 (a power of two per row)
        scale = 2.0 ** (8 - torch.ceil(torch.log2(e.abs().amax(1).double().clamp_min(1e-300))))
        scale = scale.float()[:, None]
    else:
        scale = torch.tensor(2.0 ** 10 if ls else 1.0)
    grads = torch.autograd.grad(logits, [t[2] for t in tape], grad_outputs=e * scale)
    scale = scale.double().reshape(-1)
    sq = torch.zeros(len(labels), dtype=torch.float64)
    with torch.no_grad():
        for (key, inp, _o, stride, pad), g in zip(tape, grads):
            if stride is None:
                sq += inp.double().pow(2).sum(1) * g.double().pow(2).sum(1) + g.double().pow(2).sum(1)
                continue
            w = sd[key]
            U = F.unfold(inp, w.shape[2:], padding=pad, stride=stride)
            G = g.reshape(g.shape[0], g.shape[1], -1)
            if MODE["pw"] is None:
                pw = torch.bmm(G, U.transpose(1, 2))
            else:
                Uh, Ul = _split(U, MODE["pw"])
                Gh, Gl = _split(G, MODE["pw"])
                pw = (torch.bmm(Gh, Uh.transpose(1, 2)) + torch.bmm(Gh, Ul.transpose(1, 2))
                      + torch.bmm(Gl, Uh.transpose(1, 2)))
            sq += pw.double().pow(2).sum((1, 2))
    return (sq / scale ** 2).sqrt().numpy()


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    arch = sys.argv[2] if len(sys.argv) > 2 else "resnet18"
    nc = 10 if arch == "resnet18" else 100
    torch.set_num_threads(os.cpu_count())
    images, labels = synthetic.make_images(n, nc, seed=5)
    sd = synthetic.make_checkpoint(arch, nc, seed=1)["net"]
    ref = o_pipe.grand_scores(sd, images, labels, batch_size=n, dtype=torch.float64)
    F.conv2d = conv
    rep = {}
    try:
        bf, hf = torch.bfloat16, torch.float16
        for name, fwd, bwd, pw, ls in (("fp32", None, None, None, False),
                                       ("bf16x3", bf, bf, bf, False),
                                       ("fwd_only_bf16", bf, None, None, False),
                                       ("bwd_only_bf16", None, bf, None, False),
                                       ("pw_only_bf16", None, None, bf, False),
                                       ("fwd_f16_rest_bf16", hf, bf, bf, False),
                                       ("fwd_f16_bwd_bf16_pw_fp32", hf, bf, None, False),
                                       ("f16x3+pe", hf, hf, hf, "pe"),
                                       ("fwd_f16_scaled_rest_bf16", hf, bf, bf, "ws")):
            MODE.update(dt=bf, fwd=fwd, bwd=bwd, pw=pw, wscale=ls == "ws")
            ls = ls if ls != "ws" else False
            F.conv2d = conv if fwd is not None or bwd is not None else _conv
            got = grand(sd, images, labels, ls)
            err = np.abs(got / ref - 1)
            rep[name] = {"max_rel": float(err.max()), "argmax": int(err.argmax()),
                         "p99": float(np.percentile(err, 99)), "median": float(np.median(err))}
            print(name, json.dumps(rep[name]), flush=True)
    finally:
        F.conv2d = _conv
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as f:
            json.dump(rep, f, indent=1)


if __name__ == "__main__":
    main()
