"""ORACLE (test infrastructure): the whole Data Diet scoring path on CPU (torch CPU fp32).

Restates reference get_scores_and_prune.py:8-34 under the build's parity protocol
(SURVEY §8.0): the dataset is visited unshuffled in fixed batches [b*B, (b+1)*B), so
train-mode-BN scores are well defined; per example, EL2N = ||softmax(f(x)) - onehot(y)||
(:16-18); K checkpoints are averaged; the keep-set is the stable descending top-k (:22-24).
GraNd (north star) uses eval-mode BN and the per-layer hook formulation, validated against
torch.func per-sample gradients in `grand_vmap`.

Also the timed CPU baseline of bench.py ("kind": "port").
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from . import el2n as _el2n
from . import pegrad as _pegrad
from . import resnet_fn

MEAN = (0.4914, 0.4822, 0.4465)  # data/loader.py:10
STD = (0.2023, 0.1994, 0.2010)


def normalize(images_u8: np.ndarray) -> torch.Tensor:
    """ToTensor + Normalize (data/loader.py:8-11): /255 then (x - mean) / std, fp32."""
    x = torch.from_numpy(np.ascontiguousarray(images_u8)).to(torch.float32).div(255)
    m = torch.tensor(MEAN, dtype=torch.float32)[:, None, None]
    s = torch.tensor(STD, dtype=torch.float32)[:, None, None]
    return x.sub(m).div(s)


def el2n_scores(sd, images_u8, labels, batch_size=128, stem="cifar", bn="batch"):
    """Per-example EL2N over the pinned batch partition (get_scores_and_prune.py:11-20)."""
    n = len(labels)
    out = np.empty(n, dtype=np.float32)
    with torch.no_grad():
        for lo in range(0, n, batch_size):
            hi = min(n, lo + batch_size)
            x = normalize(images_u8[lo:hi])
            y = torch.from_numpy(np.asarray(labels[lo:hi], dtype=np.int64))
            logits = resnet_fn.forward(sd, x, bn=bn, stem=stem)
            C = logits.shape[1]
            e = F.softmax(logits, dim=1) - F.one_hot(y, num_classes=C)
            out[lo:hi] = e.norm(dim=1, p=2).numpy()
    return out


def grand_scores(sd, images_u8, labels, batch_size=64, stem="cifar", params="conv_linear",
                 dtype=torch.float32, flip_rel=None, near_gates=None):
    """Per-example ||grad_W CE|| with eval-mode BN via the hook (tape) formulation:
    conv: ||unfold(a)^T g||_F^2 per example; linear: ||a||^2 ||e||^2 + ||e||^2 (bias);
    params="all" adds every BN's gamma / beta: (sum_t g xhat)^2 + (sum_t g)^2 per channel.

    dtype=torch.float64 runs forward and backward in double: the parity oracle.  In fp32 the
    computation is itself unstable on random-init checkpoints (measured: up to 35 % relative
    on near-zero scores, where p_y - 1 cancels, and 0.2 % on a large score whose ReLU
    pattern flips under CPU-conv rounding), so fp32 is only the timed CPU baseline.

    flip_rel: every ReLU gate whose pre-activation lies within flip_rel of zero (relative to
    that example's RMS of the tensor) is flipped (resnet_fn.gate_flip): the score a path takes
    when its rounding puts those gates on the other side.  near_gates (ndarray [n], int64)
    receives the number of such gates per example."""
    n = len(labels)
    out = np.empty(n, dtype=np.float32)
    if dtype != torch.float32:
        sd = {k: (v.to(dtype) if v.is_floating_point() else v) for k, v in sd.items()}
    for lo in range(0, n, batch_size):
        hi = min(n, lo + batch_size)
        x = normalize(images_u8[lo:hi]).to(dtype).requires_grad_(True)
        y = torch.from_numpy(np.asarray(labels[lo:hi], dtype=np.int64))
        tape = []
        bn_tape = [] if params == "all" else None
        cnt = torch.zeros(hi - lo, dtype=torch.int64)
        relu = F.relu if flip_rel is None else resnet_fn.gate_flip(flip_rel, cnt)
        logits = resnet_fn.forward(sd, x, bn="running", stem=stem, tape=tape, bn_tape=bn_tape,
                                   relu=relu)
        if near_gates is not None:
            near_gates[lo:hi] = cnt.numpy()
        e = (F.softmax(logits, dim=1) - F.one_hot(y, logits.shape[1])).detach()
        outs = [t[2] for t in tape] + [t[1] for t in bn_tape or ()]
        grads = torch.autograd.grad(logits, outs, grad_outputs=e)
        bn_grads = grads[len(tape):]
        grads = grads[:len(tape)]
        sq = torch.zeros(hi - lo, dtype=torch.float64)
        for (p, bn_out), g in zip(bn_tape or (), bn_grads):
            sq += torch.from_numpy(_pegrad.bn_pegrad_sqnorm(
                bn_out.detach().numpy(), g.numpy(), sd[p + ".weight"].numpy(),
                sd[p + ".bias"].numpy()))
        with torch.no_grad():
            for (key, inp, _o, stride, pad), g in zip(tape, grads):
                if stride is None:  # linear
                    a2 = inp.double().pow(2).sum(1)
                    g2 = g.double().pow(2).sum(1)
                    sq += a2 * g2 + g2
                    continue
                w = sd[key]
                U = F.unfold(inp.double(), w.shape[2:], padding=pad, stride=stride)  # B,da,T
                G = g.double().reshape(g.shape[0], g.shape[1], -1)  # B,dg,T
                pw = torch.bmm(G, U.transpose(1, 2))
                sq += pw.pow(2).sum((1, 2))
        out[lo:hi] = sq.sqrt().numpy()
    return out


def grand_vmap(sd, images_u8, labels, stem="cifar", chunk=8, params="conv_linear",
               dtype=torch.float32):
    """GraNd by definition: torch.func per-sample gradients of CE (eval BN) w.r.t. every
    Conv2d/Linear weight (+ Linear bias), and with params="all" every BN weight / bias; the
    oracle of the oracle (small N only)."""
    from torch.func import functional_call, grad, vmap  # noqa: F401

    if dtype != torch.float32:
        sd = {k: (v.to(dtype) if v.is_floating_point() else v) for k, v in sd.items()}
    keys = [k for k in sd if (k.endswith(".weight") and sd[k].dim() == 4) or k.startswith("linear.")]
    if params == "all":
        bns = [k[:-len(".running_mean")] for k in sd if k.endswith(".running_mean")]
        keys += [p + s for p in bns for s in (".weight", ".bias")]
    rest = {k: v for k, v in sd.items() if k not in keys}

    def loss(p, x, y):
        full = dict(rest)
        full.update(p)
        logits = resnet_fn.forward(full, x[None], bn="running", stem=stem)
        return F.cross_entropy(logits, y[None], reduction="sum")

    pvals = {k: sd[k] for k in keys}
    n = len(labels)
    out = np.empty(n, dtype=np.float64)
    g = vmap(grad(loss), in_dims=(None, 0, 0))
    for lo in range(0, n, chunk):
        hi = min(n, lo + chunk)
        x = normalize(images_u8[lo:hi]).to(dtype)
        y = torch.from_numpy(np.asarray(labels[lo:hi], dtype=np.int64))
        grads = g(pvals, x, y)
        tot = sum(v.double().pow(2).reshape(hi - lo, -1).sum(1) for v in grads.values())
        out[lo:hi] = tot.sqrt().numpy()
    return out


def score_pipeline(ckpts, images_u8, labels, sparsity, methods=("el2n",), select_by="el2n",
                   batch_size=128, grand_batch=64, stem="cifar"):
    """K-checkpoint ensemble + keep-set: returns (scores dict, kept indices, k)."""
    n = len(labels)
    scores = {}
    for m in methods:
        acc = np.zeros(n, dtype=np.float32)
        for sd in ckpts:
            if m == "el2n":
                acc += el2n_scores(sd, images_u8, labels, batch_size, stem)
            elif m == "grand":
                acc += grand_scores(sd, images_u8, labels, grand_batch, stem)
            else:
                raise ValueError(m)
        K = len(ckpts)
        scores[m] = acc if K == 1 else (acc / np.float32(K)).astype(np.float32)
    k = _el2n.keep_count(n, sparsity)
    kept = _el2n.stable_topk(scores[select_by], k)
    return scores, kept, k
