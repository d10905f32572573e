"""ORACLE (test infrastructure): functional ResNet forward over a state_dict, torch CPU fp32.

Restates reference models/resnet.py:7-97 directly against the checkpoint keys (no nn.Module),
so it is independent of the product's module code:
  stem  conv1 3x3/1 pad 1 -> bn1 -> relu                              (:71-72, :89)
  BasicBlock  relu(bn1(conv1)) -> bn2(conv2) + shortcut -> relu        (:27-32)
  Bottleneck  relu(bn1(conv1)) -> relu(bn2(conv2)) -> bn3(conv3) + sc  (:57-63)
  shortcut    1x1 conv(stride) + bn when present                       (:20-25, :49-54)
  head        avg_pool2d(4) -> view -> linear                          (:94-96)
The ImageNet stem (7x7/2 + 3x3/2 maxpool, adaptive pool) is the build's extension for
configs the reference cannot run.
BN mode "batch" = train-mode batch statistics (the reference never calls .eval(),
train.py:59-63); "running" = eval mode.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

EPS = 1e-5  # nn.BatchNorm2d default


def _bn_fn(sd, p, x, mode):
    if mode == "batch":
        return F.batch_norm(x, None, None, sd[p + ".weight"], sd[p + ".bias"], True, 0.0, EPS)
    return F.batch_norm(x, sd[p + ".running_mean"], sd[p + ".running_var"], sd[p + ".weight"],
                        sd[p + ".bias"], False, 0.0, EPS)


def _blocks(sd):
    for li in range(1, 5):
        bi = 0
        while f"layer{li}.{bi}.conv1.weight" in sd:
            yield li, bi, f"layer{li}.{bi}"
            bi += 1


def gate_flip(rel: float, near_count=None):
    """A ReLU that flips its gate wherever the pre-activation z lies within `rel` of zero,
    relative to the RMS of z over that example's tensor: out = z * mask with the mask inverted
    there, so the backward follows the flipped gate (the forward value moves by < rel * rms).
    This is the other side of a gate that rounding can put either way: a GPU path whose fp32
    pre-activation error is of that size may legitimately take it (tests/test_gpu_pipeline.py,
    the GraNd cross-checks).  near_count (tensor [B]) receives the number of such gates."""
    def relu(z):
        rms = z.detach().pow(2).flatten(1).mean(1).sqrt().clamp_min(1e-30)
        near = z.detach().abs() < rel * rms.view(-1, *([1] * (z.dim() - 1)))
        if near_count is not None:
            near_count.add_(near.flatten(1).sum(1).to(near_count.dtype))
        mask = (z.detach() > 0) ^ near
        return z * mask.to(z.dtype)
    return relu


def forward(sd: dict, x: torch.Tensor, bn: str = "batch", stem: str = "cifar", tape=None,
            bn_tape=None, relu=F.relu):
    """Logits of the ResNet whose weights are `sd`.  `tape` (list) receives
    (weight_key, input, output, stride, pad) for every conv and the linear layer; `bn_tape`
    receives (bn_prefix, output) for every BatchNorm; `relu` replaces every ReLU (gate_flip)."""

    def _bn(sd, p, x, mode):
        out = _bn_fn(sd, p, x, mode)
        if bn_tape is not None:
            bn_tape.append((p, out))
        return out

    def conv(key, inp, stride, pad):
        out = F.conv2d(inp, sd[key], None, stride, pad)
        if tape is not None:
            tape.append((key, inp, out, stride, pad))
        return out

    if stem == "cifar":
        out = relu(_bn(sd, "bn1", conv("conv1.weight", x, 1, 1), bn))
    else:
        out = relu(_bn(sd, "bn1", conv("conv1.weight", x, 2, 3), bn))
        out = F.max_pool2d(out, 3, 2, 1)
    bottleneck = "layer1.0.conv3.weight" in sd
    for li, bi, p in _blocks(sd):
        s = 2 if (li > 1 and bi == 0) else 1
        inp = out
        if bottleneck:
            o = relu(_bn(sd, p + ".bn1", conv(p + ".conv1.weight", inp, 1, 0), bn))
            o = relu(_bn(sd, p + ".bn2", conv(p + ".conv2.weight", o, s, 1), bn))
            o = _bn(sd, p + ".bn3", conv(p + ".conv3.weight", o, 1, 0), bn)
        else:
            o = relu(_bn(sd, p + ".bn1", conv(p + ".conv1.weight", inp, s, 1), bn))
            o = _bn(sd, p + ".bn2", conv(p + ".conv2.weight", o, 1, 1), bn)
        if p + ".shortcut.0.weight" in sd:
            sc = _bn(sd, p + ".shortcut.1", conv(p + ".shortcut.0.weight", inp, s, 0), bn)
        else:
            sc = inp
        out = relu(o + sc)
    out = F.avg_pool2d(out, 4) if stem == "cifar" else F.adaptive_avg_pool2d(out, 1)
    feat = out.reshape(out.size(0), -1)
    logits = F.linear(feat, sd["linear.weight"], sd["linear.bias"])
    if tape is not None:
        tape.append(("linear.weight", feat, logits, None, None))
    return logits
