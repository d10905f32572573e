"""ResNet backbones for Data Diet scoring, state_dict-compatible with the reference.

Mirrors `models/resnet.py` of the reference (BasicBlock :7-32, Bottleneck :35-63,
ResNet :66-97, factories :100-117): same module names, so a reference checkpoint's
`state_dict` (122 keys for ResNet-18) loads unchanged, and `ResNet18()` etc. build the
same network.  Two additions the scoring engine needs:

* `num_classes` and `stem` arguments (the reference hard-codes 10 classes and the CIFAR
  3x3 stem + `avg_pool2d(out, 4)` at :94, which cannot run at 224x224).
* `run(x, bn=..., tape=...)`: the forward with an explicit BatchNorm mode and an optional
  tape that records every Conv2d / Linear (input, output) pair.  The GraNd path uses the
  tape in place of per-module hooks: the recorded outputs are the autograd nodes whose
  gradients feed the per-example gradient-norm kernels.

`bn="batch"` reproduces the reference's scoring semantics (the net is never put in eval
mode, `train.py:59-63`, so BN uses batch statistics) without mutating running stats;
`bn="running"` is eval-mode BN (per-example independent, required for GraNd).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


class _Unit:
    """Marker base for residual blocks: children are addressed by reference names."""


class BasicBlock(nn.Module, _Unit):
    """Two 3x3 convs + identity/1x1 shortcut (reference `models/resnet.py:7-32`)."""

    expansion = 1

    def __init__(self, in_planes, planes, stride=1):
        super().__init__()
        self.conv1 = nn.Conv2d(in_planes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride=1, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.shortcut = _shortcut(in_planes, planes * self.expansion, stride)

    def chain(self):
        # (conv, bn, relu-after?) in forward order; the last bn is added to the shortcut
        return [(self.conv1, self.bn1, True), (self.conv2, self.bn2, False)]


class Bottleneck(nn.Module, _Unit):
    """1x1 -> 3x3(stride) -> 1x1(x4) + shortcut (reference `models/resnet.py:35-63`)."""

    expansion = 4

    def __init__(self, in_planes, planes, stride=1):
        super().__init__()
        self.conv1 = nn.Conv2d(in_planes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * self.expansion, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * self.expansion)
        self.shortcut = _shortcut(in_planes, planes * self.expansion, stride)

    def chain(self):
        return [(self.conv1, self.bn1, True), (self.conv2, self.bn2, True),
                (self.conv3, self.bn3, False)]


def _shortcut(in_planes, out_planes, stride):
    # reference :20-25 / :49-54: projection only when the shape changes
    if stride != 1 or in_planes != out_planes:
        return nn.Sequential(nn.Conv2d(in_planes, out_planes, 1, stride=stride, bias=False),
                             nn.BatchNorm2d(out_planes))
    return nn.Sequential()


def _bn_groups(x, bn: nn.BatchNorm2d, group: int, n_valid=None):
    """Train-mode BN over each group of `group` consecutive rows (the pinned partition's
    batches), in fp32 torch ops; rows at or past `n_valid` (the ragged last batch's padding)
    are left out of the last group's statistics."""
    G = x.shape[0] // group
    xv = x.reshape(G, group, *x.shape[1:])
    nv = x.shape[0] if n_valid is None else int(n_valid)
    full = min(G, nv // group)  # groups whose rows are all valid
    means, vars_ = [], []
    if full:
        means.append(xv[:full].mean(dim=(1, 3, 4)))
        vars_.append(xv[:full].var(dim=(1, 3, 4), unbiased=False))
    for g in range(full, G):
        rows = xv[g, :max(1, min(group, nv - g * group))]
        means.append(rows.mean(dim=(0, 2, 3))[None])
        vars_.append(rows.var(dim=(0, 2, 3), unbiased=False)[None])
    mean, var = torch.cat(means), torch.cat(vars_)
    scale = torch.rsqrt(var + bn.eps) * bn.weight
    out = (xv - mean[:, None, :, None, None]) * scale[:, None, :, None, None] + \
        bn.bias[None, None, :, None, None]
    return out.reshape(x.shape)


def _bn(x, bn: nn.BatchNorm2d, mode: str, n_valid=None, group=None):
    if mode == "groups":
        return _bn_groups(x, bn, group, n_valid)
    if mode == "batch":
        if n_valid is not None and n_valid < x.shape[0]:
            # batch statistics over the first n_valid rows only: a ragged final batch padded
            # to the full batch size normalises exactly as the unpadded batch would
            xv = x[:n_valid]
            mean = xv.mean(dim=(0, 2, 3))
            var = xv.var(dim=(0, 2, 3), unbiased=False)
            scale = torch.rsqrt(var + bn.eps) * bn.weight
            return (x - mean[None, :, None, None]) * scale[None, :, None, None] + \
                bn.bias[None, :, None, None]
        # batch statistics, running stats untouched (outputs equal the reference's
        # train-mode forward; the reference's running-stat mutation is a side effect only)
        return F.batch_norm(x, None, None, bn.weight, bn.bias, True, 0.0, bn.eps)
    if mode == "running":
        return F.batch_norm(x, bn.running_mean, bn.running_var, bn.weight, bn.bias,
                            False, 0.0, bn.eps)
    if mode == "module":
        return bn(x)
    raise ValueError(f"unknown bn mode {mode!r}")


class ResNet(nn.Module):
    """ResNet over CIFAR (3x3 stem, `avg_pool2d(4)`) or ImageNet (7x7/2 + maxpool) inputs.

    Reference `models/resnet.py:66-97`; `stem="cifar"` is the reference network.
    """

    def __init__(self, block, num_blocks, num_classes=10, stem="cifar"):
        super().__init__()
        if stem not in ("cifar", "imagenet"):
            raise ValueError(f"unknown stem {stem!r}")
        self.stem = stem
        self.in_planes = 64
        if stem == "cifar":
            self.conv1 = nn.Conv2d(3, 64, 3, stride=1, padding=1, bias=False)
        else:
            self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.layer1 = self._make_layer(block, 64, num_blocks[0], 1)
        self.layer2 = self._make_layer(block, 128, num_blocks[1], 2)
        self.layer3 = self._make_layer(block, 256, num_blocks[2], 2)
        self.layer4 = self._make_layer(block, 512, num_blocks[3], 2)
        self.linear = nn.Linear(512 * block.expansion, num_classes)

    def _make_layer(self, block, planes, n, stride):
        blocks = []
        for s in [stride] + [1] * (n - 1):
            blocks.append(block(self.in_planes, planes, s))
            self.in_planes = planes * block.expansion
        return nn.Sequential(*blocks)

    def blocks(self):
        for layer in (self.layer1, self.layer2, self.layer3, self.layer4):
            yield from layer

    def forward(self, x):
        # nn.Module semantics exactly as the reference: BN follows self.training
        return self.run(x, bn="module")

    def conv_bn_pairs(self):
        """Every (Conv2d, BatchNorm2d) pair in forward order."""
        yield self.conv1, self.bn1
        for blk in self.blocks():
            for c, b, _ in blk.chain():
                yield c, b
            if len(blk.shortcut) > 0:
                yield blk.shortcut[0], blk.shortcut[1]

    @torch.no_grad()
    def gemm_pack(self, conv):
        """The dd_conv_gemm_pack of a kh x kw conv's current weights (cached per conv; EL2N
        forward only, so in the raw packs' operand halves)."""
        from . import _capi
        key = (conv, False)
        if key not in self._gemm:
            self._gemm[key] = _capi.conv_gemm_pack(conv.weight.detach().float().contiguous(),
                                                   operands=self._raw_operands)
        return self._gemm[key]

    def stem7_pack(self, conv):
        """The dd_stem7_pack of the ImageNet stem conv's current weights (cached; EL2N forward
        only, in the raw packs' operand halves)."""
        from . import _capi
        key = (conv, "stem7")
        if key not in self._gemm:
            self._gemm[key] = _capi.stem7_pack(conv.weight.detach().float().contiguous(),
                                               operands=self._raw_operands)
        return self._gemm[key]

    @torch.no_grad()
    def prepare_fast_convs(self, raw_operands: str = "f16x3", folded_operands: str = "f16x3"):
        """Pack the conv weights (raw, and folded if fold_bn() ran) for the split MFMA conv
        kernels; `run(..., fast=True)` then uses them wherever the shape is supported.
        raw_operands / folded_operands: the operand halves of the raw weights' forward packs
        (the EL2N forward, batch-normalised activations) and of the BN-folded ones (the GraNd
        forward) -- "f16x3" (default: ~2^-22 relative per product, the weights scaled by a
        power of two) or "bf16x3"; the backward-data packs are bf16x3 (gradients span many
        octaves below fp16's normal range)."""
        from .fastconv import Down3Packs, DownPacks, Packs, Packs1x1
        self._raw_operands = raw_operands
        ro, fo = raw_operands, folded_operands
        self._packs = {}
        self._packs1 = {}   # 1x1 convs (Bottleneck conv1 / conv3, projections)
        self._down3 = {}    # stride-2 3x3 convs outside a BasicBlock head (Bottleneck conv2)
        folded = getattr(self, "_folded", None)
        for c, _ in self.conv_bn_pairs():
            if c.kernel_size == (3, 3) and c.stride == (1, 1) and c.padding == (1, 1):
                self._packs[(c, False)] = Packs(c.weight, ro)
                if folded and c in folded:
                    self._packs[(c, True)] = Packs(folded[c][0], fo)
            elif c.kernel_size == (1, 1) and c.padding == (0, 0) and c.stride[0] in (1, 2):
                self._packs1[(c, False)] = Packs1x1(c.weight, ro)
                if folded and c in folded:
                    self._packs1[(c, True)] = Packs1x1(folded[c][0], fo)
        # every other kh x kw conv (the 7x7 ImageNet stem, 3x3 at widths the 3x3 / down kernels
        # do not take) runs on the implicit-GEMM kernel, forward (EL2N) only; its packs are
        # made on first use (gemm_pack), so networks that never need them pay nothing
        self._gemm = {}
        for blk in self.blocks():
            if isinstance(blk, Bottleneck) and blk.conv2.stride == (2, 2):
                c2 = blk.conv2
                self._down3[(c2, False)] = Down3Packs(c2.weight, ro)
                if folded and c2 in folded:
                    self._down3[(c2, True)] = Down3Packs(folded[c2][0], fo)
        # downsampling heads: BasicBlock conv1 3x3/2 + its 1x1/2 projection (one kernel)
        self._down = {}
        for blk in self.blocks():
            if (isinstance(blk, BasicBlock) and blk.conv1.stride == (2, 2)
                    and blk.conv1.padding == (1, 1) and len(blk.shortcut) > 0
                    and blk.shortcut[0].kernel_size == (1, 1)
                    and blk.shortcut[0].stride == (2, 2)):
                c1, sc = blk.conv1, blk.shortcut[0]
                self._down[(blk, False)] = DownPacks(c1.weight, sc.weight, ro)
                if folded and c1 in folded and sc in folded:
                    self._down[(blk, True)] = DownPacks(folded[c1][0], folded[sc][0], fo)

    @torch.no_grad()
    def fold_bn(self):
        """Precompute eval-mode BN folded into each conv: W' = W*s, b' = beta - mean*s with
        s = gamma / sqrt(running_var + eps).  Stored outside the state_dict; call again
        after loading new weights.  `run(bn="folded")` uses it."""
        self._folded = {}
        for c, b in self.conv_bn_pairs():
            s = b.weight / torch.sqrt(b.running_var + b.eps)
            w = (c.weight * s[:, None, None, None]).contiguous()
            bias = (b.bias - b.running_mean * s).contiguous()
            self._folded[c] = (w, bias, s.contiguous())

    def run(self, x, bn="module", tape=None, n_valid=None, fast=False, group=None):
        """Forward with explicit BN mode.

        bn: "module" (nn semantics), "batch" (batch stats; `n_valid` masks padded rows out
        of the statistics), "groups" (batch stats per `group` consecutive rows, fp32 torch ops
        on MIOpen convs: many pinned batches per launch), "running" (eval), "folded" (eval
        with BN folded into the convs).
        `tape` receives (module, input, output, col_scale) per Conv2d and for the Linear;
        col_scale is the folded BN scale s (the raw conv's output gradient is s * d/d out).
        """

        packs = getattr(self, "_packs", None) if fast else None
        if fast:
            from . import fastconv

        def conv_bn(c, b, inp):
            if bn == "folded":
                w, bias, s = self._folded[c]
                pk = packs.get((c, True)) if packs else None
                if pk is not None and fastconv.supported(c, inp):
                    out = fastconv.conv3x3(inp, pk, bias)
                else:
                    out = F.conv2d(inp, w, bias, c.stride, c.padding)
                if tape is not None:
                    tape.append((c, inp, out, s))
                return out
            pk = packs.get((c, False)) if packs else None
            if pk is not None and fastconv.supported(c, inp):
                out = fastconv.conv3x3(inp, pk)
            else:
                out = c(inp)
            if tape is not None:
                tape.append((c, inp, out, None))
            return _bn(out, b, bn, n_valid, group)

        out = F.relu(conv_bn(self.conv1, self.bn1, x))
        if self.stem == "imagenet":
            out = F.max_pool2d(out, 3, stride=2, padding=1)
        for blk in self.blocks():
            inp = out
            chain = blk.chain()
            for j, (c, b, act) in enumerate(chain):
                out = conv_bn(c, b, out)
                if act:
                    out = F.relu(out)
            if len(blk.shortcut) > 0:
                sc = conv_bn(blk.shortcut[0], blk.shortcut[1], inp)
            else:
                sc = inp
            out = F.relu(out + sc)
        if self.stem == "cifar":
            out = F.avg_pool2d(out, 4)
        else:
            out = F.adaptive_avg_pool2d(out, 1)
        feat = out.reshape(out.size(0), -1)
        logits = self.linear(feat)
        if tape is not None:
            tape.append((self.linear, feat, logits, None))
        return logits


def ResNet18(num_classes=10, stem="cifar"):
    return ResNet(BasicBlock, [2, 2, 2, 2], num_classes, stem)


def ResNet34(num_classes=10, stem="cifar"):
    return ResNet(BasicBlock, [3, 4, 6, 3], num_classes, stem)


def ResNet50(num_classes=10, stem="cifar"):
    return ResNet(Bottleneck, [3, 4, 6, 3], num_classes, stem)


def ResNet101(num_classes=10, stem="cifar"):
    return ResNet(Bottleneck, [3, 4, 23, 3], num_classes, stem)


def ResNet152(num_classes=10, stem="cifar"):
    return ResNet(Bottleneck, [3, 8, 36, 3], num_classes, stem)


ARCHS = {"resnet18": ResNet18, "resnet34": ResNet34, "resnet50": ResNet50,
         "resnet101": ResNet101, "resnet152": ResNet152}


def build(arch: str, num_classes: int = 10, stem: str = "cifar") -> ResNet:
    try:
        return ARCHS[arch.lower()](num_classes, stem)
    except KeyError:
        raise ValueError(f"unknown arch {arch!r}; have {sorted(ARCHS)}") from None
