"""Hand-scheduled EL2N forward with grouped train-mode BatchNorm (reference semantics).

The reference scores with the net in train mode (train.py:59-63 never calls .eval(), and
get_scores_and_prune.py:15 runs `net(input)` per loader batch), so every BatchNorm2d uses
the statistics of the current 128-example batch.  Under the parity protocol
batch g is examples [g*B, (g+1)*B).  This module runs many such batches per launch ("BN
groups"), each normalised with its own statistics, with BN fused into the neighbouring
kernels instead of taking passes of its own:

  conv (3x3 stride 1: dd_conv3x3_forward, at 28 / 14 / 7 on its padded-width tiles; 1x1:
        dd_conv1x1_forward; 3x3 stride 2 of a Bottleneck: dd_down_forward, at 28 / 14 / 7 on its
        padded-width heads; any other kh x kw (the ImageNet 7x7 stem: dd_stem7_forward, else): dd_conv_gemm_forward;
        shapes none takes: MIOpen + dd_channel_stats)
      -> raw output y + per-(group, channel) partial sums (conv epilogue)
  dd_bn_finalize -> (scale, shift) per (group, channel)
  next conv of the unit stages relu(y * scale + shift) on the fly (no extra pass)
  unit tail: relu(bn(y_last) + shortcut), computed while the next unit's first conv stages
        it and written out once (a 3x3: dd_conv3x3_forward_unit_input; a Bottleneck's 1x1
        conv1 on the float4 layout: dd_conv1x1_forward_unit_input), or by a dd_bn_apply pass
        where that conv has no fused form (a downsampling head, 7x7 maps, 4x4 maps)
        [+ the 4x4 avg-pool head]

Network: reference models/resnet.py:7-97 (BasicBlock, Bottleneck, CIFAR stem, head).
Outputs are the logits of `ResNet.run(x, bn="batch", n_valid=...)` per group to fp32
rounding (tests/test_gpu_el2n_fast.py).
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from . import _capi, fastconv
from .resnet import ResNet


def applicable(model: ResNet) -> bool:
    return getattr(model, "_packs", None) is not None


def _conv_bn_stats(model, conv, bn, src, xf, gs, n_valid):
    """y = conv(xf(src)), plus the (scale, shift) of its train-mode BN over each group.
    xf = None or ((scale, shift), relu): the producer's pending BN.

    3x3 stride 1 -> dd_conv3x3_forward (native tiles, or the padded-width ones at widths that
    are not a tile width); 1x1 (stride 1 or 2) -> dd_conv1x1_forward (both apply
    xf while staging and leave the statistics in their epilogue); 3x3 stride 2 (ResNet-50
    Bottleneck conv2) -> dd_down_forward after a dd_bn_apply of xf; other kh x kw ->
    dd_conv_gemm_forward (xf staged, except into a dense-K pack); anything else -> MIOpen."""
    pk = model._packs.get((conv, False))
    p1 = getattr(model, "_packs1", {}).get((conv, False))
    d3 = getattr(model, "_down3", {}).get((conv, False))
    gemm_ok = (hasattr(model, "_gemm") and conv.kernel_size != (1, 1) and conv.groups == 1
               and conv.dilation == (1, 1))
    go = tuple((src.shape[i] + 2 * conv.padding[i - 2] - conv.kernel_size[i - 2])
               // conv.stride[i - 2] + 1 for i in (2, 3))
    ho, wo = (src.shape[2] // conv.stride[0], src.shape[3] // conv.stride[1])
    if pk is not None and (fastconv.supported(conv, src) or (
            conv.kernel_size == (3, 3) and conv.stride == (1, 1) and conv.padding == (1, 1)
            and _capi.conv3x3_padded_supported(src.shape[2], src.shape[3], conv.in_channels,
                                               conv.out_channels, gs))):
        y, st = _capi.conv3x3(src, pk.fwd, pk.cout, in_affine=xf[0] if xf else None,
                              in_relu=xf[1] if xf else True, group_size=gs, stats=True,
                              n_stat=n_valid)
    elif (p1 is not None and fastconv.supported1x1(conv, src)
          and _capi.lib().dd_conv1x1_tiles_per_group(ho, wo, gs) > 0):
        y, st = _capi.conv1x1(src, p1.fwd, p1.cout, stride=conv.stride[0],
                              in_affine=xf[0] if xf else None, in_relu=xf[1] if xf else True,
                              group_size=gs, stats=True, n_stat=n_valid)
    elif (d3 is not None and src.shape[2] % 2 == 0 and src.shape[3] % 2 == 0
          and (_capi.down_supported(ho, wo)
               or _capi.down_padded_supported(ho, wo, conv.in_channels, conv.out_channels, gs))
          and _capi.lib().dd_down_tiles_per_group(ho, wo, gs) > 0):
        if xf is not None and xf[1] and FUSE_UNIT_INPUT:
            # the producer's BN + ReLU computed while the head stages (no pass of its own)
            y, _, st, _ = _capi.conv_down_unit_input(src, xf[0], d3.fwd3, d3.cout, gs,
                                                     n_stat=n_valid)
        else:
            if xf is not None:
                src, _ = _capi.bn_apply(src, xf[0], gs, relu=xf[1])
            y, _, st, _ = _capi.conv_down(src, d3.fwd3, d3.cout, None, group_size=gs,
                                          stats=True, n_stat=n_valid)
    elif (gemm_ok and xf is None and conv.kernel_size == (7, 7) and conv.stride == (2, 2)
          and conv.padding == (3, 3) and STEM7
          and _capi.stem7_supported(src.shape[2], src.shape[3], conv.in_channels,
                                    conv.out_channels, gs)):
        # the ImageNet stem: input rows staged once per output-row pair (dd_stem7_forward)
        y, st = _capi.stem7(src, model.stem7_pack(conv), conv.out_channels, gs, n_stat=n_valid)
    elif (gemm_ok and _capi.lib().dd_conv1x1_tiles_per_group(go[0], go[1], gs) > 0
          and conv.stride[0] == conv.stride[1] and conv.padding[0] == conv.padding[1]
          and conv.stride[0] in (1, 2)):
        gp = model.gemm_pack(conv)  # packed on first use
        dense = _capi.lib().dd_conv_gemm_dense(conv.in_channels, *conv.kernel_size) == 1
        if xf is not None and dense:
            src, _ = _capi.bn_apply(src, xf[0], gs, relu=xf[1])
            xf = None
        y, st = _capi.conv_gemm(src, gp, conv.out_channels, conv.kernel_size, conv.stride[0],
                                conv.padding[0], in_affine=xf[0] if xf else None,
                                in_relu=xf[1] if xf else True, group_size=gs, stats=True,
                                n_stat=n_valid)
    else:
        if xf is not None:
            src, _ = _capi.bn_apply(src, xf[0], gs, relu=xf[1])
        y = F.conv2d(src, conv.weight, None, conv.stride, conv.padding).contiguous()
        st = _capi.channel_stats(y, gs, n_stat=n_valid)
    aff = _capi.bn_finalize(st, bn.weight, bn.bias, bn.eps)
    return y, aff


# the ImageNet stem on dd_stem7_forward (DD_STEM7=0: the implicit GEMM, for tests and A/B runs;
# read per call)
class _Flag:
    def __bool__(self):
        return os.environ.get("DD_STEM7", "1") != "0"


STEM7 = _Flag()

# the unit tail fused into the next unit's first conv where it can be (bitwise the same as
# the separate dd_bn_apply pass; False runs that pass everywhere, for tests and A/B runs)
FUSE_UNIT_INPUT = os.environ.get("DD_FUSE_UNIT_INPUT", "1") != "0"


def _unit_input_conv(model, blk, src, gs):
    """The packs of `blk`'s first conv when it can take the previous unit's output fused
    (a 3x3 stride-1 conv on the scoring tiles), else None."""
    if not FUSE_UNIT_INPUT:
        return None
    chain = blk.chain()
    if len(chain) < 2:
        return None
    conv = chain[0][0]
    pk = model._packs.get((conv, False))
    if pk is None or not fastconv.supported(conv, src):
        return None
    _, cin, h, w = src.shape
    if not _capi.conv3x3_unit_input_supported(h, w, cin, pk.cout, gs):
        return None
    return pk


def _unit_input_conv1x1(model, blk, src, gs):
    """The 1x1 packs of `blk`'s first conv when it can take the previous unit's output fused
    (a ResNet-50 Bottleneck's stride-1 conv1 on the float4 1x1 layout), else None."""
    if not FUSE_UNIT_INPUT:
        return None
    chain = blk.chain()
    if len(chain) < 2:
        return None
    conv = chain[0][0]
    p1 = getattr(model, "_packs1", {}).get((conv, False))
    if p1 is None or conv.stride != (1, 1) or not fastconv.supported1x1(conv, src):
        return None
    _, cin, h, w = src.shape
    if (h * w) % 4 or _capi.lib().dd_conv1x1_tiles_per_group(h, w, gs) <= 0:
        return None
    return p1


def _poolable(hw: int) -> bool:
    L = hw // 4
    return hw % 4 == 0 and L >= 1 and L <= 64 and (L & (L - 1)) == 0


@torch.inference_mode()
def forward_logits(model: ResNet, x: torch.Tensor, group_size: int, n_valid: int) -> torch.Tensor:
    """Logits [B, C] of the train-mode-BN forward of x [B, 3, H, W] (contiguous fp32), with
    BN statistics per group of `group_size` rows over rows < n_valid."""
    gs = int(group_size)
    y, aff = _conv_bn_stats(model, model.conv1, model.bn1, x, None, gs, n_valid)
    # `pending` = (y, (scale, shift), residual, residual affine): a unit output relu(bn(y) + R)
    # not yet materialised; the next unit's first conv computes it while staging when it can
    pending = None
    a = None
    if model.stem == "imagenet":
        # BN + ReLU + 3x3/2 max-pool in one pass (the 112x112 map is never materialised)
        a = _capi.bn_apply_maxpool(y, aff, gs)
    else:
        pending = (y, aff, None, None)
    blocks = list(model.blocks())
    feat = None
    down = getattr(model, "_down", {})
    for i, blk in enumerate(blocks):
        chain = blk.chain()
        res = res_aff = None
        dp = down.get((blk, False))
        cur = pending[0] if pending is not None else a  # (the unit input's shape)
        head = dp is not None and _capi.down_supported(cur.shape[2] // 2, cur.shape[3] // 2)
        pk0 = None if pending is None or head else _unit_input_conv(model, blk, pending[0], gs)
        p10 = (None if pending is None or head or pk0 is not None
               else _unit_input_conv1x1(model, blk, pending[0], gs))
        if p10 is not None:
            # the previous (Bottleneck) unit's output, fused into this unit's 1x1 conv1
            py, paff, pres, pres_aff = pending
            inp, y1, st1 = _capi.conv1x1_unit_input(py, paff, p10.fwd, p10.cout, gs,
                                                    residual=pres, res_affine=pres_aff,
                                                    n_stat=n_valid)
            c0, bn0, act0 = chain[0]
            aff1 = _capi.bn_finalize(st1, bn0.weight, bn0.bias, bn0.eps)
            src, xf = y1, (aff1, act0)
            chain = chain[1:]
        elif pk0 is not None:
            # the previous unit's output, fused into this unit's first conv
            py, paff, pres, pres_aff = pending
            inp, y1, st1 = _capi.conv3x3_unit_input(py, paff, pk0.fwd, pk0.cout, gs,
                                                    residual=pres, res_affine=pres_aff,
                                                    n_stat=n_valid)
            c0, bn0, act0 = chain[0]
            aff1 = _capi.bn_finalize(st1, bn0.weight, bn0.bias, bn0.eps)
            src, xf = y1, (aff1, act0)
            chain = chain[1:]
        elif head and pending is not None and FUSE_UNIT_INPUT and pending[3] is None \
                and pending[2] is not None:
            # the previous unit's output (identity shortcut), computed while the head stages
            # it: only this head's two convs read it, so it is never written
            py, paff, pres, _ = pending
            inp = None
        else:
            if pending is not None:
                py, paff, pres, pres_aff = pending
                a, _ = _capi.bn_apply(py, paff, gs, residual=pres, res_affine=pres_aff,
                                      relu=True)
            inp = a
            src, xf = inp, None
        fused_head = head and inp is None
        pending = None
        if head:
            # downsampling head: conv1 (3x3/2) and the 1x1/2 projection in one kernel
            if fused_head:
                y1, ys, st1, sts = _capi.conv_down_unit_input(py, paff, dp.fwd3, dp.cout, gs,
                                                              packed1x1=dp.fwd1, residual=pres,
                                                              n_stat=n_valid)
            else:
                y1, ys, st1, sts = _capi.conv_down(inp, dp.fwd3, dp.cout, dp.fwd1,
                                                   group_size=gs, stats=True, n_stat=n_valid)
            aff1 = _capi.bn_finalize(st1, blk.bn1.weight, blk.bn1.bias, blk.bn1.eps)
            sbn = blk.shortcut[1]
            res, res_aff = ys, _capi.bn_finalize(sts, sbn.weight, sbn.bias, sbn.eps)
            src, xf = y1, (aff1, chain[0][2])
            chain = chain[1:]
        for j, (c, bnm, act) in enumerate(chain):
            yj, affj = _conv_bn_stats(model, c, bnm, src, xf, gs, n_valid)
            if j < len(chain) - 1:
                src, xf = yj, (affj, act)
            else:
                y_last, aff_last = yj, affj
        if res is None and len(blk.shortcut) > 0:
            ys, affs = _conv_bn_stats(model, blk.shortcut[0], blk.shortcut[1], inp, None, gs,
                                      n_valid)
            res, res_aff = ys, affs
        elif res is None:
            res, res_aff = inp, None
        last = i == len(blocks) - 1
        hw = y_last.shape[2] * y_last.shape[3]
        if last and model.stem == "cifar" and y_last.shape[2] == 4 and _poolable(hw):
            # avg_pool2d(out, 4) on the 4x4 map (reference :94) fused into the unit tail
            feat = torch.empty((y_last.shape[0], y_last.shape[1]), dtype=torch.float32,
                               device=y_last.device)
            _capi.bn_apply(y_last, aff_last, gs, residual=res, res_affine=res_aff, relu=True,
                           pool_out=feat, write_out=False)
        else:
            pending = (y_last, aff_last, res, res_aff)
    if pending is not None:
        py, paff, pres, pres_aff = pending
        a, _ = _capi.bn_apply(py, paff, gs, residual=pres, res_affine=pres_aff, relu=True)
    if feat is None:
        out = F.avg_pool2d(a, 4) if model.stem == "cifar" else F.adaptive_avg_pool2d(a, 1)
        feat = out.reshape(out.size(0), -1)
    # per-row fixed-order classifier (dd_linear_forward): logits independent of the chunk size
    lin = model.linear
    return _capi.linear_forward(feat.float().contiguous(), lin.weight.detach(),
                                None if lin.bias is None else lin.bias.detach())


@torch.inference_mode()
def forward_logits_fp32(model: ResNet, x: torch.Tensor, group_size: int,
                        n_valid: int) -> torch.Tensor:
    """Plain-fp32 logits of the same train-mode-BN forward, for the keep-set refinement
    (ScoringEngine._refine): fp32 convs (MIOpen, no bf16 split anywhere) and the grouped BN
    as three kernels per layer -- dd_channel_stats (sums in double), dd_bn_finalize,
    dd_bn_apply with the unit's residual add and ReLU -- in place of ResNet.run(bn="groups")'s
    ~10 torch ops per BN, whose launches dominated the refinement's time.  Rows >= n_valid
    are left out of their group's statistics."""
    gs = int(group_size)

    def conv_bn(conv, bn, src):
        y = F.conv2d(src, conv.weight, None, conv.stride, conv.padding).contiguous()
        st = _capi.channel_stats(y, gs, n_stat=n_valid)
        return y, _capi.bn_finalize(st, bn.weight, bn.bias, bn.eps)

    y, aff = conv_bn(model.conv1, model.bn1, x)
    if model.stem == "imagenet":
        a = _capi.bn_apply_maxpool(y, aff, gs)
    else:
        a, _ = _capi.bn_apply(y, aff, gs, relu=True)
    for blk in model.blocks():
        inp = a
        chain = blk.chain()
        src = inp
        for j, (c, bnm, act) in enumerate(chain):
            yj, affj = conv_bn(c, bnm, src)
            if j < len(chain) - 1:
                src, _ = _capi.bn_apply(yj, affj, gs, relu=bool(act))
            else:
                y_last, aff_last = yj, affj
        if len(blk.shortcut) > 0:
            res, res_aff = conv_bn(blk.shortcut[0], blk.shortcut[1], inp)
        else:
            res, res_aff = inp, None
        a, _ = _capi.bn_apply(y_last, aff_last, gs, residual=res, res_affine=res_aff, relu=True)
    out = F.avg_pool2d(a, 4) if model.stem == "cifar" else F.adaptive_avg_pool2d(a, 1)
    lin = model.linear
    return _capi.linear_forward(out.reshape(out.size(0), -1).contiguous(), lin.weight.detach(),
                                None if lin.bias is None else lin.bias.detach())
