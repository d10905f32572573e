"""Hand-scheduled GraNd forward/backward for BasicBlock ResNets (eval BN folded into convs).

Replaces autograd for the GraNd pass of ResNet-18/34: the per-conv (input activation,
output gradient) pairs the norm kernels need are produced directly, and every 3x3 stride-1
conv runs on the split-bf16 kernel with its elementwise neighbours fused into the epilogue:

  forward   h   = relu(conv1(x) + b1)                       [bias + ReLU epilogue]
            out = relu(conv2(h) + b2 + shortcut(x))         [bias + residual + ReLU epilogue]
  backward  dz2 = d_out * (out > 0)                         (produced by the consumer below)
            dh  = conv2^T(dz2) * (h > 0)                    [ReLU-mask epilogue]
            dz2_prev = (conv1^T(dh) + dz2) * (x > 0)        [residual + ReLU-mask epilogue]
The reference's network is models/resnet.py:7-32 (BasicBlock) and :88-97 (forward); the
math is the chain rule of that forward with BN in eval mode (GraNd).
Downsampling heads (conv1 3x3/2 + the 1x1/2 projection) run forward and backward-data on
dd_down_forward / dd_down_backward; shapes those kernels do not cover fall back to MIOpen.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _capi, fastconv
from .resnet import BasicBlock, Bottleneck, ResNet


def conv_input_grad(in_shape, weight, dy, conv):
    """MIOpen backward-data with packed descriptors.  (torch.nn.grad.conv2d_input builds its
    shape-only input with expand(), a stride-0 tensor, and MIOpen then picks its naive
    non-packed kernels: ~30 ms per call.)"""
    shape_only = torch.empty(in_shape, dtype=dy.dtype, device=dy.device)
    return torch.ops.aten.convolution_backward(
        dy, shape_only, weight, None, list(conv.stride), list(conv.padding),
        list(conv.dilation), False, [0, 0], conv.groups, [True, False, False])[0]


def applicable(model: ResNet) -> bool:
    return (model.stem == "cifar" and getattr(model, "_folded", None) is not None
            and getattr(model, "_packs", None) is not None
            and all(isinstance(b, (BasicBlock, Bottleneck)) for b in model.blocks()))


@torch.no_grad()
def forward_backward(model: ResNet, x: torch.Tensor, labels: torch.Tensor, e: torch.Tensor,
                     bn_pairs: list = None, bad_labels: torch.Tensor = None):
    """Returns ([(conv, act, gout, col_scale)], feat) for one chunk; writes the CE logit
    gradient (= EL2N residual) into `e` [B, C] (bad_labels: dd_el2n's label counter).

    bn_pairs (a list, grand_params = all): receives (bn, v, r, g) per BatchNorm — g the
    gradient w.r.t. the BN output, v the tensor equal to that output (+ r) wherever g != 0
    (dd_bn_pegrad_sqnorm): the post-ReLU activation after bn1 and the stem BN, the block
    output with r = the shortcut value after bn2, the projection output after its BN."""
    folded, packs = model._folded, model._packs

    def fast(conv, inp):
        return (conv, True) in packs and fastconv.supported(conv, inp)

    # fragment-order ReLU masks of the fast convs' outputs (tensor data_ptr -> bits): the
    # backward conv that masks by such a tensor has the producer's geometry and reads 1 bit
    # per element instead of the fp32 activation
    bits = {}

    packs1 = getattr(model, "_packs1", {})
    down3 = getattr(model, "_down3", {})

    def fwd(conv, inp, relu, residual=None):
        w, b, _ = folded[conv]
        if fast(conv, inp):
            pk = packs[(conv, True)]
            m = _capi.conv3x3_mask(inp.shape[0], pk.cout, inp.shape[2], inp.shape[3], inp.device)
            y = _capi.conv3x3(inp, pk.fwd, pk.cout, bias=b, residual=residual, relu=relu,
                              mask_out=m if relu else None)
            if relu:
                bits[y.data_ptr()] = (m, y)
            return y
        p1 = packs1.get((conv, True))
        if p1 is not None and fastconv.supported1x1(conv, inp):
            return _capi.conv1x1(inp, p1.fwd, p1.cout, stride=conv.stride[0], bias=b,
                                 residual=residual, relu=relu)
        d3 = down3.get((conv, True))
        if (d3 is not None and residual is None
                and _capi.down_supported(inp.shape[2] // 2, inp.shape[3] // 2)):
            return _capi.conv_down(inp, d3.fwd3, d3.cout, None, bias=b, relu=relu)[0]
        out = F.conv2d(inp, w, b, conv.stride, conv.padding)
        if residual is not None:
            out = out + residual
        return F.relu(out) if relu else out

    def bwd(conv, dy, in_shape, residual=None, mask=None):
        """grad w.r.t. the conv input, + residual, * (mask > 0)."""
        if fast(conv, dy):  # stride-1 3x3: dy has the input's spatial shape
            pk = packs[(conv, True)]
            mb = bits.get(mask.data_ptr()) if mask is not None else None
            if mb is not None and mb[1] is mask and mask.shape[1] == pk.cin:
                return _capi.conv3x3(dy, pk.bwd, pk.cin, residual=residual, mask_in=mb[0])
            return _capi.conv3x3(dy, pk.bwd, pk.cin, residual=residual, mask_src=mask)
        p1 = packs1.get((conv, True))
        if p1 is not None and conv.stride == (1, 1) and fastconv.supported1x1(conv, dy):
            return _capi.conv1x1(dy, p1.bwd, p1.cin, residual=residual, mask_src=mask)
        d3 = down3.get((conv, True))
        if d3 is not None and residual is None and _capi.down_supported(dy.shape[2], dy.shape[3]):
            return _capi.down_backward(dy.contiguous(), d3.bwd3, d3.cin, mask_src=mask)
        dx = conv_input_grad(in_shape, folded[conv][0], dy, conv)
        if residual is not None:
            dx = dx + residual
        if mask is not None:
            dx = dx * (mask > 0)
        return dx

    down = getattr(model, "_down", {})
    a = fwd(model.conv1, x, relu=True)
    a_stem = a
    saved = []
    keep = bn_pairs is not None
    for blk in model.blocks():
        xin = a
        if isinstance(blk, Bottleneck):
            # reference models/resnet.py:57-63 with BN folded: relu(c1) -> relu(c2) ->
            # relu(c3 + shortcut) (the residual add and ReLU in the conv3 epilogue)
            h1 = fwd(blk.conv1, xin, relu=True)
            h2 = fwd(blk.conv2, h1, relu=True)
            sc = fwd(blk.shortcut[0], xin, relu=False) if len(blk.shortcut) else xin
            a = fwd(blk.conv3, h2, relu=True, residual=sc)
            saved.append((blk, xin, (h1, h2), sc if keep else None, a if keep else None))
            continue
        dp = down.get((blk, True))
        if dp is not None and _capi.down_supported(xin.shape[2] // 2, xin.shape[3] // 2):
            # conv1 (3x3/2) + bias + ReLU and the 1x1/2 projection + bias in one kernel
            h, sc, _, _ = _capi.conv_down(xin, dp.fwd3, dp.cout, dp.fwd1,
                                          bias=folded[blk.conv1][1], relu=True,
                                          bias_sc=folded[blk.shortcut[0]][1])
        else:
            h = fwd(blk.conv1, xin, relu=True)
            sc = fwd(blk.shortcut[0], xin, relu=False) if len(blk.shortcut) else xin
        a = fwd(blk.conv2, h, relu=True, residual=sc)
        saved.append((blk, xin, h, sc if bn_pairs is not None else None,
                      a if bn_pairs is not None else None))
    # head (reference models/resnet.py:94-96): avg_pool2d(out, 4) over the final 4x4 map
    feat = _capi.head_pool(a) if a.shape[2:] == (4, 4) else F.avg_pool2d(a, 4).flatten(1)
    lin = model.linear
    logits = _capi.linear_forward(feat.contiguous(), lin.weight.detach(),
                                  None if lin.bias is None else lin.bias.detach())
    _capi.el2n(logits, labels, e=e, bad_labels=bad_labels)

    # d(loss)/d(pre-activation of the last block) = broadcast(e W / 16) * (out > 0), one pass
    if a.shape[2:] == (4, 4):
        d = _capi.head_backward(a, e, model.linear.weight.detach().float().contiguous())
    else:
        dfeat = e @ model.linear.weight
        d = (dfeat / 16.0)[:, :, None, None] * (a > 0)
    pairs = []
    for blk, xin, h, sc, out in reversed(saved):
        if isinstance(blk, Bottleneck):
            d = _bottleneck_backward(blk, xin, h, sc, out, d.contiguous(), folded, bwd, packs1,
                                     pairs, bn_pairs)
            continue
        dz2 = d.contiguous()
        dh = bwd(blk.conv2, dz2, h.shape, mask=h)
        s1, s2 = folded[blk.conv1][2], folded[blk.conv2][2]
        pairs.append((blk.conv2, h, dz2, s2))
        pairs.append((blk.conv1, xin, dh, s1))
        if bn_pairs is not None:
            bn_pairs.append((blk.bn2, out, sc, dz2))
            bn_pairs.append((blk.bn1, h, None, dh))
            if len(blk.shortcut):
                bn_pairs.append((blk.shortcut[1], sc, None, dz2))
        dp = down.get((blk, True))
        if len(blk.shortcut):
            sconv = blk.shortcut[0]
            pairs.append((sconv, xin, dz2, folded[sconv][2]))
            if dp is not None and _capi.down_supported(dh.shape[2], dh.shape[3]):
                # transposed stride-2 conv1 + transposed 1x1/2 shortcut + ReLU mask, one kernel
                # the block input's ReLU mask as plane bits, converted from the fragment words
                # its producer (the previous block's conv2) wrote: 1 bit per element read
                mb = bits.get(xin.data_ptr())
                pb = None
                if (mb is not None and mb[1] is xin
                        and _capi.down_backward_mask_bits_supported(dh.shape[2], dh.shape[3])
                        and (xin.shape[2] * xin.shape[3]) % 32 == 0):
                    pb = _capi.conv3x3_mask_plane_bits(mb[0], *xin.shape)
                d = _capi.down_backward(dh.contiguous(), dp.bwd3, dp.cin, dz=dz2,
                                        packed1x1_t=dp.bwd1,
                                        mask_src=None if pb is not None else xin, mask_bits=pb)
            else:
                dsc = conv_input_grad(xin.shape, folded[sconv][0], dz2, sconv)
                d = bwd(blk.conv1, dh, xin.shape, residual=dsc, mask=xin)
        else:
            d = bwd(blk.conv1, dh, xin.shape, residual=dz2, mask=xin)
    pairs.append((model.conv1, x, d.contiguous(), folded[model.conv1][2]))
    if bn_pairs is not None:
        bn_pairs.append((model.bn1, a_stem, None, pairs[-1][2]))
    return pairs, feat


def _bottleneck_backward(blk, xin, h, sc, out, dz3, folded, bwd, packs1, pairs, bn_pairs):
    """Backward-data through one Bottleneck (BN folded), recording the (conv, act, gout, s)
    pairs of its convs; returns the gradient w.r.t. the block input's pre-activation:
      dh2 = conv3^T(dz3) * (h2 > 0);  dh1 = conv2^T(dh2) * (h1 > 0)
      d   = (conv1^T(dh1) + shortcut^T(dz3) | dz3) * (xin > 0)
    A stride-2 projection's transposed 1x1 runs on its own grid and is scattered into the
    conv1^T launch by its up2 epilogue operand."""
    h1, h2 = h
    dh2 = bwd(blk.conv3, dz3, h2.shape, mask=h2)
    dh1 = bwd(blk.conv2, dh2, h1.shape, mask=h1)
    pairs.append((blk.conv3, h2, dz3, folded[blk.conv3][2]))
    pairs.append((blk.conv2, h1, dh2, folded[blk.conv2][2]))
    pairs.append((blk.conv1, xin, dh1, folded[blk.conv1][2]))
    if bn_pairs is not None:
        bn_pairs.append((blk.bn3, out, sc, dz3))
        bn_pairs.append((blk.bn2, h2, None, dh2))
        bn_pairs.append((blk.bn1, h1, None, dh1))
    if not len(blk.shortcut):
        return bwd(blk.conv1, dh1, xin.shape, residual=dz3, mask=xin)
    sconv = blk.shortcut[0]
    pairs.append((sconv, xin, dz3, folded[sconv][2]))
    if bn_pairs is not None:
        bn_pairs.append((blk.shortcut[1], sc, None, dz3))
    ps, p1 = packs1.get((sconv, True)), packs1.get((blk.conv1, True))
    if sconv.stride == (2, 2) and ps is not None and p1 is not None:
        t = _capi.conv1x1(dz3, ps.bwd, ps.cin)  # W_sc^T dz3 on the half-resolution grid
        return _capi.conv1x1(dh1, p1.bwd, p1.cin, res_up2=t, mask_src=xin)
    t = bwd(sconv, dz3, xin.shape)
    return bwd(blk.conv1, dh1, xin.shape, residual=t, mask=xin)
