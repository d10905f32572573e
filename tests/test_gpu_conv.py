"""Backbone 3x3 stride-1 conv (split-bf16 MFMA) vs PyTorch fp32 (F.conv2d / conv2d_input).

This is a floating-point kernel, so the checker is a plain fp32 PyTorch reference of the same
op (computed on the CPU, so it cannot share code with the kernel under test).  Tolerance:
split-bf16 products carry ~2^-16 relative error; we require 5e-4 relative on the max-abs.
"""
import pytest
import torch
import torch.nn.functional as F

from data_diet_distributed_amd import _capi

pytestmark = pytest.mark.gpu

# (B, cin, cout, H, W): every 3x3 stride-1 conv of CIFAR ResNet-18/50 + ragged channels; the
# last four take the r2 tile with an odd count of 16-channel K chunks (its zero chunk) and,
# for cout = 200, a partly padded 128-output block
SHAPES = [(4, 64, 64, 32, 32), (3, 128, 128, 16, 16), (2, 256, 256, 8, 8), (2, 512, 512, 8, 8),
          (3, 3, 64, 32, 32), (2, 20, 70, 16, 16), (2, 64, 130, 8, 8), (2, 17, 64, 16, 8),
          (1, 96, 40, 64, 32), (5, 512, 512, 4, 4), (3, 64, 96, 4, 4), (3, 32, 64, 8, 8),
          (3, 48, 128, 16, 16), (2, 80, 256, 8, 8), (3, 16, 128, 4, 4), (3, 100, 200, 8, 8)]


def _close(got, want, rel=5e-4):
    err = (got.cpu() - want).abs().max().item()
    scale = want.abs().max().item()
    assert err <= rel * scale + 1e-6, (err, scale)


@pytest.mark.parametrize("B,cin,cout,H,W", SHAPES)
def test_conv3x3_forward_plain(cuda, B, cin, cout, H, W):
    g = torch.Generator().manual_seed(B * cin + cout)
    x = torch.randn(B, cin, H, W, generator=g)
    w = torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)
    want = F.conv2d(x, w, padding=1)
    packed = _capi.conv3x3_pack(w.to(cuda))
    got = _capi.conv3x3(x.to(cuda), packed, cout)
    _close(got, want)


@pytest.mark.parametrize("B,cin,cout,H,W", SHAPES[:4])
def test_conv3x3_forward_fused_epilogue(cuda, B, cin, cout, H, W):
    g = torch.Generator().manual_seed(7)
    x = torch.randn(B, cin, H, W, generator=g)
    w = torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)
    bias = torch.randn(cout, generator=g)
    res = torch.randn(B, cout, H, W, generator=g)
    mask = torch.randn(B, cout, H, W, generator=g)
    packed = _capi.conv3x3_pack(w.to(cuda))
    want = F.relu(F.conv2d(x, w, bias, padding=1) + res)
    got = _capi.conv3x3(x.to(cuda), packed, cout, bias=bias.to(cuda), residual=res.to(cuda),
                        relu=True)
    _close(got, want)
    want2 = (F.conv2d(x, w, padding=1) + res) * (mask > 0)
    got2 = _capi.conv3x3(x.to(cuda), packed, cout, residual=res.to(cuda), mask_src=mask.to(cuda))
    _close(got2, want2)


@pytest.mark.parametrize("B,cin,cout,H,W", SHAPES)
def test_conv3x3_backward_data(cuda, B, cin, cout, H, W):
    """transpose_flip packing: dx = conv2d_input(x.shape, w, dy, padding=1)."""
    g = torch.Generator().manual_seed(11 + cin)
    w = torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)
    dy = torch.randn(B, cout, H, W, generator=g)
    want = torch.nn.grad.conv2d_input((B, cin, H, W), w, dy, padding=1)
    packed = _capi.conv3x3_pack(w.to(cuda), transpose_flip=True)
    got = _capi.conv3x3(dy.to(cuda), packed, cin)
    _close(got, want)


def test_conv3x3_unsupported_shape_raises(cuda):
    w = torch.randn(8, 8, 3, 3, device=cuda)
    packed = _capi.conv3x3_pack(w)
    with pytest.raises(_capi.DDError, match="unsupported spatial shape"):
        _capi.conv3x3(torch.randn(1, 8, 7, 7, device=cuda), packed, 8)
    with pytest.raises(_capi.DDError, match="unsupported spatial shape"):
        _capi.conv3x3(torch.randn(1, 8, 8, 4, device=cuda), packed, 8)


@pytest.mark.parametrize("B,cin,cout,H,W", [(3, 64, 64, 32, 32), (5, 128, 128, 16, 16),
                                             (3, 256, 256, 8, 8), (6, 512, 512, 4, 4),
                                             (2, 20, 70, 16, 16)])
def test_conv3x3_fragment_mask_equals_fp32_mask(cuda, B, cin, cout, H, W):
    """mask_out of a producer conv, read back by a consumer of the same output geometry
    (mask_in), masks exactly like mask_src = the producer's fp32 output."""
    g = torch.Generator().manual_seed(B * H + cout)
    x = torch.randn(B, cin, H, W, generator=g).to(cuda)
    w1 = (torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)).to(cuda)
    w2 = (torch.randn(cin, cout, 3, 3, generator=g) / (3 * cout ** 0.5)).to(cuda)
    bias = torch.randn(cout, generator=g).to(cuda)
    m = _capi.conv3x3_mask(B, cout, H, W, cuda)
    h = _capi.conv3x3(x, _capi.conv3x3_pack(w1), cout, bias=bias, relu=True, mask_out=m)
    dy = torch.randn(B, cin, H, W, generator=g).to(cuda)  # consumer: conv over cin -> cout
    pk = _capi.conv3x3_pack(w2, transpose_flip=True)       # output channels = cout
    a = _capi.conv3x3(dy, pk, cout, mask_src=h)
    b = _capi.conv3x3(dy, pk, cout, mask_in=m)
    assert torch.equal(a, b)
    assert (h > 0).any() and (h == 0).any()


# the stem layout (dd_conv3x3_pack with cin <= 5 folds kx into pseudo-channels): every cin
# it covers, at every tile family's spatial shapes, with the staging transform and epilogues
STEM_SHAPES = [(2, c, 64, 32, 32) for c in (1, 2, 3, 4, 5)] + [
    (3, 3, 64, 16, 16), (2, 5, 70, 8, 8), (4, 3, 128, 4, 4), (2, 1, 40, 16, 8)]


@pytest.mark.parametrize("B,cin,cout,H,W", STEM_SHAPES)
def test_conv3x3_stem_layout(cuda, B, cin, cout, H, W):
    g = torch.Generator().manual_seed(31 * cin + H + cout)
    x = torch.randn(B, cin, H, W, generator=g)
    w = torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)
    bias = torch.randn(cout, generator=g)
    res = torch.randn(B, cout, H, W, generator=g)
    packed = _capi.conv3x3_pack(w.to(cuda))
    _close(_capi.conv3x3(x.to(cuda), packed, cout), F.conv2d(x, w, padding=1))
    got = _capi.conv3x3(x.to(cuda), packed, cout, bias=bias.to(cuda), residual=res.to(cuda),
                        relu=True)
    _close(got, F.relu(F.conv2d(x, w, bias, padding=1) + res))
    # grouped input transform (train-mode BN + ReLU of a producer), groups of 2 examples
    gs = 4 if W == 4 else 2
    G = -(-B // gs)
    sc = torch.rand(G, cin, generator=g) + 0.5
    sh = torch.randn(G, cin, generator=g)
    xf = torch.relu(x * sc.repeat_interleave(gs, 0)[:B, :, None, None]
                    + sh.repeat_interleave(gs, 0)[:B, :, None, None])
    got = _capi.conv3x3(x.to(cuda), packed, cout, in_affine=(sc.to(cuda), sh.to(cuda)),
                        group_size=gs)
    _close(got, F.conv2d(xf, w, padding=1))
    # the backward-data pack of the same weights keeps the standard layout (in = cout)
    dy = torch.randn(B, cout, H, W, generator=g)
    got = _capi.conv3x3(dy.to(cuda), _capi.conv3x3_pack(w.to(cuda), transpose_flip=True), cin)
    _close(got, torch.nn.grad.conv2d_input((B, cin, H, W), w, dy, padding=1))


@pytest.mark.parametrize("B,cin,cout,H,W", [(2, 64, c, 32, 32) for c in (1, 2, 3, 4, 5)] + [
    (3, 40, 3, 16, 16), (2, 70, 5, 8, 8), (4, 128, 3, 4, 4)])
def test_conv3x3_backward_data_small_cout(cuda, B, cin, cout, H, W):
    """Backward-data of a conv with cout <= 5: the transposed pack has <= 5 input channels, so
    it must be written in the stem layout the kernel then assumes."""
    g = torch.Generator().manual_seed(17 * cout + H)
    w = torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)
    dy = torch.randn(B, cout, H, W, generator=g)
    want = torch.nn.grad.conv2d_input((B, cin, H, W), w, dy, padding=1)
    packed = _capi.conv3x3_pack(w.to(cuda), transpose_flip=True)
    _close(_capi.conv3x3(dy.to(cuda), packed, cin), want)
    res = torch.randn(B, cin, H, W, generator=g)
    mask = torch.randn(B, cin, H, W, generator=g)
    got = _capi.conv3x3(dy.to(cuda), packed, cin, residual=res.to(cuda), mask_src=mask.to(cuda))
    _close(got, (want + res) * (mask > 0))
