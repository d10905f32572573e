"""Downsampling head (stride-2 3x3 conv + fused 1x1 stride-2 shortcut, split-bf16 MFMA) vs
PyTorch fp32 F.conv2d on the CPU.  Tolerance as for the stride-1 kernel (test_gpu_conv.py):
5e-4 of the max-abs (split-bf16 products carry ~2^-16 relative error)."""
import pytest
import torch
import torch.nn.functional as F

from data_diet_distributed_amd import _capi

pytestmark = pytest.mark.gpu

# (B, cin, cout, HI): the three ResNet-18 CIFAR downsampling heads + ragged channel counts
SHAPES = [(3, 64, 128, 32), (2, 128, 256, 16), (5, 256, 512, 8), (2, 20, 70, 16),
          (3, 17, 64, 8), (4, 64, 128, 64)]


def _close(got, want, rel=5e-4):
    err = (got.detach().cpu().double() - want.double()).abs().max().item()
    scale = want.abs().max().item()
    assert err <= rel * scale + 1e-6, (err, scale)


@pytest.mark.parametrize("B,cin,cout,HI", SHAPES)
@pytest.mark.parametrize("with_sc", [True, False])
def test_down_forward(cuda, B, cin, cout, HI, with_sc):
    g = torch.Generator().manual_seed(B + cin + cout + HI)
    x = torch.randn(B, cin, HI, HI, generator=g)
    w3 = torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)
    w1 = torch.randn(cout, cin, 1, 1, generator=g) / cin ** 0.5
    b3 = torch.randn(cout, generator=g)
    b1 = torch.randn(cout, generator=g)
    p3 = _capi.conv3x3_pack(w3.to(cuda))
    p1 = _capi.conv1x1_pack(w1.to(cuda)) if with_sc else None
    y, ys, _, _ = _capi.conv_down(x.to(cuda), p3, cout, p1, bias=b3.to(cuda), relu=True,
                                  bias_sc=b1.to(cuda) if with_sc else None)
    _close(y, F.relu(F.conv2d(x, w3, b3, stride=2, padding=1)))
    if with_sc:
        _close(ys, F.conv2d(x, w1, b1, stride=2))
    else:
        assert ys is None


def test_down_forward_grouped_stats(cuda):
    g = torch.Generator().manual_seed(9)
    B, cin, cout, HI, gs, nv = 10, 64, 128, 16, 4, 9
    x = torch.randn(B, cin, HI, HI, generator=g)
    w3 = torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)
    w1 = torch.randn(cout, cin, 1, 1, generator=g) / cin ** 0.5
    gamma, beta = torch.rand(cout, generator=g) + 0.5, torch.randn(cout, generator=g)
    y, ys, st, sts = _capi.conv_down(x.to(cuda), _capi.conv3x3_pack(w3.to(cuda)), cout,
                                     _capi.conv1x1_pack(w1.to(cuda)), group_size=gs, stats=True,
                                     n_stat=nv)
    for got_y, stats, want in ((y, st, F.conv2d(x, w3, stride=2, padding=1)),
                               (ys, sts, F.conv2d(x, w1, stride=2))):
        _close(got_y, want)
        sc, sh = _capi.bn_finalize(stats, gamma.to(cuda), beta.to(cuda), 1e-5)
        for gi in range(-(-B // gs)):
            v = want[gi * gs:min(nv, (gi + 1) * gs)].double()
            mean, var = v.mean(dim=(0, 2, 3)), v.var(dim=(0, 2, 3), unbiased=False)
            rs = gamma.double() / torch.sqrt(var + 1e-5)
            _close(sc[gi], rs, 2e-4)
            _close(sh[gi], beta.double() - mean * rs, 2e-4)


# padded-width heads (dd_down_forward ABI 10): the ImageNet-stem network's 56 -> 28, 28 -> 14,
# 14 -> 7 stride-2 conv2s and ragged cases (an overhanging last row block at 50 x 56 and
# 10 x 12 inputs, a 24 -> 12 map, 200 outputs in a padded 256-output grid), (B, cin, cout, HI,
# WI, group_size, n_valid)
PW_SHAPES = [(3, 128, 128, 56, 56, 2, 3), (4, 256, 256, 28, 28, 2, 3), (5, 512, 512, 14, 14, 2, 4),
             (3, 96, 200, 50, 56, 3, 2), (3, 80, 128, 24, 24, 3, 3), (4, 72, 128, 10, 12, 2, 3)]


@pytest.mark.parametrize("operands", ["f16x3", "bf16x3"])
@pytest.mark.parametrize("affine", [True, False])
@pytest.mark.parametrize("B,cin,cout,HI,WI,gs,nv", PW_SHAPES)
def test_down_padded_width_stats(cuda, B, cin, cout, HI, WI, gs, nv, affine, operands):
    """The EL2N launch of a Bottleneck's stride-2 conv2 at a width that is not a tile width:
    y against float64 F.conv2d, the finalized BN affine against float64 group statistics."""
    ho, wo = HI // 2, WI // 2
    assert _capi.down_padded_supported(ho, wo, cin, cout, gs)
    g = torch.Generator().manual_seed(B + cin + cout + HI + WI)
    G = -(-B // gs)
    x = torch.randn(B, cin, HI, WI, generator=g)
    w3 = torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)
    s_in = torch.rand(G, cin, generator=g) + 0.5
    t_in = torch.randn(G, cin, generator=g) * 0.3
    gamma, beta = torch.rand(cout, generator=g) + 0.5, torch.randn(cout, generator=g)
    p3 = _capi.conv3x3_pack(w3.to(cuda), operands=operands)
    if affine:
        xin = torch.relu(x * s_in.repeat_interleave(gs, 0)[:B, :, None, None] +
                         t_in.repeat_interleave(gs, 0)[:B, :, None, None])
        y, _, st, _ = _capi.conv_down_unit_input(x.to(cuda), (s_in.to(cuda), t_in.to(cuda)), p3,
                                                 cout, gs, n_stat=nv)
    else:
        xin = x
        y, _, st, _ = _capi.conv_down(x.to(cuda), p3, cout, group_size=gs, stats=True, n_stat=nv)
    want = F.conv2d(xin.double(), w3.double(), stride=2, padding=1)
    assert torch.isfinite(y).all()
    _close(y, want, 5e-4 if operands == "bf16x3" else 1e-5)
    sc, sh = _capi.bn_finalize(st, gamma.to(cuda), beta.to(cuda), 1e-5)
    for gi in range(G):
        v = want[gi * gs:min(nv, (gi + 1) * gs)]
        if v.shape[0] == 0:
            continue
        mean, var = v.mean(dim=(0, 2, 3)), v.var(dim=(0, 2, 3), unbiased=False)
        rs = gamma.double() / torch.sqrt(var + 1e-5)
        _close(sc[gi], rs, 2e-4)
        _close(sh[gi], beta.double() - mean * rs, 2e-4)


def test_down_unsupported_shape_raises(cuda):
    p3 = _capi.conv3x3_pack(torch.randn(8, 8, 3, 3, device=cuda))
    with pytest.raises(_capi.DDError, match="unsupported output shape"):
        _capi.conv_down(torch.randn(1, 8, 14, 14, device=cuda), p3, 8)


@pytest.mark.parametrize("B,cin,cout,HI", SHAPES)
@pytest.mark.parametrize("with_sc", [True, False])
def test_down_backward(cuda, B, cin, cout, HI, with_sc):
    """dx = (conv2d_input(stride 2, 3x3) + conv2d_input(stride 2, 1x1)) * (mask > 0)."""
    g = torch.Generator().manual_seed(100 + B + cin + cout + HI)
    HO = HI // 2
    w3 = torch.randn(cout, cin, 3, 3, generator=g) / (3 * cout ** 0.5)
    w1 = torch.randn(cout, cin, 1, 1, generator=g) / cout ** 0.5
    dh = torch.randn(B, cout, HO, HO, generator=g)
    dz = torch.randn(B, cout, HO, HO, generator=g)
    mask = torch.randn(B, cin, HI, HI, generator=g)
    want = torch.nn.grad.conv2d_input((B, cin, HI, HI), w3, dh, stride=2, padding=1)
    if with_sc:
        want = want + torch.nn.grad.conv2d_input((B, cin, HI, HI), w1, dz, stride=2)
    want = want * (mask > 0)
    got = _capi.down_backward(dh.to(cuda), _capi.conv3x3_pack(w3.to(cuda), transpose_flip=True),
                              cin, dz=dz.to(cuda) if with_sc else None,
                              packed1x1_t=(_capi.conv1x1_pack(w1.to(cuda), transpose=True)
                                           if with_sc else None),
                              mask_src=mask.to(cuda))
    _close(got, want)
    # without a mask
    got2 = _capi.down_backward(dh.to(cuda), _capi.conv3x3_pack(w3.to(cuda), transpose_flip=True),
                               cin)
    _close(got2, torch.nn.grad.conv2d_input((B, cin, HI, HI), w3, dh, stride=2, padding=1))


@pytest.mark.parametrize("B,c,HI", [(3, 64, 32), (2, 128, 16), (5, 256, 8), (2, 70, 16)])
def test_down_backward_plane_bit_mask(cuda, B, c, HI):
    """The head's ReLU-backward mask as plane bits (the GraNd backward of a downsampling
    head): the block input y = relu(conv3x3(x) + bias) written with its fragment-order mask
    (mask_out), converted by dd_conv3x3_mask_plane_bits, is bit-exact against (y > 0), and
    down_backward with those bits equals the fp32-mask call bit for bit."""
    g = torch.Generator(device=cuda).manual_seed(7 + B + c + HI)
    x = torch.randn(B, c, HI, HI, device=cuda, generator=g)
    w = torch.randn(c, c, 3, 3, device=cuda, generator=g) / (3 * c ** 0.5)
    bias = torch.randn(c, device=cuda, generator=g) * 0.1
    m = _capi.conv3x3_mask(B, c, HI, HI, cuda)
    y = _capi.conv3x3(x, _capi.conv3x3_pack(w), c, bias=bias, relu=True, mask_out=m)
    bits = _capi.conv3x3_mask_plane_bits(m, B, c, HI, HI)
    pos = (y > 0).reshape(-1, 32).to(torch.int64)
    want = (pos << torch.arange(32, device=cuda)).sum(1)
    assert torch.equal(bits.to(torch.int64) & 0xFFFFFFFF, want & 0xFFFFFFFF)
    cout, HO = 2 * c, HI // 2
    w3 = torch.randn(cout, c, 3, 3, device=cuda, generator=g) / (3 * cout ** 0.5)
    w1 = torch.randn(cout, c, 1, 1, device=cuda, generator=g) / cout ** 0.5
    dh = torch.randn(B, cout, HO, HO, device=cuda, generator=g)
    dz = torch.randn(B, cout, HO, HO, device=cuda, generator=g)
    p3 = _capi.conv3x3_pack(w3, transpose_flip=True)
    p1 = _capi.conv1x1_pack(w1, transpose=True)
    a = _capi.down_backward(dh, p3, c, dz=dz, packed1x1_t=p1, mask_src=y)
    b = _capi.down_backward(dh, p3, c, dz=dz, packed1x1_t=p1, mask_bits=bits)
    assert torch.equal(a, b)


def test_down_backward_mask_bits_refused_off_the_128_position_kernel(cuda):
    """A 12x16 output (down::geometry accepts it) runs the general backward kernel, which reads
    only mask_src: mask_bits there must raise, not return dx without the ReLU mask (ADVICE
    r04), and GraNd's helper must send such shapes to mask_src."""
    B, c, HO, WO = 2, 64, 12, 16
    assert not _capi.down_backward_mask_bits_supported(HO, WO)
    assert _capi.down_backward_mask_bits_supported(16, 16)
    assert _capi.down_backward_mask_bits_supported(8, 8)
    assert _capi.down_backward_mask_bits_supported(4, 4)
    w3 = torch.randn(2 * c, c, 3, 3, device=cuda) / (3 * c)
    dh = torch.randn(B, 2 * c, HO, WO, device=cuda)
    bits = torch.zeros(B * c * 4 * HO * WO // 32, dtype=torch.int32, device=cuda)
    p3 = _capi.conv3x3_pack(w3, transpose_flip=True)
    with pytest.raises(_capi.DDError, match="mask_bits needs the 128-position kernel"):
        _capi.down_backward(dh, p3, c, mask_bits=bits)
    # the mask_src form of the same shape runs and is correct
    mask = torch.randn(B, c, 2 * HO, 2 * WO, device=cuda)
    got = _capi.down_backward(dh, p3, c, mask_src=mask)
    want = torch.nn.grad.conv2d_input((B, c, 2 * HO, 2 * WO), w3.cpu(), dh.cpu(), stride=2,
                                      padding=1) * (mask.cpu() > 0)
    _close(got, want)
