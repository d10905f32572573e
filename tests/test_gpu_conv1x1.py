"""1x1 convolution (split-bf16 GEMM, dd_conv1x1_forward) vs PyTorch fp32 on the CPU.

Floating-point kernel: the checker is a plain fp32 PyTorch reference of the same op.  Tolerance
as for the 3x3 kernel: split-bf16 products carry ~2^-16 relative error; 5e-4 relative on the
max-abs.  Shapes: every 1x1 conv of ResNet-50 at CIFAR and ImageNet sizes (T = 1024 .. 16 and
3136 .. 49 positions, stride 1 and 2), plus ragged channel / batch counts.
"""
import pytest
import torch
import torch.nn.functional as F

from data_diet_distributed_amd import _capi

pytestmark = pytest.mark.gpu

# (B, cin, cout, H, W, stride)
SHAPES = [(3, 64, 64, 32, 32, 1), (2, 64, 256, 32, 32, 1), (2, 256, 64, 32, 32, 1),
          (2, 256, 512, 32, 32, 2), (3, 512, 128, 16, 16, 1), (2, 128, 512, 16, 16, 1),
          (4, 1024, 256, 8, 8, 1), (3, 512, 1024, 16, 16, 2), (9, 2048, 512, 4, 4, 1),
          (5, 512, 2048, 4, 4, 1), (3, 1024, 2048, 8, 8, 2), (2, 64, 256, 56, 56, 1),
          (3, 1024, 512, 14, 14, 1), (4, 2048, 512, 7, 7, 1), (3, 1024, 2048, 14, 14, 2),
          (5, 48, 70, 6, 10, 1), (3, 40, 200, 6, 6, 2), (1, 16, 16, 3, 3, 1),
          (3, 512, 1024, 28, 28, 2), (2, 96, 64, 12, 20, 2)]


def _close(got, want, rel=5e-4):
    err = (got.cpu() - want).abs().max().item()
    scale = want.abs().max().item()
    assert err <= rel * scale + 1e-6, (err, scale)


@pytest.mark.parametrize("B,cin,cout,H,W,s", SHAPES)
def test_conv1x1_forward(cuda, B, cin, cout, H, W, s):
    g = torch.Generator().manual_seed(B * cin + cout + H)
    x = torch.randn(B, cin, H, W, generator=g)
    w = torch.randn(cout, cin, 1, 1, generator=g) / cin ** 0.5
    want = F.conv2d(x, w, stride=s)
    pk = _capi.conv1x1_pack(w.to(cuda))
    _close(_capi.conv1x1(x.to(cuda), pk, cout, stride=s), want)
    # fused epilogue: bias + residual + ReLU; then residual + mask
    bias = torch.randn(cout, generator=g)
    res = torch.randn(want.shape, generator=g)
    got = _capi.conv1x1(x.to(cuda), pk, cout, stride=s, bias=bias.to(cuda),
                        residual=res.to(cuda), relu=True)
    _close(got, F.relu(want + bias[None, :, None, None] + res))
    mask = torch.randn(want.shape, generator=g)
    got = _capi.conv1x1(x.to(cuda), pk, cout, stride=s, residual=res.to(cuda),
                        mask_src=mask.to(cuda))
    _close(got, (want + res) * (mask > 0))


@pytest.mark.parametrize("B,cin,cout,H,W,s", SHAPES)
def test_conv1x1_backward_data(cuda, B, cin, cout, H, W, s):
    """transpose pack: dx = W^T dy (stride 1); at stride 2 the GEMM runs on the decimated
    grid and its result is the res_up2 operand of a full-resolution launch."""
    g = torch.Generator().manual_seed(3 * B + cin + cout)
    w = torch.randn(cout, cin, 1, 1, generator=g) / cout ** 0.5
    Ho, Wo = H // s, W // s
    dy = torch.randn(B, cout, Ho, Wo, generator=g)
    want = torch.nn.grad.conv2d_input((B, cin, H, W), w, dy, stride=s)
    pkt = _capi.conv1x1_pack(w.to(cuda), transpose=True)
    small = _capi.conv1x1(dy.to(cuda), pkt, cin)  # W^T dy at the output grid
    if s == 1:
        _close(small, want)
        return
    # stride 2: dx = up2(W^T dy), here added to a full-resolution conv of another input
    # (the Bottleneck block-input gradient: conv1^T(dh) + shortcut^T(dz)) and masked
    w1 = torch.randn(24, cin, 1, 1, generator=g) / 24 ** 0.5  # conv1: cin -> 24
    dh = torch.randn(B, 24, H, W, generator=g)
    mask = torch.randn(B, cin, H, W, generator=g)
    full = _capi.conv1x1(dh.to(cuda), _capi.conv1x1_pack(w1.to(cuda), transpose=True), cin,
                         res_up2=small, mask_src=mask.to(cuda))
    want_full = (torch.nn.grad.conv2d_input((B, cin, H, W), w1, dh) + want) * (mask > 0)
    _close(full, want_full)


# more tiles than resident workgroups, so every persistent workgroup walks several tiles (the
# 256-output tiles: one workgroup per CU, the two-chunk prefetch stream crossing tile ends),
# with an odd chunk count (96 channels = 3 K chunks) and a ragged tail
MANY_TILES = [(300, 96, 256, 16, 16, 1), (160, 256, 512, 16, 16, 1),
              (100, 1024, 2048, 8, 8, 2), (600, 512, 2048, 4, 4, 1)]


@pytest.mark.parametrize("B,cin,cout,H,W,s", MANY_TILES)
def test_conv1x1_forward_many_tiles(cuda, B, cin, cout, H, W, s):
    g = torch.Generator().manual_seed(7 * B + cin + cout)
    x = torch.randn(B, cin, H, W, generator=g)
    w = torch.randn(cout, cin, 1, 1, generator=g) / cin ** 0.5
    want = F.conv2d(x, w, stride=s)
    pk = _capi.conv1x1_pack(w.to(cuda))
    _close(_capi.conv1x1(x.to(cuda), pk, cout, stride=s), want)


@pytest.mark.parametrize("B,cin,cout,H,W,s,gs", [(256, 64, 128, 16, 16, 1, 128),
                                                 (256, 128, 256, 8, 8, 2, 128),
                                                 (64, 256, 64, 4, 4, 1, 32),
                                                 (130, 64, 64, 32, 32, 1, 128),
                                                 (700, 96, 256, 8, 8, 1, 128)])
def test_conv1x1_grouped_bn(cuda, B, cin, cout, H, W, s, gs):
    """Staging transform (the producer's grouped train-mode BN + ReLU) and BN statistics of
    the output per group, over the valid rows only (ragged last group), finalized by
    dd_bn_finalize: equals torch batch-norm of each group."""
    g = torch.Generator().manual_seed(B + cin)
    G = -(-B // gs)
    x = torch.randn(B, cin, H, W, generator=g)
    w = torch.randn(cout, cin, 1, 1, generator=g) / cin ** 0.5
    sc = torch.rand(G, cin, generator=g) + 0.5
    sh = torch.randn(G, cin, generator=g)
    xf = torch.relu(x * sc.repeat_interleave(gs, 0)[:B, :, None, None]
                    + sh.repeat_interleave(gs, 0)[:B, :, None, None])
    want = F.conv2d(xf, w, stride=s)
    pk = _capi.conv1x1_pack(w.to(cuda))
    n_valid = B - 1 if B % gs else B  # a ragged last group with one example left out
    y, st = _capi.conv1x1(x.to(cuda), pk, cout, stride=s, in_affine=(sc.to(cuda), sh.to(cuda)),
                          group_size=gs, stats=True, n_stat=n_valid)
    _close(y, want)
    gamma = torch.rand(cout, generator=g) + 0.5
    beta = torch.randn(cout, generator=g)
    scale, shift = _capi.bn_finalize(st, gamma.to(cuda), beta.to(cuda), 1e-5)
    for gi in range(G):
        lo, hi = gi * gs, min(n_valid, (gi + 1) * gs)
        if hi <= lo:
            continue
        yg = want[lo:hi]
        mean = yg.mean(dim=(0, 2, 3))
        var = yg.var(dim=(0, 2, 3), unbiased=False)
        s_ref = gamma / torch.sqrt(var + 1e-5)
        torch.testing.assert_close(scale[gi].cpu(), s_ref, rtol=2e-4, atol=1e-5)
        torch.testing.assert_close(shift[gi].cpu(), beta - mean * s_ref, rtol=2e-4, atol=2e-4)


def test_conv1x1_bad_args(cuda):
    pk = _capi.conv1x1_pack(torch.randn(8, 8, 1, 1, device=cuda))
    with pytest.raises(_capi.DDError, match="stride"):
        _capi.lib()  # loaded
        rc = _capi.lib().dd_conv1x1_forward(None, 1, 8, 4, 4, 3, None, 8, None, None, None,
                                            None, 0, None, None, 0, 0, 0, None, None, 0, 1.0, None)
        _capi._check(rc, "dd_conv1x1_forward")
    with pytest.raises(_capi.DDError, match="no 1x1 stats layout"):
        _capi.conv1x1(torch.randn(3, 8, 5, 5, device=cuda), pk, 8, stats=True, group_size=3)


# any kh x kw (dd_conv_gemm_forward): (B, cin, cout, H, W, k, stride, pad) -- the ResNet-50
# ImageNet-stem convs (7x7/2 stem at 224, 3x3 at 56 / 28 / 14 / 7 stride 1 and the stride-2
# 3x3 of each stage head) at small batch, plus ragged shapes and a dense-K 5x5
GEMM_SHAPES = [(2, 3, 64, 224, 224, 7, 2, 3), (2, 64, 64, 56, 56, 3, 1, 1),
               (2, 128, 128, 28, 28, 3, 1, 1), (3, 256, 256, 14, 14, 3, 1, 1),
               (4, 512, 512, 7, 7, 3, 1, 1), (2, 128, 128, 56, 56, 3, 2, 1),
               (3, 256, 256, 28, 28, 3, 2, 1), (4, 512, 512, 14, 14, 3, 2, 1),
               (3, 40, 70, 9, 11, 3, 1, 1), (2, 5, 24, 13, 10, 5, 2, 2), (3, 48, 64, 7, 7, 3, 2, 0),
               (2, 3, 16, 32, 32, 3, 1, 1)]


@pytest.mark.parametrize("B,cin,cout,H,W,k,s,p", GEMM_SHAPES)
def test_conv_gemm_forward(cuda, B, cin, cout, H, W, k, s, p):
    g = torch.Generator().manual_seed(B + cin * k + cout + H)
    x = torch.randn(B, cin, H, W, generator=g)
    w = torch.randn(cout, cin, k, k, generator=g) / (cin * k * k) ** 0.5
    want = F.conv2d(x, w, stride=s, padding=p)
    pk = _capi.conv_gemm_pack(w.to(cuda))
    assert pk.numel() == _capi.lib().dd_conv_gemm_pack_bytes(cout, cin, k, k)
    _close(_capi.conv_gemm(x.to(cuda), pk, cout, k, s, p), want)
    bias = torch.randn(cout, generator=g)
    res = torch.randn(want.shape, generator=g)
    got = _capi.conv_gemm(x.to(cuda), pk, cout, k, s, p, bias=bias.to(cuda),
                          residual=res.to(cuda), relu=True)
    _close(got, F.relu(want + bias[None, :, None, None] + res))


# group_size * ho * wo must be a multiple of 128 (a 128-position tile inside one group): at 7x7
# that is the reference's batch of 128
@pytest.mark.parametrize("B,cin,cout,H,W,k,s,p,gs", [(130, 64, 64, 14, 14, 3, 1, 1, 64),
                                                     (100, 128, 128, 14, 14, 3, 2, 1, 128),
                                                     (140, 256, 64, 7, 7, 3, 1, 1, 128),
                                                     (40, 3, 64, 56, 56, 7, 2, 3, 16)])
def test_conv_gemm_grouped_bn(cuda, B, cin, cout, H, W, k, s, p, gs):
    """Grouped train-mode BN around the GEMM conv: the producer's BN + ReLU applied while
    staging (before the zero padding), and per-group statistics of the output at map sizes
    whose 32-position partials straddle examples (7x7, 14x14, 28x28)."""
    g = torch.Generator().manual_seed(B * k + cin)
    G = -(-B // gs)
    x = torch.randn(B, cin, H, W, generator=g)
    w = torch.randn(cout, cin, k, k, generator=g) / (cin * k * k) ** 0.5
    dense = _capi.lib().dd_conv_gemm_dense(cin, k, k) == 1
    if dense:  # a dense-K pack (the stem) reads the network input: no staging transform
        xf, aff = x, None
    else:
        sc = torch.rand(G, cin, generator=g) + 0.5
        sh = torch.randn(G, cin, generator=g)
        xf = torch.relu(x * sc.repeat_interleave(gs, 0)[:B, :, None, None]
                        + sh.repeat_interleave(gs, 0)[:B, :, None, None])
        aff = (sc.to(cuda), sh.to(cuda))
    want = F.conv2d(xf, w, stride=s, padding=p)
    pk = _capi.conv_gemm_pack(w.to(cuda))
    n_valid = B - 1 if B % gs else B
    y, st = _capi.conv_gemm(x.to(cuda), pk, cout, k, s, p, in_affine=aff, group_size=gs,
                            stats=True, n_stat=n_valid)
    _close(y, want)
    gamma = torch.rand(cout, generator=g) + 0.5
    beta = torch.randn(cout, generator=g)
    scale, shift = _capi.bn_finalize(st, gamma.to(cuda), beta.to(cuda), 1e-5)
    for gi in range(G):
        lo, hi = gi * gs, min(n_valid, (gi + 1) * gs)
        if hi <= lo:
            continue
        yg = want[lo:hi]
        mean = yg.mean(dim=(0, 2, 3))
        var = yg.var(dim=(0, 2, 3), unbiased=False)
        s_ref = gamma / torch.sqrt(var + 1e-5)
        torch.testing.assert_close(scale[gi].cpu(), s_ref, rtol=2e-4, atol=1e-5)
        torch.testing.assert_close(shift[gi].cpu(), beta - mean * s_ref, rtol=2e-4, atol=2e-4)


@pytest.mark.parametrize("hw", [7, 14, 28])
def test_conv1x1_stats_straddling(cuda, hw):
    """1x1 BN statistics at ImageNet map sizes (49 / 196 / 784 positions: a 32-position
    partial spans two examples), ragged last group."""
    B, cin, cout, gs = (140, 64, 128, 128) if hw == 7 else (70, 64, 128, 32)
    g = torch.Generator().manual_seed(hw)
    x = torch.randn(B, cin, hw, hw, generator=g)
    w = torch.randn(cout, cin, 1, 1, generator=g) / cin ** 0.5
    want = F.conv2d(x, w)
    y, st = _capi.conv1x1(x.to(cuda), _capi.conv1x1_pack(w.to(cuda)), cout, group_size=gs,
                          stats=True, n_stat=B - 3)
    _close(y, want)
    ones, zeros = torch.ones(cout, device=cuda), torch.zeros(cout, device=cuda)
    scale, shift = _capi.bn_finalize(st, ones, zeros, 1e-5)
    for gi in range(-(-B // gs)):
        lo, hi = gi * gs, min(B - 3, (gi + 1) * gs)
        yg = want[lo:hi]
        s_ref = 1 / torch.sqrt(yg.var(dim=(0, 2, 3), unbiased=False) + 1e-5)
        torch.testing.assert_close(scale[gi].cpu(), s_ref, rtol=2e-4, atol=1e-5)
        torch.testing.assert_close(shift[gi].cpu(), -yg.mean(dim=(0, 2, 3)) * s_ref, rtol=2e-4,
                                   atol=2e-4)


@pytest.mark.parametrize("B,cin,H,gs", [(3, 64, 56, 2), (4, 32, 64, 1)])
def test_conv_gemm_row_quads_equal_the_tap_gather(cuda, monkeypatch, B, cin, H, gs):
    """MODE 4 (3x3 / stride 1 at a width that is a multiple of 4: one float4 of the tap's input
    row per quad of outputs, plus the edge column) stages exactly MODE 2's values in MODE 2's
    K order: outputs and BN partial statistics bitwise equal, with the producer's BN + ReLU
    staged (the padding zeroed after it), on tiles that span two examples and a ragged last
    BN group; and within the split-fp16 bar of float64."""
    g = torch.Generator().manual_seed(B * H)
    G = -(-B // gs)
    x = torch.randn(B, cin, H, H, generator=g)
    w = torch.randn(cin, cin, 3, 3, generator=g) / (cin * 9) ** 0.5
    sc = torch.rand(G, cin, generator=g) + 0.5
    sh = torch.randn(G, cin, generator=g)
    xf = torch.relu(x * sc.repeat_interleave(gs, 0)[:B, :, None, None]
                    + sh.repeat_interleave(gs, 0)[:B, :, None, None])
    want = F.conv2d(xf.double(), w.double(), padding=1)
    pk = _capi.conv_gemm_pack(w.to(cuda), operands="f16x3")
    out = {}
    for rowq in ("0", "1"):
        monkeypatch.setenv("DD_C1_ROWQ", rowq)
        y, st = _capi.conv_gemm(x.to(cuda), pk, cin, 3, 1, 1, in_affine=(sc.to(cuda), sh.to(cuda)),
                                group_size=gs, stats=True, n_stat=B - 1)
        ones, zeros = torch.ones(cin, device=cuda), torch.zeros(cin, device=cuda)
        scale, shift = _capi.bn_finalize(st, ones, zeros, 1e-5)  # (the written partials only)
        out[rowq] = (y.cpu(), scale.cpu(), shift.cpu())
    assert all(torch.equal(a, b) for a, b in zip(out["0"], out["1"]))
    err = float(((out["1"][0].double() - want).abs().max() / want.abs().max()))
    assert err < 2e-6, err
