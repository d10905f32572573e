"""fp16 operand halves (DD_OPERANDS_F16X3) of the split-MFMA forward convs, the EL2N forward's
arithmetic: every forward entry point (3x3, 1x1, downsampling head, implicit-GEMM kh x kw, and
the fused unit-input forms) against a float64 PyTorch reference of the same op.

Tolerance: fp16 halves keep 22 significant bits per operand (~2^-22 relative per product, fp32
accumulation), so the max error over the max-abs output is held to 2e-6 and to at most half
the bf16-halves kernel's on the same inputs (bf16 halves: ~2^-17 per product).  At fp16's
precision the fp32 accumulation over K = 576-4608 terms in the kernel's order is a comparable
share of what is left: measured 7.3e-7 (fp16) against 4.6e-6 (bf16) at 64 -> 64 on 32x32,
1.3e-6 against 4.5e-6 at 256 -> 256 on 8x8, where PyTorch's fp32 CPU conv (blocked sums)
reaches 2.9e-7.
"""
import pytest
import torch
import torch.nn.functional as F

from data_diet_distributed_amd import _capi

pytestmark = pytest.mark.gpu

F16_REL = 2e-6


def _err(got, want):
    return ((got.detach().cpu().double() - want).abs().max() / want.abs().max()).item()


def _check(errs, e32):
    """fp16 halves: within F16_REL and at most half the bf16 halves' error (e32: PyTorch's
    fp32 CPU conv, reported beside them)."""
    assert errs["f16x3"] <= F16_REL, (errs, e32)
    assert errs["f16x3"] <= 0.5 * errs["bf16x3"], (errs, e32)


SHAPES = [(4, 64, 64, 32, 32), (3, 128, 128, 16, 16), (2, 256, 256, 8, 8), (5, 512, 512, 4, 4),
          (3, 3, 64, 32, 32), (2, 20, 70, 16, 16), (2, 64, 130, 8, 8), (3, 100, 200, 8, 8)]


@pytest.mark.parametrize("B,cin,cout,H,W", SHAPES)
def test_conv3x3_f16_forward(cuda, B, cin, cout, H, W):
    g = torch.Generator().manual_seed(B * cin + cout + 1)
    x = torch.randn(B, cin, H, W, generator=g)
    w = torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)
    want = F.conv2d(x.double(), w.double(), padding=1)
    errs = {}
    for ops in ("f16x3", "bf16x3"):
        pk = _capi.conv3x3_pack(w.to(cuda), operands=ops)
        assert _capi.pack_operands(pk) == _capi.OPERANDS[ops]
        errs[ops] = _err(_capi.conv3x3(x.to(cuda), pk, cout), want)
    _check(errs, _err(F.conv2d(x, w, padding=1), want))


@pytest.mark.parametrize("B,cin,cout,H,W", [(256, 64, 64, 32, 32), (256, 128, 128, 16, 16),
                                             (256, 256, 256, 8, 8), (256, 512, 512, 4, 4)])
def test_conv3x3_f16_grouped_stats(cuda, B, cin, cout, H, W):
    """The EL2N launch shape: the producer's grouped BN + ReLU staged, BN partial statistics out
    (groups of 128), in fp16 halves; y and the finalized (scale, shift) against float64."""
    g = torch.Generator().manual_seed(cin + H)
    gs = 128
    G = B // gs
    x = torch.randn(B, cin, H, W, generator=g)
    w = torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)
    sc = torch.rand(G, cin, generator=g) + 0.5
    sh = torch.randn(G, cin, generator=g) * 0.2
    xf = torch.relu(x * sc.repeat_interleave(gs, 0)[:, :, None, None]
                    + sh.repeat_interleave(gs, 0)[:, :, None, None])
    want = F.conv2d(xf.double(), w.double(), padding=1)
    pk = _capi.conv3x3_pack(w.to(cuda), operands="f16x3")
    y, st = _capi.conv3x3(x.to(cuda), pk, cout, in_affine=(sc.to(cuda), sh.to(cuda)),
                          group_size=gs, stats=True)
    assert _err(y, want) <= F16_REL
    gamma = torch.rand(cout, device=cuda) + 0.5
    beta = torch.randn(cout, device=cuda)
    scale, shift = _capi.bn_finalize(st, gamma, beta, 1e-5)
    yg = want.reshape(G, gs, cout, H * W)
    var = yg.var(dim=(1, 3), unbiased=False)
    mean = yg.mean(dim=(1, 3))
    rs = gamma.double().cpu() / torch.sqrt(var + 1e-5)
    assert torch.allclose(scale.cpu().double(), rs, rtol=2e-5)
    assert torch.allclose(shift.cpu().double(), beta.double().cpu() - mean * rs, rtol=2e-5,
                          atol=2e-5)


@pytest.mark.parametrize("H,cin,cout,res_kind", [(32, 64, 64, "none"), (32, 64, 64, "identity"),
                                                  (16, 128, 128, "bn"), (8, 256, 256, "identity")])
def test_conv3x3_f16_unit_input_is_bn_apply_then_conv(cuda, H, cin, cout, res_kind):
    """The fused unit input in fp16 halves is bitwise bn_apply followed by the fp16 conv."""
    B, gs = 256, 128
    G = B // gs
    g = torch.Generator(device=cuda).manual_seed(H + cin)
    yp = torch.randn(B, cin, H, H, device=cuda, generator=g)
    aff = (torch.rand(G * cin, device=cuda, generator=g) + 0.5,
           torch.randn(G * cin, device=cuda, generator=g) * 0.1)
    res = torch.randn(B, cin, H, H, device=cuda, generator=g) if res_kind != "none" else None
    raff = ((torch.rand(G * cin, device=cuda, generator=g) + 0.5,
             torch.randn(G * cin, device=cuda, generator=g) * 0.1) if res_kind == "bn" else None)
    w = torch.randn(cout, cin, 3, 3, device=cuda, generator=g) / (3 * cin ** 0.5)
    pk = _capi.conv3x3_pack(w, operands="f16x3")
    assert _capi.conv3x3_unit_input_supported(H, H, cin, cout, gs)
    xo, y, st = _capi.conv3x3_unit_input(yp, aff, pk, cout, gs, residual=res, res_affine=raff)
    a, _ = _capi.bn_apply(yp, aff, gs, residual=res, res_affine=raff, relu=True)
    y2, st2 = _capi.conv3x3(a, pk, cout, group_size=gs, stats=True)
    assert torch.equal(xo, a)
    assert torch.equal(y, y2)
    assert torch.equal(st.buf, st2.buf)


@pytest.mark.parametrize("B,cin,cout,H,stride", [(4, 256, 64, 32, 1), (4, 64, 256, 32, 1),
                                                  (2, 1024, 256, 8, 1), (2, 512, 2048, 4, 1),
                                                  (3, 256, 512, 32, 2), (3, 70, 90, 6, 1)])
def test_conv1x1_f16_forward(cuda, B, cin, cout, H, stride):
    g = torch.Generator().manual_seed(cin + cout + stride)
    x = torch.randn(B, cin, H, H, generator=g)
    w = torch.randn(cout, cin, generator=g) / cin ** 0.5
    want = F.conv2d(x.double(), w.double()[:, :, None, None], stride=stride)
    errs = {}
    for ops in ("f16x3", "bf16x3"):
        pk = _capi.conv1x1_pack(w.to(cuda), operands=ops)
        errs[ops] = _err(_capi.conv1x1(x.to(cuda), pk, cout, stride=stride), want)
    _check(errs, _err(F.conv2d(x, w[:, :, None, None], stride=stride), want))


@pytest.mark.parametrize("B,cin,cout,HI", [(3, 64, 128, 32), (2, 128, 256, 16), (8, 256, 512, 8),
                                            (2, 64, 64, 64)])
def test_down_f16_forward(cuda, B, cin, cout, HI):
    g = torch.Generator().manual_seed(HI + cout)
    x = torch.randn(B, cin, HI, HI, generator=g)
    w3 = torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)
    w1 = torch.randn(cout, cin, 1, 1, generator=g) / cin ** 0.5
    want = F.conv2d(x.double(), w3.double(), stride=2, padding=1)
    want_s = F.conv2d(x.double(), w1.double(), stride=2)
    p3 = _capi.conv3x3_pack(w3.to(cuda), operands="f16x3")
    p1 = _capi.conv1x1_pack(w1.to(cuda), operands="f16x3")
    y, ys, _, _ = _capi.conv_down(x.to(cuda), p3, cout, p1)
    assert _err(y, want) <= F16_REL and _err(ys, want_s) <= F16_REL
    # the statistics launch (EL2N) and the 3x3-only form (a Bottleneck's stride-2 conv2)
    gs = 4 if HI == 8 else 1
    y2, ys2, st, sts = _capi.conv_down(x.to(cuda), p3, cout, p1, group_size=gs * (B // gs),
                                       stats=True)
    assert _err(y2, want) <= F16_REL and _err(ys2, want_s) <= F16_REL
    y3, _, _, _ = _capi.conv_down(x.to(cuda), p3, cout)
    assert _err(y3, want) <= F16_REL
    with pytest.raises(ValueError, match="same operands"):
        _capi.conv_down(x.to(cuda), p3, cout, _capi.conv1x1_pack(w1.to(cuda)))


@pytest.mark.parametrize("HI,cin,cout,unit", [(32, 64, 128, True), (16, 128, 256, True),
                                               (8, 256, 512, True), (32, 128, 128, False)])
def test_down_f16_unit_input_is_bn_apply_then_down(cuda, HI, cin, cout, unit):
    B, gs = 256, 128
    G = B // gs
    g = torch.Generator(device=cuda).manual_seed(HI + cin + 1)
    yp = torch.randn(B, cin, HI, HI, device=cuda, generator=g)
    aff = (torch.rand(G * cin, device=cuda, generator=g) + 0.5,
           torch.randn(G * cin, device=cuda, generator=g) * 0.1)
    res = torch.randn(B, cin, HI, HI, device=cuda, generator=g) if unit else None
    w3 = torch.randn(cout, cin, 3, 3, device=cuda, generator=g) / (3 * cin ** 0.5)
    w1 = torch.randn(cout, cin, 1, 1, device=cuda, generator=g) / cin ** 0.5
    p3 = _capi.conv3x3_pack(w3, operands="f16x3")
    p1 = _capi.conv1x1_pack(w1, operands="f16x3") if unit else None
    y, ys, st, sts = _capi.conv_down_unit_input(yp, aff, p3, cout, gs, packed1x1=p1,
                                                residual=res)
    a, _ = _capi.bn_apply(yp, aff, gs, residual=res, relu=True)
    y2, ys2, st2, sts2 = _capi.conv_down(a, p3, cout, p1, group_size=gs, stats=True)
    assert torch.equal(y, y2) and torch.equal(st.buf, st2.buf)
    if unit:
        assert torch.equal(ys, ys2) and torch.equal(sts.buf, sts2.buf)


@pytest.mark.parametrize("cin,cout,k,stride,pad,H", [(3, 64, 7, 2, 3, 56), (64, 64, 3, 1, 1, 14),
                                                      (128, 128, 3, 2, 1, 14)])
def test_conv_gemm_f16_forward(cuda, cin, cout, k, stride, pad, H):
    g = torch.Generator().manual_seed(cin + k)
    B = 2
    x = torch.randn(B, cin, H, H, generator=g)
    w = torch.randn(cout, cin, k, k, generator=g) / (k * cin ** 0.5)
    want = F.conv2d(x.double(), w.double(), stride=stride, padding=pad)
    errs = {}
    for ops in ("f16x3", "bf16x3"):
        pk = _capi.conv_gemm_pack(w.to(cuda), operands=ops)
        errs[ops] = _err(_capi.conv_gemm(x.to(cuda), pk, cout, k, stride, pad), want)
    _check(errs, _err(F.conv2d(x, w, stride=stride, padding=pad), want))


def test_operands_code_is_checked(cuda):
    w = torch.randn(64, 64, 3, 3, device=cuda)
    with pytest.raises(ValueError, match="operands must be one of"):
        _capi.conv3x3_pack(w, operands="fp8")
    L = _capi.lib()
    import ctypes
    pk = torch.empty(L.dd_conv3x3_pack_bytes(64, 64), dtype=torch.uint8, device=cuda)
    rc = L.dd_conv3x3_pack(ctypes.c_void_p(w.data_ptr()), 64, 64, 0, 7, 1.0,
                           ctypes.c_void_p(pk.data_ptr()), None)
    assert rc == -1 and b"operands" in L.dd_last_error()  # DD_EINVAL


def test_f16_pack_scale_is_a_power_of_two_and_exact(cuda):
    """fp16 packs hold W * 2^s with max|W| * 2^s in [2^12, 2^13) and the forward multiplies
    the accumulators by 2^-s: small weights keep their lo halves normal (a pack of W * 1e-4
    gives the same relative error as one of W), and bf16 packs are unscaled."""
    g = torch.Generator().manual_seed(9)
    x = torch.randn(2, 64, 16, 16, generator=g)
    w = torch.randn(128, 64, 3, 3, generator=g) / 24
    errs = []
    for f in (1.0, 1e-4, 1e3):
        pk = _capi.conv3x3_pack((w * f).to(cuda), operands="f16x3")
        s = pk.dd_scale
        import math
        assert math.frexp(s)[0] == 0.5 and 2 ** 12 <= float((w * f).abs().max()) * s < 2 ** 13
        want = F.conv2d(x.double(), (w * f).double(), padding=1)
        errs.append(_err(_capi.conv3x3(x.to(cuda), pk, 128), want))
    assert max(errs) <= F16_REL and max(errs) <= 3 * min(errs), errs
    assert _capi.conv3x3_pack(w.to(cuda)).dd_scale == 1.0


def test_a_copied_pack_without_its_tag_is_refused(cuda):
    """a pack's operand code and scale live on the tensor as attributes, which
    clone() / .to() / slicing drop.  A copy must not be read as an unscaled bf16 pack (an fp16
    pack of W * 2^s would then run as garbage with no error): the launch raises DDError."""
    w = torch.randn(64, 64, 3, 3, generator=torch.Generator().manual_seed(3)).to(cuda) / 24
    x = torch.randn(2, 64, 16, 16, device=cuda)
    for op in ("f16x3", "bf16x3"):
        pk = _capi.conv3x3_pack(w, operands=op)
        _capi.conv3x3(x, pk, 64)
        with pytest.raises(_capi.DDError, match="operand tag"):
            _capi.conv3x3(x, pk.clone(), 64)
