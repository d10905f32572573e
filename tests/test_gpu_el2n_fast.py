"""Grouped train-mode BatchNorm kernels and the hand-scheduled EL2N forward vs PyTorch fp32.

Floating-point kernels, so the checkers are plain fp32 PyTorch references of the same ops
(F.conv2d / F.batch_norm(training=True) per group, computed on the CPU).  Tolerances: the
split-bf16 conv carries ~2^-16 relative per product (5e-4 of the max-abs as in
test_gpu_conv.py); BN statistics are summed in double (1e-5); logits of the whole network
1e-3 relative to their max-abs (the north-star bar for scores is 1e-3 relative).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from data_diet_distributed_amd import _capi, checkpoints, el2n_fast, synthetic
from data_diet_distributed_amd.scoring import ScoreConfig, ScoringEngine
from oracle import pipeline as o_pipe

pytestmark = pytest.mark.gpu


def _close(got, want, rel=5e-4):
    got = got.detach().cpu().double()
    want = want.detach().cpu().double()
    err = (got - want).abs().max().item()
    scale = want.abs().max().item()
    assert err <= rel * scale + 1e-6, (err, scale)


def _group_bn_ref(y, gs, n_valid, gamma, beta, eps=1e-5):
    """Per-group train-mode BN affine (scale, shift) of y (CPU fp64) over rows < n_valid."""
    B, C = y.shape[:2]
    G = -(-B // gs)
    sc = torch.zeros(G, C, dtype=torch.float64)
    sh = torch.zeros(G, C, dtype=torch.float64)
    for g in range(G):
        lo, hi = g * gs, min(B, (g + 1) * gs, max(n_valid, 0))
        if hi <= lo:
            continue
        v = y[lo:hi].double()
        mean = v.mean(dim=(0, 2, 3))
        var = v.var(dim=(0, 2, 3), unbiased=False)
        sc[g] = gamma.double() / torch.sqrt(var + eps)
        sh[g] = beta.double() - mean * sc[g]
    return sc, sh


@pytest.mark.parametrize("B,cin,cout,H,W,gs,n_valid", [
    (6, 64, 64, 32, 32, 2, 5), (8, 128, 128, 16, 16, 4, 8), (8, 256, 256, 8, 8, 4, 7),
    (12, 512, 512, 4, 4, 4, 10), (6, 3, 64, 32, 32, 3, 6), (5, 64, 96, 8, 8, 3, 5)])
def test_conv3x3_input_affine_and_stats(cuda, B, cin, cout, H, W, gs, n_valid):
    g = torch.Generator().manual_seed(B * cin + cout + H)
    G = -(-B // gs)
    x = torch.randn(B, cin, H, W, generator=g)
    w = torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)
    s_in = torch.rand(G, cin, generator=g) + 0.5
    t_in = torch.randn(G, cin, generator=g) * 0.3
    xin = torch.relu(x * s_in.repeat_interleave(gs, 0)[:B, :, None, None] +
                     t_in.repeat_interleave(gs, 0)[:B, :, None, None])
    want = F.conv2d(xin, w, padding=1)
    packed = _capi.conv3x3_pack(w.to(cuda))
    y, st = _capi.conv3x3(x.to(cuda), packed, cout, in_affine=(s_in.to(cuda), t_in.to(cuda)),
                          group_size=gs, stats=True, n_stat=n_valid)
    _close(y, want)
    gamma = torch.rand(cout, generator=g) + 0.5
    beta = torch.randn(cout, generator=g)
    sc, sh = _capi.bn_finalize(st, gamma.to(cuda), beta.to(cuda), 1e-5)
    rsc, rsh = _group_bn_ref(want, gs, n_valid, gamma, beta)
    _close(sc, rsc, 2e-4)
    _close(sh, rsh, 2e-4)


# padded-width tiles (dd_conv3x3_forward ABI 10): the ImageNet-stem network's 56 / 28 / 14 / 7
# maps and ragged cases -- an overhanging last row block (37, 27, 13 rows), a width past 16 that is
# not a tile width (20), a 6 x 5 map two to a tile, 200 outputs in a padded 256-output grid --
# with and without the producer's BN staged, in both operand types
PW_SHAPES = [(3, 64, 64, 56, 56, 2, 3), (3, 40, 96, 37, 44, 2, 2), (5, 128, 128, 28, 28, 2, 5), (4, 256, 256, 14, 14, 2, 3), (6, 512, 512, 7, 7, 2, 5),
             (3, 96, 200, 13, 14, 3, 3), (5, 64, 128, 27, 20, 5, 4), (4, 48, 128, 5, 6, 2, 4)]


@pytest.mark.parametrize("operands", ["f16x3", "bf16x3"])
@pytest.mark.parametrize("affine", [True, False])
@pytest.mark.parametrize("B,cin,cout,H,W,gs,n_valid", PW_SHAPES)
def test_conv3x3_padded_width_stats(cuda, B, cin, cout, H, W, gs, n_valid, affine, operands):
    assert _capi.conv3x3_padded_supported(H, W, cin, cout, gs)
    g = torch.Generator().manual_seed(B * cin + cout + H + W)
    G = -(-B // gs)
    x = torch.randn(B, cin, H, W, generator=g)
    w = torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)
    s_in = torch.rand(G, cin, generator=g) + 0.5
    t_in = torch.randn(G, cin, generator=g) * 0.3
    xin = x
    if affine:
        xin = torch.relu(x * s_in.repeat_interleave(gs, 0)[:B, :, None, None] +
                         t_in.repeat_interleave(gs, 0)[:B, :, None, None])
    want = F.conv2d(xin.double(), w.double(), padding=1)
    packed = _capi.conv3x3_pack(w.to(cuda), operands=operands)
    # poisoned output: every (example, channel, position) of the image must be written
    out = torch.full((B, cout, H, W), float("nan"), device=cuda)
    y, st = _capi.conv3x3(x.to(cuda), packed, cout, out=out, group_size=gs, stats=True,
                          in_affine=(s_in.to(cuda), t_in.to(cuda)) if affine else None,
                          n_stat=n_valid)
    assert torch.isfinite(y).all()
    _close(y, want, 5e-4 if operands == "bf16x3" else 1e-5)
    gamma = torch.rand(cout, generator=g) + 0.5
    beta = torch.randn(cout, generator=g)
    sc, sh = _capi.bn_finalize(st, gamma.to(cuda), beta.to(cuda), 1e-5)
    rsc, rsh = _group_bn_ref(want, gs, n_valid, gamma, beta)
    _close(sc, rsc, 2e-4)
    _close(sh, rsh, 2e-4)


@pytest.mark.parametrize("operands", ["f16x3", "bf16x3"])
@pytest.mark.parametrize("B,cout,H,W,gs,n_valid", [(5, 64, 224, 224, 2, 4), (3, 64, 30, 40, 2, 3),
                                                   (2, 40, 16, 256, 1, 2)])
def test_stem7_forward_and_stats(cuda, B, cout, H, W, gs, n_valid, operands):
    """The ImageNet stem (dd_stem7_forward): y against float64 F.conv2d(7x7, stride 2, pad 3),
    the finalized BN affine against float64 group statistics; odd output heights (an
    overhanging row pair), the widest map (128 outputs) and fewer than 64 outputs."""
    assert _capi.stem7_supported(H, W, 3, cout, gs)
    g = torch.Generator().manual_seed(B + cout + H + W)
    x = torch.randn(B, 3, H, W, generator=g)
    w = torch.randn(cout, 3, 7, 7, generator=g) / (7 * 3 ** 0.5)
    want = F.conv2d(x.double(), w.double(), stride=2, padding=3)
    y, st = _capi.stem7(x.to(cuda), _capi.stem7_pack(w.to(cuda), operands=operands), cout, gs,
                        n_stat=n_valid)
    assert torch.isfinite(y).all()
    _close(y, want, 5e-4 if operands == "bf16x3" else 1e-5)
    gamma = torch.rand(cout, generator=g) + 0.5
    beta = torch.randn(cout, generator=g)
    sc, sh = _capi.bn_finalize(st, gamma.to(cuda), beta.to(cuda), 1e-5)
    rsc, rsh = _group_bn_ref(want, gs, n_valid, gamma, beta)
    _close(sc, rsc, 2e-4)
    _close(sh, rsh, 2e-4)


def test_conv3x3_padded_width_refuses_other_epilogues(cuda):
    w = torch.randn(128, 64, 3, 3, device=cuda)
    packed = _capi.conv3x3_pack(w)
    x = torch.randn(2, 64, 28, 28, device=cuda)
    with pytest.raises(_capi.DDError, match="unsupported spatial shape"):
        _capi.conv3x3(x, packed, 128, relu=True)
    with pytest.raises(_capi.DDError, match="unsupported spatial shape"):
        _capi.conv3x3(x, packed, 128, bias=torch.zeros(128, device=cuda), group_size=2,
                      stats=True)


@pytest.mark.parametrize("B,C,H,W,gs,n_valid", [(7, 64, 16, 16, 3, 6), (4, 512, 4, 4, 2, 4),
                                                (5, 24, 7, 7, 5, 3)])
def test_channel_stats_finalize(cuda, B, C, H, W, gs, n_valid):
    g = torch.Generator().manual_seed(3 + B)
    y = torch.randn(B, C, H, W, generator=g) * 3 + 1
    gamma = torch.rand(C, generator=g) + 0.5
    beta = torch.randn(C, generator=g)
    st = _capi.channel_stats(y.to(cuda), gs, n_stat=n_valid)
    sc, sh = _capi.bn_finalize(st, gamma.to(cuda), beta.to(cuda), 1e-5)
    rsc, rsh = _group_bn_ref(y, gs, n_valid, gamma, beta)
    _close(sc, rsc, 1e-5)
    _close(sh, rsh, 1e-5)


@pytest.mark.parametrize("B,C,H,W,gs", [(5, 64, 112, 112, 2), (3, 16, 16, 24, 3),
                                        (3, 8, 15, 15, 2), (2, 8, 12, 12, 1)])
def test_bn_apply_maxpool(cuda, B, C, H, W, gs):
    """The ImageNet stem tail max_pool2d(relu(bn(y)), 3, 2, 1): the 4-output float4 kernel
    (w = 2 wo, w % 8 == 0) and the scalar one (other shapes, or a misaligned input) against
    fp64, and bitwise against each other."""
    g = torch.Generator().manual_seed(B + C + H + W)
    G = -(-B // gs)
    y = torch.randn(B, C, H, W, generator=g) * 2
    sc = torch.rand(G, C, generator=g) + 0.5
    sh = torch.randn(G, C, generator=g) * 0.5
    aff = (sc.to(cuda), sh.to(cuda))
    got = _capi.bn_apply_maxpool(y.to(cuda), aff, gs)
    z = torch.relu(y.double() * sc.double().repeat_interleave(gs, 0)[:B, :, None, None]
                   + sh.double().repeat_interleave(gs, 0)[:B, :, None, None])
    _close(got, F.max_pool2d(z, 3, 2, 1), 1e-6)
    # the same input at a 4-byte offset: the scalar kernel everywhere
    buf = torch.empty(y.numel() + 1, device=cuda)
    ym = buf[1:].view(B, C, H, W)
    ym.copy_(y.to(cuda))
    assert torch.equal(_capi.bn_apply_maxpool(ym, aff, gs), got)


@pytest.mark.parametrize("res_mode", ["none", "raw", "affine"])
@pytest.mark.parametrize("B,C,H,W,gs", [(6, 64, 7, 7, 4), (3, 4, 5, 3, 2)])
def test_bn_apply_quad_equals_scalar(cuda, monkeypatch, res_mode, B, C, H, W, gs):
    """Widths that are not a multiple of 4 (the ImageNet network's 7x7 unit tails): the
    4-element kernel is bitwise the scalar one (DD_BN_QUAD=0) and matches fp64."""
    g = torch.Generator().manual_seed(B + C + H)
    G = -(-B // gs)
    y = torch.randn(B, C, H, W, generator=g)
    r = torch.randn(B, C, H, W, generator=g)
    sc, sh = torch.rand(G, C, generator=g) + 0.5, torch.randn(G, C, generator=g)
    rs, rt = torch.rand(G, C, generator=g) + 0.5, torch.randn(G, C, generator=g)
    kw = {}
    if res_mode != "none":
        kw["residual"] = r.to(cuda)
    if res_mode == "affine":
        kw["res_affine"] = (rs.to(cuda), rt.to(cuda))
    got, _ = _capi.bn_apply(y.to(cuda), (sc.to(cuda), sh.to(cuda)), gs, **kw)
    monkeypatch.setenv("DD_BN_QUAD", "0")
    ref, _ = _capi.bn_apply(y.to(cuda), (sc.to(cuda), sh.to(cuda)), gs, **kw)
    assert torch.equal(got, ref)
    ex = lambda t: t.double().repeat_interleave(gs, 0)[:B, :, None, None]  # noqa: E731
    want = y.double() * ex(sc) + ex(sh)
    if res_mode == "raw":
        want = want + r.double()
    elif res_mode == "affine":
        want = want + r.double() * ex(rs) + ex(rt)
    _close(got, torch.relu(want), 1e-6)


@pytest.mark.parametrize("res_mode", ["none", "raw", "affine"])
def test_bn_apply_and_pool(cuda, res_mode):
    g = torch.Generator().manual_seed(5)
    B, C, H, W, gs = 6, 32, 4, 4, 4
    G = -(-B // gs)
    y = torch.randn(B, C, H, W, generator=g)
    r = torch.randn(B, C, H, W, generator=g)
    sc, sh = torch.rand(G, C, generator=g) + 0.5, torch.randn(G, C, generator=g)
    rs, rt = torch.rand(G, C, generator=g) + 0.5, torch.randn(G, C, generator=g)
    ex = lambda t: t.repeat_interleave(gs, 0)[:B, :, None, None]  # noqa: E731
    want = y * ex(sc) + ex(sh)
    kw = {}
    if res_mode == "raw":
        want = want + r
        kw = dict(residual=r.to(cuda))
    elif res_mode == "affine":
        want = want + torch.relu(r * ex(rs) + ex(rt))
        kw = dict(residual=r.to(cuda), res_affine=(rs.to(cuda), rt.to(cuda)), res_relu=True)
    want = torch.relu(want)
    pool = torch.empty(B, C, device=cuda)
    out, _ = _capi.bn_apply(y.to(cuda), (sc.to(cuda), sh.to(cuda)), gs, relu=True,
                            pool_out=pool, **kw)
    _close(out, want, 1e-6)
    _close(pool, want.mean(dim=(2, 3)), 1e-6)


@pytest.mark.parametrize("B,cin,cout,H,W,gs,n_valid", [
    (6, 64, 64, 32, 32, 2, 5), (8, 128, 128, 16, 16, 4, 8), (10, 256, 256, 8, 8, 4, 7)])
@pytest.mark.parametrize("res_mode", ["none", "raw", "affine"])
def test_conv3x3_unit_input_is_bn_apply_then_conv(cuda, B, cin, cout, H, W, gs, n_valid,
                                                   res_mode):
    """dd_conv3x3_forward_unit_input == dd_bn_apply (relu(bn(y) + R)) followed by
    dd_conv3x3_forward on its output, bitwise: the unit output it writes, the conv output and
    the BN partial statistics (ragged last group, rows past n_valid)."""
    assert _capi.conv3x3_unit_input_supported(H, W, cin, cout, gs)
    g = torch.Generator().manual_seed(B + cin + H)
    G = -(-B // gs)
    y = torch.randn(B, cin, H, W, generator=g).to(cuda)
    r = torch.randn(B, cin, H, W, generator=g).to(cuda)
    aff = ((torch.rand(G, cin, generator=g) + 0.5).to(cuda),
           torch.randn(G, cin, generator=g).to(cuda))
    raff = ((torch.rand(G, cin, generator=g) + 0.5).to(cuda),
            torch.randn(G, cin, generator=g).to(cuda))
    w = torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)
    packed = _capi.conv3x3_pack(w.to(cuda))
    kw = {} if res_mode == "none" else dict(residual=r) if res_mode == "raw" else \
        dict(residual=r, res_affine=raff)
    x_ref, _ = _capi.bn_apply(y, aff, gs, relu=True, **kw)
    tiles = _capi.conv3x3_tiles_per_group(H, W, gs)
    # (zeroed: the slots of a ragged last group past B are never written by either launch)
    sbuf = [torch.zeros(G * cout * tiles * 2, device=cuda) for _ in range(2)]
    y_ref, st_ref = _capi.conv3x3(x_ref, packed, cout, group_size=gs, stats=True,
                                  n_stat=n_valid, stats_buf=sbuf[0])
    x_out = torch.full_like(y, float("nan"))  # every element must be written
    x, yy, st = _capi.conv3x3_unit_input(y, aff, packed, cout, gs, n_stat=n_valid, x_out=x_out,
                                         stats_buf=sbuf[1], **kw)
    assert torch.equal(x, x_ref)
    assert torch.equal(yy, y_ref)
    assert torch.equal(st.buf, st_ref.buf)


@pytest.mark.parametrize("B,cin,cout,H,gs,unit", [
    (6, 64, 128, 32, 2, True), (10, 128, 256, 16, 2, True), (12, 256, 512, 8, 4, True),
    (6, 128, 128, 32, 2, False), (8, 256, 256, 8, 4, False)])
def test_down_unit_input_is_bn_apply_then_down(cuda, B, cin, cout, H, gs, unit):
    """dd_down_forward_unit_input == dd_bn_apply (relu(bn(y) + shortcut), or relu(bn(y)) for
    a Bottleneck's stride-2 conv2) followed by dd_down_forward on its output, bitwise: both
    outputs and the BN partial statistics (ragged last group, rows past n_valid)."""
    g = torch.Generator().manual_seed(B + cin + H)
    G = -(-B // gs)
    n_valid = B - 1
    y = torch.randn(B, cin, H, H, generator=g).to(cuda)
    r = torch.randn(B, cin, H, H, generator=g).to(cuda)
    aff = ((torch.rand(G, cin, generator=g) + 0.5).to(cuda),
           torch.randn(G, cin, generator=g).to(cuda))
    w3 = (torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)).to(cuda)
    p3 = _capi.conv3x3_pack(w3)
    p1 = _capi.conv1x1_pack((torch.randn(cout, cin, generator=g) / cin ** 0.5).to(cuda)) \
        if unit else None
    x_ref, _ = _capi.bn_apply(y, aff, gs, relu=True, **(dict(residual=r) if unit else {}))
    want = _capi.conv_down(x_ref, p3, cout, p1, group_size=gs, stats=True, n_stat=n_valid)
    got = _capi.conv_down_unit_input(y, aff, p3, cout, gs, packed1x1=p1,
                                     residual=r if unit else None, n_stat=n_valid)
    assert torch.equal(got[0], want[0])
    assert torch.equal(got[2].buf, want[2].buf)
    if unit:
        assert torch.equal(got[1], want[1])
        assert torch.equal(got[3].buf, want[3].buf)


def test_forward_logits_unit_input_fusion_is_bitwise(cuda):
    """The EL2N forward with the unit tails fused into the next convs' staging gives the
    logits of the separate-pass forward bit for bit (ResNet-18: the stem output and the 32x32,
    16x16 and 8x8 unit outputs take the fused form)."""
    images, _ = synthetic.make_images(256, 10, seed=6)
    sd = synthetic.make_checkpoint("resnet18", 10, seed=5)["net"]
    model = checkpoints.build_models([sd], "resnet18", 10, device=cuda)[0]
    model.eval()
    model.prepare_fast_convs()
    x = o_pipe.normalize(images).to(cuda).contiguous()
    _capi.kernel_log = []
    try:
        got = el2n_fast.forward_logits(model, x, 128, 200)
        tags = [e[0] for e in _capi.kernel_log]
        fused = tags.count("conv3x3_unit")
    finally:
        _capi.kernel_log = None
    el2n_fast.FUSE_UNIT_INPUT = False
    try:
        want = el2n_fast.forward_logits(model, x, 128, 200)
    finally:
        el2n_fast.FUSE_UNIT_INPUT = True
    assert torch.equal(got, want)
    # fused into the next conv's staging: the stem output and the outputs of layer1.0, 2.0
    # and 3.0 (written out once by the first convs of layer1.0, 1.1, 2.1, 3.1) and those of
    # layer1.1, 2.1, 3.1 (computed by the next stage's downsampling head, never written); a
    # separate pass: the output of layer4.0 (4x4 maps) and the pooled tail of layer4.1
    assert fused == 4 and tags.count("down_fwd_unit") == 3, tags
    assert tags.count("bn_apply") == 2, tags


@pytest.mark.parametrize("arch,classes,B,gs,n_valid,rel", [
    ("resnet18", 10, 512, 128, 400, 1e-5), ("resnet50", 100, 64, 16, 60, 3e-5)])
def test_forward_logits_fp32_matches_grouped_run(cuda, arch, classes, B, gs, n_valid, rel):
    """The refinement's plain-fp32 forward (fp32 convs, grouped BN by the stats / finalize /
    apply kernels) == ResNet.run(bn="groups") (fp32 convs, torch BN ops) to fp32 rounding:
    1e-5 of the max-abs logit on ResNet-18, 3e-5 through ResNet-50's 53 train-mode BNs over
    16-row groups (measured 1.65e-5: dd_channel_stats sums in double, as PyTorch's CPU
    batch_norm -- the reference's -- does, torch's GPU reduction in float; the split-bf16 path
    is at 1e-4)."""
    images, _ = synthetic.make_images(B, classes, seed=8)
    sd = synthetic.make_checkpoint(arch, classes, seed=9)["net"]
    model = checkpoints.build_models([sd], arch, classes, device=cuda)[0]
    model.eval()
    x = o_pipe.normalize(images).to(cuda).contiguous()
    x[n_valid:] = 0
    got = el2n_fast.forward_logits_fp32(model, x, gs, n_valid)[:n_valid]
    with torch.inference_mode():
        want = model.run(x, bn="groups", group=gs, n_valid=n_valid)[:n_valid]
    _close(got, want, rel)


def _grouped_run_ref(model, x, gs, n_valid):
    """ResNet.run(bn="batch") per group on the GPU (MIOpen fp32), rows >= n_valid dropped."""
    outs = []
    with torch.inference_mode():
        for lo in range(0, n_valid, gs):
            hi = min(n_valid, lo + gs)
            outs.append(model.run(x[lo:hi], bn="batch"))
    return torch.cat(outs)


@pytest.mark.parametrize("arch,classes,B,gs,n_valid", [
    ("resnet18", 10, 256, 128, 256), ("resnet18", 10, 256, 128, 200),
    ("resnet50", 100, 32, 16, 27)])
def test_forward_logits_matches_train_bn_forward(cuda, arch, classes, B, gs, n_valid):
    images, labels = synthetic.make_images(B, classes, seed=4)
    sd = synthetic.make_checkpoint(arch, classes, seed=3)["net"]
    model = checkpoints.build_models([sd], arch, classes, device=cuda)[0]
    model.eval()
    model.prepare_fast_convs()
    x = o_pipe.normalize(images).to(cuda)
    x[n_valid:] = 0
    got = el2n_fast.forward_logits(model, x.contiguous(), gs, n_valid)[:n_valid]
    want = _grouped_run_ref(model, x, gs, n_valid)
    _close(got, want, 1e-3)


def test_engine_fast_el2n_equals_reference_path(cuda):
    """Grouped fast path == the per-batch MIOpen path, ragged final batch, chunk boundaries."""
    images, labels = synthetic.make_images(700, 10, seed=12)
    sds = [synthetic.make_checkpoint("resnet18", 10, seed=s)["net"] for s in (1, 2)]
    img, lab = torch.from_numpy(images).to(cuda), torch.from_numpy(labels).to(cuda)
    out = {}
    for fast in (True, False):
        eng = ScoringEngine(checkpoints.build_models(sds, device=cuda),
                            ScoreConfig(fast_el2n=fast, el2n_chunk=256), cuda)
        out[fast] = eng.score_shard(img, lab, 0, 700)["el2n"].cpu().numpy()
    np.testing.assert_allclose(out[True], out[False], rtol=1e-3)
    ref = np.zeros(700, np.float32)
    for sd in sds:
        ref += o_pipe.el2n_scores(sd, images, labels, batch_size=128)
    np.testing.assert_allclose(out[True], ref / np.float32(2), rtol=1e-3)


@pytest.mark.parametrize("B,cin,cout,H,gs,n_valid,res_mode,ops", [
    (4, 64, 64, 32, 2, 3, "none", "f16x3"), (4, 256, 64, 32, 2, 4, "raw", "f16x3"),
    (6, 256, 128, 16, 2, 5, "affine", "f16x3"), (8, 512, 128, 8, 4, 8, "raw", "bf16x3"),
    (16, 1024, 256, 4, 8, 13, "affine", "bf16x3"), (4, 512, 512, 16, 2, 4, "raw", "f16x3")])
def test_conv1x1_unit_input_is_bn_apply_then_conv(cuda, B, cin, cout, H, gs, n_valid, res_mode,
                                                  ops):
    """dd_conv1x1_forward_unit_input (ABI 8) == dd_bn_apply (relu(bn(y) [+ R | + bn_r(R)]))
    followed by dd_conv1x1_forward(stats) on its output, bitwise: the unit output it writes
    (every element, from the output-block-0 tiles), the conv output and the BN partials, on
    the Bottleneck conv1 shapes (cout > 128: several output blocks re-stage the input)."""
    g = torch.Generator().manual_seed(B + cin + H + cout)
    G = -(-B // gs)
    y = torch.randn(B, cin, H, H, generator=g).to(cuda)
    r = torch.randn(B, cin, H, H, generator=g).to(cuda)
    aff = ((torch.rand(G, cin, generator=g) + 0.5).to(cuda),
           torch.randn(G, cin, generator=g).to(cuda))
    raff = ((torch.rand(G, cin, generator=g) + 0.5).to(cuda),
            torch.randn(G, cin, generator=g).to(cuda))
    w = torch.randn(cout, cin, generator=g) / cin ** 0.5
    packed = _capi.conv1x1_pack(w.to(cuda), operands=ops)
    kw = {} if res_mode == "none" else dict(residual=r) if res_mode == "raw" else \
        dict(residual=r, res_affine=raff)
    x_ref, _ = _capi.bn_apply(y, aff, gs, relu=True, **kw)
    y_ref, st_ref = _capi.conv1x1(x_ref, packed, cout, group_size=gs, stats=True, n_stat=n_valid)
    x, yy, st = _capi.conv1x1_unit_input(y, aff, packed, cout, gs, n_stat=n_valid, **kw)
    assert torch.equal(x, x_ref)
    assert torch.equal(yy, y_ref)
    assert torch.equal(st.buf, st_ref.buf)


def test_forward_logits_resnet50_unit_input_fusion_is_bitwise(cuda):
    """ResNet-50 (CIFAR-100): the Bottleneck unit tails fused into the next unit's 1x1 conv1
    give the logits of the separate-pass forward bit for bit; every tail but the pooled last
    one (and the stride-2 conv2 heads' own fusions) leaves dd_bn_apply."""
    images, _ = synthetic.make_images(256, 100, seed=7)
    sd = synthetic.make_checkpoint("resnet50", 100, seed=5)["net"]
    model = checkpoints.build_models([sd], "resnet50", 100, device=cuda)[0]
    model.eval()
    model.prepare_fast_convs()
    x = o_pipe.normalize(images).to(cuda).contiguous()
    _capi.kernel_log = []
    try:
        got = el2n_fast.forward_logits(model, x, 128, 200)
        tags = [e[0] for e in _capi.kernel_log]
    finally:
        _capi.kernel_log = None
    el2n_fast.FUSE_UNIT_INPUT = False
    _capi.kernel_log = []
    try:
        want = el2n_fast.forward_logits(model, x, 128, 200)
        tags_sep = [e[0] for e in _capi.kernel_log]
    finally:
        el2n_fast.FUSE_UNIT_INPUT = True
        _capi.kernel_log = None
    assert torch.equal(got, want)
    # the stem output and the outputs of the first 15 of the 16 units feed a 1x1 conv1; the
    # last unit's tail is the pooled dd_bn_apply (the separate forward also applies the
    # stride-2 conv2s' producer BN in passes of their own)
    assert tags.count("conv1x1_unit") == 16, tags
    assert tags.count("bn_apply") == 1, tags
    assert tags_sep.count("bn_apply") == 1 + 16 + 3, tags_sep
