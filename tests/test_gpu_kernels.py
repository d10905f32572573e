"""Kernel-level parity of libdd.so against the NumPy oracle (GPU, through the C-ABI)."""
import numpy as np
import pytest
import torch

from data_diet_distributed_amd import _capi
from oracle import el2n as o_el2n
from oracle import pegrad as o_pegrad

pytestmark = pytest.mark.gpu

RTOL = 1e-3  # north star: scores within 1e-3 relative (fp32)


# ---- EL2N ------------------------------------------------------------------------------------
@pytest.mark.parametrize("B,C", [(1, 10), (128, 10), (1000, 10), (77, 100), (256, 1000),
                                 (33, 3000), (5, 1), (64, 17), (300, 64), (257, 10),
                                 (70001, 10), (513, 7), (600, 128), (300, 129), (1024, 100),
                                 (255, 33)])
def test_el2n_matches_oracle(cuda, B, C):
    rng = np.random.default_rng(B * 1000 + C)
    logits = (rng.normal(size=(B, C)) * 4).astype(np.float32)
    labels = rng.integers(0, C, size=B)
    s_ref, e_ref = o_el2n.el2n_rows(logits, labels, with_e=True)
    lg = torch.from_numpy(logits).to(cuda)
    lb = torch.from_numpy(labels).to(cuda)
    score = torch.empty(B, device=cuda)
    e = torch.empty(B, C, device=cuda)
    acc = torch.full((B,), 0.5, device=cuda)
    _capi.el2n(lg, lb, score=score, e=e, accum=acc)
    np.testing.assert_allclose(score.cpu().numpy(), s_ref, rtol=RTOL, atol=1e-6)
    np.testing.assert_allclose(e.cpu().numpy(), e_ref, rtol=RTOL, atol=1e-6)
    np.testing.assert_allclose(acc.cpu().numpy(), s_ref + 0.5, rtol=RTOL, atol=1e-6)


@pytest.mark.parametrize("C", [10, 7, 100])
def test_el2n_unaligned_buffers(cuda, C):
    """Row slices whose start is not 16-byte aligned take the scalar staging path."""
    B = 700
    rng = np.random.default_rng(C)
    logits = (rng.normal(size=(B + 1, C)) * 3).astype(np.float32)
    labels = rng.integers(0, C, size=B + 1)
    s_ref, e_ref = o_el2n.el2n_rows(logits[1:], labels[1:], with_e=True)
    lg = torch.from_numpy(logits).to(cuda)[1:]
    lb = torch.from_numpy(labels).to(cuda)[1:]
    e_all = torch.empty(B + 1, C, device=cuda)
    score = torch.empty(B, device=cuda)
    _capi.el2n(lg, lb, score=score, e=e_all[1:])
    np.testing.assert_allclose(score.cpu().numpy(), s_ref, rtol=RTOL, atol=1e-6)
    np.testing.assert_allclose(e_all[1:].cpu().numpy(), e_ref, rtol=RTOL, atol=1e-6)


def test_el2n_extreme_logits(cuda):
    # saturated softmax rows: one logit dominates by 1e4 (exp underflow must not NaN)
    logits = np.zeros((4, 10), np.float32)
    logits[:, 3] = 1e4
    labels = np.array([3, 0, 3, 9])
    s_ref = o_el2n.el2n_rows(logits, labels)
    score = torch.empty(4, device=cuda)
    _capi.el2n(torch.from_numpy(logits).to(cuda), torch.from_numpy(labels).to(cuda), score=score)
    np.testing.assert_allclose(score.cpu().numpy(), s_ref, rtol=RTOL, atol=1e-6)


@pytest.mark.parametrize("B,C", [(300, 10), (200, 100), (130, 1000), (40, 3000)],
                         ids=["lds16", "lds32x4", "rows", "wide"])
def test_el2n_counts_bad_labels(cuda, B, C):
    """A label outside [0, C) (where the reference's one_hot raises, get_scores_and_prune.py:17)
    is counted in bad_labels and its row's score, accum term and e row are NaN, on every kernel
    family; the other rows are exactly those of a run without the bad rows; check_labels raises
    LabelError (a ValueError and a RuntimeError)."""
    rng = np.random.default_rng(B + C)
    logits = (rng.normal(size=(B, C)) * 4).astype(np.float32)
    labels = rng.integers(0, C, size=B)
    bad_rows = np.array([0, 7, B // 2, B - 1])
    bad_labels = labels.copy()
    bad_labels[bad_rows] = [-1, C, C + 5, -(2 ** 40)]
    lg = torch.from_numpy(logits).to(cuda)
    out = {}
    for name, lab in (("good", labels), ("bad", bad_labels)):
        score = torch.empty(B, device=cuda)
        e = torch.empty(B, C, device=cuda)
        acc = torch.zeros(B, device=cuda)
        cnt = _capi.label_counter(cuda)
        _capi.el2n(lg, torch.from_numpy(lab).to(cuda), score=score, e=e, accum=acc,
                   bad_labels=cnt)
        out[name] = (score.cpu().numpy(), e.cpu().numpy(), acc.cpu().numpy(), int(cnt.item()))
    assert out["good"][3] == 0 and out["bad"][3] == bad_rows.size
    ok = np.setdiff1d(np.arange(B), bad_rows)
    for i in range(3):
        assert np.isnan(out["bad"][i][bad_rows]).all()
        assert np.array_equal(out["bad"][i][ok], out["good"][i][ok])
    _capi.check_labels(_capi.label_counter(cuda), C)  # zero: no raise
    cnt = torch.tensor([bad_rows.size], dtype=torch.int32, device=cuda)
    with pytest.raises(ValueError, match="outside"):
        _capi.check_labels(cnt, C)
    with pytest.raises(RuntimeError):
        _capi.check_labels(cnt, C)


def test_el2n_empty(cuda):
    _capi.el2n(torch.empty(0, 10, device=cuda), torch.empty(0, dtype=torch.int64, device=cuda),
               score=torch.empty(0, device=cuda))


# ---- normalisation ---------------------------------------------------------------------------
@pytest.mark.parametrize("shape", [(5, 3, 32, 32), (3, 3, 7, 5), (2, 1, 4, 4)])
def test_normalize_matches_torch(cuda, shape):
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, size=shape, dtype=np.uint8)
    C = shape[1]
    mean, std = [0.4914, 0.4822, 0.4465][:C], [0.2023, 0.1994, 0.2010][:C]
    ref = torch.from_numpy(img).float().div(255)
    ref = ref.sub(torch.tensor(mean)[:, None, None]).div(torch.tensor(std)[:, None, None])
    out = torch.empty(shape, dtype=torch.float32, device=cuda)
    _capi.normalize_u8(torch.from_numpy(img).to(cuda), mean, std, out)
    np.testing.assert_allclose(out.cpu().numpy(), ref.numpy(), rtol=1e-6, atol=1e-6)
    # gathered variant
    idx = torch.tensor(list(range(shape[0]))[::-1], dtype=torch.int64, device=cuda)
    out2 = torch.empty(shape, dtype=torch.float32, device=cuda)
    _capi.normalize_u8(torch.from_numpy(img).to(cuda), mean, std, out2, index=idx)
    np.testing.assert_allclose(out2.cpu().numpy(), ref.numpy()[::-1], rtol=1e-6, atol=1e-6)


# ---- GraNd per-layer norms -------------------------------------------------------------------
# (B, cin, h, w, cout, k, stride, pad): every Conv2d shape of CIFAR ResNet-18 and ResNet-50,
# plus odd/ragged shapes
R18 = [(3, 3, 32, 32, 64, 3, 1, 1), (3, 64, 32, 32, 64, 3, 1, 1), (3, 64, 32, 32, 128, 3, 2, 1),
       (3, 128, 16, 16, 128, 3, 1, 1), (3, 64, 32, 32, 128, 1, 2, 0),
       (3, 128, 16, 16, 256, 3, 2, 1), (3, 256, 8, 8, 256, 3, 1, 1), (3, 128, 16, 16, 256, 1, 2, 0),
       (3, 256, 8, 8, 512, 3, 2, 1), (3, 512, 4, 4, 512, 3, 1, 1), (3, 256, 8, 8, 512, 1, 2, 0)]
R50 = [(2, 64, 32, 32, 64, 1, 1, 0), (2, 64, 32, 32, 256, 1, 1, 0), (2, 256, 32, 32, 64, 1, 1, 0),
       (2, 128, 32, 32, 128, 3, 2, 1), (2, 256, 16, 16, 1024, 1, 1, 0),
       (2, 512, 4, 4, 2048, 1, 1, 0), (2, 2048, 4, 4, 512, 1, 1, 0),
       # 1x1 stride-2 projections (split-bf16 1x1 direct kernel, strided gather)
       (2, 256, 32, 32, 512, 1, 2, 0), (3, 40, 10, 14, 70, 1, 2, 0), (2, 130, 16, 16, 260, 1, 1, 0),
       # split-bf16 1x1 kernel on its scalar gather paths (T = 49; stride 2 onto a 7-wide map)
       (2, 256, 7, 7, 64, 1, 1, 0), (2, 128, 14, 14, 256, 1, 2, 0)]
ODD = [(5, 5, 9, 7, 13, 3, 1, 1), (4, 7, 5, 5, 3, 3, 2, 1), (2, 3, 11, 11, 70, 7, 2, 3),
       (6, 33, 3, 3, 65, 1, 1, 0), (1, 1, 1, 1, 1, 1, 1, 0), (3, 65, 6, 6, 129, 3, 1, 1)]
# shapes the split-bf16 all-taps 3x3 kernel takes (W in {8,16,32}), incl. ragged channel
# counts and non-square inputs (H a multiple of 32/W)
D3 = [(2, 96, 32, 32, 40, 3, 1, 1), (3, 17, 16, 16, 130, 3, 1, 1), (2, 128, 8, 8, 70, 3, 1, 1),
      (2, 64, 8, 32, 64, 3, 1, 1), (2, 64, 12, 16, 64, 3, 1, 1), (1, 3, 32, 32, 64, 3, 1, 1),
      # odd step counts: 10 rows at 16 wide (persistent form, 5 steps), 9 rows at 32 wide,
      # 12 rows at 8 wide (3 steps of 4 rows)
      (2, 64, 10, 16, 64, 3, 1, 1), (2, 64, 9, 32, 64, 3, 1, 1), (2, 32, 12, 8, 48, 3, 1, 1),
      # stride 2 over 32-wide inputs (decimated staging): ragged channels, non-square
      (2, 40, 32, 32, 70, 3, 2, 1), (2, 64, 16, 32, 64, 3, 2, 1), (1, 130, 8, 32, 20, 3, 2, 1)]


def _conv_case(cuda, case, seed):
    B, cin, h, w, cout, k, s, p = case
    ho = (h + 2 * p - k) // s + 1
    wo = (w + 2 * p - k) // s + 1
    rng = np.random.default_rng(seed)
    act = np.maximum(rng.normal(size=(B, cin, h, w)), 0).astype(np.float32)
    gout = (rng.normal(size=(B, cout, ho, wo)) * 1e-2).astype(np.float32)
    return act, gout, k, s, p


@pytest.mark.parametrize("prec", ["fp32", "bf16x3"])
@pytest.mark.parametrize("method", ["direct", "ghost", "auto"])
@pytest.mark.parametrize("case", R18 + R50 + ODD + D3, ids=lambda c: "x".join(map(str, c)))
def test_conv_pegrad_matches_oracle(cuda, case, method, prec):
    act, gout, k, s, p = _conv_case(cuda, case, hash(case) % 2**31)
    ref = o_pegrad.conv_pegrad_sqnorm(act, gout, k, k, s, p)
    a = torch.from_numpy(act).to(cuda)
    g = torch.from_numpy(gout).to(cuda)
    geom = _capi.conv_geom(a, g, (k, k), s, p)
    ws = torch.empty(max(_capi.conv_workspace_bytes(geom, method, prec), 4), dtype=torch.uint8,
                     device=cuda)
    sq = torch.full((act.shape[0],), 1.0, device=cuda)
    _capi.conv_pegrad_sqnorm(a, g, (k, k), s, p, sq, ws, method=method, precision=prec)
    np.testing.assert_allclose(sq.cpu().numpy().astype(np.float64) - 1.0, ref, rtol=RTOL,
                               atol=1e-7 * max(1.0, ref.max()))


def test_conv_pegrad_col_scale(cuda):
    act, gout, k, s, p = _conv_case(cuda, (3, 64, 8, 8, 96, 3, 1, 1), 5)
    scale = np.random.default_rng(9).uniform(0.2, 2.0, size=96).astype(np.float32)
    ref = o_pegrad.conv_pegrad_sqnorm(act, gout, k, k, s, p, col_scale=scale)
    for method, prec in (("direct", "fp32"), ("ghost", "fp32"), ("direct", "bf16x3"),
                         ("ghost", "bf16x3")):
        a, g = torch.from_numpy(act).to(cuda), torch.from_numpy(gout).to(cuda)
        geom = _capi.conv_geom(a, g, (k, k), s, p)
        ws = torch.empty(_capi.conv_workspace_bytes(geom, method, prec), dtype=torch.uint8,
                         device=cuda)
        sq = torch.zeros(3, device=cuda)
        _capi.conv_pegrad_sqnorm(a, g, (k, k), s, p, sq, ws, method=method,
                                 col_scale=torch.from_numpy(scale).to(cuda), precision=prec)
        np.testing.assert_allclose(sq.cpu().numpy(), ref, rtol=RTOL)


@pytest.mark.parametrize("case", [(4, 64, 32, 32, 64, 3, 1, 1), (4, 128, 16, 16, 128, 3, 1, 1),
                                  (4, 64, 32, 32, 128, 3, 2, 1)])
def test_direct3x3_accuracy_on_signed_data(cuda, case):
    """Split-bf16 accuracy on signed, cancellation-prone data (gradients of both signs and
    activations with a large common offset): far inside the 1e-3 norm tolerance."""
    B, cin, h, w, cout, k, s, p = case
    rng = np.random.default_rng(7)
    act = (rng.normal(size=(B, cin, h, w)) + 3.0).astype(np.float32)
    gout = rng.normal(size=(B, cout, h // s, w // s)).astype(np.float32)
    ref = o_pegrad.conv_pegrad_sqnorm(act, gout, k, k, s, p)
    a, g = torch.from_numpy(act).to(cuda), torch.from_numpy(gout).to(cuda)
    geom = _capi.conv_geom(a, g, (k, k), s, p)
    assert _capi.conv_method(geom, "direct", "bf16x3") == "direct3x3"
    ws = torch.empty(_capi.conv_workspace_bytes(geom, "direct", "bf16x3"), dtype=torch.uint8,
                     device=cuda)
    sq = torch.zeros(B, device=cuda)
    _capi.conv_pegrad_sqnorm(a, g, (k, k), s, p, sq, ws, method="direct", precision="bf16x3")
    err = np.abs(sq.cpu().numpy() / ref - 1).max()
    assert err < 1e-4, err


def test_conv_pegrad_deterministic(cuda):
    act, gout, k, s, p = _conv_case(cuda, (16, 64, 32, 32, 64, 3, 1, 1), 3)
    a, g = torch.from_numpy(act).to(cuda), torch.from_numpy(gout).to(cuda)
    geom = _capi.conv_geom(a, g, (k, k), s, p)
    ws = torch.empty(_capi.conv_workspace_bytes(geom, "auto", "fp32"), dtype=torch.uint8,
                     device=cuda)
    outs = []
    for _ in range(3):
        sq = torch.zeros(16, device=cuda)
        _capi.conv_pegrad_sqnorm(a, g, (k, k), s, p, sq, ws)
        outs.append(sq.cpu().numpy())
    assert all((o == outs[0]).all() for o in outs)


def test_auto_method_choice(cuda):
    # direct wins for T >= 256 on R18, ghost for layer3/layer4
    def m(cin, h, cout, k, s, p, prec="fp32"):
        ho = (h + 2 * p - k) // s + 1
        g = _capi.ConvGeom(8, cin, h, h, cout, ho, ho, k, k, s, p)
        return _capi.conv_method(g, "auto", prec)
    assert m(64, 32, 64, 3, 1, 1) == "direct"
    assert m(128, 16, 128, 3, 1, 1) == "direct"
    assert m(256, 8, 256, 3, 1, 1) == "ghost"
    assert m(512, 4, 512, 3, 1, 1) == "ghost"
    assert m(64, 32, 64, 3, 1, 1, "bf16x3") == "direct3x3"
    # 16x16 at stride 1 (ResNet-18 layer2): the quarter-tiled shifted-Gram ghost (dd_pgram.hip)
    assert m(128, 16, 128, 3, 1, 1, "bf16x3") == "direct3x3"  # (measured faster: DESIGN §4.2)
    g16 = _capi.ConvGeom(8, 128, 16, 16, 128, 16, 16, 3, 3, 1, 1)
    assert _capi.conv_method(g16, "direct", "bf16x3") == "direct3x3"
    assert _capi.conv_method(g16, "ghost", "bf16x3") == "pgram_q"
    # maps of <= 64 positions: the shifted-Gram ghost (dd_pgram.hip)
    assert m(512, 4, 512, 3, 1, 1, "bf16x3") == "pgram"
    assert m(256, 8, 256, 3, 1, 1, "bf16x3") == "pgram"
    assert m(256, 8, 512, 3, 2, 1, "bf16x3") == "pgram"
    assert m(256, 8, 512, 1, 2, 0, "bf16x3") == "pgram"
    assert m(128, 16, 256, 3, 2, 1, "bf16x3") == "pgram"  # 256 inputs: 4 parity classes
    assert m(64, 32, 128, 3, 2, 1, "bf16x3") == "direct3x3"  # 1024 input positions
    assert m(3, 32, 64, 3, 1, 1, "bf16x3") == "stem"  # the input conv: 27 im2col rows
    assert m(3, 32, 64, 3, 1, 1) == "direct"
    assert m(512, 4, 512, 3, 1, 1, "bf16x3") != m(512, 4, 512, 3, 1, 1, "fp32")


# the input conv (cin * 9 <= 32): one 32-row block of G, g read once (dd_stem.hip); 1-3
# channels, 10-64 outputs, widths 8/16/32, non-square, signed data with a large common offset
STEM = [(5, 3, 32, 32, 64), (3, 3, 32, 32, 10), (2, 1, 16, 16, 64), (3, 2, 8, 32, 33),
        (4, 3, 8, 8, 64), (2, 3, 64, 32, 64)]


@pytest.mark.parametrize("case", STEM, ids=lambda c: "x".join(map(str, c)))
@pytest.mark.parametrize("scaled", [False, True])
def test_stem_matches_oracle(cuda, case, scaled):
    B, cin, h, w, cout = case
    rng = np.random.default_rng(h * 100 + cout + cin)
    act = (rng.normal(size=(B, cin, h, w)) + 2.0).astype(np.float32)
    gout = (rng.normal(size=(B, cout, h, w)) * 1e-2).astype(np.float32)
    scale = rng.uniform(0.2, 2.0, size=cout).astype(np.float32) if scaled else None
    ref = o_pegrad.conv_pegrad_sqnorm(act, gout, 3, 3, 1, 1, col_scale=scale)
    a, g = torch.from_numpy(act).to(cuda), torch.from_numpy(gout).to(cuda)
    geom = _capi.conv_geom(a, g, (3, 3), 1, 1)
    for method in ("auto", "direct"):
        assert _capi.conv_method(geom, method, "bf16x3") == "stem"
    assert _capi.conv_method(geom, "ghost", "bf16x3") != "stem"
    ws = torch.empty(max(_capi.conv_workspace_bytes(geom, "auto", "bf16x3"), 4),
                     dtype=torch.uint8, device=cuda)
    sq = torch.full((B,), 0.5, device=cuda)
    cs = torch.from_numpy(scale).to(cuda) if scaled else None
    _capi.conv_pegrad_sqnorm(a, g, (3, 3), 1, 1, sq, ws, col_scale=cs, precision="bf16x3")
    err = np.abs((sq.cpu().numpy().astype(np.float64) - 0.5) / ref - 1).max()
    assert err < 1e-4, err


@pytest.mark.parametrize("B,din,dout,bias", [(1, 512, 10, True), (300, 2048, 100, True),
                                             (7, 5, 3, False)])
def test_linear_pegrad(cuda, B, din, dout, bias):
    rng = np.random.default_rng(B)
    a = rng.normal(size=(B, din)).astype(np.float32)
    g = rng.normal(size=(B, dout)).astype(np.float32)
    ref = o_pegrad.linear_pegrad_sqnorm(a, g, bias)
    sq = torch.zeros(B, device=cuda)
    _capi.linear_pegrad_sqnorm(torch.from_numpy(a).to(cuda), torch.from_numpy(g).to(cuda), sq, bias)
    np.testing.assert_allclose(sq.cpu().numpy(), ref, rtol=RTOL)


def test_sqrt_accumulate_and_finalize(cuda):
    sq = torch.tensor([0.0, 4.0, 9.0, 2.0], device=cuda)
    acc = torch.tensor([1.0, 1.0, 1.0, 1.0], device=cuda)
    _capi.sqrt_accumulate(sq, acc)
    np.testing.assert_allclose(acc.cpu().numpy(), [1, 3, 4, 1 + np.sqrt(np.float32(2))], rtol=1e-6)
    out = torch.empty(4, device=cuda)
    _capi.ensemble_finalize(acc, 1, out)
    assert torch.equal(out, acc)  # K == 1 is the single-checkpoint score, bit for bit
    _capi.ensemble_finalize(acc, 3, out)
    np.testing.assert_allclose(out.cpu().numpy(), acc.cpu().numpy() / np.float32(3), rtol=1e-7)


# shifted-Gram ghost (pgram): every tile configuration (input / output positions 16 or 64),
# stride 1 and 2, 3x3 and 1x1, ragged channel counts (chunks of 64), signed activations
PGRAM = [(5, 256, 8, 8, 256, 3, 1, 1), (3, 512, 4, 4, 512, 3, 1, 1), (4, 256, 8, 8, 512, 3, 2, 1),
         (4, 256, 8, 8, 512, 1, 2, 0), (3, 17, 8, 8, 70, 3, 1, 1), (2, 100, 4, 4, 33, 3, 1, 1),
         (2, 3, 8, 8, 5, 1, 1, 0), (3, 130, 16, 16, 64, 1, 2, 0),
         # stride 2 over 16x16 inputs: four 8x8 parity classes (layer3 head + its shortcut)
         (3, 128, 16, 16, 256, 3, 2, 1), (3, 128, 16, 16, 256, 1, 2, 0),
         (2, 70, 16, 16, 33, 3, 2, 1)]


@pytest.mark.parametrize("case", PGRAM, ids=lambda c: "x".join(map(str, c)))
@pytest.mark.parametrize("signed", [False, True])
def test_pgram_matches_oracle(cuda, case, signed):
    act, gout, k, s, p = _conv_case(cuda, case, 7 + hash(case) % 1000)
    if signed:
        act = act - 0.5
    ref = o_pegrad.conv_pegrad_sqnorm(act, gout, k, k, s, p)
    a, g = torch.from_numpy(act).to(cuda), torch.from_numpy(gout).to(cuda)
    geom = _capi.conv_geom(a, g, (k, k), s, p)
    if case[2] * case[3] <= 64 or (case[2:4] == (16, 16) and case[6] == 2):
        assert _capi.conv_method(geom, "auto", "bf16x3") == "pgram"
    ws = torch.empty(max(_capi.conv_workspace_bytes(geom, "auto", "bf16x3"), 4),
                     dtype=torch.uint8, device=cuda)
    sq = torch.full((act.shape[0],), 2.0, device=cuda)
    _capi.conv_pegrad_sqnorm(a, g, (k, k), s, p, sq, ws, precision="bf16x3")
    np.testing.assert_allclose(sq.cpu().numpy().astype(np.float64) - 2.0, ref, rtol=1e-4,
                               atol=1e-7 * max(1.0, ref.max()))


# quarter-tiled shifted-Gram ghost (pgram_q, 16x16 at stride 1): the ResNet-18 layer2 shape,
# ragged / asymmetric channel counts (16-channel K steps), a batch that is not a multiple of 8
# (the grid covers whole groups of 8 examples), signed activations and a BN-folded col_scale
PGQ = [(5, 128, 16, 16, 128, 3, 1, 1), (3, 100, 16, 16, 70, 3, 1, 1), (9, 17, 16, 16, 33, 3, 1, 1),
       (1, 256, 16, 16, 64, 3, 1, 1)]


@pytest.mark.parametrize("case", PGQ, ids=lambda c: "x".join(map(str, c)))
@pytest.mark.parametrize("signed", [False, True])
def test_pgram_q_matches_oracle_and_direct(cuda, case, signed):
    act, gout, k, s, p = _conv_case(cuda, case, 11 + hash(case) % 1000)
    if signed:
        act = act - 0.5
    scale = np.random.default_rng(case[1]).uniform(0.3, 2.0, size=case[4]).astype(np.float32)
    ref = o_pegrad.conv_pegrad_sqnorm(act, gout, k, k, s, p, col_scale=scale)
    a, g = torch.from_numpy(act).to(cuda), torch.from_numpy(gout).to(cuda)
    geom = _capi.conv_geom(a, g, (k, k), s, p)
    assert _capi.conv_method(geom, "ghost", "bf16x3") == "pgram_q"
    out = {}
    for method in ("ghost", "direct"):
        ws = torch.empty(max(_capi.conv_workspace_bytes(geom, method, "bf16x3"), 4),
                         dtype=torch.uint8, device=cuda)
        sq = torch.full((act.shape[0],), 2.0, device=cuda)
        _capi.conv_pegrad_sqnorm(a, g, (k, k), s, p, sq, ws, method=method, precision="bf16x3",
                                 col_scale=torch.from_numpy(scale).to(cuda))
        out[method] = sq.cpu().numpy().astype(np.float64) - 2.0
    np.testing.assert_allclose(out["ghost"], ref, rtol=1e-4, atol=1e-7 * max(1.0, ref.max()))
    np.testing.assert_allclose(out["ghost"], out["direct"], rtol=2e-4)


def test_pgram_q_is_deterministic(cuda):
    """The quarter sums go to per-example partials reduced in a fixed order: bitwise repeatable."""
    act, gout, k, s, p = _conv_case(cuda, (64, 128, 16, 16, 128, 3, 1, 1), 3)
    a, g = torch.from_numpy(act).to(cuda), torch.from_numpy(gout).to(cuda)
    geom = _capi.conv_geom(a, g, (k, k), s, p)
    ws = torch.empty(_capi.conv_workspace_bytes(geom, "ghost", "bf16x3"), dtype=torch.uint8,
                     device=cuda)
    outs = []
    for _ in range(3):
        sq = torch.zeros(64, device=cuda)
        _capi.conv_pegrad_sqnorm(a, g, (k, k), s, p, sq, ws, method="ghost", precision="bf16x3")
        outs.append(sq.cpu())
    assert all(torch.equal(o, outs[0]) for o in outs)


# ---- BN affine per-example gradient norm (grand_params: all) ----------------------------------
@pytest.mark.parametrize("B,C,H,W,res", [(5, 64, 32, 32, False), (3, 128, 16, 16, True),
                                         (4, 256, 8, 8, False), (6, 512, 4, 4, True),
                                         (2, 7, 5, 5, True), (3, 33, 2, 2, False)])
def test_bn_pegrad_matches_oracle(cuda, B, C, H, W, res):
    rng = np.random.default_rng(B * C + H)
    out = rng.normal(size=(B, C, H, W)).astype(np.float32)
    r = rng.normal(size=(B, C, H, W)).astype(np.float32) if res else None
    g = (rng.normal(size=(B, C, H, W)) * (rng.random((B, C, H, W)) > 0.4)).astype(np.float32)
    gamma = rng.uniform(0.5, 1.5, C).astype(np.float32)
    beta = rng.normal(size=C).astype(np.float32) * 0.3
    v = out + r if res else out  # the tensor holding BN output + residual
    want = o_pegrad.bn_pegrad_sqnorm(out, g, gamma, beta) + 0.25
    sq = torch.full((B,), 0.25, device=cuda)
    t = lambda a: torch.from_numpy(a).to(cuda)  # noqa: E731
    _capi.bn_pegrad_sqnorm(t(v), t(g), t(gamma), t(beta), sq, r=t(r) if res else None)
    np.testing.assert_allclose(sq.cpu().numpy(), want, rtol=1e-4)


# ---- CIFAR head of the GraNd pass (avg-pool + linear backward) --------------------------------
@pytest.mark.parametrize("B,C,ncls,hw", [(5, 512, 10, 4), (3, 2048, 100, 4), (2, 70, 7, 3)])
def test_head_pool_and_backward(cuda, B, C, ncls, hw):
    g = torch.Generator().manual_seed(B * C + ncls)
    a = torch.randn(B, C, hw, hw, generator=g)
    e = torch.randn(B, ncls, generator=g)
    w = torch.randn(ncls, C, generator=g)
    feat = _capi.head_pool(a.to(cuda))
    torch.testing.assert_close(feat.cpu(), a.mean(dim=(2, 3)), rtol=1e-6, atol=1e-6)
    d = _capi.head_backward(a.to(cuda), e.to(cuda), w.to(cuda))
    want = (e @ w / (hw * hw))[:, :, None, None] * (a > 0)
    torch.testing.assert_close(d.cpu(), want, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("B,d,C,bias", [(1000, 512, 10, True), (37, 2048, 1000, True),
                                        (5, 100, 7, False), (130, 2048, 100, True),
                                        (3, 4096, 65, True), (1026, 2048, 1000, True),
                                        (9, 512, 300, False)])
def test_linear_forward_matches_fp64_and_is_batch_independent(cuda, B, d, C, bias):
    """dd_linear_forward (the classifier of the fast EL2N / GraNd passes, reference
    models/resnet.py:96) vs a float64 GEMM, and each row bitwise the same whatever the batch
    it is computed in (rows of a 1-, 3- and B-row call: the kernel's 4-row groups and 256-class
    slices cut differently, C = 300 ends in a partial slice)."""
    g = torch.Generator().manual_seed(B + d + C)
    feat = torch.randn(B, d, generator=g).relu()  # post-ReLU pooled features
    w = torch.randn(C, d, generator=g) / d ** 0.5
    b = torch.randn(C, generator=g) if bias else None
    want = feat.double() @ w.double().T + (b.double() if bias else 0)
    fd, wd = feat.to(cuda), w.to(cuda)
    bd = b.to(cuda) if bias else None
    got = _capi.linear_forward(fd, wd, bd)
    np.testing.assert_allclose(got.cpu().double().numpy(), want.numpy(), rtol=1e-5,
                               atol=1e-5 * float(want.abs().max()))
    for lo, hi in ((0, 1), (B // 2, min(B, B // 2 + 3))):
        part = _capi.linear_forward(fd[lo:hi].contiguous(), wd, bd)
        assert torch.equal(part, got[lo:hi])
