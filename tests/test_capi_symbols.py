"""libdd.so loads on a CPU-only host and exports every symbol include/dd_capi.h declares."""
import os
import re

from data_diet_distributed_amd import _capi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "dd_capi.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dd_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_binding_surface():
    assert set(declared_symbols()) == set(_capi.EXPORTS)


def test_library_exports_every_declared_symbol():
    lib = _capi.lib()
    for name in declared_symbols():
        assert hasattr(lib, name), name


def test_host_only_entry_points():
    # no device work: ABI version, keep-count, workspace queries, method planning
    assert _capi.lib().dd_abi_version() == 10
    assert _capi.keep_count(50000, 0.9) == 4999
    assert _capi.keep_count(2000, 0.8) == 399
    assert _capi.select_workspace_bytes(50000) > 50000 * 16
    g = _capi.ConvGeom(128, 64, 32, 32, 64, 32, 32, 3, 3, 1, 1)
    assert _capi.conv_method(g, "auto", "fp32") == "direct"
    assert _capi.conv_workspace_bytes(g, "direct", "fp32") == 128 * 9 * 4
    assert _capi.conv_method(g, "auto", "bf16x3") == "direct3x3"
    assert _capi.conv_workspace_bytes(g, "direct", "bf16x3") == 128 * 4
    g3 = _capi.ConvGeom(128, 256, 8, 8, 256, 8, 8, 3, 3, 1, 1)
    assert _capi.conv_method(g3, "auto", "fp32") == "ghost"
    g2 = _capi.ConvGeom(128, 64, 32, 32, 128, 16, 16, 3, 3, 2, 1)  # stride 2, 32-wide input
    assert _capi.conv_method(g2, "direct", "bf16x3") == "direct3x3"
    assert _capi.conv_method(g2, "direct", "fp32") == "direct"
    g5 = _capi.ConvGeom(8, 64, 30, 30, 128, 15, 15, 3, 3, 2, 1)  # stride 2, other widths
    assert _capi.conv_method(g5, "direct", "bf16x3") == "direct"
    g1 = _capi.ConvGeom(16, 256, 32, 32, 64, 32, 32, 1, 1, 1, 0)  # 1x1: split-bf16 GEMM form
    assert _capi.conv_method(g1, "direct", "bf16x3") == "direct1x1"
    assert _capi.conv_method(g1, "direct", "fp32") == "direct"
    # layout cin 256, cout 64 -> 4 waves along c: 256 c x 64 o per workgroup, one partial
    assert _capi.conv_workspace_bytes(g1, "direct", "bf16x3") == 16 * 4
    bad = _capi.ConvGeom(1, 3, 32, 32, 8, 31, 32, 3, 3, 1, 1)  # inconsistent ho
    assert _capi.conv_workspace_bytes(bad, "auto") == 0
    # the fused residual-unit input exists on the scoring tiles of the 3x3 conv only
    sup = _capi.conv3x3_unit_input_supported
    assert sup(32, 32, 64, 64, 128) and sup(16, 16, 128, 128, 128) and sup(8, 8, 256, 256, 128)
    assert not sup(4, 4, 512, 512, 128)     # 4x4: its residual registers would spill
    assert not sup(16, 16, 64, 64, 128)     # cout 64 at 16x16: the narrow tile, no fused form
    assert not sup(32, 32, 3, 64, 128)      # the stem layout
    assert not sup(8, 8, 256, 256, 3)       # 8x8 stages two images: the group must be even


def test_errors_are_reported_not_crashing():
    import ctypes
    rc = _capi.lib().dd_el2n(None, None, 4, 0, None, None, None, None, None)
    assert rc == -1
    assert b"C must be positive" in _capi.lib().dd_last_error()
    rc = _capi.lib().dd_select_topk(None, 10, 11, None, None, None, None, 0, None)
    assert rc == -1
    g = _capi.ConvGeom(4, 3, 8, 8, 8, 8, 8, 3, 3, 1, 1)
    rc = _capi.lib().dd_conv_pegrad_sqnorm(ctypes.c_void_p(16), ctypes.c_void_p(16),
                                           ctypes.byref(g), None, 0, 0, ctypes.c_void_p(16),
                                           None, 0, None)
    assert rc == -3  # workspace too small, detected before any launch


def test_round2_entry_points_validate_before_launching():
    """The round-2 symbols reject bad arguments with an error code and a message, before any
    device work (so this runs without a GPU)."""
    L = _capi.lib()
    P16 = __import__("ctypes").c_void_p(16)
    # implicit-GEMM conv: stride 3, then an empty output (7x7 kernel on a 3x3 map, no pad)
    assert L.dd_conv_gemm_forward(P16, 2, 3, 8, 8, 3, 3, 3, 1, P16, 8, None, None, 0, None,
                                  None, 1, 0, 0, None, P16, 0, 1.0, None) == -1
    assert b"stride" in L.dd_last_error()
    assert L.dd_conv_gemm_forward(P16, 2, 3, 3, 3, 7, 7, 1, 0, P16, 8, None, None, 0, None,
                                  None, 1, 0, 0, None, P16, 0, 1.0, None) == -1
    assert b"empty output" in L.dd_last_error()
    # ABI 7: the operand halves are checked (DD_OPERANDS_BF16X3 = 0, DD_OPERANDS_F16X3 = 1)
    assert L.dd_conv_gemm_forward(P16, 2, 3, 8, 8, 3, 3, 1, 1, P16, 8, None, None, 0, None,
                                  None, 1, 0, 0, None, P16, 5, 1.0, None) == -1
    assert b"operands" in L.dd_last_error()
    assert L.dd_conv3x3_pack(P16, 8, 8, 0, 2, 1.0, P16, None) == -1
    assert b"operands" in L.dd_last_error()
    assert L.dd_conv1x1_pack(P16, 8, 8, 0, -1, 1.0, P16, None) == -1
    assert b"operands" in L.dd_last_error()
    # weight / accumulator scales: 1 for bf16 packs, a power of two for fp16 ones
    assert L.dd_conv3x3_pack(P16, 8, 8, 0, 0, 2.0, P16, None) == -1
    assert b"scale" in L.dd_last_error()
    assert L.dd_conv1x1_pack(P16, 8, 8, 0, 1, 3.0, P16, None) == -1
    assert b"scale" in L.dd_last_error()
    assert L.dd_conv_gemm_forward(P16, 2, 3, 8, 8, 3, 3, 1, 1, P16, 8, None, None, 0, None,
                                  None, 1, 0, 0, None, P16, 1, 0.0, None) == -1
    assert b"acc_scale" in L.dd_last_error()
    # grouped layouts need whole 128-position tiles per group (32 x 49 positions is not)
    assert L.dd_conv1x1_tiles_per_group(7, 7, 32) < 0
    assert L.dd_conv1x1_tiles_per_group(7, 7, 128) == 128 * 49 // 64
    assert L.dd_conv_gemm_dense(3, 7, 7) == 1 and L.dd_conv_gemm_dense(64, 3, 3) == 0
    assert L.dd_conv_gemm_pack_bytes(64, 3, 7, 7) == 64 * 160 * 2 * 2  # K = 147 -> 160
    assert L.dd_conv_gemm_pack_bytes(64, 64, 3, 3) == 64 * 9 * 64 * 2 * 2
    # padded-width conv3x3 tiles (the statistics launch at widths that are not a tile width)
    assert L.dd_conv3x3_tiles_per_group(28, 28, 128) == 128 * 28 * 32 // 32
    assert L.dd_conv3x3_tiles_per_group(14, 14, 128) == 128 * 16 * 16 // 32
    assert L.dd_conv3x3_tiles_per_group(7, 7, 128) == 128 * 8 * 8 // 32
    assert L.dd_conv3x3_tiles_per_group(7, 7, 3) < 0  # two images per tile: an even group
    assert L.dd_conv3x3_tiles_per_group(32, 32, 128) == 128 * 32  # native, unchanged
    assert L.dd_conv3x3_padded_supported(28, 28, 128, 128, 128) == 1
    assert L.dd_conv3x3_padded_supported(14, 14, 256, 256, 128) == 1
    assert L.dd_conv3x3_padded_supported(7, 7, 512, 512, 128) == 1
    assert L.dd_conv3x3_padded_supported(56, 56, 64, 64, 128) == 1  # the 64-wide tile
    assert L.dd_conv3x3_tiles_per_group(56, 56, 128) == 128 * 56 * 64 // 32
    assert L.dd_conv3x3_padded_supported(72, 72, 64, 64, 128) == 0  # wider than a tile
    assert L.dd_conv3x3_padded_supported(28, 28, 64, 64, 128) == 0  # 128-output tiles
    assert L.dd_conv3x3_padded_supported(16, 16, 128, 128, 128) == 0  # native
    assert L.dd_conv3x3_padded_supported(30, 30, 128, 128, 128) == 0  # w % 4 past 16
    # padded-width stride-2 heads (a Bottleneck's conv2 statistics launch)
    assert L.dd_down_tiles_per_group(28, 28, 128) == 128 * 14 * 2
    assert L.dd_down_tiles_per_group(14, 14, 128) == 128 * 4 * 2
    assert L.dd_down_tiles_per_group(7, 7, 128) == 128 * 1 * 2
    assert L.dd_down_tiles_per_group(16, 16, 128) == 128 * 4 * 2  # native, unchanged
    assert L.dd_down_padded_supported(28, 28, 128, 128, 128) == 1
    assert L.dd_down_padded_supported(14, 14, 256, 256, 128) == 1
    assert L.dd_down_padded_supported(7, 7, 512, 512, 128) == 1
    assert L.dd_down_padded_supported(28, 28, 64, 128, 128) == 0  # cin <= 64: persistent heads
    assert L.dd_down_padded_supported(28, 28, 128, 64, 128) == 0  # 128-output tiles
    assert L.dd_down_padded_supported(16, 16, 128, 128, 128) == 0  # native
    assert L.dd_down_padded_supported(13, 13, 128, 128, 128) == 0  # odd past 8
    # the ImageNet stem conv
    assert L.dd_stem7_supported(224, 224, 3, 64, 128) == 1
    assert L.dd_stem7_tiles_per_group(224, 224, 128) == 128 * 56 * 8
    assert L.dd_stem7_supported(224, 224, 4, 64, 128) == 0  # 3 input channels
    assert L.dd_stem7_supported(224, 260, 3, 64, 128) == 0  # at most 128 output columns
    assert L.dd_stem7_supported(224, 228, 3, 128, 128) == 0  # 114 % 4, and 128 outputs
    # head kernels and the fused stem max-pool
    assert L.dd_head_backward(P16, P16, P16, 2, 0, 16, 10, 1.0, P16, None) == -1
    assert L.dd_head_pool(None, 2, 4, 16, None, None) == -1
    assert L.dd_bn_apply_maxpool(P16, 2, 4, 8, 8, 0, P16, P16, P16, None) == -1
    assert L.dd_bn_apply_maxpool(P16, 0, 4, 8, 8, 2, None, None, None, None) == 0  # B = 0


def test_product_path_fails_loudly_without_library(monkeypatch, tmp_path):
    import importlib
    import pytest
    monkeypatch.setenv("DD_LIB", str(tmp_path / "missing.so"))
    mod = importlib.reload(_capi)
    try:
        with pytest.raises(mod.DDError):
            mod.lib()
    finally:
        monkeypatch.delenv("DD_LIB")
        importlib.reload(_capi)
