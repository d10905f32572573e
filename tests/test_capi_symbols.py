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
    assert _capi.lib().dd_abi_version() == 3
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


def test_errors_are_reported_not_crashing():
    import ctypes
    rc = _capi.lib().dd_el2n(None, None, 4, 0, None, None, None, None)
    assert rc == -1
    assert b"C must be positive" in _capi.lib().dd_last_error()
    rc = _capi.lib().dd_select_topk(None, 10, 11, None, None, None, None, 0, None)
    assert rc == -1
    g = _capi.ConvGeom(4, 3, 8, 8, 8, 8, 8, 3, 3, 1, 1)
    rc = _capi.lib().dd_conv_pegrad_sqnorm(ctypes.c_void_p(16), ctypes.c_void_p(16),
                                           ctypes.byref(g), None, 0, 0, ctypes.c_void_p(16),
                                           None, 0, None)
    assert rc == -3  # workspace too small, detected before any launch


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
