"""ctypes binding of libdd.so (declared in include/dd_capi.h).

This is the only route from the host side to the HIP kernels.  There is no CPU or eager
PyTorch fallback: if the library is missing or a call fails, an exception is raised.
Tensors are checked for device/dtype/contiguity/shape here, so the C side only sees
consistent pointers and sizes.
"""
from __future__ import annotations

import ctypes
import math
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DD_LIB", os.path.join(_HERE, "libdd.so"))

(DD_PEGRAD_AUTO, DD_PEGRAD_DIRECT, DD_PEGRAD_GHOST, DD_PEGRAD_DIRECT3X3, DD_PEGRAD_PGRAM,
 DD_PEGRAD_STEM, DD_PEGRAD_DIRECT1X1, DD_PEGRAD_PGRAM_Q) = 0, 1, 2, 3, 4, 5, 6, 7
METHODS = {"auto": DD_PEGRAD_AUTO, "direct": DD_PEGRAD_DIRECT, "ghost": DD_PEGRAD_GHOST}
KERNELS = {DD_PEGRAD_DIRECT: "direct", DD_PEGRAD_GHOST: "ghost", DD_PEGRAD_DIRECT3X3: "direct3x3",
           DD_PEGRAD_PGRAM: "pgram", DD_PEGRAD_STEM: "stem", DD_PEGRAD_DIRECT1X1: "direct1x1",
           DD_PEGRAD_PGRAM_Q: "pgram_q"}
PRECISIONS = {"fp32": 0, "bf16x3": 1}
DEFAULT_PRECISION = "bf16x3"

# every symbol include/dd_capi.h declares (checked by tests/test_capi_symbols.py)
EXPORTS = (
    "dd_abi_version", "dd_last_error", "dd_normalize_u8", "dd_normalize_u8_gather", "dd_el2n",
    "dd_conv_pegrad_method", "dd_conv_pegrad_workspace_bytes", "dd_conv_pegrad_sqnorm",
    "dd_linear_pegrad_sqnorm", "dd_sqrt_accumulate", "dd_ensemble_finalize", "dd_keep_count",
    "dd_select_workspace_bytes", "dd_select_topk", "dd_conv3x3_pack_bytes", "dd_conv3x3_pack",
    "dd_conv3x3_tiles_per_group", "dd_conv3x3_padded_supported", "dd_conv3x3_mask_bytes", "dd_conv3x3_forward", "dd_channel_stats", "dd_bn_finalize",
    "dd_bn_apply", "dd_conv1x1_pack_bytes", "dd_conv1x1_pack", "dd_down_tiles_per_group",
    "dd_down_padded_supported", "dd_stem7_pack_bytes", "dd_stem7_pack", "dd_stem7_supported",
    "dd_stem7_tiles_per_group", "dd_stem7_forward",
    "dd_down_forward", "dd_down_backward", "dd_synth_images_u8", "dd_bn_pegrad_sqnorm",
    "dd_conv1x1_tiles_per_group", "dd_conv1x1_forward", "dd_conv_gemm_dense",
    "dd_conv_gemm_pack_bytes", "dd_conv_gemm_pack", "dd_conv_gemm_forward", "dd_head_pool",
    "dd_head_backward", "dd_bn_apply_maxpool", "dd_linear_forward",
    "dd_conv3x3_mask_plane_bits", "dd_conv3x3_unit_input_supported",
    "dd_conv3x3_forward_unit_input", "dd_down_forward_unit_input",
    "dd_conv1x1_forward_unit_input",
)


class DDError(RuntimeError):
    pass


class LabelError(ValueError, RuntimeError):
    """A label outside [0, C): the reference's one_hot(target, num_classes=10) raises a
    RuntimeError there (get_scores_and_prune.py:17); this is a ValueError too (a bad input)."""


class ConvGeom(ctypes.Structure):
    _fields_ = [("batch", ctypes.c_int64),
                ("cin", ctypes.c_int32), ("h", ctypes.c_int32), ("w", ctypes.c_int32),
                ("cout", ctypes.c_int32), ("ho", ctypes.c_int32), ("wo", ctypes.c_int32),
                ("kh", ctypes.c_int32), ("kw", ctypes.c_int32),
                ("stride", ctypes.c_int32), ("pad", ctypes.c_int32)]


_lib = None
_lock = threading.Lock()
P, I32, I64, F64, SZ = (ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_double,
                        ctypes.c_size_t)
F32 = ctypes.c_float


def lib():
    """Load libdd.so once; raise if it is absent (the product path has no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise DDError(f"libdd.so not found at {LIB_PATH}: build it with "
                              f"`python -c 'import __graft_entry__ as g; g.build()'`")
            L = ctypes.CDLL(LIB_PATH)
            sig = {
                "dd_abi_version": (I32, []),
                "dd_last_error": (ctypes.c_char_p, []),
                "dd_normalize_u8": (I32, [P, I64, I32, I64, P, P, P, P]),
                "dd_normalize_u8_gather": (I32, [P, P, I64, I32, I64, P, P, P, P]),
                "dd_synth_images_u8": (I32, [ctypes.c_uint64, I64, I64, I32, I32, I32, I32, P,
                                             P, P]),
                "dd_el2n": (I32, [P, P, I64, I32, P, P, P, P, P]),
                "dd_conv_pegrad_method": (I32, [ctypes.POINTER(ConvGeom), I32, I32]),
                "dd_conv_pegrad_workspace_bytes": (SZ, [ctypes.POINTER(ConvGeom), I32, I32]),
                "dd_conv_pegrad_sqnorm": (I32, [P, P, ctypes.POINTER(ConvGeom), P, I32, I32, P,
                                                P, SZ, P]),
                "dd_linear_pegrad_sqnorm": (I32, [P, P, I64, I32, I32, I32, P, P]),
                "dd_linear_forward": (I32, [P, P, P, I64, I32, I32, P, P]),
                "dd_sqrt_accumulate": (I32, [P, I64, P, P]),
                "dd_ensemble_finalize": (I32, [P, I64, I32, P, P]),
                "dd_keep_count": (I64, [I64, F64]),
                "dd_select_workspace_bytes": (SZ, [I64]),
                "dd_select_topk": (I32, [P, I64, I64, P, P, P, P, SZ, P]),
                "dd_conv3x3_pack_bytes": (SZ, [I32, I32]),
                "dd_conv3x3_pack": (I32, [P, I32, I32, I32, I32, F32, P, P]),
                "dd_conv3x3_tiles_per_group": (I32, [I32, I32, I32]),
                "dd_conv3x3_padded_supported": (I32, [I32, I32, I32, I32, I32]),
                "dd_conv3x3_mask_bytes": (SZ, [I64, I32, I32, I32]),
                "dd_conv3x3_forward": (I32, [P, I64, I32, I32, I32, P, I32, P, P, P, I32, P, P,
                                             I32, I32, I64, P, P, P, P, I32, F32, P]),
                "dd_channel_stats": (I32, [P, I64, I32, I64, I32, I64, P, P]),
                "dd_bn_finalize": (I32, [P, I64, I32, I64, I32, I32, I32, I32, I64, P, P, F32,
                                         P, P, P]),
                "dd_bn_apply": (I32, [P, I64, I32, I64, I32, P, P, P, P, P, I32, I32, P, P, P]),
                "dd_conv1x1_pack_bytes": (SZ, [I32, I32]),
                "dd_conv1x1_pack": (I32, [P, I32, I32, I32, I32, F32, P, P]),
                "dd_down_tiles_per_group": (I32, [I32, I32, I32]),
                "dd_down_padded_supported": (I32, [I32, I32, I32, I32, I32]),
                "dd_stem7_pack_bytes": (SZ, []),
                "dd_stem7_pack": (I32, [P, I32, I32, F32, P, P]),
                "dd_stem7_supported": (I32, [I32, I32, I32, I32, I32]),
                "dd_stem7_tiles_per_group": (I32, [I32, I32, I32]),
                "dd_stem7_forward": (I32, [P, I64, I32, I32, P, I32, I32, I64, P, P, I32, F32,
                                           P]),
                "dd_down_forward": (I32, [P, I64, I32, I32, I32, P, P, I32, P, I32, P, P, P,
                                          I32, P, P, I32, I64, I32, F32, F32, P]),
                "dd_down_backward": (I32, [P, P, I64, I32, I32, I32, P, P, I32, P, P, P, P]),
                "dd_conv3x3_mask_plane_bits": (I32, [P, I64, I32, I32, I32, P, P]),
                "dd_conv3x3_unit_input_supported": (I32, [I32, I32, I32, I32, I32]),
                "dd_down_forward_unit_input": (I32, [P, P, P, P, I64, I32, I32, I32, P, P, I32,
                                                     P, P, P, P, I32, I64, I32, F32, F32, P]),
                "dd_conv3x3_forward_unit_input": (I32, [P, P, P, P, P, P, P, I64, I32, I32, I32,
                                                        P, I32, I32, I64, P, P, I32, F32, P]),
                "dd_bn_pegrad_sqnorm": (I32, [P, P, P, I64, I32, I64, P, P, P, P]),
                "dd_conv1x1_tiles_per_group": (I32, [I32, I32, I32]),
                "dd_conv1x1_forward": (I32, [P, I64, I32, I32, I32, I32, P, I32, P, P, P, P, I32,
                                             P, P, I32, I32, I64, P, P, I32, F32, P]),
                "dd_conv1x1_forward_unit_input": (I32, [P, P, P, P, P, P, P, I64, I32, I32, I32,
                                                        P, I32, I32, I64, P, P, I32, F32, P]),
                "dd_conv_gemm_dense": (I32, [I32, I32, I32]),
                "dd_head_pool": (I32, [P, I64, I32, I32, P, P]),
                "dd_bn_apply_maxpool": (I32, [P, I64, I32, I32, I32, I32, P, P, P, P]),
                "dd_head_backward": (I32, [P, P, P, I64, I32, I32, I32, F32, P, P]),
                "dd_conv_gemm_pack_bytes": (SZ, [I32, I32, I32, I32]),
                "dd_conv_gemm_pack": (I32, [P, I32, I32, I32, I32, I32, F32, P, P]),
                "dd_conv_gemm_forward": (I32, [P, I64, I32, I32, I32, I32, I32, I32, I32, P, I32,
                                               P, P, I32, P, P, I32, I32, I64, P, P, I32, F32,
                                               P]),
            }
            for name, (res, args) in sig.items():
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            if L.dd_abi_version() != 10:
                raise DDError("libdd.so ABI mismatch")
            _lib = L
    return _lib


# ---- live kernel timing (bench.py) -----------------------------------------------------------
# When `kernel_log` is a list, every compute entry point below appends (kind, work, start,
# end, tag) per launch; `work` is the algorithmic flop (MFMA-bound kinds) or bytes (HBM-bound
# kinds) of the call, per SURVEY §8(d).  A pseudo-random 1 in `kernel_log_every` launches is
# bracketed with HIP events on its launch stream (start, end); the others are logged with
# start = end = None, so counts are exact and each (kind, shape) key's mean duration comes
# from its sampled launches.  Timing every launch costs ~3 % of wall time on this path (each
# event record is a queue marker between kernels).
kernel_log = None
kernel_log_every = 8
_sample_state = [0x9E3779B9]


def _t0(t: torch.Tensor, always: bool = False):
    """always: time every launch (kinds launched a few times per step, e.g. the select)."""
    if kernel_log is None:
        return None
    st = (_sample_state[0] * 1103515245 + 12345) & 0x7FFFFFFF
    _sample_state[0] = st
    if not always and (st >> 16) % kernel_log_every:
        return False  # counted, not timed
    e = torch.cuda.Event(enable_timing=True)
    e.record(torch.cuda.current_stream(t.device))
    return e


def _t1(e0, kind: str, work: float, t: torch.Tensor, tag: str = "", nbytes: float = 0.0):
    """Log one launch: kind, algorithmic work (flop or bytes, per bench.KINDS) and, for the
    matrix kernels, their algorithmic HBM bytes (operands read once, outputs written once),
    from which bench.py decides whether the MFMA or the HBM roofline binds."""
    if e0 is None or kernel_log is None:
        return
    if e0 is False:
        kernel_log.append((kind, float(work), None, None, tag, float(nbytes)))
        return
    e1 = torch.cuda.Event(enable_timing=True)
    e1.record(torch.cuda.current_stream(t.device))
    kernel_log.append((kind, float(work), e0, e1, tag, float(nbytes)))


def _conv_bytes(B, cin, h, w, cout, ho, wo, stride=1, k=1, extra=0):
    """Algorithmic HBM bytes of a conv launch: the input read once (a 1x1 stride-2 conv reads
    only the decimated positions), the output written once, plus `extra` same-size operands
    (residual, mask)."""
    inp = B * cin * (ho * wo if (k == 1 and stride > 1) else h * w)
    return 4.0 * (inp + B * cout * ho * wo * (1 + extra))


def pegrad_flop(g, kind: str) -> float:
    """Algorithmic flop of one dd_conv_pegrad_sqnorm call:
    direct 2 B T d_a d_g, ghost 2 B T^2 (d_a + d_g), shifted-Gram ghost 2 B (Ti^2 cin +
    T^2 cout) (unpadded shapes)."""
    T = g.ho * g.wo
    da = g.cin * g.kh * g.kw
    if kind in ("direct", "direct3x3", "direct1x1", "stem"):
        return 2.0 * g.batch * T * da * g.cout
    if kind == "pgram_q":  # the identity's work (the quarters also redo P's halo rows)
        return 2.0 * g.batch * ((g.h * g.w) ** 2 * g.cin + T * T * g.cout)
    if kind == "pgram":
        Ti = g.h * g.w
        if Ti > 64:  # stride 2: Grams of the parity classes the taps read (1 class for 1x1)
            ncls = 4 if g.kh == 3 else 1
            return 2.0 * g.batch * (ncls * (Ti // 4) ** 2 * g.cin + T * T * g.cout)
        return 2.0 * g.batch * (Ti * Ti * g.cin + T * T * g.cout)
    return 2.0 * g.batch * T * T * (da + g.cout)


def _check(rc: int, what: str):
    if rc != 0:
        msg = lib().dd_last_error().decode(errors="replace")
        raise DDError(f"{what} failed (rc={rc}): {msg}")


def _stream(t: torch.Tensor):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _dev(t, dtype, name, ndim=None):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if t.device.type != "cuda":
        raise ValueError(f"{name} must be a GPU tensor (got {t.device}); libdd has no CPU path")
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype} (got {t.dtype})")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if ndim is not None and t.dim() != ndim:
        raise ValueError(f"{name} must be {ndim}-D (got shape {tuple(t.shape)})")
    return ctypes.c_void_p(t.data_ptr())


def _opt(t, dtype, name, numel=None):
    if t is None:
        return ctypes.c_void_p(0)
    p = _dev(t, dtype, name)
    if numel is not None and t.numel() != numel:
        raise ValueError(f"{name} must have {numel} elements (got {t.numel()})")
    return p


# ---- input feed ------------------------------------------------------------------------------
def normalize_u8(img: torch.Tensor, mean, std, out: torch.Tensor, index: torch.Tensor = None):
    """out = (img / 255 - mean) / std  (reference data/loader.py:8-11).  img uint8 [n,C,H,W]
    (or the whole set when `index` gathers rows of it)."""
    _dev(img, torch.uint8, "img")
    n = out.shape[0]
    C = img.shape[1]
    hw = img[0, 0].numel()
    if out.shape[1:] != img.shape[1:]:
        raise ValueError("out must be [n, C, H, W] like img")
    if index is None and img.shape[0] != n:
        raise ValueError("img and out batch sizes differ")
    m = (ctypes.c_float * C)(*[float(v) for v in mean])
    s = (ctypes.c_float * C)(*[float(v) for v in std])
    if index is None:
        rc = lib().dd_normalize_u8(_dev(img, torch.uint8, "img"), n, C, hw, m, s,
                                   _dev(out, torch.float32, "out"), _stream(out))
    else:
        if index.numel() != n:
            raise ValueError("index must have n entries")
        rc = lib().dd_normalize_u8_gather(_dev(img, torch.uint8, "img"),
                                          _dev(index, torch.int64, "index"), n, C, hw, m, s,
                                          _dev(out, torch.float32, "out"), _stream(out))
    _check(rc, "dd_normalize_u8")
    return out


def synth_images_u8(seed: int, idx0: int, n: int, num_classes: int, hw: int = 32,
                    channels: int = 3, device="cuda"):
    """Examples idx0 .. idx0+n-1 of the synthetic set `seed`, generated in HBM
    (dd_synth_images_u8): (uint8 [n, channels, hw, hw], int64 labels [n])."""
    img = torch.empty((n, channels, hw, hw), dtype=torch.uint8, device=device)
    lab = torch.empty((n,), dtype=torch.int64, device=device)
    if n:
        e0 = _t0(img)
        rc = lib().dd_synth_images_u8(int(seed) & (2**64 - 1), idx0, n, channels, hw, hw,
                                      num_classes, _dev(img, torch.uint8, "img"),
                                      _dev(lab, torch.int64, "labels"), _stream(img))
        _t1(e0, "synth", float(img.numel() + 8 * n), img)
        _check(rc, "dd_synth_images_u8")
    return img, lab


# ---- EL2N ------------------------------------------------------------------------------------
def el2n(logits: torch.Tensor, labels: torch.Tensor, score=None, e=None, accum=None,
         bad_labels=None):
    """EL2N rows (reference get_scores_and_prune.py:16-18); writes whichever outputs given.
    bad_labels: int32 [1] device counter += rows whose label is outside [0, C) (their score,
    accum term and e row are NaN; check_labels() turns a non-zero count into LabelError)."""
    _dev(logits, torch.float32, "logits", 2)
    B, C = logits.shape
    if labels.numel() != B:
        raise ValueError("labels must have B entries")
    if e is not None and tuple(e.shape) != (B, C):
        raise ValueError("e must be [B, C]")
    e0 = _t0(logits)
    rc = lib().dd_el2n(_dev(logits, torch.float32, "logits"), _dev(labels, torch.int64, "labels"),
                       B, C, _opt(score, torch.float32, "score", B),
                       _opt(e, torch.float32, "e", B * C),
                       _opt(accum, torch.float32, "accum", B),
                       _opt(bad_labels, torch.int32, "bad_labels", 1), _stream(logits))
    _check(rc, "dd_el2n")
    # logits + int64 label + each output written (accum: read-modify-write)
    _t1(e0, "el2n", B * (4 * C + 8 + (4 if score is not None else 0) +
                         (4 * C if e is not None else 0) + (8 if accum is not None else 0)),
        logits)


def label_counter(device) -> torch.Tensor:
    """A zeroed int32 [1] device counter for el2n(bad_labels=)."""
    return torch.zeros(1, dtype=torch.int32, device=device)


def check_labels(counter: torch.Tensor, num_classes: int, where: str = "scoring"):
    """Raise LabelError if el2n counted labels outside [0, num_classes) (one device -> host
    read), as the reference's one_hot raises on the first such batch (:17)."""
    c = int(counter.item())
    if c:
        raise LabelError(f"{where}: {c} label(s) outside [0, {num_classes}) -- the reference's "
                         f"one_hot(target, num_classes={num_classes}) rejects them")


# ---- GraNd -----------------------------------------------------------------------------------
def conv_geom(act: torch.Tensor, gout: torch.Tensor, kernel_size, stride, padding) -> ConvGeom:
    B, cin, h, w = act.shape
    B2, cout, ho, wo = gout.shape
    if B != B2:
        raise ValueError("act/gout batch mismatch")
    kh, kw = kernel_size
    return ConvGeom(B, cin, h, w, cout, ho, wo, kh, kw, stride, padding)


def conv_method(g: ConvGeom, method: str = "auto", precision: str = DEFAULT_PRECISION) -> str:
    """Kernel a request resolves to: "direct", "ghost", "direct3x3", "pgram" or "stem"."""
    m = lib().dd_conv_pegrad_method(ctypes.byref(g), METHODS[method], PRECISIONS[precision])
    _check(0 if m > 0 else m, "dd_conv_pegrad_method")
    return KERNELS[m]


def conv_workspace_bytes(g: ConvGeom, method: str = "auto",
                         precision: str = DEFAULT_PRECISION) -> int:
    return int(lib().dd_conv_pegrad_workspace_bytes(ctypes.byref(g), METHODS[method],
                                                    PRECISIONS[precision]))


def conv_pegrad_sqnorm(act, gout, kernel_size, stride, padding, sq_accum, workspace,
                       method="auto", col_scale=None, precision=DEFAULT_PRECISION):
    """sq_accum[b] += ||grad_W loss_b||_F^2 for one Conv2d (no bias)."""
    _dev(act, torch.float32, "act", 4)
    _dev(gout, torch.float32, "gout", 4)
    g = conv_geom(act, gout, kernel_size, stride, padding)
    need = conv_workspace_bytes(g, method, precision)
    if workspace.numel() * workspace.element_size() < need:
        raise DDError(f"workspace too small: {workspace.numel() * workspace.element_size()} < {need}")
    if sq_accum.numel() != g.batch:
        raise ValueError("sq_accum must have B entries")
    e0 = _t0(act)
    rc = lib().dd_conv_pegrad_sqnorm(
        _dev(act, torch.float32, "act"), _dev(gout, torch.float32, "gout"), ctypes.byref(g),
        _opt(col_scale, torch.float32, "col_scale", g.cout), METHODS[method],
        PRECISIONS[precision], _dev(sq_accum, torch.float32, "sq_accum"), ctypes.c_void_p(workspace.data_ptr()),
        workspace.numel() * workspace.element_size(), _stream(act))
    _check(rc, "dd_conv_pegrad_sqnorm")
    if e0 is not None:
        kind = conv_method(g, method, precision)
        # the stem kernel is bound by reading its operands once: its work unit is bytes
        nbytes = 4.0 * (act.numel() + gout.numel())  # both operands read once
        work = nbytes if kind == "stem" else pegrad_flop(g, kind)
        _t1(e0, kind, work, act, nbytes=0.0 if kind == "stem" else nbytes)


def linear_forward(feat: torch.Tensor, weight: torch.Tensor, bias=None, out=None):
    """Classifier logits feat W^T + bias [B, C] (dd_linear_forward): each row reduced in a fixed
    order from that row alone, so logits do not depend on the batch size (a library GEMM picks
    its kernel, and its rounding, per batch size)."""
    _dev(feat, torch.float32, "feat", 2)
    _dev(weight, torch.float32, "weight", 2)
    B, d = feat.shape
    C = weight.shape[0]
    if weight.shape[1] != d:
        raise ValueError(f"feat has {d} features, weight {tuple(weight.shape)}")
    if bias is not None:
        _dev(bias, torch.float32, "bias", 1)
        if bias.numel() != C:
            raise ValueError("bias must have C entries")
    if out is None:
        out = torch.empty((B, C), dtype=torch.float32, device=feat.device)
    elif tuple(out.shape) != (B, C):
        raise ValueError("out must be [B, C]")
    e0 = _t0(feat)
    rc = lib().dd_linear_forward(_dev(feat, torch.float32, "feat"),
                                 _dev(weight, torch.float32, "weight"),
                                 _opt(bias, torch.float32, "bias", C), B, d, C,
                                 _dev(out, torch.float32, "out"), _stream(feat))
    _check(rc, "dd_linear_forward")
    _t1(e0, "linear", 4.0 * (B * d + C * d + B * C), feat)
    return out


def linear_pegrad_sqnorm(act, gout, sq_accum, has_bias=True):
    _dev(act, torch.float32, "act", 2)
    _dev(gout, torch.float32, "gout", 2)
    B, din = act.shape
    if gout.shape[0] != B or sq_accum.numel() != B:
        raise ValueError("batch mismatch")
    rc = lib().dd_linear_pegrad_sqnorm(_dev(act, torch.float32, "act"),
                                       _dev(gout, torch.float32, "gout"), B, din,
                                       gout.shape[1], int(bool(has_bias)),
                                       _dev(sq_accum, torch.float32, "sq_accum"), _stream(act))
    _check(rc, "dd_linear_pegrad_sqnorm")


def bn_pegrad_sqnorm(v, g, gamma, beta, sq_accum, r=None):
    """sq_accum[b] += ||d loss_b / d(gamma, beta)||^2 of an eval-mode BN (dd_bn_pegrad_sqnorm):
    v = the BN output (+ r) wherever g != 0, g = d loss / d BN output, both [B, C, H, W]."""
    _dev(v, torch.float32, "v", 4)
    _dev(g, torch.float32, "g", 4)
    B, C, h, w = v.shape
    if tuple(g.shape) != tuple(v.shape) or (r is not None and tuple(r.shape) != tuple(v.shape)):
        raise ValueError("v, g (and r) must have the same shape")
    if sq_accum.numel() != B:
        raise ValueError("sq_accum must have B entries")
    e0 = _t0(v)
    rc = lib().dd_bn_pegrad_sqnorm(_dev(v, torch.float32, "v"), _opt(r, torch.float32, "r"),
                                   _dev(g, torch.float32, "g"), B, C, h * w,
                                   _opt(gamma, torch.float32, "gamma", C),
                                   _opt(beta, torch.float32, "beta", C),
                                   _dev(sq_accum, torch.float32, "sq_accum"), _stream(v))
    _check(rc, "dd_bn_pegrad_sqnorm")
    _t1(e0, "bn_pegrad", 4.0 * v.numel() * (2 + (r is not None)), v)


def sqrt_accumulate(sq, accum):
    if sq.numel() != accum.numel():
        raise ValueError("size mismatch")
    rc = lib().dd_sqrt_accumulate(_dev(sq, torch.float32, "sq"), sq.numel(),
                                  _dev(accum, torch.float32, "accum"), _stream(sq))
    _check(rc, "dd_sqrt_accumulate")


def ensemble_finalize(accum, K: int, out):
    if accum.numel() != out.numel():
        raise ValueError("size mismatch")
    rc = lib().dd_ensemble_finalize(_dev(accum, torch.float32, "accum"), accum.numel(), int(K),
                                    _dev(out, torch.float32, "out"), _stream(accum))
    _check(rc, "dd_ensemble_finalize")


# ---- selection -------------------------------------------------------------------------------
def keep_count(train_samples: int, sparsity: float) -> int:
    return int(lib().dd_keep_count(int(train_samples), float(sparsity)))


def select_workspace_bytes(n: int) -> int:
    return int(lib().dd_select_workspace_bytes(int(n)))


def select_topk(keys: torch.Tensor, k: int, idx_out=None, workspace=None, check_nan=True):
    """Indices of the k largest keys, descending, ties by ascending index (stable sort).

    Returns (idx int64[k], threshold fp32[1] tensor, nan_count int32[1] tensor) on device.
    With check_nan the NaN count is read back (one sync) and a NaN raises ValueError.
    """
    _dev(keys, torch.float32, "keys", 1)
    n = keys.numel()
    if not 0 <= k <= n:
        raise ValueError(f"k={k} outside [0, {n}]")
    dev = keys.device
    if idx_out is None:
        idx_out = torch.empty(k, dtype=torch.int64, device=dev)
    need = select_workspace_bytes(n)
    if workspace is None or workspace.numel() * workspace.element_size() < need:
        workspace = torch.empty(need, dtype=torch.uint8, device=dev)
    thr = torch.empty(1, dtype=torch.float32, device=dev)
    nan = torch.empty(1, dtype=torch.int32, device=dev)
    e0 = _t0(keys, always=True)
    rc = lib().dd_select_topk(_dev(keys, torch.float32, "keys"), n, int(k),
                              _opt(idx_out, torch.int64, "idx_out", k), _dev(thr, torch.float32, "thr"),
                              _dev(nan, torch.int32, "nan"), ctypes.c_void_p(workspace.data_ptr()),
                              workspace.numel() * workspace.element_size(), _stream(keys))
    _check(rc, "dd_select_topk")
    _t1(e0, "select", 4.0 * n + 8.0 * k, keys)  # algorithmic minimum: keys once + int64 idx
    if check_nan:
        c = int(nan.item())
        if c != 0:
            raise ValueError(f"{c} NaN score(s): the keep-set is undefined")
    return idx_out, thr, nan


# ---- operand halves of the split MFMA convs (include/dd_capi.h DD_OPERANDS_*) -----------------
OPERANDS = {"bf16x3": 0, "f16x3": 1}


def _operands_code(operands: str) -> int:
    try:
        return OPERANDS[operands]
    except KeyError:
        raise ValueError(f"operands must be one of {sorted(OPERANDS)}") from None


def _pack_tag(packed: torch.Tensor, name: str):
    """A pack's operand tag.  Every pack function tags the tensor it returns (_tag_pack);
    clone(), .to(), slicing or torch.save/load return a tensor without the Python attributes,
    and reading such a copy as bf16 would run an fp16 pack's bit patterns (scaled by 2^s) as
    bf16 with no error: refuse it instead."""
    try:
        return getattr(packed, name)
    except AttributeError:
        raise DDError("weight pack without its operand tag (a copy of a pack loses the "
                      "dd_operands / dd_scale attributes): re-pack from the weights") from None


def pack_operands(packed: torch.Tensor) -> int:
    """DD_OPERANDS_* code a pack was made with (carried on the pack tensor)."""
    return _pack_tag(packed, "dd_operands")


def pack_acc_scale(packed: torch.Tensor) -> float:
    """The accumulator scale of a pack's forward: 1 / its weight scale (a power of two)."""
    return 1.0 / _pack_tag(packed, "dd_scale")


def _pack_scale(weight: torch.Tensor, code: int) -> float:
    """Weight scale of a pack (include/dd_capi.h): 1 for bf16; for fp16 the power of two that
    puts max|W| in [2^12, 2^13), so the lo halves of small weights stay normal fp16 numbers.
    (One device -> host read per pack: packs are made once per checkpoint.)"""
    if code == OPERANDS["bf16x3"]:
        return 1.0
    m = float(weight.detach().abs().max().item()) if weight.numel() else 0.0
    if not math.isfinite(m):
        raise ValueError("non-finite weights cannot be packed")
    if m == 0.0:
        return 1.0
    e = 13 - math.frexp(m)[1]  # m < 2^frexp_e: m * 2^e < 2^13
    return float(2.0 ** max(-100, min(100, e)))


def _tag_pack(packed: torch.Tensor, code: int, scale: float = 1.0) -> torch.Tensor:
    packed.dd_operands = code
    packed.dd_scale = scale
    return packed


# ---- backbone 3x3 stride-1 conv (split MFMA) ---------------------------------------------------
def conv3x3_pack(weight: torch.Tensor, transpose_flip: bool = False,
                 operands: str = "bf16x3") -> torch.Tensor:
    """Pack fp32 weights [cout, cin, 3, 3] for dd_conv3x3_forward (transpose_flip: the
    backward-data conv of this weight; operands: "bf16x3" or "f16x3" halves, carried on the
    returned tensor so the forward launches with the matching kernels)."""
    code = _operands_code(operands)
    _dev(weight, torch.float32, "weight", 4)
    cout, cin, kh, kw = weight.shape
    if (kh, kw) != (3, 3):
        raise ValueError("3x3 weights only")
    oc, ic = (cin, cout) if transpose_flip else (cout, cin)
    packed = torch.empty(lib().dd_conv3x3_pack_bytes(oc, ic), dtype=torch.uint8,
                         device=weight.device)
    scale = _pack_scale(weight, code)
    rc = lib().dd_conv3x3_pack(_dev(weight, torch.float32, "weight"), cout, cin,
                               int(bool(transpose_flip)), code, scale,
                               ctypes.c_void_p(packed.data_ptr()), _stream(weight))
    _check(rc, "dd_conv3x3_pack")
    return _tag_pack(packed, code, scale)


def conv3x3_mask_bytes(B: int, out_channels: int, h: int, w: int) -> int:
    return int(lib().dd_conv3x3_mask_bytes(int(B), int(out_channels), int(h), int(w)))


def conv3x3_mask(B: int, out_channels: int, h: int, w: int, device) -> torch.Tensor:
    """Buffer for a fragment-order ReLU mask (conv3x3 mask_out / mask_in)."""
    return torch.empty(conv3x3_mask_bytes(B, out_channels, h, w), dtype=torch.uint8,
                       device=device)


def _mask_ptr(m, B, cout, h, w):
    if m is None:
        return None
    _dev(m, torch.uint8, "mask")
    need = conv3x3_mask_bytes(B, cout, h, w)
    if m.numel() < need:
        raise ValueError(f"mask buffer must have {need} bytes (got {m.numel()})")
    return ctypes.c_void_p(m.data_ptr())


def conv3x3_tiles_per_group(h: int, w: int, group_size: int) -> int:
    t = int(lib().dd_conv3x3_tiles_per_group(int(h), int(w), int(group_size)))
    if t < 0:
        raise DDError(f"no conv3x3 tile geometry for {h}x{w} with group_size {group_size}")
    return t


class BNStats:
    """Partial BN statistics of one producer: buffer [G, C, tiles, 2] + its tile geometry."""

    def __init__(self, buf, groups, group_size, n_valid, tiles, images_per_tile, row_tiles,
                 channels, hw):
        self.buf, self.groups, self.group_size, self.n_valid = buf, groups, group_size, n_valid
        self.tiles, self.images_per_tile, self.row_tiles = tiles, images_per_tile, row_tiles
        self.channels, self.hw = channels, hw


def _stats_buffer(buf, G, C, tiles, device):
    need = G * C * tiles * 2
    if buf is None or buf.numel() < need:
        return torch.empty(need, dtype=torch.float32, device=device)
    return buf


def conv3x3(x: torch.Tensor, packed: torch.Tensor, out_channels: int, bias=None, residual=None,
            mask_src=None, relu=False, out=None, in_affine=None, in_relu=True, group_size=None,
            stats=False, n_stat=None, stats_buf=None, mask_out=None, mask_in=None):
    """y = epilogue(conv3x3_s1_p1(xf(x))) with the packed weights (see include/dd_capi.h).

    in_affine = (scale, shift) [G, cin]: the producer's grouped train-mode BN (+ ReLU if
    in_relu) applied while x is staged.  stats=True also returns the BN partial statistics of
    y over rows < n_stat (default all) as a BNStats: returns (y, BNStats).
    mask_out (uint8 tensor of conv3x3_mask_bytes bytes) receives the ReLU mask (y > 0) in
    fragment order; mask_in (such a tensor from a launch of the same geometry) replaces
    mask_src."""
    _dev(x, torch.float32, "x", 4)
    B, cin, h, w = x.shape
    shape = (B, out_channels, h, w)
    if out is None:
        out = torch.empty(shape, dtype=torch.float32, device=x.device)
    for name, t in (("residual", residual), ("mask_src", mask_src), ("out", out)):
        if t is not None and tuple(t.shape) != shape:
            raise ValueError(f"{name} must be {shape}")
    grouped = in_affine is not None or stats
    gs = int(group_size) if group_size is not None else 0
    if grouped and gs <= 0:
        raise ValueError("group_size is required with in_affine / stats")
    G = -(-B // gs) if grouped else 1
    sc = sh = None
    if in_affine is not None:
        sc, sh = in_affine
        for name, t in (("in_scale", sc), ("in_shift", sh)):
            _dev(t, torch.float32, name)
            if t.numel() != G * cin:
                raise ValueError(f"{name} must have G*cin = {G * cin} entries")
    st = None
    nst = B if n_stat is None else int(n_stat)
    if stats:
        tiles = conv3x3_tiles_per_group(h, w, gs)
        sbuf = _stats_buffer(stats_buf, G, out_channels, tiles, x.device)
        # one partial per 32 consecutive positions of a group (two images at 4x4)
        ipt = max(1, 32 // (h * w))
        st = BNStats(sbuf, G, gs, min(max(nst, 0), B), tiles, ipt, tiles // (gs // ipt),
                     out_channels, h * w)
    e0 = _t0(x)
    rc = lib().dd_conv3x3_forward(_dev(x, torch.float32, "x"), B, cin, h, w,
                                  ctypes.c_void_p(packed.data_ptr()), out_channels,
                                  _opt(bias, torch.float32, "bias", out_channels),
                                  _opt(residual, torch.float32, "residual"),
                                  _opt(mask_src, torch.float32, "mask_src"), int(bool(relu)),
                                  _opt(sc, torch.float32, "in_scale"),
                                  _opt(sh, torch.float32, "in_shift"), int(bool(in_relu)),
                                  gs, nst, ctypes.c_void_p(st.buf.data_ptr()) if st else None,
                                  _mask_ptr(mask_out, B, out_channels, h, w),
                                  _mask_ptr(mask_in, B, out_channels, h, w),
                                  _dev(out, torch.float32, "out"), pack_operands(packed),
                                  pack_acc_scale(packed), _stream(x))
    _check(rc, "dd_conv3x3_forward")
    _t1(e0, "conv3x3", 2.0 * B * h * w * cin * out_channels * 9, x,
        tag="stats" if stats else "mask" if mask_src is not None else
        "bias" if bias is not None else "plain",
        nbytes=_conv_bytes(B, cin, h, w, out_channels, h, w, 1, 3,
                           (residual is not None) + (mask_src is not None)))
    return (out, st) if stats else out


def conv3x3_padded_supported(h: int, w: int, cin: int, cout: int, group_size: int) -> bool:
    """A statistics launch of this shape runs on the padded-width tiles (dd_conv3x3_forward,
    ABI 10: widths that are not a tile width, e.g. the ImageNet-stem network's 28 / 14 / 7)."""
    return lib().dd_conv3x3_padded_supported(int(h), int(w), int(cin), int(cout),
                                             int(group_size)) == 1


def conv3x3_unit_input_supported(h: int, w: int, cin: int, cout: int, group_size: int) -> bool:
    return lib().dd_conv3x3_unit_input_supported(int(h), int(w), int(cin), int(cout),
                                                 int(group_size)) == 1


def conv3x3_unit_input(y_prev: torch.Tensor, affine, packed: torch.Tensor, out_channels: int,
                       group_size: int, residual=None, res_affine=None, n_stat=None,
                       stats_buf=None, x_out=None, out=None):
    """The residual unit's output x = relu(y_prev * scale + shift + R) (R = 0, residual, or
    residual * res_scale + res_shift; grouped train-mode BN) computed while the next unit's
    first conv stages it: returns (x, y = conv3x3(x), BNStats of y).  x is bitwise
    bn_apply's output and y bitwise conv3x3's on it (include/dd_capi.h)."""
    _dev(y_prev, torch.float32, "y_prev", 4)
    B, cin, h, w = y_prev.shape
    gs = int(group_size)
    G = -(-B // gs)
    scale, shift = affine
    for name, t in (("scale", scale), ("shift", shift)):
        _dev(t, torch.float32, name)
        if t.numel() != G * cin:
            raise ValueError(f"{name} must have G*cin = {G * cin} entries")
    if residual is not None:
        _dev(residual, torch.float32, "residual")
        if residual.shape != y_prev.shape:
            raise ValueError("residual must match y_prev")
    rs = rt = None
    if res_affine is not None:
        if residual is None:
            raise ValueError("res_affine needs residual")
        rs, rt = res_affine
        for name, t in (("res_scale", rs), ("res_shift", rt)):
            _dev(t, torch.float32, name)
            if t.numel() != G * cin:
                raise ValueError(f"{name} must have G*cin = {G * cin} entries")
    if x_out is None:
        x_out = torch.empty_like(y_prev)
    elif x_out.shape != y_prev.shape:
        raise ValueError("x_out must match y_prev")
    shape = (B, out_channels, h, w)
    if out is None:
        out = torch.empty(shape, dtype=torch.float32, device=y_prev.device)
    elif tuple(out.shape) != shape:
        raise ValueError(f"out must be {shape}")
    nst = B if n_stat is None else int(n_stat)
    tiles = conv3x3_tiles_per_group(h, w, gs)
    sbuf = _stats_buffer(stats_buf, G, out_channels, tiles, y_prev.device)
    ipt = max(1, 32 // (h * w))
    st = BNStats(sbuf, G, gs, min(max(nst, 0), B), tiles, ipt, tiles // (gs // ipt),
                 out_channels, h * w)
    e0 = _t0(y_prev)
    rc = lib().dd_conv3x3_forward_unit_input(
        _dev(y_prev, torch.float32, "y_prev"), _dev(scale, torch.float32, "scale"),
        _dev(shift, torch.float32, "shift"), _opt(residual, torch.float32, "residual"),
        _opt(rs, torch.float32, "res_scale"), _opt(rt, torch.float32, "res_shift"),
        _dev(x_out, torch.float32, "x_out"), B, cin, h, w, ctypes.c_void_p(packed.data_ptr()),
        out_channels, gs, nst, ctypes.c_void_p(sbuf.data_ptr()), _dev(out, torch.float32, "out"),
        pack_operands(packed), pack_acc_scale(packed), _stream(y_prev))
    _check(rc, "dd_conv3x3_forward_unit_input")
    # the conv's bytes plus the residual read and the unit output written
    _t1(e0, "conv3x3_unit", 2.0 * B * h * w * cin * out_channels * 9, y_prev, tag="stats",
        nbytes=_conv_bytes(B, cin, h, w, out_channels, h, w, 1, 3)
        + 4.0 * B * cin * h * w * (1 + (residual is not None)))
    return x_out, out, st


def channel_stats(y: torch.Tensor, group_size: int, n_stat=None, stats_buf=None) -> BNStats:
    """BN partial statistics of an NCHW tensor (any producer) per group of examples."""
    _dev(y, torch.float32, "y", 4)
    B, C, h, w = y.shape
    G = -(-B // group_size)
    sbuf = _stats_buffer(stats_buf, G, C, group_size, y.device)
    nst = B if n_stat is None else min(max(int(n_stat), 0), B)
    rc = lib().dd_channel_stats(_dev(y, torch.float32, "y"), B, C, h * w, int(group_size), nst,
                                ctypes.c_void_p(sbuf.data_ptr()), _stream(y))
    _check(rc, "dd_channel_stats")
    return BNStats(sbuf, G, int(group_size), nst, int(group_size), 1, 1, C, h * w)


def bn_finalize(st: BNStats, gamma: torch.Tensor, beta: torch.Tensor, eps: float,
                scale=None, shift=None):
    """(scale, shift) [G, C] of grouped train-mode BN from partial statistics."""
    G, C = st.groups, st.channels
    dev = st.buf.device
    if scale is None:
        scale = torch.empty((G, C), dtype=torch.float32, device=dev)
    if shift is None:
        shift = torch.empty((G, C), dtype=torch.float32, device=dev)
    for name, t in (("gamma", gamma), ("beta", beta)):
        _dev(t, torch.float32, name)
        if t.numel() != C:
            raise ValueError(f"{name} must have {C} entries")
    rc = lib().dd_bn_finalize(ctypes.c_void_p(st.buf.data_ptr()), G, st.group_size, st.n_valid,
                              st.tiles, st.images_per_tile, st.row_tiles, C, st.hw,
                              _dev(gamma, torch.float32, "gamma"),
                              _dev(beta, torch.float32, "beta"), float(eps),
                              _opt(scale, torch.float32, "scale", G * C),
                              _opt(shift, torch.float32, "shift", G * C), _stream(gamma))
    _check(rc, "dd_bn_finalize")
    return scale, shift


def bn_apply_maxpool(y: torch.Tensor, affine, group_size: int) -> torch.Tensor:
    """max_pool2d(relu(y * scale + shift), 3, stride 2, padding 1): the ImageNet stem tail."""
    _dev(y, torch.float32, "y", 4)
    B, C, h, w = y.shape
    G = -(-B // group_size)
    scale, shift = affine
    for name, t in (("scale", scale), ("shift", shift)):
        _dev(t, torch.float32, name)
        if t.numel() != G * C:
            raise ValueError(f"{name} must have G*C = {G * C} entries")
    out = torch.empty((B, C, (h - 1) // 2 + 1, (w - 1) // 2 + 1), dtype=torch.float32,
                      device=y.device)
    e0 = _t0(y)
    rc = lib().dd_bn_apply_maxpool(_dev(y, torch.float32, "y"), B, C, h, w, int(group_size),
                                   _dev(scale, torch.float32, "scale"),
                                   _dev(shift, torch.float32, "shift"),
                                   _dev(out, torch.float32, "out"), _stream(y))
    _check(rc, "dd_bn_apply_maxpool")
    _t1(e0, "bn_apply", 4.0 * (y.numel() + out.numel()), y, tag="maxpool")
    return out


def bn_apply(y: torch.Tensor, affine, group_size: int, residual=None, res_affine=None,
             res_relu=False, relu=True, out=None, pool_out=None, write_out=True):
    """out = relu?(y * scale + shift + R) (grouped BN apply + residual); pool_out [B, C] gets
    the spatial mean.  Returns (out or None, pool_out or None)."""
    _dev(y, torch.float32, "y", 4)
    B, C, h, w = y.shape
    G = -(-B // group_size)
    scale, shift = affine
    for name, t in (("scale", scale), ("shift", shift)):
        _dev(t, torch.float32, name)
        if t.numel() != G * C:
            raise ValueError(f"{name} must have G*C = {G * C} entries")
    if residual is not None:
        _dev(residual, torch.float32, "residual")
        if residual.shape != y.shape:
            raise ValueError("residual must match y")
    rs = rt = None
    if res_affine is not None:
        rs, rt = res_affine
    if write_out and out is None:
        out = torch.empty_like(y)
    e0 = _t0(y)
    rc = lib().dd_bn_apply(_dev(y, torch.float32, "y"), B, C, h * w, int(group_size),
                           _dev(scale, torch.float32, "scale"), _dev(shift, torch.float32, "shift"),
                           _opt(residual, torch.float32, "residual"),
                           _opt(rs, torch.float32, "res_scale", G * C),
                           _opt(rt, torch.float32, "res_shift", G * C), int(bool(res_relu)),
                           int(bool(relu)), _opt(out if write_out else None, torch.float32, "out"),
                           _opt(pool_out, torch.float32, "pool_out", B * C), _stream(y))
    _check(rc, "dd_bn_apply")
    _t1(e0, "bn_apply", 4.0 * y.numel() * (1 + (residual is not None) + bool(write_out)), y)
    return (out if write_out else None), pool_out


# ---- 1x1 convolution (split-bf16 GEMM) ---------------------------------------------------------
def conv1x1(x: torch.Tensor, packed: torch.Tensor, out_channels: int, stride: int = 1,
            bias=None, residual=None, res_up2=None, mask_src=None, relu=False, out=None,
            in_affine=None, in_relu=True, group_size=None, stats=False, n_stat=None):
    """y = epi(conv1x1_stride(xf(x))) (dd_conv1x1_forward; packed = conv1x1_pack(W) or
    conv1x1_pack(W, transpose=True) for the backward-data GEMM).  stats=True also returns the
    grouped BN partial statistics (BNStats) of y."""
    _dev(x, torch.float32, "x", 4)
    B, cin, h, w = x.shape
    ho, wo = h // stride, w // stride
    shape = (B, out_channels, ho, wo)
    if out is None:
        out = torch.empty(shape, dtype=torch.float32, device=x.device)
    for name, t in (("residual", residual), ("mask_src", mask_src), ("out", out)):
        if t is not None and tuple(t.shape) != shape:
            raise ValueError(f"{name} must be {shape}")
    if res_up2 is not None and tuple(res_up2.shape) != (B, out_channels, ho // 2, wo // 2):
        raise ValueError("res_up2 must be [B, cout, ho/2, wo/2]")
    grouped = in_affine is not None or stats
    gs = int(group_size) if group_size is not None else 0
    if grouped and gs <= 0:
        raise ValueError("group_size is required with in_affine / stats")
    G = -(-B // gs) if grouped else 1
    sc = sh = None
    if in_affine is not None:
        sc, sh = in_affine
        for name, t in (("in_scale", sc), ("in_shift", sh)):
            _dev(t, torch.float32, name)
            if t.numel() != G * cin:
                raise ValueError(f"{name} must have G*cin = {G * cin} entries")
    st = None
    nst = B if n_stat is None else min(max(int(n_stat), 0), B)
    if stats:
        tiles = int(lib().dd_conv1x1_tiles_per_group(ho, wo, gs))
        if tiles < 0:
            raise DDError(f"no 1x1 stats layout for {ho}x{wo} with group_size {gs}")
        # position-granular partials (one per 64 consecutive positions of the group)
        st = BNStats(_stats_buffer(None, G, out_channels, tiles, x.device), G, gs, nst, tiles,
                     -64, 1, out_channels, ho * wo)
    e0 = _t0(x)
    rc = lib().dd_conv1x1_forward(_dev(x, torch.float32, "x"), B, cin, h, w, int(stride),
                                  ctypes.c_void_p(packed.data_ptr()), out_channels,
                                  _opt(bias, torch.float32, "bias", out_channels),
                                  _opt(residual, torch.float32, "residual"),
                                  _opt(res_up2, torch.float32, "res_up2"),
                                  _opt(mask_src, torch.float32, "mask_src"), int(bool(relu)),
                                  _opt(sc, torch.float32, "in_scale"),
                                  _opt(sh, torch.float32, "in_shift"), int(bool(in_relu)), gs,
                                  nst, ctypes.c_void_p(st.buf.data_ptr()) if st else None,
                                  _dev(out, torch.float32, "out"), pack_operands(packed),
                                  pack_acc_scale(packed), _stream(x))
    _check(rc, "dd_conv1x1_forward")
    _t1(e0, "conv1x1", 2.0 * B * ho * wo * cin * out_channels, x,
        tag="stats" if stats else "mask" if mask_src is not None else "plain",
        nbytes=_conv_bytes(B, cin, h, w, out_channels, ho, wo, stride, 1,
                           (residual is not None) + (mask_src is not None)))
    return (out, st) if stats else out


def conv1x1_unit_input(y_prev: torch.Tensor, affine, packed: torch.Tensor, out_channels: int,
                       group_size: int, residual=None, res_affine=None, n_stat=None):
    """The previous ResNet-50 unit's output relu(bn(y_prev) [+ bn_r(residual) | + residual])
    computed while the next unit's first 1x1 conv stages it (dd_conv1x1_forward_unit_input):
    returns (that unit output, written once; y = conv1x1(unit output); the grouped BN partial
    statistics of y) -- bitwise bn_apply(...) followed by conv1x1(..., stats=True)."""
    _dev(y_prev, torch.float32, "y_prev", 4)
    B, cin, h, w = y_prev.shape
    gs = int(group_size)
    if gs <= 0:
        raise ValueError("group_size must be positive")
    G = -(-B // gs)
    sc, sh = affine
    rs = rt = None
    if res_affine is not None:
        if residual is None:
            raise ValueError("res_affine needs residual")
        rs, rt = res_affine
    for name, t in (("scale", sc), ("shift", sh), ("res_scale", rs), ("res_shift", rt)):
        if t is not None:
            _dev(t, torch.float32, name)
            if t.numel() != G * cin:
                raise ValueError(f"{name} must have G*cin = {G * cin} entries")
    if residual is not None and tuple(residual.shape) != tuple(y_prev.shape):
        raise ValueError("residual must have y_prev's shape")
    xout = torch.empty_like(y_prev)
    out = torch.empty((B, out_channels, h, w), dtype=torch.float32, device=y_prev.device)
    tiles = int(lib().dd_conv1x1_tiles_per_group(h, w, gs))
    if tiles < 0:
        raise DDError(f"no 1x1 stats layout for {h}x{w} with group_size {gs}")
    nst = B if n_stat is None else min(max(int(n_stat), 0), B)
    st = BNStats(_stats_buffer(None, G, out_channels, tiles, y_prev.device), G, gs, nst, tiles,
                 -64, 1, out_channels, h * w)
    e0 = _t0(y_prev)
    rc = lib().dd_conv1x1_forward_unit_input(
        _dev(y_prev, torch.float32, "y_prev"), _dev(sc, torch.float32, "scale"),
        _dev(sh, torch.float32, "shift"), _opt(residual, torch.float32, "residual"),
        _opt(rs, torch.float32, "res_scale"), _opt(rt, torch.float32, "res_shift"),
        _dev(xout, torch.float32, "xout"), B, cin, h, w, ctypes.c_void_p(packed.data_ptr()),
        out_channels, gs, nst, ctypes.c_void_p(st.buf.data_ptr()), _dev(out, torch.float32, "y"),
        pack_operands(packed), pack_acc_scale(packed), _stream(y_prev))
    _check(rc, "dd_conv1x1_forward_unit_input")
    _t1(e0, "conv1x1_unit", 2.0 * B * h * w * cin * out_channels, y_prev, tag="stats",
        nbytes=_conv_bytes(B, cin, h, w, out_channels, h, w, 1, 1)
        + 4.0 * B * cin * h * w * (1 + (residual is not None)))
    return xout, out, st


# ---- downsampling head: stride-2 3x3 conv + fused 1x1 stride-2 shortcut --------------------
def conv1x1_pack(weight: torch.Tensor, transpose: bool = False,
                 operands: str = "bf16x3") -> torch.Tensor:
    """Pack fp32 1x1 weights [cout, cin(, 1, 1)] for dd_conv1x1_forward / dd_down_forward
    (transpose: W^T; operands as conv3x3_pack)."""
    code = _operands_code(operands)
    w = weight.reshape(weight.shape[0], weight.shape[1]).contiguous()
    _dev(w, torch.float32, "weight", 2)
    cout, cin = w.shape
    oc, ic = (cin, cout) if transpose else (cout, cin)
    packed = torch.empty(lib().dd_conv1x1_pack_bytes(oc, ic), dtype=torch.uint8, device=w.device)
    scale = _pack_scale(w, code)
    rc = lib().dd_conv1x1_pack(_dev(w, torch.float32, "weight"), cout, cin, int(bool(transpose)),
                               code, scale, ctypes.c_void_p(packed.data_ptr()), _stream(w))
    _check(rc, "dd_conv1x1_pack")
    return _tag_pack(packed, code, scale)


# ---- CIFAR head of the GraNd pass --------------------------------------------------------------
def head_pool(a: torch.Tensor, out=None) -> torch.Tensor:
    """feat [B, C] = spatial mean of a [B, C, H, W] (avg_pool2d over the whole 4x4 map)."""
    _dev(a, torch.float32, "a", 4)
    B, C, h, w = a.shape
    if out is None:
        out = torch.empty((B, C), dtype=torch.float32, device=a.device)
    rc = lib().dd_head_pool(_dev(a, torch.float32, "a"), B, C, h * w,
                            _dev(out, torch.float32, "out"), _stream(a))
    _check(rc, "dd_head_pool")
    return out


def head_backward(a: torch.Tensor, e: torch.Tensor, weight: torch.Tensor, out=None) -> torch.Tensor:
    """d [B, C, H, W] = (e @ weight / (H W)) broadcast * (a > 0): the gradient reaching the
    last block's pre-ReLU output through avg-pool + linear."""
    _dev(a, torch.float32, "a", 4)
    B, C, h, w = a.shape
    ncls = weight.shape[0]
    if tuple(weight.shape) != (ncls, C) or tuple(e.shape) != (B, ncls):
        raise ValueError("weight must be [ncls, C] and e [B, ncls]")
    if out is None:
        out = torch.empty_like(a)
    rc = lib().dd_head_backward(_dev(a, torch.float32, "a"), _dev(e, torch.float32, "e"),
                                _dev(weight, torch.float32, "weight"), B, C, h * w, ncls,
                                1.0 / (h * w), _dev(out, torch.float32, "out"), _stream(a))
    _check(rc, "dd_head_backward")
    return out


# ---- any kh x kw convolution as an implicit GEMM (same kernel) -------------------------------
def stem7_supported(h: int, w: int, cin: int, cout: int, group_size: int) -> bool:
    """The ImageNet 7x7 / stride 2 / pad 3 stem's EL2N launch runs on dd_stem7_forward."""
    return lib().dd_stem7_supported(int(h), int(w), int(cin), int(cout), int(group_size)) == 1


def stem7_pack(weight: torch.Tensor, operands: str = "bf16x3") -> torch.Tensor:
    """Pack fp32 weights [cout <= 64, 3, 7, 7] for dd_stem7_forward."""
    code = _operands_code(operands)
    _dev(weight, torch.float32, "weight", 4)
    cout, cin, kh, kw = weight.shape
    if (cin, kh, kw) != (3, 7, 7):
        raise ValueError("3 x 7 x 7 weights only")
    packed = torch.empty(lib().dd_stem7_pack_bytes(), dtype=torch.uint8, device=weight.device)
    scale = _pack_scale(weight, code)
    rc = lib().dd_stem7_pack(_dev(weight, torch.float32, "weight"), cout, code, scale,
                             ctypes.c_void_p(packed.data_ptr()), _stream(weight))
    _check(rc, "dd_stem7_pack")
    return _tag_pack(packed, code, scale)


def stem7(x: torch.Tensor, packed: torch.Tensor, out_channels: int, group_size: int,
          n_stat=None):
    """(y, BNStats): the 7x7 / stride 2 / pad 3 stem conv of x [B, 3, h, w] with grouped BN
    partial statistics (dd_stem7_forward; packed = stem7_pack(W))."""
    _dev(x, torch.float32, "x", 4)
    B, cin, h, w = x.shape
    gs = int(group_size)
    if not stem7_supported(h, w, cin, out_channels, gs):
        raise DDError(f"no stem7 geometry for {cin} -> {out_channels} at {h}x{w}")
    G = -(-B // gs)
    tiles = int(lib().dd_stem7_tiles_per_group(h, w, gs))
    ho, wo = h // 2, w // 2
    y = torch.empty((B, out_channels, ho, wo), dtype=torch.float32, device=x.device)
    nst = B if n_stat is None else min(max(int(n_stat), 0), B)
    st = BNStats(_stats_buffer(None, G, out_channels, tiles, x.device), G, gs, nst, tiles, 1,
                 tiles // gs, out_channels, ho * wo)
    e0 = _t0(x)
    rc = lib().dd_stem7_forward(_dev(x, torch.float32, "x"), B, h, w,
                                ctypes.c_void_p(packed.data_ptr()), out_channels, gs, nst,
                                ctypes.c_void_p(st.buf.data_ptr()), _dev(y, torch.float32, "y"),
                                pack_operands(packed), pack_acc_scale(packed), _stream(x))
    _check(rc, "dd_stem7_forward")
    _t1(e0, "stem7", 2.0 * B * ho * wo * 147 * out_channels, x,
        nbytes=4.0 * (B * 3 * h * w + B * out_channels * ho * wo))
    return y, st


def conv_gemm_pack(weight: torch.Tensor, operands: str = "bf16x3") -> torch.Tensor:
    """Pack fp32 weights [cout, cin, kh, kw] for dd_conv_gemm_forward (operands as
    conv3x3_pack)."""
    code = _operands_code(operands)
    _dev(weight, torch.float32, "weight", 4)
    cout, cin, kh, kw = weight.shape
    packed = torch.empty(lib().dd_conv_gemm_pack_bytes(cout, cin, kh, kw), dtype=torch.uint8,
                         device=weight.device)
    scale = _pack_scale(weight, code)
    rc = lib().dd_conv_gemm_pack(_dev(weight, torch.float32, "weight"), cout, cin, kh, kw,
                                 code, scale, ctypes.c_void_p(packed.data_ptr()),
                                 _stream(weight))
    _check(rc, "dd_conv_gemm_pack")
    return _tag_pack(packed, code, scale)


def conv_gemm(x: torch.Tensor, packed: torch.Tensor, out_channels: int, kernel_size, stride=1,
              padding=0, bias=None, residual=None, relu=False, out=None, in_affine=None,
              in_relu=True, group_size=None, stats=False, n_stat=None):
    """y = epi(conv_{kh x kw, stride, pad}(xf(x))) (dd_conv_gemm_forward, packed =
    conv_gemm_pack(W)); stats=True also returns the grouped BN partial statistics of y."""
    _dev(x, torch.float32, "x", 4)
    kh, kw = (kernel_size, kernel_size) if isinstance(kernel_size, int) else kernel_size
    B, cin, h, w = x.shape
    ho = (h + 2 * padding - kh) // stride + 1
    wo = (w + 2 * padding - kw) // stride + 1
    shape = (B, out_channels, ho, wo)
    if out is None:
        out = torch.empty(shape, dtype=torch.float32, device=x.device)
    for name, t in (("residual", residual), ("out", out)):
        if t is not None and tuple(t.shape) != shape:
            raise ValueError(f"{name} must be {shape}")
    grouped = in_affine is not None or stats
    gs = int(group_size) if group_size is not None else 0
    if grouped and gs <= 0:
        raise ValueError("group_size is required with in_affine / stats")
    G = -(-B // gs) if grouped else 1
    sc = sh = None
    if in_affine is not None:
        sc, sh = in_affine
        for name, t in (("in_scale", sc), ("in_shift", sh)):
            _dev(t, torch.float32, name)
            if t.numel() != G * cin:
                raise ValueError(f"{name} must have G*cin = {G * cin} entries")
    st = None
    nst = B if n_stat is None else min(max(int(n_stat), 0), B)
    if stats:
        tiles = int(lib().dd_conv1x1_tiles_per_group(ho, wo, gs))
        if tiles < 0:
            raise DDError(f"no GEMM-conv stats layout for {ho}x{wo} with group_size {gs}")
        st = BNStats(_stats_buffer(None, G, out_channels, tiles, x.device), G, gs, nst, tiles,
                     -64, 1, out_channels, ho * wo)
    e0 = _t0(x)
    rc = lib().dd_conv_gemm_forward(_dev(x, torch.float32, "x"), B, cin, h, w, kh, kw,
                                    int(stride), int(padding), ctypes.c_void_p(packed.data_ptr()),
                                    out_channels, _opt(bias, torch.float32, "bias", out_channels),
                                    _opt(residual, torch.float32, "residual"), int(bool(relu)),
                                    _opt(sc, torch.float32, "in_scale"),
                                    _opt(sh, torch.float32, "in_shift"), int(bool(in_relu)), gs,
                                    nst, ctypes.c_void_p(st.buf.data_ptr()) if st else None,
                                    _dev(out, torch.float32, "out"), pack_operands(packed),
                                    pack_acc_scale(packed), _stream(x))
    _check(rc, "dd_conv_gemm_forward")
    _t1(e0, "conv_gemm", 2.0 * B * ho * wo * cin * kh * kw * out_channels, x,
        tag=f"{kh}x{kw}s{stride}",
        nbytes=_conv_bytes(B, cin, h, w, out_channels, ho, wo, stride, kh,
                           residual is not None))
    return (out, st) if stats else out


def down_supported(h_out: int, w_out: int) -> bool:
    return ((w_out == 32 and h_out % 2 == 0) or (w_out == 16 and h_out % 4 == 0)
            or (h_out, w_out) in ((8, 8), (4, 4)))


def down_padded_supported(h_out: int, w_out: int, cin: int, cout: int, group_size: int) -> bool:
    """A stride-2 statistics launch without a shortcut runs on the padded-width heads at this
    output shape (dd_down_forward, ABI 10: the ImageNet-stem network's 28 / 14 / 7 outputs)."""
    return lib().dd_down_padded_supported(int(h_out), int(w_out), int(cin), int(cout),
                                          int(group_size)) == 1


def down_backward_mask_bits_supported(h_out: int, w_out: int) -> bool:
    """Whether dd_down_backward takes `mask_bits` at this output shape: only its 128-position
    kernel reads them (16-wide maps with h_out % 8 == 0, 8x8, 4x4); other shapes need mask_src
    (the library refuses mask_bits there rather than run without the ReLU mask)."""
    return (w_out == 16 and h_out % 8 == 0) or (h_out, w_out) in ((8, 8), (4, 4))


def _head_operands(packed3x3, packed1x1):
    """(operands code, accumulator scale of the 3x3 pack, of the 1x1 pack) of a head."""
    code = pack_operands(packed3x3)
    if packed1x1 is not None and pack_operands(packed1x1) != code:
        raise ValueError("the 3x3 and 1x1 packs of a head must have the same operands")
    return (code, pack_acc_scale(packed3x3),
            pack_acc_scale(packed1x1) if packed1x1 is not None else 1.0)


def conv_down(x: torch.Tensor, packed3x3: torch.Tensor, out_channels: int, packed1x1=None,
              bias=None, relu=False, bias_sc=None, relu_sc=False, group_size=None,
              stats=False, n_stat=None):
    """(y, y_sc or None, BNStats or None, BNStats or None): stride-2 3x3 conv and the fused
    1x1 stride-2 shortcut of a downsampling block (see include/dd_capi.h)."""
    _dev(x, torch.float32, "x", 4)
    B, cin, hi, wi = x.shape
    if hi % 2 or wi % 2:
        raise ValueError("input height and width must be even")
    ho, wo = hi // 2, wi // 2
    shape = (B, out_channels, ho, wo)
    y = torch.empty(shape, dtype=torch.float32, device=x.device)
    ys = torch.empty(shape, dtype=torch.float32, device=x.device) if packed1x1 is not None else None
    gs = int(group_size) if group_size is not None else 0
    if stats and gs <= 0:
        raise ValueError("group_size is required with stats")
    st = sts = None
    nst = B if n_stat is None else min(max(int(n_stat), 0), B)
    if stats:
        G = -(-B // gs)
        tiles = int(lib().dd_down_tiles_per_group(ho, wo, gs))
        if tiles < 0:
            raise DDError(f"no downsample tile geometry for {ho}x{wo} with group_size {gs}")
        ipt = 4 if (ho, wo) == (4, 4) else 1
        mk = lambda: BNStats(_stats_buffer(None, G, out_channels, tiles, x.device), G, gs, nst,  # noqa: E731
                             tiles, ipt, tiles // (gs // ipt), out_channels, ho * wo)
        st = mk()
        sts = mk() if ys is not None else None
    ptr = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
    e0 = _t0(x)
    rc = lib().dd_down_forward(_dev(x, torch.float32, "x"), B, cin, ho, wo, ptr(packed3x3),
                               ptr(packed1x1), out_channels,
                               _opt(bias, torch.float32, "bias", out_channels), int(bool(relu)),
                               ptr(st.buf) if st else None, ptr(y),
                               _opt(bias_sc, torch.float32, "bias_sc", out_channels),
                               int(bool(relu_sc)), ptr(sts.buf) if sts else None, ptr(ys),
                               gs, nst, *_head_operands(packed3x3, packed1x1), _stream(x))
    _check(rc, "dd_down_forward")
    # algorithmic bytes: x read once, y (and the shortcut output) written once
    _t1(e0, "down_fwd", 2.0 * B * ho * wo * cin * out_channels * (9 + (ys is not None)), x,
        nbytes=4.0 * (B * cin * hi * wi + B * out_channels * ho * wo * (1 + (ys is not None))))
    return y, ys, st, sts


def conv_down_unit_input(y_prev: torch.Tensor, affine, packed3x3: torch.Tensor,
                         out_channels: int, group_size: int, packed1x1=None, residual=None,
                         n_stat=None):
    """conv_down of x = relu(y_prev * scale + shift (+ residual)) with x computed while the
    head stages it (dd_down_forward_unit_input; EL2N statistics epilogue): returns
    (y, y_sc or None, BNStats, BNStats or None), bitwise conv_down(bn_apply(...))."""
    _dev(y_prev, torch.float32, "y_prev", 4)
    B, cin, hi, wi = y_prev.shape
    if hi % 2 or wi % 2:
        raise ValueError("input height and width must be even")
    if (residual is None) != (packed1x1 is None):
        raise ValueError("the unit form (residual) goes with the fused shortcut (packed1x1)")
    gs = int(group_size)
    G = -(-B // gs)
    scale, shift = affine
    for name, t in (("scale", scale), ("shift", shift)):
        _dev(t, torch.float32, name)
        if t.numel() != G * cin:
            raise ValueError(f"{name} must have G*cin = {G * cin} entries")
    if residual is not None:
        _dev(residual, torch.float32, "residual")
        if residual.shape != y_prev.shape:
            raise ValueError("residual must match y_prev")
    ho, wo = hi // 2, wi // 2
    shape = (B, out_channels, ho, wo)
    y = torch.empty(shape, dtype=torch.float32, device=y_prev.device)
    ys = torch.empty(shape, dtype=torch.float32, device=y_prev.device) \
        if packed1x1 is not None else None
    nst = B if n_stat is None else min(max(int(n_stat), 0), B)
    tiles = int(lib().dd_down_tiles_per_group(ho, wo, gs))
    if tiles < 0:
        raise DDError(f"no downsample tile geometry for {ho}x{wo} with group_size {gs}")
    ipt = 4 if (ho, wo) == (4, 4) else 1
    mk = lambda: BNStats(_stats_buffer(None, G, out_channels, tiles, y_prev.device), G, gs,  # noqa: E731
                         nst, tiles, ipt, tiles // (gs // ipt), out_channels, ho * wo)
    st = mk()
    sts = mk() if ys is not None else None
    ptr = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
    e0 = _t0(y_prev)
    rc = lib().dd_down_forward_unit_input(
        _dev(y_prev, torch.float32, "y_prev"), ptr(scale), ptr(shift), ptr(residual), B, cin,
        ho, wo, ptr(packed3x3), ptr(packed1x1), out_channels, ptr(st.buf), ptr(y),
        ptr(sts.buf) if sts else None, ptr(ys), gs, nst, *_head_operands(packed3x3, packed1x1),
        _stream(y_prev))
    _check(rc, "dd_down_forward_unit_input")
    _t1(e0, "down_fwd_unit", 2.0 * B * ho * wo * cin * out_channels * (9 + (ys is not None)),
        y_prev, nbytes=4.0 * (B * cin * hi * wi * (1 + (residual is not None))
                              + B * out_channels * ho * wo * (1 + (ys is not None))))
    return y, ys, st, sts


def conv3x3_mask_plane_bits(mask: torch.Tensor, B: int, cout: int, h: int, w: int,
                            out: torch.Tensor = None) -> torch.Tensor:
    """Plane bits (int32 [B * cout * h * w / 32], bit p & 31 of word ((b cout + o) h w + p) >> 5)
    of a conv3x3 launch's fragment-order ReLU mask (its mask_out)."""
    if (h * w) % 32:
        raise ValueError("h * w must be a multiple of 32")
    n = B * cout * h * w // 32
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=mask.device)
    rc = lib().dd_conv3x3_mask_plane_bits(ctypes.c_void_p(mask.data_ptr()), int(B), int(cout),
                                          int(h), int(w), ctypes.c_void_p(out.data_ptr()),
                                          _stream(mask))
    _check(rc, "dd_conv3x3_mask_plane_bits")
    return out


def down_backward(dh: torch.Tensor, packed3x3_t: torch.Tensor, in_channels: int, dz=None,
                  packed1x1_t=None, mask_src=None, mask_bits=None) -> torch.Tensor:
    """dx = (conv3x3_s2^T(dh) + conv1x1_s2^T(dz)) * mask for a downsampling head (packs from
    conv3x3_pack(W, transpose_flip=True) / conv1x1_pack(Ws, transpose=True)); the mask is
    (mask_src > 0) or the plane bits `mask_bits` (conv3x3_mask_plane_bits)."""
    _dev(dh, torch.float32, "dh", 4)
    B, cout, ho, wo = dh.shape
    shape = (B, in_channels, 2 * ho, 2 * wo)
    if dz is not None:
        _dev(dz, torch.float32, "dz", 4)
        if dz.shape != dh.shape:
            raise ValueError("dz must match dh")
    if mask_src is not None:
        _dev(mask_src, torch.float32, "mask_src", 4)
        if tuple(mask_src.shape) != shape:
            raise ValueError(f"mask_src must be {shape}")
    if mask_bits is not None:
        if mask_src is not None:
            raise ValueError("mask_src and mask_bits are exclusive")
        if mask_bits.dtype != torch.int32 or mask_bits.numel() * 32 != math.prod(shape):
            raise ValueError(f"mask_bits must be int32 [{math.prod(shape) // 32}]")
    dx = torch.empty(shape, dtype=torch.float32, device=dh.device)
    ptr = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
    e0 = _t0(dh)
    rc = lib().dd_down_backward(_dev(dh, torch.float32, "dh"), ptr(dz), B, cout, ho, wo,
                                ptr(packed3x3_t), ptr(packed1x1_t), int(in_channels),
                                ptr(mask_src), ptr(mask_bits), ptr(dx), _stream(dh))
    _check(rc, "dd_down_backward")
    # algorithmic bytes: dh (and dz) read once, the mask read once (4 B or 1 bit per
    # element), dx written once
    nx = B * in_channels * 4 * ho * wo
    mb = 4.0 * nx if mask_src is not None else (nx / 8.0 if mask_bits is not None else 0.0)
    _t1(e0, "down_bwd", 2.0 * B * ho * wo * in_channels * cout * (9 + (dz is not None)), dh,
        nbytes=4.0 * (B * cout * ho * wo * (1 + (dz is not None)) + nx) + mb)
    return dx
