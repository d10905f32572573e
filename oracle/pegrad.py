"""ORACLE (test infrastructure): per-example weight-gradient squared norms in NumPy float64.

GraNd is not in the reference (it scores EL2N only, get_scores_and_prune.py:15-18); the
definition is the Data Diet paper's: ||grad_W CE(f(x_i), y_i)||_2 over the network weights.
For a Conv2d (no bias) the per-example weight gradient is G_i = sum_t u_t g_t^T with
u_t the im2col column at output position t and g_t the output gradient there; this module
computes ||G_i||_F^2 explicitly (direct) and via the ghost identity for cross-checking.
"""
from __future__ import annotations

import numpy as np


def im2col(act: np.ndarray, kh: int, kw: int, stride: int, pad: int) -> np.ndarray:
    """act [B, C, H, W] -> U [B, T, C*kh*kw] with m = (c, ky, kx) (PyTorch's unfold order)."""
    B, C, H, W = act.shape
    Ho = (H + 2 * pad - kh) // stride + 1
    Wo = (W + 2 * pad - kw) // stride + 1
    xp = np.zeros((B, C, H + 2 * pad, W + 2 * pad), dtype=np.float64)
    xp[:, :, pad:pad + H, pad:pad + W] = act
    cols = np.empty((B, C, kh, kw, Ho, Wo), dtype=np.float64)
    for ky in range(kh):
        for kx in range(kw):
            cols[:, :, ky, kx] = xp[:, :, ky:ky + stride * Ho:stride, kx:kx + stride * Wo:stride]
    return cols.reshape(B, C * kh * kw, Ho * Wo).transpose(0, 2, 1)


def conv_pegrad_sqnorm(act, gout, kh, kw, stride, pad, col_scale=None, method="direct"):
    """||U_i^T G_i||_F^2 per example (float64).  gout [B, Cout, Ho, Wo]."""
    U = im2col(np.asarray(act, np.float64), kh, kw, stride, pad)  # B,T,da
    B, Cout = gout.shape[:2]
    G = np.asarray(gout, np.float64).reshape(B, Cout, -1)  # B,dg,T
    if col_scale is not None:
        G = G * np.asarray(col_scale, np.float64)[None, :, None]
    if method == "direct":
        W = np.einsum("btm,bot->bmo", U, G)
        return (W * W).sum(axis=(1, 2))
    if method == "ghost":
        GA = np.einsum("btm,bsm->bts", U, U)
        GG = np.einsum("bot,bos->bts", G, G)
        return (GA * GG).sum(axis=(1, 2))
    raise ValueError(method)


def linear_pegrad_sqnorm(act, gout, has_bias=True):
    """||a g^T||^2 + ||g||^2 (bias) per example: the Linear layer (models/resnet.py:78)."""
    a2 = (np.asarray(act, np.float64) ** 2).sum(axis=1)
    g2 = (np.asarray(gout, np.float64) ** 2).sum(axis=1)
    return a2 * g2 + (g2 if has_bias else 0.0)


def bn_pegrad_sqnorm(out, g, gamma, beta):
    """||d loss / d(gamma, beta)||^2 per example of an eval-mode BatchNorm2d (float64), from its
    output out = gamma xhat + beta and the gradient g w.r.t. it:
    d/dgamma_c = sum_t g xhat, d/dbeta_c = sum_t g (grand_params: all)."""
    out = np.asarray(out, np.float64)
    g = np.asarray(g, np.float64)
    ga = np.asarray(gamma, np.float64)[None, :, None, None]
    be = np.asarray(beta, np.float64)[None, :, None, None]
    dgam = (g * (out - be) / ga).sum(axis=(2, 3))
    dbet = g.sum(axis=(2, 3))
    return (dgam ** 2).sum(axis=1) + (dbet ** 2).sum(axis=1)
