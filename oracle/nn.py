"""numpy fp32 restatement of the torch ops the reference path uses (CPU oracle).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg as the checker. Never part of the product path.

All tensors are NCHW / [N, L, C] float32 numpy arrays, as in the reference modules.
"""
from __future__ import annotations

import numpy as np
from numpy.lib.stride_tricks import sliding_window_view
from scipy.special import erf

f32 = np.float32


def conv2d(x, w, b=None, stride=1, pad=0):
    """torch.nn.functional.conv2d, zero padding. x [B,C,H,W], w [O,C,kh,kw]."""
    B, C, H, W = x.shape
    O, C2, kh, kw = w.shape
    assert C == C2
    if pad:
        x = np.pad(x, ((0, 0), (0, 0), (pad, pad), (pad, pad)))
    if kh == 1 and kw == 1 and stride == 1:
        cols = x.transpose(0, 2, 3, 1).reshape(-1, C)
        Ho, Wo = x.shape[2], x.shape[3]
    else:
        win = sliding_window_view(x, (kh, kw), axis=(2, 3))[:, :, ::stride, ::stride]
        Ho, Wo = win.shape[2], win.shape[3]
        cols = win.transpose(0, 2, 3, 1, 4, 5).reshape(B * Ho * Wo, C * kh * kw)
    y = cols @ w.reshape(O, -1).T
    if b is not None:
        y = y + b
    return np.ascontiguousarray(y.reshape(B, Ho, Wo, O).transpose(0, 3, 1, 2)).astype(f32)


def linear(x, w, b=None):
    y = x @ w.T
    return (y + b if b is not None else y).astype(f32)


def silu(x):
    return (x / (1 + np.exp(-x))).astype(f32)


def gelu(x):
    """nn.GELU() default (erf form)."""
    return (0.5 * x * (1 + erf(x / np.sqrt(f32(2))))).astype(f32)


def softmax(x, axis):
    m = x.max(axis=axis, keepdims=True)
    e = np.exp(x - m)
    return (e / e.sum(axis=axis, keepdims=True)).astype(f32)


def layer_norm(x, w, b, eps=1e-5):
    """nn.LayerNorm over the last dim (biased variance)."""
    mu = x.mean(-1, keepdims=True)
    var = ((x - mu) ** 2).mean(-1, keepdims=True)
    y = (x - mu) / np.sqrt(var + f32(eps))
    return (y * w + b).astype(f32)


def channel_layer_norm(x, g, eps=1e-5):
    """module_util.py:77-86 LayerNorm over dim 1 of NCHW, gain only; eps 1e-5 for fp32."""
    mu = x.mean(1, keepdims=True)
    var = ((x - mu) ** 2).mean(1, keepdims=True)
    return ((x - mu) / np.sqrt(var + f32(eps)) * g).astype(f32)


def group_norm(x, groups, w, b, eps=1e-6):
    B, C, H, W = x.shape
    xg = x.reshape(B, groups, -1)
    mu = xg.mean(-1, keepdims=True)
    var = ((xg - mu) ** 2).mean(-1, keepdims=True)
    y = ((xg - mu) / np.sqrt(var + f32(eps))).reshape(B, C, H, W)
    return (y * w[None, :, None, None] + b[None, :, None, None]).astype(f32)


def upsample_nearest2x(x):
    return x.repeat(2, axis=2).repeat(2, axis=3)


def reflect_pad(x, ph, pw):
    """F.pad(x, (0, pw, 0, ph), 'reflect') (DenoisingUNet_arch.py:111-116)."""
    if ph == 0 and pw == 0:
        return x
    return np.pad(x, ((0, 0), (0, 0), (0, ph), (0, pw)), mode="reflect")
