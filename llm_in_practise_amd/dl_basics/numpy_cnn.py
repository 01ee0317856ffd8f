"""Convolution / pooling by hand plus LeNet-5 (``DL_Basics/CNN_and_RNN.ipynb``: "卷积操作 / 池化操作 /
单层卷积与多层连续卷积对比 / 展平层 / CNN正向传播和反向传播 / LeNet-5示例").

``conv2d_forward`` builds the strided window view of the padded input once
(``sliding_window_view``) and contracts it with the filters in one ``einsum``; the backward
reuses the same view for ``dW`` and scatters ``dX`` one kernel tap at a time (kh·kw strided adds
instead of a col2im buffer).  Semantics match ``torch.nn.functional.conv2d`` / ``max_pool2d``
(NCHW, cross-correlation, zero padding).
"""
from __future__ import annotations

import numpy as np
import torch
from torch import nn
from numpy.lib.stride_tricks import sliding_window_view


def _windows(xp: np.ndarray, kh: int, kw: int, stride: int) -> np.ndarray:
    v = sliding_window_view(xp, (kh, kw), axis=(2, 3))            # (N, C, H-kh+1, W-kw+1, kh, kw)
    return v[:, :, ::stride, ::stride]


def conv2d_forward(x, w, b=None, stride: int = 1, padding: int = 0):
    xp = np.pad(x, ((0, 0), (0, 0), (padding, padding), (padding, padding)))
    cols = _windows(xp, w.shape[2], w.shape[3], stride)
    out = np.einsum("nchwij,fcij->nfhw", cols, w, optimize=True)
    if b is not None:
        out = out + b[None, :, None, None]
    return out, (x.shape, xp.shape, cols, w, stride, padding)


def conv2d_backward(dout, cache):
    x_shape, xp_shape, cols, w, stride, padding = cache
    dw = np.einsum("nfhw,nchwij->fcij", dout, cols, optimize=True)
    db = dout.sum(axis=(0, 2, 3))
    dxp = np.zeros(xp_shape)
    Ho, Wo = dout.shape[2], dout.shape[3]
    for i in range(w.shape[2]):
        for j in range(w.shape[3]):
            dxp[:, :, i:i + stride * Ho:stride, j:j + stride * Wo:stride] += np.einsum("nfhw,fc->nchw", dout, w[:, :, i, j])
    H, W = x_shape[2], x_shape[3]
    return dxp[:, :, padding:padding + H, padding:padding + W], dw, db


def maxpool2d_forward(x, k: int = 2, stride: int | None = None):
    s = stride or k
    win = _windows(x, k, k, s)
    N, C, Ho, Wo = win.shape[:4]
    flat = win.reshape(N, C, Ho, Wo, k * k)
    idx = flat.argmax(axis=-1)                                     # first max, like torch
    return np.take_along_axis(flat, idx[..., None], -1)[..., 0], (x.shape, idx, k, s)


def maxpool2d_backward(dout, cache):
    x_shape, idx, k, s = cache
    dx = np.zeros(x_shape)
    Ho, Wo = dout.shape[2], dout.shape[3]
    for t in range(k * k):
        i, j = divmod(t, k)
        dx[:, :, i:i + s * Ho:s, j:j + s * Wo:s] += dout * (idx == t)
    return dx


class LeNet5(nn.Module):
    """LeNet-5 for 1×28×28 inputs: conv5(pad 2)→tanh→avgpool→conv5→tanh→avgpool→120→84→classes."""

    def __init__(self, num_classes: int = 10, act: type[nn.Module] = nn.Tanh):
        super().__init__()
        self.features = nn.Sequential(nn.Conv2d(1, 6, 5, padding=2), act(), nn.AvgPool2d(2),
                                      nn.Conv2d(6, 16, 5), act(), nn.AvgPool2d(2))
        self.classifier = nn.Sequential(nn.Flatten(), nn.Linear(16 * 5 * 5, 120), act(), nn.Linear(120, 84), act(),
                                        nn.Linear(84, num_classes))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.classifier(self.features(x))
