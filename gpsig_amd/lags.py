"""Fractional lags by linear interpolation in time, on device (torch).

Restates gpsig/lags.py:7-63 (lin_interp / add_lags_to_sequences) with torch ops so the
pre-processing of SignatureKernel._apply_scaling_and_lags_to_sequences (gpsig/kernels.py:344-365)
runs on the GPU next to the HIP kernels.  Semantics kept: time grid t_k = k/(L-1), query
max(t - lag, 0), left index = argmax over {t <= query + jitter} of (t - query) (first maximum, as
tf.argmax), right index = left + 1.
"""
from __future__ import annotations

import torch


def lin_interp(time: torch.Tensor, X: torch.Tensor, time_query: torch.Tensor, jitter: float) -> torch.Tensor:
    """lags.py:7-38.  time (L,), X (N,L,D), time_query (L,nl) -> (N,L,nl,D)."""
    pairwise = time[:, None, None] - time_query[None, :, :]
    masked = torch.where(pairwise > jitter, torch.full_like(pairwise, -float("inf")), pairwise)
    left = torch.argmax(masked, dim=0)            # (L, nl)
    right = left + 1
    Xl = X[:, left, :]                            # (N, L, nl, D)
    Xr = X[:, right, :]
    tl = time[left]
    tr = time[right]
    w = (time_query - tl) / (tr - tl)
    return Xl + w[None, :, :, None] * (Xr - Xl)


def add_lags_to_sequences(X: torch.Tensor, lags: torch.Tensor, jitter: float) -> torch.Tensor:
    """lags.py:41-63.  X (N,L,D), lags (nl,) -> (N,L,nl+1,D)."""
    L = X.shape[1]
    time = torch.arange(L, dtype=X.dtype, device=X.device) / float(L - 1)
    time_lags = torch.clamp(time[:, None] - lags.to(X.dtype)[None, :], min=0.0)
    Xq = lin_interp(time, X, time_lags, jitter)
    return torch.cat((X[:, :, None, :], Xq), dim=2)
