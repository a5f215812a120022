"""Signature features on MI355X: the iisignature-backed pieces of the VOSF inducing-feature path.

Reference: gpsig/iisignature_tensorflow.py:87 (``Sig``: iisignature.sig as a TF py_func with
iisignature.sigbackprop as gradient), gpsig/utils.py:102-134 (``compute_trunc``, ``get_powers``) and
the signature branch of the VOSF Kuf (gpsig/inducing_variables_vosf.py:96-146).  ``Sig`` runs the
gfx950 kernels gpsig_signature / gpsig_signature_vjp (gpsig_amd/csrc/sig_features.hip) on torch
tensors; the rest is O(M d) host arithmetic.
"""
from __future__ import annotations

import itertools

import numpy as np
import torch

from . import autograd as _ag


def Sig(x, m):
    """iisignature_tensorflow.Sig: x (N, L, d) -> (N, d + d^2 + ... + d^m), differentiable in x."""
    if not isinstance(x, torch.Tensor):
        x = torch.as_tensor(np.asarray(x), device="cuda")
    out = _ag.Signature.apply(x, int(m))
    return out.to(x.dtype) if x.is_floating_point() else out


def compute_trunc(M, d):
    """utils.py:102-108: the smallest truncation level whose signature has at least M - 1 coordinates
    beyond level 0 (d + d^2 + ... >= M - 1, counted as the reference does from d + 1)."""
    count, level = d + 1, 1
    while count < M:
        level += 1
        count += d ** level
    return level


def get_powers(d, sig_level):
    """utils.py:110-134: (num_features, d) multiplicities of each channel in the multi-index of every
    signature coordinate up to sig_level, in signature order (level-major, first index most significant)."""
    rows = []
    for level in range(1, sig_level + 1):
        for idx in itertools.product(range(d), repeat=level):
            rows.append(np.bincount(np.asarray(idx), minlength=d))
    return np.asarray(rows, dtype=np.float64)


def vosf_Kuf(kern, X_new, M, d, compute_and_diff_sig=False, precomputed=False):
    """The signature branch of Kuf for UntruncInducingOrthogonalTensors
    (inducing_variables_vosf.py:96-146): (M, N) with row 0 = sqrt(sigma) and rows 1.. the first M-1
    signature coordinates (lengthscale-scaled paths, or raw signatures divided by the ARD powers)."""
    sig_level = compute_trunc(M, d)
    if precomputed:
        S = torch.as_tensor(X_new)
    else:
        X = torch.as_tensor(X_new)
        N = X.shape[0]
        X = X.reshape(N, -1, d)
        if compute_and_diff_sig:
            X = kern._apply_scaling_and_lags_to_sequences(X)
        S = Sig(X, sig_level)[:, :M - 1]
    if not compute_and_diff_sig:
        powers = torch.as_tensor(get_powers(d, sig_level)[:M - 1], device=S.device, dtype=S.dtype)
        ls = kern.lengthscales.to(S.device, S.dtype)
        S = S / torch.prod(ls[None, :] ** powers, dim=1)[None, :]
    ones = torch.ones((S.shape[0], 1), device=S.device, dtype=S.dtype)
    full = torch.cat([ones, S], 1) * torch.sqrt(torch.as_tensor(kern.sigma, dtype=S.dtype, device=S.device))
    return full.T
