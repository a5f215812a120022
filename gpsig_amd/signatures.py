"""Signature features on MI355X: the iisignature-backed pieces of the VOSF inducing-feature path.

Reference: gpsig/iisignature_tensorflow.py:87 (``Sig``: iisignature.sig as a TF py_func with
iisignature.sigbackprop as gradient), gpsig/utils.py:102-134 (``compute_trunc``, ``get_powers``) and
the VOSF features built on them (gpsig_amd/inducing_variables_vosf.py).  ``Sig`` runs the
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
