"""VOSF orthogonal inducing variables on MI355X: drop-in for gpsig.inducing_variables_vosf.

Reference gpsig/inducing_variables_vosf.py.  The reference registers Kuu / Kuf / Kuu_Kuf_Kff with
GPflow's multiple dispatch; GPflow is not part of this build, so the same three computations are
methods of the two feature classes (and module functions with the reference's names), on torch
tensors:

  * Kzz = I_M                                                     (:148-152, :271-275)
  * Kzx = [1, S(x)_{:M-1}]^T, the first M-1 signature coordinates of each path, computed by the
    gfx950 signature kernel (gpsig_amd.signatures.Sig, replacing iisignature) -- scaled by the ARD
    lengthscale powers or computed on the scaled paths (:96-146, :212-269)
  * Kxx = the PDE kernel's Kdiag (UntruncInducingOrthogonalTensors, :68-93) or the truncated
    kernel's Kdiag / K (TruncInducingOrthogonalTensors, :180-210), with the normalisation
    correction of Kzx through K_norms (:204-207).

Kzx and Kxx are differentiable (signature backprop, PDE adjoint, Gram VJP kernels).
"""
from __future__ import annotations

import numpy as np
import torch

from .kernels import SignatureKernel, _as_tensor
from .kernels_pde import UntruncSignatureKernel
from .signatures import Sig, compute_trunc, get_powers


class SignatureOrthogonalInducing:
    """Base class (inducing_variables_vosf.py:31-37)."""


class _VOSF(SignatureOrthogonalInducing):
    def __init__(self, input_dim, d, M, compute_sig=False, compute_and_diff_sig=False, num_lags=0, **kwargs):
        self.input_dim = input_dim
        self.d = d
        self.num_lags = num_lags
        self.M = M
        self.compute_sig = compute_sig
        self.compute_and_diff_sig = compute_and_diff_sig
        self.sig_level = compute_trunc(M, (num_lags + 1) * d)

    def __len__(self):
        return self.M

    def Kuu(self, kern, dtype=torch.float64, device="cuda"):
        return torch.eye(self.M, dtype=dtype, device=device)

    def _signatures(self, kern, X_new):
        """(N, M-1) signature coordinates (the compute_* branches of Kuf)."""
        X_new = _as_tensor(X_new)
        N = X_new.shape[0]
        if self.compute_and_diff_sig:
            X = kern._apply_scaling_and_lags_to_sequences(X_new.reshape(N, -1, self.d))
            return Sig(X, self.sig_level)[:, :self.M - 1]
        if self.compute_sig:
            S = Sig(X_new.reshape(N, -1, self.d), self.sig_level)[:, :self.M - 1]
        else:
            S = X_new  # the signatures are the input
        powers = torch.as_tensor(get_powers(self.d, self.sig_level)[:self.M - 1], dtype=S.dtype, device=S.device)
        ls = kern.lengthscales.to(S.device, S.dtype)
        return S / torch.prod(ls[None, :] ** powers, dim=1)[None, :]

    def _full(self, kern, X_new):
        S = self._signatures(kern, X_new)
        ones = torch.ones((S.shape[0], 1), dtype=S.dtype, device=S.device)
        return torch.cat([ones, S], 1).T  # (M, N)


class UntruncInducingOrthogonalTensors(_VOSF):
    """inducing_variables_vosf.py:40-152 (with the PDE signature kernel)."""

    def Kuf(self, kern: UntruncSignatureKernel, X_new):
        """:96-146."""
        Kzx = self._full(kern, X_new)
        return Kzx * torch.sqrt(torch.as_tensor(kern.sigma, dtype=Kzx.dtype, device=Kzx.device))

    def Kuu_Kuf_Kff(self, kern: UntruncSignatureKernel, X_new, *, jitter=0.0, full_f_cov=False, fast=False):
        """:68-93."""
        X_new = _as_tensor(X_new)
        Kzz = self.Kuu(kern, device=X_new.device)
        if fast:
            Kzx = None
        elif self.compute_sig or self.compute_and_diff_sig:
            Kzx = self.Kuf(kern, X_new)
        else:
            Kzx = self.Kuf(kern, X_new[:, self.input_dim:])
        if full_f_cov:
            raise ValueError('Not implemented')
        Kxx = kern.Kdiag(X_new[:, :self.input_dim]) + jitter
        return Kzz, Kzx, Kxx


class TruncInducingOrthogonalTensors(_VOSF):
    """inducing_variables_vosf.py:154-275 (with the truncated signature kernel)."""

    def _level_repeat(self, v, device, dtype):
        """(sig_level+1,) per-level values repeated d^i times, first M entries (:207, :266)."""
        reps = torch.as_tensor([self.d ** i for i in range(self.sig_level + 1)], device=device)
        return torch.repeat_interleave(v[:self.sig_level + 1].to(device, dtype), reps, dim=0)[:self.M]

    def Kuf(self, kern: SignatureKernel, X_new):
        """:212-269."""
        Kzx = self._full(kern, X_new)
        Kzx = Kzx * torch.sqrt(self._level_repeat(kern.variances, Kzx.device, Kzx.dtype))[:, None]
        return Kzx * torch.sqrt(torch.as_tensor(kern.sigma, dtype=Kzx.dtype, device=Kzx.device))

    def Kuu_Kuf_Kff(self, kern: SignatureKernel, X_new, *, jitter=0.0, full_f_cov=False, fast=False):
        """:180-210."""
        X_new = _as_tensor(X_new)
        Kzz = self.Kuu(kern, device=X_new.device)
        if fast:
            Kzx = None
        elif self.compute_sig or self.compute_and_diff_sig:
            Kzx = self.Kuf(kern, X_new)
        else:
            Kzx = self.Kuf(kern, X_new[:, self.input_dim:])
        Xin = X_new[:, :self.input_dim]
        if full_f_cov:
            Kxx = kern.K(Xin, return_levels=False)
            Kxx = Kxx + jitter * torch.eye(Kxx.shape[0], dtype=Kxx.dtype, device=Kxx.device)
        else:
            if kern.normalization:
                Kxx, Kxx_un = kern.K_norms(Xin)
                if Kzx is not None:
                    norm = torch.sqrt(self._level_repeat(Kxx_un, Kzx.device, Kzx.dtype) + kern.jitter)
                    Kzx = Kzx / norm
            else:
                Kxx = kern.Kdiag(Xin, return_levels=False)
            Kxx = Kxx + jitter
        return Kzz, Kzx, Kxx


def Kuu(feat, kern):
    return feat.Kuu(kern)


def Kuf(feat, kern, X_new):
    return feat.Kuf(kern, X_new)


def Kuu_Kuf_Kff(feat, kern, X_new, *, jitter=0.0, full_f_cov=False, fast=False):
    return feat.Kuu_Kuf_Kff(kern, X_new, jitter=jitter, full_f_cov=full_f_cov, fast=fast)
