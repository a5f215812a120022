"""Inducing tensors / inducing sequences on MI355X: drop-in for gpsig.inducing_variables.

Reference gpsig/inducing_variables.py.  The reference registers Kuu / Kuf / Kuu_Kuf_Kff for its
feature classes with GPflow's multiple dispatch; GPflow is not part of this build, so the same
computations are methods of the feature classes and module functions with the reference's names,
on torch tensors (differentiable: Z, the optional per-level weights W, and the kernel's lengthscales
and variances get gradients through the gfx950 VJP kernels).  The reference's full_f_cov branches
add jitter to `tf.eye(tf.shape(X)[0])` with X undefined (NameError, :64, :134); here X_new's size.
"""
from __future__ import annotations

import numpy as np
import torch

from .kernels import SignatureKernel, _as_tensor


class SignatureInducing:
    """inducing_variables.py:14-27: Z and, with learn_weights, per-level mixing matrices W
    (num_levels, M, M) initialised to identities."""

    def __init__(self, Z, num_levels, learn_weights=False):
        self.Z = _as_tensor(Z)
        self.num_levels = num_levels
        self.learn_weights = learn_weights
        if learn_weights:
            eye = torch.eye(len(self), dtype=torch.float64, device=self.Z.device)
            self.W = eye[None].repeat(num_levels, 1, 1)

    def __len__(self):
        return self.Z.shape[0]

    def _mix_sym(self, K):
        """Kzz[0] + sum_m W_m Kzz[m] W_m^T (inducing_variables.py:57, :84, :106)."""
        W = self.W.to(K.device, K.dtype)
        return K[0] + torch.sum(W @ K[1:] @ W.transpose(1, 2), dim=0)

    def _mix_cross(self, K):
        """Kzx[0] + sum_m W_m Kzx[m] (inducing_variables.py:58, :74, :117)."""
        W = self.W.to(K.device, K.dtype)
        return K[0] + torch.sum(W @ K[1:], dim=0)


class InducingTensors(SignatureInducing):
    """inducing_variables.py:29-49: Z (LT, T, D) or (LT, T, 2, D) with increments."""

    def __init__(self, Z, num_levels, increments=False, **kwargs):
        len_tensors = int(num_levels * (num_levels + 1) / 2)
        Zt = _as_tensor(Z)
        assert Zt.shape[0] == len_tensors
        if increments:
            assert Zt.ndim == 4
            assert Zt.shape[2] == 2
        self.len_tensors = len_tensors
        self.increments = increments
        super().__init__(Zt, num_levels, **kwargs)

    def __len__(self):
        return self.Z.shape[1]

    def Kuu_Kuf_Kff(self, kern: SignatureKernel, X_new, *, jitter=0.0, full_f_cov=False):
        """inducing_variables.py:51-67."""
        if self.learn_weights:
            Kzz, Kzx, Kxx = kern.K_tens_n_seq_covs(self.Z, X_new, full_X_cov=full_f_cov, return_levels=True,
                                                   increments=self.increments)
            Kzz, Kzx, Kxx = self._mix_sym(Kzz), self._mix_cross(Kzx), Kxx.sum(0)
        else:
            Kzz, Kzx, Kxx = kern.K_tens_n_seq_covs(self.Z, X_new, full_X_cov=full_f_cov, increments=self.increments)
        Kzz = Kzz + jitter * torch.eye(len(self), dtype=Kzz.dtype, device=Kzz.device)
        if full_f_cov:
            Kxx = Kxx + jitter * torch.eye(Kxx.shape[0], dtype=Kxx.dtype, device=Kxx.device)
        else:
            Kxx = Kxx + jitter
        return Kzz, Kzx, Kxx

    def Kuf(self, kern: SignatureKernel, X_new):
        """inducing_variables.py:69-77."""
        if self.learn_weights:
            return self._mix_cross(kern.K_tens_vs_seq(self.Z, X_new, return_levels=True, increments=self.increments))
        return kern.K_tens_vs_seq(self.Z, X_new, increments=self.increments)

    def Kuu(self, kern: SignatureKernel, *, jitter=0.0, full_f_cov=False):
        """inducing_variables.py:79-88."""
        if self.learn_weights:
            Kzz = self._mix_sym(kern.K_tens(self.Z, return_levels=True, increments=self.increments))
        else:
            Kzz = kern.K_tens(self.Z, increments=self.increments)
        return Kzz + jitter * torch.eye(len(self), dtype=Kzz.dtype, device=Kzz.device)


class InducingSequences(SignatureInducing):
    """inducing_variables.py:90-99: Z (num_inducing, len_inducing, num_features), presliced."""

    def __init__(self, Z, num_levels, **kwargs):
        super().__init__(Z, num_levels, **kwargs)
        self.len_inducing = self.Z.shape[1]

    def _Zflat(self):
        return self.Z.reshape(self.Z.shape[0], -1)

    def Kuu(self, kern: SignatureKernel, *, jitter=0.0):
        """inducing_variables.py:102-111."""
        if self.learn_weights:
            Kzz = self._mix_sym(kern.K(self._Zflat(), return_levels=True, presliced=True))
        else:
            Kzz = kern.K(self._Zflat(), presliced=True)
        return Kzz + jitter * torch.eye(len(self), dtype=Kzz.dtype, device=Kzz.device)

    def Kuf(self, kern: SignatureKernel, X_new):
        """inducing_variables.py:113-121."""
        if self.learn_weights:
            return self._mix_cross(kern.K(self._Zflat(), X_new, presliced_X=True, return_levels=True))
        return kern.K(self._Zflat(), X_new, presliced_X=True)

    def Kuu_Kuf_Kff(self, kern: SignatureKernel, X_new, *, jitter=0.0, full_f_cov=False):
        """inducing_variables.py:123-137."""
        if self.learn_weights:
            Kzz, Kzx, Kxx = kern.K_seq_n_seq_covs(self._Zflat(), X_new, full_X2_cov=full_f_cov, return_levels=True)
            Kzz, Kzx, Kxx = self._mix_sym(Kzz), self._mix_cross(Kzx), Kxx.sum(0)
        else:
            Kzz, Kzx, Kxx = kern.K_seq_n_seq_covs(self._Zflat(), X_new, full_X2_cov=full_f_cov)
        Kzz = Kzz + jitter * torch.eye(len(self), dtype=Kzz.dtype, device=Kzz.device)
        if full_f_cov:
            Kxx = Kxx + jitter * torch.eye(Kxx.shape[0], dtype=Kxx.dtype, device=Kxx.device)
        else:
            Kxx = Kxx + jitter
        return Kzz, Kzx, Kxx


def Kuu(feat, kern, **kw):
    return feat.Kuu(kern, **kw)


def Kuf(feat, kern, X_new):
    return feat.Kuf(kern, X_new)


def Kuu_Kuf_Kff(feat, kern, X_new, *, jitter=0.0, full_f_cov=False):
    return feat.Kuu_Kuf_Kff(kern, X_new, jitter=jitter, full_f_cov=full_f_cov)
