"""Truncated signature kernels on MI355X: drop-in for gpsig.kernels (reference gpsig/kernels.py).

Same constructor arguments, method names, argument meaning, return shapes and error behaviour as
the reference's GPflow kernels, on torch tensors (or NumPy arrays for the ``compute_*`` helpers,
which mirror the reference's autoflow functions and return NumPy).  Inputs are the reference's
flattened ``(N, L*D)`` sequences.  The level recursion and its normalisation epilogue run in the
gfx950 kernels of gpsig_amd/libgpsig_amd.so; slicing, lags and lengthscale scaling (O(N*L*D)
elementwise) run as torch ops on the same device.

The low-rank mode (``low_rank=True``: Nystrom features + randomized Hadamard projections,
gpsig/low_rank_calculations.py) runs through gpsig_amd/low_rank_calculations.py (torch GEMMs /
eigh on the device; the fused gfx950 Gram kernels are exact and are not used there).  Not carried
over ("Out of scope"): GPflow Parameter transforms/priors (parameters are plain
tensors here), and base kernels without a gfx950 seed (Cosine, Poly, Mix, Spectral, Matern*).
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib as L
from . import autograd as _ag
from . import lags as _lags
from . import low_rank_calculations as _lr
from . import ops

DEFAULT_JITTER = 1e-6  # GPflow 1.5.1 settings.jitter (third-party default, unpinned in this image)


def _params_to(obj, device, names):
    """Move the named hyperparameter tensors of a kernel object to `device` (leaves stay leaves)."""
    for n in names:
        t = getattr(obj, n, None)
        if isinstance(t, torch.Tensor):
            setattr(obj, n, t.detach().to(device).requires_grad_(t.requires_grad))


def _as_tensor(X, device=None):
    if isinstance(X, torch.Tensor):
        return X if device is None else X.to(device)
    t = torch.as_tensor(np.asarray(X))
    return t.to(device if device is not None else "cuda")


class SignatureKernel:
    """Reference gpsig/kernels.py:16-940 (non-low-rank paths)."""

    base = None  # set by subclasses: "rbf" | "linear"

    def __init__(self, input_dim, num_features, num_levels, active_dims=None, variances=1, lengthscales=1, order=1,
                 normalization=True, difference=True, num_lags=None, low_rank=False, num_components=50,
                 rank_bound=None, sparsity='sqrt', name=None, jitter=DEFAULT_JITTER):
        # kernels.py:54-89
        self.input_dim = input_dim
        self.active_dims = active_dims
        self.name = name
        self.num_features = num_features
        self.num_levels = num_levels
        self.len_examples = self._validate_number_of_features(input_dim, num_features)
        self.order = num_levels if (order <= 0 or order >= num_levels) else order
        if self.order != 1 and low_rank:
            raise NotImplementedError('Higher-order algorithms not compatible with low-rank mode (yet).')
        self.normalization = normalization
        self.difference = difference
        self.jitter = float(jitter)
        self.variances = torch.as_tensor(self._validate_signature_param("variances", variances, num_levels + 1))
        self.sigma = torch.tensor(1.0, dtype=torch.float64)
        self.low_rank, self.num_components, self.rank_bound, self.sparsity = self._validate_low_rank_params(
            low_rank, num_components, rank_bound, sparsity)
        if num_lags is None:
            self.num_lags = 0
        else:
            if not isinstance(num_lags, int) or num_lags < 0:
                raise ValueError('The variable num_lags most be a nonnegative integer or None.')
            self.num_lags = int(num_lags)
            if num_lags > 0:
                self.lags = torch.as_tensor(0.1 * np.asarray(range(1, num_lags + 1)), dtype=torch.float64)
                gamma = 1. / np.asarray(range(1, self.num_lags + 2))
                gamma /= np.sum(gamma)
                self.gamma = torch.as_tensor(gamma, dtype=torch.float64)
        if lengthscales is not None:
            self.lengthscales = torch.as_tensor(self._validate_signature_param("lengthscales", lengthscales,
                                                                               self.num_features))
        else:
            self.lengthscales = None

    # ------------------------------------------------------------------ validators (kernels.py:95-134)
    def _validate_number_of_features(self, input_dim, num_features):
        if input_dim % num_features == 0:
            return int(input_dim / num_features)
        raise ValueError("The arguments num_features and input_dim are not consistent.")

    def _validate_low_rank_params(self, low_rank, num_components, rank_bound, sparsity):
        if low_rank is not None and low_rank == True:  # noqa: E712  (reference semantics)
            if not type(low_rank) == bool:
                raise ValueError("Unknown low-rank argument: %s. It should be True of False." % low_rank)
            if sparsity not in ['log', 'sqrt', 'lin']:
                raise ValueError("Unknown sparsity argument %s. Possible values are 'sqrt', 'log', 'lin'" % sparsity)
            if rank_bound is not None and rank_bound <= 0:
                raise ValueError("The rank-bound in the low-rank algorithm must be either None or a positiv integer.")
            if num_components is None or num_components <= 0:
                raise ValueError("The number of components in the kernel approximation must be a positive integer.")
            if rank_bound is None:
                rank_bound = num_components
        else:
            low_rank = False
        return low_rank, num_components, rank_bound, sparsity

    def _validate_signature_param(self, name, value, length):
        value = value * np.ones(length, dtype=np.float64)
        correct_shape = () if length == 1 else (length,)
        if np.asarray(value).squeeze().shape != correct_shape:
            raise ValueError("shape of parameter {} is not what is expected ({})".format(name, length))
        return value

    # ------------------------------------------------------------------ preprocessing
    def _slice(self, X, X2=None):
        if self.active_dims is None:
            return X, X2
        idx = self.active_dims
        return X[..., idx], (None if X2 is None else X2[..., idx])

    def _apply_scaling_and_lags_to_sequences(self, X):
        """kernels.py:344-365 on device; X (N,L,D) -> (N,L,(lags+1)*D)."""
        N, Ln, _ = X.shape
        num_features = self.num_features * (self.num_lags + 1)
        if self.num_lags > 0:
            X = _lags.add_lags_to_sequences(X, self.lags.to(X.device, X.dtype), self.jitter)
        X = X.reshape(N, Ln, self.num_lags + 1, self.num_features)
        if self.lengthscales is not None:
            X = X / self.lengthscales.to(X.device, X.dtype)[None, None, None, :]
        if self.num_lags > 0:
            X = X * self.gamma.to(X.device, X.dtype)[None, None, :, None]
        return X.reshape(N, Ln, num_features)

    def _apply_scaling_to_tensors(self, Z):
        """kernels.py:367-382."""
        LT, T = Z.shape[0], Z.shape[1]
        if self.lengthscales is not None:
            Z = Z.reshape(LT, T, self.num_lags + 1, self.num_features) / \
                self.lengthscales.to(Z.device, Z.dtype)[None, None, None, :]
            if self.num_lags > 0:
                Z = Z * self.gamma.to(Z.device, Z.dtype)[None, None, :, None]
            Z = Z.reshape(LT, T, -1)
        return Z

    def _apply_scaling_to_incremental_tensors(self, Z):
        """kernels.py:384-399."""
        LT, T, D = Z.shape[0], Z.shape[1], Z.shape[-1]
        if self.lengthscales is not None:
            Z = Z.reshape(LT, T, 2, self.num_lags + 1, self.num_features) / \
                self.lengthscales.to(Z.device, Z.dtype)[None, None, None, None, :]
            if self.num_lags > 0:
                Z = Z * self.gamma.to(Z.device, Z.dtype)[None, None, None, :, None]
        return Z.reshape(LT, T, 2, D)

    def _prep(self, X, presliced=False):
        X = _as_tensor(X)
        if not presliced:
            X, _ = self._slice(X)
        N = X.shape[0]
        X = X.reshape(N, int(np.prod(X.shape[1:])) // self.num_features, self.num_features)  # (N = 0 allowed)
        return self._apply_scaling_and_lags_to_sequences(X)

    def _scale_vec(self, device):
        return (self.sigma * self.variances).to(device=device, dtype=torch.float32)

    def _out_dtype(self, X):
        return X.dtype if (isinstance(X, torch.Tensor) and X.is_floating_point()) else torch.float64

    # ------------------------------------------------------------------ algorithm seam (kernels.py:190-341)
    def _cfg(self, return_levels=False):
        return dict(num_levels=self.num_levels, order=self.order, base=self.base, difference=self.difference,
                    normalization=self.normalization, jitter=self.jitter, return_levels=bool(return_levels))

    def _K_seq_diag(self, X):
        """(N,L,D) scaled -> (num_levels+1, N) unnormalised diagonal (kernels.py:190-207); differentiable."""
        return _ag.SigDiag.apply(X, self._cfg())

    def _K_seq(self, X, X2=None):
        """(N,L,D) scaled -> (num_levels+1, N, N2) unnormalised per-level Gram (kernels.py:209-238)."""
        return ops.sig_gram(X, X2, self.num_levels, self.order, self.base, self.difference)

    def _rsqrt_diag(self, X):
        return ops.sig_diag(X, self.num_levels, self.order, self.base, self.difference, jitter=self.jitter,
                            rsqrt=True)

    # ------------------------------------------------------------------ low-rank mode (kernels.py:240-312)
    def _base_kern(self, X, X2=None):
        """Base kernel matrix between point sets (kernels.py:946-957, 979-986, 1042-1044)."""
        X2 = X if X2 is None else X2
        if self.base == "rbf":
            sq = (X ** 2).sum(-1)[:, None] + (X2 ** 2).sum(-1)[None, :] - 2.0 * X @ X2.T
            return torch.exp(-sq / 2.0)
        return X @ X2.T

    def _lr_seeds(self, device):
        return torch.randint(0, 2 ** 31 - 1, (max(self.num_levels - 1, 1), 2), device="cpu")

    def _K_seq_lr_feat(self, X, nys_samples=None, seeds=None):
        """kernels.py:240-262: (num_levels+1,) low-rank factors of scaled sequences X (N, L, D)."""
        N, Ln, D = X.shape
        X = X.to(torch.float64)
        feat = _lr.Nystrom_map(X.reshape(N * Ln, D), self._base_kern, nys_samples, self.num_components)
        feat = feat.reshape(N, Ln, -1)
        if self.order != 1:
            raise NotImplementedError('Low-rank mode not implemented for order higher than 1.')
        return _lr.signature_kern_first_order_lr_feature(feat, self.num_levels, self.rank_bound, self.sparsity,
                                                         seeds, difference=self.difference)

    def _K_tens_lr_feat(self, Z, increments=False, nys_samples=None, seeds=None):
        """kernels.py:286-312."""
        if self.order > 1:
            raise NotImplementedError('higher order not implemented yet for low-rank mode')
        Z = Z.to(torch.float64)
        LT, T, D = Z.shape[0], Z.shape[1], Z.shape[-1]
        if increments:
            f = _lr.Nystrom_map(Z.reshape(LT * T * 2, D), self._base_kern, nys_samples, self.num_components)
            f = f.reshape(LT, T, 2, -1)
            f = f[:, :, 1, :] - f[:, :, 0, :]
        else:
            f = _lr.Nystrom_map(Z.reshape(LT * T, D), self._base_kern, nys_samples, self.num_components)
            f = f.reshape(LT, T, -1)
        return _lr.tensor_kern_lr_feature(f, self.num_levels, self.rank_bound, self.sparsity, seeds)

    def _nys_from(self, *sets):
        """Shared Nystrom samples drawn from the union of point sets (kernels.py:443-446, 593-595)."""
        pts = torch.cat([s.reshape(-1, s.shape[-1]).to(torch.float64) for s in sets], 0)
        idx, _ = _lr._draw_indices(pts.shape[0], self.num_components, device=pts.device)
        return pts[idx]

    @staticmethod
    def _gram_of(P, Q=None):
        return torch.stack([p @ (p if Q is None else q).T for p, q in zip(P, P if Q is None else Q)], 0)

    def _K_lowrank(self, Xs, X2s, return_levels):
        """The low_rank branch of K (kernels.py:423-476), on the scaled sequences (the reference feeds
        the unscaled X to _K_seq_lr_feat in K only, kernels.py:426,448 -- not reproduced)."""
        if X2s is None:
            Phi = self._K_seq_lr_feat(Xs)
            K = self._gram_of(Phi)
            if self.normalization:
                K = K + self.jitter * torch.eye(K.shape[1], dtype=K.dtype, device=K.device)[None]
                d = torch.sqrt(torch.diagonal(K, dim1=1, dim2=2))
                K = K / (d[:, :, None] * d[:, None, :])
        else:
            seeds = self._lr_seeds(Xs.device)
            nys = self._nys_from(Xs, X2s)
            Phi = self._K_seq_lr_feat(Xs, nys, seeds)
            Phi2 = self._K_seq_lr_feat(X2s, nys, seeds)
            K = self._gram_of(Phi, Phi2)
            if self.normalization:
                d1 = torch.sqrt(torch.stack([(p ** 2).sum(-1) for p in Phi], 0) + self.jitter)
                d2 = torch.sqrt(torch.stack([(p ** 2).sum(-1) for p in Phi2], 0) + self.jitter)
                K = K / (d1[:, :, None] * d2[:, None, :])
        K = K * (self.sigma * self.variances).to(K.device, K.dtype)[:, None, None]
        return K if return_levels else K.sum(0)

    # ------------------------------------------------------------------ public API
    def to(self, device):
        """Keep variances, lengthscales, lags and gamma on `device` (sigma stays a host scalar), so a
        call makes no host-to-device copies -- required for hipGraph capture (gpsig_amd.graphs).
        Returns self."""
        _params_to(self, device, ("variances", "lengthscales", "lags", "gamma"))
        return self

    def K(self, X, X2=None, presliced=False, return_levels=False, presliced_X=False, presliced_X2=False):
        """kernels.py:402-477: (N, N2) or (num_levels+1, N, N2) with return_levels."""
        if presliced:
            presliced_X = presliced_X2 = True
        dt = self._out_dtype(X)
        if self.low_rank:
            Xs = self._prep(X, presliced_X)
            X2s = None if X2 is None else self._prep(X2, presliced_X2)
            return self._K_lowrank(Xs, X2s, return_levels).to(dt)
        Xs = self._prep(X, presliced_X)
        X2s = None if X2 is None else self._prep(X2, presliced_X2)
        scale = (self.sigma * self.variances).to(Xs.device)
        # forward: fused Gram kernel; backward (autograd): gpsig_sig_gram_vjp (gpsig_amd/autograd.py)
        out = _ag.SigGram.apply(Xs, X2s, scale, self._cfg(return_levels))
        return out.to(dt)

    def K_norms(self, X, presliced=False):
        """kernels.py:481-506."""
        Xs = self._prep(X, presliced)
        N = Xs.shape[0]
        const = torch.full((N,), float(self.sigma * self.variances.sum()), dtype=self._out_dtype(X), device=Xs.device)
        return const, self._K_seq_diag(Xs).to(self._out_dtype(X))

    def Kdiag(self, X, presliced=False, return_levels=False):
        """kernels.py:510-541."""
        Xt = _as_tensor(X)
        N = Xt.shape[0]
        dt = self._out_dtype(X)
        if self.normalization:
            sv = (self.sigma * self.variances).to(Xt.device, dt)
            if return_levels:
                return sv[:, None].repeat(1, N)
            return torch.full((N,), float(sv.sum()), dtype=dt, device=Xt.device)
        Xs = self._prep(Xt, presliced)
        if self.low_rank:
            Kd = torch.stack([(p ** 2).sum(-1) for p in self._K_seq_lr_feat(Xs)], 0)
            Kd = Kd * (self.sigma * self.variances).to(Xs.device, Kd.dtype)[:, None]
            return (Kd if return_levels else Kd.sum(0)).to(dt)
        Kd = self._K_seq_diag(Xs) * (self.sigma * self.variances).to(Xs.device, torch.float32)[:, None]
        return (Kd if return_levels else Kd.sum(0)).to(dt)

    # ------------------------------------------------------------------ inducing tensors (kernels.py:544-704)
    def _K_tens(self, Z, increments=False):
        """Raw per-level (num_levels+1, T, T) (kernels.py:264-284); differentiable in Z."""
        cfg = self._cfg()
        cfg["increments"] = bool(increments)
        return _ag.TensGram.apply(Z, cfg)

    def _rs_diff(self, Xs):
        """1/sqrt(diag + jitter) per level, differentiable (SigDiag backward = diagonal VJP launch)."""
        return torch.rsqrt(self._K_seq_diag(Xs) + self.jitter)

    def _K_tens_vs_seq(self, Z, X, increments=False):
        """Raw per-level (num_levels+1, T, N) (kernels.py:314-341); differentiable in Z and X."""
        cfg = self._cfg()
        cfg["increments"] = bool(increments)
        return _ag.TensVsSeq.apply(Z, X, cfg)

    def K_tens(self, Z, return_levels=False, increments=False):
        """kernels.py:544-567."""
        Zt = _as_tensor(Z)
        dt = self._out_dtype(Z)
        Zs = self._apply_scaling_to_incremental_tensors(Zt) if increments else self._apply_scaling_to_tensors(Zt)
        if self.low_rank:
            K = self._gram_of(self._K_tens_lr_feat(Zs, increments))
        else:
            K = self._K_tens(Zs, increments)
        K = K * (self.sigma * self.variances).to(Zs.device, K.dtype)[:, None, None]
        return (K if return_levels else K.sum(0)).to(dt)

    def K_tens_vs_seq(self, Z, X, return_levels=False, increments=False, presliced=False):
        """kernels.py:571-620."""
        Zt = _as_tensor(Z)
        dt = self._out_dtype(X)
        Xs = self._prep(X, presliced)
        Zs = self._apply_scaling_to_incremental_tensors(Zt) if increments else self._apply_scaling_to_tensors(Zt)
        if self.low_rank:
            PhiZ, PhiX = self._lr_tens_seq_feats(Zs, Xs, increments)
            Kzx = self._gram_of(PhiZ, PhiX)
            if self.normalization:
                Kzx = Kzx / torch.sqrt(torch.stack([(p ** 2).sum(-1) for p in PhiX], 0) + self.jitter)[:, None, :]
        else:
            Kzx = self._K_tens_vs_seq(Zs, Xs, increments)
            if self.normalization:
                Kzx = Kzx * self._rs_diff(Xs)[:, None, :]
        Kzx = Kzx * (self.sigma * self.variances).to(Xs.device, Kzx.dtype)[:, None, None]
        return (Kzx if return_levels else Kzx.sum(0)).to(dt)

    def _lr_tens_seq_feats(self, Zs, Xs, increments):
        """Shared seeds and Nystrom samples for tensors and sequences (kernels.py:592-598, 645-652)."""
        seeds = self._lr_seeds(Xs.device)
        nys = self._nys_from(Zs, Xs)
        return self._K_tens_lr_feat(Zs, increments, nys, seeds), self._K_seq_lr_feat(Xs, nys, seeds)

    def _sv(self, device):
        """sigma * variances as float32 on device, differentiable in variances."""
        return (self.sigma * self.variances).to(device, torch.float32)

    def _gram_levels(self, Xs, X2s=None):
        """Normalised (if self.normalization) per-level K(X[, X2]) x sigma*variances, differentiable."""
        return _ag.SigGram.apply(Xs, X2s, (self.sigma * self.variances).to(Xs.device), self._cfg(True))

    def K_tens_n_seq_covs(self, Z, X, full_X_cov=False, return_levels=False, increments=False, presliced=False):
        """kernels.py:624-704 (differentiable in Z, X, lengthscales, variances)."""
        Zt = _as_tensor(Z)
        dt = self._out_dtype(X)
        Xs = self._prep(X, presliced)
        N = Xs.shape[0]
        Zs = self._apply_scaling_to_incremental_tensors(Zt) if increments else self._apply_scaling_to_tensors(Zt)
        if self.low_rank:
            return self._lr_tens_n_seq_covs(Zs, Xs, full_X_cov, return_levels, increments, dt)
        sv = self._sv(Xs.device)
        Kzz = self._K_tens(Zs, increments) * sv[:, None, None]
        Kzx = self._K_tens_vs_seq(Zs, Xs, increments)
        if self.normalization:
            Kzx = Kzx * self._rs_diff(Xs)[:, None, :]
        Kzx = Kzx * sv[:, None, None]
        if full_X_cov:
            Kxx = self._gram_levels(Xs)
        elif self.normalization:
            Kxx = sv[:, None].repeat(1, N)
        else:
            Kxx = self._K_seq_diag(Xs) * sv[:, None]
        out = (Kzz, Kzx, Kxx)
        if not return_levels:
            out = tuple(o.sum(0) for o in out)
        return tuple(o.to(dt) for o in out)

    def K_seq_n_seq_covs(self, X, X2, full_X2_cov=False, return_levels=False, presliced=False):
        """kernels.py:707-794 (differentiable).  Two reference defects are not reproduced: the
        NameError branch at :756-761 is restated with the intended names, and in the diagonal branch
        Kxx2 is normalised once by each side's norms (:768 and :784 divide it by X's norms twice)."""
        dt = self._out_dtype(X)
        Xs = self._prep(X, True)  # reference slices only X2 here (kernels.py:712-713)
        X2s = self._prep(X2, presliced)
        N2 = X2s.shape[0]
        if self.low_rank:
            return self._lr_seq_n_seq_covs(Xs, X2s, full_X2_cov, return_levels, dt)
        sv = self._sv(Xs.device)
        Kxx = self._gram_levels(Xs)
        Kxx2 = self._gram_levels(Xs, X2s)
        if full_X2_cov:
            Kd = self._gram_levels(X2s)
        elif self.normalization:
            Kd = sv[:, None].repeat(1, N2)
        else:
            Kd = self._K_seq_diag(X2s) * sv[:, None]
        out = (Kxx, Kxx2, Kd)
        if not return_levels:
            out = tuple(o.sum(0) for o in out)
        return tuple(o.to(dt) for o in out)

    def _lr_norm_sym(self, Phi):
        """Gram of low-rank factors with jitter + diagonal normalisation (kernels.py:431-434), and the
        square roots of its diagonal."""
        K = self._gram_of(Phi)
        if not self.normalization:
            return K, None
        K = K + self.jitter * torch.eye(K.shape[1], dtype=K.dtype, device=K.device)[None]
        d = torch.sqrt(torch.diagonal(K, dim1=1, dim2=2))
        return K / (d[:, :, None] * d[:, None, :]), d

    def _lr_tens_n_seq_covs(self, Zs, Xs, full_X_cov, return_levels, increments, dt):
        """Low-rank branch of K_tens_n_seq_covs (kernels.py:645-704)."""
        N = Xs.shape[0]
        PhiZ, PhiX = self._lr_tens_seq_feats(Zs, Xs, increments)
        sv = (self.sigma * self.variances).to(Xs.device, torch.float64)
        Kzz = self._gram_of(PhiZ) * sv[:, None, None]
        Kzx = self._gram_of(PhiZ, PhiX)
        if full_X_cov:
            Kxx, d = self._lr_norm_sym(PhiX)
            if d is not None:
                Kzx = Kzx / d[:, None, :]
            Kxx = Kxx * sv[:, None, None]
        else:
            Kd = torch.stack([(p ** 2).sum(-1) for p in PhiX], 0)
            if self.normalization:
                Kzx = Kzx / torch.sqrt(Kd + self.jitter)[:, None, :]
                Kxx = sv[:, None].repeat(1, N)
            else:
                Kxx = Kd * sv[:, None]
        out = (Kzz, Kzx * sv[:, None, None], Kxx)
        if not return_levels:
            out = tuple(o.sum(0) for o in out)
        return tuple(o.to(dt) for o in out)

    def _lr_seq_n_seq_covs(self, Xs, X2s, full_X2_cov, return_levels, dt):
        """Low-rank branch of K_seq_n_seq_covs (kernels.py:720-794, intended semantics)."""
        N2 = X2s.shape[0]
        seeds = self._lr_seeds(Xs.device)
        nys = self._nys_from(Xs, X2s)
        Phi, Phi2 = self._K_seq_lr_feat(Xs, nys, seeds), self._K_seq_lr_feat(X2s, nys, seeds)
        sv = (self.sigma * self.variances).to(Xs.device, torch.float64)
        Kxx, d = self._lr_norm_sym(Phi)
        Kxx2 = self._gram_of(Phi, Phi2)
        if d is not None:
            Kxx2 = Kxx2 / d[:, :, None]
        if full_X2_cov:
            Kd, d2 = self._lr_norm_sym(Phi2)
            if d2 is not None:
                Kxx2 = Kxx2 / d2[:, None, :]
            Kd = Kd * sv[:, None, None]
        else:
            Kd = torch.stack([(p ** 2).sum(-1) for p in Phi2], 0)
            if self.normalization:
                Kxx2 = Kxx2 / torch.sqrt(Kd + self.jitter)[:, None, :]
                Kd = sv[:, None].repeat(1, N2)
            else:
                Kd = Kd * sv[:, None]
        out = (Kxx * sv[:, None, None], Kxx2 * sv[:, None, None], Kd)
        if not return_levels:
            out = tuple(o.sum(0) for o in out)
        return tuple(o.to(dt) for o in out)

    # ------------------------------------------------------------------ VOSF helpers (kernels.py:800-940)
    def _Mahalanobis_term_approx_posterior(self, Z, X):
        """kernels.py:800-822 (linear embedding): (num_levels+1, N, T)."""
        return ops.rescaled(Z, X, self.num_levels, embedding="linear")

    def Mahalanobis_term_approx_posterior(self, Z, X, presliced=False):
        """kernels.py:876-895."""
        Zt = _as_tensor(Z)
        dt = self._out_dtype(X)
        Xs = self._prep(X, presliced)
        K = self._Mahalanobis_term_approx_posterior(Zt[1:], Xs) * float(self.sigma)
        return (K.sum(0) + 1.0 - Zt[0, :, 0].to(K)[None, :]).to(dt)

    def norms_tens(self, Z):
        """kernels.py:897-906 (O(M^2 T) host arithmetic)."""
        Zt = _as_tensor(Z)
        M = torch.sum(Zt[1:] ** 2, dim=2)
        return _tensor_inner_product(M, self.num_levels).sum(0) - 1.0 + Zt[0, :, 0] ** 2

    def logs_tens(self, Z):
        """kernels.py:908-917."""
        Zt = _as_tensor(Z)
        M = torch.sum(torch.log(Zt[1:]), dim=2)
        return _tensor_logs(M, self.num_levels, Zt.shape[2]).sum(0) + torch.log(Zt[0, :, 0])

    def inner_product_tens_vs_seq(self, Z, X, presliced=False):
        """kernels.py:919-940: linear inner products <S(X), m_r> at order = num_levels."""
        Zt = _as_tensor(Z)
        dt = self._out_dtype(X)
        Xs = self._prep(X, presliced)
        K = ops.tens_vs_seq(Zt[1:], Xs, self.num_levels, self.num_levels, "linear", True, False)
        s = float(self.sigma) ** 0.5
        return (K.sum(0) * s + s * (Zt[0, :, 0].to(K)[:, None] - 1.0)).to(dt)

    # ------------------------------------------------------------------ autoflow-style helpers (kernels.py:142-187)
    def compute_K(self, X, Y):
        return self.K(_as_tensor(X), _as_tensor(Y)).cpu().numpy()

    def compute_K_symm(self, X):
        return self.K(_as_tensor(X)).cpu().numpy()

    def compute_K_level_diags(self, X):
        return self.Kdiag(_as_tensor(X), return_levels=True).cpu().numpy()

    def compute_K_levels(self, X, X2):
        return self.K(_as_tensor(X), _as_tensor(X2), return_levels=True).cpu().numpy()

    def compute_Kdiag(self, X):
        return self.Kdiag(_as_tensor(X)).cpu().numpy()

    def compute_K_tens(self, Z):
        return self.K_tens(_as_tensor(Z), return_levels=False).cpu().numpy()

    def compute_K_tens_vs_seq(self, Z, X):
        return self.K_tens_vs_seq(_as_tensor(Z), _as_tensor(X), return_levels=False).cpu().numpy()

    def compute_K_incr_tens(self, Z):
        return self.K_tens(_as_tensor(Z), increments=True, return_levels=False).cpu().numpy()

    def compute_K_incr_tens_vs_seq(self, Z, X):
        return self.K_tens_vs_seq(_as_tensor(Z), _as_tensor(X), increments=True, return_levels=False).cpu().numpy()

    def compute_base_kern_symm(self, X):
        """kernels.py:151-158: the base-kernel tensor M[a, b, i, j] = k(x_{a,i}, x_{b,j}) of the scaled
        sequences, (N, N, L, L) -- the tensor the reference's recursion consumes (here for inspection
        only: the gfx950 kernels never materialise it)."""
        Xt = _as_tensor(X)
        N = Xt.shape[0]
        Xs = self._apply_scaling_and_lags_to_sequences(Xt.reshape(N, -1, self.num_features)).to(torch.float64)
        Ln = Xs.shape[1]
        P = Xs.reshape(N * Ln, -1)
        return self._base_kern(P).reshape(N, Ln, N, Ln).permute(0, 2, 1, 3).cpu().numpy()


def _tensor_inner_product(M, num_levels):
    """signature_algs_vosf.py:51-74."""
    out = [torch.ones_like(M[0])]
    k = 0
    for i in range(1, num_levels + 1):
        R = M[k]
        k += 1
        for _ in range(1, i):
            R = M[k] * R
            k += 1
        out.append(R)
    return torch.stack(out, 0)


def _tensor_logs(M, num_levels, d):
    """signature_algs_vosf.py:76-100."""
    out = [torch.zeros_like(M[0])]
    k = 0
    for i in range(1, num_levels + 1):
        R = M[k]
        k += 1
        for _ in range(1, i):
            R = M[k] + R
            k += 1
        out.append(float(d) ** (i - 1) * R)
    return torch.stack(out, 0)


class SignatureLinear(SignatureKernel):
    """kernels.py:966-986: identity state-space embedding."""
    base = "linear"


class SignatureRBF(SignatureKernel):
    """kernels.py:1030-1044: Gaussian state-space embedding."""
    base = "rbf"


SignatureGauss = SignatureRBF


class _Unsupported(SignatureKernel):
    def __init__(self, *args, **kwargs):
        raise NotImplementedError(f"{type(self).__name__}: this base kernel has no gfx950 seed in this build "
                                  "(supported: SignatureRBF/SignatureGauss, SignatureLinear); see DESIGN.md")


class SignatureCosine(_Unsupported):
    """kernels.py:988-1008 (not built)."""


class SignaturePoly(_Unsupported):
    """kernels.py:1011-1028 (not built)."""


class SignatureMix(_Unsupported):
    """kernels.py:1050-1072 (not built)."""


class SignatureSpectral(_Unsupported):
    """kernels.py:1074-1122 (not built)."""


class SignatureMatern12(_Unsupported):
    """kernels.py:1124-1138 (not built)."""


class SignatureMatern32(_Unsupported):
    """kernels.py:1144-1157 (not built)."""


class SignatureMatern52(_Unsupported):
    """kernels.py:1161-1173 (not built)."""


SignatureLaplace = SignatureMatern12
SignatureExponential = SignatureMatern12
