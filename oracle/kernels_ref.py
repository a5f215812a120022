"""CPU oracle: float64 NumPy restatement of the reference kernel orchestration.

TEST INFRASTRUCTURE ONLY (see oracle/sigalgs.py header).

Restates, on NumPy float64 arrays, what the GPflow kernels of the reference do
around the recursions (file:line relative to /root/reference):
  * SignatureKernel.__init__ parameters            gpsig/kernels.py:19-89
  * _K_seq_diag / _K_seq                            gpsig/kernels.py:190-238
  * _K_tens / _K_tens_vs_seq                        gpsig/kernels.py:264-284, 314-341
  * _apply_scaling_and_lags_to_sequences            gpsig/kernels.py:344-365
  * _apply_scaling_to_tensors / _incremental_       gpsig/kernels.py:367-399
  * K (jitter + diag normalisation + sigma*var)     gpsig/kernels.py:402-477
  * K_norms / Kdiag                                 gpsig/kernels.py:481-541
  * K_tens / K_tens_vs_seq                          gpsig/kernels.py:544-620
  * K_tens_n_seq_covs / K_seq_n_seq_covs            gpsig/kernels.py:624-794
  * VOSF helpers                                    gpsig/kernels.py:800-940
  * base kernels _square_dist/_lin/_cos/_poly/_rbf/_mix/_Matern*   gpsig/kernels.py:946-1173
  * lags.lin_interp / add_lags_to_sequences         gpsig/lags.py:7-63

Third-party defaults that are not in this container and are therefore
"parity unpinned": GPflow 1.5.1 ``settings.jitter`` (1e-6) and
``settings.float_type`` (float64).  They are explicit constructor arguments
here (``jitter=1e-6``).

Known reference defects are NOT reproduced: the
``K_x2x2_lvls`` NameError branch of K_seq_n_seq_covs (kernels.py:756-761) is
restated with the evidently intended names, and its diagonal branch normalises
Kxx2 once by each side's norms (kernels.py:768 and :784 both divide it by the
norms of X, i.e. twice).
"""
from __future__ import annotations

import numpy as np

from . import sigalgs

JITTER = 1e-6


# ----------------------------------------------------------------------------- lags
def lin_interp(time, X, time_query, jitter=JITTER):
    """lags.py:7-38."""
    pairwise = time[:, None, None] - time_query[None, :, :]
    masked = np.where(pairwise > jitter, -np.inf, pairwise)
    left = np.argmax(masked, axis=0)
    right = left + 1
    Xl = np.take(X, left, axis=-2)
    Xr = np.take(X, right, axis=-2)
    tl = time[left]
    tr = time[right]
    if X.ndim == 3:
        return Xl + (time_query[None, ..., None] - tl[None, ..., None]) * (Xr - Xl) / (tr[None, ..., None] - tl[None, ..., None])
    raise ValueError("lin_interp: X must be 3-D here")


def add_lags_to_sequences(X, lags, jitter=JITTER):
    """lags.py:41-63.  X (N,L,D), lags (nl,) -> (N,L,nl+1,D)."""
    L = X.shape[1]
    time = np.arange(L, dtype=np.float64) / float(L - 1)
    time_lags = np.maximum(time[:, None] - np.asarray(lags, dtype=np.float64)[None, :], 0.0)
    Xq = lin_interp(time, X, time_lags, jitter)
    return np.concatenate((X[:, :, None, :], Xq), axis=2)


# ----------------------------------------------------------------------------- base kernels
def square_dist(X, X2=None):
    """kernels.py:946-957 (batched over leading dims)."""
    Xs = np.sum(X * X, axis=-1)
    if X2 is None:
        dist = -2.0 * (X @ np.swapaxes(X, -1, -2))
        return dist + Xs[..., :, None] + Xs[..., None, :]
    X2s = np.sum(X2 * X2, axis=-1)
    dist = -2.0 * (X @ np.swapaxes(X2, -1, -2))
    return dist + Xs[..., :, None] + X2s[..., None, :]


def base_rbf(X, X2=None):
    """kernels.py:1042-1044."""
    return np.exp(-square_dist(X, X2) / 2.0)


def base_lin(X, X2=None):
    """kernels.py:979-986."""
    Y = X if X2 is None else X2
    return X @ np.swapaxes(Y, -1, -2)


def base_cos(X, X2=None):
    """kernels.py:1000-1008."""
    n1 = np.sqrt(np.sum(X * X, axis=-1))
    Y = X if X2 is None else X2
    n2 = np.sqrt(np.sum(Y * Y, axis=-1))
    return (X @ np.swapaxes(Y, -1, -2)) / (n1[..., :, None] * n2[..., None, :])


def make_base_poly(gamma=1.0, degree=3.0):
    """kernels.py:1023-1028."""
    def base_poly(X, X2=None):
        Y = X if X2 is None else X2
        return (X @ np.swapaxes(Y, -1, -2) + gamma) ** degree
    return base_poly


def make_base_mix(mixing=0.5):
    """kernels.py:1061-1072."""
    def base_mix(X, X2=None):
        Y = X if X2 is None else X2
        inner = X @ np.swapaxes(Y, -1, -2)
        ds = np.sum(X * X, -1)[..., :, None] + np.sum(Y * Y, -1)[..., None, :] - 2 * inner
        return mixing * np.exp(-ds / 2) + (1.0 - mixing) * inner
    return base_mix


def _euclid(X, X2=None):
    """kernels.py:959-961."""
    return np.sqrt(np.maximum(square_dist(X, X2), 1e-40))


def base_matern12(X, X2=None):
    """kernels.py:1135-1138."""
    return np.exp(-_euclid(X, X2))


def base_matern32(X, X2=None):
    """kernels.py:1154-1157."""
    r = _euclid(X, X2)
    return (1.0 + np.sqrt(3.0) * r) * np.exp(-np.sqrt(3.0) * r)


def base_matern52(X, X2=None):
    """kernels.py:1171-1173."""
    r = _euclid(X, X2)
    return (1.0 + np.sqrt(5.0) * r + 5.0 / 3.0 * r * r) * np.exp(-np.sqrt(5.0) * r)


BASE_KERNELS = {
    "rbf": base_rbf,
    "linear": base_lin,
    "cosine": base_cos,
    "matern12": base_matern12,
    "matern32": base_matern32,
    "matern52": base_matern52,
}


# ----------------------------------------------------------------------------- kernel
class SignatureKernelRef:
    """Restatement of gpsig.kernels.SignatureKernel (non-low-rank paths) on NumPy float64."""

    def __init__(self, input_dim, num_features, num_levels, base="rbf", active_dims=None, variances=1.0,
                 lengthscales=1.0, order=1, normalization=True, difference=True, num_lags=None,
                 sigma=1.0, lags=None, gamma=None, jitter=JITTER, base_kern=None):
        if input_dim % num_features != 0:
            raise ValueError("The arguments num_features and input_dim are not consistent.")
        self.input_dim = input_dim
        self.num_features = num_features
        self.num_levels = num_levels
        self.len_examples = input_dim // num_features
        self.order = num_levels if (order <= 0 or order >= num_levels) else order
        self.normalization = normalization
        self.difference = difference
        self.active_dims = active_dims
        self.variances = np.asarray(variances, dtype=np.float64) * np.ones(num_levels + 1)
        self.sigma = float(sigma)
        self.jitter = float(jitter)
        self.num_lags = 0 if num_lags is None else int(num_lags)
        if self.num_lags > 0:
            # kernels.py:80-83 initial values (the Logistic/positive transforms only constrain them)
            self.lags = np.asarray(lags if lags is not None else 0.1 * np.arange(1, self.num_lags + 1), dtype=np.float64)
            g = 1.0 / np.arange(1, self.num_lags + 2)
            self.gamma = np.asarray(gamma if gamma is not None else g / g.sum(), dtype=np.float64)
        self.lengthscales = None if lengthscales is None else np.asarray(lengthscales, dtype=np.float64) * np.ones(num_features)
        self._base_kern = base_kern if base_kern is not None else BASE_KERNELS[base]

    # -- helpers
    def _slice(self, X):
        if self.active_dims is None:
            return X
        return X[..., self.active_dims]

    def scale_sequences(self, X):
        """kernels.py:344-365.  X (N,L,D) -> (N,L,(nl+1)*D)."""
        N, L, _ = X.shape
        if self.num_lags > 0:
            X = add_lags_to_sequences(X, self.lags, self.jitter)
        X = X.reshape(N, L, self.num_lags + 1, self.num_features)
        if self.lengthscales is not None:
            X = X / self.lengthscales[None, None, None, :]
        if self.num_lags > 0:
            X = X * self.gamma[None, None, :, None]
        return X.reshape(N, L, (self.num_lags + 1) * self.num_features)

    def scale_tensors(self, Z):
        """kernels.py:367-382."""
        LT, T = Z.shape[0], Z.shape[1]
        if self.lengthscales is not None:
            Z = Z.reshape(LT, T, self.num_lags + 1, self.num_features) / self.lengthscales[None, None, None, :]
            if self.num_lags > 0:
                Z = Z * self.gamma[None, None, :, None]
            Z = Z.reshape(LT, T, -1)
        return Z

    def scale_incr_tensors(self, Z):
        """kernels.py:384-399."""
        LT, T, D = Z.shape[0], Z.shape[1], Z.shape[-1]
        if self.lengthscales is not None:
            Z = Z.reshape(LT, T, 2, self.num_lags + 1, self.num_features) / self.lengthscales[None, None, None, None, :]
            if self.num_lags > 0:
                Z = Z * self.gamma[None, None, None, :, None]
        return Z.reshape(LT, T, 2, D)

    def _algo(self, M):
        if self.order == 1:
            return sigalgs.signature_kern_first_order(M, self.num_levels, difference=self.difference)
        return sigalgs.signature_kern_higher_order(M, self.num_levels, order=self.order, difference=self.difference)

    def K_seq_diag(self, Xs):
        """kernels.py:190-207: 3-D base-kernel tensor (N,L,L)."""
        return self._algo(self._base_kern(Xs))

    def K_seq(self, Xs, X2s=None):
        """kernels.py:209-238: 4-D base-kernel tensor (N1,L1,N2,L2)."""
        N, L, D = Xs.shape
        if X2s is None:
            flat = Xs.reshape(N * L, D)
            M = self._base_kern(flat).reshape(N, L, N, L)
        else:
            N2, L2 = X2s.shape[0], X2s.shape[1]
            M = self._base_kern(Xs.reshape(N * L, D), X2s.reshape(N2 * L2, D)).reshape(N, L, N2, L2)
        return self._algo(M)

    def K_tens_raw(self, Z, increments=False):
        """kernels.py:264-284."""
        LT, T, D = Z.shape[0], Z.shape[1], Z.shape[-1]
        if increments:
            Zr = Z.reshape(LT, 2 * T, D)
            M = self._base_kern(Zr).reshape(LT, T, 2, T, 2)
            M = M[:, :, 1, :, 1] + M[:, :, 0, :, 0] - M[:, :, 1, :, 0] - M[:, :, 0, :, 1]
        else:
            M = self._base_kern(Z)
        return sigalgs.tensor_kern(M, self.num_levels)

    def K_tens_vs_seq_raw(self, Z, Xs, increments=False):
        """kernels.py:314-341."""
        LT, T, D = Z.shape[0], Z.shape[1], Z.shape[-1]
        N, L = Xs.shape[0], Xs.shape[1]
        Xf = Xs.reshape(N * L, D)
        if increments:
            M = self._base_kern(Z.reshape(2 * T * LT, D), Xf).reshape(LT, T, 2, N, L)
            M = M[:, :, 1] - M[:, :, 0]
        else:
            M = self._base_kern(Z.reshape(T * LT, D), Xf).reshape(LT, T, N, L)
        if self.order == 1:
            return sigalgs.signature_kern_tens_vs_seq_first_order(M, self.num_levels, difference=self.difference)
        return sigalgs.signature_kern_tens_vs_seq_higher_order(M, self.num_levels, order=self.order, difference=self.difference)

    def _prep(self, X):
        X = self._slice(np.asarray(X, dtype=np.float64))
        N = X.shape[0]
        X = X.reshape(N, -1, self.num_features)
        return self.scale_sequences(X)

    # -- public API (kernels.py)
    def K(self, X, X2=None, return_levels=False):
        """kernels.py:402-477 (non-low-rank)."""
        Xs = self._prep(X)
        N = Xs.shape[0]
        if X2 is None:
            K = self.K_seq(Xs)
            if self.normalization:
                K = K + self.jitter * np.eye(N)[None]
                ds = np.sqrt(np.diagonal(K, axis1=1, axis2=2))
                K = K / (ds[:, :, None] * ds[:, None, :])
        else:
            X2s = self._prep(X2)
            K = self.K_seq(Xs, X2s)
            if self.normalization:
                d1 = np.sqrt(self.K_seq_diag(Xs) + self.jitter)
                d2 = np.sqrt(self.K_seq_diag(X2s) + self.jitter)
                K = K / (d1[:, :, None] * d2[:, None, :])
        K = K * (self.sigma * self.variances[:, None, None])
        return K if return_levels else np.sum(K, axis=0)

    def K_norms(self, X):
        """kernels.py:481-506."""
        Xs = self._prep(X)
        return np.full((Xs.shape[0],), self.sigma * np.sum(self.variances)), self.K_seq_diag(Xs)

    def Kdiag(self, X, return_levels=False):
        """kernels.py:510-541."""
        N = np.asarray(X).shape[0]
        if self.normalization:
            if return_levels:
                return np.tile(self.sigma * self.variances[:, None], (1, N))
            return np.full((N,), self.sigma * np.sum(self.variances))
        Kd = self.K_seq_diag(self._prep(X)) * (self.sigma * self.variances[:, None])
        return Kd if return_levels else np.sum(Kd, axis=0)

    def K_tens(self, Z, return_levels=False, increments=False):
        """kernels.py:544-567."""
        Z = self.scale_incr_tensors(Z) if increments else self.scale_tensors(Z)
        K = self.K_tens_raw(Z, increments) * (self.sigma * self.variances[:, None, None])
        return K if return_levels else np.sum(K, axis=0)

    def K_tens_vs_seq(self, Z, X, return_levels=False, increments=False):
        """kernels.py:571-620."""
        Xs = self._prep(X)
        Z = self.scale_incr_tensors(Z) if increments else self.scale_tensors(Z)
        Kzx = self.K_tens_vs_seq_raw(Z, Xs, increments)
        if self.normalization:
            dx = np.sqrt(self.K_seq_diag(Xs) + self.jitter)
            Kzx = Kzx / dx[:, None, :]
        Kzx = Kzx * (self.sigma * self.variances[:, None, None])
        return Kzx if return_levels else np.sum(Kzx, axis=0)

    def K_tens_n_seq_covs(self, Z, X, full_X_cov=False, return_levels=False, increments=False):
        """kernels.py:624-704."""
        Xs = self._prep(X)
        N = Xs.shape[0]
        Z = self.scale_incr_tensors(Z) if increments else self.scale_tensors(Z)
        Kzz = self.K_tens_raw(Z, increments)
        Kzx = self.K_tens_vs_seq_raw(Z, Xs, increments)
        sv = self.sigma * self.variances
        if full_X_cov:
            Kxx = self.K_seq(Xs)
            if self.normalization:
                Kxx = Kxx + self.jitter * np.eye(N)[None]
                ds = np.sqrt(np.diagonal(Kxx, axis1=1, axis2=2))
                Kxx = Kxx / (ds[:, :, None] * ds[:, None, :])
                Kzx = Kzx / ds[:, None, :]
            Kxx = Kxx * sv[:, None, None]
            Kzz = Kzz * sv[:, None, None]
            Kzx = Kzx * sv[:, None, None]
            if return_levels:
                return Kzz, Kzx, Kxx
            return Kzz.sum(0), Kzx.sum(0), Kxx.sum(0)
        Kxx = self.K_seq_diag(Xs)
        if self.normalization:
            ds = np.sqrt(Kxx + self.jitter)
            Kzx = Kzx / ds[:, None, :]
            Kxx = np.tile(sv[:, None], (1, N))
        else:
            Kxx = Kxx * sv[:, None]
        Kzz = Kzz * sv[:, None, None]
        Kzx = Kzx * sv[:, None, None]
        if return_levels:
            return Kzz, Kzx, Kxx
        return Kzz.sum(0), Kzx.sum(0), Kxx.sum(0)

    def K_seq_n_seq_covs(self, X, X2, full_X2_cov=False, return_levels=False):
        """kernels.py:707-794 (intended semantics of the typo'd branch)."""
        Xs = self._prep(X)
        X2s = self._prep(X2)
        N, N2 = Xs.shape[0], X2s.shape[0]
        Kxx = self.K_seq(Xs)
        Kxx2 = self.K_seq(Xs, X2s)
        sv = self.sigma * self.variances
        if self.normalization:
            Kxx = Kxx + self.jitter * np.eye(N)[None]
            ds = np.sqrt(np.diagonal(Kxx, axis1=1, axis2=2))
            Kxx = Kxx / (ds[:, :, None] * ds[:, None, :])
            Kxx2 = Kxx2 / ds[:, :, None]
        if full_X2_cov:
            Kx2x2 = self.K_seq(X2s)
            if self.normalization:
                Kx2x2 = Kx2x2 + self.jitter * np.eye(N2)[None]
                ds2 = np.sqrt(np.diagonal(Kx2x2, axis1=1, axis2=2))
                Kxx2 = Kxx2 / ds2[:, None, :]
                Kx2x2 = Kx2x2 / (ds2[:, :, None] * ds2[:, None, :])
            out = (Kxx * sv[:, None, None], Kxx2 * sv[:, None, None], Kx2x2 * sv[:, None, None])
        else:
            Kd = self.K_seq_diag(X2s)
            if self.normalization:
                ds2 = np.sqrt(Kd + self.jitter)
                Kxx2 = Kxx2 / ds2[:, None, :]
                Kd = np.tile(sv[:, None], (1, N2))
            else:
                Kd = Kd * sv[:, None]
            out = (Kxx * sv[:, None, None], Kxx2 * sv[:, None, None], Kd)
        if return_levels:
            return out
        return tuple(o.sum(0) for o in out)

    # -- VOSF helpers (kernels.py:800-940)
    def mahalanobis_raw(self, Z, Xs):
        """kernels.py:800-822 (linear embedding).  Z (LT,T,D), Xs (N,L,D) -> (M+1, N, T)."""
        Zc = np.concatenate([Z, np.ones_like(Z)], axis=1)        # (LT, 2T, D)
        # M[n,p,r,t,q] = sum_d x[n,p,d] * Zc[r,t,d] * x[n,q,d]
        M = np.einsum("npd,rtd,nqd->nprtq", Xs, Zc, Xs)
        return sigalgs.signature_kern_rescaled_higher_order(M, self.num_levels)

    def Mahalanobis_term_approx_posterior(self, Z, X):
        """kernels.py:876-895."""
        Xs = self._prep(X)
        K = self.mahalanobis_raw(Z[1:], Xs) * self.sigma
        return np.sum(K, axis=0) + 1.0 - Z[0, :, 0][None, :]

    def norms_tens(self, Z):
        """kernels.py:897-906."""
        M = np.sum(Z[1:] ** 2, axis=2)
        return np.sum(sigalgs.tensor_inner_product(M, self.num_levels), axis=0) - 1.0 + Z[0, :, 0] ** 2

    def logs_tens(self, Z):
        """kernels.py:908-917."""
        M = np.sum(np.log(Z[1:]), axis=2)
        return np.sum(sigalgs.tensor_logs(M, self.num_levels, Z.shape[2]), axis=0) + np.log(Z[0, :, 0])

    def inner_product_tens_vs_seq(self, Z, X):
        """kernels.py:919-940 (linear inner product, order = num_levels)."""
        Xs = self._prep(X)
        Zi = Z[1:]
        LT, T, D = Zi.shape
        N, L = Xs.shape[0], Xs.shape[1]
        M = (Zi.reshape(T * LT, D) @ Xs.reshape(N * L, D).T).reshape(LT, T, N, L)
        K = sigalgs.signature_kern_tens_vs_seq_higher_order(M, self.num_levels, order=self.num_levels, difference=True)
        K = K * np.sqrt(self.sigma)
        return np.sum(K, axis=0) + np.sqrt(self.sigma) * (Z[0, :, 0][:, None] - 1.0)
