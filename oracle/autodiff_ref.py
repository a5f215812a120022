"""CPU oracle for GRADIENTS: float64 torch restatement of the reference graph, differentiated by
torch.autograd the way the reference is differentiated by TF autodiff.

TEST INFRASTRUCTURE ONLY (see oracle/sigalgs.py header): only tests/ may import it, as the checker
of gpsig_sig_gram_vjp / gpsig_amd.autograd.

The reference has no hand-written gradient for the truncated signature kernel: SVGP training
differentiates K through TF-1.15 autodiff of the graph (file:line relative to /root/reference)

  * base kernels                 gpsig/kernels.py:946-957 (_square_dist), :979-986 (_lin), :1042-1044 (_rbf)
  * second difference + recursion gpsig/signature_algs.py:8-35 (signature_kern_first_order),
                                 :37-74 (signature_kern_higher_order)
  * scaling                      gpsig/kernels.py:344-365 (X / lengthscales; num_lags=0)
  * K: jitter, normalisation by sqrt(diag), sigma*variances, level sum   gpsig/kernels.py:402-477
  * Kdiag (unnormalised)         gpsig/kernels.py:510-541

restated here op for op on torch float64 tensors (materialised base-kernel tensor, exclusive cumsums
as shifted cumsums, diag of the Gram for K(X)).  Reverse-mode autodiff of the same function in fp64
is the reference's gradient up to fp64 rounding.  Pinning: the forward values equal oracle/sigalgs.py
/ oracle/kernels_ref.py (the pinned NumPy restatement) and the gradients equal central finite
differences of that NumPy oracle (tests/test_oracle.py).
"""
from __future__ import annotations

import torch


def _xcumsum(a: torch.Tensor, dim: int) -> torch.Tensor:
    """tf.cumsum(a, exclusive=True, axis=dim)."""
    c = torch.cumsum(a, dim)
    z = torch.zeros_like(c.narrow(dim, 0, 1))
    return torch.cat([z, c.narrow(dim, 0, c.shape[dim] - 1)], dim)


def square_dist(X, X2):
    """kernels.py:946-957: |x|^2 + |y|^2 - 2 x.y."""
    Xs = (X ** 2).sum(-1)
    X2s = (X2 ** 2).sum(-1)
    return -2.0 * X @ X2.T + Xs[:, None] + X2s[None, :]


def base_kern(X, X2, base):
    if base == "rbf":
        return torch.exp(-square_dist(X, X2) / 2.0)  # kernels.py:1042-1044
    return X @ X2.T  # kernels.py:979-986


def first_order(M: torch.Tensor, num_levels: int, difference: bool = True) -> torch.Tensor:
    """signature_algs.py:8-35 on a 4-D (n1, l1, n2, l2) tensor -> (num_levels+1, n1, n2)."""
    K = [torch.ones((M.shape[0], M.shape[2]), dtype=M.dtype)]
    if difference:
        M = M[:, 1:, :, 1:] + M[:, :-1, :, :-1] - M[:, :-1, :, 1:] - M[:, 1:, :, :-1]
    K.append(M.sum(dim=(1, -1)))
    R = M
    for _ in range(2, num_levels + 1):
        R = M * _xcumsum(_xcumsum(R, 1), -1)
        K.append(R.sum(dim=(1, -1)))
    return torch.stack(K, 0)


def higher_order(M: torch.Tensor, num_levels: int, order: int, difference: bool = True) -> torch.Tensor:
    """signature_algs.py:37-74 on a 4-D (n1, l1, n2, l2) tensor -> (num_levels+1, n1, n2): the d x d
    array of tensors R with the 1/j, 1/(jk) corrections, cumsums over axis 1 (x time) and -1 (y time)."""
    K = [torch.ones((M.shape[0], M.shape[2]), dtype=M.dtype)]
    if difference:
        M = M[:, 1:, :, 1:] + M[:, :-1, :, :-1] - M[:, :-1, :, 1:] - M[:, 1:, :, :-1]
    K.append(M.sum(dim=(1, -1)))
    R = [[M]]
    for i in range(2, num_levels + 1):
        d = min(i, order)
        Rn = [[None] * d for _ in range(d)]
        Rn[0][0] = M * _xcumsum(_xcumsum(sum(r for row in R for r in row), 1), -1)
        for j in range(2, d + 1):
            Rn[0][j - 1] = M * _xcumsum(sum(R[a][j - 2] for a in range(len(R))), 1) / j
            Rn[j - 1][0] = M * _xcumsum(sum(R[j - 2][b] for b in range(len(R))), -1) / j
            for k in range(2, d + 1):
                Rn[j - 1][k - 1] = M * R[j - 2][k - 2] / (j * k)
        K.append(sum(r for row in Rn for r in row).sum(dim=(1, -1)))
        R = Rn
    return torch.stack(K, 0)


def _recursion(M, num_levels, difference, order):
    return first_order(M, num_levels, difference) if order == 1 else higher_order(M, num_levels, order, difference)


def k_seq(Xs, X2s, num_levels, base="rbf", difference=True, order=1):
    """_K_seq (kernels.py:209-238): Xs (n1,l1,d), X2s (n2,l2,d) or None."""
    n1, l1, d = Xs.shape
    Y = Xs if X2s is None else X2s
    n2, l2, _ = Y.shape
    M = base_kern(Xs.reshape(n1 * l1, d), Y.reshape(n2 * l2, d), base).reshape(n1, l1, n2, l2)
    return _recursion(M, num_levels, difference, order)


def k_seq_diag(Xs, num_levels, base="rbf", difference=True, order=1):
    """_K_seq_diag (kernels.py:190-207): per-sequence (n, l, l) base kernel -> (num_levels+1, n)."""
    n, l, d = Xs.shape
    Ms = torch.stack([base_kern(Xs[a], Xs[a], base) for a in range(n)], 0)  # (n, l, l)
    M = Ms[:, :, None, :]  # run the 3-D branch as a (n, l, 1, l) tensor
    K = _recursion(M, num_levels, difference, order)  # (M+1, n, 1)
    return K[:, :, 0]


def K(Xs, X2s, num_levels, base="rbf", normalization=True, scale=None, jitter=1e-6, return_levels=False,
      difference=True, order=1):
    """SignatureKernel.K (kernels.py:402-477) on scaled sequences; scale = sigma * variances (M+1)."""
    K_l = k_seq(Xs, X2s, num_levels, base, difference, order)
    if normalization:
        if X2s is None:
            n = Xs.shape[0]
            K_l = K_l + jitter * torch.eye(n, dtype=K_l.dtype)[None]
            dsq = torch.sqrt(torch.diagonal(K_l, dim1=1, dim2=2))
            K_l = K_l / (dsq[:, :, None] * dsq[:, None, :])
        else:
            d1 = torch.sqrt(k_seq_diag(Xs, num_levels, base, difference, order) + jitter)
            d2 = torch.sqrt(k_seq_diag(X2s, num_levels, base, difference, order) + jitter)
            K_l = K_l / (d1[:, :, None] * d2[:, None, :])
    if scale is None:
        scale = torch.ones(num_levels + 1, dtype=K_l.dtype)
    K_l = K_l * scale[:, None, None]
    return K_l if return_levels else K_l.sum(0)


def tens_vs_seq_first_order(M: torch.Tensor, num_levels: int, difference: bool = True) -> torch.Tensor:
    """signature_algs.py:101-127: M (LT, T, N, L) -> (num_levels+1, T, N)."""
    if difference:
        M = M[..., 1:] - M[..., :-1]
    K = [torch.ones((M.shape[1], M.shape[2]), dtype=M.dtype)]
    k = 0
    for i in range(1, num_levels + 1):
        R = M[k]
        k += 1
        for _ in range(1, i):
            R = M[k] * _xcumsum(R, 2)
            k += 1
        K.append(R.sum(2))
    return torch.stack(K, 0)


def k_tens_vs_seq(Zs, Xs, num_levels, base="rbf", increments=False, difference=True):
    """_K_tens_vs_seq (kernels.py:314-341): Zs (LT,T,d) or (LT,T,2,d), Xs (N,L,d) -> (M+1, T, N) raw."""
    LT, T, d = Zs.shape[0], Zs.shape[1], Zs.shape[-1]
    N, L = Xs.shape[0], Xs.shape[1]
    Xf = Xs.reshape(N * L, d)
    if increments:
        M = base_kern(Zs.reshape(2 * T * LT, d), Xf, base).reshape(LT, T, 2, N, L)
        M = M[:, :, 1] - M[:, :, 0]
    else:
        M = base_kern(Zs.reshape(T * LT, d), Xf, base).reshape(LT, T, N, L)
    return tens_vs_seq_first_order(M, num_levels, difference)


def K_tens_vs_seq(Zs, Xs, num_levels, base="rbf", increments=False, normalization=True, scale=None, jitter=1e-6,
                  return_levels=False, difference=True):
    """SignatureKernel.K_tens_vs_seq (kernels.py:571-620) on scaled tensors / sequences."""
    Kzx = k_tens_vs_seq(Zs, Xs, num_levels, base, increments, difference)
    if normalization:
        Kzx = Kzx / torch.sqrt(k_seq_diag(Xs, num_levels, base, difference) + jitter)[:, None, :]
    if scale is None:
        scale = torch.ones(num_levels + 1, dtype=Kzx.dtype)
    Kzx = Kzx * scale[:, None, None]
    return Kzx if return_levels else Kzx.sum(0)


def k_tens(Zs, num_levels, base="rbf", increments=False):
    """_K_tens (kernels.py:264-284) + tensor_kern (signature_algs.py:76-99): (M+1, T, T) raw."""
    LT, T, d = Zs.shape[0], Zs.shape[1], Zs.shape[-1]
    if increments:
        Zr = Zs.reshape(LT, 2 * T, d)
        M = torch.stack([base_kern(Zr[c], Zr[c], base) for c in range(LT)], 0).reshape(LT, T, 2, T, 2)
        M = M[:, :, 1, :, 1] + M[:, :, 0, :, 0] - M[:, :, 1, :, 0] - M[:, :, 0, :, 1]
    else:
        M = torch.stack([base_kern(Zs[c], Zs[c], base) for c in range(LT)], 0)
    K = [torch.ones((T, T), dtype=Zs.dtype)]
    k = 0
    for i in range(1, num_levels + 1):
        R = M[k]
        k += 1
        for _ in range(1, i):
            R = M[k] * R
            k += 1
        K.append(R)
    return torch.stack(K, 0)


def signature(x: torch.Tensor, depth: int) -> torch.Tensor:
    """Truncated signature of one path x (L, D) (Chen's identity, oracle/chen.py's definition) as a
    differentiable torch fp64 function: levels 1..depth flattened first-index-major, concatenated --
    the object iisignature.sig returns (iisignature_tensorflow.py:87)."""
    D = x.shape[1]
    S = [torch.ones(1, dtype=x.dtype)] + [torch.zeros(D ** m, dtype=x.dtype) for m in range(1, depth + 1)]
    for k in range(x.shape[0] - 1):
        v = x[k + 1] - x[k]
        E = [torch.ones(1, dtype=x.dtype)]
        for m in range(1, depth + 1):
            E.append(torch.outer(E[-1], v).reshape(-1) / m)
        S = [sum(torch.outer(S[j], E[m - j]).reshape(-1) for j in range(m + 1)) for m in range(depth + 1)]
    return torch.cat(S[1:])
