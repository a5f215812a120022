"""CPU oracle: float64 NumPy restatement of the reference's signature-kernel algorithms.

TEST INFRASTRUCTURE ONLY.  Nothing in `gpsig_amd/` imports this module; only
`tests/`, `__graft_entry__.smoke()` and the `cpu_baseline` leg of `bench.py`
may use it, and only as the checker / the CPU baseline -- never as the thing
measured or shipped.

What it restates (file:line relative to /root/reference):
  * signature_kern_first_order          gpsig/signature_algs.py:8-35
  * signature_kern_higher_order         gpsig/signature_algs.py:37-74
  * tensor_kern                         gpsig/signature_algs.py:76-99
  * signature_kern_tens_vs_seq_first_order   gpsig/signature_algs.py:101-127
  * signature_kern_tens_vs_seq_higher_order  gpsig/signature_algs.py:129-160
  * signature_kern_rescaled_higher_order     gpsig/signature_algs_vosf.py:11-48
  * tensor_inner_product / tensor_logs       gpsig/signature_algs_vosf.py:51-100

The reference runs these as TF-1.15 graph ops in float64; TF is not importable
in this container (see DESIGN.md "Oracle"), so this restatement follows the
formulas and slicing line by line with the same dataflow (materialised base
kernel tensor, exclusive cumsums, level stacking).  TF's
``tf.cumsum(exclusive=True)`` is restated as a shifted cumsum (``_xcumsum``),
not ``cumsum - x``, so the summation order matches.

Pinning: for ``order == num_levels`` and the linear base kernel, the
higher-order recursion equals the exact truncated-signature inner product; the
tests pin that against ``oracle/chen.py`` (Chen-identity signatures, the
esig-equivalent used by reference notebooks/signature_kernel.ipynb:52-140).
"""
from __future__ import annotations

import numpy as np


def _xcumsum(a: np.ndarray, axis: int) -> np.ndarray:
    """tf.cumsum(a, exclusive=True, axis=axis): [0, a0, a0+a1, ...]."""
    c = np.cumsum(a, axis=axis)
    out = np.zeros_like(c)
    src = [slice(None)] * a.ndim
    dst = [slice(None)] * a.ndim
    src[axis] = slice(0, -1)
    dst[axis] = slice(1, None)
    out[tuple(dst)] = c[tuple(src)]
    return out


def _second_difference(M: np.ndarray) -> np.ndarray:
    """signature_algs.py:26  M[:,1:,...,1:] + M[:,:-1,...,:-1] - M[:,:-1,...,1:] - M[:,1:,...,:-1]."""
    return (M[:, 1:, ..., 1:] + M[:, :-1, ..., :-1]) - M[:, :-1, ..., 1:] - M[:, 1:, ..., :-1]


def signature_kern_first_order(M: np.ndarray, num_levels: int, difference: bool = True) -> np.ndarray:
    """signature_algs.py:8-35.  M: (n1,l1,n2,l2) or (n,l,l) -> (num_levels+1, n1, n2) or (num_levels+1, n)."""
    if M.ndim == 4:
        K = [np.ones((M.shape[0], M.shape[2]))]
    else:
        K = [np.ones((M.shape[0],))]
    if difference:
        M = _second_difference(M)
    K.append(np.sum(M, axis=(1, -1)))
    R = M
    for _ in range(2, num_levels + 1):
        R = M * _xcumsum(_xcumsum(R, axis=1), axis=-1)
        K.append(np.sum(R, axis=(1, -1)))
    return np.stack(K, axis=0)


def signature_kern_higher_order(M: np.ndarray, num_levels: int, order: int = 2, difference: bool = True) -> np.ndarray:
    """signature_algs.py:37-74 (d = min(i, order) block recursion with 1/j, 1/(jk) weights)."""
    if M.ndim == 4:
        K = [np.ones((M.shape[0], M.shape[2]))]
    else:
        K = [np.ones((M.shape[0],))]
    if difference:
        M = _second_difference(M)
    K.append(np.sum(M, axis=(1, -1)))
    R = [[M]]
    for i in range(2, num_levels + 1):
        d = min(i, order)
        Rn = [[None] * d for _ in range(d)]
        tot = sum(x for row in R for x in row)
        Rn[0][0] = M * _xcumsum(_xcumsum(tot, axis=1), axis=-1)
        for j in range(2, d + 1):
            col = sum(R[a][j - 2] for a in range(len(R)))
            row = sum(R[j - 2][b] for b in range(len(R)))
            Rn[0][j - 1] = 1.0 / j * M * _xcumsum(col, axis=1)
            Rn[j - 1][0] = 1.0 / j * M * _xcumsum(row, axis=-1)
            for k in range(2, d + 1):
                Rn[j - 1][k - 1] = 1.0 / (j * k) * M * R[j - 2][k - 2]
        K.append(np.sum(sum(x for row in Rn for x in row), axis=(1, -1)))
        R = Rn
    return np.stack(K, axis=0)


def tensor_kern(M: np.ndarray, num_levels: int) -> np.ndarray:
    """signature_algs.py:76-99.  M: (LT, T1, T2) -> (num_levels+1, T1, T2)."""
    K = [np.ones((M.shape[1], M.shape[2]))]
    k = 0
    for i in range(1, num_levels + 1):
        R = M[k]
        k += 1
        for _ in range(1, i):
            R = M[k] * R
            k += 1
        K.append(R)
    return np.stack(K, axis=0)


def signature_kern_tens_vs_seq_first_order(M: np.ndarray, num_levels: int, difference: bool = True) -> np.ndarray:
    """signature_algs.py:101-127.  M: (LT, T, N, L) -> (num_levels+1, T, N)."""
    if difference:
        M = M[..., 1:] - M[..., :-1]
    K = [np.ones((M.shape[1], M.shape[2]))]
    k = 0
    for i in range(1, num_levels + 1):
        R = M[k]
        k += 1
        for _ in range(1, i):
            R = M[k] * _xcumsum(R, axis=2)
            k += 1
        K.append(np.sum(R, axis=2))
    return np.stack(K, axis=0)


def signature_kern_tens_vs_seq_higher_order(M: np.ndarray, num_levels: int, order: int = 2, difference: bool = True) -> np.ndarray:
    """signature_algs.py:129-160."""
    if difference:
        M = M[..., 1:] - M[..., :-1]
    K = [np.ones((M.shape[1], M.shape[2]))]
    k = 0
    for i in range(1, num_levels + 1):
        R = [M[k]]
        k += 1
        for j in range(1, i):
            d = min(j + 1, order)
            Rn = [None] * d
            Rn[0] = M[k] * _xcumsum(sum(R), axis=2)
            for l in range(1, d):
                Rn[l] = 1.0 / (l + 1) * M[k] * R[l - 1]
            R = Rn
            k += 1
        K.append(np.sum(sum(R), axis=2))
    return np.stack(K, axis=0)


def signature_kern_rescaled_higher_order(M: np.ndarray, num_levels: int) -> np.ndarray:
    """signature_algs_vosf.py:11-48.

    M: (N, L, LT, 2T, L) -> (num_levels+1, N, T) after ``-first half + second half``.
    """
    num_tensors = M.shape[3]
    K = [np.ones((M.shape[0], num_tensors))]
    M = _second_difference(M)
    r = 0
    for i in range(1, num_levels + 1):
        R = [[M[:, :, r, :, :]]]
        r += 1
        for j in range(1, i):
            d = min(j + 1, num_levels)
            Mr = M[:, :, r, :, :]
            Rn = [[None] * d for _ in range(d)]
            tot = sum(x for row in R for x in row)
            Rn[0][0] = Mr * _xcumsum(_xcumsum(tot, axis=1), axis=-1)
            for l in range(1, d):
                col = sum(R[a][l - 1] for a in range(len(R)))
                row = sum(R[l - 1][b] for b in range(len(R)))
                Rn[0][l] = 1.0 / (l + 1) * Mr * _xcumsum(col, axis=1)
                Rn[l][0] = 1.0 / (l + 1) * Mr * _xcumsum(row, axis=-1)
                for k in range(1, d):
                    Rn[l][k] = 1.0 / ((l + 1) * (k + 1)) * Mr * R[l - 1][k - 1]
            R = Rn
            r += 1
        K.append(np.sum(sum(x for row in R for x in row), axis=(1, -1)))
    K = [-e[:, : num_tensors // 2] + e[:, num_tensors // 2:] for e in K]
    return np.stack(K, axis=0)


def tensor_inner_product(M: np.ndarray, num_levels: int) -> np.ndarray:
    """signature_algs_vosf.py:51-74.  M: (LT, T) -> (num_levels+1, T)."""
    K = [np.ones(M.shape[1])]
    k = 0
    for i in range(1, num_levels + 1):
        R = M[k]
        k += 1
        for _ in range(1, i):
            R = M[k] * R
            k += 1
        K.append(R)
    return np.stack(K, axis=0)


def tensor_logs(M: np.ndarray, num_levels: int, d: int) -> np.ndarray:
    """signature_algs_vosf.py:76-100.  M: (LT, T) -> (num_levels+1, T)."""
    K = [np.zeros(M.shape[1])]
    k = 0
    for i in range(1, num_levels + 1):
        R = M[k]
        k += 1
        for _ in range(1, i):
            R = M[k] + R
            k += 1
        K.append(float(d) ** (i - 1) * R)
    return np.stack(K, axis=0)
