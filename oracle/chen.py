"""CPU oracle: exact truncated signatures of piecewise-linear paths (Chen identity).

TEST INFRASTRUCTURE ONLY (see oracle/sigalgs.py header).

The reference validates its kernels against ``esig.tosig.stream2sig``
(reference notebooks/signature_kernel.ipynb:52-140, Inf-norm 2.24e-8 for the
Gram, 1.30e-10 tensor-vs-seq, 1.66e-12 tensor-vs-tensor).  esig / iisignature
(requirements.txt:11) are not installable offline, so this module computes the
same object from its definition: for a path with increments v_1..v_{L-1},
S(x) = exp(v_1) (x) exp(v_2) (x) ... (x) exp(v_{L-1}) in the truncated tensor
algebra, exp(v)_m = v^{(x)m} / m!.  Levels are flattened first-index-major,
matching the notebook's tensor flattening (signature_kernel.ipynb:157-167).
"""
from __future__ import annotations

import math

import numpy as np


def signature(x: np.ndarray, num_levels: int):
    """x: (L, D) -> list of level tensors, level m flattened to (D**m,)."""
    x = np.asarray(x, dtype=np.float64)
    D = x.shape[1]
    S = [np.ones(1)] + [np.zeros(D ** m) for m in range(1, num_levels + 1)]
    for v in np.diff(x, axis=0):
        # E[m] = v^{(x)m} / m!
        E = [np.ones(1)] + [_power(v, m) / math.factorial(m) for m in range(1, num_levels + 1)]
        new = []
        for m in range(num_levels + 1):
            acc = np.zeros(D ** m)
            for k in range(m + 1):
                acc += np.multiply.outer(S[k], E[m - k]).reshape(-1)
            new.append(acc)
        S = new
    return S


def _power(v, m):
    out = v.copy()
    for _ in range(1, m):
        out = np.multiply.outer(out, v).reshape(-1)
    return out


def signature_levels_kernel(X: np.ndarray, Y: np.ndarray, num_levels: int) -> np.ndarray:
    """Per-level exact signature inner products. X (N1,L,D), Y (N2,L2,D) -> (M+1, N1, N2)."""
    SX = [signature(x, num_levels) for x in X]
    SY = [signature(y, num_levels) for y in Y]
    out = np.zeros((num_levels + 1, len(SX), len(SY)))
    for m in range(num_levels + 1):
        A = np.stack([s[m] for s in SX])
        B = np.stack([s[m] for s in SY])
        out[m] = A @ B.T
    return out


def simple_tensors(Z: np.ndarray, num_levels: int) -> list:
    """Z (LT, T, D) components -> per-level flattened rank-1 tensors (signature_kernel.ipynb:157-167)."""
    T = Z.shape[1]
    tens = [np.ones((T, 1))]
    k = 0
    for m in range(1, num_levels + 1):
        Zm = Z[k]
        k += 1
        for _ in range(1, m):
            Zm = (Zm[..., None] * Z[k, :, None, :]).reshape(T, -1)
            k += 1
        tens.append(Zm)
    return tens
