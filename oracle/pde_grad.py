"""CPU oracle for the PDE-kernel gradient: NumPy restatement of the reference's adjoint formula.

TEST INFRASTRUCTURE ONLY (see oracle/sigalgs.py header).

The reference differentiates the Goursat-PDE kernel with a hand-written gradient
(gpsig/kernels_pde.py:465-509, _KdiagGrad; same formula in
gpsig/covariance_op/_untrunc_cov_grad.py:25-77) over the grids K and K_rev that
sig_kern_diag (gpsig/sigKer_fast.pyx:15-62) returns:

  K, K_rev symmetrised (only the lower triangle is computed)              kernels_pde.py:481-486
  inc_X = repeat((X[:,1:]-X[:,:-1]) / 2^n, 2^n)                           :489-490
  K_rev_rev = K_rev flipped in both axes                                  :493-494
  KK = K[:, :-1, :-1] * K_rev_rev[:, 1:, 1:]                              :496
  K_grad = 2^-n sum_t KK[s, t] inc_X[t], summed over each coarse row      :498-504
  grad_points = -2 [K_grad, 0] + 2 [0, K_grad]                            :508
  (times the upstream gradient of K[:, -1, -1])                           :510

kdiag_grad() restates exactly that from the grids (pinned: the grids of tests/golden/pde.npz are
the reference's own sig_kern_diag outputs).  pair_grids()/pair_grad() extend the same adjoint to a
cross pair (x, y) -- the reference has no cross-Gram PDE gradient, so that case is "parity
unpinned" beyond its consistency with kdiag_grad() for y = x (tests/test_pde_grad.py).
"""
from __future__ import annotations

import numpy as np


def kdiag_grad(X, K, K_rev, n):
    """_KdiagGrad (kernels_pde.py:465-509) for unit upstream gradient: X (A, L, D) -> (A, L, D)."""
    X = np.asarray(X, dtype=np.float64)
    A, L, D = X.shape
    c = 2 ** n
    K = K + np.transpose(K, (0, 2, 1)) - np.einsum("aii->ai", K)[:, :, None] * np.eye(K.shape[1])[None]
    K_rev = K_rev + np.transpose(K_rev, (0, 2, 1)) - np.einsum("aii->ai", K_rev)[:, :, None] * np.eye(K.shape[1])[None]
    inc = np.repeat((X[:, 1:, :] - X[:, :-1, :]) / c, c, axis=1)
    Krr = K_rev[:, ::-1, ::-1]
    KK = K[:, :-1, :-1] * Krr[:, 1:, 1:]
    Kg = np.einsum("ast,atd->asd", KK, inc) / c
    Kg = Kg.reshape(A, L - 1, c, D).sum(2)
    z = np.zeros((A, 1, D))
    return -2.0 * np.concatenate([Kg, z], 1) + 2.0 * np.concatenate([z, Kg], 1)


def pair_grids(x, y, n, solver=1, rev_solver=0):
    """Full (I+1) x (J+1) grids K (scheme `solver`) on (x, y) and K_rev (scheme `rev_solver`) on the
    time-reversed paths; the update rules of sigKer_fast.pyx:5-10 / :46-48."""
    x = np.asarray(x, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    c = 2 ** n
    dx, dy = np.diff(x, axis=0), np.diff(y, axis=0)
    I, J = c * len(dx), c * len(dy)

    def solve(ix, iy, sch):
        G = np.ones((I + 1, J + 1))
        for i in range(I):
            for j in range(J):
                inc = float(ix[i // c] @ iy[j // c]) / (c * c)
                if sch == 1:
                    G[i + 1, j + 1] = (G[i, j + 1] + G[i + 1, j]) * (1 + 0.5 * inc + inc * inc / 12) \
                        - G[i, j] * (1 - inc * inc / 12)
                else:
                    G[i + 1, j + 1] = G[i, j + 1] + G[i + 1, j] + G[i, j] * (inc - 1)
        return G

    return solve(dx, dy, solver), solve(-dx[::-1], -dy[::-1], rev_solver)


def pair_grad(x, y, n, solver=1):
    """The same adjoint for a cross pair: (dK/dx (Lx, D), dK/dy (Ly, D)) of K[-1, -1]."""
    x = np.asarray(x, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    c = 2 ** n
    K, Kr = pair_grids(x, y, n, solver)
    KK = K[:-1, :-1] * Kr[::-1, ::-1][1:, 1:]
    incx = np.repeat(np.diff(x, axis=0), c, axis=0)
    incy = np.repeat(np.diff(y, axis=0), c, axis=0)
    Gx = (KK @ incy).reshape(-1, c, x.shape[1]).sum(1) / (c * c)
    Gy = (KK.T @ incx).reshape(-1, c, y.shape[1]).sum(1) / (c * c)
    zx, zy = np.zeros((1, x.shape[1])), np.zeros((1, y.shape[1]))
    gx = np.concatenate([zx, Gx], 0) - np.concatenate([Gx, zx], 0)
    gy = np.concatenate([zy, Gy], 0) - np.concatenate([Gy, zy], 0)
    return gx, gy
