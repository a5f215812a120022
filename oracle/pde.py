"""ctypes front-end of the C PDE oracle (oracle/pde/sigpde_oracle.c).

TEST INFRASTRUCTURE ONLY (see oracle/sigalgs.py header).  Builds with gcc on
first use if the shared object is missing (the build is also driven by
__graft_entry__.build()).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SRC = os.path.join(_HERE, "pde", "sigpde_oracle.c")
_SO = os.path.join(_HERE, "_build", "libsigpde_oracle.so")
_lib = None


def build(force: bool = False) -> str:
    os.makedirs(os.path.dirname(_SO), exist_ok=True)
    if force or not os.path.exists(_SO) or os.path.getmtime(_SO) < os.path.getmtime(_SRC):
        subprocess.check_call(["gcc", "-O2", "-fopenmp", "-fPIC", "-shared", "-ffp-contract=off",
                               _SRC, "-o", _SO, "-lm"])
    return _SO


def _load():
    global _lib
    if _lib is None:
        _lib = ctypes.CDLL(build())
        dp, i = ctypes.POINTER(ctypes.c_double), ctypes.c_int
        _lib.sigpde_pair.restype = ctypes.c_double
        _lib.sigpde_pair.argtypes = [dp, i, dp, i, i, i, i, i, i, dp]
        _lib.sigpde_gram.argtypes = [dp, i, i, dp, i, i, i, i, i, i, dp]
        _lib.sigpde_diag.argtypes = [dp, i, i, i, i, i, dp]
        _lib.sigpde_diag_grids.argtypes = [dp, i, i, i, i, i, dp, dp]
        _lib.sigpde_gram_grad.argtypes = [dp, i, i, dp, i, i, i, i, i, dp, dp, dp]
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def pde_gram(X, Y=None, dyadic=0, solver=1):
    """Final-corner PDE Gram.  X (n1,l1,d), Y (n2,l2,d) or None (symmetric)."""
    lib = _load()
    X = np.ascontiguousarray(X, dtype=np.float64)
    sym = Y is None
    Y = X if sym else np.ascontiguousarray(Y, dtype=np.float64)
    out = np.zeros((X.shape[0], Y.shape[0]))
    lib.sigpde_gram(_p(X), X.shape[0], X.shape[1], _p(Y), Y.shape[0], Y.shape[1], X.shape[2],
                    dyadic, solver, int(sym), _p(out))
    return out


def pde_diag(X, dyadic=0, solver=1):
    lib = _load()
    X = np.ascontiguousarray(X, dtype=np.float64)
    out = np.zeros(X.shape[0])
    lib.sigpde_diag(_p(X), X.shape[0], X.shape[1], X.shape[2], dyadic, solver, _p(out))
    return out


def pde_diag_grids(X, dyadic=0, solver=1):
    """Restatement of sig_kern_diag(x, n, solver) -> (K, K_rev) full grids."""
    lib = _load()
    X = np.ascontiguousarray(X, dtype=np.float64)
    A, L, D = X.shape
    G = (1 << dyadic) * (L - 1) + 1
    K = np.zeros((A, G, G))
    Kr = np.zeros((A, G, G))
    lib.sigpde_diag_grids(_p(X), A, L, D, dyadic, solver, _p(K), _p(Kr))
    return K, Kr


def pde_gram_grad(X, Y, W, dyadic=0, solver=1):
    """sum_ab W[a, b] (dK(x_a, y_b)/dX, dK/dY) by the reference's adjoint (oracle/pde_grad.py pair_grad, in C):
    X (n1,l1,d), Y (n2,l2,d), W (n1,n2) -> (gX, gY)."""
    lib = _load()
    X = np.ascontiguousarray(X, dtype=np.float64)
    Y = np.ascontiguousarray(Y, dtype=np.float64)
    W = np.ascontiguousarray(W, dtype=np.float64)
    gX, gY = np.zeros_like(X), np.zeros_like(Y)
    lib.sigpde_gram_grad(_p(X), X.shape[0], X.shape[1], _p(Y), Y.shape[0], Y.shape[1], X.shape[2], dyadic, solver,
                         _p(W), _p(gX), _p(gY))
    return gX, gY
