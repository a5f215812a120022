"""GPU parity at wide channel counts (runtime channel loop, gpsig_amd/csrc/wide.h) vs the float64 oracle.

The reference places no bound on the channel count: _square_dist is one tf.matmul over D
(/root/reference/gpsig/kernels.py:946-957).  Its own training runners feed (D + 1) * 2 channels after
add_time and num_lags=1 (benchmarks/run_gpsig_benchmarks.py:32, train_gpsig.py:29): 26 (JapaneseVowels),
46 (AUSLAN), 126 (CMUsubject16 / KickvsPunch / WalkvsRun) and more.  Criterion as tests/test_gram_gpu.py:
norm-relative max|K32 - K64| <= 1e-5 * max|K64| per level.
"""
import numpy as np
import pytest
import torch

from conftest import norm_rel_err
from oracle import kernels_ref as kr

pytestmark = pytest.mark.gpu
TOL = 1e-5
DEV = "cuda"


def t(x):
    return torch.as_tensor(np.asarray(x), device=DEV)


def walks(rng, n, L, D, scale=1.0):
    return np.cumsum(rng.standard_normal((n, L, D)), 1) * scale / np.sqrt(L * D)


@pytest.mark.parametrize("D,L", [(33, 20), (46, 136), (126, 136), (46, 500), (126, 64), (200, 30)])
def test_wide_rbf_gram_and_diag(D, L):
    """K(X), K(X, X2) (raw levels) and the diagonal at the reference runners' channel counts; L = 500 runs in
    column blocks (max_len 500 of benchmarks/run_gpsig_benchmarks.py)."""
    from gpsig_amd import ops
    rng = np.random.default_rng(D * 1000 + L)
    M = 4
    X = walks(rng, 5, L, D)
    Y = walks(rng, 3, max(L - 7, 2), D)
    ref = kr.SignatureKernelRef(L * D, D, M, normalization=False)
    got = ops.sig_gram(t(X), t(Y), M).cpu().numpy()
    err = norm_rel_err(got[1:], ref.K_seq(X, Y)[1:], axis_levels=True)
    assert (err < TOL).all(), err
    sym = ops.sig_gram(t(X), None, M).cpu().numpy()
    err = norm_rel_err(sym[1:], ref.K_seq(X)[1:], axis_levels=True)
    assert (err < TOL).all(), err
    dg = ops.sig_diag(t(X), M).cpu().numpy()
    err = norm_rel_err(dg[1:], ref.K_seq_diag(X)[1:], axis_levels=True)
    assert (err < TOL).all(), err


@pytest.mark.parametrize("D", [46, 126])
def test_wide_normalised_K_and_Kdiag(D):
    """The full SignatureRBF K / Kdiag orchestration (scaling, jitter, normalisation, sigma * variances,
    level sum; kernels.py:402-541) at wide channel counts, with lengthscales."""
    import gpsig_amd
    rng = np.random.default_rng(D)
    N, L, M = 7, 40, 5
    X = walks(rng, N, L, D, 3.0)
    X2 = walks(rng, 4, L, D, 3.0)
    ls = rng.uniform(0.5, 2.0, D)
    k = gpsig_amd.SignatureRBF(L * D, D, M, lengthscales=ls)
    ref = kr.SignatureKernelRef(L * D, D, M, lengthscales=ls)
    K = k.K(t(X.reshape(N, -1))).cpu().numpy()
    assert norm_rel_err(K, ref.K(X.reshape(N, -1))) < TOL
    Kc = k.K(t(X.reshape(N, -1)), t(X2.reshape(4, -1)), return_levels=True).cpu().numpy()
    exp = ref.K(X.reshape(N, -1), X2.reshape(4, -1), return_levels=True)
    assert (norm_rel_err(Kc, exp, axis_levels=True) < TOL).all()
    ku = gpsig_amd.SignatureRBF(L * D, D, M, lengthscales=ls, normalization=False)
    refu = kr.SignatureKernelRef(L * D, D, M, lengthscales=ls, normalization=False)
    assert norm_rel_err(ku.Kdiag(t(X.reshape(N, -1))).cpu().numpy(), refu.Kdiag(X.reshape(N, -1))) < TOL


@pytest.mark.parametrize("base,difference", [("linear", True), ("linear", False), ("rbf", False)])
def test_wide_other_seeds(base, difference):
    from gpsig_amd import ops
    rng = np.random.default_rng(7)
    D, L, M = 46, 70, 3
    X = walks(rng, 4, L, D)
    Y = walks(rng, 3, L + 5, D)
    ref = kr.SignatureKernelRef(L * D, D, M, normalization=False, difference=difference,
                                base="linear" if base == "linear" else "rbf")
    got = ops.sig_gram(t(X), t(Y), M, base=base, difference=difference).cpu().numpy()
    err = norm_rel_err(got[1:], ref.K_seq(X, Y)[1:], axis_levels=True)
    assert (err < TOL).all(), err
    sym = ops.sig_gram(t(X), None, M, base=base, difference=difference).cpu().numpy()
    assert (norm_rel_err(sym[1:], ref.K_seq(X)[1:], axis_levels=True) < TOL).all()


@pytest.mark.parametrize("scale,jumps", [(0.02, False), (0.2, False), (0.05, True)])
def test_wide_seed_regimes(scale, jumps):
    """The wide RBF seed's regimes (the cubic expm1(c) under the |dx||dy| bound, the quintic, and slow rows
    with large jumps: corner differences and re-evaluated chained expm1(p)), D = 46."""
    import gpsig_amd
    rng = np.random.default_rng(12)
    N, L, D, M = 10, 45, 46, 4
    inc = rng.standard_normal((N, L, D)) * scale / np.sqrt(D)
    if jumps:
        inc[:, ::9, :] *= 25.0
    X = np.cumsum(inc, 1)
    k = gpsig_amd.SignatureRBF(L * D, D, M)
    got = k.K(t(X.reshape(N, -1)), return_levels=True).cpu().numpy()
    exp = kr.SignatureKernelRef(L * D, D, M).K(X.reshape(N, -1), return_levels=True)
    assert (norm_rel_err(got, exp, axis_levels=True) < TOL).all()
