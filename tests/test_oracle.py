"""CPU: the oracle against the committed golden vectors and against independent restatements."""
import numpy as np
import pytest

from conftest import golden
from oracle import chen, pde, sigalgs
from oracle import kernels_ref as kr


def test_rbf_gram_fixture_reproduced():
    g = golden("rbf_gram.npz")
    X, X2, M = g["X"], g["X2"], int(g["num_levels"])
    N, L, D = X.shape
    k = kr.SignatureKernelRef(L * D, D, M)
    np.testing.assert_allclose(k.K(X.reshape(N, -1)), g["K"], rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(k.K(X.reshape(N, -1), X2.reshape(len(X2), -1), return_levels=True),
                               g["K_cross_levels"], rtol=1e-12, atol=1e-14)


def test_linear_order_M_equals_chen_signatures():
    g = golden("linear_chen.npz")
    np.testing.assert_allclose(g["K_levels"], g["K_chen"], rtol=1e-10, atol=1e-9)
    X, M = g["X"], int(g["num_levels"])
    k = kr.SignatureKernelRef(X.shape[1] * X.shape[2], X.shape[2], M, base="linear", order=M, normalization=False)
    np.testing.assert_allclose(k.K_seq(X[:4]), chen.signature_levels_kernel(X[:4], X[:4], M), rtol=1e-10, atol=1e-9)


def test_normalised_diagonal_and_level0():
    g = golden("rbf_gram.npz")
    K = g["K_levels"]
    for m in range(K.shape[0]):
        np.testing.assert_allclose(np.diag(K[m]), 1.0, rtol=1e-12)
    off = K[0][~np.eye(K.shape[1], dtype=bool)]
    np.testing.assert_allclose(off, 1.0 / (1.0 + 1e-6), rtol=1e-12)
    np.testing.assert_allclose(g["K_cross_levels"][0], 1.0 / (1.0 + 1e-6), rtol=1e-12)
    np.testing.assert_allclose(g["Kdiag_norm"], 5.0)


def test_gram_symmetric_psd():
    g = golden("rbf_gram.npz")
    K = g["K"]
    np.testing.assert_allclose(K, K.T, rtol=0, atol=1e-12)
    assert np.linalg.eigvalsh(K).min() > -1e-8


def test_first_order_equals_higher_order_with_order1():
    rng = np.random.default_rng(11)
    X = np.cumsum(rng.standard_normal((5, 15, 2)), 1) * 0.2
    M = kr.base_rbf(X.reshape(-1, 2)).reshape(5, 15, 5, 15)
    a = sigalgs.signature_kern_first_order(M, 4)
    b = sigalgs.signature_kern_higher_order(M, 4, order=1)
    np.testing.assert_allclose(a, b, rtol=1e-12, atol=1e-15)


def test_tensor_fixtures_pinned_to_chen():
    g = golden("tensors.npz")
    Z, X, M = g["Z"], g["X"], int(g["num_levels"])
    tens = chen.simple_tensors(Z, M)
    SX = [chen.signature(x, M) for x in X]
    ref = np.stack([tens[m] @ np.stack([s[m] for s in SX]).T for m in range(M + 1)])
    np.testing.assert_allclose(g["lin_tvs_order5"], ref, rtol=1e-10, atol=1e-10)


def test_rescaled_fixture_matches_naive():
    g = golden("rescaled.npz")
    np.testing.assert_allclose(g["K_linear"], g["K_naive"], rtol=1e-10, atol=1e-10)


def test_pde_oracle_matches_reference_cython_outputs():
    """pde.npz grids are the reference's sig_kern_diag outputs (generated from its .pyx)."""
    g = golden("pde.npz")
    X = g["X"]
    for n in (0, 1):
        for solver in (0, 1):
            K, Kr = pde.pde_diag_grids(X, n, solver)
            tril = np.tril(np.ones(K.shape[1:], bool))
            np.testing.assert_array_equal(K[:, tril], g[f"grid_n{n}_s{solver}"][:, tril])
            np.testing.assert_array_equal(Kr[:, tril], g[f"gridrev_n{n}_s{solver}"][:, tril])
    for solver in (0, 1):
        np.testing.assert_array_equal(pde.pde_diag(X, 2, solver), g[f"diag_n2_s{solver}"])


def test_pde_cross_gram_symmetry_and_diag():
    g = golden("pde.npz")
    X = g["X"]
    S = pde.pde_gram(X, None, 1, 1)
    np.testing.assert_array_equal(S, S.T)
    np.testing.assert_array_equal(np.diag(S), g["diag_n1_s1"])


def test_pde_converges_to_signature_kernel():
    """Dyadic refinement approaches sum_m <S_m(x), S_m(y)> (untruncated kernel) for the linear kernel."""
    rng = np.random.default_rng(12)
    x = np.cumsum(rng.standard_normal((1, 6, 2)), 1) * 0.3
    y = np.cumsum(rng.standard_normal((1, 7, 2)), 1) * 0.3
    exact = chen.signature_levels_kernel(x, y, 8).sum()
    errs = [abs(pde.pde_gram(x, y, n, 1)[0, 0] - exact) for n in (0, 1, 2, 3)]
    assert errs[3] < errs[0] and errs[3] < 1e-4


@pytest.mark.parametrize("nl", [1, 2])
def test_lags_fixture(nl):
    g = golden("lags.npz")
    X, M = g["X"], int(g["num_levels"])
    N, L, D = X.shape
    k = kr.SignatureKernelRef(L * D, D, M, num_lags=nl)
    np.testing.assert_allclose(k.scale_sequences(X), g[f"lags{nl}_scaled"], rtol=1e-13, atol=1e-15)
