"""GPU parity: the gfx950 Goursat-PDE kernel vs the reference's Cython solver outputs (pde.npz holds
sig_kern_diag results generated from gpsig/sigKer_fast.pyx) and the C restatement (cross Gram)."""
import numpy as np
import pytest
import torch

from conftest import golden, norm_rel_err
from oracle import pde

pytestmark = pytest.mark.gpu
TOL = 1e-5


def t(x):
    return torch.as_tensor(np.asarray(x), device="cuda")


@pytest.mark.parametrize("n", [0, 1, 2])
@pytest.mark.parametrize("solver", [0, 1])
def test_pde_diag_matches_reference_cython(n, solver):
    from gpsig_amd import ops
    g = golden("pde.npz")
    got = ops.pde_diag(t(g["X"]), n, solver).cpu().numpy()
    exp = g[f"diag_n{n}_s{solver}"]
    assert np.abs(got - exp).max() / np.abs(exp).max() < TOL, (got, exp)


@pytest.mark.parametrize("n", [0, 1])
def test_pde_cross_and_symmetric_gram(n):
    from gpsig_amd import ops
    g = golden("pde.npz")
    X, Y = t(g["X"]), t(g["Y"])
    assert norm_rel_err(ops.pde_gram(X, Y, n, 1).cpu().numpy(), g[f"cross_n{n}"]) < TOL
    S = ops.pde_gram(X, None, n, 1).cpu().numpy()
    assert norm_rel_err(S, g[f"sym_n{n}"]) < TOL
    np.testing.assert_array_equal(S, S.T)


def test_pde_kernel_class():
    import gpsig_amd
    g = golden("pde.npz")
    X = g["X"]
    A, L, D = X.shape
    k = gpsig_amd.UntruncSignatureKernel(L * D, D, order=1)
    kd = k.Kdiag(t(X.reshape(A, -1))).cpu().numpy()
    assert np.abs(kd - g["diag_n1_s1"]).max() / np.abs(g["diag_n1_s1"]).max() < TOL
    K = k.K(t(X.reshape(A, -1)), t(g["Y"].reshape(len(g["Y"]), -1))).cpu().numpy()
    assert norm_rel_err(K, g["cross_n1"]) < TOL


@pytest.mark.parametrize("L,n", [(2, 0), (65, 0), (66, 0), (129, 1), (200, 1), (257, 2), (300, 0)])
def test_pde_sizes(L, n):
    from gpsig_amd import ops
    rng = np.random.default_rng(L + n)
    X = np.cumsum(rng.standard_normal((3, L, 5)), 1) / np.sqrt(L * 5) * 2
    Y = np.cumsum(rng.standard_normal((2, L, 5)), 1) / np.sqrt(L * 5) * 2
    exp = pde.pde_gram(X, Y, n, 1)
    got = ops.pde_gram(t(X), t(Y), n, 1).cpu().numpy()
    assert norm_rel_err(got, exp) < TOL
