"""CPU: pin the gradient oracle (oracle/autodiff_ref.py, torch fp64 autodiff of the reference graph).

Forward values must equal the pinned NumPy oracle (oracle/kernels_ref.py); gradients must equal
central finite differences of that NumPy oracle -- i.e. the derivative TF autodiff computes for the
reference graph (gpsig/kernels.py:402-477 over signature_algs.py:8-35).
"""
import numpy as np
import pytest
import torch

from oracle import autodiff_ref as ar
from oracle import kernels_ref as kr


def walks(n, l, d, seed):
    rng = np.random.default_rng(seed)
    return np.cumsum(rng.standard_normal((n, l, d)), axis=1) / np.sqrt(l * d)


@pytest.mark.parametrize("base", ["rbf", "linear"])
@pytest.mark.parametrize("cross", [False, True])
def test_autodiff_oracle_forward_matches_numpy_oracle(base, cross):
    X, X2 = walks(5, 7, 2, 0), walks(4, 9, 2, 1)
    M = 3
    k = kr.SignatureKernelRef(7 * 2, 2, M, base=base)
    ref = k.K(X.reshape(5, -1), None if not cross else X2.reshape(4, -1), return_levels=True) if not cross else None
    if cross:
        k2 = kr.SignatureKernelRef(7 * 2, 2, M, base=base)
        # the NumPy oracle takes sequences of one length per call; cross lengths differ here
        ref = k2.K(X.reshape(5, -1), X2[:, :7].reshape(4, -1), return_levels=True)
        got = ar.K(torch.tensor(X), torch.tensor(X2[:, :7]), M, base=base, return_levels=True).numpy()
    else:
        got = ar.K(torch.tensor(X), None, M, base=base, return_levels=True).numpy()
    np.testing.assert_allclose(got, ref, rtol=1e-11, atol=1e-13)


@pytest.mark.parametrize("base", ["rbf", "linear"])
def test_autodiff_oracle_gradient_matches_finite_differences(base):
    X, X2 = walks(3, 6, 2, 3), walks(2, 6, 2, 4)
    M = 3
    rng = np.random.default_rng(5)
    G = rng.standard_normal((3, 2))
    k = kr.SignatureKernelRef(6 * 2, 2, M, base=base)

    def loss(Xv, X2v):
        return float((k.K(Xv.reshape(3, -1), X2v.reshape(2, -1)) * G).sum())

    Xt = torch.tensor(X, requires_grad=True)
    X2t = torch.tensor(X2, requires_grad=True)
    (ar.K(Xt, X2t, M, base=base) * torch.tensor(G)).sum().backward()
    h = 1e-6
    for arr, gt, which in ((X, Xt.grad.numpy(), 0), (X2, X2t.grad.numpy(), 1)):
        fd = np.zeros_like(arr)
        for idx in np.ndindex(arr.shape):
            p, m_ = arr.copy(), arr.copy()
            p[idx] += h
            m_[idx] -= h
            fp = loss(p, X2) if which == 0 else loss(X, p)
            fm = loss(m_, X2) if which == 0 else loss(X, m_)
            fd[idx] = (fp - fm) / (2 * h)
        np.testing.assert_allclose(gt, fd, rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("base", ["rbf", "linear"])
@pytest.mark.parametrize("increments", [False, True])
def test_autodiff_oracle_tens_vs_seq(base, increments):
    """Forward equals the NumPy oracle; dLoss/dZ and dLoss/dX equal central differences of it."""
    M, T, N, L, D = 3, 2, 3, 5, 2
    LT = M * (M + 1) // 2
    rng = np.random.default_rng(7)
    Z = 0.5 * rng.standard_normal((LT, T, 2, D) if increments else (LT, T, D))
    X = walks(N, L, D, 8)
    k = kr.SignatureKernelRef(L * D, D, M, base=base)
    ref = k.K_tens_vs_seq(Z, X.reshape(N, -1), return_levels=True, increments=increments)
    Zt, Xt = torch.tensor(Z, requires_grad=True), torch.tensor(X, requires_grad=True)
    got = ar.K_tens_vs_seq(Zt, Xt, M, base=base, increments=increments, return_levels=True)
    np.testing.assert_allclose(got.detach().numpy(), ref, rtol=1e-11, atol=1e-13)
    G = rng.standard_normal((T, N))
    (ar.K_tens_vs_seq(Zt, Xt, M, base=base, increments=increments) * torch.tensor(G)).sum().backward()

    def loss(Zv, Xv):
        return float((k.K_tens_vs_seq(Zv, Xv.reshape(N, -1), increments=increments) * G).sum())

    h = 1e-6
    for arr, gt, which in ((Z, Zt.grad.numpy(), 0), (X, Xt.grad.numpy(), 1)):
        fd = np.zeros_like(arr)
        for idx in np.ndindex(arr.shape):
            p, m_ = arr.copy(), arr.copy()
            p[idx] += h
            m_[idx] -= h
            fd[idx] = ((loss(p, X) - loss(m_, X)) if which == 0 else (loss(Z, p) - loss(Z, m_))) / (2 * h)
        np.testing.assert_allclose(gt, fd, rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("base", ["rbf", "linear"])
@pytest.mark.parametrize("increments", [False, True])
def test_autodiff_oracle_tens_gram(base, increments):
    M, T, D = 3, 4, 2
    LT = M * (M + 1) // 2
    rng = np.random.default_rng(9)
    Z = 0.5 * rng.standard_normal((LT, T, 2, D) if increments else (LT, T, D))
    k = kr.SignatureKernelRef(2 * D, D, M, base=base)
    ref = k.K_tens_raw(Z, increments)
    Zt = torch.tensor(Z, requires_grad=True)
    np.testing.assert_allclose(ar.k_tens(Zt, M, base, increments).detach().numpy(), ref, rtol=1e-11, atol=1e-13)
    G = rng.standard_normal((M + 1, T, T))
    (ar.k_tens(Zt, M, base, increments) * torch.tensor(G)).sum().backward()
    h = 1e-6
    fd = np.zeros_like(Z)
    for idx in np.ndindex(Z.shape):
        p, m_ = Z.copy(), Z.copy()
        p[idx] += h
        m_[idx] -= h
        fd[idx] = ((k.K_tens_raw(p, increments) * G).sum() - (k.K_tens_raw(m_, increments) * G).sum()) / (2 * h)
    np.testing.assert_allclose(Zt.grad.numpy(), fd, rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("base,order", [("linear", 5), ("linear", 2), ("rbf", 3)])
def test_autodiff_oracle_higher_order_matches_numpy_oracle_and_chen(base, order):
    """The torch restatement of signature_algs.py:37-74 equals the NumPy oracle; with the linear base
    kernel and order = num_levels it is the exact signature kernel (Chen), the golden linear_chen.npz."""
    from conftest import golden
    M = 5
    X, X2 = walks(4, 9, 2, 5), walks(3, 9, 2, 6)
    k = kr.SignatureKernelRef(9 * 2, 2, M, base=base, order=order, normalization=False)
    ref = k.K(X.reshape(4, -1), X2.reshape(3, -1), return_levels=True)
    got = ar.K(torch.tensor(X), torch.tensor(X2), M, base=base, order=order, normalization=False,
               return_levels=True).numpy()
    np.testing.assert_allclose(got, ref, rtol=1e-10, atol=1e-13)
    if base == "linear" and order == M:
        g = golden("linear_chen.npz")
        Xg = g["X"]
        Kg = ar.k_seq(torch.tensor(Xg), None, int(g["num_levels"]), "linear", True, order=int(g["num_levels"]))
        np.testing.assert_allclose(Kg.numpy(), g["K_chen"], rtol=1e-9, atol=1e-12)
