"""Low-rank mode (gpsig/low_rank_calculations.py, signature_algs.py:162-222): randomised, so parity
with the reference is distributional.  Deterministic pieces are checked exactly; the
random projections by their defining property (unbiased for the exact Hadamard / signature kernels),
by Monte Carlo."""
import math

import numpy as np
import pytest
import torch

from gpsig_amd import low_rank_calculations as lr

F64 = dict(dtype=torch.float64)


def test_lr_hadamard_prod_exact():
    A, B = torch.randn(3, 4, 5, **F64), torch.randn(3, 4, 6, **F64)
    C = lr.lr_hadamard_prod(A, B)
    assert C.shape == (3, 4, 30)
    torch.testing.assert_close(C.reshape(3, 4, 5, 6), A[..., :, None] * B[..., None, :])
    # feature inner products are products of inner products (the property the low-rank mode uses)
    torch.testing.assert_close(C[0] @ C[1].T, (A[0] @ A[1].T) * (B[0] @ B[1].T))


def test_draw_indices():
    s, ns, inv = lr._draw_indices(20, 7, need_inv=True, device="cpu")
    idx = torch.cat([s, ns])
    assert sorted(idx.tolist()) == list(range(20)) and len(s) == 7
    torch.testing.assert_close(idx[inv], torch.arange(20))


def test_nystrom_with_all_points_is_exact():
    X = torch.randn(30, 3, **F64)
    kern = lambda a, b: torch.exp(-0.5 * torch.cdist(a, b) ** 2)  # noqa: E731
    F = lr.Nystrom_map(X, kern, nys_samples=X)
    torch.testing.assert_close(F @ F.T, kern(X, X), atol=1e-4, rtol=0)


def test_sparse_projection_matches_gather_formula():
    """lr_hadamard_prod_sparse evaluates sum_i A_i (B @ R_i) instead of gathering the nonzero (i, j)
    combinations (low_rank_calculations.py:172-193); same projection R from the same seed."""
    A, B = torch.randn(7, 5, **F64), torch.randn(7, 4, **F64)
    rank, seed = 6, (11, 12)
    C = lr.lr_hadamard_prod_sparse(A, B, rank, 'sqrt', seed)
    D = 5 * 4
    s = math.sqrt(D)
    R = lr._draw_n_sparse_gaussian_samples(D * rank, s, device="cpu", generator=lr._gen(seed, "cpu")).reshape(D, rank)
    comb = [(i, j) for j in range(4) for i in range(5)]  # reference order: idx1 fastest
    nz = (R != 0).any(1)
    Cg = torch.stack([A[:, i] * B[:, j] for (i, j), keep in zip(comb, nz) if keep], 1) @ R[nz]
    torch.testing.assert_close(C, math.sqrt(s / rank) * Cg)
    torch.testing.assert_close(lr.lr_hadamard_prod_sparse(A, B, rank, 'sqrt', seed), C)  # stateless seeds


@pytest.mark.parametrize("sparsity", ["sqrt", "log", "lin"])
def test_random_hadamard_projection_unbiased(sparsity):
    torch.manual_seed(0)
    A, B = torch.randn(2, 6, **F64), torch.randn(2, 5, **F64)
    exact = (A @ A.T) * (B @ B.T)
    acc = torch.zeros(2, 2, **F64)
    n = 3000
    for k in range(n):
        C = lr.lr_hadamard_prod_rand(A, B, 8, sparsity, (k, 7))
        acc += C @ C.T
    est = acc / n
    # the subsampling estimator is unbiased up to the k1*k2 / rank scaling the reference leaves out
    if sparsity == "lin":
        est = est * (30 / 8)
    assert (est - exact).abs().max() < 0.15 * exact.abs().max()


def test_signature_lr_features_level_structure():
    U = torch.randn(4, 9, 5, **F64)
    Phi = lr.signature_kern_first_order_lr_feature(U, 3, 16, 'sqrt', seeds=[(1, 2), (3, 4)])
    assert [p.shape for p in Phi] == [(4, 1), (4, 5), (4, 16), (4, 16)]
    torch.testing.assert_close(Phi[1], (U[:, 1:] - U[:, :-1]).sum(1))
    bug = lr.signature_kern_first_order_lr_feature(U, 3, 16, 'sqrt', seeds=[(1, 2), (3, 4)], reference_level_bug=True)
    torch.testing.assert_close(bug[2], bug[1])  # signature_algs.py:191 appends the level-1 sum


@pytest.mark.gpu
def test_low_rank_K_estimates_exact_kernel():
    """SignatureLinear(low_rank=True) with Nystrom on all points (exact level 1): the averaged
    low-rank Gram approaches the exact first-order Gram at every level (unbiased projections)."""
    import gpsig_amd
    rng = np.random.default_rng(0)
    N, L, D, M = 4, 6, 2, 3
    X = np.cumsum(rng.standard_normal((N, L, D)), 1) / np.sqrt(L)
    Xt = torch.tensor(X.reshape(N, -1), device="cuda")
    exact = gpsig_amd.SignatureLinear(L * D, D, M, normalization=False).K(Xt, return_levels=True).cpu()
    k = gpsig_amd.SignatureLinear(L * D, D, M, normalization=False, low_rank=True, num_components=N * L,
                                  rank_bound=24)
    # deterministic: every projection / Nystrom draw comes from the seeded global generators
    torch.manual_seed(1234)
    runs = 400
    draws = torch.stack([k.K(Xt, return_levels=True).cpu() for _ in range(runs)])
    acc = draws.mean(0)
    torch.testing.assert_close(acc[1], exact[1], atol=1e-3 * exact[1].abs().max().item(), rtol=0)
    # the sparse-JL estimator is heavy-tailed: bound the bias by the Monte Carlo standard error of the
    # mean, per entry (an unbiased estimator sits within a few SE; a biased one drifts past it as runs grow)
    se = draws.std(0) / math.sqrt(runs)
    for m in (2, 3):
        dev = (acc[m] - exact[m]).abs()
        assert (dev <= 5.0 * se[m] + 1e-6 * exact[m].abs().max()).all(), (m, (dev / se[m]).max().item())
        assert dev.max() < 0.25 * exact[m].abs().max()
    # the other entry points run and have the reference shapes
    Z = torch.tensor(rng.standard_normal((6, 5, D)), device="cuda")
    assert k.K_tens(Z).shape == (5, 5)
    assert k.K_tens_vs_seq(Z, Xt).shape == (5, N)
    assert k.Kdiag(Xt).shape == (N,)
    kn = gpsig_amd.SignatureRBF(L * D, D, M, low_rank=True, num_components=12, rank_bound=10)
    Kzz, Kzx, Kxx = kn.K_tens_n_seq_covs(Z, Xt, full_X_cov=True)
    assert Kzz.shape == (5, 5) and Kzx.shape == (5, N) and Kxx.shape == (N, N)
    np.testing.assert_allclose(torch.diagonal(kn.K(Xt, return_levels=True), dim1=1, dim2=2).cpu().numpy(), 1.0,
                               rtol=1e-6)
    Kxx, Kxx2, Kd = kn.K_seq_n_seq_covs(Xt, Xt[:3])
    assert Kxx.shape == (N, N) and Kxx2.shape == (N, 3) and Kd.shape == (3,)
