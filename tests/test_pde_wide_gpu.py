"""GPU parity of the PDE increment-tile mode (pde.hip pde_tiled_run, pde_bwd.hip pde_adj_tiled): channel
counts above the fixed instantiations (d = 40, 128: the reference's sigpde runners feed 46 / 126-channel
series, kernels_pde.py:21-25 takes any d) and dyadic orders past the fixed kernels' refinement (forward
dyadic 3 at L = 200 and dyadic 4-5 by tile sub-refinement; adjoint dyadic 4). Oracle: the C restatement
(oracle/pde, forward and the reference's adjoint kernels_pde.py:465-509)."""
import numpy as np
import pytest
import torch

from conftest import norm_rel_err
from oracle import pde

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = 1e-5


def paths(rng, n, L, d, scale=2.0):
    return np.cumsum(rng.standard_normal((n, L, d)), 1) / np.sqrt(L * d) * scale


@pytest.mark.parametrize("L,d,n", [(30, 128, 0), (30, 128, 1), (64, 40, 2), (129, 46, 1), (20, 17, 0)])
def test_pde_wide_channels_gram_and_diag(L, d, n):
    from gpsig_amd import ops
    rng = np.random.default_rng(L * d + n)
    X, Y = paths(rng, 4, L, d), paths(rng, 3, L - 3, d)
    got = ops.pde_gram(torch.tensor(X, device=DEV), torch.tensor(Y, device=DEV), n, 1).cpu().numpy()
    assert norm_rel_err(got, pde.pde_gram(X, Y, n, 1)) < TOL
    S = ops.pde_gram(torch.tensor(X, device=DEV), None, n, 1).cpu().numpy()
    assert norm_rel_err(S, pde.pde_gram(X, X, n, 1)) < TOL
    np.testing.assert_array_equal(S, S.T)
    kd = ops.pde_diag(torch.tensor(X, device=DEV), n, 0).cpu().numpy()
    exp = pde.pde_diag(X, n, 0)
    assert np.abs(kd - exp).max() / np.abs(exp).max() < TOL


@pytest.mark.parametrize("L,d,n", [(200, 5, 3), (100, 5, 4), (40, 3, 5), (100, 40, 4)])
def test_pde_high_dyadic_forward(L, d, n):
    """Refined grids of 1592 (dyadic 3, REP 8 kernel), 1584 (dyadic 4, REP 16) and 1248 (dyadic 5: tile
    cells split once more, value / 4) columns."""
    from gpsig_amd import ops
    rng = np.random.default_rng(L + 7 * n)
    X, Y = paths(rng, 2, L, d), paths(rng, 2, L, d)
    got = ops.pde_gram(torch.tensor(X, device=DEV), torch.tensor(Y, device=DEV), n, 1).cpu().numpy()
    assert norm_rel_err(got, pde.pde_gram(X, Y, n, 1)) < TOL
    kd = ops.pde_diag(torch.tensor(X, device=DEV), n, 1).cpu().numpy()
    exp = pde.pde_diag(X, n, 1)
    assert np.abs(kd - exp).max() / np.abs(exp).max() < TOL


@pytest.mark.parametrize("L,d,n", [(30, 40, 0), (30, 128, 1), (100, 5, 4), (60, 3, 5), (200, 4, 3)])
def test_pde_tiled_vjp(L, d, n):
    """Adjoint in tile mode (d > 16 or dyadic > 3): dLoss/d<dx_i, dy_j> tiles contracted with the
    increments by the matrix-core GEMM, cross and diagonal."""
    from gpsig_amd import ops
    rng = np.random.default_rng(3 * L + d + n)
    X, Y = paths(rng, 3, L, d), paths(rng, 2, L - 2, d)
    G = rng.standard_normal((3, 2))
    Xt, Yt, Gt = (torch.tensor(v, device=DEV, dtype=torch.float32) for v in (X, Y, G))
    gX, gY = ops.pde_gram_vjp(Xt, Yt, Gt, n, 1)
    rx, ry = pde.pde_gram_grad(X, Y, G, n, 1)
    assert norm_rel_err(gX.cpu().numpy(), rx) < TOL
    assert norm_rel_err(gY.cpu().numpy(), ry) < TOL
    w = rng.standard_normal(3)
    gd = ops.pde_diag_vjp(Xt, torch.tensor(w, device=DEV, dtype=torch.float32), n, 1).cpu().numpy()
    ref = np.zeros_like(X)
    for a in range(3):
        gx, gy = pde.pde_gram_grad(X[a:a + 1], X[a:a + 1], np.ones((1, 1)), n, 1)
        ref[a] = w[a] * (gx[0] + gy[0])
    assert norm_rel_err(gd, ref) < TOL


@pytest.mark.parametrize("d,n", [(40, 1), (5, 4)])
def test_pde_tiled_fronts_and_autograd(d, n):
    """Training-step split in tile mode: gpsig_pde_fronts_ex values equal gpsig_pde_gram_ex's, the
    adjoint from the fronts equals the one-call adjoint; autograd through UntruncSignatureKernel.K."""
    import gpsig_amd
    from gpsig_amd import ops
    rng = np.random.default_rng(90 + d + n)
    L = 24
    X = torch.tensor(paths(rng, 5, L, d), device=DEV, dtype=torch.float32)
    Y = torch.tensor(paths(rng, 4, L, d), device=DEV, dtype=torch.float32)
    G = torch.randn(5, 4, device=DEV)
    fr = torch.empty(ops.pde_fronts_bytes(20, L, L, n) // 4, device=DEV)
    K = ops.pde_fronts(X, Y, n, 1, fr)
    torch.testing.assert_close(K, ops.pde_gram(X, Y, n, 1), rtol=0, atol=0)
    gX, gY = ops.pde_vjp_fronts(X, Y, G, n, 1, fr)
    rX, rY = ops.pde_gram_vjp(X, Y, G, n, 1)
    assert norm_rel_err(gX.cpu().numpy(), rX.cpu().numpy()) < 1e-6
    assert norm_rel_err(gY.cpu().numpy(), rY.cpu().numpy()) < 1e-6
    kp = gpsig_amd.UntruncSignatureKernel(L * d, d, order=n)
    Xf = X.reshape(5, -1).double().requires_grad_(True)
    Kg = kp.K(Xf)
    torch.testing.assert_close(Kg.detach(), kp.K(Xf.detach()), rtol=1e-7, atol=0)
    (Kg * torch.randn(5, 5, device=DEV, dtype=torch.float64)).sum().backward()
    assert torch.isfinite(Xf.grad).all()


@pytest.mark.parametrize("n", [6, 7, 8])
def test_pde_dyadic_6_to_8_forward_and_vjp(n):
    """The forward's dyadic cap (8) is the adjoint's too: dyadic 6-8 forward (tile cells split 2^(n-4) ways)
    and the adjoint on the REP-8 layout (cells split 2^(n-3) ways) against the C oracle; autograd through
    UntruncSignatureKernel.K at the same order."""
    import gpsig_amd
    from gpsig_amd import ops
    rng = np.random.default_rng(600 + n)
    L, d = 9, 3
    X, Y = paths(rng, 2, L, d), paths(rng, 2, L - 1, d)
    Xt, Yt = torch.tensor(X, device=DEV), torch.tensor(Y, device=DEV)
    got = ops.pde_gram(Xt, Yt, n, 1).cpu().numpy()
    assert norm_rel_err(got, pde.pde_gram(X, Y, n, 1)) < TOL
    kd = ops.pde_diag(Xt, n, 1).cpu().numpy()
    exp = pde.pde_diag(X, n, 1)
    assert np.abs(kd - exp).max() / np.abs(exp).max() < TOL
    G = rng.standard_normal((2, 2))
    gX, gY = ops.pde_gram_vjp(Xt.float(), Yt.float(), torch.tensor(G, device=DEV, dtype=torch.float32), n, 1)
    rx, ry = pde.pde_gram_grad(X, Y, G, n, 1)
    assert norm_rel_err(gX.cpu().numpy(), rx) < TOL
    assert norm_rel_err(gY.cpu().numpy(), ry) < TOL
    kp = gpsig_amd.UntruncSignatureKernel(L * d, d, order=n)
    Xf = Xt.reshape(2, -1).double().requires_grad_(True)
    kp.K(Xf).sum().backward()
    assert torch.isfinite(Xf.grad).all()


def test_pde_tiled_vjp_column_side_split_k():
    """Tiled adjoint with n2 (l2 - 1) >> rows per chunk: the dLoss/d dy contraction (M = n2 (l2 - 1), K = the
    chunk's rows) splits K and must stay inside the scratch (gemm_f32 clamps the split).  The loss weights
    three y-paths only, so the C oracle runs on those; the other y-gradients must be exactly zero."""
    from gpsig_amd import ops
    rng = np.random.default_rng(64)
    n1, n2, L, d = 64, 1000, 64, 32
    X, Y = paths(rng, n1, L, d), paths(rng, n2, L, d)
    sel = [0, 500, 999]
    G = np.zeros((n1, n2))
    G[:, sel] = rng.standard_normal((n1, len(sel)))
    f = lambda v: torch.tensor(v, device=DEV, dtype=torch.float32)
    gX, gY = ops.pde_gram_vjp(f(X), f(Y), f(G), 0, 1)
    rx, ry = pde.pde_gram_grad(X, Y[sel], G[:, sel], 0, 1)
    assert norm_rel_err(gX.cpu().numpy(), rx) < TOL
    gy = gY.cpu().numpy()
    assert norm_rel_err(gy[sel], ry) < TOL
    assert not np.any(np.delete(gy, sel, axis=0))
