"""PDE-kernel gradient: the oracle restatement of the reference's adjoint (oracle/pde_grad.py) pinned
to the reference's own grids (tests/golden/pde.npz), and the gfx950 gpsig_pde_vjp against it."""
import numpy as np
import pytest
import torch

from conftest import golden, norm_rel_err
from oracle import pde, pde_grad

DEV = "cuda"


@pytest.mark.parametrize("n,solver", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_kdiag_grad_oracle_pinned_and_consistent(n, solver):
    g = golden("pde.npz")
    X = g["X"]
    ref = pde_grad.kdiag_grad(X, g[f"grid_n{n}_s{solver}"], g[f"gridrev_n{n}_s{solver}"], n)
    # the C restatement's grids give the same gradient (it matches sig_kern_diag bitwise)
    K, Kr = pde.pde_diag_grids(X, n, solver)  # full grids; the reference stores the lower triangle
    np.testing.assert_allclose(pde_grad.kdiag_grad(X, np.tril(K), np.tril(Kr), n), ref, rtol=1e-12, atol=1e-10)
    # the cross-pair extension with y = x reproduces the diagonal formula (x-part + y-part = 2 x-part)
    if solver == 1:
        for a in range(3):
            gx, gy = pde_grad.pair_grad(X[a], X[a], n, solver)
            np.testing.assert_allclose(gx + gy, ref[a], rtol=1e-9, atol=1e-11)


def test_pair_grad_approximates_derivative():
    """The adjoint is the continuous-PDE derivative (K_rev by the first-order scheme): it approximates
    finite differences of the discrete solve up to the discretisation error (a few % at dyadic 2)."""
    rng = np.random.default_rng(3)
    x = np.cumsum(rng.standard_normal((8, 2)), 0) * 0.2
    y = np.cumsum(rng.standard_normal((6, 2)), 0) * 0.2
    n = 2
    gx, gy = pde_grad.pair_grad(x, y, n)
    h = 1e-6
    fd = np.zeros_like(x)
    for idx in np.ndindex(x.shape):
        p, m = x.copy(), x.copy()
        p[idx] += h
        m[idx] -= h
        fd[idx] = (pde_grad.pair_grids(p, y, n)[0][-1, -1] - pde_grad.pair_grids(m, y, n)[0][-1, -1]) / (2 * h)
    assert np.abs(gx - fd).max() < 0.1 * np.abs(fd).max()


@pytest.mark.gpu
@pytest.mark.parametrize("n,solver", [(0, 0), (0, 1), (1, 0), (1, 1), (2, 1)])
def test_pde_kdiag_vjp_matches_reference_adjoint(n, solver):
    import gpsig_amd
    g = golden("pde.npz")
    X = g["X"]
    A, L, D = X.shape
    w = np.random.default_rng(4).standard_normal(A)
    K, Kr = pde.pde_diag_grids(X, n, solver)
    ref = pde_grad.kdiag_grad(X, np.tril(K), np.tril(Kr), n) * w[:, None, None]
    k = gpsig_amd.UntruncSignatureKernel(L * D, D, order=n)
    k.solver = solver
    Xt = torch.tensor(X.reshape(A, -1), device=DEV, requires_grad=True)
    (k.Kdiag(Xt) * torch.as_tensor(w, device=DEV)).sum().backward()
    assert norm_rel_err(Xt.grad.reshape(X.shape).cpu().numpy(), ref) < 1e-5


@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 1])
def test_pde_cross_vjp_matches_adjoint(n):
    from gpsig_amd import ops
    rng = np.random.default_rng(5)
    X = np.cumsum(rng.standard_normal((3, 9, 2)), 1) * 0.3
    Y = np.cumsum(rng.standard_normal((4, 7, 2)), 1) * 0.3
    G = rng.standard_normal((3, 4))
    gX, gY = ops.pde_gram_vjp(torch.tensor(X, device=DEV), torch.tensor(Y, device=DEV),
                              torch.tensor(G, device=DEV), n, 1)
    rx, ry = np.zeros_like(X), np.zeros_like(Y)
    for a in range(3):
        for b in range(4):
            gx, gy = pde_grad.pair_grad(X[a], Y[b], n, 1)
            rx[a] += G[a, b] * gx
            ry[b] += G[a, b] * gy
    assert norm_rel_err(gX.cpu().numpy(), rx) < 1e-5
    assert norm_rel_err(gY.cpu().numpy(), ry) < 1e-5


@pytest.mark.gpu
@pytest.mark.parametrize("L,n", [(100, 1), (200, 1), (129, 2), (300, 1), (500, 0), (500, 1)])
def test_pde_kdiag_vjp_wide_grids(L, n):
    """Wide grids of the adjoint kernel: 2^n (L-1) = 198 (W = 4), 398 and 512 (W = 8), 598 refined
    columns (W = 16), and the reference's VOSF training length (train_gpsig_vosf.py:25,100: max_len 500,
    UntruncSignatureKernel order 0; order 1 = 998 refined columns)."""
    from gpsig_amd import ops
    rng = np.random.default_rng(L + n)
    X = np.cumsum(rng.standard_normal((3, L, 3)), 1) / np.sqrt(L * 3) * 2
    w = rng.standard_normal(3)
    K, Kr = pde.pde_diag_grids(X, n, 1)
    ref = pde_grad.kdiag_grad(X, np.tril(K), np.tril(Kr), n) * w[:, None, None]
    got = ops.pde_diag_vjp(torch.tensor(X, device=DEV), torch.tensor(w, device=DEV), n, 1)
    assert norm_rel_err(got.cpu().numpy(), ref) < 1e-5


@pytest.mark.gpu
@pytest.mark.parametrize("l2,n", [(300, 0), (700, 0), (130, 1)])
def test_pde_cross_vjp_wide_grids(l2, n):
    """Cross pairs whose refined column count J = 2^n (l2 - 1) is 299 / 258 (W = 8) and 699 (W = 16)."""
    from gpsig_amd import ops
    rng = np.random.default_rng(l2)
    X = np.cumsum(rng.standard_normal((2, 12, 2)), 1) * 0.3
    Y = np.cumsum(rng.standard_normal((2, l2, 2)), 1) * 0.3 / np.sqrt(l2 / 10)
    G = rng.standard_normal((2, 2))
    gX, gY = ops.pde_gram_vjp(torch.tensor(X, device=DEV), torch.tensor(Y, device=DEV),
                              torch.tensor(G, device=DEV), n, 1)
    rx, ry = np.zeros_like(X), np.zeros_like(Y)
    for a in range(2):
        for b in range(2):
            gx, gy = pde_grad.pair_grad(X[a], Y[b], n, 1)
            rx[a] += G[a, b] * gx
            ry[b] += G[a, b] * gy
    assert norm_rel_err(gX.cpu().numpy(), rx) < 1e-5
    assert norm_rel_err(gY.cpu().numpy(), ry) < 1e-5


@pytest.mark.gpu
@pytest.mark.parametrize("n,solver", [(0, 1), (1, 1), (1, 0), (2, 1)])
def test_pde_fronts_forward_and_vjp(n, solver):
    """The training step's split adjoint: gpsig_pde_fronts returns gpsig_pde_gram's / gpsig_pde_diag's
    values (same cells) and leaves the forward fronts; gpsig_pde_vjp_fronts from them equals gpsig_pde_vjp.
    Also through autograd (UntruncSignatureKernel.K / Kdiag take this path when a gradient is needed)."""
    import gpsig_amd
    from gpsig_amd import ops
    rng = np.random.default_rng(60 + n)
    X = torch.tensor(np.cumsum(rng.standard_normal((6, 13, 3)), 1) * 0.3, device=DEV, dtype=torch.float32)
    Y = torch.tensor(np.cumsum(rng.standard_normal((5, 11, 3)), 1) * 0.3, device=DEV, dtype=torch.float32)
    G = torch.randn(6, 5, device=DEV)
    fr = torch.empty(ops.pde_fronts_bytes(30, 13, 11, n) // 4, device=DEV)
    K = ops.pde_fronts(X, Y, n, solver, fr)
    torch.testing.assert_close(K, ops.pde_gram(X, Y, n, solver), rtol=0, atol=0)
    gX, gY = ops.pde_vjp_fronts(X, Y, G, n, solver, fr)
    rX, rY = ops.pde_gram_vjp(X, Y, G, n, solver)
    assert norm_rel_err(gX.cpu().numpy(), rX.cpu().numpy()) < 1e-6
    assert norm_rel_err(gY.cpu().numpy(), rY.cpu().numpy()) < 1e-6
    w = torch.randn(6, device=DEV)
    frd = torch.empty(ops.pde_fronts_bytes(6, 13, 13, n) // 4, device=DEV)
    kd = ops.pde_fronts(X, None, n, solver, frd, diag=True)
    torch.testing.assert_close(kd, ops.pde_diag(X, n, solver), rtol=0, atol=0)
    gd = ops.pde_vjp_fronts(X, None, w, n, solver, frd, diag=True)
    assert norm_rel_err(gd.cpu().numpy(), ops.pde_diag_vjp(X, w, n, solver).cpu().numpy()) < 1e-6
    # autograd: symmetric K(X) with a gradient (fronts path) vs without (forward only)
    kp = gpsig_amd.UntruncSignatureKernel(13 * 3, 3, order=n)
    kp.solver = solver
    Xf = X.reshape(6, -1).double().requires_grad_(True)
    Kg = kp.K(Xf)
    torch.testing.assert_close(Kg.detach(), kp.K(Xf.detach()), rtol=1e-7, atol=0)
    assert torch.equal(Kg, Kg.T)


@pytest.mark.gpu
@pytest.mark.parametrize("L,n,d", [(600, 1, 3), (150, 3, 3), (1100, 0, 5)])
def test_pde_kdiag_vjp_column_blocks(L, n, d):
    """Grids wider than one wave's 64 W refined columns, swept in column blocks: 1198 columns = 2 blocks of
    1024 (W = 16), 1192 at dyadic order 3 = 3 blocks of 512 (W = 8), and 1099 at order 0 with d = 5, where
    x's per-pair LDS (row accumulators and increments, 66 KB) leaves 2 pairs per workgroup."""
    from gpsig_amd import ops
    rng = np.random.default_rng(L + n)
    X = np.cumsum(rng.standard_normal((3, L, d)), 1) / np.sqrt(L * d) * 2
    w = rng.standard_normal(3)
    K, Kr = pde.pde_diag_grids(X, n, 1)
    ref = pde_grad.kdiag_grad(X, np.tril(K), np.tril(Kr), n) * w[:, None, None]
    got = ops.pde_diag_vjp(torch.tensor(X, device=DEV), torch.tensor(w, device=DEV), n, 1)
    assert norm_rel_err(got.cpu().numpy(), ref) < 1e-5


@pytest.mark.gpu
@pytest.mark.parametrize("l2,n,solver", [(1500, 0, 1), (300, 2, 1), (1500, 0, 0)])
def test_pde_cross_vjp_column_blocks(l2, n, solver):
    """Cross pairs in column blocks (J = 1499 at order 0, 1196 at order 2: 2 blocks of 1024), against the
    adjoint restated from the reference; then the training-step split (gpsig_pde_fronts forward, whose
    values equal gpsig_pde_gram's, and gpsig_pde_vjp_fronts) against the one-launch adjoint."""
    from gpsig_amd import ops
    rng = np.random.default_rng(l2 + n)
    X = np.cumsum(rng.standard_normal((3, 12, 2)), 1) * 0.3
    Y = np.cumsum(rng.standard_normal((2, l2, 2)), 1) * 0.3 / np.sqrt(l2 / 10)
    G = rng.standard_normal((3, 2))
    Xt, Yt, Gt = (torch.tensor(v, device=DEV, dtype=torch.float32) for v in (X, Y, G))
    gX, gY = ops.pde_gram_vjp(Xt, Yt, Gt, n, solver)
    rx, ry = np.zeros_like(X), np.zeros_like(Y)
    for a in range(3):
        for b in range(2):
            gx, gy = pde_grad.pair_grad(X[a], Y[b], n, solver)
            rx[a] += G[a, b] * gx
            ry[b] += G[a, b] * gy
    assert norm_rel_err(gX.cpu().numpy(), rx) < 1e-5
    assert norm_rel_err(gY.cpu().numpy(), ry) < 1e-5
    fr = torch.empty(ops.pde_fronts_bytes(6, 12, l2, n) // 4, device=DEV)
    K = ops.pde_fronts(Xt, Yt, n, solver, fr)
    torch.testing.assert_close(K, ops.pde_gram(Xt, Yt, n, solver), rtol=0, atol=0)
    fX, fY = ops.pde_vjp_fronts(Xt, Yt, Gt, n, solver, fr)
    assert norm_rel_err(fX.cpu().numpy(), gX.cpu().numpy()) < 1e-6
    assert norm_rel_err(fY.cpu().numpy(), gY.cpu().numpy()) < 1e-6
