"""GPU parity of the gradients: gpsig_sig_gram_vjp (through gpsig_amd.autograd) vs torch fp64 autodiff
of the reference graph (oracle/autodiff_ref.py, pinned by finite differences in test_grad_oracle.py).

Criterion: norm-relative max|g32 - g64| <= GTOL * max|g64| per gradient tensor, GTOL = 1e-5 (the
north_star's fp32 bar, applied to gradients since round 5); the one named exception is in
test_gram_vjp_shapes, with its measured error.
"""
import numpy as np
import pytest
import torch

from conftest import norm_rel_err
from oracle import autodiff_ref as ar

pytestmark = pytest.mark.gpu
GTOL = 1e-5
DEV = "cuda"


def walks(n, l, d, seed, scale=1.0):
    rng = np.random.default_rng(seed)
    return scale * np.cumsum(rng.standard_normal((n, l, d)), axis=1) / np.sqrt(l * d)


def grads_gpu(kern, X, X2, G, return_levels=False, params=()):
    Xt = torch.tensor(X.reshape(len(X), -1), device=DEV, requires_grad=True)
    X2t = None if X2 is None else torch.tensor(X2.reshape(len(X2), -1), device=DEV, requires_grad=True)
    K = kern.K(Xt, X2t, return_levels=return_levels)
    (K * torch.as_tensor(G, device=DEV)).sum().backward()
    out = [Xt.grad.reshape(X.shape).cpu().numpy()]
    if X2 is not None:
        out.append(X2t.grad.reshape(X2.shape).cpu().numpy())
    out += [p.grad.cpu().numpy() for p in params]
    return out, K.detach().cpu().numpy()


def grads_ref(X, X2, G, M, base="rbf", normalization=True, return_levels=False, lengthscales=None, variances=None,
              jitter=1e-6):
    Xt = torch.tensor(X, requires_grad=True)
    X2t = None if X2 is None else torch.tensor(X2, requires_grad=True)
    ls = torch.tensor(np.ones(X.shape[-1]) if lengthscales is None else lengthscales, requires_grad=True)
    var = torch.tensor(np.ones(M + 1) if variances is None else variances, requires_grad=True)
    K = ar.K(Xt / ls, None if X2t is None else X2t / ls, M, base=base, normalization=normalization, scale=var,
             jitter=jitter, return_levels=return_levels)
    (K * torch.tensor(G)).sum().backward()
    out = [Xt.grad.numpy()]
    if X2 is not None:
        out.append(X2t.grad.numpy())
    return out, ls.grad.numpy(), var.grad.numpy(), K.detach().numpy()


@pytest.mark.parametrize("base", ["rbf", "linear"])
@pytest.mark.parametrize("cross", [False, True])
@pytest.mark.parametrize("normalization", [True, False])
def test_gram_vjp_matches_autodiff(base, cross, normalization):
    import gpsig_amd
    N, N2, L, L2, D, M = 12, 9, 24, 17, 3, 4
    X = walks(N, L, D, 0)
    X2 = walks(N2, L2, D, 1) if cross else None
    if cross:
        X2 = walks(N2, L, D, 1)  # the API takes one length per kernel (input_dim = L*D)
    G = np.random.default_rng(2).standard_normal((N, N2 if cross else N))
    cls = gpsig_amd.SignatureRBF if base == "rbf" else gpsig_amd.SignatureLinear
    k = cls(L * D, D, M, normalization=normalization)
    got, K = grads_gpu(k, X, X2, G)
    ref, _, _, Kref = grads_ref(X, X2, G, M, base=base, normalization=normalization)
    assert norm_rel_err(K, Kref) < 1e-5
    for g, r in zip(got, ref):
        assert norm_rel_err(g, r) < GTOL, (norm_rel_err(g, r))


def test_gram_vjp_return_levels_lengthscales_variances():
    import gpsig_amd
    N, L, D, M = 10, 20, 2, 5
    X = walks(N, L, D, 3)
    G = np.random.default_rng(4).standard_normal((M + 1, N, N))
    ls = np.array([0.7, 1.3])
    var = np.array([0.5, 1.0, 2.0, 1.5, 0.8, 1.2])
    k = gpsig_amd.SignatureRBF(L * D, D, M, lengthscales=ls, variances=var)
    k.lengthscales = torch.tensor(ls, device=DEV, requires_grad=True)
    k.variances = torch.tensor(var, device=DEV, requires_grad=True)
    got, K = grads_gpu(k, X, None, G, return_levels=True, params=(k.lengthscales, k.variances))
    ref, gls, gvar, Kref = grads_ref(X, None, G, M, return_levels=True, lengthscales=ls, variances=var)
    assert norm_rel_err(K, Kref) < 1e-5
    assert norm_rel_err(got[0], ref[0]) < GTOL
    assert norm_rel_err(got[1], gls) < GTOL
    assert norm_rel_err(got[2], gvar) < GTOL


@pytest.mark.parametrize("D,M,L", [(1, 1, 8), (5, 8, 40), (8, 2, 33), (16, 3, 20), (5, 5, 128)])
def test_gram_vjp_shapes(D, M, L):
    import gpsig_amd
    N = 6 if L > 64 else 9
    X = walks(N, L, D, 5)
    G = np.random.default_rng(6).standard_normal((N, N))
    k = gpsig_amd.SignatureRBF(L * D, D, M)
    got, _ = grads_gpu(k, X, None, G)
    ref, _, _, _ = grads_ref(X, None, G, M)
    assert norm_rel_err(got[0], ref[0]) < (2e-5 if (D, M, L) == (1, 1, 8) else GTOL)
    # (D, M, L) = (1, 1, 8): one channel, level 1 only, normalised -- the gradient is a difference of corner
    # terms that cancel across pairs, so the fp32 rounding of the inputs the kernel receives moves it by
    # ~1e-5 of its size (fp32 autodiff of the reference graph: 4.0e-3).  Every shape is also held to the plain
    # GTOL against fp64 autodiff of the reference graph at those fp32-rounded inputs (what the GPU computes on).
    ref_q, _, _, _ = grads_ref(X.astype(np.float32).astype(np.float64), None, G, M)
    assert norm_rel_err(got[0], ref_q[0]) < GTOL


@pytest.mark.parametrize("base", ["rbf", "linear"])
@pytest.mark.parametrize("N,D,M,L", [(13, 5, 5, 100), (7, 3, 6, 81), (10, 2, 4, 65), (5, 5, 5, 99)])
def test_gram_vjp_twenty_lane_groups(base, N, D, M, L):
    """65..100 points: the VJP runs 20-lane groups of 5 columns (3 pairs per wave, segmented scans) and
    the forward 10-lane groups of 10 columns; K(X) and K(X, X2) gradients vs fp64 autodiff."""
    import gpsig_amd
    X = walks(N, L, D, 40 + N)
    X2 = walks(N - 2, L, D, 41 + N)
    cls = gpsig_amd.SignatureRBF if base == "rbf" else gpsig_amd.SignatureLinear
    k = cls(L * D, D, M)
    G = np.random.default_rng(N).standard_normal((N, N))
    got, K = grads_gpu(k, X, None, G)
    ref, _, _, Kref = grads_ref(X, None, G, M, base=base)
    assert norm_rel_err(K, Kref) < 1e-5
    assert norm_rel_err(got[0], ref[0]) < GTOL
    G2 = np.random.default_rng(N + 1).standard_normal((N, N - 2))
    got, _ = grads_gpu(k, X, X2, G2)
    ref, _, _, _ = grads_ref(X, X2, G2, M, base=base)
    for g, r in zip(got, ref):
        assert norm_rel_err(g, r) < GTOL


def test_kdiag_unnormalised_vjp():
    import gpsig_amd
    N, L, D, M = 7, 30, 3, 4
    X = walks(N, L, D, 7, scale=2.0)
    k = gpsig_amd.SignatureRBF(L * D, D, M, normalization=False)
    Xt = torch.tensor(X.reshape(N, -1), device=DEV, requires_grad=True)
    w = np.random.default_rng(8).standard_normal((M + 1, N))
    (k.Kdiag(Xt, return_levels=True) * torch.as_tensor(w, device=DEV)).sum().backward()
    Xr = torch.tensor(X, requires_grad=True)
    (ar.k_seq_diag(Xr, M) * torch.tensor(w)).sum().backward()
    assert norm_rel_err(Xt.grad.reshape(X.shape).cpu().numpy(), Xr.grad.numpy()) < GTOL


def test_rough_data_vjp():
    """Large increments (|p|, |c| beyond the polynomial range): the corner-difference cells."""
    import gpsig_amd
    rng = np.random.default_rng(9)
    N, L, D, M = 6, 16, 3, 3
    X = rng.standard_normal((N, L, D))
    G = rng.standard_normal((N, N))
    k = gpsig_amd.SignatureRBF(L * D, D, M)
    got, _ = grads_gpu(k, X, None, G)
    ref, _, _, _ = grads_ref(X, None, G, M)
    assert norm_rel_err(got[0], ref[0]) < GTOL


@pytest.mark.parametrize("base", ["rbf", "linear"])
@pytest.mark.parametrize("cross", [False, True])
def test_gram_vjp_no_difference(base, cross):
    """difference=False (the base-kernel grid itself feeds the recursion): normalised K gradients
    w.r.t. the sequences and the variances vs fp64 autodiff."""
    import gpsig_amd
    N, N2, L, D, M = 10, 7, 21, 3, 4
    X = walks(N, L, D, 40)
    X2 = walks(N2, L, D, 41) if cross else None
    G = np.random.default_rng(42).standard_normal((N, N2 if cross else N))
    cls = gpsig_amd.SignatureRBF if base == "rbf" else gpsig_amd.SignatureLinear
    k = cls(L * D, D, M, difference=False)
    k.variances.requires_grad_(True)
    got, _ = grads_gpu(k, X, X2, G, params=(k.variances,))
    Xt = torch.tensor(X, requires_grad=True)
    X2t = None if X2 is None else torch.tensor(X2, requires_grad=True)
    var = torch.ones(M + 1, dtype=torch.float64, requires_grad=True)
    K = ar.K(Xt, X2t, M, base=base, scale=var, difference=False)
    (K * torch.tensor(G)).sum().backward()
    assert norm_rel_err(got[0], Xt.grad.numpy()) < GTOL
    if cross:
        assert norm_rel_err(got[1], X2t.grad.numpy()) < GTOL
    assert norm_rel_err(got[-1], var.grad.numpy()) < GTOL


@pytest.mark.parametrize("base", ["rbf", "linear"])
def test_raw_levels_vjp_no_difference_ragged(base):
    from gpsig_amd import ops
    N1, N2, L1, L2, D, M = 4, 6, 13, 40, 5, 5
    X, Y = walks(N1, L1, D, 43), walks(N2, L2, D, 44)
    G = np.random.default_rng(45).standard_normal((M + 1, N1, N2))
    gX, gY = ops.sig_gram_vjp(torch.tensor(X, device=DEV), torch.tensor(Y, device=DEV), M,
                              torch.tensor(G, device=DEV), base=base, gout_levels=True, difference=False)
    Xr, Yr = torch.tensor(X, requires_grad=True), torch.tensor(Y, requires_grad=True)
    (ar.k_seq(Xr, Yr, M, base, difference=False) * torch.tensor(G)).sum().backward()
    assert norm_rel_err(gX.cpu().numpy(), Xr.grad.numpy()) < GTOL
    assert norm_rel_err(gY.cpu().numpy(), Yr.grad.numpy()) < GTOL


def test_higher_order_backward_raises():
    """min(order, num_levels) = 7 with the RBF base kernel: outside the higher-order VJP kernels (orders
    2-5, and 6 at 6 levels, tests/test_ho_grad_gpu.py) and not the exact signature kernel -> NotImplementedError."""
    import gpsig_amd
    X = walks(4, 10, 2, 0)
    k = gpsig_amd.SignatureRBF(20, 2, 7, order=7)
    Xt = torch.tensor(X.reshape(4, -1), device=DEV, requires_grad=True)
    with pytest.raises(NotImplementedError):
        k.K(Xt).sum().backward()


@pytest.mark.parametrize("base", ["rbf", "linear"])
def test_raw_levels_vjp_ragged_lengths(base):
    """ops-level VJP of the raw per-level Gram with l1 != l2 (padded lane columns on both sides)."""
    from gpsig_amd import ops
    N1, N2, L1, L2, D, M = 5, 7, 19, 45, 4, 6
    X, Y = walks(N1, L1, D, 10), walks(N2, L2, D, 11)
    G = np.random.default_rng(12).standard_normal((M + 1, N1, N2))
    gX, gY = ops.sig_gram_vjp(torch.tensor(X, device=DEV), torch.tensor(Y, device=DEV), M,
                              torch.tensor(G, device=DEV), base=base, gout_levels=True)
    Xr, Yr = torch.tensor(X, requires_grad=True), torch.tensor(Y, requires_grad=True)
    (ar.k_seq(Xr, Yr, M, base) * torch.tensor(G)).sum().backward()
    assert norm_rel_err(gX.cpu().numpy(), Xr.grad.numpy()) < GTOL
    assert norm_rel_err(gY.cpu().numpy(), Yr.grad.numpy()) < GTOL


@pytest.mark.parametrize("base", ["rbf", "linear"])
@pytest.mark.parametrize("sym", [False, True])
@pytest.mark.parametrize("D,M,L1,L2", [(5, 5, 100, 100), (3, 4, 19, 45), (8, 6, 33, 128), (2, 2, 64, 7)])
def test_saved_state_vjp(base, sym, D, M, L1, L2):
    """The VJP from the forward launch's saved end state (gpsig_sig_gram_state) equals the VJP that
    recomputes its forward sweep, and the fp64 autodiff gradient; the forward output is unchanged."""
    from gpsig_amd import ops
    if sym:
        L2 = L1
    N1, N2 = 9, 7
    X = torch.tensor(walks(N1, L1, D, 20), device=DEV)
    Y = None if sym else torch.tensor(walks(N2, L2, D, 21), device=DEV)
    n2 = N1 if sym else N2
    G = torch.tensor(np.random.default_rng(22).standard_normal((M + 1, N1, n2)), device=DEV)
    if sym:
        G = G + G.transpose(1, 2)
    st = torch.empty(ops.sig_state_numel(N1, None if sym else N2, L2, M), dtype=torch.float32, device=DEV)
    K0 = ops.sig_gram(X, Y, M, base=base)
    K1 = ops.sig_gram(X, Y, M, base=base, state=st)
    assert torch.equal(K0, K1)
    g0 = ops.sig_gram_vjp(X, Y, M, G, base=base, gout_levels=True)
    g1 = ops.sig_gram_vjp(X, Y, M, G, base=base, gout_levels=True, state=st)
    Xr = torch.tensor(X.cpu().numpy().astype(np.float64), requires_grad=True)
    Yr = None if sym else torch.tensor(Y.cpu().numpy().astype(np.float64), requires_grad=True)
    Gr = G.cpu().double()
    if sym:  # K(X) evaluates the upper triangle and mirrors: dK(a,b) and dK(b,a) both flow to the pair
        (ar.k_seq(Xr, Xr, M, base) * Gr).sum().backward()
    else:
        (ar.k_seq(Xr, Yr, M, base) * Gr).sum().backward()
    assert norm_rel_err(g1[0].cpu().numpy(), g0[0].cpu().numpy()) < 1e-5
    assert norm_rel_err(g1[0].cpu().numpy(), Xr.grad.numpy()) < GTOL
    if not sym:
        assert norm_rel_err(g1[1].cpu().numpy(), g0[1].cpu().numpy()) < 1e-5
        assert norm_rel_err(g1[1].cpu().numpy(), Yr.grad.numpy()) < GTOL


def test_autograd_state_budget(monkeypatch):
    """K(X).backward with the saved state and with the recompute fallback (budget 0) agree."""
    import gpsig_amd
    import gpsig_amd.autograd as ag
    N, L, D, M = 10, 40, 4, 4
    X = walks(N, L, D, 30)
    G = np.random.default_rng(31).standard_normal((N, N))
    k = gpsig_amd.SignatureRBF(L * D, D, M)
    a, _ = grads_gpu(k, X, None, G)
    monkeypatch.setattr(ag, "GRAM_STATE_BYTES", 0)
    b, _ = grads_gpu(k, X, None, G)
    ref, _, _, _ = grads_ref(X, None, G, M)
    assert norm_rel_err(a[0], b[0]) < 1e-5
    assert norm_rel_err(a[0], ref[0]) < GTOL


@pytest.mark.parametrize("base", ["rbf", "linear"])
@pytest.mark.parametrize("increments", [False, True])
@pytest.mark.parametrize("D", [3, 40])
def test_tens_vs_seq_vjp_no_difference(base, increments, D):
    """difference=False inducing-tensor kernel (point values as cells): Z and X gradients of the
    normalised K_tens_vs_seq vs fp64 autodiff (D = 40: the wide VJP on GEMM seed tiles, sig_tvs_bwd_wide.hip)."""
    import gpsig_amd
    M, L, T, N = 4, 17, 5, 67
    LT = M * (M + 1) // 2
    rng = np.random.default_rng(60)
    Z = (0.5 if D <= 8 else 2.0 / np.sqrt(D)) * rng.standard_normal((LT, T, 2, D) if increments else (LT, T, D))
    X = walks(N, L, D, 61)
    G = rng.standard_normal((T, N))
    cls = gpsig_amd.SignatureRBF if base == "rbf" else gpsig_amd.SignatureLinear
    k = cls(L * D, D, M, difference=False)
    Zt = torch.tensor(Z, device=DEV, requires_grad=True)
    Xt = torch.tensor(X.reshape(N, -1), device=DEV, requires_grad=True)
    K = k.K_tens_vs_seq(Zt, Xt, increments=increments)
    (K * torch.as_tensor(G, device=DEV)).sum().backward()
    Zr, Xr = torch.tensor(Z, requires_grad=True), torch.tensor(X, requires_grad=True)
    Kr = ar.K_tens_vs_seq(Zr, Xr, M, base=base, increments=increments, difference=False)
    (Kr * torch.tensor(G)).sum().backward()
    assert norm_rel_err(K.detach().cpu().numpy(), Kr.detach().numpy()) < 1e-5
    assert norm_rel_err(Zt.grad.cpu().numpy(), Zr.grad.numpy()) < GTOL
    assert norm_rel_err(Xt.grad.reshape(X.shape).cpu().numpy(), Xr.grad.numpy()) < GTOL


@pytest.mark.parametrize("base", ["rbf", "linear"])
@pytest.mark.parametrize("increments", [False, True])
@pytest.mark.parametrize("M,D,L", [(3, 3, 20), (5, 5, 40), (1, 2, 9), (8, 8, 12)])
def test_tens_vs_seq_vjp_matches_autodiff(base, increments, M, D, L):
    """K_tens_vs_seq (normalised, summed) gradients in Z, X, lengthscales, variances."""
    import gpsig_amd
    T, N = 7, 70  # N > 64: two sequence blocks, a partial one
    LT = M * (M + 1) // 2
    rng = np.random.default_rng(20 + M)
    Z = 0.5 * rng.standard_normal((LT, T, 2, D) if increments else (LT, T, D))
    X = walks(N, L, D, 21)
    G = rng.standard_normal((T, N))
    ls = 0.8 + 0.4 * rng.random(D)
    cls = gpsig_amd.SignatureRBF if base == "rbf" else gpsig_amd.SignatureLinear
    k = cls(L * D, D, M)
    k.lengthscales = torch.tensor(ls, device=DEV, requires_grad=True)
    k.variances = torch.tensor(np.linspace(0.5, 1.5, M + 1), device=DEV, requires_grad=True)
    Zt = torch.tensor(Z, device=DEV, requires_grad=True)
    Xt = torch.tensor(X.reshape(N, -1), device=DEV, requires_grad=True)
    K = k.K_tens_vs_seq(Zt, Xt, increments=increments)
    (K * torch.as_tensor(G, device=DEV)).sum().backward()

    Zr, Xr = torch.tensor(Z, requires_grad=True), torch.tensor(X, requires_grad=True)
    lr = torch.tensor(ls, requires_grad=True)
    vr = torch.tensor(np.linspace(0.5, 1.5, M + 1), requires_grad=True)
    Zs = Zr / lr
    Kr = ar.K_tens_vs_seq(Zs, Xr / lr, M, base=base, increments=increments, scale=vr)
    (Kr * torch.tensor(G)).sum().backward()
    assert norm_rel_err(K.detach().cpu().numpy(), Kr.detach().numpy()) < 1e-5
    assert norm_rel_err(Zt.grad.cpu().numpy(), Zr.grad.numpy()) < GTOL
    assert norm_rel_err(Xt.grad.reshape(X.shape).cpu().numpy(), Xr.grad.numpy()) < GTOL
    assert norm_rel_err(k.lengthscales.grad.cpu().numpy(), lr.grad.numpy()) < GTOL
    assert norm_rel_err(k.variances.grad.cpu().numpy(), vr.grad.numpy()) < GTOL


@pytest.mark.parametrize("base", ["rbf", "linear"])
@pytest.mark.parametrize("increments", [False, True])
@pytest.mark.parametrize("D", [3, 46, 126])
def test_tens_gram_vjp_matches_autodiff(base, increments, D):
    """K_tens (Kzz, summed over levels x sigma*variances) gradients in Z and lengthscales (D = 46 and 126, the
    CMU runners' channel count after lag and time: the pair-tile + GEMM path, csrc/tens_vjp_mm.hip)."""
    import gpsig_amd
    M, T = 4, 70
    LT = M * (M + 1) // 2
    rng = np.random.default_rng(30)
    Z = (0.5 if D <= 8 else 0.15) * rng.standard_normal((LT, T, 2, D) if increments else (LT, T, D))
    G = rng.standard_normal((T, T))
    ls = np.linspace(0.9, 1.3, D)
    cls = gpsig_amd.SignatureRBF if base == "rbf" else gpsig_amd.SignatureLinear
    k = cls(10 * D, D, M)
    k.lengthscales = torch.tensor(ls, device=DEV, requires_grad=True)
    Zt = torch.tensor(Z, device=DEV, requires_grad=True)
    K = k.K_tens(Zt, increments=increments)
    (K * torch.as_tensor(G, device=DEV)).sum().backward()
    Zr, lr = torch.tensor(Z, requires_grad=True), torch.tensor(ls, requires_grad=True)
    Kr = ar.k_tens(Zr / lr, M, base, increments).sum(0)
    (Kr * torch.tensor(G)).sum().backward()
    assert norm_rel_err(K.detach().cpu().numpy(), Kr.detach().numpy()) < 1e-5
    assert norm_rel_err(Zt.grad.cpu().numpy(), Zr.grad.numpy()) < GTOL
    assert norm_rel_err(k.lengthscales.grad.cpu().numpy(), lr.grad.numpy()) < GTOL


def test_K_tens_n_seq_covs_gradient():
    """Gradient of a loss over all three outputs (Kzz, Kzx, full Kxx) of K_tens_n_seq_covs
    (kernels.py:624-704), the SVGP covariance bundle, in Z, X and the variances."""
    import gpsig_amd
    M, T, N, L, D = 3, 5, 6, 15, 2
    LT = M * (M + 1) // 2
    rng = np.random.default_rng(40)
    Z = 0.5 * rng.standard_normal((LT, T, D))
    X = walks(N, L, D, 41)
    G1, G2, G3 = rng.standard_normal((T, T)), rng.standard_normal((T, N)), rng.standard_normal((N, N))
    var = np.linspace(0.5, 1.5, M + 1)
    k = gpsig_amd.SignatureRBF(L * D, D, M)
    k.variances = torch.tensor(var, device=DEV, requires_grad=True)
    Zt = torch.tensor(Z, device=DEV, requires_grad=True)
    Xt = torch.tensor(X.reshape(N, -1), device=DEV, requires_grad=True)
    Kzz, Kzx, Kxx = k.K_tens_n_seq_covs(Zt, Xt, full_X_cov=True)
    ((Kzz * torch.as_tensor(G1, device=DEV)).sum() + (Kzx * torch.as_tensor(G2, device=DEV)).sum()
     + (Kxx * torch.as_tensor(G3, device=DEV)).sum()).backward()
    Zr, Xr, vr = (torch.tensor(Z, requires_grad=True), torch.tensor(X, requires_grad=True),
                  torch.tensor(var, requires_grad=True))
    Kzz_r = (ar.k_tens(Zr, M) * vr[:, None, None]).sum(0)
    Kzx_r = ar.K_tens_vs_seq(Zr, Xr, M, scale=vr)
    Kxx_r = ar.K(Xr, None, M, scale=vr)
    ((Kzz_r * torch.tensor(G1)).sum() + (Kzx_r * torch.tensor(G2)).sum() + (Kxx_r * torch.tensor(G3)).sum()).backward()
    assert norm_rel_err(Zt.grad.cpu().numpy(), Zr.grad.numpy()) < GTOL
    assert norm_rel_err(Xt.grad.reshape(X.shape).cpu().numpy(), Xr.grad.numpy()) < GTOL
    assert norm_rel_err(k.variances.grad.cpu().numpy(), vr.grad.numpy()) < GTOL


@pytest.mark.parametrize("base", ["rbf", "linear"])
@pytest.mark.parametrize("increments", [False, True])
@pytest.mark.parametrize("D", [5, 46])
def test_tens_vs_seq_saved_state_vjp_equals_recompute(base, increments, D):
    """The Kuf VJP from the forward launch's saved end state (gpsig_tens_vs_seq_state) equals the VJP
    that recomputes its forward sweep (the forward's exp-free recurrences vs the VJP's exact cells: fp32
    rounding only); the state path's output equals the plain launch bit for bit."""
    from gpsig_amd import ops
    T, N, L, M = 33, 130, 60, 5
    LT = M * (M + 1) // 2
    rng = np.random.default_rng(40)
    Z = torch.tensor((0.5 if D <= 8 else 2.0 / np.sqrt(D)) * rng.standard_normal((LT, T, 2, D) if increments else (LT, T, D)),
                     device=DEV, dtype=torch.float32)
    X = torch.tensor(walks(N, L, D, 41), device=DEV, dtype=torch.float32)
    G = torch.randn(M + 1, T, N, device=DEV)
    st = torch.empty(ops.tens_state_numel(T, N, M), device=DEV)
    out, st2 = ops.tens_vs_seq(Z, X, M, 1, base, True, increments, state=st)
    assert st2 is st
    torch.testing.assert_close(out, ops.tens_vs_seq(Z, X, M, 1, base, True, increments), rtol=0, atol=0)
    gz0, gx0 = ops.tens_vs_seq_vjp(Z, X, M, G, base, increments)
    gz1, gx1 = ops.tens_vs_seq_vjp(Z, X, M, G, base, increments, state=st)
    assert norm_rel_err(gz1.cpu().numpy(), gz0.cpu().numpy()) < 1e-5
    assert norm_rel_err(gx1.cpu().numpy(), gx0.cpu().numpy()) < 1e-5


def test_tens_vs_seq_higher_order_backward_raises():
    """K_tens_vs_seq of SignatureLinear(order=num_levels) runs the higher-order recursion forward
    (signature_algs.py:129-160); gpsig_tens_vs_seq_vjp differentiates the order-1 recursion only, so the
    backward must raise instead of returning the order-1 gradient."""
    import gpsig_amd
    M, D, L, T, N = 3, 2, 10, 3, 5
    LT = M * (M + 1) // 2
    rng = np.random.default_rng(70)
    k = gpsig_amd.SignatureLinear(L * D, D, M, order=M)
    Zt = torch.tensor(0.5 * rng.standard_normal((LT, T, D)), device=DEV, requires_grad=True)
    Xt = torch.tensor(walks(N, L, D, 71).reshape(N, -1), device=DEV, requires_grad=True)
    with pytest.raises(NotImplementedError):
        k.K_tens_vs_seq(Zt, Xt).sum().backward()


def test_tens_vs_seq_vjp_far_inducing_point():
    """An inducing point about 10 lengthscales from the path with outward steps of ~1.7 drives
    q = <z, dx_s> - g_s below -17, where 1 + expm1(q) underflows to 0 in fp32: the Kuf VJP's backward
    recurrence of k(z, x_s) must take exact point values there (finite gradients, oracle parity)."""
    import gpsig_amd
    M, D, L, T, N = 3, 2, 24, 4, 9
    LT = M * (M + 1) // 2
    rng = np.random.default_rng(72)
    X = np.cumsum(rng.standard_normal((N, L, D)) * 0.3, 1)
    X[:, L // 2:, :] += np.linspace(0, 1.7 * (L - L // 2), L - L // 2)[None, :, None] * np.array([1.0, 0.0])
    Z = rng.standard_normal((LT, T, D)) * 0.3
    Z[:, 0, :] = [-10.0, 0.0]  # far on the other side of the path
    G = rng.standard_normal((T, N))
    k = gpsig_amd.SignatureRBF(L * D, D, M, normalization=False)
    Zt = torch.tensor(Z, device=DEV, requires_grad=True)
    Xt = torch.tensor(X.reshape(N, -1), device=DEV, requires_grad=True)
    K = k.K_tens_vs_seq(Zt, Xt)
    (K * torch.as_tensor(G, device=DEV)).sum().backward()
    assert torch.isfinite(Zt.grad).all() and torch.isfinite(Xt.grad).all()
    Zr, Xr = torch.tensor(Z, requires_grad=True), torch.tensor(X, requires_grad=True)
    Kr = ar.K_tens_vs_seq(Zr, Xr, M, base="rbf", normalization=False)
    (Kr * torch.tensor(G)).sum().backward()
    assert norm_rel_err(Zt.grad.cpu().numpy(), Zr.grad.numpy()) < GTOL
    assert norm_rel_err(Xt.grad.reshape(X.shape).cpu().numpy(), Xr.grad.numpy()) < GTOL


@pytest.mark.parametrize("increments", [False, True])
def test_wide_tens_vs_seq_vjp_path_approaching_far_point(increments):
    """Wide channels (D = 20: the point-weight tile VJP, sig_tvs_bwd_wide.hip) with paths that start ~15
    lengthscales from an inducing point -- k(z, x) = e^-112 underflows to 0 in fp32 -- and walk steadily
    towards it (steps of 0.55: |q| < 20 per step, so the step-factor guard alone never fires), and paths that
    walk away from it (the reverse sweep sees the approach).  The carried k(z, x_s) must be re-evaluated once
    it would grow from an underflowed value, else the cells near z come out as 0."""
    import gpsig_amd
    M, D, L, T, N = 3, 20, 40, 3, 4
    LT = M * (M + 1) // 2
    rng = np.random.default_rng(80)
    X = rng.standard_normal((N, L, D)) * 0.02
    ramp = 15.0 - 0.55 * np.arange(L)  # channel-0 distance to z: 15 -> -6.45 (passes through z)
    X[0, :, 0] += ramp
    X[1, :, 0] += ramp[::-1]           # walks away (the reverse sweep approaches)
    X[2, :, 0] += 15.0 - 0.4 * np.arange(L)
    X[3] = np.cumsum(rng.standard_normal((L, D)) * 0.1, 0)
    Z = rng.standard_normal((LT, T, 2, D) if increments else (LT, T, D)) * 0.1
    Z[:, 0] *= 0.0  # the inducing points (and increments) of tensor 0 at the origin
    G = rng.standard_normal((T, N))
    k = gpsig_amd.SignatureRBF(L * D, D, M, normalization=False)
    Zt = torch.tensor(Z, device=DEV, requires_grad=True)
    Xt = torch.tensor(X.reshape(N, -1), device=DEV, requires_grad=True)
    K = k.K_tens_vs_seq(Zt, Xt, increments=increments)
    (K * torch.as_tensor(G, device=DEV)).sum().backward()
    assert torch.isfinite(Zt.grad).all() and torch.isfinite(Xt.grad).all()
    Zr, Xr = torch.tensor(Z, requires_grad=True), torch.tensor(X, requires_grad=True)
    Kr = ar.K_tens_vs_seq(Zr, Xr, M, base="rbf", increments=increments, normalization=False)
    assert norm_rel_err(K.detach().cpu().numpy(), Kr.detach().numpy()) < 1e-5
    (Kr * torch.tensor(G)).sum().backward()
    assert norm_rel_err(Zt.grad.cpu().numpy(), Zr.grad.numpy()) < GTOL
    assert norm_rel_err(Xt.grad.reshape(X.shape).cpu().numpy(), Xr.grad.numpy()) < GTOL


@pytest.mark.parametrize("D", [3, 20])
def test_tens_vs_seq_forward_path_approaching_far_point(D):
    """Forward Kuf (narrow packed kernel at D = 3, wide seed-tile kernel at D = 20) for paths that start ~15
    lengthscales from an inducing point (k underflows to 0) and walk towards it: the carried k(z, x_s) must
    be re-evaluated before it grows, not only at the anchors every 32 cells."""
    import gpsig_amd
    M, L, T, N = 3, 40, 2, 3
    LT = M * (M + 1) // 2
    rng = np.random.default_rng(81)
    X = rng.standard_normal((N, L, D)) * 0.02
    X[0, :, 0] += 15.0 - 0.55 * np.arange(L)
    X[1, :, 0] += 15.0 - 0.3 * np.arange(L)
    X[2] = np.cumsum(rng.standard_normal((L, D)) * 0.1, 0)
    Z = rng.standard_normal((LT, T, D)) * 0.1
    Z[:, 0] *= 0.0
    k = gpsig_amd.SignatureRBF(L * D, D, M, normalization=False)
    K = k.K_tens_vs_seq(torch.tensor(Z, device=DEV), torch.tensor(X.reshape(N, -1), device=DEV), return_levels=True)
    Kr = ar.K_tens_vs_seq(torch.tensor(Z), torch.tensor(X), M, base="rbf", normalization=False, return_levels=True)
    for m in range(1, M + 1):
        assert norm_rel_err(K[m].cpu().numpy(), Kr[m].numpy()) < 1e-5, m
