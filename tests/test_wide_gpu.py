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


# ----------------------------------------------------------------------------- gradients
GTOL = 1e-5  # observed <= 2.2e-6 (tools/grad_err_scan.py, profiles/r4_wide_grad_err.jsonl)


@pytest.mark.parametrize("D,L", [(46, 136), (126, 136), (46, 500), (33, 20)])
@pytest.mark.parametrize("sym", [False, True])
def test_wide_gram_vjp_raw_levels(D, L, sym):
    """ops-level VJP of the raw per-level Gram (point-weight tiles + the emission GEMMs) vs fp64 autodiff of
    the reference graph (oracle/autodiff_ref.py), with and without the forward's saved state."""
    from gpsig_amd import ops
    from oracle import autodiff_ref as ar
    rng = np.random.default_rng(D + L + sym)
    N1, N2, M = 3, 2, 3
    X = walks(rng, N1, L, D)
    Y = None if sym else walks(rng, N2, L - 5, D)
    n2 = N1 if sym else N2
    G = rng.standard_normal((M + 1, N1, n2))
    Xt = torch.tensor(X, device=DEV, dtype=torch.float32)
    Yt = None if sym else torch.tensor(Y, device=DEV, dtype=torch.float32)
    Gt = torch.tensor(G, device=DEV, dtype=torch.float32)
    st = torch.empty(ops.sig_state_numel(N1, None if sym else N2, L if sym else L - 5, M), dtype=torch.float32,
                     device=DEV)
    K0 = ops.sig_gram(Xt, Yt, M)
    K1 = ops.sig_gram(Xt, Yt, M, state=st)
    assert torch.equal(K0, K1)
    g0 = ops.sig_gram_vjp(Xt, Yt, M, Gt, gout_levels=True)
    g1 = ops.sig_gram_vjp(Xt, Yt, M, Gt, gout_levels=True, state=st)
    Xr = torch.tensor(X, requires_grad=True)
    Yr = Xr if sym else torch.tensor(Y, requires_grad=True)
    (ar.k_seq(Xr, Yr, M, "rbf") * torch.tensor(G)).sum().backward()
    for g in (g0, g1):
        assert norm_rel_err(g[0].cpu().numpy(), Xr.grad.numpy()) < GTOL
        if not sym:
            assert norm_rel_err(g[1].cpu().numpy(), Yr.grad.numpy()) < GTOL


@pytest.mark.parametrize("D", [46, 126])
def test_wide_K_gradient_normalised(D):
    """K(X, X2) of SignatureRBF (normalised: diagonal VJP chained through rs) with lengthscales and
    variances, gradients in X, X2, lengthscales, variances vs fp64 autodiff."""
    import gpsig_amd
    from oracle import autodiff_ref as ar
    rng = np.random.default_rng(D + 1)
    N1, N2, L, M = 4, 3, 30, 4
    X, X2 = walks(rng, N1, L, D, 2.0), walks(rng, N2, L, D, 2.0)
    G = rng.standard_normal((N1, N2))
    ls = rng.uniform(0.7, 1.5, D)
    var = np.linspace(0.5, 1.5, M + 1)
    k = gpsig_amd.SignatureRBF(L * D, D, M)
    k.lengthscales = torch.tensor(ls, device=DEV, requires_grad=True)
    k.variances = torch.tensor(var, device=DEV, requires_grad=True)
    Xt = torch.tensor(X.reshape(N1, -1), device=DEV, requires_grad=True)
    X2t = torch.tensor(X2.reshape(N2, -1), device=DEV, requires_grad=True)
    (k.K(Xt, X2t) * torch.as_tensor(G, device=DEV)).sum().backward()
    Xr, X2r = torch.tensor(X, requires_grad=True), torch.tensor(X2, requires_grad=True)
    lr, vr = torch.tensor(ls, requires_grad=True), torch.tensor(var, requires_grad=True)
    (ar.K(Xr / lr, X2r / lr, M, scale=vr) * torch.tensor(G)).sum().backward()
    assert norm_rel_err(Xt.grad.reshape(X.shape).cpu().numpy(), Xr.grad.numpy()) < GTOL
    assert norm_rel_err(X2t.grad.reshape(X2.shape).cpu().numpy(), X2r.grad.numpy()) < GTOL
    assert norm_rel_err(k.lengthscales.grad.cpu().numpy(), lr.grad.numpy()) < GTOL
    assert norm_rel_err(k.variances.grad.cpu().numpy(), vr.grad.numpy()) < GTOL


@pytest.mark.parametrize("base,difference", [("linear", True), ("rbf", False), ("linear", False)])
def test_wide_vjp_other_seeds(base, difference):
    from gpsig_amd import ops
    from oracle import autodiff_ref as ar
    rng = np.random.default_rng(9)
    D, L, M = 40, 25, 3
    X, Y = walks(rng, 3, L, D), walks(rng, 2, L + 3, D)
    G = rng.standard_normal((M + 1, 3, 2))
    gX, gY = ops.sig_gram_vjp(torch.tensor(X, device=DEV), torch.tensor(Y, device=DEV), M,
                              torch.tensor(G, device=DEV), base=base, gout_levels=True, difference=difference)
    Xr, Yr = torch.tensor(X, requires_grad=True), torch.tensor(Y, requires_grad=True)
    (ar.k_seq(Xr, Yr, M, base, difference=difference) * torch.tensor(G)).sum().backward()
    assert norm_rel_err(gX.cpu().numpy(), Xr.grad.numpy()) < GTOL
    assert norm_rel_err(gY.cpu().numpy(), Yr.grad.numpy()) < GTOL


# ----------------------------------------------------------------------------- inducing tensors
@pytest.mark.parametrize("D,L", [(46, 136), (126, 136), (46, 500), (9, 33), (12, 40)])
@pytest.mark.parametrize("increments", [False, True])
def test_wide_tens_vs_seq(D, L, increments):
    """K_tens_vs_seq raw levels (the wide port of the packed recursion) vs the oracle at the runners'
    channel counts (InducingTensors with increments=True is what train_gpsig.py trains)."""
    from gpsig_amd import ops
    M, T, N = 4, 5, 70
    LT = M * (M + 1) // 2
    rng = np.random.default_rng(D + L + increments)
    Z = rng.standard_normal((LT, T, 2, D) if increments else (LT, T, D)) * (2.0 / np.sqrt(D))
    X = walks(rng, N, L, D, 2.0)
    ref = kr.SignatureKernelRef(L * D, D, M, normalization=False)
    exp = ref.K_tens_vs_seq_raw(Z, X, increments=increments)
    got = ops.tens_vs_seq(t(Z), t(X), M, increments=increments).cpu().numpy()
    assert (norm_rel_err(got[1:], exp[1:], axis_levels=True) < TOL).all()


@pytest.mark.parametrize("D", [46, 126])
def test_wide_tens_vs_seq_corner(D):
    """Kuf raw levels with increments far apart: |q| or |c| >= 2 on many steps, so the forward takes the
    corner differences of directly evaluated base-kernel values (|z1 - x|^2 from the exact pass and the
    step's seeds) rather than the chained expm1 recurrences."""
    from gpsig_amd import ops
    M, T, N, L = 4, 6, 24, 60
    LT = M * (M + 1) // 2
    rng = np.random.default_rng(D + 7)
    Z = rng.standard_normal((LT, T, 2, D)) * (1.0 / np.sqrt(D))
    inc = rng.standard_normal((N, L, D)) * (1.5 / np.sqrt(D))
    inc[:, ::7, :] *= 3.0
    X = np.cumsum(inc, 1)
    dx = np.diff(X, axis=1)
    q = np.einsum("ktd,nsd->ktns", Z[:, :, 0], dx) - np.einsum("nsd,nsd->ns", X[:, :-1], dx) \
        - 0.5 * np.einsum("nsd,nsd->ns", dx, dx)
    assert (np.abs(q) >= 2.0).mean() > 0.1  # the corner regime is exercised
    ref = kr.SignatureKernelRef(L * D, D, M, normalization=False)
    exp = ref.K_tens_vs_seq_raw(Z, X, increments=True)
    got = ops.tens_vs_seq(t(Z), t(X), M, increments=True).cpu().numpy()
    assert (norm_rel_err(got[1:], exp[1:], axis_levels=True) < TOL).all()


@pytest.mark.parametrize("order,difference,base", [(2, True, "rbf"), (1, False, "rbf"), (1, True, "linear"),
                                                   (3, True, "linear")])
def test_wide_tens_vs_seq_generic(order, difference, base):
    """The generic kernel (orders > 1, difference=False) and the linear seed at a wide channel count."""
    from gpsig_amd import ops
    M, T, N, D, L = 3, 4, 20, 40, 18
    LT = M * (M + 1) // 2
    rng = np.random.default_rng(order * 10 + difference)
    Z = rng.standard_normal((LT, T, 2, D)) * (2.0 / np.sqrt(D))
    X = walks(rng, N, L, D, 2.0)
    ref = kr.SignatureKernelRef(L * D, D, M, normalization=False, order=order, difference=difference, base=base)
    exp = ref.K_tens_vs_seq_raw(Z, X, increments=True)
    got = ops.tens_vs_seq(t(Z), t(X), M, order=order, base=base, difference=difference, increments=True).cpu().numpy()
    assert (norm_rel_err(got[1:], exp[1:], axis_levels=True) < TOL).all()


@pytest.mark.parametrize("increments", [False, True])
def test_wide_tens_gram(increments):
    from gpsig_amd import ops
    M, T, D = 4, 37, 46
    LT = M * (M + 1) // 2
    rng = np.random.default_rng(3 + increments)
    Z = rng.standard_normal((LT, T, 2, D) if increments else (LT, T, D)) * (2.0 / np.sqrt(D))
    exp = kr.SignatureKernelRef(4 * D, D, M).K_tens_raw(Z, increments=increments)
    got = ops.tens_gram(t(Z), M, increments=increments).cpu().numpy()
    assert (norm_rel_err(got[1:], exp[1:], axis_levels=True) < TOL).all()


@pytest.mark.parametrize("D,L", [(46, 136), (126, 40), (46, 500)])
@pytest.mark.parametrize("base", ["rbf", "linear"])
@pytest.mark.parametrize("increments", [True, False])
def test_wide_tens_vs_seq_vjp(D, L, base, increments):
    """Kuf gradients (point-weight tiles + the emission GEMMs) vs fp64 autodiff, normalised K_tens_vs_seq,
    with and without the forward's saved end state."""
    import gpsig_amd
    from oracle import autodiff_ref as ar
    M, T, N = 3, 3, 67
    LT = M * (M + 1) // 2
    rng = np.random.default_rng(D + L)
    Z = rng.standard_normal((LT, T, 2, D) if increments else (LT, T, D)) * (2.0 / np.sqrt(D))
    X = walks(rng, N, L, D, 2.0)
    G = rng.standard_normal((T, N))
    cls = gpsig_amd.SignatureRBF if base == "rbf" else gpsig_amd.SignatureLinear
    k = cls(L * D, D, M)
    Zt = torch.tensor(Z, device=DEV, requires_grad=True)
    Xt = torch.tensor(X.reshape(N, -1), device=DEV, requires_grad=True)
    (k.K_tens_vs_seq(Zt, Xt, increments=increments) * torch.as_tensor(G, device=DEV)).sum().backward()
    Zr, Xr = torch.tensor(Z, requires_grad=True), torch.tensor(X, requires_grad=True)
    (ar.K_tens_vs_seq(Zr, Xr, M, base=base, increments=increments) * torch.tensor(G)).sum().backward()
    assert norm_rel_err(Zt.grad.cpu().numpy(), Zr.grad.numpy()) < GTOL
    assert norm_rel_err(Xt.grad.reshape(X.shape).cpu().numpy(), Xr.grad.numpy()) < GTOL


@pytest.mark.parametrize("embedding", ["linear", "rbf"])
def test_wide_rescaled(embedding):
    """VOSF <S(x), (I - Lambda) S(x)> per level (signature_algs_vosf.py:11-48) at a wide channel count."""
    from gpsig_amd import ops
    M, T, N, D, L = 3, 4, 6, 30, 20
    LT = M * (M + 1) // 2
    rng = np.random.default_rng(5)
    Z = rng.uniform(0.0, 1.0, (LT, T, D))
    X = walks(rng, N, L, D, 2.0)
    if embedding == "linear":
        exp = kr.SignatureKernelRef(L * D, D, M, base="linear", normalization=False).mahalanobis_raw(Z, X)
    else:  # per-coordinate RBF embedding (kernels_pde.py:191-222), as tests/golden/make_golden.py F5
        from oracle import sigalgs
        Zc = np.concatenate([Z, np.ones_like(Z)], axis=1)
        E = np.exp(-(X[:, :, None, :] - X[:, None, :, :]) ** 2 / 2.0)
        exp = sigalgs.signature_kern_rescaled_higher_order(np.einsum("npqd,rtd->nprtq", E, Zc), M)
    got = ops.rescaled(t(Z), t(X), M, embedding=embedding).cpu().numpy()
    assert (norm_rel_err(got[1:], exp[1:], axis_levels=True) < TOL).all()


# ----------------------------------------------------------------------------- higher order, tile mode
@pytest.mark.parametrize("D,L,M,order", [(46, 40, 4, 2), (63, 60, 5, 5), (40, 150, 5, 5), (100, 30, 4, 4)])
def test_wide_higher_order_linear(D, L, M, order):
    """Higher-order recursion past 32 channels with the linear base kernel (the exact signature kernel at
    order >= M, as benchmarks/models/train_gpsig_vosf.py:102 trains it with add_time: 63 channels for
    CMUsubject16): cells from the increment-Gram tile (a matrix-core GEMM), recursion as sig_ho; L = 150
    runs in column blocks.  Cross, symmetric and diagonal against the fp64 oracle."""
    from gpsig_amd import ops
    rng = np.random.default_rng(D + L + order)
    X, Y = walks(rng, 4, L, D), walks(rng, 3, L - 7, D)
    ref = kr.SignatureKernelRef(L * D, D, M, normalization=False, base="linear", order=order)
    got = ops.sig_gram(t(X), t(Y), M, order=order, base="linear").cpu().numpy()
    assert (norm_rel_err(got[1:], ref.K_seq(X, Y)[1:], axis_levels=True) < TOL).all()
    S = ops.sig_gram(t(X), None, M, order=order, base="linear").cpu().numpy()
    exp = ref.K_seq(X, X)
    assert (norm_rel_err(S[1:], exp[1:], axis_levels=True) < TOL).all()
    d = ops.sig_diag(t(X), M, order=order, base="linear").cpu().numpy()
    assert (norm_rel_err(d[1:], np.stack([np.diagonal(e) for e in exp])[1:], axis_levels=True) < TOL).all()


@pytest.mark.parametrize("D,L,M,order", [(46, 40, 3, 2), (33, 100, 4, 3), (126, 60, 5, 5), (46, 170, 3, 2)])
def test_wide_higher_order_rbf(D, L, M, order):
    """Higher-order recursion past 32 channels with the RBF base kernel (signature_algs.py:37-74 over
    kernels.py:946-957 at any D): the difference-seed cells of each chunk of pairs come from the matrix-core
    wide seed in cell-producer mode (sig_fo_mf.h; column blocks at L = 170), the recursion reads them as the
    linear path reads its increment Gram, level 1 in the RBF closed form.  Cross, symmetric and diagonal
    against the fp64 oracle."""
    from gpsig_amd import ops
    rng = np.random.default_rng(D + L + order + 1)
    X, Y = walks(rng, 4, L, D), walks(rng, 3, L - 5, D)
    ref = kr.SignatureKernelRef(L * D, D, M, normalization=False, order=order)
    got = ops.sig_gram(t(X), t(Y), M, order=order, base="rbf").cpu().numpy()
    assert (norm_rel_err(got[1:], ref.K_seq(X, Y)[1:], axis_levels=True) < TOL).all()
    S = ops.sig_gram(t(X), None, M, order=order, base="rbf").cpu().numpy()
    exp = ref.K_seq(X, X)
    assert (norm_rel_err(S[1:], exp[1:], axis_levels=True) < TOL).all()
    dg = ops.sig_diag(t(X), M, order=order, base="rbf").cpu().numpy()
    assert (norm_rel_err(dg[1:], np.stack([np.diagonal(e) for e in exp])[1:], axis_levels=True) < TOL).all()


# ----------------------------------------------------------------------------- edge cases
@pytest.mark.parametrize("D,L1,L2", [(33, 2, 2), (40, 2, 17), (64, 3, 130), (50, 129, 2)])
def test_wide_edge_lengths(D, L1, L2):
    """Shortest sequences (one increment), ragged lengths across the 128-point geometry switch, one
    sequence per side: raw levels of the RBF and linear Gram against the oracle."""
    from gpsig_amd import ops
    rng = np.random.default_rng(D + L1 + L2)
    X, Y = walks(rng, 1, L1, D), walks(rng, 2, L2, D)
    for base in ("rbf", "linear"):
        ref = kr.SignatureKernelRef(L1 * D, D, 4, normalization=False, base=base)
        got = ops.sig_gram(t(X), t(Y), 4, base=base).cpu().numpy()
        assert (norm_rel_err(got[1:], ref.K_seq(X, Y)[1:], axis_levels=True) < TOL).all(), base


def test_wide_empty_and_single():
    """An empty batch returns an empty Gram (the reference's graph does the same); N = 1 symmetric."""
    from gpsig_amd import ops
    X0 = torch.zeros((0, 20, 40), device=DEV)
    assert ops.sig_gram(X0, None, 3).shape == (4, 0, 0)
    rng = np.random.default_rng(1)
    X = walks(rng, 1, 20, 40)
    ref = kr.SignatureKernelRef(20 * 40, 40, 3, normalization=False)
    got = ops.sig_gram(t(X), None, 3).cpu().numpy()
    assert (norm_rel_err(got[1:], ref.K_seq(X, X)[1:], axis_levels=True) < TOL).all()


@pytest.mark.parametrize("L", [2, 3, 65])
def test_wide_higher_order_and_pde_short(L):
    """Tile modes at the shortest lengths: higher-order linear (d = 40) and the PDE (d = 40, dyadic 2)."""
    from gpsig_amd import ops
    from oracle import pde
    rng = np.random.default_rng(L)
    X, Y = walks(rng, 3, L, 40), walks(rng, 2, L, 40)
    ref = kr.SignatureKernelRef(L * 40, 40, 3, normalization=False, base="linear", order=3)
    got = ops.sig_gram(t(X), t(Y), 3, order=3, base="linear").cpu().numpy()
    assert (norm_rel_err(got[1:], ref.K_seq(X, Y)[1:], axis_levels=True) < TOL).all()
    gp = ops.pde_gram(t(X), t(Y), 2, 1).cpu().numpy()
    assert norm_rel_err(gp, pde.pde_gram(X, Y, 2, 1)) < TOL


@pytest.mark.parametrize("L1,L2", [(3, 130), (130, 9), (20, 300)])
def test_wide_vjp_ragged_records(L1, L2):
    """x and y records of different padded lengths (wide_lw(L1) != wide_lw(L2)): the row side strides by
    the x record, the columns by the y record, in the forward seed and the VJP's regenerated cells."""
    from gpsig_amd import ops
    from oracle import autodiff_ref as ar
    D, M = 46, 3
    rng = np.random.default_rng(L1 * 7 + L2)
    X, Y = walks(rng, 2, L1, D), walks(rng, 3, L2, D)
    G = rng.standard_normal((M + 1, 2, 3))
    Xt, Yt = t(X).float(), t(Y).float()
    got = ops.sig_gram(Xt, Yt, M).cpu().numpy()
    ref = kr.SignatureKernelRef(L1 * D, D, M, normalization=False)
    assert (norm_rel_err(got[1:], ref.K_seq(X, Y)[1:], axis_levels=True) < TOL).all()
    gX, gY = ops.sig_gram_vjp(Xt, Yt, M, torch.tensor(G, device=DEV, dtype=torch.float32), gout_levels=True)
    Xr, Yr = torch.tensor(X, requires_grad=True), torch.tensor(Y, requires_grad=True)
    (ar.k_seq(Xr, Yr, M, "rbf") * torch.tensor(G)).sum().backward()
    assert norm_rel_err(gX.cpu().numpy(), Xr.grad.numpy()) < GTOL
    assert norm_rel_err(gY.cpu().numpy(), Yr.grad.numpy()) < GTOL
    if L2 <= 256:  # the higher-order VJP's range
        gX2, gY2 = ops.sig_gram_vjp(Xt, Yt, M, torch.tensor(G, device=DEV, dtype=torch.float32), gout_levels=True,
                                    order=2)
        Xr, Yr = torch.tensor(X, requires_grad=True), torch.tensor(Y, requires_grad=True)
        (ar.k_seq(Xr, Yr, M, "rbf", order=2) * torch.tensor(G)).sum().backward()
        assert norm_rel_err(gX2.cpu().numpy(), Xr.grad.numpy()) < GTOL
        assert norm_rel_err(gY2.cpu().numpy(), Yr.grad.numpy()) < GTOL


@pytest.mark.parametrize("path", ["wide", "ho_tile", "pde_tile", "pde_sub"])
def test_tile_paths_row_windows(path):
    """Row windows (rows=(r0, r1), the row sharding of gpsig_amd/distributed.py) on the wide and tile
    paths: every evaluated entry (a in the window, b >= a) equals the full symmetric call's."""
    from gpsig_amd import ops
    rng = np.random.default_rng(11)
    n = 13
    if path == "wide":
        X = t(walks(rng, n, 40, 46)).float()
        full = ops.sig_gram(X, None, 3)
        part = lambda r0, r1: ops.sig_gram(X, None, 3, rows=(r0, r1))  # noqa: E731
    elif path == "ho_tile":
        X = t(walks(rng, n, 30, 40)).float()
        full = ops.sig_gram(X, None, 4, order=2, base="linear")
        part = lambda r0, r1: ops.sig_gram(X, None, 4, order=2, base="linear", rows=(r0, r1))  # noqa: E731
    else:
        dy = 1 if path == "pde_tile" else 5
        X = t(walks(rng, n, 20, 40 if path == "pde_tile" else 3)).float()
        full = ops.pde_gram(X, None, dy, 1)[None]
        part = lambda r0, r1: ops.pde_gram(X, None, dy, 1, rows=(r0, r1))[None]  # noqa: E731
    for r0, r1 in [(0, 5), (5, 6), (6, 13), (3, 11)]:
        got = part(r0, r1)
        for a in range(r0, r1):
            torch.testing.assert_close(got[:, a - r0, a:], full[:, a, a:], rtol=1e-6, atol=1e-7)


def test_wide_vjp_column_side_split_k():
    """RECT VJP with far more column-side points than one row chunk holds (n2 * l2 >> rows * l1): the
    column-side emission GEMM splits K on its own, and its partial products must stay inside the workspace
    (gemm_f32 clamps the split to the capacity it is given).  The loss weights only four y-sequences, so the
    fp64 oracle runs on those; every other y-gradient must be exactly zero."""
    from gpsig_amd import ops
    from oracle import autodiff_ref as ar
    rng = np.random.default_rng(400)
    N1, N2, L, D, M = 8, 400, 100, 32, 2
    X = walks(rng, N1, L, D)
    Y = walks(rng, N2, L, D)
    sel = [0, 1, 398, 399]
    G = np.zeros((M + 1, N1, N2))
    G[:, :, sel] = rng.standard_normal((M + 1, N1, len(sel)))
    gX, gY = ops.sig_gram_vjp(t(X).float(), t(Y).float(), M, t(G).float(), gout_levels=True)
    Xr = torch.tensor(X, requires_grad=True)
    Yr = torch.tensor(Y[sel], requires_grad=True)
    (ar.k_seq(Xr, Yr, M, "rbf") * torch.tensor(G[:, :, sel])).sum().backward()
    assert norm_rel_err(gX.cpu().numpy(), Xr.grad.numpy()) < GTOL
    gy = gY.cpu().numpy()
    assert norm_rel_err(gy[sel], Yr.grad.numpy()) < GTOL
    rest = np.setdiff1d(np.arange(N2), sel)
    assert not np.any(gy[rest])


@pytest.mark.parametrize("D,L,M,base", [(46, 161, 2, "rbf"), (46, 300, 6, "rbf"), (126, 300, 3, "rbf"),
                                        (46, 300, 4, "linear"), (200, 170, 3, "rbf")])
def test_wide_mf_column_blocks(D, L, M, base):
    """Matrix-core wide Gram past 160 points (sig_fo_mf.h): column blocks of 127 cells, each with its own B
    image (the block's increments and its first point y_{j0}), the levels' column sums carried from block to
    block through the workspace; K(X, X2) at ragged lengths and K(X), raw levels against the oracle."""
    from gpsig_amd import ops
    rng = np.random.default_rng(D + L + M)
    X = walks(rng, 5, L, D)
    Y = walks(rng, 3, L - 11, D)
    ref = kr.SignatureKernelRef(L * D, D, M, normalization=False, base=base)
    got = ops.sig_gram(t(X), t(Y), M, base=base).cpu().numpy()
    assert (norm_rel_err(got[1:], ref.K_seq(X, Y)[1:], axis_levels=True) < TOL).all()
    sym = ops.sig_gram(t(X), None, M, base=base).cpu().numpy()
    assert (norm_rel_err(sym[1:], ref.K_seq(X)[1:], axis_levels=True) < TOL).all()
    np.testing.assert_array_equal(sym, np.swapaxes(sym, 1, 2))


@pytest.mark.parametrize("increments", [True, False])
def test_wide_tens_vs_seq_seed_chunks(increments, monkeypatch):
    """Kuf forward and VJP with the seed tiles split over several chunks of sequences (GPSIG_TVS_TILE_BYTES
    forces chunks of 64 sequences): the forward equals the one-chunk launch bit for bit, the gradients to
    fp32 rounding (the emission GEMMs accumulate the chunks in another order)."""
    from gpsig_amd import ops
    M, T, N, D, L = 3, 5, 150, 40, 30
    LT = M * (M + 1) // 2
    rng = np.random.default_rng(77)
    Z = t(rng.standard_normal((LT, T, 2, D) if increments else (LT, T, D)) * (2.0 / np.sqrt(D)))
    X = t(walks(rng, N, L, D, 2.0))
    G = torch.randn(M + 1, T, N, device=DEV)
    out1 = ops.tens_vs_seq(Z, X, M, increments=increments)
    gz1, gx1 = ops.tens_vs_seq_vjp(Z, X, M, G, "rbf", increments)
    monkeypatch.setenv("GPSIG_TVS_TILE_BYTES", "65536")
    out2 = ops.tens_vs_seq(Z, X, M, increments=increments)
    gz2, gx2 = ops.tens_vs_seq_vjp(Z, X, M, G, "rbf", increments)
    torch.testing.assert_close(out2, out1, rtol=0, atol=0)
    assert norm_rel_err(gz2.cpu().numpy(), gz1.cpu().numpy()) < 1e-6
    assert norm_rel_err(gx2.cpu().numpy(), gx1.cpu().numpy()) < 1e-6


@pytest.mark.parametrize("case", ["offset", "tiny", "huge_lin", "zero_seq"])
def test_wide_split_operand_scales(case):
    """The matrix-core wide Gram's operand split (sig_fo_mf.h: f16 parts at per-row / per-sequence power-of-two
    scales) on inputs whose magnitudes stress the scales: points offset by 10 lengthscales with increments ~0.02
    (RBF is translation invariant, so the kernel values stay O(1)), everything ~1e-3 or ~1e4 times the unit walk
    (linear base kernel) and an all-zero sequence.  Against the fp64 oracle at the fp32-rounded inputs the kernels
    receive.  (Where the scales do not hold -- offsets of ~1e3 lengthscales, every third point pulled to 0 -- is
    measured in DESIGN.md 2.10 "Range".)"""
    from gpsig_amd import ops
    rng = np.random.default_rng(["offset", "tiny", "huge_lin", "zero_seq"].index(case) + 900)
    D, L, M = 46, 40, 4
    X = walks(rng, 5, L, D)
    Y = walks(rng, 3, L - 5, D)
    base = "rbf"
    if case == "offset":
        off = rng.standard_normal(D) * 10.0 / np.sqrt(D)
        X, Y = X + off, Y + off
    elif case == "tiny":
        X, Y, base = X * 1e-3, Y * 1e-3, "linear"
    elif case == "huge_lin":
        X, Y, base = X * 1e4, Y * 1e4, "linear"
    elif case == "zero_seq":
        X[1] = 0.0
        Y[2] = 0.0
    X = X.astype(np.float32).astype(np.float64)
    Y = Y.astype(np.float32).astype(np.float64)
    ref = kr.SignatureKernelRef(L * D, D, M, normalization=False, base=base)
    got = ops.sig_gram(t(X), t(Y), M, base=base).cpu().numpy()
    exp = ref.K_seq(X, Y)
    assert np.isfinite(got).all()
    err = norm_rel_err(got[1:], exp[1:], axis_levels=True)
    assert (err < TOL).all(), err
    sym = ops.sig_gram(t(X), None, M, base=base).cpu().numpy()
    err = norm_rel_err(sym[1:], ref.K_seq(X)[1:], axis_levels=True)
    assert (err < TOL).all(), err


@pytest.mark.parametrize("M", [1, 2, 7, 8])
@pytest.mark.parametrize("L", [60, 150])
def test_wide_matrix_core_level_counts(M, L):
    """The matrix-core wide Gram (sig_fo_mf.h) at the level counts the other wide tests do not reach (level 1 alone
    is the closed form; 7 and 8 levels at W = 4 / 10 columns per lane), raw levels vs the fp64 oracle."""
    from gpsig_amd import ops
    rng = np.random.default_rng(M * 100 + L)
    D = 40
    X = walks(rng, 4, L, D)
    Y = walks(rng, 3, L - 3, D)
    ref = kr.SignatureKernelRef(L * D, D, M, normalization=False)
    got = ops.sig_gram(t(X), t(Y), M).cpu().numpy()
    err = norm_rel_err(got[1:], ref.K_seq(X, Y)[1:], axis_levels=True)
    assert (err < TOL).all(), err
    sym = ops.sig_gram(t(X), None, M).cpu().numpy()
    err = norm_rel_err(sym[1:], ref.K_seq(X)[1:], axis_levels=True)
    assert (err < TOL).all(), err
