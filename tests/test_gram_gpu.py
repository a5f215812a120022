"""GPU parity: the gfx950 truncated-signature kernels vs the float64 oracle / golden fixtures.

Criterion (BASELINE.json north_star "within 1e-5 relative fp32"): norm-relative
max|K32 - K64| <= TOL * max|K64|, per level and for the summed normalised Gram.
"""
import numpy as np
import pytest
import torch

from conftest import golden, norm_rel_err
from oracle import kernels_ref as kr

pytestmark = pytest.mark.gpu
TOL = 1e-5
DEV = "cuda"


def t(x):
    return torch.as_tensor(np.asarray(x), device=DEV)


def test_rbf_gram_matches_fixture():
    import gpsig_amd
    g = golden("rbf_gram.npz")
    X, X2, M = g["X"], g["X2"], int(g["num_levels"])
    N, L, D = X.shape
    k = gpsig_amd.SignatureRBF(L * D, D, M)
    K = k.K(t(X.reshape(N, -1))).cpu().numpy()
    assert norm_rel_err(K, g["K"]) < TOL
    Kl = k.K(t(X.reshape(N, -1)), return_levels=True).cpu().numpy()
    assert (norm_rel_err(Kl[1:], g["K_levels"][1:], axis_levels=True) < TOL).all()
    Kc = k.K(t(X.reshape(N, -1)), t(X2.reshape(len(X2), -1)), return_levels=True).cpu().numpy()
    assert (norm_rel_err(Kc, g["K_cross_levels"], axis_levels=True) < TOL).all()
    # float64 in -> float64 out (drop-in dtype), symmetric, unit diagonal per level
    assert k.K(t(X.reshape(N, -1))).dtype == torch.float64
    np.testing.assert_allclose(K, K.T, atol=1e-6)
    for m in range(M + 1):
        np.testing.assert_allclose(np.diag(Kl[m]), 1.0, atol=2e-6)


def test_rbf_raw_levels_and_diag():
    import gpsig_amd
    from gpsig_amd import ops
    g = golden("rbf_gram.npz")
    X, M = g["X"], int(g["num_levels"])
    raw = ops.sig_gram(t(X), None, M).cpu().numpy()
    err = norm_rel_err(raw[1:], g["K_raw"][1:], axis_levels=True)
    assert (err < TOL).all(), err
    d = ops.sig_diag(t(X), M).cpu().numpy()
    assert (norm_rel_err(d[1:], g["Kdiag_raw"][1:], axis_levels=True) < TOL).all()
    k = gpsig_amd.SignatureRBF(X.shape[1] * X.shape[2], X.shape[2], M, normalization=False)
    assert norm_rel_err(k.Kdiag(t(X.reshape(len(X), -1))).cpu().numpy(), g["Kdiag_unnorm"]) < TOL
    kn = gpsig_amd.SignatureRBF(X.shape[1] * X.shape[2], X.shape[2], M)
    np.testing.assert_allclose(kn.Kdiag(t(X.reshape(len(X), -1))).cpu().numpy(), g["Kdiag_norm"])


def test_rbf_rough_data_with_lengthscales_and_variances():
    import gpsig_amd
    g = golden("rbf_rough.npz")
    X, M = g["X"], int(g["num_levels"])
    N, L, D = X.shape
    k = gpsig_amd.SignatureRBF(L * D, D, M, lengthscales=g["lengthscales"], variances=g["variances"])
    Kl = k.K(t(X.reshape(N, -1)), return_levels=True).cpu().numpy()
    assert (norm_rel_err(Kl, g["K_levels"], axis_levels=True) < TOL).all()


def test_linear_order_M_matches_chen_signatures():
    """esig-equivalent check (reference notebooks/signature_kernel.ipynb:52-140, 2.24e-8 in fp64)."""
    import gpsig_amd
    g = golden("linear_chen.npz")
    X, M = g["X"], int(g["num_levels"])
    N, L, D = X.shape
    k = gpsig_amd.SignatureLinear(L * D, D, M, order=M, normalization=False)
    Kl = k.K(t(X.reshape(N, -1)), return_levels=True).cpu().numpy()
    err = norm_rel_err(Kl, g["K_chen"], axis_levels=True)
    assert (err < TOL).all(), err


@pytest.mark.parametrize("order", [2, 3, 4])
@pytest.mark.parametrize("base", ["rbf", "lin"])
def test_higher_order(order, base):
    from gpsig_amd import ops
    g = golden("higher_order.npz")
    X, M = g["X"], int(g["num_levels"])
    got = ops.sig_gram(t(X), None, M, order=order, base="rbf" if base == "rbf" else "linear").cpu().numpy()
    err = norm_rel_err(got[1:], g[f"{base}_order{order}"][1:], axis_levels=True)
    assert (err < TOL).all(), err


@pytest.mark.parametrize("nl", [1, 2])
def test_lags(nl):
    import gpsig_amd
    g = golden("lags.npz")
    X, M = g["X"], int(g["num_levels"])
    N, L, D = X.shape
    k = gpsig_amd.SignatureRBF(L * D, D, M, num_lags=nl)
    Kl = k.K(t(X.reshape(N, -1)), return_levels=True).cpu().numpy()
    assert (norm_rel_err(Kl, g[f"lags{nl}_K_levels"], axis_levels=True) < TOL).all()


@pytest.mark.parametrize("base", ["rbf", "linear"])
def test_no_difference(base):
    from gpsig_amd import ops
    g = golden("nodiff.npz")
    X, M = g["X"], int(g["num_levels"])
    got = ops.sig_gram(t(X), None, M, base=base, difference=False).cpu().numpy()
    assert (norm_rel_err(got[1:], g[f"{base}_nodiff"][1:], axis_levels=True) < TOL).all()


@pytest.mark.parametrize("L", [2, 3, 17, 33, 64, 65, 81, 100, 101, 128, 129, 200, 257, 300])
def test_lengths_and_geometries(L):
    """Every lane-geometry branch (LP=16/32/64, W=4/8, and the 10-lane groups of 10 columns at 65..100
    points) incl. ragged edges, vs the oracle."""
    from gpsig_amd import ops
    rng = np.random.default_rng(L)
    N1, N2, D, M = 5, 3, 4, 4
    X = np.cumsum(rng.standard_normal((N1, L, D)), 1) / np.sqrt(L * D)
    Y = np.cumsum(rng.standard_normal((N2, max(L - 1, 2), D)), 1) / np.sqrt(L * D)
    ref = kr.SignatureKernelRef(L * D, D, M, normalization=False)
    exp = ref.K_seq(X, Y)
    got = ops.sig_gram(t(X), t(Y), M).cpu().numpy()
    assert (norm_rel_err(got[1:], exp[1:], axis_levels=True) < TOL).all()
    sym = ops.sig_gram(t(X), None, M).cpu().numpy()
    exps = ref.K_seq(X)
    assert (norm_rel_err(sym[1:], exps[1:], axis_levels=True) < TOL).all()


@pytest.mark.parametrize("D", [1, 2, 3, 5, 6, 7, 8, 11, 16, 20])
@pytest.mark.parametrize("M", [1, 2, 6, 8])
def test_channels_and_levels(D, M):
    from gpsig_amd import ops
    rng = np.random.default_rng(100 * D + M)
    X = np.cumsum(rng.standard_normal((6, 24, D)), 1) / np.sqrt(24 * D)
    exp = kr.SignatureKernelRef(24 * D, D, M, normalization=False).K_seq(X)
    got = ops.sig_gram(t(X), None, M).cpu().numpy()
    assert (norm_rel_err(got[1:], exp[1:], axis_levels=True) < TOL).all()


@pytest.mark.parametrize("N", [1, 5, 6, 7, 23, 61])
def test_ten_lane_groups_tiles(N):
    """The 10-lane geometry (6 pairs per wave, tile rows starting at B tile floor(4r/6)): every pair of
    the upper triangle is evaluated exactly once and mirrored, for N around the tile sizes; D = 5, M = 5,
    L = 100 (C2's shape), raw levels and the normalised sum, against the oracle."""
    from gpsig_amd import ops
    rng = np.random.default_rng(7 * N)
    L, D, M = 100, 5, 5
    X = np.cumsum(rng.standard_normal((N, L, D)), 1) / np.sqrt(L * D)
    ref = kr.SignatureKernelRef(L * D, D, M, normalization=False)
    got = ops.sig_gram(t(X), None, M).cpu().numpy()
    assert (norm_rel_err(got[1:], ref.K_seq(X)[1:], axis_levels=True) < TOL).all()
    # row windows of the upper-triangle launch (the distributed row shards): tile_base from the exact prefix
    if N >= 7:
        full = torch.as_tensor(got, device=DEV)
        for r0, r1 in [(0, 3), (3, N // 2), (N // 2, N)]:
            up = torch.zeros(M + 1, r1 - r0, N, device=DEV)
            ops.sig_gram(t(X), None, M, rows=(r0, r1), out=up)
            mask = torch.arange(N, device=DEV)[None, :] >= torch.arange(r0, r1, device=DEV)[:, None]
            torch.testing.assert_close(up[:, mask], full[:, r0:r1][:, mask], rtol=1e-5, atol=1e-6)


def test_row_windows_and_rect_tiles():
    """Row sharding windows: (rows, out_row0) of both pair modes reproduce the full Gram."""
    from gpsig_amd import ops
    import gpsig_amd._lib as L
    rng = np.random.default_rng(5)
    X = torch.as_tensor(np.cumsum(rng.standard_normal((37, 30, 3)), 1) / 10, device=DEV, dtype=torch.float32)
    full = ops.sig_gram(X, None, 4)
    for r0, r1 in [(0, 9), (9, 21), (21, 37), (3, 4)]:
        part = ops.sig_gram(X, X, 4, rows=(r0, r1))
        torch.testing.assert_close(part, full[:, r0:r1], rtol=1e-5, atol=1e-6)
        up = torch.zeros(5, r1 - r0, 37, device=DEV)
        ops.sig_gram(X, None, 4, rows=(r0, r1), out=up)
        mask = torch.arange(37, device=DEV)[None, :] >= torch.arange(r0, r1, device=DEV)[:, None]
        torch.testing.assert_close(up[:, mask], full[:, r0:r1][:, mask], rtol=1e-5, atol=1e-6)


def test_full_size_properties_headline():
    """At the headline sequence shape (L=128, D=5, M=5): a 256-row subsample vs the oracle, plus
    size-independent properties of the full normalised Gram (symmetry, unit diagonal, PSD)."""
    import gpsig_amd
    rng = np.random.default_rng(0)
    N, L, D, M = 512, 128, 5, 5
    X = np.cumsum(rng.standard_normal((N, L, D)), 1) / np.sqrt(L * D)
    k = gpsig_amd.SignatureRBF(L * D, D, M)
    Xt = torch.as_tensor(X.reshape(N, -1), device=DEV, dtype=torch.float32)
    K = k.K(Xt).double()
    torch.testing.assert_close(K, K.T, rtol=0, atol=1e-6)
    torch.testing.assert_close(torch.diagonal(K), torch.full((N,), 6.0, dtype=K.dtype, device=DEV), rtol=0, atol=1e-5)
    assert torch.linalg.eigvalsh(K).min().item() > -1e-4
    idx = np.arange(0, N, 64)
    ref = kr.SignatureKernelRef(L * D, D, M)
    exp = ref.K(X[idx].reshape(len(idx), -1), X[:40].reshape(40, -1))
    got = k.K(Xt[idx], Xt[:40]).cpu().numpy()
    assert norm_rel_err(got, exp) < TOL


@pytest.mark.parametrize("case", ["order", "levels", "length"])
def test_unsupported_configurations_raise(case):
    """Configurations outside the compiled instantiations fail loudly (GpsigError), never silently."""
    import gpsig_amd
    from gpsig_amd import ops
    # order 9 > the higher-order kernel's 8; 9 levels; LDS carry of the column blocks > 160 KiB
    D, M, L, order = {"order": (3, 10, 10, 9), "levels": (3, 9, 10, 1), "length": (4, 3, 6000, 1)}[case]
    X = torch.zeros((2, L, D), device=DEV)
    with pytest.raises(gpsig_amd.GpsigError):
        ops.sig_gram(X, None, M, order=order)


@pytest.mark.parametrize("L,D,M", [(20, 3, 4), (50, 5, 5), (100, 5, 5), (128, 8, 6), (200, 2, 3)])
def test_mfma_seed_arm_matches_valu_arm(L, D, M):
    """The matrix-core seed (GPSIG_BASE_SEED_MFMA, v_mfma_f32_4x4x1_16b_f32 for <y_j, dx_i> and
    <dy_j, dx_i>) is the A/B arm of the packed-VALU seed: same cells (an MFMA is a k-ordered fp32 fma
    chain), so the Gram agrees with the VALU arm to rounding of the recursion's association and with the
    oracle within the north_star tolerance, for the Gram, the cross Gram and the diagonal."""
    from gpsig_amd import _lib as Lb
    from gpsig_amd import ops
    rng = np.random.default_rng(L + D)
    N = 12
    X = np.cumsum(rng.standard_normal((N, L, D)), 1) / np.sqrt(L * D)
    Y = np.cumsum(rng.standard_normal((7, L - 3, D)), 1) / np.sqrt(L * D)
    mf = Lb.BASE_RBF | Lb.BASE_SEED_MFMA
    ref = kr.SignatureKernelRef(L * D, D, M, normalization=False)
    for Yin in (None, Y):
        a = ops.sig_gram(t(X), None if Yin is None else t(Yin), M, base=mf).cpu().numpy()
        v = ops.sig_gram(t(X), None if Yin is None else t(Yin), M).cpu().numpy()
        e = ref.K_seq(X, X if Yin is None else Yin)
        assert (norm_rel_err(a[1:], v[1:], axis_levels=True) < 5e-6).all()
        assert (norm_rel_err(a[1:], e[1:], axis_levels=True) < TOL).all()
    dm = ops.sig_diag(t(X), M, base=mf).cpu().numpy()
    dv = ops.sig_diag(t(X), M).cpu().numpy()
    assert (norm_rel_err(dm[1:], dv[1:], axis_levels=True) < 5e-6).all()


@pytest.mark.parametrize("N,L,D,M", [(70, 50, 3, 4), (40, 128, 5, 5), (36, 100, 8, 6)])
def test_split_diagnostic_matches_fused(N, L, D, M):
    """The split design of SURVEY.md 8d (GPSIG_GRAM_SPLIT: producer writes the cells dM to HBM, consumer
    streams them through the recursion) gives the fused kernel's Gram: same cell instructions, same
    recursion; K(X) (upper pairs, mirror) and K(X, X2), raw levels and the fused normalised sum."""
    from gpsig_amd import _lib as Lb
    from gpsig_amd import ops

    def walks(n, seed):
        rng = np.random.default_rng(seed)
        return np.cumsum(rng.standard_normal((n, L, D)), axis=1) / np.sqrt(L * D)
    X = torch.as_tensor(walks(N, 7), device=DEV, dtype=torch.float32)
    Y = torch.as_tensor(walks(N // 2 + 3, 8), device=DEV, dtype=torch.float32)
    for Yt in (None, Y):
        ref = ops.sig_gram(X, Yt, M, base=Lb.BASE_RBF)
        got = ops.sig_gram(X, Yt, M, base=Lb.BASE_RBF | Lb.GRAM_SPLIT)
        torch.testing.assert_close(got, ref, rtol=0, atol=1e-6 * float(ref.abs().max()))


def test_empty_and_single_sequence_batches():
    """Edge batches: no sequences (empty outputs of the right shapes, as the reference's graph), one
    sequence, one increment (L = 2), a constant path (zero increments: only level 0 survives)."""
    import gpsig_amd
    L, D, M = 12, 3, 4
    k = gpsig_amd.SignatureRBF(L * D, D, M)
    kp = gpsig_amd.UntruncSignatureKernel(L * D, D, order=1)
    E = torch.zeros((0, L * D), device=DEV, dtype=torch.float64)
    X1 = torch.as_tensor(np.cumsum(np.random.default_rng(3).standard_normal((1, L, D)), 1).reshape(1, -1) * 0.2,
                         device=DEV)
    assert k.K(E).shape == (0, 0) and k.Kdiag(E).shape == (0,)
    assert k.K(E, X1).shape == (0, 1) and k.K(X1, E).shape == (1, 0)
    assert kp.Kdiag(E).shape == (0,) and kp.K(E).shape == (0, 0)
    Z = torch.zeros((M * (M + 1) // 2, 2, D), device=DEV, dtype=torch.float64)
    assert k.K_tens_vs_seq(Z, E).shape == (2, 0)
    ref = kr.SignatureKernelRef(L * D, D, M)
    np.testing.assert_allclose(k.K(X1).cpu().numpy(), ref.K(X1.cpu().numpy()), rtol=1e-5)
    # one increment and a constant path
    for X in (np.random.default_rng(4).standard_normal((3, 2, D)) * 0.3, np.ones((2, 5, D))):
        n, l, _ = X.shape
        kk = gpsig_amd.SignatureRBF(l * D, D, M, normalization=False)
        rr = kr.SignatureKernelRef(l * D, D, M, normalization=False)
        got = kk.K(torch.as_tensor(X.reshape(n, -1), device=DEV), return_levels=True).cpu().numpy()
        exp = rr.K(X.reshape(n, -1), return_levels=True)
        np.testing.assert_allclose(got, exp, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("scale,jumps,D", [(0.02, False, 3), (0.15, False, 3), (0.05, True, 3), (0.03, True, 8)])
def test_seed_regimes(scale, jumps, D):
    """The RBF seed's regimes (sig_common.h RbfSeedPk::row) vs the oracle: small increments (expm1(c) by
    the cubic under the |dx||dy| < 1/16 bound), medium ones (bound fails: the quintic), and rows with a few
    large jumps (slow rows: cells outside the polynomial range take the corner difference, the in-range
    cells after them re-evaluate their chained expm1(p)); D = 8 re-reads the points of column pairs >= 1
    on anchor rows (YG)."""
    import gpsig_amd
    rng = np.random.default_rng(11)
    N, L, M = 24, 40, 4
    inc = rng.standard_normal((N, L, D)) * scale
    if jumps:
        inc[:, ::9, :] *= 25.0
    X = np.cumsum(inc, 1)
    k = gpsig_amd.SignatureRBF(L * D, D, M)
    got = k.K(t(X.reshape(N, -1)), return_levels=True).cpu().numpy()
    exp = kr.SignatureKernelRef(L * D, D, M).K(X.reshape(N, -1), return_levels=True)
    assert (norm_rel_err(got, exp, axis_levels=True) < TOL).all()


@pytest.mark.parametrize("scale,D,M", [(0.01, 5, 5), (0.06, 5, 5), (0.03, 8, 6)])
def test_anchor_spans_long_sequences(scale, D, M):
    """Sequences of 480 points: the packed recurrences (k by (1 + expm1(p)), Eq by the expm1 chain) run for
    GPSIG_PK_ANCHOR = 128 rows between exact re-evaluations, four spans per pair here; the accumulated
    rounding must stay inside the parity tolerance against the oracle (small and medium increments, and
    D = 8, whose column pairs >= 1 re-read their points on anchor rows)."""
    import gpsig_amd
    rng = np.random.default_rng(23)
    N, L = 5, 480
    X = np.cumsum(rng.standard_normal((N, L, D)) * scale, 1)
    k = gpsig_amd.SignatureRBF(L * D, D, M)
    got = k.K(t(X.reshape(N, -1)), return_levels=True).cpu().numpy()
    exp = kr.SignatureKernelRef(L * D, D, M).K(X.reshape(N, -1), return_levels=True)
    assert (norm_rel_err(got, exp, axis_levels=True) < TOL).all()
