"""GPU parity of higher-order gradients: SignatureLinear(order = num_levels) -- the exact signature
kernel, trained through TF autodiff of signature_algs.py:37-74 by benchmarks/models/train_gpsig_vosf.py:102
-- differentiated through the signature features (ops.sig_gram_ho_vjp -> gpsig_signature_vjp), vs fp64
autodiff of the reference graph (oracle/autodiff_ref.py higher_order), on the linear_chen.npz shapes
(N = 16, L = 20, D = 3, M = 5).  Criterion as tests/test_grad_gpu.py (norm-relative, GTOL)."""
import numpy as np
import pytest
import torch

from conftest import golden, norm_rel_err
from oracle import autodiff_ref as ar

pytestmark = pytest.mark.gpu
GTOL = 1e-5
DEV = "cuda"


@pytest.mark.parametrize("normalization", [True, False])
@pytest.mark.parametrize("cross", [False, True])
@pytest.mark.parametrize("return_levels", [False, True])
def test_higher_order_signature_kernel_gradient(normalization, cross, return_levels):
    import gpsig_amd
    g = golden("linear_chen.npz")
    X = g["X"]
    N, L, D = X.shape
    M = int(g["num_levels"])
    X2 = np.cumsum(np.random.default_rng(3).standard_normal((7, L, D)), 1) / np.sqrt(L * D) if cross else None
    rng = np.random.default_rng(4)
    G = rng.standard_normal(((M + 1,) if return_levels else ()) + (N, 7 if cross else N))
    ls = np.array([0.7, 1.3, 1.0])
    var = np.linspace(0.5, 1.5, M + 1)
    k = gpsig_amd.SignatureLinear(L * D, D, M, order=M, normalization=normalization)
    k.lengthscales = torch.tensor(ls, device=DEV, requires_grad=True)
    k.variances = torch.tensor(var, device=DEV, requires_grad=True)
    Xt = torch.tensor(X.reshape(N, -1), device=DEV, requires_grad=True)
    X2t = None if X2 is None else torch.tensor(X2.reshape(7, -1), device=DEV, requires_grad=True)
    K = k.K(Xt, X2t, return_levels=return_levels)
    (K * torch.as_tensor(G, device=DEV)).sum().backward()

    Xr = torch.tensor(X, requires_grad=True)
    X2r = None if X2 is None else torch.tensor(X2, requires_grad=True)
    lr = torch.tensor(ls, requires_grad=True)
    vr = torch.tensor(var, requires_grad=True)
    Kr = ar.K(Xr / lr, None if X2r is None else X2r / lr, M, base="linear", normalization=normalization, scale=vr,
              return_levels=return_levels, order=M)
    (Kr * torch.tensor(G)).sum().backward()
    assert norm_rel_err(K.detach().cpu().numpy(), Kr.detach().numpy()) < 1e-5
    assert norm_rel_err(Xt.grad.reshape(X.shape).cpu().numpy(), Xr.grad.numpy()) < GTOL
    if cross:
        assert norm_rel_err(X2t.grad.reshape(X2.shape).cpu().numpy(), X2r.grad.numpy()) < GTOL
    # The sequences' and variances' gradients are held to the plain GTOL against fp64 autodiff of the reference
    # graph evaluated at the fp32-rounded scaled inputs the kernels receive (x / l -> fp32).
    Xq = _fp32_scaled(X, ls)
    X2q = None if X2 is None else _fp32_scaled(X2, ls)
    xs = torch.tensor(Xq, requires_grad=True)
    x2s = None if X2q is None else torch.tensor(X2q, requires_grad=True)
    vq = torch.tensor(var, requires_grad=True)
    Kq = ar.K(xs, x2s, M, base="linear", normalization=normalization, scale=vq, return_levels=return_levels, order=M)
    (Kq * torch.tensor(G)).sum().backward()
    assert norm_rel_err(Xt.grad.reshape(X.shape).cpu().numpy(), xs.grad.numpy() / ls) < GTOL
    if cross:
        assert norm_rel_err(X2t.grad.reshape(X2.shape).cpu().numpy(), x2s.grad.numpy() / ls) < GTOL
    assert norm_rel_err(k.variances.grad.cpu().numpy(), vq.grad.numpy()) < GTOL
    # dLoss/dl_c = -sum_i x_ic dLoss/dx_ic / l_c contracts every point's gradient along the scaling direction of
    # channel c; the normalised kernel is invariant to a common scaling of all channels (sum_c l_c dLoss/dl_c = 0),
    # so the small components are cancellations of the large ones.  The backward evaluates those contractions in
    # closed form from the signatures (autograd._scaling_contraction, round 6; the fp32 VJP alone read 1.006e-5 at
    # [True-False-True]), so the plain GTOL holds against both references.
    gl_q = -(X * xs.grad.numpy()).reshape(-1, D).sum(0) / ls ** 2
    if cross:
        gl_q = gl_q - (X2 * x2s.grad.numpy()).reshape(-1, D).sum(0) / ls ** 2
    gl = k.lengthscales.grad.cpu().numpy()
    assert norm_rel_err(gl, gl_q) < GTOL
    assert norm_rel_err(gl, lr.grad.numpy()) < GTOL


def _fp32_scaled(X, ls):
    """The scaled sequences as the kernels receive them: x / l in float64 (kernels.py:344-365, the host
    scaling) rounded to float32 (ops._f32), back in float64 for the fp64 reference."""
    return (X / ls).astype(np.float32).astype(np.float64)


def test_higher_order_diag_and_norms_gradient():
    """Kdiag (unnormalised) and K_norms of the exact signature kernel (the VOSF Kuu_Kuf_Kff terms,
    inducing_variables_vosf.py:200-208)."""
    import gpsig_amd
    g = golden("linear_chen.npz")
    X = g["X"][:6]
    N, L, D = X.shape
    M = int(g["num_levels"])
    G = np.random.default_rng(5).standard_normal(N)
    k = gpsig_amd.SignatureLinear(L * D, D, M, order=M, normalization=False)
    Xt = torch.tensor(X.reshape(N, -1), device=DEV, requires_grad=True)
    (k.Kdiag(Xt) * torch.as_tensor(G, device=DEV)).sum().backward()
    Xr = torch.tensor(X, requires_grad=True)
    (ar.k_seq_diag(Xr, M, "linear", True, order=M).sum(0) * torch.tensor(G)).sum().backward()
    assert norm_rel_err(Xt.grad.reshape(X.shape).cpu().numpy(), Xr.grad.numpy()) < GTOL
    kn = gpsig_amd.SignatureLinear(L * D, D, M, order=M)
    Xt2 = torch.tensor(X.reshape(N, -1), device=DEV, requires_grad=True)
    _, Kun = kn.K_norms(Xt2)
    (Kun * torch.as_tensor(np.random.default_rng(6).standard_normal(Kun.shape), device=DEV)).sum().backward()
    assert torch.isfinite(Xt2.grad).all()


def test_unsupported_higher_order_gradients_raise():
    """Orders past the VJP kernels (min(order, num_levels) = 7; order 6 at 7 levels, whose slab does not fit the
    LDS) that are not the exact linear kernel evaluate forward; their backward raises."""
    import gpsig_amd
    X = torch.tensor(golden("linear_chen.npz")["X"][:4].reshape(4, -1), device=DEV, requires_grad=True)
    for k in (gpsig_amd.SignatureRBF(60, 3, 7, order=7), gpsig_amd.SignatureLinear(60, 3, 7, order=6)):
        K = k.K(X)
        with pytest.raises(NotImplementedError):
            K.sum().backward()


def _walks(n, l, d, seed):
    return np.cumsum(np.random.default_rng(seed).standard_normal((n, l, d)), 1) / np.sqrt(l * d)


@pytest.mark.parametrize("L,D,M,order,base", [
    (12, 3, 3, 2, "rbf"), (30, 4, 5, 2, "linear"), (40, 46, 4, 2, "rbf"), (200, 3, 4, 2, "rbf"),
    (25, 3, 4, 3, "rbf"), (20, 2, 5, 3, "linear"), (18, 3, 3, 3, "linear"), (16, 2, 8, 2, "rbf"),
    # the LDS-state kernel (csrc/sig_ho_bwd_lds.h): orders 4-5, order 3 past 5 levels, 257-512 points
    (25, 3, 5, 4, "rbf"), (20, 2, 5, 5, "linear"), (22, 3, 6, 3, "rbf"), (16, 2, 7, 5, "rbf"),
    (19, 4, 4, 4, "linear"), (300, 3, 4, 2, "rbf"), (270, 2, 5, 5, "linear"), (400, 3, 5, 4, "rbf"),
    # 257-509 points: one pair over the 4 SIMDs of a CU (csrc/sig_ho_bwd_split.h), 3 and 4 column blocks
    (381, 3, 4, 3, "rbf"), (509, 2, 3, 2, "linear"),
    # effective order 6 (6 levels, up to 256 points: the LDS-state kernel at W = 4)
    (20, 3, 6, 6, "rbf"), (18, 2, 6, 7, "rbf"), (200, 2, 6, 6, "linear"),
    # 510-512 points at levels the 8-wave form does not hold: the one-wave W = 8 kernel
    (511, 2, 7, 3, "linear"),
])
def test_higher_order_vjp_kernel_raw_levels(L, D, M, order, base):
    """gpsig_sig_gram_vjp_ho (csrc/sig_ho_bwd.h, sig_ho_bwd_lds.h) against fp64 autodiff of
    signature_kern_higher_order (signature_algs.py:37-74, restated in oracle/autodiff_ref.py): per-level
    upstream gradients, cross K(X, Y), symmetric K(X) (UPPER pairs) and the diagonal."""
    from gpsig_amd import ops
    X, Y = _walks(3, L, D, L + order), _walks(4, L - 3, D, L + order + 1)
    G = np.random.default_rng(7).standard_normal((M + 1, 3, 4))
    Gs = np.random.default_rng(8).standard_normal((M + 1, 3, 3))
    Gd = np.random.default_rng(9).standard_normal((M + 1, 3))
    Xt, Yt = torch.tensor(X, device=DEV, dtype=torch.float32), torch.tensor(Y, device=DEV, dtype=torch.float32)
    gX, gY = ops.sig_gram_vjp(Xt, Yt, M, torch.tensor(G, device=DEV), base=base, gout_levels=True, order=order)
    Xr, Yr = torch.tensor(X, requires_grad=True), torch.tensor(Y, requires_grad=True)
    (ar.k_seq(Xr, Yr, M, base, order=order) * torch.tensor(G)).sum().backward()
    assert norm_rel_err(gX.cpu().numpy(), Xr.grad.numpy()) < GTOL
    assert norm_rel_err(gY.cpu().numpy(), Yr.grad.numpy()) < GTOL
    gS, _ = ops.sig_gram_vjp(Xt, None, M, torch.tensor(Gs, device=DEV), base=base, gout_levels=True, order=order)
    Xr = torch.tensor(X, requires_grad=True)
    (ar.k_seq(Xr, Xr, M, base, order=order) * torch.tensor(Gs)).sum().backward()
    assert norm_rel_err(gS.cpu().numpy(), Xr.grad.numpy()) < GTOL
    gD, _ = ops.sig_gram_vjp(Xt, None, M, torch.tensor(Gd, device=DEV), base=base, diag=True, order=order)
    Xr = torch.tensor(X, requires_grad=True)
    (ar.k_seq_diag(Xr, M, base, order=order) * torch.tensor(Gd)).sum().backward()
    assert norm_rel_err(gD.cpu().numpy(), Xr.grad.numpy()) < GTOL


@pytest.mark.parametrize("cross", [False, True])
@pytest.mark.parametrize("base", ["rbf", "linear"])
def test_higher_order_normalised_K_gradient(cross, base):
    """SignatureKernel(order=2).K normalised, through autograd: sequences, lengthscales and variances, vs
    fp64 autodiff of the reference graph (kernels.py:402-477 over signature_algs.py:37-74)."""
    import gpsig_amd
    N, L, D, M = 5, 24, 3, 4
    X = _walks(N, L, D, 11)
    X2 = _walks(3, L + 4, D, 12) if cross else None
    G = np.random.default_rng(13).standard_normal((N, 3 if cross else N))
    ls = np.array([0.8, 1.2, 1.0])
    var = np.linspace(0.5, 1.5, M + 1)
    cls = gpsig_amd.SignatureRBF if base == "rbf" else gpsig_amd.SignatureLinear
    k = cls(L * D, D, M, order=2)
    k.lengthscales = torch.tensor(ls, device=DEV, requires_grad=True)
    k.variances = torch.tensor(var, device=DEV, requires_grad=True)
    Xt = torch.tensor(X.reshape(N, -1), device=DEV, requires_grad=True)
    X2t = None if X2 is None else torch.tensor(X2.reshape(3, -1), device=DEV, requires_grad=True)
    K = k.K(Xt, X2t)
    (K * torch.as_tensor(G, device=DEV)).sum().backward()
    Xr = torch.tensor(X, requires_grad=True)
    X2r = None if X2 is None else torch.tensor(X2, requires_grad=True)
    lr, vr = torch.tensor(ls, requires_grad=True), torch.tensor(var, requires_grad=True)
    Kr = ar.K(Xr / lr, None if X2r is None else X2r / lr, M, base=base, scale=vr, order=2)
    (Kr * torch.tensor(G)).sum().backward()
    assert norm_rel_err(K.detach().cpu().numpy(), Kr.detach().numpy()) < 1e-5
    assert norm_rel_err(Xt.grad.reshape(X.shape).cpu().numpy(), Xr.grad.numpy()) < GTOL
    if cross:
        assert norm_rel_err(X2t.grad.reshape(X2.shape).cpu().numpy(), X2r.grad.numpy()) < GTOL
    assert norm_rel_err(k.lengthscales.grad.cpu().numpy(), lr.grad.numpy()) < GTOL
    assert norm_rel_err(k.variances.grad.cpu().numpy(), vr.grad.numpy()) < GTOL


def test_higher_order_vjp_unsupported_raises():
    """min(order, M) = 7, order 6 at 7 levels or past 256 points, sequences past 1017 points, (order, levels)
    whose multiplier slab does not fit the LDS at 257-509 points or whose state does not fit the 8-wave form past
    509 are outside the VJP kernels: the error names the entry point (autograd then uses the signature-feature
    path for the exact linear kernel, or raises)."""
    from gpsig_amd import _lib as Lb
    from gpsig_amd import ops
    for L, M, order in ((10, 7, 7), (10, 7, 6), (300, 6, 6), (1100, 3, 2), (700, 8, 2), (600, 6, 4), (300, 6, 4),
                        (300, 8, 3)):
        X = torch.zeros((2, L, 2), device=DEV)
        with pytest.raises(Lb.GpsigError):
            ops.sig_gram_vjp(X, None, M, torch.zeros((M + 1, 2, 2), device=DEV), gout_levels=True, order=order)


@pytest.mark.parametrize("normalization", [True, False])
def test_higher_order_long_sequences_gradient(normalization):
    """SignatureLinear(num_levels=5, order=5) at the VOSF trainer's sequence shape (d = 24, L = 500,
    benchmarks/models/train_gpsig_vosf.py:102): K (symmetric and cross) and Kdiag gradients through the
    LDS-state VJP kernel (W = 8 columns per lane), vs fp64 autodiff of the reference graph, plain
    norm-relative criterion on the gradient itself.

    Normalised, the Gram term and the diagonal term of the gradient cancel ~270x (the normalised kernel is
    scale-invariant in each sequence): autograd.SigGram folds the diagonal terms into the weights of the
    diagonal pairs of ONE VJP launch (K(X, X2): over the concatenation [X; X2]), and the kernel accumulates
    its adjoint column sums in fp64 (sig_ho_bwd_lds.h); DESIGN.md 2.3, tools/diag_ho_grad.py."""
    import gpsig_amd
    from gpsig_amd import ops
    N, L, D, M = 2, 500, 24, 5
    assert ops.ho_vjp_supported(L, M, M, "linear")
    X, X2 = _walks(N, L, D, 21), _walks(2, L - 20, D, 22)
    k = gpsig_amd.SignatureLinear(L * D, D, M, order=M, normalization=normalization)
    Xt = torch.tensor(X.reshape(N, -1), device=DEV, dtype=torch.float32, requires_grad=True)
    X2t = torch.tensor(X2.reshape(2, -1), device=DEV, dtype=torch.float32, requires_grad=True)
    G, G2 = np.random.default_rng(23).standard_normal((N, N)), np.random.default_rng(24).standard_normal((N, 2))
    Gd = np.random.default_rng(25).standard_normal(N)
    (k.K(Xt) * torch.as_tensor(G, device=DEV)).sum().backward()
    gs = Xt.grad.reshape(X.shape).cpu().numpy()
    Xt.grad = None
    (k.K(Xt, X2t) * torch.as_tensor(G2, device=DEV)).sum().backward()
    gc, gc2 = Xt.grad.reshape(X.shape).cpu().numpy(), X2t.grad.reshape(X2.shape).cpu().numpy()

    def ref(Y, Gm):
        Xr = torch.tensor(X, requires_grad=True)
        Yr = None if Y is None else torch.tensor(Y, requires_grad=True)
        (ar.K(Xr, Yr, M, base="linear", normalization=normalization, order=M) * torch.tensor(Gm)).sum().backward()
        return [Xr.grad.numpy()] + ([] if Y is None else [Yr.grad.numpy()])

    (rs,) = ref(None, G)
    assert norm_rel_err(gs, rs) < GTOL
    rc, rc2 = ref(X2, G2)
    assert norm_rel_err(gc, rc) < GTOL
    assert norm_rel_err(gc2, rc2) < GTOL
    if not normalization:
        Xt.grad = None  # the unnormalised diagonal (normalised it is the constant sum of the variances)
        (k.Kdiag(Xt) * torch.as_tensor(Gd, device=DEV)).sum().backward()
        gd = Xt.grad.reshape(X.shape).cpu().numpy()
        Xr = torch.tensor(X, requires_grad=True)
        (ar.k_seq_diag(Xr, M, "linear", True, order=M).sum(0) * torch.tensor(Gd)).sum().backward()
        assert norm_rel_err(gd, Xr.grad.numpy()) < GTOL


@pytest.mark.parametrize("L1,L2,D", [(2, 2, 3), (3, 40, 2), (2, 9, 40)])
def test_higher_order_vjp_short_sequences(L1, L2, D):
    """Order-2 VJP with one- and two-increment sequences (the recursion's shortest grids), cross pairs."""
    from gpsig_amd import ops
    M = 3
    X, Y = _walks(2, L1, D, L1 + L2), _walks(3, L2, D, L1 + L2 + 1)
    G = np.random.default_rng(5).standard_normal((M + 1, 2, 3))
    gX, gY = ops.sig_gram_vjp(torch.tensor(X, device=DEV, dtype=torch.float32),
                              torch.tensor(Y, device=DEV, dtype=torch.float32), M,
                              torch.tensor(G, device=DEV), base="rbf", gout_levels=True, order=2)
    Xr, Yr = torch.tensor(X, requires_grad=True), torch.tensor(Y, requires_grad=True)
    (ar.k_seq(Xr, Yr, M, "rbf", order=2) * torch.tensor(G)).sum().backward()
    assert norm_rel_err(gX.cpu().numpy(), Xr.grad.numpy()) < GTOL
    assert norm_rel_err(gY.cpu().numpy(), Yr.grad.numpy()) < GTOL


@pytest.mark.parametrize("L,base,order,M", [(256, "linear", 2, 3), (256, "rbf", 3, 4), (400, "linear", 3, 4),
                                            (400, "rbf", 4, 4)])
def test_higher_order_vjp_unit_scale_long(L, base, order, M):
    """The reverse sweep recovers the forward column sums by subtraction, CB_m(i) = CB_m(i+1) - colsum R_m(i),
    over every row: unit-scale increments (walks of N(0, 1) steps, not 1/sqrt(L d)) at 256 (register kernel)
    and 400 points (LDS-state kernel), cross pairs, per-level upstream gradients, vs fp64 autodiff."""
    from gpsig_amd import ops
    D = 2
    rng = np.random.default_rng(L + order)
    X = np.cumsum(rng.standard_normal((2, L, D)), 1) * (0.1 if base == "rbf" else 1.0)
    Y = np.cumsum(rng.standard_normal((2, L - 7, D)), 1) * (0.1 if base == "rbf" else 1.0)
    G = rng.standard_normal((M + 1, 2, 2))
    gX, gY = ops.sig_gram_vjp(torch.tensor(X, device=DEV, dtype=torch.float32),
                              torch.tensor(Y, device=DEV, dtype=torch.float32), M, torch.tensor(G, device=DEV),
                              base=base, gout_levels=True, order=order)
    Xr, Yr = torch.tensor(X, requires_grad=True), torch.tensor(Y, requires_grad=True)
    (ar.k_seq(Xr, Yr, M, base, order=order) * torch.tensor(G)).sum().backward()
    assert norm_rel_err(gX.cpu().numpy(), Xr.grad.numpy()) < GTOL
    assert norm_rel_err(gY.cpu().numpy(), Yr.grad.numpy()) < GTOL


def test_higher_order_vjp_chunked_upper_vs_rect():
    """The LDS-state VJP over several chunks of x-rows (N = 64 sequences of 300 points: the point-weight tile
    budget holds 44 rows per chunk): the symmetric K(X) gradient (UPPER pairs, one workgroup per pair from
    each chunk's row window) equals the cross K(X, Y) one with Y a copy of X, dK/dX + dK/dY (RECT pairs)."""
    from gpsig_amd import ops
    N, L, D, M, order = 64, 300, 3, 4, 3
    X = _walks(N, L, D, 90)
    G = np.random.default_rng(91).standard_normal((M + 1, N, N))
    Xt = torch.tensor(X, device=DEV, dtype=torch.float32)
    Gt = torch.tensor(G, device=DEV, dtype=torch.float32)
    gS, _ = ops.sig_gram_vjp(Xt, None, M, Gt, base="rbf", gout_levels=True, order=order)
    gX, gY = ops.sig_gram_vjp(Xt, Xt.clone(), M, Gt, base="rbf", gout_levels=True, order=order)
    assert norm_rel_err(gS.cpu().numpy(), (gX + gY).cpu().numpy()) < 1e-5


@pytest.mark.parametrize("L,M,order,base", [(300, 4, 2, "rbf"), (500, 5, 5, "linear"), (390, 3, 3, "rbf")])
def test_higher_order_vjp_split_matches_one_wave_kernel(L, M, order, base, monkeypatch):
    """The 4-wave split of the LDS-state VJP (sig_ho_bwd_split.h) against the one-wave kernel it replaces
    (GPSIG_HO_SPLIT=0): the same recursion with the column scans combined across blocks, so the gradients
    agree to fp32 rounding of the scans; UPPER, RECT and DIAG pairs."""
    from gpsig_amd import ops
    D = 5
    X, Y = _walks(3, L, D, L + 1), _walks(2, L - 7, D, L + 2)
    G = np.random.default_rng(17).standard_normal((M + 1, 3, 2))
    Gs = np.random.default_rng(18).standard_normal((M + 1, 3, 3))
    Gd = np.random.default_rng(19).standard_normal((M + 1, 3))
    Xt, Yt = torch.tensor(X, device=DEV, dtype=torch.float32), torch.tensor(Y, device=DEV, dtype=torch.float32)

    def grads():
        out = list(ops.sig_gram_vjp(Xt, Yt, M, torch.tensor(G, device=DEV), base=base, gout_levels=True,
                                    order=order))
        out.append(ops.sig_gram_vjp(Xt, None, M, torch.tensor(Gs, device=DEV), base=base, gout_levels=True,
                                    order=order)[0])
        out.append(ops.sig_gram_vjp(Xt, None, M, torch.tensor(Gd, device=DEV), base=base, diag=True,
                                    order=order)[0])
        return [g.cpu().numpy() for g in out]

    split = grads()
    monkeypatch.setenv("GPSIG_HO_SPLIT", "0")
    one = grads()
    for g, r in zip(split, one):
        assert norm_rel_err(g, r) < 2e-6


@pytest.mark.parametrize("L,D,M,order,base", [(700, 3, 4, 3, "rbf"), (1017, 2, 3, 2, "linear"), (600, 3, 5, 5, "rbf"),
                                               (510, 2, 5, 4, "linear")])
def test_higher_order_vjp_past_512_points(L, D, M, order, base):
    """510-1017 points: one pair over 8 waves (2 per SIMD), the multiplier slab in a global-memory region of the
    workspace (csrc/sig_ho_bwd_split.h, NW = 8), against fp64 autodiff of signature_kern_higher_order on cross,
    symmetric and diagonal pairs."""
    from gpsig_amd import ops
    X, Y = _walks(2, L, D, L + order), _walks(2, L - 5, D, L + order + 1)
    G = np.random.default_rng(7).standard_normal((M + 1, 2, 2))
    Gd = np.random.default_rng(9).standard_normal((M + 1, 2))
    Xt, Yt = torch.tensor(X, device=DEV, dtype=torch.float32), torch.tensor(Y, device=DEV, dtype=torch.float32)
    gX, gY = ops.sig_gram_vjp(Xt, Yt, M, torch.tensor(G, device=DEV), base=base, gout_levels=True, order=order)
    Xr, Yr = torch.tensor(X, requires_grad=True), torch.tensor(Y, requires_grad=True)
    (ar.k_seq(Xr, Yr, M, base, order=order) * torch.tensor(G)).sum().backward()
    assert norm_rel_err(gX.cpu().numpy(), Xr.grad.numpy()) < GTOL
    assert norm_rel_err(gY.cpu().numpy(), Yr.grad.numpy()) < GTOL
    gS, _ = ops.sig_gram_vjp(Xt, None, M, torch.tensor(G, device=DEV), base=base, gout_levels=True, order=order)
    Xr = torch.tensor(X, requires_grad=True)
    (ar.k_seq(Xr, Xr, M, base, order=order) * torch.tensor(G)).sum().backward()
    assert norm_rel_err(gS.cpu().numpy(), Xr.grad.numpy()) < GTOL
    gD, _ = ops.sig_gram_vjp(Xt, None, M, torch.tensor(Gd, device=DEV), base=base, diag=True, order=order)
    Xr = torch.tensor(X, requires_grad=True)
    (ar.k_seq_diag(Xr, M, base, order=order) * torch.tensor(Gd)).sum().backward()
    assert norm_rel_err(gD.cpu().numpy(), Xr.grad.numpy()) < GTOL


def test_folded_cross_backward_in_blocks(monkeypatch):
    """The folded K(X, X2) backward cut into block launches (autograd._fold_blocks: lopsided shapes or
    weights past GPSIG_FOLD_WEIGHT_BYTES) gives the gradient of the single launch, against fp64 autodiff."""
    import gpsig_amd
    from gpsig_amd import autograd as ag
    g = golden("linear_chen.npz")
    X = g["X"]
    N, L, D = X.shape
    M = int(g["num_levels"])
    X2 = np.cumsum(np.random.default_rng(3).standard_normal((7, L, D)), 1) / np.sqrt(L * D)
    G = np.random.default_rng(4).standard_normal((N, 7))
    monkeypatch.setattr(ag, "_fold_blocks", lambda n1, n2, M, budget=None: (5, 3))
    k = gpsig_amd.SignatureLinear(L * D, D, M, order=M)
    Xt = torch.tensor(X.reshape(N, -1), device=DEV, requires_grad=True)
    X2t = torch.tensor(X2.reshape(7, -1), device=DEV, requires_grad=True)
    (k.K(Xt, X2t) * torch.as_tensor(G, device=DEV)).sum().backward()
    Xr = torch.tensor(X, requires_grad=True)
    X2r = torch.tensor(X2, requires_grad=True)
    (ar.K(Xr, X2r, M, base="linear", order=M) * torch.tensor(G)).sum().backward()
    assert norm_rel_err(Xt.grad.reshape(X.shape).cpu().numpy(), Xr.grad.numpy()) < GTOL
    assert norm_rel_err(X2t.grad.reshape(X2.shape).cpu().numpy(), X2r.grad.numpy()) < GTOL
