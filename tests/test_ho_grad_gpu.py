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
GTOL = 5e-5
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
    assert norm_rel_err(k.lengthscales.grad.cpu().numpy(), lr.grad.numpy()) < GTOL
    assert norm_rel_err(k.variances.grad.cpu().numpy(), vr.grad.numpy()) < GTOL


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
    """RBF (or linear with order < num_levels) higher orders evaluate forward; their backward raises."""
    import gpsig_amd
    X = torch.tensor(golden("linear_chen.npz")["X"][:4].reshape(4, -1), device=DEV, requires_grad=True)
    for k in (gpsig_amd.SignatureRBF(60, 3, 4, order=2), gpsig_amd.SignatureLinear(60, 3, 4, order=2)):
        K = k.K(X)
        with pytest.raises(NotImplementedError):
            K.sum().backward()
