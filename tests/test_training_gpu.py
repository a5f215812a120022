"""End to end: hyperparameter learning through the gfx950 forward and VJP kernels.

An exact GP marginal likelihood on a small sequence regression task, NLL(theta) with
K = SignatureRBF(lengthscales, variances).K(X) + noise * I (the quantity GPSig's models differentiate,
gpsig/models.py over gpsig/kernels.py:402-477).  Checks: the gradient of the NLL w.r.t. the log
lengthscales and log variances equals fp64 autodiff of the reference graph (oracle/autodiff_ref.py),
and Adam on the GPU gradients lowers the NLL."""
import numpy as np
import pytest
import torch

from oracle import autodiff_ref as ar

pytestmark = pytest.mark.gpu
DEV = "cuda"


def nll(K, y, noise):
    Kn = K + noise * torch.eye(K.shape[0], dtype=K.dtype, device=K.device)
    Lc = torch.linalg.cholesky(Kn)
    alpha = torch.cholesky_solve(y[:, None], Lc)[:, 0]
    return 0.5 * (y * alpha).sum() + torch.log(torch.diagonal(Lc)).sum()


def data(N=40, L=20, D=2, seed=0):
    rng = np.random.default_rng(seed)
    X = np.cumsum(rng.standard_normal((N, L, D)), 1) / np.sqrt(L)
    y = np.sin(2.0 * X[:, -1, 0]) + 0.5 * X[:, :, 1].mean(1) + 0.05 * rng.standard_normal(N)
    return X, y - y.mean()


def test_nll_gradient_matches_autodiff_and_training_descends():
    import gpsig_amd
    X, y = data()
    N, L, D = X.shape
    M = 3
    log_ls0 = np.log(np.array([0.7, 1.4]))
    log_var0 = np.zeros(M + 1)
    noise = 0.05
    k = gpsig_amd.SignatureRBF(L * D, D, M)
    Xt = torch.tensor(X.reshape(N, -1), device=DEV)
    yt = torch.tensor(y, device=DEV)
    log_ls = torch.tensor(log_ls0, device=DEV, requires_grad=True)
    log_var = torch.tensor(log_var0, device=DEV, requires_grad=True)

    def loss_gpu():
        k.lengthscales = torch.exp(log_ls)
        k.variances = torch.exp(log_var)
        return nll(k.K(Xt), yt, noise)

    f = loss_gpu()
    f.backward()
    # fp64 autodiff of the reference graph at the same parameters
    lr_, lv_ = torch.tensor(log_ls0, requires_grad=True), torch.tensor(log_var0, requires_grad=True)
    Kr = ar.K(torch.tensor(X) / torch.exp(lr_), None, M, scale=torch.exp(lv_))
    fr = nll(Kr, torch.tensor(y), noise)
    fr.backward()
    assert abs(f.item() - fr.item()) < 1e-4 * abs(fr.item())
    np.testing.assert_allclose(log_ls.grad.cpu().numpy(), lr_.grad.numpy(), rtol=1e-3, atol=1e-4)
    np.testing.assert_allclose(log_var.grad.cpu().numpy(), lv_.grad.numpy(), rtol=1e-3, atol=1e-4)

    opt = torch.optim.Adam([log_ls, log_var], lr=0.05)
    start = f.item()
    for _ in range(40):
        opt.zero_grad()
        loss = loss_gpu()
        loss.backward()
        opt.step()
    end = loss_gpu().item()
    assert end < start - 0.05 * abs(start), (start, end)
