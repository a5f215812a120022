"""GPU parity of the gradients for long sequences: the Gram VJP in column blocks (sig_bwd_kernel `nblk`,
forward and adjoint carries per row and level in the workspace) vs torch fp64 autodiff of the reference
graph (oracle/autodiff_ref.py), and the reference's own SVGP training shapes
(benchmarks/run_gpsig_benchmarks.py:32: num_levels=4, num_inducing=500, max_len=500, num_lags=1,
increments=True; train_gpsig.py:20 minibatch 50), where lags double the 3 + time channels to 8.

Criterion as tests/test_grad_gpu.py: norm-relative max|g32 - g64| <= GTOL * max|g64|.
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


@pytest.mark.parametrize("L,D,M,base,cross,diff", [
    (300, 3, 4, "rbf", False, True),    # 2 blocks (255 cells each at W = 4)
    (600, 2, 3, "rbf", True, True),     # 3 blocks
    (400, 12, 3, "rbf", False, True),   # d > 8: W = 2, 127 cells per block, 4 blocks
    (300, 3, 4, "linear", True, True),
    (300, 3, 3, "rbf", False, False),   # point cells (difference=False)
    (280, 4, 1, "rbf", False, True),    # one level: no carries
])
def test_long_gram_vjp_matches_autodiff(L, D, M, base, cross, diff):
    import gpsig_amd
    N, N2 = 3, 2
    X = walks(N, L, D, L)
    X2 = walks(N2, L, D, L + 1) if cross else None
    rng = np.random.default_rng(7)
    G = rng.standard_normal((N, N2 if cross else N))
    cls = gpsig_amd.SignatureRBF if base == "rbf" else gpsig_amd.SignatureLinear
    k = cls(L * D, D, M, difference=diff)
    Xt = torch.tensor(X.reshape(N, -1), device=DEV, requires_grad=True)
    X2t = None if X2 is None else torch.tensor(X2.reshape(N2, -1), device=DEV, requires_grad=True)
    (k.K(Xt, X2t) * torch.as_tensor(G, device=DEV)).sum().backward()
    Xr = torch.tensor(X, requires_grad=True)
    X2r = None if X2 is None else torch.tensor(X2, requires_grad=True)
    (ar.K(Xr, X2r, M, base=base, difference=diff) * torch.tensor(G)).sum().backward()
    assert norm_rel_err(Xt.grad.reshape(X.shape).cpu().numpy(), Xr.grad.numpy()) < GTOL
    if cross:
        assert norm_rel_err(X2t.grad.reshape(X2.shape).cpu().numpy(), X2r.grad.numpy()) < GTOL


def test_long_gram_vjp_saved_state_equals_recompute():
    """The training forward saves the end-of-sweep state (gpsig_sig_gram_state); the blocked VJP then
    skips the last block's forward sweep and reads its end state from it: same gradient."""
    from gpsig_amd import ops
    N, L, D, M = 4, 530, 3, 4
    X = torch.tensor(walks(N, L, D, 5), device=DEV, dtype=torch.float32)
    G = torch.tensor(np.random.default_rng(1).standard_normal((N, N)), device=DEV, dtype=torch.float32)
    st = torch.zeros(ops.sig_state_numel(N, None, L, M), dtype=torch.float32, device=DEV)
    ops.sig_gram(X, None, M, state=st, out_mode=2)
    g1, _ = ops.sig_gram_vjp(X, None, M, G)
    g2, _ = ops.sig_gram_vjp(X, None, M, G, state=st)
    assert norm_rel_err(g2.cpu().numpy(), g1.cpu().numpy()) < 1e-5


def test_reference_training_shapes_covariance_gradients():
    """K_tens_n_seq_covs (kernels.py:624-704) at the reference's SVGP training shapes: T = 500 inducing
    tensors (increments=True), a minibatch of N = 50 sequences of L = 500 points in 8 channels (3 + time,
    one lag), num_levels = 4; normalised.  The GPU gradient for all 50 sequences and the 500 tensors runs
    in one backward; the fp64 autodiff oracle checks it on a subsample of the sequences (the loss is a
    sum of per-sequence terms in Kzx and diag(Kxx), so the rows of dLoss/dX for the subsample equal the
    oracle's on the subsample; dLoss/dZ is checked on a second GPU call over the subsample)."""
    import gpsig_amd
    M, T, N, L, D = 4, 500, 50, 500, 8
    LT = M * (M + 1) // 2
    rng = np.random.default_rng(11)
    Z = 0.3 * rng.standard_normal((LT, T, 2, D))
    X = walks(N, L, D, 12, scale=2.0)
    G2, G3 = rng.standard_normal((T, N)), rng.standard_normal(N)
    k = gpsig_amd.SignatureRBF(L * D, D, M)

    def gpu_grads(Xs, G2s, G3s):
        Zt = torch.tensor(Z, device=DEV, requires_grad=True)
        Xt = torch.tensor(Xs.reshape(len(Xs), -1), device=DEV, requires_grad=True)
        Kzz, Kzx, Kxx = k.K_tens_n_seq_covs(Zt, Xt, increments=True)
        ((Kzx * torch.as_tensor(G2s, device=DEV)).sum() + (Kxx * torch.as_tensor(G3s, device=DEV)).sum()
         + Kzz.sum()).backward()
        return Zt.grad.cpu().numpy(), Xt.grad.reshape(Xs.shape).cpu().numpy(), Kzx.detach().cpu().numpy()

    gZ_full, gX_full, Kzx_full = gpu_grads(X, G2, G3)
    assert np.isfinite(gX_full).all() and np.isfinite(gZ_full).all()
    S = [0, 31]
    gZ_sub, gX_sub, _ = gpu_grads(X[S], G2[:, S], G3[S])
    np.testing.assert_allclose(gX_full[S], gX_sub, rtol=1e-5, atol=1e-6 * np.abs(gX_sub).max())

    Zr = torch.tensor(Z, requires_grad=True)
    Xr = torch.tensor(X[S], requires_grad=True)
    Kzz_r = ar.k_tens(Zr, M, increments=True).sum(0)
    Kzx_r = ar.K_tens_vs_seq(Zr, Xr, M, increments=True)
    Kxx_r = torch.full((len(S),), float(M + 1), dtype=torch.float64)  # normalised diag: sigma * sum(variances)
    ((Kzx_r * torch.tensor(G2[:, S])).sum() + (Kxx_r * torch.tensor(G3[S])).sum() + Kzz_r.sum()).backward()
    assert norm_rel_err(Kzx_full[:, S], Kzx_r.detach().numpy()) < 1e-5
    assert norm_rel_err(gX_sub, Xr.grad.numpy()) < GTOL
    assert norm_rel_err(gZ_sub, Zr.grad.numpy()) < GTOL
