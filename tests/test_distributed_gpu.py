"""GPU, one process: the sharded entry points of gpsig_amd.distributed at world size 1 run the
gfx950 kernels and agree with the unsharded calls (the N > 1 partition / gather logic is covered by
the gloo tests in test_distributed.py)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def walks(n, l, d, seed):
    rng = np.random.default_rng(seed)
    return np.cumsum(rng.standard_normal((n, l, d)), axis=1) / np.sqrt(l * d)


def test_sharded_entry_points_world1():
    import gpsig_amd
    from gpsig_amd import distributed as D
    N, L, Dm, M = 20, 16, 3, 4
    X = torch.tensor(walks(N, L, Dm, 0).reshape(N, -1), device=DEV)
    X2 = torch.tensor(walks(7, L, Dm, 1).reshape(7, -1), device=DEV)
    k = gpsig_amd.SignatureRBF(L * Dm, Dm, M)
    np.testing.assert_allclose(D.sharded_K(k, X).cpu().numpy(), k.K(X).cpu().numpy(), rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(D.sharded_K(k, X, X2).cpu().numpy(), k.K(X, X2).cpu().numpy(), rtol=1e-6, atol=1e-7)
    Z = torch.tensor(np.random.default_rng(2).standard_normal((M * (M + 1) // 2, 5, Dm)) * 0.5, device=DEV)
    np.testing.assert_allclose(D.sharded_K_tens_vs_seq(k, Z, X, return_levels=True).cpu().numpy(),
                               k.K_tens_vs_seq(Z, X, return_levels=True).cpu().numpy(), rtol=1e-6, atol=1e-7)
    kp = gpsig_amd.UntruncSignatureKernel(L * Dm, Dm, order=1)
    np.testing.assert_allclose(D.sharded_pde_K(kp, X).cpu().numpy(), kp.K(X).cpu().numpy(), rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(D.sharded_pde_K(kp, X, X2).cpu().numpy(), kp.K(X, X2).cpu().numpy(), rtol=1e-6,
                               atol=1e-7)
