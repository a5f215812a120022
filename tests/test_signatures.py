"""Signature features (iisignature.sig / sigbackprop replacement): host helpers on CPU, the gfx950
kernels vs the Chen-identity oracle (oracle/chen.py, pinned to the esig relation in test_oracle.py)."""
import numpy as np
import pytest
import torch

from conftest import norm_rel_err
from oracle import autodiff_ref as ar
from oracle import chen

DEV = "cuda"


def test_compute_trunc_and_powers():
    from gpsig_amd import signatures as sg
    assert sg.compute_trunc(6, 5) == 1 and sg.compute_trunc(7, 5) == 2 and sg.compute_trunc(100, 5) == 3
    P = sg.get_powers(3, 2)
    assert P.shape == (3 + 9, 3)
    np.testing.assert_array_equal(P[3], [2, 0, 0])  # (1,1)
    np.testing.assert_array_equal(P[4], [1, 1, 0])  # (1,2)
    np.testing.assert_array_equal(P[3 + 5], [0, 1, 1])  # (2,3)
    np.testing.assert_array_equal(P.sum(1), [1] * 3 + [2] * 9)


def test_torch_signature_oracle_matches_chen():
    rng = np.random.default_rng(0)
    x = np.cumsum(rng.standard_normal((7, 3)), 0) * 0.3
    ref = np.concatenate(chen.signature(x, 4)[1:])
    np.testing.assert_allclose(ar.signature(torch.tensor(x), 4).numpy(), ref, rtol=1e-12, atol=1e-14)


@pytest.mark.gpu
@pytest.mark.parametrize("d,depth,L", [(2, 6, 30), (3, 4, 50), (5, 5, 40), (1, 3, 10), (8, 3, 20),
                                       (6, 6, 12), (40, 3, 8)])
def test_signature_matches_chen(d, depth, L):
    """(6, 6) and (40, 3) have 55 986 / 65 640 coordinates: past the 160 KiB of LDS, the levels live in
    per-path slabs of the workspace (gpsig_signature_workspace_bytes)."""
    from gpsig_amd import ops
    rng = np.random.default_rng(d + depth)
    X = np.cumsum(rng.standard_normal((9, L, d)), 1) / np.sqrt(L)
    got = ops.signature(torch.tensor(X, device=DEV), depth).cpu().numpy()
    off = 0
    for m in range(1, depth + 1):
        ref = np.stack([chen.signature(x, depth)[m] for x in X])
        assert norm_rel_err(got[:, off:off + d ** m], ref) < 1e-5, m
        off += d ** m
    assert off == got.shape[1]


@pytest.mark.gpu
@pytest.mark.parametrize("d,depth,L", [(2, 4, 12), (3, 3, 20), (5, 3, 15), (4, 7, 8), (12, 4, 6)])
def test_signature_backprop_matches_autodiff(d, depth, L):
    """(4, 7) and (12, 4): 21 844 / 22 620 coordinates, the VJP's levels, adjoints and exponential tables
    (4 x the coordinates) past the LDS, in the workspace slabs."""
    from gpsig_amd import signatures as sg
    rng = np.random.default_rng(10 + d)
    X = np.cumsum(rng.standard_normal((5, L, d)), 1) / np.sqrt(L)
    C = sum(d ** m for m in range(1, depth + 1))
    G = rng.standard_normal((5, C))
    Xt = torch.tensor(X, device=DEV, requires_grad=True)
    (sg.Sig(Xt, depth) * torch.as_tensor(G, device=DEV)).sum().backward()
    ref = np.zeros_like(X)
    for a in range(5):
        xa = torch.tensor(X[a], requires_grad=True)
        (ar.signature(xa, depth) * torch.tensor(G[a])).sum().backward()
        ref[a] = xa.grad.numpy()
    assert norm_rel_err(Xt.grad.cpu().numpy(), ref) < 1e-5


@pytest.mark.gpu
def test_vosf_untrunc_features():
    """UntruncInducingOrthogonalTensors.Kuu_Kuf_Kff (inducing_variables_vosf.py:68-146)."""
    import gpsig_amd
    from gpsig_amd import inducing_variables_vosf as iv
    from gpsig_amd import signatures as sg
    from oracle import pde
    rng = np.random.default_rng(3)
    N, L, d, M = 6, 20, 3, 10
    X = np.cumsum(rng.standard_normal((N, L, d)), 1) / np.sqrt(L)
    ls = np.array([0.5, 1.0, 2.0])
    k = gpsig_amd.UntruncSignatureKernel(L * d, d, lengthscales=ls, order=1)
    feat = iv.UntruncInducingOrthogonalTensors(L * d, d, M, compute_sig=True)
    Kzz, Kzx, Kxx = iv.Kuu_Kuf_Kff(feat, k, torch.tensor(X.reshape(N, -1), device=DEV))
    lvl = sg.compute_trunc(M, d)
    S = np.stack([np.concatenate(chen.signature(x, lvl)[1:]) for x in X])[:, :M - 1]
    S = S / np.prod(ls[None, :] ** sg.get_powers(d, lvl)[:M - 1], axis=1)[None, :]
    np.testing.assert_allclose(Kzz.cpu().numpy(), np.eye(M))
    assert Kzx.shape == (M, N)
    np.testing.assert_allclose(Kzx[0].cpu().numpy(), 1.0)
    assert norm_rel_err(Kzx[1:].T.cpu().numpy(), S) < 1e-5
    assert norm_rel_err(Kxx.cpu().numpy(), pde.pde_diag(X / ls, 1, 1)) < 1e-5
    # compute_and_diff_sig: signatures of the scaled paths, differentiable in the lengthscales
    feat2 = iv.UntruncInducingOrthogonalTensors(L * d, d, M, compute_and_diff_sig=True)
    k.lengthscales = torch.tensor(ls, device=DEV, requires_grad=True)
    Kzx2 = feat2.Kuf(k, torch.tensor(X.reshape(N, -1), device=DEV))
    assert norm_rel_err(Kzx2[1:].T.detach().cpu().numpy(), S) < 1e-5  # same numbers, other route
    Kzx2.sum().backward()
    assert torch.isfinite(k.lengthscales.grad).all()


@pytest.mark.gpu
@pytest.mark.parametrize("normalization", [True, False])
def test_vosf_trunc_features(normalization):
    """TruncInducingOrthogonalTensors.Kuu_Kuf_Kff (inducing_variables_vosf.py:180-269)."""
    import gpsig_amd
    from gpsig_amd import inducing_variables_vosf as iv
    from gpsig_amd import signatures as sg
    from oracle import kernels_ref as kr
    rng = np.random.default_rng(4)
    N, L, d, M, lev = 5, 16, 2, 9, 4
    X = np.cumsum(rng.standard_normal((N, L, d)), 1) / np.sqrt(L)
    var = np.array([1.0, 0.5, 2.0, 1.5, 0.7])
    k = gpsig_amd.SignatureLinear(L * d, d, lev, variances=var, normalization=normalization)
    feat = iv.TruncInducingOrthogonalTensors(L * d, d, M, compute_sig=True)
    Kzz, Kzx, Kxx = feat.Kuu_Kuf_Kff(k, torch.tensor(X.reshape(N, -1), device=DEV))
    slv = sg.compute_trunc(M, d)
    S = np.stack([np.concatenate([[1.0]] + chen.signature(x, slv)[1:]) for x in X])[:, :M].T  # (M, N)
    reps = np.repeat(np.arange(slv + 1), [d ** i for i in range(slv + 1)])[:M]
    S = S * np.sqrt(var[reps])[:, None]
    ref = kr.SignatureKernelRef(L * d, d, lev, base="linear", variances=var, normalization=normalization)
    if normalization:
        Kun = ref.K_seq_diag(X)
        S = S / np.sqrt(Kun[reps] + 1e-6)
        np.testing.assert_allclose(Kxx.cpu().numpy(), var.sum())
    else:
        assert norm_rel_err(Kxx.cpu().numpy(), ref.Kdiag(X.reshape(N, -1))) < 1e-5
    assert norm_rel_err(Kzx.cpu().numpy(), S) < 1e-5
