"""GPU parity at the BASELINE.json full sizes (SURVEY.md 8 configs C2-C5 and the headline H), through
size-independent properties plus bounded oracle subsamples:

  * the normalised Gram restricted to a subset S equals the Gram of X[S] (pairs are independent:
    the full-size launch reproduces the small launch bit for bit where each pair's recursion is the
    same instructions in any lane-group slot, and to fp32 rounding for the 10-lane groups);
  * symmetry, the constant normalised diagonal (sum of sigma * variances), positive semi-definiteness;
  * a subsample of rows against the float64 oracle (1e-5 norm-relative, the north_star bar)."""
import numpy as np
import pytest
import torch

from conftest import norm_rel_err
from oracle import kernels_ref as kr
from oracle import pde

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = 1e-5


def walks(n, l, d, seed=0):
    rng = np.random.default_rng(seed)
    return (np.cumsum(rng.standard_normal((n, l, d)), axis=1) / np.sqrt(l * d)).astype(np.float32)


@pytest.mark.parametrize("cfg", [("C2", 1024, 100, 5, 5), ("H", 4096, 128, 5, 5), ("C5", 8192, 128, 8, 6)])
def test_gram_full_size(cfg):
    import gpsig_amd
    name, N, L, D, M = cfg
    X = walks(N, L, D)
    Xt = torch.as_tensor(X.reshape(N, -1), device=DEV)
    k = gpsig_amd.SignatureRBF(L * D, D, M)
    K = k.K(Xt)
    assert torch.equal(K, K.T)  # the mirror store writes the identical value
    torch.testing.assert_close(torch.diagonal(K), torch.full((N,), float(M + 1), device=DEV), rtol=0, atol=2e-5)
    S = np.unique(np.linspace(0, N - 1, 48).astype(int))
    St = torch.as_tensor(S, device=DEV)
    sub = K[St][:, St]
    # Every pair's recursion runs as the same instructions in any slot, the 10-lane groups at 65..100 points
    # (C2) included (their scans are slot-independent Hillis-Steele trees, common.h): bitwise.
    torch.testing.assert_close(sub, k.K(Xt[St]), rtol=0, atol=0)
    if N <= 1024:
        assert torch.linalg.eigvalsh(K.double()).min().item() > -1e-4
    # the symmetric oracle on a subset (K(X) and K(X, X2) differ on the diagonal by design: jitter
    # normalises K(X)'s diagonal to exactly 1 per level, K(x, x) / (K(x, x) + jitter) in K(X, X2))
    R = S[::2]
    Rt = torch.as_tensor(R, device=DEV)
    ref = kr.SignatureKernelRef(L * D, D, M)
    exp = ref.K(X[R].astype(np.float64).reshape(len(R), -1))
    assert norm_rel_err(K[Rt][:, Rt].cpu().numpy(), exp) < TOL


def test_pde_gram_full_size_C3():
    import gpsig_amd
    N, L, D = 1024, 200, 5
    X = walks(N, L, D)
    Xt = torch.as_tensor(X.reshape(N, -1), device=DEV)
    kp = gpsig_amd.UntruncSignatureKernel(L * D, D, order=1)
    K = kp.K(Xt)
    assert torch.equal(K, K.T)
    d = kp.Kdiag(Xt)
    torch.testing.assert_close(torch.diagonal(K), d, rtol=1e-6, atol=0)
    S = np.unique(np.linspace(0, N - 1, 16).astype(int))
    St = torch.as_tensor(S, device=DEV)
    torch.testing.assert_close(K[St][:, St], kp.K(Xt[St]), rtol=0, atol=0)
    exp = pde.pde_gram(X[S].astype(np.float64), None, 1, 1)
    assert norm_rel_err(K[St][:, St].cpu().numpy(), exp) < TOL


@pytest.mark.parametrize("increments", [False, True])
def test_kuf_full_size_C4(increments):
    import gpsig_amd
    T, N, L, D, M = 512, 4096, 100, 5, 5
    LT = M * (M + 1) // 2
    X = walks(N, L, D)
    rng = np.random.default_rng(2)
    Z = rng.standard_normal((LT, T, 2, D) if increments else (LT, T, D)).astype(np.float32)
    Xt = torch.as_tensor(X.reshape(N, -1), device=DEV)
    Zt = torch.as_tensor(Z, device=DEV)
    k = gpsig_amd.SignatureRBF(L * D, D, M)
    K = k.K_tens_vs_seq(Zt, Xt, increments=increments, return_levels=True)
    assert K.shape == (M + 1, T, N)
    S = np.unique(np.linspace(0, N - 1, 24).astype(int))
    St = torch.as_tensor(S, device=DEV)
    # column subset = the call on the subset of sequences (per-sequence independence)
    torch.testing.assert_close(K[:, :, St], k.K_tens_vs_seq(Zt, Xt[St], increments=increments, return_levels=True),
                               rtol=0, atol=0)
    Ts = np.arange(0, T, 64)
    ref = kr.SignatureKernelRef(L * D, D, M)
    exp = ref.K_tens_vs_seq(Z[:, Ts].astype(np.float64), X[S].astype(np.float64).reshape(len(S), -1),
                            return_levels=True, increments=increments)
    got = K[:, torch.as_tensor(Ts, device=DEV)][:, :, St].cpu().numpy()
    assert (norm_rel_err(got[1:], exp[1:], axis_levels=True) < TOL).all()


def test_vosf_kuf_full_size_C4():
    """The VOSF reading of C4 (BASELINE.json configs[3], inducing_variables_vosf.py:212-269): Kuf of
    Mz = 512 orthogonal signature features against N = 4096 sequences, L = 100, D = 5 (signature level
    4, the first 511 coordinates, computed on the device and scaled per level), the normalised kernel
    (Kuf divided by the per-level K_norms of each sequence).  Column subset = the call on the subset;
    a subsample against exact Chen signatures (oracle/chen.py) and the float64 oracle's diagonal."""
    import gpsig_amd
    from gpsig_amd import inducing_variables_vosf as iv
    from gpsig_amd import signatures as sg
    from oracle import chen
    Mz, N, L, D, lev = 512, 4096, 100, 5, 5
    X = walks(N, L, D)
    Xt = torch.as_tensor(X.reshape(N, -1), device=DEV)
    var = np.linspace(0.5, 1.5, lev + 1)
    k = gpsig_amd.SignatureLinear(L * D, D, lev, order=lev, variances=var)
    feat = iv.TruncInducingOrthogonalTensors(L * D, D, Mz, compute_sig=True)
    Kzz, Kzx, Kxx = feat.Kuu_Kuf_Kff(k, Xt)
    assert Kzz.shape == (Mz, Mz) and Kzx.shape == (Mz, N) and Kxx.shape == (N,)
    torch.testing.assert_close(Kxx, torch.full((N,), float(var.sum()), device=DEV, dtype=Kxx.dtype))
    S = np.unique(np.linspace(0, N - 1, 12).astype(int))
    St = torch.as_tensor(S, device=DEV)
    _, Kzx_s, _ = feat.Kuu_Kuf_Kff(k, Xt[St])
    # per-sequence independence; the exact signature kernel's norms (the feature path: signatures and a
    # library reduction per level, ops._sig_feature_path) sum in a batch-size dependent order
    torch.testing.assert_close(Kzx[:, St], Kzx_s, rtol=1e-6, atol=0)
    slv = sg.compute_trunc(Mz, D)
    assert slv == 4
    Xs = X[S].astype(np.float64)
    sig = [chen.signature(x, slv) for x in Xs]
    ref = np.stack([np.concatenate([[1.0]] + s[1:]) for s in sig])[:, :Mz].T  # (Mz, |S|)
    reps = np.repeat(np.arange(slv + 1), [D ** i for i in range(slv + 1)])[:Mz]
    # normalised kernel: level m of k(x, x) is |S_m(x)|^2 (the exact signature kernel, order = num_levels)
    knorm = np.stack([[1.0] + [float(np.dot(s[m], s[m])) for m in range(1, slv + 1)] for s in
                      [chen.signature(x, lev) for x in Xs]]).T  # (slv + 1, |S|)
    ref = ref * np.sqrt(var[reps])[:, None] / np.sqrt(knorm[reps] + 1e-6)
    assert norm_rel_err(Kzx_s.cpu().numpy(), ref) < TOL
