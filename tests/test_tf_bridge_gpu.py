"""GPU: the host bodies of the TF 1.15 binding (gpsig_amd/tf_bridge.py), called as
tf.py_func calls them -- float64 NumPy in, float64 NumPy out -- checked forward against the NumPy oracle
and backward against fp64 autodiff of the reference graph (oracle/autodiff_ref.py) or the reference's
PDE adjoint restated on its own grids (oracle/pde_grad.py).

Criterion: norm-relative max error, forward TOL = 1e-5 per level, gradients GTOL = 1e-5
(the north_star's 1e-5 relative fp32)."""
import numpy as np
import pytest
import torch

from conftest import golden, norm_rel_err
from oracle import autodiff_ref as ar
from oracle import kernels_ref as kr
from oracle import pde, pde_grad

pytestmark = pytest.mark.gpu
TOL = 1e-5
GTOL = 1e-5


def _walk(rng, n, l, d, s=1.0):
    return np.cumsum(rng.standard_normal((n, l, d)), 1) * s / np.sqrt(l * d)


def _autodiff(f, args, dy):
    """fp64 reverse-mode gradient of sum(f(*args) * dy) w.r.t. every arg."""
    ts = [torch.tensor(a, dtype=torch.float64, requires_grad=True) for a in args]
    (f(*ts) * torch.as_tensor(dy)).sum().backward()
    return [t.grad.numpy() for t in ts]


@pytest.mark.parametrize("base", ["rbf", "linear"])
@pytest.mark.parametrize("cross", [False, True])
def test_K_seq_forward_and_vjp(base, cross):
    from gpsig_amd import tf_bridge as tfb
    rng = np.random.default_rng(11)
    M = 4
    X = _walk(rng, 6, 20, 3)
    X2 = _walk(rng, 5, 17, 3) if cross else None
    got = tfb.K_seq(X, X2, M, base=base)
    assert got.dtype == np.float64 and got.shape == (M + 1, 6, 5 if cross else 6)
    ref = kr.SignatureKernelRef(20 * 3, 3, M, base=base).K_seq(X, X2)
    assert (norm_rel_err(got, ref, axis_levels=True) < TOL).all()
    dK = rng.standard_normal(got.shape)
    g = tfb.K_seq_vjp(X, X2, M, dK, base=base)
    if cross:
        rx, ry = _autodiff(lambda x, y: ar.k_seq(x, y, M, base), [X, X2], dK)
        assert norm_rel_err(g[0], rx) < GTOL and norm_rel_err(g[1], ry) < GTOL
    else:
        (rx,) = _autodiff(lambda x: ar.k_seq(x, None, M, base), [X], dK)
        assert g.shape == X.shape and norm_rel_err(g, rx) < GTOL


@pytest.mark.parametrize("order", [1, 3])
def test_K_seq_diag_forward_and_vjp(order):
    from gpsig_amd import tf_bridge as tfb
    rng = np.random.default_rng(12)
    M = 4
    X = _walk(rng, 7, 24, 3)
    got = tfb.K_seq_diag(X, M, order=order)
    ref = ar.k_seq_diag(torch.tensor(X), M, order=order).numpy()
    assert got.shape == (M + 1, 7) and (norm_rel_err(got, ref, axis_levels=True) < TOL).all()
    dK = rng.standard_normal(got.shape)
    g = tfb.K_seq_diag_vjp(X, M, dK, order=order)
    (rx,) = _autodiff(lambda x: ar.k_seq_diag(x, M, order=order), [X], dK)
    assert norm_rel_err(g, rx) < GTOL


def test_K_seq_higher_order_vjp():
    """_K_seq at order 2 (the higher-order VJP kernel) through the bridge."""
    from gpsig_amd import tf_bridge as tfb
    rng = np.random.default_rng(13)
    M = 3
    X = _walk(rng, 5, 16, 2)
    got = tfb.K_seq(X, None, M, order=2)
    ref = ar.k_seq(torch.tensor(X), None, M, order=2).numpy()
    assert (norm_rel_err(got, ref, axis_levels=True) < TOL).all()
    dK = rng.standard_normal(got.shape)
    g = tfb.K_seq_vjp(X, None, M, dK, order=2)
    (rx,) = _autodiff(lambda x: ar.k_seq(x, None, M, order=2), [X], dK)
    assert norm_rel_err(g, rx) < GTOL


@pytest.mark.parametrize("base", ["rbf", "linear"])
@pytest.mark.parametrize("incr", [False, True])
def test_K_tens_forward_and_vjp(base, incr):
    """Kzz: _K_tens (kernels.py:264-284), the inducing-tensor SVGP's Kuu."""
    from gpsig_amd import tf_bridge as tfb
    g0 = golden("tensors.npz")
    M = int(g0["num_levels"])
    Z = g0["Zi"] if incr else g0["Z"] * 0.3
    got = tfb.K_tens(Z, M, base=base, increments=incr)
    exp = g0[f"{base}_tens_incr" if incr else f"{base}_tens"]
    assert (norm_rel_err(got, exp, axis_levels=True) < TOL).all()
    dK = np.random.default_rng(14).standard_normal(got.shape)
    gz = tfb.K_tens_vjp(Z, M, dK, base=base, increments=incr)
    (rz,) = _autodiff(lambda z: ar.k_tens(z, M, base, incr), [Z], dK)
    assert gz.shape == Z.shape and norm_rel_err(gz, rz) < GTOL


@pytest.mark.parametrize("base", ["rbf", "linear"])
@pytest.mark.parametrize("incr", [False, True])
def test_K_tens_vs_seq_forward_and_vjp(base, incr):
    """Kuf: _K_tens_vs_seq (kernels.py:314-341), the path C4 measures and the default SVGP trainer runs."""
    from gpsig_amd import tf_bridge as tfb
    g0 = golden("tensors.npz")
    M = int(g0["num_levels"])
    Z = g0["Zi"] if incr else g0["Z"] * 0.3
    X = g0["X"]
    got = tfb.K_tens_vs_seq(Z, X, M, base=base, increments=incr)
    exp = g0[f"{base}_tvs_incr_o1" if incr else f"{base}_tvs_o1"]
    assert (norm_rel_err(got, exp, axis_levels=True) < TOL).all()
    dK = np.random.default_rng(15).standard_normal(got.shape)
    gz, gx = tfb.K_tens_vs_seq_vjp(Z, X, M, dK, base=base, increments=incr)
    rz, rx = _autodiff(lambda z, x: ar.k_tens_vs_seq(z, x, M, base, incr), [Z, X], dK)
    assert norm_rel_err(gz, rz) < GTOL and norm_rel_err(gx, rx) < GTOL


def test_K_tens_vs_seq_higher_order_vjp_raises():
    from gpsig_amd import tf_bridge as tfb
    g0 = golden("tensors.npz")
    M = int(g0["num_levels"])
    with pytest.raises(NotImplementedError):
        tfb.K_tens_vs_seq_vjp(g0["Z"], g0["X"], M, np.zeros((M + 1, g0["Z"].shape[1], g0["X"].shape[0])), order=2)


@pytest.mark.parametrize("n", [0, 1, 2])
def test_pde_Kdiag_forward_and_vjp(n):
    """UntruncSignatureKernel.Kdiag's solve (kernels_pde.py:174-183) and its gradient (_KdiagGrad,
    kernels_pde.py:465-509), against the reference's own Cython grids (tests/golden/pde.npz)."""
    from gpsig_amd import tf_bridge as tfb
    g0 = golden("pde.npz")
    X = g0["X"]
    got = tfb.pde_Kdiag(X, n)
    assert got.shape == (X.shape[0],) and norm_rel_err(got, pde.pde_diag(X, n, 1)) < TOL
    w = np.random.default_rng(16).standard_normal(X.shape[0])
    g = tfb.pde_Kdiag_vjp(X, w, n)
    K, Kr = pde.pde_diag_grids(X, n, 1)
    ref = pde_grad.kdiag_grad(X, np.tril(K), np.tril(Kr), n) * w[:, None, None]
    assert norm_rel_err(g, ref) < GTOL


def test_bridge_rejects_unsupported_base():
    from gpsig_amd import tf_bridge as tfb
    with pytest.raises(ValueError):
        tfb.K_seq(np.zeros((2, 5, 2)), None, 3, base="cosine")
