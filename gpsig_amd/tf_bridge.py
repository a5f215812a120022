"""Host bodies of the TensorFlow 1.15 binding: NumPy in, NumPy out, no TensorFlow.

GPSig (TF 1.15.3 / GPflow 1.5.1, graph mode) reaches the hot path through five methods.  INTEGRATION.md's
``enable()`` replaces each with a ``tf.py_func`` + ``tf.custom_gradient`` pair whose Python bodies are the
functions below; the upstream gradient goes to the matching VJP:

  ================================================  =====================  ==========================
  reference method (file:line)                       forward                backward
  ================================================  =====================  ==========================
  ``SignatureKernel._K_seq`` (kernels.py:209-238)    :func:`K_seq`          :func:`K_seq_vjp`
  ``SignatureKernel._K_seq_diag`` (:190-207)         :func:`K_seq_diag`     :func:`K_seq_diag_vjp`
  ``SignatureKernel._K_tens`` (:264-284)             :func:`K_tens`         :func:`K_tens_vjp`
  ``SignatureKernel._K_tens_vs_seq`` (:314-341)      :func:`K_tens_vs_seq`  :func:`K_tens_vs_seq_vjp`
  ``UntruncSignatureKernel.Kdiag`` solve             :func:`pde_Kdiag`      :func:`pde_Kdiag_vjp`
    (kernels_pde.py:160-185; its gradients
    ``_KdiagGrad`` :465-509 and
    ``_untrunc_cov_grad`` covariance_op/
    _untrunc_cov_grad.py:25-77)
  ================================================  =====================  ==========================

Every function takes the reference's own arguments after its scaling (``_apply_scaling_and_lags_to_sequences``
and ``_apply_scaling_to_*tensors`` stay in TensorFlow, so the lengthscale gradient flows through TF as
before), moves the float64 arrays to the GPU as float32, calls the gfx950 kernels through
:mod:`gpsig_amd.ops` and returns float64 NumPy (``settings.float_type``).  Shapes follow the reference:
sequences (N, L, D); inducing tensors (LT, T, D), or (LT, T, 2, D) with ``increments``; outputs
(num_levels + 1, ...) raw levels.  Errors are the ops' ``GpsigError`` / ``ValueError`` /
``NotImplementedError`` (raised inside ``tf.py_func``, they surface as TF's ``InvalidArgumentError``).

There is no CPU fallback: without a GPU, or without the built library, every call raises.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib as L
from . import ops

_BASES = ("rbf", "linear")


def _device(device=None) -> torch.device:
    if device is not None:
        return torch.device(device)
    if not torch.cuda.is_available():
        raise L.GpsigError("gpsig_amd.tf_bridge needs a ROCm GPU (torch.cuda); there is no CPU path")
    return torch.device("cuda", torch.cuda.current_device())


def _dev(a, device=None) -> torch.Tensor:
    """float64 NumPy (what TF hands a py_func) -> contiguous float32 device tensor."""
    return torch.from_numpy(np.ascontiguousarray(np.asarray(a), dtype=np.float64)).to(_device(device), torch.float32)


def _host(t) -> np.ndarray:
    """Device tensor -> float64 NumPy (settings.float_type), after the stream has finished."""
    return t.detach().to(torch.float64).cpu().numpy()


def _base(base) -> str:
    b = {"lin": "linear"}.get(base, base)
    if b not in _BASES:
        raise ValueError(f"base must be one of {_BASES} (the fused gfx950 seeds), got {base!r}")
    return b


def _signature_case(num_levels, order, base, difference) -> bool:
    """The exact signature kernel (linear, order >= num_levels): its gradient goes through the signature
    features when the higher-order VJP kernel does not cover the length (autograd._ho_signature_case)."""
    return order >= num_levels and _base(base) == "linear" and difference


# ----------------------------------------------------------------------------- _K_seq / _K_seq_diag
def K_seq(X, X2, num_levels: int, order: int = 1, base="rbf", difference: bool = True, device=None) -> np.ndarray:
    """SignatureKernel._K_seq (kernels.py:209-238): X (N, L, D), X2 (N2, L2, D) or None ->
    (num_levels + 1, N, N2) raw levels (signature_algs.py:8-74)."""
    kw = dict(order=order, base=_base(base), difference=difference)
    x = _dev(X, device)
    return _host(ops.sig_gram(x, None if X2 is None else _dev(X2, x.device), num_levels, **kw))


def K_seq_vjp(X, X2, num_levels: int, dK, order: int = 1, base="rbf", difference: bool = True, device=None):
    """Gradient of :func:`K_seq` given dK (num_levels + 1, N, N2): ``dX`` for X2 None (K(X), both slots of
    every pair), else ``(dX, dX2)``.  TF autodiff of kernels.py:209-238 in the reference."""
    b = _base(base)
    x = _dev(X, device)
    y = None if X2 is None else _dev(X2, x.device)
    g = _dev(dK, x.device)
    lengths = (x.shape[1],) if y is None else (x.shape[1], y.shape[1])
    if order > 1 and num_levels > 1 and not all(ops.ho_vjp_supported(l, num_levels, order, b) for l in lengths):
        if not _signature_case(num_levels, order, b, difference):
            raise NotImplementedError(f"no gfx950 VJP for order {order}, num_levels {num_levels} at lengths {lengths}")
        gx, gy = ops.sig_gram_ho_vjp(x, y, num_levels, g)
    else:
        gx, gy = ops.sig_gram_vjp(x, y, num_levels, g, base=b, gout_levels=True, difference=difference, order=order)
    return _host(gx) if y is None else (_host(gx), _host(gy))


def K_seq_diag(X, num_levels: int, order: int = 1, base="rbf", difference: bool = True, device=None) -> np.ndarray:
    """SignatureKernel._K_seq_diag (kernels.py:190-207): X (N, L, D) -> (num_levels + 1, N)."""
    return _host(ops.sig_diag(_dev(X, device), num_levels, order, _base(base), difference))


def K_seq_diag_vjp(X, num_levels: int, dK, order: int = 1, base="rbf", difference: bool = True,
                   device=None) -> np.ndarray:
    """Gradient of :func:`K_seq_diag` given dK (num_levels + 1, N) -> dX (N, L, D)."""
    b = _base(base)
    x = _dev(X, device)
    g = _dev(dK, x.device)
    if order > 1 and num_levels > 1 and not ops.ho_vjp_supported(x.shape[1], num_levels, order, b):
        if not _signature_case(num_levels, order, b, difference):
            raise NotImplementedError(f"no gfx950 VJP for order {order}, num_levels {num_levels} at length {x.shape[1]}")
        gx, _ = ops.sig_gram_ho_vjp(x, None, num_levels, None, g)
    else:
        gx, _ = ops.sig_gram_vjp(x, None, num_levels, g, base=b, diag=True, difference=difference, order=order)
    return _host(gx)


# ----------------------------------------------------------------------------- _K_tens / _K_tens_vs_seq
def K_tens(Z, num_levels: int, base="rbf", increments: bool = False, device=None) -> np.ndarray:
    """SignatureKernel._K_tens (kernels.py:264-284, tensor_kern signature_algs.py:76-99): Z (LT, T, D) or
    (LT, T, 2, D) -> (num_levels + 1, T, T).  Kzz of the inducing-tensor SVGP (inducing_variables.py:52-60)."""
    return _host(ops.tens_gram(_dev(Z, device), num_levels, _base(base), increments))


def K_tens_vjp(Z, num_levels: int, dK, base="rbf", increments: bool = False, device=None) -> np.ndarray:
    """Gradient of :func:`K_tens` given dK (num_levels + 1, T, T) -> dZ, Z's shape."""
    z = _dev(Z, device)
    return _host(ops.tens_gram_vjp(z, num_levels, _dev(dK, z.device), _base(base), increments))


def K_tens_vs_seq(Z, X, num_levels: int, order: int = 1, base="rbf", difference: bool = True,
                  increments: bool = False, device=None) -> np.ndarray:
    """SignatureKernel._K_tens_vs_seq (kernels.py:314-341, signature_algs.py:101-160): Z (LT, T, D) or
    (LT, T, 2, D), X (N, L, D) -> (num_levels + 1, T, N).  Kuf of the inducing-tensor SVGP (C4)."""
    z = _dev(Z, device)
    return _host(ops.tens_vs_seq(z, _dev(X, z.device), num_levels, order, _base(base), difference, increments))


def K_tens_vs_seq_vjp(Z, X, num_levels: int, dK, order: int = 1, base="rbf", difference: bool = True,
                      increments: bool = False, device=None):
    """Gradient of :func:`K_tens_vs_seq` given dK (num_levels + 1, T, N) -> (dZ, dX).  Order 1 (the
    reference's default, kernels.py:19): gpsig_tens_vs_seq_vjp; higher orders raise NotImplementedError."""
    if order != 1:
        raise NotImplementedError("gpsig_tens_vs_seq_vjp differentiates the order-1 recursion "
                                  "(signature_algs.py:101-127)")
    z = _dev(Z, device)
    x = _dev(X, z.device)
    gz, gx = ops.tens_vs_seq_vjp(z, x, num_levels, _dev(dK, z.device), _base(base), increments, difference=difference)
    return _host(gz), _host(gx)


# ----------------------------------------------------------------------------- UntruncSignatureKernel.Kdiag
def pde_Kdiag(X, order: int = 0, device=None) -> np.ndarray:
    """k(x, x) of the Goursat PDE at dyadic order ``order``: X (N, L, D) scaled -> (N,).  Replaces both
    branches of UntruncSignatureKernel.Kdiag (kernels_pde.py:174-183: sig_kern_diag's K[:, -1, -1], or the
    UntruncCov op's; the explicit scheme, sigKer_fast.pyx:48 / untrunc_cov_op_gpu.cu:29).  sigma stays in TF."""
    return _host(ops.pde_diag(_dev(X, device), order, 1))


def pde_Kdiag_vjp(X, dK, order: int = 0, device=None) -> np.ndarray:
    """Gradient of :func:`pde_Kdiag` given dK (N,) -> dX (N, L, D): the reference's adjoint
    (``_KdiagGrad`` kernels_pde.py:465-509 / ``_untrunc_cov_grad`` _untrunc_cov_grad.py:25-77 --
    grad_points weighted by the upstream gradient of k(x, x)) on the gfx950 adjoint sweeps."""
    x = _dev(X, device)
    return _host(ops.pde_diag_vjp(x, _dev(dK, x.device), order, 1))


# the five reference methods enable() patches, for INTEGRATION.md and tests/test_integration_doc.py
PATCHED = (
    ("gpsig.kernels.SignatureKernel", "_K_seq", "K_seq", "K_seq_vjp"),
    ("gpsig.kernels.SignatureKernel", "_K_seq_diag", "K_seq_diag", "K_seq_diag_vjp"),
    ("gpsig.kernels.SignatureKernel", "_K_tens", "K_tens", "K_tens_vjp"),
    ("gpsig.kernels.SignatureKernel", "_K_tens_vs_seq", "K_tens_vs_seq", "K_tens_vs_seq_vjp"),
    ("gpsig.kernels_pde.UntruncSignatureKernel", "Kdiag", "pde_Kdiag", "pde_Kdiag_vjp"),
)
