"""Low-rank (Nystrom + randomized Hadamard projection) signature features on MI355X.

Drop-in for gpsig/low_rank_calculations.py (same function names, arguments and meaning, on torch
tensors) and for the low-rank feature maps of gpsig/signature_algs.py:162-222.  The reference runs
these as TF graph ops; here the GEMM-shaped work (the Nystrom cross-kernel, the projections) goes
through torch.matmul (hipBLASLt on gfx950) and the small Nystrom eigendecomposition through
torch.linalg.eigh on the device.  Randomness: the reference draws from TF's stateful / stateless
generators; here a torch.Generator on the device, seeded from the (num_levels-1, 2) integer seeds
when given (tf.contrib.stateless semantics: equal seeds -> equal draws).  Parity with the reference
is therefore distributional: the estimators are unbiased for the exact kernels, which
tests/test_low_rank.py checks by Monte Carlo, and the deterministic pieces are exact.

The sparse Johnson-Lindenstrauss product lr_hadamard_prod_sparse evaluates
    C[n, r] = sum_{i,j} A[n, i] B[n, j] R[i k2 + j, r]
as  sum_i A[n, i] (B @ R_i)[n, r]  (one GEMM over the dense (k1, k2, rank) projection, zero rows
included) instead of gathering the nonzero (i, j) combinations -- the same sum without materialising
the (..., n_nonzero) product matrix.
"""
from __future__ import annotations

import math

import torch

JITTER = 1e-6        # GPflow 1.5.1 settings.jitter (third-party default, unpinned here)
JITTER_LEVEL = 1e-6  # GPflow 1.5.1 settings.numerics.jitter_level


def _gen(seed, device):
    if seed is None:
        return None
    g = torch.Generator(device=device)
    s = [int(v) for v in (seed.tolist() if isinstance(seed, torch.Tensor) else seed)] if not isinstance(seed, int) \
        else [seed]
    h = 0
    for v in s:
        h = (h * 1000003 + (v & 0xFFFFFFFF)) & 0x7FFFFFFFFFFFFFFF
    g.manual_seed(h)
    return g


def _draw_indices(n, l, need_inv=False, device="cuda", generator=None):
    """low_rank_calculations.py:12-24: l of range(n) without replacement, the rest, [inverse map]."""
    idx = torch.randperm(int(n), device=device, generator=generator)
    idx_sampled, idx_not_sampled = idx[:l], idx[l:]
    if need_inv:
        inv_map = torch.argsort(idx)
        return idx_sampled, idx_not_sampled, inv_map
    return idx_sampled, idx_not_sampled


def Nystrom_map(X, kern, nys_samples=None, num_components=None, generator=None):
    """low_rank_calculations.py:27-63: Nystrom features (num_samples, num_components) with
    W = kern(S, S) + diag(jitter_level U[0,1)), W = U diag(S) U^T, features kern(X, S) U / sqrt(S + jitter)."""
    if nys_samples is None and num_components is None:
        raise ValueError('One of num_components or nys_samples should be given')
    if nys_samples is None:
        idx, _ = _draw_indices(X.shape[0], num_components, device=X.device, generator=generator)
        nys_samples = X[idx]
    c = nys_samples.shape[0]
    W = kern(nys_samples, nys_samples)
    W = W + torch.diag(JITTER_LEVEL * torch.rand(c, dtype=W.dtype, device=W.device, generator=generator))
    S, U = torch.linalg.eigh(W)
    D = torch.sqrt(S + JITTER)
    return (kern(X, nys_samples) @ U) / D[None, :]


def lr_hadamard_prod(A, B):
    """low_rank_calculations.py:66-76: [..., k1], [..., k2] -> [..., k1*k2] outer products."""
    C = A[..., :, None] * B[..., None, :]
    return C.reshape(*C.shape[:-2], C.shape[-2] * C.shape[-1])


def lr_hadamard_prod_rand(A, B, rank_bound, sparsity='sqrt', seeds=None):
    """low_rank_calculations.py:78-92."""
    if sparsity == 'lin':
        return lr_hadamard_prod_subsample(A, B, rank_bound, seeds)
    return lr_hadamard_prod_sparse(A, B, rank_bound, sparsity, seeds)


def _draw_n_rademacher_samples(n, seed=None, dtype=torch.float64, device="cuda", generator=None):
    """low_rank_calculations.py:94-103."""
    g = generator if generator is not None else _gen(seed, device)
    u = torch.rand(n, dtype=dtype, device=device, generator=g)
    return torch.where(u <= 0.5, torch.ones_like(u), -torch.ones_like(u))


def lr_hadamard_prod_subsample(A, B, num_components, seed=None):
    """low_rank_calculations.py:106-129: a random subset of num_components (i, j) products with
    Rademacher signs."""
    g = _gen(seed, A.device)
    k1, k2 = A.shape[-1], B.shape[-1]
    perm = torch.randperm(k1 * k2, device=A.device, generator=g)[:num_components]
    i, j = perm % k1, perm // k1  # reference combination order: idx1 varies fastest
    D = _draw_n_rademacher_samples(num_components, dtype=A.dtype, device=A.device, generator=g)
    return A[..., i] * B[..., j] * D


def _draw_n_gaussian_samples(n, seed=None, dtype=torch.float64, device="cuda", generator=None):
    """low_rank_calculations.py:132-139."""
    g = generator if generator is not None else _gen(seed, device)
    return torch.randn(n, dtype=dtype, device=device, generator=g)


def _draw_n_sparse_gaussian_samples(n, s, seed=None, dtype=torch.float64, device="cuda", generator=None):
    """low_rank_calculations.py:141-151: N(0,1) with probability 1/s, else 0."""
    g = generator if generator is not None else _gen(seed, device)
    u = torch.rand(n, dtype=dtype, device=device, generator=g)
    z = torch.randn(n, dtype=dtype, device=device, generator=g)
    return torch.where(u <= 1.0 / float(s), z, torch.zeros_like(z))


def lr_hadamard_prod_sparse(A, B, num_components, sparse_scale, seed=None):
    """low_rank_calculations.py:154-193: very sparse JL projection of the k1*k2 Hadamard products,
    scaled by sqrt(s / num_components)."""
    g = _gen(seed, A.device)
    k1, k2 = A.shape[-1], B.shape[-1]
    D = k1 * k2
    if sparse_scale == 'log':
        s = D / math.log(D)
    elif sparse_scale == 'sqrt':
        s = math.sqrt(D)
    else:
        raise ValueError("Unknown sparsity argument %s. Possible values are 'sqrt', 'log', 'lin'" % sparse_scale)
    R = _draw_n_sparse_gaussian_samples(D * num_components, s, dtype=A.dtype, device=A.device,
                                        generator=g).reshape(D, num_components)
    # reference combination (i, j) at row j * k1 + i (idx1 fastest); R3[i, j, r]
    R3 = R.reshape(k2, k1, num_components).permute(1, 0, 2)
    batch = A.shape[:-1]
    A2 = A.reshape(-1, k1)
    B2 = B.reshape(-1, k2)
    out = torch.empty((A2.shape[0], num_components), dtype=A.dtype, device=A.device)
    Rk = R3.permute(1, 0, 2).reshape(k2, k1 * num_components)  # (k2, k1 * rank)
    step = max(1, (1 << 27) // max(1, k1 * num_components))    # bound the (rows, k1, rank) temporary
    for r0 in range(0, A2.shape[0], step):
        T = (B2[r0:r0 + step] @ Rk).reshape(-1, k1, num_components)
        out[r0:r0 + step] = torch.einsum('nk,nkr->nr', A2[r0:r0 + step], T)
    return math.sqrt(s / num_components) * out.reshape(*batch, num_components)


# ----------------------------------------------------------------------------- signature_algs.py:162-222
def signature_kern_first_order_lr_feature(U, num_levels, rank_bound, sparsity='sqrt', seeds=None, difference=True,
                                          reference_level_bug=False):
    """signature_algs.py:162-193: (num_levels+1,) low-rank factors of the first-order signature kernel.

    The reference appends reduce_sum(U) at every level >= 2 (:191), so its levels 2..M repeat level 1;
    the evident intent, reduce_sum(P), is the default here (reference_level_bug=True reproduces :191)."""
    N = U.shape[0]
    Phi = [torch.ones((N, 1), dtype=U.dtype, device=U.device)]
    if difference:
        U = U[:, 1:, :] - U[:, :-1, :]
    Phi.append(U.sum(1))
    P = U
    for i in range(2, num_levels + 1):
        Pc = torch.cumsum(P, dim=1)
        P = torch.cat([torch.zeros_like(Pc[:, :1]), Pc[:, :-1]], 1)  # tf.cumsum(exclusive=True)
        P = lr_hadamard_prod_rand(U, P, rank_bound, sparsity, None if seeds is None else seeds[i - 2])
        Phi.append(U.sum(1) if reference_level_bug else P.sum(1))
    return Phi


def tensor_kern_lr_feature(U, num_levels, rank_bound, sparsity='sqrt', seeds=None):
    """signature_algs.py:195-222: (num_levels+1,) low-rank factors for inducing tensors."""
    T = U.shape[1]
    Phi = [torch.ones((T, 1), dtype=U.dtype, device=U.device)]
    k = 0
    for i in range(1, num_levels + 1):
        R = U[k]
        k += 1
        for j in range(1, i):
            R = lr_hadamard_prod_rand(U[k], R, rank_bound, sparsity, None if seeds is None else seeds[j - 1])
            k += 1
        Phi.append(R)
    return Phi
