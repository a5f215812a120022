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


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("levels_out", [False, True])
def test_multi_rank_layout_assembles_bitwise_on_one_gpu(world, levels_out):
    """The world-2/4/8 data path on one GPU: every rank's share is computed by the real HIP kernel
    (sym_local_blocks: chunks r and 2P-1-r of the upper triangle, fused normalisation), the shares are
    concatenated in rank order exactly as all_gather_into_tensor lays them out, and gpsig_sym_assemble
    rebuilds the matrix from distributed.row_offsets -- bitwise the single-call Gram.  Also the
    row-block cross Gram (cross_local_block + cross_from_gathered)."""
    import gpsig_amd
    from gpsig_amd import _lib as Lb
    from gpsig_amd import distributed as D
    N, L, Dm, M = 37, 24, 3, 4  # N not a multiple of 2 * world: ragged chunks
    X = torch.tensor(walks(N, L, Dm, 3).reshape(N, -1), device=DEV)
    X2 = torch.tensor(walks(11, L, Dm, 4).reshape(11, -1), device=DEV)
    k = gpsig_amd.SignatureRBF(L * Dm, Dm, M)
    Xs = k._prep(X)
    rs = k._rsqrt_diag(Xs)
    mode = Lb.OUT_NORM_LEVELS if levels_out else Lb.OUT_NORM_SUM
    kw = dict(rs1=rs, rs2=rs, scale=k._scale_vec(Xs.device), jitter=k.jitter, order=1, base="rbf", difference=True)
    full = D.sharded_sym_gram(Xs, M, out_mode=mode, **kw)  # world 1: one launch over all rows
    levels = M + 1 if levels_out else 1
    shares = [D.sym_local_blocks(Xs, M, r, world, out_mode=mode, **kw) for r in range(world)]
    gathered = torch.cat([s.reshape(-1, N) for s in shares], 0)
    got = D.sym_from_gathered(gathered, N, world, levels)
    assert torch.equal(got.reshape(full.shape), full)
    # cross Gram: P row blocks
    X2s = k._prep(X2)
    rs2 = k._rsqrt_diag(X2s)
    kwc = dict(rs1=rs, rs2=rs2, scale=k._scale_vec(Xs.device), jitter=k.jitter, order=1, base="rbf", difference=True)
    fullc = D.sharded_cross_gram(Xs, X2s, M, out_mode=mode, **kwc)
    blocks = torch.stack([D.cross_local_block(Xs, X2s, M, r, world, out_mode=mode, **kwc) for r in range(world)])
    gotc = D.cross_from_gathered(blocks, N)
    assert torch.equal(gotc.reshape(fullc.shape), fullc)
