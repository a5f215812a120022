"""GPU parity for long sequences: the first-order Gram in column blocks (sig_fo_kernel `nblk`, LP = 64,
carries in LDS) beyond the 64 * fo_wmax points one lane group covers -- the reference's cython/TF
paths have no length cap (signature_algs.py:8-35 over any L).  Checked against the float64 oracle
(oracle/kernels_ref.py) at sizes it finishes in seconds, and for consistency across the block
boundary: a pair of sequences and their truncation at a block edge agree with the unblocked kernel."""
import numpy as np
import pytest
import torch

from conftest import norm_rel_err
from oracle import kernels_ref as kr

pytestmark = pytest.mark.gpu
TOL = 1e-5
DEV = "cuda"


def t(x):
    return torch.as_tensor(np.asarray(x), device=DEV)


def walks(n, l, d, seed):
    rng = np.random.default_rng(seed)
    return np.cumsum(rng.standard_normal((n, l, d)), 1) / np.sqrt(l * d)


@pytest.mark.parametrize("L,D,M,base,diff", [
    (600, 3, 4, "rbf", True),      # 2 blocks at W = 8 (511 cells per block)
    (1100, 2, 3, "rbf", True),     # 3 blocks
    (600, 8, 6, "rbf", True),      # W = 4: 255 cells per block, 3 blocks
    (520, 4, 5, "linear", True),
    (600, 3, 4, "rbf", False),     # point seeds (difference=False)
    (513, 5, 2, "linear", False),
])
def test_long_sequences_match_oracle(L, D, M, base, diff):
    from gpsig_amd import ops
    X = walks(5, L, D, L + D)
    Y = walks(3, L - 37, D, L + D + 1)
    ref = kr.SignatureKernelRef(L * D, D, M, normalization=False, base=base, difference=diff)
    got = ops.sig_gram(t(X), None, M, base=base, difference=diff).cpu().numpy()
    exp = ref.K_seq(X, X)
    assert (norm_rel_err(got[1:], exp[1:], axis_levels=True) < TOL).all()
    got = ops.sig_gram(t(X), t(Y), M, base=base, difference=diff).cpu().numpy()
    exp = ref.K_seq(X, Y)
    assert (norm_rel_err(got[1:], exp[1:], axis_levels=True) < TOL).all()
    d = ops.sig_diag(t(X), M, base=base, difference=diff).cpu().numpy()
    assert (norm_rel_err(d[1:], np.stack([np.diagonal(e) for e in ref.K_seq(X, X)])[1:], axis_levels=True) < TOL).all()


@pytest.mark.parametrize("L,D,M,order,base", [
    (300, 3, 5, 2, "rbf"),       # W = 4: 255 cells per block, 2 blocks
    (300, 4, 5, 3, "linear"),
    (300, 3, 5, 4, "rbf"),
    (300, 2, 5, 5, "linear"),    # W = 2: 127 cells per block, 3 blocks
    (600, 2, 4, 2, "rbf"),       # 3 blocks
    (200, 3, 8, 8, "linear"),    # order 8 (exact signature at M = 8): W = 1, 4 blocks of 63 cells
])
def test_long_higher_order_matches_oracle(L, D, M, order, base):
    """Higher-order recursion (signature_algs.py:37-74) in column blocks: the exclusive column scans of
    every level and block index carry across the block seams through LDS."""
    from gpsig_amd import ops
    X = walks(4, L, D, L + 7 * order)
    Y = walks(2, L - 29, D, L + 7 * order + 1)
    ref = kr.SignatureKernelRef(L * D, D, M, normalization=False, base=base, order=order)
    got = ops.sig_gram(t(X), None, M, order=order, base=base).cpu().numpy()
    assert (norm_rel_err(got[1:], ref.K_seq(X, X)[1:], axis_levels=True) < TOL).all()
    got = ops.sig_gram(t(X), t(Y), M, order=order, base=base).cpu().numpy()
    assert (norm_rel_err(got[1:], ref.K_seq(X, Y)[1:], axis_levels=True) < TOL).all()
    d = ops.sig_diag(t(X), M, order=order, base=base).cpu().numpy()
    exp = np.stack([np.diagonal(e) for e in ref.K_seq(X, X)])
    assert (norm_rel_err(d[1:], exp[1:], axis_levels=True) < TOL).all()


def test_long_normalised_K_and_saved_state_gradient_path():
    """SignatureRBF.K at L = 700 (normalised, fused epilogue) vs the oracle; the training forward (saved
    VJP state, gpsig_sig_gram_state) at the same length writes the same Gram."""
    import gpsig_amd
    from gpsig_amd import _lib as Lb
    from gpsig_amd import ops
    N, L, D, M = 6, 700, 3, 4
    X = walks(N, L, D, 3)
    k = gpsig_amd.SignatureRBF(L * D, D, M)
    got = k.K(t(X.reshape(N, -1))).cpu().numpy()
    exp = kr.SignatureKernelRef(L * D, D, M).K(X.reshape(N, -1))
    assert norm_rel_err(got, exp) < TOL
    Xd = t(X).float()
    st = torch.zeros(ops.sig_state_numel(N, None, L, M), dtype=torch.float32, device=DEV)
    a = ops.sig_gram(Xd, None, M, state=st).cpu().numpy()
    b = ops.sig_gram(Xd, None, M).cpu().numpy()
    np.testing.assert_array_equal(a, b)
    assert torch.isfinite(st).all()


def test_block_boundary_consistency():
    """Cells on either side of a block edge: the Gram of sequences of exactly 512 points (one block of
    511 cells at W = 8, LP = 64) and of 513 points (two blocks, the second holding one cell) both match
    the oracle -- the halo point and carry are exact at the seam."""
    from gpsig_amd import ops
    for L in (512, 513, 1023, 1024):
        X = walks(4, L, 3, L)
        ref = kr.SignatureKernelRef(L * 3, 3, 5, normalization=False)
        got = ops.sig_gram(t(X), None, 5).cpu().numpy()
        assert (norm_rel_err(got[1:], ref.K_seq(X, X)[1:], axis_levels=True) < TOL).all(), L


def test_carry_too_large_raises():
    from gpsig_amd import _lib as Lb
    from gpsig_amd import ops
    X = torch.zeros((2, 6000, 2), device=DEV)  # 4 waves x 5999 rows x 7 levels x 4 B > 160 KiB of LDS
    with pytest.raises(Lb.GpsigError):
        ops.sig_gram(X, None, 8)


@pytest.mark.parametrize("L,n,solver", [(500, 2, 1), (500, 2, 0), (300, 2, 1), (600, 1, 1), (1200, 0, 1), (257, 2, 1)])
def test_long_pde_matches_oracle(L, n, solver):
    """Goursat PDE beyond 64 W refined columns (column blocks of pde_rep_kernel, boundary column in LDS):
    L = 500 at dyadic 2 is 1996 refined columns, which the reference's gpu_op refuses
    (kernels_pde.py:53) and its Cython path (sigKer_fast.pyx:15-62) solves; here both the diagonal
    (solver 0 takes the solver-1 update on the diagonal, sigKer_fast.pyx:59) and the cross Gram vs the
    C restatement (oracle/pde), which is bitwise the reference's Cython solver (tests/test_oracle.py)."""
    from oracle import pde
    from gpsig_amd import ops
    rng = np.random.default_rng(L + n)
    X = np.cumsum(rng.standard_normal((3, L, 4)), 1) / np.sqrt(L * 4) * 2
    Y = np.cumsum(rng.standard_normal((2, L - 11, 4)), 1) / np.sqrt(L * 4) * 2
    got = ops.pde_diag(t(X), n, solver).cpu().numpy()
    exp = pde.pde_diag(X, n, solver)
    assert np.abs(got - exp).max() / np.abs(exp).max() < TOL
    if solver == 1:
        assert norm_rel_err(ops.pde_gram(t(X), t(Y), n, 1).cpu().numpy(), pde.pde_gram(X, Y, n, 1)) < TOL
        assert norm_rel_err(ops.pde_gram(t(X), None, n, 1).cpu().numpy(), pde.pde_gram(X, X, n, 1)) < TOL


def test_long_pde_kernel_class_kdiag():
    """UntruncSignatureKernel(order=2).Kdiag at L = 500 (the reference's gpu_op asserts here)."""
    import gpsig_amd
    from oracle import pde
    L, D = 500, 3
    X = walks(4, L, D, 9) * 2
    k = gpsig_amd.UntruncSignatureKernel(L * D, D, order=2)
    got = k.Kdiag(t(X.reshape(4, -1))).cpu().numpy()
    exp = pde.pde_diag(X, 2, 1)
    assert np.abs(got - exp).max() / np.abs(exp).max() < TOL


@pytest.mark.parametrize("L,M,order,base", [(200, 5, 5, "linear"), (500, 5, 5, "linear"), (300, 4, 3, "rbf"),
                                            (260, 6, 2, "rbf")])
def test_higher_order_split_forward_matches_plain(L, M, order, base, monkeypatch):
    """The split higher-order forward (sig_ho.hip SPLIT: one pair per workgroup, column blocks side by side on
    the 4 waves, the block carries exchanged through LDS) against the plain kernel (column blocks one after
    another on one wave, GPSIG_HO_SPLIT=0): the same cells and recursion, the column scans combined in another
    order, so the levels agree to fp32 rounding; K(X, Y), K(X) and the diagonal."""
    from gpsig_amd import ops
    D = 24 if base == "linear" else 4  # linear order >= M at few channels runs as signature features instead
    rng = np.random.default_rng(L + M)
    X = np.cumsum(rng.standard_normal((3, L, D)), 1) / np.sqrt(L * D)
    Y = np.cumsum(rng.standard_normal((2, L - 9, D)), 1) / np.sqrt(L * D)
    Xt, Yt = (torch.tensor(v, device="cuda", dtype=torch.float32) for v in (X, Y))

    def levels():
        return [ops.sig_gram(Xt, Yt, M, order=order, base=base).cpu().numpy(),
                ops.sig_gram(Xt, None, M, order=order, base=base).cpu().numpy(),
                ops.sig_diag(Xt, M, order=order, base=base).cpu().numpy()]

    split = levels()
    monkeypatch.setenv("GPSIG_HO_SPLIT", "0")
    plain = levels()
    for g, r in zip(split, plain):
        for m in range(1, M + 1):
            assert np.abs(g[m] - r[m]).max() <= 2e-6 * np.abs(r[m]).max(), m
