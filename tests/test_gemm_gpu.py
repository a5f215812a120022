"""The matrix-core fp32 GEMM (gpsig_amd/csrc/gemm.hip, v_mfma_f32_32x32x2_f32) that the wide-channel paths
use for their inner-product GEMMs, against a float64 torch matmul: every transpose combination, ragged
shapes (partial 128-tiles and 16-steps of K), alpha / beta."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("ta", [0, 1])
@pytest.mark.parametrize("tb", [0, 1])
@pytest.mark.parametrize("M,N,K", [(1, 1, 1), (37, 130, 5), (128, 128, 16), (300, 77, 129), (513, 260, 46)])
def test_gemm_matches_float64(ta, tb, M, N, K):
    from gpsig_amd import _lib as L
    rng = np.random.default_rng(M * 7 + N * 3 + K + 10 * ta + 20 * tb)
    A = rng.standard_normal((K, M) if ta else (M, K))
    B = rng.standard_normal((N, K) if tb else (K, N))
    C0 = rng.standard_normal((M, N))
    At = torch.as_tensor(A, device=DEV, dtype=torch.float32)
    Bt = torch.as_tensor(B, device=DEV, dtype=torch.float32)
    C = torch.as_tensor(C0, device=DEV, dtype=torch.float32)
    lib = L.load()
    rc = lib.gpsig_gemm_f32(ta, tb, M, N, K, 0.5, At.data_ptr(), At.shape[1], Bt.data_ptr(), Bt.shape[1], 2.0,
                            C.data_ptr(), N, torch.cuda.current_stream().cuda_stream)
    L.check(rc, "gpsig_gemm_f32")
    opA = A.T if ta else A
    opB = B.T if tb else B
    exp = 0.5 * opA @ opB + 2.0 * C0
    got = C.cpu().double().numpy()
    scale = 0.5 * np.abs(opA) @ np.abs(opB) + 2.0 * np.abs(C0)
    assert (np.abs(got - exp) <= 2e-6 * scale + 1e-6).all()
