// gpsig_amd -- host entry of the fp32 matrix-core GEMM (gemm.hip), shared by every translation unit that
// issues one (wide-channel VJPs, PDE increment tiles, higher-order tiles).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

namespace gpsig {

// C[b] = alpha op(A[b]) op(B[b]) + beta C[b] (row-major; transA / transB select op).  skip_rb/skip_cb > 0:
// op(A) rows and op(B) columns come in blocks of skip_rb / skip_cb and the inputs vanish for row block >
// column block (upper-triangle pair layouts): those output tiles are left untouched.
// partial / partial_bytes: scratch that lets an unbatched product split K into partial products (summed in a
// fixed order).  The split is clamped to what partial_bytes holds (no split when it holds fewer than two
// partial products), so a caller can never be overrun by a split it did not size for.
int gemm_f32(hipStream_t s, bool transA, bool transB, int M, int N, int K, float alpha, const float *A, long long lda,
             long long sA, const float *B, long long ldb, long long sB, float beta, float *C, long long ldc,
             long long sC, int batch, int skip_rb, int skip_cb, float *partial, size_t partial_bytes);

// Bytes of partial products gemm_f32 would use for an unbatched (M, N, K) product with unlimited scratch
// (0: it would not split).
size_t gemm_splitk_bytes(int M, int N, int K);

}  // namespace gpsig
