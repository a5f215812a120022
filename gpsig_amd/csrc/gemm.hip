// gpsig_amd -- fp32 GEMM on the gfx950 matrix cores (v_mfma_f32_32x32x2_f32).
//
// The batched inner-product GEMMs of the wide-channel paths: the increment Gram <dx_i, dy_j> of the
// Goursat PDE (the reference builds it with tf.matmul, kernels_pde.py:176, before the solver) and the
// emission GEMMs of the wide-channel VJPs (point gradients = weights x points, the transpose of the
// reference's _square_dist GEMM, kernels.py:946-957).  f32 in / f32 accumulate: an MFMA is a k-ordered
// fp32 fma chain, the same numerics as the VALU dots of the fixed-channel kernels.
//
//   C[b] = alpha * op(A[b]) * op(B[b]) + beta * C[b]      op(X) = X or X^T, row-major, batch b = blockIdx.z
//
// 128 x 128 output tile per 4-wave workgroup (each wave 2 x 2 tiles of 32 x 32), K in steps of 16
// staged through double-buffered LDS (k-major images, so every MFMA operand read is conflict-free);
// operands of the next step are loaded while the current one is multiplied.
#include <hip/hip_runtime.h>

#include "../../include/gpsig_amd.h"
#include "gemm.h"

namespace gpsig {

typedef float f16v __attribute__((ext_vector_type(16)));
typedef float f4v __attribute__((ext_vector_type(4)));

struct GemmArgs {
  const float *A, *B;
  float *C;
  int M, N, K;
  long long lda, ldb, ldc, sA, sB, sC;
  float alpha, beta;
  int skip_lower;  // skip output tiles whose rows all lie below the block diagonal of (rb x cb) blocks
  int rb, cb;      // (tile rows -> block index row / rb, tile cols -> block index col / cb)
  int ksplit;      // > 1: blockIdx.z = K slice of kchunk columns, alpha * partial product -> P[slice] (M x N)
  int kchunk;
  float *P;
};

constexpr int GBM = 128, GBN = 128, GBK = 16, GPAD = 4;

// element (r, k) of op(X) with op = transpose flag T: X[r * ld + k] (N) or X[k * ld + r] (T)
template <bool T>
__device__ __forceinline__ void load_tile(const float *__restrict__ X, long long ld, int R, int Kd, int r0, int k0,
                                          float (&v)[8], int t) {
  if constexpr (!T) {
    // row-major rows r (128) x k (16): thread t -> k = 4 (t & 3) .. + 3, rows (t >> 2) + 64 e, one 16-byte
    // load per row, so a wave's load covers 16 rows x 64 contiguous bytes (a lane per row would touch 64
    // cache lines per instruction); v[4 e + c] = (row (t >> 2) + 64 e, k + c)
    typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));
    const int k = k0 + 4 * (t & 3), rb = r0 + (t >> 2);
    const float *p = X + (long long)rb * ld + k;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int r = rb + 64 * e;
      const float *q = p + (long long)64 * e * ld;
      if (r < R && k + 3 < Kd) {
        const f4u w = *reinterpret_cast<const f4u *>(q);
#pragma unroll
        for (int c = 0; c < 4; ++c) v[4 * e + c] = w[c];
      } else {
#pragma unroll
        for (int c = 0; c < 4; ++c) v[4 * e + c] = (r < R && k + c < Kd) ? q[c] : 0.0f;
      }
    }
  } else {
    // k-major: k (16) rows x r (128) contiguous: thread t -> k = t >> 4, r chunk (t & 15) * 8
    const int k = k0 + (t >> 4), rb = r0 + (t & 15) * 8;
    const float *p = X + (long long)k * ld + rb;
    const bool kok = k < Kd;
    if (kok && rb + 7 < R) {
      // two 16-byte loads (align 4: an odd ld leaves rows 4-byte aligned)
      typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));
      const f4u lo = *reinterpret_cast<const f4u *>(p), hi = *reinterpret_cast<const f4u *>(p + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = lo[e];
        v[4 + e] = hi[e];
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = (kok && rb + e < R) ? p[e] : 0.0f;
    }
  }
}

template <bool T>
__device__ __forceinline__ void store_tile(float (*S)[GBM + GPAD], const float (&v)[8], int t) {
  if constexpr (!T) {
    // (GBM + GPAD) = 4 mod 64 banks: a wave's 4 k-groups x 16 rows hit 64 distinct banks per store
    const int k = 4 * (t & 3), r = t >> 2;
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
      for (int c = 0; c < 4; ++c) S[k + c][r + 64 * e] = v[4 * e + c];
  } else {
    const int k = t >> 4, rb = (t & 15) * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) S[k][rb + e] = v[e];
  }
}

template <bool TA, bool TB>
__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) float As[2][GBK][GBM + GPAD];
  __shared__ __attribute__((aligned(16))) float Bs[2][GBK][GBN + GPAD];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int m0 = blockIdx.y * GBM, n0 = blockIdx.x * GBN;
  // every row block of this tile lies strictly below every column block: nothing to add (workgroup-uniform,
  // before any barrier)
  if (g.skip_lower && m0 / g.rb > (n0 + GBN - 1) / g.cb) return;
  const bool split = g.ksplit > 1;
  const int kz = split ? (int)blockIdx.z * g.kchunk : 0;  // first K column of this slice
  const int Kd = split ? min(g.K - kz, g.kchunk) : g.K;
  const long long zb = split ? 0 : blockIdx.z;
  // the slice's K offset moves the operand base: op(A) column kz, op(B) row kz
  const float *A = g.A + zb * g.sA + (TA ? (long long)kz * g.lda : (long long)kz);
  const float *B = g.B + zb * g.sB + (TB ? (long long)kz : (long long)kz * g.ldb);
  float *C = split ? g.P + (long long)blockIdx.z * g.M * g.N : g.C + zb * g.sC;
  const long long ldc = split ? g.N : g.ldc;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;

  f16v acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

  float va[8], vb[8];
  load_tile<TA>(A, g.lda, g.M, Kd, m0, 0, va, t);
  load_tile<!TB>(B, g.ldb, g.N, Kd, n0, 0, vb, t);
  store_tile<TA>(As[0], va, t);
  store_tile<!TB>(Bs[0], vb, t);
  __syncthreads();
  const int nk = (Kd + GBK - 1) / GBK;
  for (int ks = 0; ks < nk; ++ks) {
    const int buf = ks & 1;
    const bool more = ks + 1 < nk;
    if (more) {
      load_tile<TA>(A, g.lda, g.M, Kd, m0, (ks + 1) * GBK, va, t);
      load_tile<!TB>(B, g.ldb, g.N, Kd, n0, (ks + 1) * GBK, vb, t);
    }
#pragma unroll
    for (int kk = 0; kk < GBK; kk += 2) {
      const int kr = kk + (lane >> 5);
      float a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = As[buf][kr][wm + 32 * i + (lane & 31)];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = Bs[buf][kr][wn + 32 * j + (lane & 31)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(b[j], a[i], acc[i][j], 0, 0, 0);
    }
    if (more) {
      store_tile<TA>(As[buf ^ 1], va, t);
      store_tile<!TB>(Bs[buf ^ 1], vb, t);
    }
    __syncthreads();
  }
  // The MFMA runs with B as its first operand, so each 32 x 32 tile holds C^T: lane -> C row (lane & 31),
  // register r -> C column 4 (lane >> 5) + 8 (r >> 2) + (r & 3).  Four consecutive registers are four
  // consecutive columns of one row: one 16-byte store each (align 4: rows of an odd ldc are not 16-byte
  // aligned), a quarter of the store instructions of a column-per-lane epilogue.
  typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));
  const bool plain = split || g.beta == 0.0f;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = m0 + wm + 32 * i + (lane & 31);
    if (row >= g.M) continue;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int col = n0 + wn + 32 * j + 4 * (lane >> 5) + 8 * q;
        float *c = C + (long long)row * ldc + col;
        f4u v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = g.alpha * acc[i][j][4 * q + e];
        if (col + 3 < g.N) {
          if (!plain) {
            const f4u o = *reinterpret_cast<const f4u *>(c);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = __builtin_fmaf(g.beta, o[e], v[e]);
          }
          *reinterpret_cast<f4u *>(c) = v;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (col + e < g.N) c[e] = plain ? v[e] : __builtin_fmaf(g.beta, c[e], v[e]);
        }
      }
  }
}

// C = beta C + sum of the ksplit partial products (fixed order: deterministic)
__global__ __launch_bounds__(256) void gemm_splitk_reduce(const float *__restrict__ P, int ksplit, int M, int N,
                                                          float beta, float *__restrict__ C, long long ldc) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long long)M * N) return;
  const int row = (int)(idx / N), col = (int)(idx % N);
  float v = 0.0f;
  for (int z = 0; z < ksplit; ++z) v += P[(long long)z * M * N + idx];
  float *c = C + (long long)row * ldc + col;
  *c = beta == 0.0f ? v : __builtin_fmaf(beta, *c, v);
}

// Split-K slices for a single (unbatched) product whose output tiles alone would not fill the chip:
// about 512 workgroups, slices of at least 512 K columns.  Partial buffer: ksplit * M * N floats.
inline int gemm_ksplit(int M, int N, int K) {
  const long long tiles = (long long)((M + GBM - 1) / GBM) * ((N + GBN - 1) / GBN);
  int ks = (int)((512 + tiles - 1) / tiles);
  const int kmax = (K + 511) / 512;
  if (ks > kmax) ks = kmax;
  if (ks > 64) ks = 64;
  return ks < 1 ? 1 : ks;
}
size_t gemm_splitk_bytes(int M, int N, int K) {
  const int ks = gemm_ksplit(M, N, K);
  return ks > 1 ? (size_t)ks * M * N * sizeof(float) : 0;
}

// see gemm.h
int gemm_f32(hipStream_t s, bool transA, bool transB, int M, int N, int K, float alpha, const float *A,
             long long lda, long long sA, const float *B, long long ldb, long long sB, float beta, float *C,
             long long ldc, long long sC, int batch, int skip_rb, int skip_cb, float *partial, size_t partial_bytes) {
  if (M <= 0 || N <= 0 || batch <= 0) return GPSIG_OK;
  if (K <= 0) return GPSIG_EINVAL;
  int ks = (batch == 1 && partial && skip_rb == 0) ? gemm_ksplit(M, N, K) : 1;
  int kc = K, nsl = 1;
  // the largest split (up to gemm_ksplit's) whose nsl partial products fit the caller's scratch
  for (; ks > 1; --ks) {
    kc = (((K + ks - 1) / ks + GBK - 1) / GBK) * GBK;
    nsl = (K + kc - 1) / kc;
    if (nsl > 1 && (size_t)nsl * (size_t)M * (size_t)N * sizeof(float) <= partial_bytes) break;
  }
  if (ks <= 1) {
    kc = K;
    nsl = 1;
  }
  GemmArgs g{A, B, C, M, N, K, lda, ldb, ldc, sA, sB, sC, alpha, beta, skip_rb > 0 ? 1 : 0,
             skip_rb > 0 ? skip_rb : 1, skip_cb > 0 ? skip_cb : 1, nsl, kc, partial};
  dim3 grid((N + GBN - 1) / GBN, (M + GBM - 1) / GBM, nsl > 1 ? nsl : batch);
  if (grid.y > 65535 || grid.z > 65535) return GPSIG_EUNSUPPORTED;
  if (!transA && !transB) hipLaunchKernelGGL((gemm_f32_kernel<false, false>), grid, dim3(256), 0, s, g);
  else if (!transA && transB) hipLaunchKernelGGL((gemm_f32_kernel<false, true>), grid, dim3(256), 0, s, g);
  else if (transA && !transB) hipLaunchKernelGGL((gemm_f32_kernel<true, false>), grid, dim3(256), 0, s, g);
  else hipLaunchKernelGGL((gemm_f32_kernel<true, true>), grid, dim3(256), 0, s, g);
  if (nsl > 1) {
    const long long tot = (long long)M * N;
    hipLaunchKernelGGL(gemm_splitk_reduce, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, partial, nsl, M, N,
                       beta, C, ldc);
  }
  return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
}

}  // namespace gpsig

// Test entry of the GEMM (include/gpsig_amd.h)
extern "C" int gpsig_gemm_f32(int transA, int transB, int M, int N, int K, float alpha, const float *A, long long lda,
                              const float *B, long long ldb, float beta, float *C, long long ldc,
                              gpsig_stream_t stream) {
  if (!A || !B || !C) return GPSIG_EINVAL;
  return gpsig::gemm_f32(reinterpret_cast<hipStream_t>(stream), transA != 0, transB != 0, M, N, K, alpha, A, lda, 0,
                         B, ldb, 0, beta, C, ldc, 0, 1, 0, 0, nullptr, 0);
}

// As gpsig_gemm_f32 with K split over partial products summed in a fixed order (workspace of
// gpsig_gemm_splitk_bytes(M, N, K) bytes).
extern "C" size_t gpsig_gemm_splitk_bytes(int M, int N, int K) { return gpsig::gemm_splitk_bytes(M, N, K); }
extern "C" int gpsig_gemm_f32_splitk(int transA, int transB, int M, int N, int K, float alpha, const float *A,
                                     long long lda, const float *B, long long ldb, float beta, float *C, long long ldc,
                                     void *workspace, size_t workspace_bytes, gpsig_stream_t stream) {
  if (!A || !B || !C) return GPSIG_EINVAL;
  const size_t need = gpsig::gemm_splitk_bytes(M, N, K);
  if (need && (!workspace || workspace_bytes < need)) return GPSIG_EWORKSPACE;
  return gpsig::gemm_f32(reinterpret_cast<hipStream_t>(stream), transA != 0, transB != 0, M, N, K, alpha, A, lda, 0,
                         B, ldb, 0, beta, C, ldc, 0, 1, 0, 0, need ? static_cast<float *>(workspace) : nullptr,
                         need ? workspace_bytes : 0);
}
