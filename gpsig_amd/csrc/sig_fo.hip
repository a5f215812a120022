// gpsig_amd -- first-order truncated signature kernel Gram on gfx950.
//
// Replaces, for order == 1, the dataflow of gpsig/kernels.py:209-238 (_K_seq) +
// gpsig/signature_algs.py:8-35 (signature_kern_first_order):
//     dM = second difference of the base-kernel grid M(x_i, y_j)        (signature_algs.py:26)
//     K_1 = sum dM,  R_m = dM * cumsum_x(cumsum_x(R_{m-1})), K_m = sum R_m   (:28-33)
// without materialising M or R: one lane group of LP lanes owns one pair (a, b) and streams the
// rows i of the dM grid; each lane keeps W columns j.  Per row and level the exclusive column
// prefix S_m(i, j) = sum_{i'<i, j'<j} R_m(i', j') is the exclusive scan over j of the running
// column sums C_m(j) = sum_{i'<i} R_m(i', j), so per pair the state is (M x W) registers per lane
// and the only cross-lane traffic is one DPP scan per level per row.  K_m = sum_j C_m(j) at the end.
//
#include "sig_fo.h"

namespace gpsig {

// ------------------------------------------------------------------------------------ features
template <int DP>
__global__ __launch_bounds__(256) void features_kernel(const float *__restrict__ X, int n, int l, int d,
                                                       float *__restrict__ F) {
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long long)n * l) return;
  const int i = (int)(idx % l);
  const float *x = X + idx * d;
  constexpr int FS = feat_stride(DP);
  float *f = F + idx * FS;
  float h = 0.0f;
  double gx = 0.0;  // <x, dx> accumulated in fp64, rounded once
#pragma unroll
  for (int k = 0; k < DP; ++k) {
    const float xv = k < d ? x[k] : 0.0f;
    const float dv = (k < d && i + 1 < l) ? x[d + k] - xv : 0.0f;
    f[k] = xv;
    f[DP + k] = dv;
    h = __builtin_fmaf(dv, dv, h);
    gx = __builtin_fma((double)xv, (double)dv, gx);
  }
  f[2 * DP] = 0.5f * h;
  f[2 * DP + 1] = (float)(gx + 0.5 * (double)h);
#pragma unroll
  for (int k = 2 * DP + 2; k < FS; ++k) f[k] = 0.0f;
}

// ------------------------------------------------------------------------------------ launchers
template <int DP>
static int launch_features(const float *X, int n, int l, int d, float *F, hipStream_t s) {
  const long long tot = (long long)n * l;
  const int blocks = (int)((tot + 255) / 256);
  hipLaunchKernelGGL(features_kernel<DP>, dim3(blocks), dim3(256), 0, s, X, n, l, d, F);
  return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
}

int features(const float *X, int n, int l, int d, int DP, float *F, hipStream_t s) {
  switch (DP) {
#define CASE(v) \
  case v: return launch_features<v>(X, n, l, d, F, s);
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8) CASE(16) CASE(32) CASE(64)
#undef CASE
    default: return GPSIG_EUNSUPPORTED;
  }
}

template <int DP, int M>
int sig_fo_launch_dpm(const SigArgs &a, int seed, long long nblocks, hipStream_t s);

template <int DP>
static int fo_dp(const SigArgs &a, int seed, long long nblocks, hipStream_t s) {
  switch (a.M) {
    case 1: return sig_fo_launch_dpm<DP, 1>(a, seed, nblocks, s);
    case 2: return sig_fo_launch_dpm<DP, 2>(a, seed, nblocks, s);
    case 3: return sig_fo_launch_dpm<DP, 3>(a, seed, nblocks, s);
    case 4: return sig_fo_launch_dpm<DP, 4>(a, seed, nblocks, s);
    case 5: return sig_fo_launch_dpm<DP, 5>(a, seed, nblocks, s);
    case 6: return sig_fo_launch_dpm<DP, 6>(a, seed, nblocks, s);
    case 7: return sig_fo_launch_dpm<DP, 7>(a, seed, nblocks, s);
    case 8: return sig_fo_launch_dpm<DP, 8>(a, seed, nblocks, s);
    default: return GPSIG_EUNSUPPORTED;
  }
}

int sig_fo_launch(const SigArgs &a0, int DP, int seed, long long nblocks, hipStream_t s) {
  const Geo g = DP == 0 ? fo_geometry_wide(a0.l2, seed) : fo_geometry(a0.l2, DP, a0.M, a0.mfma != 0, a0.dmbuf ? -1 : seed);
  if (g.W == 0) return GPSIG_EUNSUPPORTED;
  SigArgs a = a0;
  a.nblk = fo_blocks(a0.l2, seed == SEED_RBF_DIFF || seed == SEED_LIN_DIFF, g);
  switch (DP) {
#define CASE(v) \
  case v: return fo_dp<v>(a, seed, nblocks, s);
    CASE(0) CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(8)
#undef CASE
    default: return GPSIG_EUNSUPPORTED;
  }
}

int fo_lanes_per_pair(int l2, int DP, int M, bool mf, int seed, bool split) {
  return (DP == 0 ? fo_geometry_wide(l2, seed) : fo_geometry(l2, DP, M, mf, split ? -1 : seed)).LP;
}
// the wide forward's (columns per lane, lanes per pair)
void fo_wide_geo(int l2, int seed, int *W, int *LP) {
  const Geo g = fo_geometry_wide(l2, seed);
  *W = g.W;
  *LP = g.LP;
}

// ------------------------------------------------------------------------------------ wide records
__global__ __launch_bounds__(256) void wide_records_kernel(const float *__restrict__ X, int n, int l, int d,
                                                           float *__restrict__ R) {
  const int lw = wide_lw(l);
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long long)n * lw) return;
  const int sq = (int)(idx / lw), j = (int)(idx % lw);
  const int jj = j < l ? j : l - 1;
  const bool inc = j + 1 < l;
  const float *x = X + ((long long)sq * l + jj) * d;
  float *r = R + (long long)sq * wide_rec_floats(d, l) + j;
  float h = 0.0f;
  double gx = 0.0;
  for (int k = 0; k < d; ++k) {
    const float xv = x[k];
    const float dv = inc ? x[d + k] - xv : 0.0f;
    r[(long long)k * lw] = xv;
    r[(long long)(d + k) * lw] = dv;
    h = __builtin_fmaf(dv, dv, h);
    gx = __builtin_fma((double)xv, (double)dv, gx);
  }
  r[(long long)2 * d * lw] = 0.5f * h;
  r[(long long)(2 * d + 1) * lw] = (float)(gx + 0.5 * (double)h);
}

int wide_records(const float *X, int n, int l, int d, float *R, hipStream_t s) {
  const long long tot = (long long)n * wide_lw(l);
  hipLaunchKernelGGL(wide_records_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, X, n, l, d, R);
  return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
}

// one chunk of the split diagnostic: FO_SPLIT_BLOCKS workgroups x 4 waves x G pairs, (l1 - 1) rows of
// LP * W cells each (0: the geometry has column blocks or W < 4, where the split does not apply)
size_t fo_split_bytes(int l1, int l2, int DP, int M) {
  const Geo g = fo_geometry(l2, DP, M, false);
  if (g.W < 4 || fo_blocks(l2, true, g) != 1) return 0;
  return (size_t)FO_SPLIT_BLOCKS * 4 * (64 / g.LP) * (size_t)(l1 - 1) * g.LP * g.W * sizeof(float);
}

}  // namespace gpsig
