// gpsig_amd -- extern "C" entry of the tens-vs-seq VJP (include/gpsig_amd.h, gpsig_tens_vs_seq_vjp):
// argument checks, time-major features, the kernel (sig_tvs_bwd.h) and the transpose of the
// time-major sequence gradient into the caller's (n, l, d) buffer.
#include "sig_tvs_bwd.h"

namespace gpsig {
size_t tvs_features_bytes(int n, int l, int d);
int tvs_features_launch(const float *X, int n, int l, int d, float *Ft, hipStream_t s);
template <int DP, bool INCR>
int tvs_bwd_launch_dp(const TvsBwdArgs &a, int M, bool rbf, bool diff, hipStream_t s);
size_t tvs_bwd_wide_workspace(int n, int l, int d, int lt, int t);
int tvs_bwd_wide(const float *Z, int lt, int t, int incr, int d, const float *X, int n, int l, int M, bool rbf,
                 bool diff, const float *gout, float *gZ, float *gX, const float *state, void *workspace,
                 size_t workspace_bytes, hipStream_t s);

// gX[seq][s][q] += gXt[(s * d + q) * n + seq]
__global__ __launch_bounds__(256) void tvs_gx_add_kernel(const float *__restrict__ gXt, int n, int l, int d,
                                                         float *__restrict__ gX) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long long)n * l * d) return;
  const int seq = (int)(idx / ((long long)l * d));
  const int r = (int)(idx % ((long long)l * d));
  gX[idx] += gXt[(long long)r * n + seq];
}

static size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }
static int tvs_bwd_pad(int d) { return d <= 2 ? 2 : d <= 4 ? 4 : d <= 6 ? 6 : d <= 8 ? 8 : d <= 12 ? 12 : d <= 16 ? 16 : 0; }

}  // namespace gpsig

using namespace gpsig;

extern "C" size_t gpsig_tens_vjp_workspace_bytes(int n, int l, int d) {
  return tvs_features_bytes(n, l, d) + align256((size_t)n * l * d * sizeof(float));
}

// Channel counts past the instantiations (d > 16): point-weight tiles + GEMMs (sig_tvs_bwd_wide.hip); the
// workspace depends on the tensors too
extern "C" size_t gpsig_tens_vjp_wide_workspace_bytes(int n, int l, int d, int lt, int t) {
  return tvs_bwd_wide_workspace(n, l, d, lt, t);
}

extern "C" int gpsig_tens_vs_seq_vjp(const float *Z, int lt, int t, int increments, int d, const float *X, int n,
                                     int l, int num_levels, int base_kind, int difference, const float *gout,
                                     float *gZ, float *gX, const float *state,
                                     void *workspace, size_t workspace_bytes, gpsig_stream_t stream) {
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (!Z || !X || !gout || !gZ || !gX || lt <= 0 || t <= 0 || n <= 0 || d <= 0 || l < (difference ? 2 : 1) ||
      num_levels < 1)
    return GPSIG_EINVAL;
  if (lt != num_levels * (num_levels + 1) / 2) return GPSIG_EINVAL;
  if (state && !difference) return GPSIG_EINVAL;  // the saved state comes from the difference fast paths
  if (base_kind != GPSIG_BASE_RBF && base_kind != GPSIG_BASE_LINEAR) return GPSIG_EUNSUPPORTED;
  const int DP = tvs_bwd_pad(d);
  if (num_levels > 8 || t > 65535) return GPSIG_EUNSUPPORTED;
  if (DP == 0)
    return tvs_bwd_wide(Z, lt, t, increments, d, X, n, l, num_levels, base_kind == GPSIG_BASE_RBF, difference != 0, gout,
                        gZ, gX, state, workspace, workspace_bytes, s);
  if (!workspace || workspace_bytes < gpsig_tens_vjp_workspace_bytes(n, l, d)) return GPSIG_EWORKSPACE;
  float *Ft = static_cast<float *>(workspace);
  float *gXt = reinterpret_cast<float *>(static_cast<char *>(workspace) + tvs_features_bytes(n, l, d));
  int rc = tvs_features_launch(X, n, l, d, Ft, s);
  if (rc) return rc;
  if (hipMemsetAsync(gXt, 0, (size_t)n * l * d * sizeof(float), s) != hipSuccess) return GPSIG_ELAUNCH;
  TvsBwdArgs a{Z, Ft, t, n, l, d, gout, gZ, gXt, state};
  const bool rbf = base_kind == GPSIG_BASE_RBF;
  switch (DP * 2 + (increments ? 1 : 0)) {
    case 4: rc = tvs_bwd_launch_dp<2, false>(a, num_levels, rbf, difference != 0, s); break;
    case 5: rc = tvs_bwd_launch_dp<2, true>(a, num_levels, rbf, difference != 0, s); break;
    case 8: rc = tvs_bwd_launch_dp<4, false>(a, num_levels, rbf, difference != 0, s); break;
    case 9: rc = tvs_bwd_launch_dp<4, true>(a, num_levels, rbf, difference != 0, s); break;
    case 12: rc = tvs_bwd_launch_dp<6, false>(a, num_levels, rbf, difference != 0, s); break;
    case 13: rc = tvs_bwd_launch_dp<6, true>(a, num_levels, rbf, difference != 0, s); break;
    case 16: rc = tvs_bwd_launch_dp<8, false>(a, num_levels, rbf, difference != 0, s); break;
    case 17: rc = tvs_bwd_launch_dp<8, true>(a, num_levels, rbf, difference != 0, s); break;
    case 24: rc = tvs_bwd_launch_dp<12, false>(a, num_levels, rbf, difference != 0, s); break;
    case 25: rc = tvs_bwd_launch_dp<12, true>(a, num_levels, rbf, difference != 0, s); break;
    case 32: rc = tvs_bwd_launch_dp<16, false>(a, num_levels, rbf, difference != 0, s); break;
    case 33: rc = tvs_bwd_launch_dp<16, true>(a, num_levels, rbf, difference != 0, s); break;
    default: return GPSIG_EUNSUPPORTED;
  }
  if (rc) return rc;
  const long long tot = (long long)n * l * d;
  hipLaunchKernelGGL(tvs_gx_add_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, gXt, n, l, d, gX);
  return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
}
