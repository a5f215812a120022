// gpsig_amd -- extern "C" entry of the first-order Gram VJP (include/gpsig_amd.h, gpsig_sig_gram_vjp):
// argument checks, feature records, tile counts, dispatch to the per-(DP, M) instantiations of
// sig_bwd_kernel (sig_bwd.h, sig_bwd_inst.hip).
#include "sig_bwd_pk.h"

namespace gpsig {
int features(const float *X, int n, int l, int d, int DP, float *F, hipStream_t s);
size_t sig_bwd_wide_workspace(int n1, int l1, int n2, int l2, int d);
int sig_bwd_wide(BwdArgs a, const float *X, const float *Y, int seed, void *workspace, size_t workspace_bytes,
                 hipStream_t s, int order = 1);
bool ho_bwd_supported(int l2, int order, int M, int seed);
size_t ho_bwd_slab_bytes(int l2, int order, int M);
// channel counts past the VJP's instantiations: the wide-channel VJP (point-weight tiles + GEMMs; slower
// than the register form at few channels: d = 5 69.7 vs 31.8 ms fwd+bwd at N = 1024, L = 100).
// GPSIG_VJP_FIXED_MAX lowers the crossover for A/B runs.
static int vjp_fixed_max() {
  static const int v = [] {
    const char *e = getenv("GPSIG_VJP_FIXED_MAX");
    const int x = e ? atoi(e) : 16;
    return x < 16 ? (x < 0 ? 0 : x) : 16;
  }();
  return v;
}
static bool bwd_wide(int d) { return d > vjp_fixed_max(); }
template <int DP, int M>
int sig_bwd_launch_dpm(const BwdArgs &a, int seed, long long nblocks, hipStream_t s);
template <int DP, int M>
int sig_bwd_pk_launch_dpm(const BwdArgs &a, int seed, BwdGeo geo, long long nblocks, hipStream_t s);

// The packed column-pair VJP (sig_bwd_pk.h) for the difference seeds in one column block; GPSIG_BWD_PK=0
// keeps sig_bwd_kernel everywhere (A/B runs)
static bool bwd_pk_enabled() {
  static const bool v = [] {
    const char *e = getenv("GPSIG_BWD_PK");
    return !(e && atoi(e) == 0);
  }();
  return v;
}
// Measured (tools/kbench_vjp.hip, N = 1024, D = 5, M = 5, saved state; profiles/r6_vjp_ab.txt): at the same
// geometry the packed kernel is 1-4 % faster (L = 64: 11.12 -> 10.99 ms, L = 128: 27.28 -> 26.13 ms), but at
// 65-100 points sig_bwd_kernel's 20-lane groups (3 pairs per wave, W = 5) beat its 32-lane W = 4 (2 pairs):
// C2 21.79 vs 24.15 ms.  So the packed kernel takes every one-block shape except that segmented geometry.
static BwdGeo bwd_pk_geo(int l2, int DP, int M, int seed) {
  if (!bwd_pk_enabled() || (seed != SEED_RBF_DIFF && seed != SEED_LIN_DIFF)) return {0, 0};
  const BwdGeo old = bwd_geometry(l2, DP, M);
  if (old.LP == 20) return {0, 0};
  return bwd_pk_geometry(l2, DP, M, seed == SEED_RBF_DIFF);
}
template <int DP>
static int bwd_pk_dp(const BwdArgs &a, int seed, BwdGeo geo, long long nblocks, hipStream_t s) {
  switch (a.M) {
    case 1: return sig_bwd_pk_launch_dpm<DP, 1>(a, seed, geo, nblocks, s);
    case 2: return sig_bwd_pk_launch_dpm<DP, 2>(a, seed, geo, nblocks, s);
    case 3: return sig_bwd_pk_launch_dpm<DP, 3>(a, seed, geo, nblocks, s);
    case 4: return sig_bwd_pk_launch_dpm<DP, 4>(a, seed, geo, nblocks, s);
    case 5: return sig_bwd_pk_launch_dpm<DP, 5>(a, seed, geo, nblocks, s);
    case 6: return sig_bwd_pk_launch_dpm<DP, 6>(a, seed, geo, nblocks, s);
    case 7: return sig_bwd_pk_launch_dpm<DP, 7>(a, seed, geo, nblocks, s);
    case 8: return sig_bwd_pk_launch_dpm<DP, 8>(a, seed, geo, nblocks, s);
    default: return GPSIG_EUNSUPPORTED;
  }
}

template <int DP>
static int bwd_dp(const BwdArgs &a, int seed, long long nblocks, hipStream_t s) {
  switch (a.M) {
    case 1: return sig_bwd_launch_dpm<DP, 1>(a, seed, nblocks, s);
    case 2: return sig_bwd_launch_dpm<DP, 2>(a, seed, nblocks, s);
    case 3: return sig_bwd_launch_dpm<DP, 3>(a, seed, nblocks, s);
    case 4: return sig_bwd_launch_dpm<DP, 4>(a, seed, nblocks, s);
    case 5: return sig_bwd_launch_dpm<DP, 5>(a, seed, nblocks, s);
    case 6: return sig_bwd_launch_dpm<DP, 6>(a, seed, nblocks, s);
    case 7: return sig_bwd_launch_dpm<DP, 7>(a, seed, nblocks, s);
    case 8: return sig_bwd_launch_dpm<DP, 8>(a, seed, nblocks, s);
    default: return GPSIG_EUNSUPPORTED;
  }
}

// channel padding of the VJP instantiations (never wider than the forward's workspace padding)
static int bwd_pad(int d) {
  if (d <= 6) return d;
  if (d <= 8) return 8;
  if (d <= 16) return 16;
  return 0;
}

static size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }
static constexpr size_t GSC_BYTES = GSCALE_SLOTS * 9 * sizeof(float);  // dscale partials (M <= 8)

// gscale[m] += sum of the GSCALE_SLOTS partial sums of level m
__global__ void gscale_reduce_kernel(const float *__restrict__ slots, int levels, float *__restrict__ gscale) {
  const int m = threadIdx.x;
  if (m >= levels) return;
  float s = 0.0f;
  for (int k = 0; k < GSCALE_SLOTS; ++k) s += slots[k * levels + m];
  gscale[m] += s;
}

// The VJPs with point-weight tiles and emission GEMMs (sig_bwd_wide.hip): order 1 at wide channel counts,
// and every order > 1
static int tile_vjp(const float *X, int n1, int l1, const float *Y, int n2, int l2, int d, int num_levels, int order,
                    int seed, int pair_mode, int row_begin, int row_end, const float *gout, int gout_levels,
                    const float *rs1, const float *rs2, const float *scale, float jitter, float *gX, float *gY,
                    float *grs1, float *grs2, float *gscale, const float *state, void *workspace,
                    size_t workspace_bytes, hipStream_t s) {
  if (row_end == row_begin) return GPSIG_OK;
  if (!workspace || workspace_bytes < GSC_BYTES + sig_bwd_wide_workspace(n1, l1, n2, l2, d)) return GPSIG_EWORKSPACE;
  float *gsc_slots = static_cast<float *>(workspace);
  BwdArgs a{};
  a.n1 = n1; a.l1 = l1; a.n2 = n2; a.l2 = l2; a.d = d;
  a.M = num_levels;
  a.pair_mode = pair_mode;
  a.row_begin = row_begin;
  a.row_end = row_end;
  a.gout = gout;
  a.gout_levels = gout_levels ? 1 : 0;
  a.g_ld = n2;
  a.g_lvl = pair_mode == GPSIG_PAIRS_DIAG ? (long long)n1 : (long long)n1 * n2;
  a.rs1 = rs1; a.rs2 = rs2; a.scale = scale;
  a.jitter = jitter;
  a.gX = gX;
  a.gY = pair_mode == GPSIG_PAIRS_RECT ? gY : gX;
  a.grs1 = grs1;
  a.grs2 = pair_mode == GPSIG_PAIRS_RECT ? grs2 : grs1;
  a.gscale = nullptr;
  if (gscale && pair_mode != GPSIG_PAIRS_DIAG) {
    if (hipMemsetAsync(gsc_slots, 0, GSC_BYTES, s) != hipSuccess) return GPSIG_ELAUNCH;
    a.gscale = gsc_slots;
  }
  a.state = state;
  // the 8-wave higher-order VJP's global slabs (past 509 points) after the wide workspace
  const size_t wide_b = sig_bwd_wide_workspace(n1, l1, n2, l2, d);
  const size_t slab_b = order > 1 ? ho_bwd_slab_bytes(l2, order, num_levels) : 0;
  if (workspace_bytes < GSC_BYTES + wide_b + slab_b) return GPSIG_EWORKSPACE;
  a.scratch = slab_b ? reinterpret_cast<float *>(static_cast<char *>(workspace) + GSC_BYTES + wide_b) : nullptr;
  const int rc = sig_bwd_wide(a, X, pair_mode == GPSIG_PAIRS_RECT ? Y : X, seed, static_cast<char *>(workspace) + GSC_BYTES,
                              wide_b, s, order);
  if (rc) return rc;
  if (a.gscale) {
    hipLaunchKernelGGL(gscale_reduce_kernel, dim3(1), dim3(64), 0, s, gsc_slots, num_levels + 1, gscale);
    if (hipGetLastError() != hipSuccess) return GPSIG_ELAUNCH;
  }
  return GPSIG_OK;
}

}  // namespace gpsig

using namespace gpsig;

extern "C" int gpsig_sig_gram_vjp(const float *X, int n1, int l1, const float *Y, int n2, int l2, int d,
                                  int num_levels, int base_kind, int difference, int pair_mode, int row_begin, int row_end,
                                  const float *gout, int gout_levels, const float *rs1, const float *rs2,
                                  const float *scale, float jitter, float *gX, float *gY, float *grs1, float *grs2,
                                  float *gscale, const float *state, void *workspace, size_t workspace_bytes,
                                  gpsig_stream_t stream) {
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (!X || !Y || !gout || !gX || n1 <= 0 || n2 <= 0 || d <= 0 || num_levels < 1) return GPSIG_EINVAL;
  if (l1 < 1 || l2 < 1 || (difference && (l1 < 2 || l2 < 2))) return GPSIG_EINVAL;
  if (pair_mode < GPSIG_PAIRS_RECT || pair_mode > GPSIG_PAIRS_DIAG) return GPSIG_EINVAL;
  if (row_begin < 0 || row_end > n1 || row_begin > row_end) return GPSIG_EINVAL;
  if (pair_mode != GPSIG_PAIRS_RECT && (n1 != n2 || l1 != l2 || X != Y)) return GPSIG_EINVAL;
  if (pair_mode == GPSIG_PAIRS_RECT && !gY) return GPSIG_EINVAL;
  if (pair_mode == GPSIG_PAIRS_DIAG && !gout_levels) return GPSIG_EINVAL;
  if ((rs1 == nullptr) != (rs2 == nullptr)) return GPSIG_EINVAL;
  if (state && (pair_mode == GPSIG_PAIRS_DIAG || !difference)) return GPSIG_EINVAL;
  const int seed = base_kind == GPSIG_BASE_RBF ? (difference ? SEED_RBF_DIFF : SEED_RBF_POINT)
                   : base_kind == GPSIG_BASE_LINEAR ? (difference ? SEED_LIN_DIFF : SEED_LIN_POINT) : -1;
  const bool wide = bwd_wide(d);
  const int DP = wide ? 0 : bwd_pad(d);
  if (seed < 0 || (DP == 0 && !wide) || num_levels > 8) return GPSIG_EUNSUPPORTED;
  if (wide)
    return tile_vjp(X, n1, l1, Y, n2, l2, d, num_levels, 1, seed, pair_mode, row_begin, row_end, gout, gout_levels,
                    rs1, rs2, scale, jitter, gX, gY, grs1, grs2, gscale, state, workspace, workspace_bytes, s);
  const BwdGeo pkgeo = bwd_pk_geo(l2, DP, num_levels, seed);
  const bool pk = pkgeo.W != 0;
  const BwdGeo geo = pk ? pkgeo : bwd_geometry(l2, DP, num_levels);
  if (geo.W == 0) return GPSIG_EUNSUPPORTED;
  if (row_end == row_begin) return GPSIG_OK;
  const int nblk = pk ? 1 : bwd_blocks(l2, difference != 0, geo);
  const long long scr_stride = bwd_scratch_floats(difference ? l1 - 1 : l1, num_levels, geo.W, nblk);

  const bool same = (X == Y && n1 == n2 && l1 == l2);
  const size_t fx_b = align256((size_t)n1 * l1 * feat_stride(DP) * sizeof(float));
  const size_t fy_b = same ? 0 : align256((size_t)n2 * l2 * feat_stride(DP) * sizeof(float));
  const size_t scr_b = (size_t)scr_stride * 4 * BWD_CHUNK_BLOCKS * sizeof(float);
  if (!workspace || workspace_bytes < fx_b + fy_b + scr_b + GSC_BYTES) return GPSIG_EWORKSPACE;
  float *gsc_slots = reinterpret_cast<float *>(static_cast<char *>(workspace) + fx_b + fy_b + scr_b);
  float *FX = static_cast<float *>(workspace);
  float *FY = same ? FX : reinterpret_cast<float *>(static_cast<char *>(workspace) + fx_b);
  int rc = features(X, n1, l1, d, DP, FX, s);
  if (rc) return rc;
  if (!same && (rc = features(Y, n2, l2, d, DP, FY, s))) return rc;

  BwdArgs a{};
  a.FX = FX;
  a.FY = FY;
  a.n1 = n1; a.l1 = l1; a.n2 = n2; a.l2 = l2; a.d = d;
  a.M = num_levels;
  a.pair_mode = pair_mode;
  a.row_begin = row_begin;
  a.row_end = row_end;
  a.gout = gout;
  a.gout_levels = gout_levels ? 1 : 0;
  a.g_ld = n2;
  a.g_lvl = pair_mode == GPSIG_PAIRS_DIAG ? (long long)n1 : (long long)n1 * n2;
  a.rs1 = rs1; a.rs2 = rs2; a.scale = scale;
  a.jitter = jitter;
  a.gX = gX;
  a.gY = pair_mode == GPSIG_PAIRS_RECT ? gY : gX;
  a.grs1 = grs1;
  a.grs2 = pair_mode == GPSIG_PAIRS_RECT ? grs2 : grs1;
  a.gscale = nullptr;
  if (gscale && pair_mode != GPSIG_PAIRS_DIAG) {
    if (hipMemsetAsync(gsc_slots, 0, GSC_BYTES, s) != hipSuccess) return GPSIG_ELAUNCH;
    a.gscale = gsc_slots;
  }
  a.state = state;
  a.nblk = nblk;
  a.scratch = scr_stride ? reinterpret_cast<float *>(static_cast<char *>(workspace) + fx_b + fy_b) : nullptr;
  a.scr_stride = scr_stride;

  const int G = 64 / geo.LP;
  long long nblocks;
  if (pair_mode == GPSIG_PAIRS_DIAG) {
    nblocks = (row_end - row_begin + 3) / 4;
  } else {
    const int ta0 = row_begin / 4, ta1 = (row_end + 3) / 4;
    const int ntb = (n2 + G - 1) / G;
    a.tiles_a0 = ta0;
    a.ntb = ntb;
    if (pair_mode == GPSIG_PAIRS_RECT) {
      nblocks = (long long)(ta1 - ta0) * ntb;
    } else {
      a.tile_base = upper_prefix_g(ta0, ntb, G);
      nblocks = upper_prefix_g(ta1, ntb, G) - a.tile_base;
    }
  }
  if (nblocks > 0x7fffffffLL) return GPSIG_EUNSUPPORTED;
  if (nblocks <= 0) return GPSIG_OK;
  // column-block launches go in chunks of BWD_CHUNK_BLOCKS workgroups (the scratch holds one chunk)
  const long long chunk = scr_stride ? BWD_CHUNK_BLOCKS : nblocks;
  for (long long c = 0; c < nblocks; c += chunk) {
    a.blk0 = c;
    const long long nb = nblocks - c < chunk ? nblocks - c : chunk;
    switch (DP) {
#define CASE(v) \
  case v: rc = pk ? bwd_pk_dp<v>(a, seed, geo, nb, s) : bwd_dp<v>(a, seed, nb, s); break;
      CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(8) CASE(16)
#undef CASE
      default: return GPSIG_EUNSUPPORTED;
    }
    if (rc) return rc;
  }
  if (a.gscale) {
    hipLaunchKernelGGL(gscale_reduce_kernel, dim3(1), dim3(64), 0, s, gsc_slots, num_levels + 1, gscale);
    if (hipGetLastError() != hipSuccess) return GPSIG_ELAUNCH;
  }
  return GPSIG_OK;
}

extern "C" size_t gpsig_sig_vjp_workspace_bytes(int n1, int l1, int n2, int l2, int d, int num_levels, int difference) {
  if (n1 <= 0 || n2 <= 0 || l1 < 1 || l2 < 1 || d <= 0) return 0;
  if (bwd_wide(d)) return GSC_BYTES + sig_bwd_wide_workspace(n1, l1, n2, l2, d);
  const int DP = bwd_pad(d);
  if (DP == 0 || n1 <= 0 || n2 <= 0 || l1 < 1 || l2 < 1) return 0;
  const BwdGeo geo = bwd_geometry(l2, DP);
  const int nblk = bwd_blocks(l2, difference != 0, geo);
  const long long scr = bwd_scratch_floats(difference ? l1 - 1 : l1, num_levels, geo.W, nblk);
  return align256((size_t)n1 * l1 * feat_stride(DP) * sizeof(float)) +
         align256((size_t)n2 * l2 * feat_stride(DP) * sizeof(float)) + (size_t)scr * 4 * BWD_CHUNK_BLOCKS * sizeof(float) +
         GSC_BYTES;
}

extern "C" int gpsig_sig_gram_vjp_ho(const float *X, int n1, int l1, const float *Y, int n2, int l2, int d,
                                     int num_levels, int order, int base_kind, int pair_mode, int row_begin,
                                     int row_end, const float *gout, int gout_levels, const float *rs1,
                                     const float *rs2, const float *scale, float jitter, float *gX, float *gY,
                                     float *grs1, float *grs2, float *gscale, void *workspace,
                                     size_t workspace_bytes, gpsig_stream_t stream) {
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (!X || !Y || !gout || !gX || n1 <= 0 || n2 <= 0 || d <= 0 || num_levels < 1 || order < 1) return GPSIG_EINVAL;
  if (l1 < 2 || l2 < 2) return GPSIG_EINVAL;
  if (pair_mode < GPSIG_PAIRS_RECT || pair_mode > GPSIG_PAIRS_DIAG) return GPSIG_EINVAL;
  if (row_begin < 0 || row_end > n1 || row_begin > row_end) return GPSIG_EINVAL;
  if (pair_mode != GPSIG_PAIRS_RECT && (n1 != n2 || l1 != l2 || X != Y)) return GPSIG_EINVAL;
  if (pair_mode == GPSIG_PAIRS_RECT && !gY) return GPSIG_EINVAL;
  if (pair_mode == GPSIG_PAIRS_DIAG && !gout_levels) return GPSIG_EINVAL;
  if ((rs1 == nullptr) != (rs2 == nullptr)) return GPSIG_EINVAL;
  if (order == 1 || num_levels == 1)  // the first-order recursion
    return gpsig_sig_gram_vjp(X, n1, l1, Y, n2, l2, d, num_levels, base_kind, 1, pair_mode, row_begin, row_end, gout,
                              gout_levels, rs1, rs2, scale, jitter, gX, gY, grs1, grs2, gscale, nullptr, workspace,
                              workspace_bytes, stream);
  const int seed = base_kind == GPSIG_BASE_RBF ? SEED_RBF_DIFF : base_kind == GPSIG_BASE_LINEAR ? SEED_LIN_DIFF : -1;
  if (seed < 0 || !ho_bwd_supported(l2, order, num_levels, seed)) return GPSIG_EUNSUPPORTED;
  return tile_vjp(X, n1, l1, Y, n2, l2, d, num_levels, order, seed, pair_mode, row_begin, row_end, gout, gout_levels,
                  rs1, rs2, scale, jitter, gX, gY, grs1, grs2, gscale, nullptr, workspace, workspace_bytes, s);
}

extern "C" size_t gpsig_sig_vjp_ho_workspace_bytes(int n1, int l1, int n2, int l2, int d, int num_levels, int order,
                                                   int base_kind) {
  if (n1 <= 0 || n2 <= 0 || l1 < 2 || l2 < 2 || d <= 0 || order < 1) return 0;
  if (order == 1 || num_levels == 1) return gpsig_sig_vjp_workspace_bytes(n1, l1, n2, l2, d, num_levels, 1);
  const int seed = base_kind == GPSIG_BASE_RBF ? SEED_RBF_DIFF : base_kind == GPSIG_BASE_LINEAR ? SEED_LIN_DIFF : -1;
  if (seed < 0 || !ho_bwd_supported(l2, order, num_levels, seed)) return 0;
  return GSC_BYTES + sig_bwd_wide_workspace(n1, l1, n2, l2, d) + ho_bwd_slab_bytes(l2, order, num_levels);
}
