// gpsig_amd -- C ABI of the Goursat-PDE gradient (kernels in pde_bwd.h, one instantiation unit per
// channel count: pde_bwd_inst.hip).
#include "pde_bwd.h"

namespace gpsig {
#define DECL(v) extern template int pde_bwd_launch_dp<v>(const PdeBwdArgs &, long long, int, hipStream_t);
DECL(1) DECL(2) DECL(3) DECL(4) DECL(5) DECL(6) DECL(7) DECL(8) DECL(16)
#undef DECL
}  // namespace gpsig

using namespace gpsig;

extern "C" size_t gpsig_pde_vjp_workspace_bytes(int npairs, int l1, int l2, int dyadic) {
  if (npairs <= 0 || l1 < 2 || l2 < 2 || dyadic < 0 || dyadic > 6) return 0;
  return (size_t)npairs * (size_t)pde_front_floats(l1, l2, dyadic) * sizeof(float);
}

// mode 0: gpsig_pde_vjp, 1: gpsig_pde_fronts, 2: gpsig_pde_vjp_fronts (pde_adj_kernel's MODE)
static int pde_adj_impl(int mode, const float *X, int n1, int l1, const float *Y, int n2, int l2, int d, int dyadic,
                        int solver, int pair_mode, int row_begin, int row_end, const float *gout, float *gX, float *gY,
                        float *out, void *workspace, size_t workspace_bytes, hipStream_t s) {
  if (!X || !Y || n1 <= 0 || n2 <= 0 || d <= 0 || l1 < 2 || l2 < 2) return GPSIG_EINVAL;
  if (mode == 1 ? !out : (!gout || !gX)) return GPSIG_EINVAL;
  if (dyadic < 0 || dyadic > 6 || (solver != 0 && solver != 1)) return GPSIG_EINVAL;
  if (pair_mode != GPSIG_PAIRS_RECT && pair_mode != GPSIG_PAIRS_DIAG) return GPSIG_EINVAL;
  if (row_begin < 0 || row_end > n1 || row_begin > row_end) return GPSIG_EINVAL;
  if (pair_mode == GPSIG_PAIRS_DIAG && (n1 != n2 || l1 != l2 || X != Y)) return GPSIG_EINVAL;
  if (mode != 1 && pair_mode == GPSIG_PAIRS_RECT && !gY) return GPSIG_EINVAL;
  if (row_end == row_begin) return GPSIG_OK;
  const int rows = row_end - row_begin;
  const int npairs = pair_mode == GPSIG_PAIRS_DIAG ? rows : rows * n2;
  if (pde_front_floats(l1, l2, dyadic) == 0) return GPSIG_EUNSUPPORTED;  // dyadic > 3
  if (!workspace || workspace_bytes < gpsig_pde_vjp_workspace_bytes(npairs, l1, l2, dyadic)) return GPSIG_EWORKSPACE;
  PdeBwdArgs a{};
  a.X = X; a.Y = Y;
  a.n1 = n1; a.l1 = l1; a.n2 = n2; a.l2 = l2; a.d = d;
  a.dyadic = dyadic; a.solver = solver;
  a.pair_mode = pair_mode; a.row_begin = row_begin; a.row_end = row_end;
  a.gout = gout; a.gX = gX; a.gY = gY;
  a.fronts = static_cast<float *>(workspace);
  a.out = out;
  // pairs per workgroup: 4 unless the per-wave LDS (row accumulators and dx of x) of long x needs fewer
  const int dp = d <= 8 ? d : (d <= 16 ? 16 : 0);
  int wpb = 4;
  while (wpb > 1 && (size_t)wpb * pde_lds_wave_doubles(l1 - 1, dp) * sizeof(double) > 160 * 1024) wpb /= 2;
  a.wpb = wpb;
  long long nblocks;
  if (pair_mode == GPSIG_PAIRS_DIAG) {
    nblocks = (rows + wpb - 1) / wpb;
  } else {
    const int ta0 = row_begin / wpb, ta1 = (row_end + wpb - 1) / wpb;
    a.ntb = n2;
    a.tiles_a0 = ta0;
    nblocks = (long long)(ta1 - ta0) * n2;
  }
  if (nblocks > 0x7fffffffLL) return GPSIG_EUNSUPPORTED;
  switch (dp) {
#define CASE(v) \
  case v: return pde_bwd_launch_dp<v>(a, nblocks, mode, s);
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8) CASE(16)
#undef CASE
    default: return GPSIG_EUNSUPPORTED;
  }
}

extern "C" int gpsig_pde_vjp(const float *X, int n1, int l1, const float *Y, int n2, int l2, int d, int dyadic,
                             int solver, int pair_mode, int row_begin, int row_end, const float *gout, float *gX,
                             float *gY, void *workspace, size_t workspace_bytes, gpsig_stream_t stream) {
  return pde_adj_impl(0, X, n1, l1, Y, n2, l2, d, dyadic, solver, pair_mode, row_begin, row_end, gout, gX, gY,
                      nullptr, workspace, workspace_bytes, reinterpret_cast<hipStream_t>(stream));
}

extern "C" int gpsig_pde_fronts(const float *X, int n1, int l1, const float *Y, int n2, int l2, int d, int dyadic,
                                int solver, int pair_mode, int row_begin, int row_end, float *out, void *fronts,
                                size_t fronts_bytes, gpsig_stream_t stream) {
  return pde_adj_impl(1, X, n1, l1, Y, n2, l2, d, dyadic, solver, pair_mode, row_begin, row_end, nullptr, nullptr,
                      nullptr, out, fronts, fronts_bytes, reinterpret_cast<hipStream_t>(stream));
}

extern "C" int gpsig_pde_vjp_fronts(const float *X, int n1, int l1, const float *Y, int n2, int l2, int d, int dyadic,
                                    int solver, int pair_mode, int row_begin, int row_end, const float *gout,
                                    float *gX, float *gY, const void *fronts, size_t fronts_bytes,
                                    gpsig_stream_t stream) {
  return pde_adj_impl(2, X, n1, l1, Y, n2, l2, d, dyadic, solver, pair_mode, row_begin, row_end, gout, gX, gY,
                      nullptr, const_cast<void *>(fronts), fronts_bytes, reinterpret_cast<hipStream_t>(stream));
}
