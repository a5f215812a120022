// gpsig_amd -- C ABI of the Goursat-PDE gradient (kernels in pde_bwd.h, one instantiation unit per
// channel count: pde_bwd_inst.hip).
#include "pde_bwd.h"
#include "gemm.h"

namespace gpsig {
#define DECL(v) extern template int pde_bwd_launch_dp<v>(const PdeBwdArgs &, long long, int, hipStream_t);
DECL(0) DECL(1) DECL(2) DECL(3) DECL(4) DECL(5) DECL(6) DECL(7) DECL(8) DECL(16)
#undef DECL
int increments_launch(const float *X, int n, int l, int d, float *dX, hipStream_t s);

// The adjoint on increment tiles: channel counts past the instantiations, dyadic orders past 3
bool pde_bwd_tiled(int d, int dyadic) { return d > 16 || dyadic > 3; }

static size_t al256b(size_t b) { return (b + 255) & ~(size_t)255; }
constexpr size_t PDE_BWD_TILE_BYTES = (size_t)1 << 30;  // increment tile (and as much adjoint tile) of a chunk

struct PdeBwdPlan {
  int rows;
  long long cols;
  size_t dx, dy, gdx, gdy, inc, gt, part;
};
static PdeBwdPlan pde_bwd_plan(int n1, int l1, int n2, int l2, int d, int pair_mode) {
  PdeBwdPlan p{};
  const int IC = l1 - 1, JC = l2 - 1;
  p.cols = pair_mode == GPSIG_PAIRS_DIAG ? (long long)IC : (long long)n2 * JC;
  long long r = (long long)(PDE_BWD_TILE_BYTES / ((size_t)IC * p.cols * sizeof(float)));
  r = r < 4 ? 4 : (r / 4) * 4;
  if (r > ((n1 + 3) / 4) * 4) r = ((n1 + 3) / 4) * 4;
  p.rows = (int)r;
  const bool rect = pair_mode == GPSIG_PAIRS_RECT;
  p.dx = al256b((size_t)n1 * IC * d * sizeof(float));
  p.dy = rect ? al256b((size_t)n2 * JC * d * sizeof(float)) : 0;
  p.gdx = p.dx;
  p.gdy = p.dy;
  p.inc = al256b((size_t)r * IC * p.cols * sizeof(float));
  p.gt = p.inc;
  // split-K partials of the two adjoint contractions of a full chunk (gdX: R x d, K = cols; gdY: cols x d,
  // K = R); gemm_f32 clamps any split to this capacity
  if (rect) {
    const size_t pr = gemm_splitk_bytes((int)(r * IC), d, (int)p.cols);
    const size_t pc = gemm_splitk_bytes((int)p.cols, d, (int)(r * IC));
    p.part = al256b(pr > pc ? pr : pc);
  }
  return p;
}
static size_t pde_bwd_plan_bytes(const PdeBwdPlan &p) { return p.dx + p.dy + p.gdx + p.gdy + p.inc + p.gt + p.part; }

// g[a][i][k] += G[a][i-1][k] - G[a][i][k] (increment gradients -> point gradients)
__global__ __launch_bounds__(256) void incr_to_points_kernel(const float *__restrict__ G, int n, int l, int d,
                                                             float *__restrict__ g) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long long)n * l * d) return;
  const int k = (int)(idx % d);
  const long long r = idx / d;
  const int i = (int)(r % l);
  const long long a = r / l;
  const float *Ga = G + a * (l - 1) * d;
  const float gp = i > 0 ? Ga[(long long)(i - 1) * d + k] : 0.0f;
  const float gc = i < l - 1 ? Ga[(long long)i * d + k] : 0.0f;
  g[idx] += gp - gc;
}
}  // namespace gpsig

using namespace gpsig;

extern "C" size_t gpsig_pde_vjp_scratch_bytes(int n1, int l1, int n2, int l2, int d, int dyadic, int pair_mode) {
  if (n1 <= 0 || n2 <= 0 || l1 < 2 || l2 < 2 || d <= 0 || !pde_bwd_tiled(d, dyadic)) return 0;
  return pde_bwd_plan_bytes(pde_bwd_plan(n1, l1, n2, l2, d, pair_mode));
}

extern "C" size_t gpsig_pde_vjp_workspace_bytes(int npairs, int l1, int l2, int dyadic) {
  if (npairs <= 0 || l1 < 2 || l2 < 2 || dyadic < 0 || dyadic > 8) return 0;
  return (size_t)npairs * (size_t)pde_front_floats(l1, l2, dyadic) * sizeof(float);
}

// The tiled adjoint: per chunk of x-rows the increment tile (GEMM), the kernel (fronts / adjoint sums into
// the adjoint tile), and the contractions dLoss/d dx = G dY, dLoss/d dy = G^T dX (GEMMs); point gradients at
// the end.  a: filled by pde_adj_impl (mode fields, rows, fronts of the whole call).
static int pde_adj_tiled(PdeBwdArgs a, int mode, void *scratch, size_t scratch_bytes, hipStream_t s) {
  const int n1 = a.n1, l1 = a.l1, n2 = a.n2, l2 = a.l2, d = a.d, pm = a.pair_mode;
  const int IC = l1 - 1;
  const PdeBwdPlan pl = pde_bwd_plan(n1, l1, n2, l2, d, pm);
  if (!scratch || scratch_bytes < pde_bwd_plan_bytes(pl)) return GPSIG_EWORKSPACE;
  char *w = static_cast<char *>(scratch);
  float *dX = reinterpret_cast<float *>(w); w += pl.dx;
  float *dY = pl.dy ? reinterpret_cast<float *>(w) : dX; w += pl.dy;
  float *gdX = reinterpret_cast<float *>(w); w += pl.gdx;
  float *gdY = pl.gdy ? reinterpret_cast<float *>(w) : nullptr; w += pl.gdy;
  float *Tin = reinterpret_cast<float *>(w); w += pl.inc;
  float *Tg = reinterpret_cast<float *>(w); w += pl.gt;
  float *part = pl.part ? reinterpret_cast<float *>(w) : nullptr;
  int rc = increments_launch(a.X, n1, l1, d, dX, s);
  if (rc) return rc;
  if (pm == GPSIG_PAIRS_RECT && (rc = increments_launch(a.Y, n2, l2, d, dY, s))) return rc;
  const bool adj = mode != 1;
  if (adj && hipMemsetAsync(gdX, 0, pl.gdx, s) != hipSuccess) return GPSIG_ELAUNCH;
  if (adj && gdY && hipMemsetAsync(gdY, 0, pl.gdy, s) != hipSuccess) return GPSIG_ELAUNCH;
  a.sub = pde_bwd_sub(a.dyadic);
  a.inc = Tin;
  a.gt = Tg;
  a.wpb = 4;  // no per-wave LDS on tiles
  const long long pf = pde_front_floats(l1, l2, a.dyadic);
  const int rb0 = a.row_begin, rb1 = a.row_end;
  for (int r0 = (rb0 / 4) * 4; r0 < rb1; r0 += pl.rows) {
    const int r1 = r0 + pl.rows < rb1 ? r0 + pl.rows : rb1;
    const int c0 = r0 > rb0 ? r0 : rb0;
    PdeBwdArgs c = a;
    c.row_begin = c0;
    c.row_end = r1;
    const long long poff = (long long)(c0 - rb0) * (pm == GPSIG_PAIRS_DIAG ? 1 : n2);  // pairs before the chunk
    c.fronts = a.fronts + poff * pf;
    if (a.out) c.out = a.out + poff;
    long long nblocks;
    if (pm == GPSIG_PAIRS_DIAG) {
      c.inc_a0 = c0;
      c.inc_b0 = 0;
      c.inc_as = (long long)IC * IC;
      c.inc_ld = IC;
      nblocks = (r1 - c0 + 3) / 4;
      rc = gemm_f32(s, false, true, IC, IC, d, 1.0f, dX + (long long)c0 * IC * d, d, (long long)IC * d,
                    dX + (long long)c0 * IC * d, d, (long long)IC * d, 0.0f, Tin, IC, (long long)IC * IC, r1 - c0, 0, 0,
                    nullptr, 0);
    } else {
      c.inc_a0 = r0;
      c.inc_b0 = 0;
      c.inc_as = (long long)IC * pl.cols;
      c.inc_ld = pl.cols;
      c.ntb = n2;
      c.tiles_a0 = r0 / 4;
      nblocks = (long long)((r1 + 3) / 4 - r0 / 4) * n2;
      rc = gemm_f32(s, false, true, (r1 - r0) * IC, (int)pl.cols, d, 1.0f, dX + (long long)r0 * IC * d, d, 0, dY, d, 0,
                    0.0f, Tin, pl.cols, 0, 1, 0, 0, nullptr, 0);
    }
    if (rc) return rc;
    if (nblocks > 0x7fffffffLL) return GPSIG_EUNSUPPORTED;
    const size_t tbytes = (size_t)(r1 - (pm == GPSIG_PAIRS_DIAG ? c0 : r0)) * IC * pl.cols * sizeof(float);
    if (adj && hipMemsetAsync(Tg, 0, tbytes, s) != hipSuccess) return GPSIG_ELAUNCH;
    if ((rc = pde_bwd_launch_dp<0>(c, nblocks, mode, s))) return rc;
    if (!adj) continue;
    if (pm == GPSIG_PAIRS_DIAG) {
      rc = gemm_f32(s, false, false, IC, d, IC, 1.0f, Tg, IC, (long long)IC * IC, dX + (long long)c0 * IC * d, d,
                    (long long)IC * d, 0.0f, gdX + (long long)c0 * IC * d, d, (long long)IC * d, r1 - c0, 0, 0, nullptr, 0);
    } else {
      const int R = (r1 - r0) * IC;
      rc = gemm_f32(s, false, false, R, d, (int)pl.cols, 1.0f, Tg, pl.cols, 0, dY, d, 0, 1.0f,
                    gdX + (long long)r0 * IC * d, d, 0, 1, 0, 0, part, pl.part);
      if (!rc)
        rc = gemm_f32(s, true, false, (int)pl.cols, d, R, 1.0f, Tg, pl.cols, 0, dX + (long long)r0 * IC * d, d, 0, 1.0f,
                      gdY, d, 0, 1, 0, 0, part, pl.part);
    }
    if (rc) return rc;
  }
  if (adj) {
    const long long tx = (long long)(rb1 - rb0) * l1 * d;
    hipLaunchKernelGGL(incr_to_points_kernel, dim3((unsigned)((tx + 255) / 256)), dim3(256), 0, s,
                       gdX + (long long)rb0 * IC * d, rb1 - rb0, l1, d, a.gX + (long long)rb0 * l1 * d);
    if (pm == GPSIG_PAIRS_RECT) {
      const long long ty = (long long)n2 * l2 * d;
      hipLaunchKernelGGL(incr_to_points_kernel, dim3((unsigned)((ty + 255) / 256)), dim3(256), 0, s, gdY, n2, l2, d,
                         a.gY);
    }
  }
  return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
}

// mode 0: gpsig_pde_vjp, 1: gpsig_pde_fronts, 2: gpsig_pde_vjp_fronts (pde_adj_kernel's MODE)
static int pde_adj_impl(int mode, const float *X, int n1, int l1, const float *Y, int n2, int l2, int d, int dyadic,
                        int solver, int pair_mode, int row_begin, int row_end, const float *gout, float *gX, float *gY,
                        float *out, void *workspace, size_t workspace_bytes, hipStream_t s, void *scratch = nullptr,
                        size_t scratch_bytes = 0) {
  if (!X || !Y || n1 <= 0 || n2 <= 0 || d <= 0 || l1 < 2 || l2 < 2) return GPSIG_EINVAL;
  if (mode == 1 ? !out : (!gout || !gX)) return GPSIG_EINVAL;
  if (dyadic < 0 || dyadic > 8 || (solver != 0 && solver != 1)) return GPSIG_EINVAL;
  if (pair_mode != GPSIG_PAIRS_RECT && pair_mode != GPSIG_PAIRS_DIAG) return GPSIG_EINVAL;
  if (row_begin < 0 || row_end > n1 || row_begin > row_end) return GPSIG_EINVAL;
  if (pair_mode == GPSIG_PAIRS_DIAG && (n1 != n2 || l1 != l2 || X != Y)) return GPSIG_EINVAL;
  if (mode != 1 && pair_mode == GPSIG_PAIRS_RECT && !gY) return GPSIG_EINVAL;
  if (row_end == row_begin) return GPSIG_OK;
  const int rows = row_end - row_begin;
  const int npairs = pair_mode == GPSIG_PAIRS_DIAG ? rows : rows * n2;
  if (pde_front_floats(l1, l2, dyadic) == 0) return GPSIG_EUNSUPPORTED;
  if (!workspace || workspace_bytes < gpsig_pde_vjp_workspace_bytes(npairs, l1, l2, dyadic)) return GPSIG_EWORKSPACE;
  PdeBwdArgs a{};
  a.X = X; a.Y = Y;
  a.n1 = n1; a.l1 = l1; a.n2 = n2; a.l2 = l2; a.d = d;
  a.dyadic = dyadic; a.solver = solver;
  a.pair_mode = pair_mode; a.row_begin = row_begin; a.row_end = row_end;
  a.gout = gout; a.gX = gX; a.gY = gY;
  a.fronts = static_cast<float *>(workspace);
  a.out = out;
  if (pde_bwd_tiled(d, dyadic)) return pde_adj_tiled(a, mode, scratch, scratch_bytes, s);
  // pairs per workgroup: 4 unless the per-wave LDS (row accumulators and dx of x) of long x needs fewer
  const int dp = d <= 8 ? d : (d <= 16 ? 16 : 0);
  int wpb = 4;
  // cross pairs also keep their lanes' column sums in LDS (W / REP coarse columns per lane)
  const int wc = pair_mode == GPSIG_PAIRS_RECT && mode != 1 ? pde_layout(l1, l2, dyadic).W >> dyadic : 0;
  while (wpb > 1 && (size_t)wpb * pde_lds_wave_doubles(l1 - 1, dp, wc) * sizeof(double) > 160 * 1024) wpb /= 2;
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

extern "C" int gpsig_pde_vjp_ex(const float *X, int n1, int l1, const float *Y, int n2, int l2, int d, int dyadic,
                                int solver, int pair_mode, int row_begin, int row_end, const float *gout, float *gX,
                                float *gY, void *workspace, size_t workspace_bytes, void *scratch, size_t scratch_bytes,
                                gpsig_stream_t stream) {
  return pde_adj_impl(0, X, n1, l1, Y, n2, l2, d, dyadic, solver, pair_mode, row_begin, row_end, gout, gX, gY,
                      nullptr, workspace, workspace_bytes, reinterpret_cast<hipStream_t>(stream), scratch, scratch_bytes);
}

extern "C" int gpsig_pde_fronts_ex(const float *X, int n1, int l1, const float *Y, int n2, int l2, int d, int dyadic,
                                   int solver, int pair_mode, int row_begin, int row_end, float *out, void *fronts,
                                   size_t fronts_bytes, void *scratch, size_t scratch_bytes, gpsig_stream_t stream) {
  return pde_adj_impl(1, X, n1, l1, Y, n2, l2, d, dyadic, solver, pair_mode, row_begin, row_end, nullptr, nullptr,
                      nullptr, out, fronts, fronts_bytes, reinterpret_cast<hipStream_t>(stream), scratch, scratch_bytes);
}

extern "C" int gpsig_pde_vjp_fronts_ex(const float *X, int n1, int l1, const float *Y, int n2, int l2, int d,
                                       int dyadic, int solver, int pair_mode, int row_begin, int row_end,
                                       const float *gout, float *gX, float *gY, const void *fronts,
                                       size_t fronts_bytes, void *scratch, size_t scratch_bytes,
                                       gpsig_stream_t stream) {
  return pde_adj_impl(2, X, n1, l1, Y, n2, l2, d, dyadic, solver, pair_mode, row_begin, row_end, gout, gX, gY,
                      nullptr, const_cast<void *>(fronts), fronts_bytes, reinterpret_cast<hipStream_t>(stream), scratch,
                      scratch_bytes);
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
