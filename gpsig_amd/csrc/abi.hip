// gpsig_amd -- extern "C" entry points (include/gpsig_amd.h): argument checks, workspace carving,
// tile counts, and dispatch to the templated kernels.  No allocation, no synchronisation.
#include "sig_common.h"
#include "wide.h"

#include <stdlib.h>

namespace gpsig {
int features(const float *X, int n, int l, int d, int DP, float *F, hipStream_t s);
int sig_fo_launch(const SigArgs &a, int DP, int seed, long long nblocks, hipStream_t s);
int fo_lanes_per_pair(int l2, int DP, int M, bool mf, int seed, bool split);
void fo_wide_geo(int l2, int seed, int *W, int *LP);
size_t fo_split_bytes(int l1, int l2, int DP, int M);
int sig_ho_launch(const SigArgs &a, int DP, int seed, long long nblocks, hipStream_t s);
bool ho_tiled(int d, int order);
size_t ho_tile_bytes(int n1, int l1, int n2, int l2, int d, int pair_mode);
int sig_ho_tiled(SigArgs a, const float *X, const float *Y, int d, int seed, void *workspace, size_t workspace_bytes,
                 hipStream_t s);
int ho_lanes_per_pair(int l2, int order, int M);
int pde_launch(const float *X, int n1, int l1, const float *Y, int n2, int l2, int d, int dyadic, int solver,
               int pair_mode, int row_begin, int row_end, float *out, int out_row0, int out_rows,
               long long out_ld, hipStream_t s);
int sym_assemble_launch(const float *src, const long long *row_off, long long level_stride, int n, int levels,
                        float *dst, hipStream_t s);
bool pde_tiled(int d, int dyadic);
int mf_records(const float *X, int n, int l, int d, float *R, hipStream_t s);
size_t mf_records_bytes(int n, int l, int d);
bool mf_gram_applies(int d, int l2);
size_t mf_gram_scratch_bytes(int l1, int l2, int d);
int sig_fo_mf(const SigArgs &a, int d, int seed, float *scratch, hipStream_t s);
size_t pde_tile_scratch_bytes(int n1, int l1, int n2, int l2, int d, int pair_mode);
int pde_launch_tiled(const float *X, int n1, int l1, const float *Y, int n2, int l2, int d, int dyadic, int solver,
                     int pair_mode, int row_begin, int row_end, float *out, int out_row0, int out_rows,
                     long long out_ld, void *scratch, size_t scratch_bytes, hipStream_t s);
}  // namespace gpsig

using namespace gpsig;

// Channel padding of the feature records: exact for the first-order kernels up to 6 channels,
// multiples the instantiation tables cover otherwise (sig_fo_inst / sig_ho).
static int pad_channels(int d, int order) {
  if (order == 1 && d <= 6) return d;
  if (order > 1 && d <= 4) return 4;
  if (d <= 8) return 8;
  if (d <= 16) return 16;
  if (d <= 32) return 32;
  return 0;
}

static size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

// Channel counts past the fixed instantiations (8) run the first-order forward on channel-major records
// with a runtime channel loop (wide.h), which beats the padded fixed kernels from 9 channels on
// (N = 1024, L = 128, M = 4: d = 16 12.7 vs 15.4 ms, d = 32 23.5 vs 35.6 ms; d = 8 7.7 vs 6.4 ms).
// GPSIG_FO_FIXED_MAX lowers the crossover for A/B runs (0 sends every channel count to the wide kernels).
namespace gpsig {
int fo_fixed_max() {
  static const int v = [] {
    const char *e = getenv("GPSIG_FO_FIXED_MAX");
    const int x = e ? atoi(e) : 8;
    return x < 8 ? (x < 0 ? 0 : x) : 8;
  }();
  return v;
}
}  // namespace gpsig
static bool wide_channels(int d, int order) { return order == 1 && d > fo_fixed_max(); }

// The wide-channel Gram with the increment GEMM on the matrix cores (sig_fo_mf.h) for the difference seeds
// of the Gram pair modes; GPSIG_WIDE_MF=0 keeps the runtime-channel-loop kernel (A/B runs).
namespace gpsig {
bool wide_mf_enabled() {
  static const bool v = [] {
    const char *e = getenv("GPSIG_WIDE_MF");
    return !(e && atoi(e) == 0);
  }();
  return v;
}
}  // namespace gpsig

static size_t feat_bytes(int n, int l, int d) {
  size_t wb = d > fo_fixed_max() ? align256((size_t)n * wide_rec_floats(d, l) * sizeof(float)) : 0;
  const size_t mb = d > fo_fixed_max() ? align256(mf_records_bytes(n, l, d)) : 0;
  wb = mb > wb ? mb : wb;
  const int DP = pad_channels(d, 2);  // the wider of the two paddings
  const size_t fb = DP ? align256((size_t)n * l * feat_stride(DP) * sizeof(float)) : 0;
  return wb > fb ? wb : fb;
}

static int seed_of(int base_kind, int difference) {
  if (base_kind == GPSIG_BASE_RBF) return difference ? SEED_RBF_DIFF : SEED_RBF_POINT;
  if (base_kind == GPSIG_BASE_LINEAR) return difference ? SEED_LIN_DIFF : SEED_LIN_POINT;
  return -1;
}

// the matrix-core wide Gram's column-block carries (sequences past 160 points), after the records
static size_t mf_scratch(int l1, int l2, int d) {
  return d > fo_fixed_max() && wide_mf_enabled() ? align256(mf_gram_scratch_bytes(l1, l2, d)) : 0;
}

// the wide diagonal's seed tiles (wide.h DiagTiles, RBF difference seed): one chunk of pairs
static bool diag_tiled(int n, int l, int d, int order) {
  if (order != 1 || d <= fo_fixed_max() || n <= 0) return false;
  int W, LP;
  fo_wide_geo(l, SEED_RBF_DIFF, &W, &LP);
  return (long long)LP * W >= l && diag_tiles_apply(l, d, W, LP, SEED_RBF_DIFF, 1);
}
static size_t diag_tile_bytes(int n, int l, int d, int order) {
  if (!diag_tiled(n, l, d, order)) return 0;
  int W, LP;
  fo_wide_geo(l, SEED_RBF_DIFF, &W, &LP);
  const DiagTiles dt = diag_tiles_of(l, W, LP);
  return align256((size_t)diag_tile_pairs(dt, n) * dt.pair * sizeof(float));
}

extern "C" size_t gpsig_sig_workspace_bytes(int n1, int l1, int n2, int l2, int d) {
  return feat_bytes(n1, l1, d) + feat_bytes(n2, l2, d) + mf_scratch(l1, l2, d) + diag_tile_bytes(n1, l1, d, 1);
}

// The workspace of one gpsig_sig_gram / gpsig_sig_diag call: the feature records, or for the higher-order
// recursion past 32 channels the increments and one chunk's increment tile (sig_ho.hip tile mode).
extern "C" size_t gpsig_sig_workspace_bytes_ex(int n1, int l1, int n2, int l2, int d, int order, int pair_mode) {
  if (n1 <= 0 || n2 <= 0 || l1 < 1 || l2 < 1 || d <= 0) return 0;
  if (ho_tiled(d, order) && l1 >= 2 && l2 >= 2) return ho_tile_bytes(n1, l1, n2, l2, d, pair_mode);
  return gpsig_sig_workspace_bytes(n1, l1, n2, l2, d);
}

extern "C" size_t gpsig_sig_split_bytes(int l1, int l2, int d, int num_levels) {
  const int DP = pad_channels(d, 1);
  if (DP == 0 || l1 < 2 || l2 < 2 || num_levels < 1 || num_levels > 8) return 0;
  return fo_split_bytes(l1, l2, DP, num_levels);
}


static int sig_gram_impl(const float *X, int n1, int l1, const float *Y, int n2, int l2, int d, int num_levels,
                         int order, int base_kind, int difference, int pair_mode, int row_begin, int row_end,
                         const float *rs1, const float *rs2, const float *scale, float jitter, int out_mode,
                         float *out, int out_row0, int out_rows, float *state, void *workspace,
                         size_t workspace_bytes, gpsig_stream_t stream) {
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (!X || !Y || !out || n1 <= 0 || n2 <= 0 || d <= 0 || num_levels < 1) return GPSIG_EINVAL;
  if (l1 < 1 || l2 < 1 || (difference && (l1 < 2 || l2 < 2))) return GPSIG_EINVAL;
  if (pair_mode < GPSIG_PAIRS_RECT || pair_mode > GPSIG_PAIRS_DIAG) return GPSIG_EINVAL;
  if (row_begin < 0 || row_end > n1 || row_begin > row_end) return GPSIG_EINVAL;
  if (pair_mode != GPSIG_PAIRS_RECT && (n1 != n2 || l1 != l2)) return GPSIG_EINVAL;
  if (out_mode < GPSIG_OUT_LEVELS || out_mode > GPSIG_OUT_RSQRT) return GPSIG_EINVAL;
  if (out_mode == GPSIG_OUT_RSQRT && pair_mode != GPSIG_PAIRS_DIAG) return GPSIG_EINVAL;
  if ((rs1 == nullptr) != (rs2 == nullptr)) return GPSIG_EINVAL;
  if (order < 1) return GPSIG_EINVAL;
  const bool mfma = (base_kind & GPSIG_BASE_SEED_MFMA) != 0;
  const bool split = (base_kind & GPSIG_GRAM_SPLIT) != 0;
  base_kind &= ~(GPSIG_BASE_SEED_MFMA | GPSIG_GRAM_SPLIT);
  const int seed = seed_of(base_kind, difference);
  if (mfma && (seed != SEED_RBF_DIFF || order != 1 || state)) return GPSIG_EUNSUPPORTED;
  if (split && (mfma || seed != SEED_RBF_DIFF || order != 1 || state || pair_mode == GPSIG_PAIRS_DIAG))
    return GPSIG_EUNSUPPORTED;
  const bool tiled = ho_tiled(d, order);  // higher order past 32 channels: cells from an increment-Gram tile
  if (tiled && ((seed != SEED_LIN_DIFF && seed != SEED_RBF_DIFF) || mfma || split || state)) return GPSIG_EUNSUPPORTED;
  const bool wide = wide_channels(d, order);
  const int DP = (wide || tiled) ? 0 : pad_channels(d, order);
  if (seed < 0 || (DP == 0 && !wide && !tiled)) return GPSIG_EUNSUPPORTED;
  if (wide && (mfma || split)) return GPSIG_EUNSUPPORTED;
  if (row_end == row_begin) return GPSIG_OK;
  if (tiled) {
    SigArgs a{};
    a.n1 = n1; a.l1 = l1; a.n2 = n2; a.l2 = l2;
    a.M = num_levels;
    a.order = order;
    a.pair_mode = pair_mode;
    a.row_begin = row_begin;
    a.row_end = row_end;
    a.rs1 = rs1; a.rs2 = rs2; a.scale = scale;
    a.jitter = jitter;
    a.out_mode = out_mode;
    a.out = out;
    a.out_row0 = out_row0;
    a.out_rows = out_rows;
    a.out_ld = n2;
    a.out_lvl = pair_mode == GPSIG_PAIRS_DIAG ? (long long)n1 : (long long)out_rows * n2;
    return sig_ho_tiled(a, X, Y, d, seed, workspace, workspace_bytes, s);
  }

  const bool same = (X == Y && n1 == n2 && l1 == l2);
  const bool mf = wide && wide_mf_enabled() && pair_mode != GPSIG_PAIRS_DIAG &&
                  (seed == SEED_RBF_DIFF || seed == SEED_LIN_DIFF) && mf_gram_applies(d, l2);
  const size_t fx_b = wide ? feat_bytes(n1, l1, d) : align256((size_t)n1 * l1 * feat_stride(DP) * sizeof(float));
  const size_t fy_b = same ? 0 : (wide ? feat_bytes(n2, l2, d) : align256((size_t)n2 * l2 * feat_stride(DP) * sizeof(float)));
  const size_t dm_b = split ? gpsig_sig_split_bytes(l1, l2, d, num_levels) : 0;
  if (split && dm_b == 0) return GPSIG_EUNSUPPORTED;
  const size_t mc_b = mf ? mf_scratch(l1, l2, d) : 0;
  const bool dtiles = wide && pair_mode == GPSIG_PAIRS_DIAG && seed == SEED_RBF_DIFF && !state &&
                      diag_tiled(n1, l1, d, order);
  const size_t dt_b = dtiles ? diag_tile_bytes(n1, l1, d, order) : 0;
  if (!workspace || workspace_bytes < fx_b + fy_b + dm_b + mc_b + dt_b) return GPSIG_EWORKSPACE;
  float *FX = static_cast<float *>(workspace);
  float *FY = same ? FX : reinterpret_cast<float *>(static_cast<char *>(workspace) + fx_b);
  int rc = mf ? mf_records(X, n1, l1, d, FX, s) : wide ? wide_records(X, n1, l1, d, FX, s) : features(X, n1, l1, d, DP, FX, s);
  if (rc) return rc;
  if (!same && (rc = mf ? mf_records(Y, n2, l2, d, FY, s)
                        : wide ? wide_records(Y, n2, l2, d, FY, s) : features(Y, n2, l2, d, DP, FY, s)))
    return rc;

  SigArgs a{};
  a.FX = FX;
  a.FY = FY;
  a.n1 = n1; a.l1 = l1; a.n2 = n2; a.l2 = l2;
  a.fs = feat_stride(DP);
  a.M = num_levels;
  a.order = order;
  a.pair_mode = pair_mode;
  a.row_begin = row_begin;
  a.row_end = row_end;
  a.rs1 = rs1; a.rs2 = rs2; a.scale = scale;
  a.jitter = jitter;
  a.out_mode = out_mode;
  a.out = out;
  a.out_row0 = out_row0;
  a.out_rows = out_rows;
  a.out_ld = n2;
  a.out_lvl = (long long)out_rows * n2;
  a.state = state;
  a.mfma = mfma ? 1 : 0;
  a.dmbuf = split ? reinterpret_cast<float *>(static_cast<char *>(workspace) + fx_b + fy_b) : nullptr;
  a.wd = d;
  a.lw1 = wide_lw(l1);
  a.lw2 = wide_lw(l2);
  a.sx = wide_rec_floats(d, l1);
  a.sy = wide_rec_floats(d, l2);
  if (mf)
    return sig_fo_mf(a, d, seed, mc_b ? reinterpret_cast<float *>(static_cast<char *>(workspace) + fx_b + fy_b) : nullptr, s);

  if (dtiles) {
    // the diagonal's pairs in chunks: their seed tiles (two batched GEMMs + the anchors), then the launch
    int gW, gLP;
    fo_wide_geo(l2, seed, &gW, &gLP);
    const DiagTiles dt = diag_tiles_of(l1, gW, gLP);
    const int cp = diag_tile_pairs(dt, n1);
    float *T = reinterpret_cast<float *>(static_cast<char *>(workspace) + fx_b + fy_b + dm_b + mc_b);
    a.out_lvl = n1;
    a.dtile = T;
    a.dt_pair = dt.pair;
    a.dt_rows = dt.rows;
    a.dt_ld = dt.ld;
    for (int c0 = row_begin; c0 < row_end; c0 += cp) {
      const int c1 = c0 + cp < row_end ? c0 + cp : row_end;
      if ((rc = wide_diag_tiles(FX, a.sx, d, a.lw1, c0, c1 - c0, dt, T, s))) return rc;
      SigArgs c = a;
      c.row_begin = c0;
      c.row_end = c1;
      c.dt_a0 = c0;
      if ((rc = sig_fo_launch(c, DP, seed, (c1 - c0 + 3) / 4, s))) return rc;
    }
    return GPSIG_OK;
  }
  const int LP = (order == 1) ? fo_lanes_per_pair(l2, DP, num_levels, mfma, seed, split) : ho_lanes_per_pair(l2, order, num_levels);
  if (LP == 0) return GPSIG_EUNSUPPORTED;
  const int G = 64 / LP;
  long long nblocks = 0;
  if (pair_mode == GPSIG_PAIRS_DIAG) {
    a.out_lvl = n1;
    nblocks = (row_end - row_begin + 3) / 4;
  } else {
    const int ta0 = row_begin / 4, ta1 = (row_end + 3) / 4;
    const int ntb = (n2 + G - 1) / G;
    a.tiles_a0 = ta0;
    a.ntb = ntb;
    if (pair_mode == GPSIG_PAIRS_RECT) {
      nblocks = (long long)(ta1 - ta0) * ntb;
    } else {
      // tile row r starts at B tile floor(4 r / G) (G = 6 for the 10-lane groups: not a whole ratio)
      a.tile_base = upper_prefix_g(ta0, ntb, G);
      nblocks = upper_prefix_g(ta1, ntb, G) - a.tile_base;
    }
  }
  if (nblocks > 0x7fffffffLL) return GPSIG_EUNSUPPORTED;
  return (order == 1) ? sig_fo_launch(a, DP, seed, nblocks, s) : sig_ho_launch(a, DP, seed, nblocks, s);
}

extern "C" int gpsig_sig_gram(const float *X, int n1, int l1, const float *Y, int n2, int l2, int d, int num_levels,
                              int order, int base_kind, int difference, int pair_mode, int row_begin, int row_end,
                              const float *rs1, const float *rs2, const float *scale, float jitter, int out_mode,
                              float *out, int out_row0, int out_rows, void *workspace, size_t workspace_bytes,
                              gpsig_stream_t stream) {
  return sig_gram_impl(X, n1, l1, Y, n2, l2, d, num_levels, order, base_kind, difference, pair_mode, row_begin,
                       row_end, rs1, rs2, scale, jitter, out_mode, out, out_row0, out_rows, nullptr, workspace,
                       workspace_bytes, stream);
}

extern "C" size_t gpsig_sig_state_bytes(int n1, int n2, int l2, int num_levels, int pair_mode) {
  if (n1 <= 0 || n2 <= 0 || l2 < 2 || num_levels < 1) return 0;
  long long slots;
  if (pair_mode == GPSIG_PAIRS_RECT) slots = (long long)n1 * n2;
  else if (pair_mode == GPSIG_PAIRS_UPPER && n1 == n2) slots = (long long)n1 * (n1 + 1) / 2;
  else return 0;
  return (size_t)slots * (size_t)state_stride(num_levels, l2) * sizeof(float);
}

extern "C" int gpsig_sig_gram_state(const float *X, int n1, int l1, const float *Y, int n2, int l2, int d,
                                    int num_levels, int base_kind, int pair_mode, int row_begin, int row_end,
                                    const float *rs1, const float *rs2, const float *scale, float jitter,
                                    int out_mode, float *out, int out_row0, int out_rows, float *state,
                                    size_t state_bytes, void *workspace, size_t workspace_bytes,
                                    gpsig_stream_t stream) {
  if (!state) return GPSIG_EINVAL;
  if (pair_mode != GPSIG_PAIRS_RECT && pair_mode != GPSIG_PAIRS_UPPER) return GPSIG_EINVAL;
  const size_t need = gpsig_sig_state_bytes(n1, n2, l2, num_levels, pair_mode);
  if (need == 0) return GPSIG_EINVAL;
  if (state_bytes < need) return GPSIG_EWORKSPACE;
  return sig_gram_impl(X, n1, l1, Y, n2, l2, d, num_levels, 1, base_kind, 1, pair_mode, row_begin, row_end, rs1,
                       rs2, scale, jitter, out_mode, out, out_row0, out_rows, state, workspace, workspace_bytes,
                       stream);
}

extern "C" int gpsig_sig_diag(const float *X, int n, int l, int d, int num_levels, int order, int base_kind,
                              int difference, float jitter, int out_mode, float *out, void *workspace,
                              size_t workspace_bytes, gpsig_stream_t stream) {
  if (out_mode != GPSIG_OUT_LEVELS && out_mode != GPSIG_OUT_RSQRT) return GPSIG_EINVAL;
  return gpsig_sig_gram(X, n, l, X, n, l, d, num_levels, order, base_kind, difference, GPSIG_PAIRS_DIAG, 0, n,
                        nullptr, nullptr, nullptr, jitter, out_mode, out, 0, n, workspace, workspace_bytes, stream);
}

extern "C" size_t gpsig_pde_scratch_bytes(int n1, int l1, int n2, int l2, int d, int dyadic, int pair_mode) {
  if (!pde_tiled(d, dyadic)) return 0;
  return pde_tile_scratch_bytes(n1, l1, n2, l2, d, pair_mode);
}

extern "C" int gpsig_pde_gram_ex(const float *X, int n1, int l1, const float *Y, int n2, int l2, int d, int dyadic,
                                 int solver, int pair_mode, int row_begin, int row_end, float *out, int out_row0,
                                 int out_rows, void *scratch, size_t scratch_bytes, gpsig_stream_t stream) {
  if (!X || !Y || !out || n1 <= 0 || n2 <= 0 || d <= 0 || l1 < 2 || l2 < 2) return GPSIG_EINVAL;
  if (dyadic < 0 || dyadic > 8 || (solver != 0 && solver != 1)) return GPSIG_EINVAL;
  if (pair_mode < GPSIG_PAIRS_RECT || pair_mode > GPSIG_PAIRS_DIAG) return GPSIG_EINVAL;
  if (row_begin < 0 || row_end > n1 || row_begin > row_end) return GPSIG_EINVAL;
  if (pair_mode != GPSIG_PAIRS_RECT && (n1 != n2 || l1 != l2)) return GPSIG_EINVAL;
  if (row_end == row_begin) return GPSIG_OK;
  if (pde_tiled(d, dyadic))
    return pde_launch_tiled(X, n1, l1, Y, n2, l2, d, dyadic, solver, pair_mode, row_begin, row_end, out, out_row0,
                            out_rows, n2, scratch, scratch_bytes, reinterpret_cast<hipStream_t>(stream));
  return pde_launch(X, n1, l1, Y, n2, l2, d, dyadic, solver, pair_mode, row_begin, row_end, out, out_row0,
                    out_rows, n2, reinterpret_cast<hipStream_t>(stream));
}

extern "C" int gpsig_pde_gram(const float *X, int n1, int l1, const float *Y, int n2, int l2, int d, int dyadic,
                              int solver, int pair_mode, int row_begin, int row_end, float *out, int out_row0,
                              int out_rows, gpsig_stream_t stream) {
  return gpsig_pde_gram_ex(X, n1, l1, Y, n2, l2, d, dyadic, solver, pair_mode, row_begin, row_end, out, out_row0,
                           out_rows, nullptr, 0, stream);
}

extern "C" int gpsig_pde_diag_ex(const float *X, int n, int l, int d, int dyadic, int solver, float *out,
                                 void *scratch, size_t scratch_bytes, gpsig_stream_t stream) {
  return gpsig_pde_gram_ex(X, n, l, X, n, l, d, dyadic, solver, GPSIG_PAIRS_DIAG, 0, n, out, 0, n, scratch,
                           scratch_bytes, stream);
}

extern "C" int gpsig_pde_diag(const float *X, int n, int l, int d, int dyadic, int solver, float *out,
                              gpsig_stream_t stream) {
  return gpsig_pde_diag_ex(X, n, l, d, dyadic, solver, out, nullptr, 0, stream);
}

extern "C" int gpsig_sym_assemble(const float *src, const long long *row_off, long long level_stride, int n,
                                  int levels, float *dst, gpsig_stream_t stream) {
  if (!src || !dst || !row_off || n <= 0 || levels <= 0 || level_stride < 0) return GPSIG_EINVAL;
  return sym_assemble_launch(src, row_off, level_stride, n, levels, dst, reinterpret_cast<hipStream_t>(stream));
}

extern "C" const char *gpsig_version(void) { return "gpsig_amd 0.1 (gfx950)"; }
