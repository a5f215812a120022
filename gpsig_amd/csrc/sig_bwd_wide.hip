// gpsig_amd -- host side of the wide-channel Gram VJP (sig_bwd_wide.h): chunks of x-rows, the point-weight
// tile of each chunk, and the emission GEMMs on the matrix cores (gemm.hip):
//   [gX | rowsum] += W [Y | 1],   [gY | colsum] += W^T [X | 1],   then  g -= rowsum * x  (RBF)
// (UPPER / DIAG: Y = X, both sides go to gX).
#include "sig_bwd_wide.h"
#include "gemm.h"

namespace gpsig {

template <int M>
int sig_bwd_wide_launch_m(const BwdArgs &a, int seed, long long nblocks, hipStream_t s);
bool ho_bwd_supported(int l2, int order, int M, int seed);
int sig_ho_bwd_launch(const BwdArgs &a, int order, int seed, long long nblocks, hipStream_t s);

// Xa[r][k] = X[r][k] (k < d), Xa[r][d] = 1
__global__ __launch_bounds__(256) void aug_ones_kernel(const float *__restrict__ X, long long rows, int d,
                                                       float *__restrict__ Xa) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= rows * (d + 1)) return;
  const long long r = idx / (d + 1);
  const int k = (int)(idx % (d + 1));
  Xa[idx] = k < d ? X[r * d + k] : 1.0f;
}

// g[r][k] += G[r][k] - G[r][d] x[r][k] (RBF: the base kernel's derivative k (y - x) puts -x * rowsum(W)
// on every point), linear: g[r][k] += G[r][k]
__global__ __launch_bounds__(256) void emit_correct_kernel(const float *__restrict__ G, const float *__restrict__ X,
                                                           long long rows, int d, int rbf, float *__restrict__ g) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= rows * d) return;
  const long long r = idx / d;
  const int k = (int)(idx % d);
  const float *Gr = G + r * (d + 1);
  g[idx] += rbf ? __builtin_fmaf(-Gr[d], X[idx], Gr[k]) : Gr[k];
}

static size_t al256(size_t b) { return (b + 255) & ~(size_t)255; }

DiagTiles diag_tiles_of(int l, int W, int LP) {
  const long long rp = (((long long)(l - 1) + 7) / 8) * 8;
  const long long nc = (long long)LP * W;
  return {rp, nc, 2 * rp * nc + 2 * (rp / DIAG_TILE_ANCHOR) * nc};
}
bool diag_tiles_apply(int l, int d, int W, int LP, int seed, int order) {
  return seed == SEED_RBF_DIFF && order == 1 && W > 0 && (long long)LP * W <= wide_lw(l) && l >= 2 && d > 0 &&
         (((long long)(l - 1) + 7) / 8) * 8 <= wide_lw(l);
}

// anchor rows: thread per (pair, group of ANCHOR_G anchor rows, column j); the pair and the group are
// workgroup-uniform (grid y / z), so the anchor points x_i come in as scalar loads and every thread reuses its
// column's x_j and dx_j across the group's rows
constexpr int ANCHOR_G = 8;
__global__ __launch_bounds__(256) void wide_diag_anchor_kernel(const float *__restrict__ R, long long sx, int d, int lw,
                                                               DiagTiles dt, float *__restrict__ T) {
  const int na = (int)(dt.rows / DIAG_TILE_ANCHOR);
  const int j = blockIdx.x * 256 + threadIdx.x;
  const int t0 = blockIdx.y * ANCHOR_G, a = blockIdx.z;
  if (j >= dt.ld) return;
  const float *rec = R + (long long)a * sx;
  float s[ANCHOR_G], qq[ANCHOR_G];
  const float q0 = -rec[(long long)2 * d * lw + j];
#pragma unroll
  for (int g = 0; g < ANCHOR_G; ++g) {
    s[g] = 0.0f;
    qq[g] = q0;
  }
#pragma unroll 4
  for (int k = 0; k < d; ++k) {
    const float xj = rec[(long long)k * lw + j], dxj = rec[(long long)(d + k) * lw + j];
    const float *xk = rec + (long long)k * lw;
#pragma unroll
    for (int g = 0; g < ANCHOR_G; ++g) {
      // a group past the last anchor repeats the last one (not stored)
      const int t = t0 + g < na ? t0 + g : na - 1;
      const float df = xk[DIAG_TILE_ANCHOR * t] - xj;
      s[g] = __builtin_fmaf(df, df, s[g]);
      qq[g] = __builtin_fmaf(df, dxj, qq[g]);
    }
  }
  constexpr float NHL2E = -0.72134752044448170f, L2E = 1.4426950408889634f;
#pragma unroll
  for (int g = 0; g < ANCHOR_G; ++g) {
    const int t = t0 + g;
    if (t >= na) break;
    float *o = T + (long long)a * dt.pair + 2 * dt.rows * dt.ld + (long long)(2 * t) * dt.ld + j;
    o[0] = __builtin_amdgcn_exp2f(s[g] * NHL2E);
    o[dt.ld] = __builtin_fabsf(qq[g]) < EM1_TAU ? em1_small(qq[g]) : __builtin_amdgcn_exp2f(qq[g] * L2E) - 1.0f;
  }
}

int wide_diag_tiles(const float *FX, long long sx, int d, int lw, int a0, int npairs, DiagTiles dt, float *T,
                           hipStream_t s) {
  const float *rec = FX + (long long)a0 * sx;
  int rc;
  if (npairs > 65535) return GPSIG_EUNSUPPORTED;  // the anchor launch's grid z; checked before any launch
  // c_ij: op(A)[i][k] = dx_k[i], op(B)[k][j] = dx_k[j]
  if ((rc = gemm_f32(s, true, false, (int)dt.rows, (int)dt.ld, d, 1.0f, rec + (long long)d * lw, lw, sx,
                     rec + (long long)d * lw, lw, sx, 0.0f, T, dt.ld, dt.pair, npairs, 0, 0, nullptr, 0)))
    return rc;
  // <dx_i, x_j>
  if ((rc = gemm_f32(s, true, false, (int)dt.rows, (int)dt.ld, d, 1.0f, rec + (long long)d * lw, lw, sx, rec, lw, sx,
                     0.0f, T + dt.rows * dt.ld, dt.ld, dt.pair, npairs, 0, 0, nullptr, 0)))
    return rc;
  const long long na = dt.rows / DIAG_TILE_ANCHOR;
  hipLaunchKernelGGL(wide_diag_anchor_kernel,
                     dim3((unsigned)((dt.ld + 255) / 256), (unsigned)((na + ANCHOR_G - 1) / ANCHOR_G), (unsigned)npairs),
                     dim3(256), 0, s, rec, sx, d, lw, dt, T);
  return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
}
static inline long long up_prefix(long long r, long long ntb, long long k) { return r * ntb - k * r * (r - 1) / 2; }

// point-weight tile budget of one chunk of x-rows
constexpr size_t WIDE_TILE_BYTES = (size_t)1 << 30;

struct WidePlan {
  int rows;  // x-rows per chunk (multiple of 4)
  size_t rec_x, rec_y, aug_x, aug_y, gx, gc, tile, part, dtile;
};

static WidePlan wide_plan(int n1, int l1, int n2, int l2, int d, int pair_mode) {
  WidePlan p{};
  const bool same = pair_mode != GPSIG_PAIRS_RECT;
  const long long cols = pair_mode == GPSIG_PAIRS_DIAG ? (long long)l1 : (long long)n2 * l2;
  long long rows = (long long)(WIDE_TILE_BYTES / ((size_t)l1 * cols * sizeof(float)));
  rows = rows < 4 ? 4 : (rows / 4) * 4;
  const BwdGeo dg = bwd_geometry_wide(l1);
  if (pair_mode == GPSIG_PAIRS_DIAG && dg.W > 0) {  // a chunk's pairs also fit the seed-tile budget
    const long long tp = ((long long)diag_tile_pairs(diag_tiles_of(l1, dg.W, dg.LP), 1 << 30) / 4) * 4;
    if (rows > tp) rows = tp < 4 ? 4 : tp;
  }
  if (rows > ((n1 + 3) / 4) * 4) rows = ((n1 + 3) / 4) * 4;
  p.rows = (int)rows;
  p.rec_x = al256((size_t)n1 * wide_rec_floats(d, l1) * sizeof(float));
  p.rec_y = same ? 0 : al256((size_t)n2 * wide_rec_floats(d, l2) * sizeof(float));
  p.aug_x = al256((size_t)n1 * l1 * (d + 1) * sizeof(float));
  p.aug_y = same ? 0 : al256((size_t)n2 * l2 * (d + 1) * sizeof(float));
  p.gx = al256((size_t)n1 * l1 * (d + 1) * sizeof(float));
  p.gc = pair_mode == GPSIG_PAIRS_DIAG ? 0 : al256((size_t)n2 * l2 * (d + 1) * sizeof(float));
  p.tile = al256((size_t)rows * l1 * cols * sizeof(float));
  // split-K partials of the row-side (rows * l1 x (d + 1), K = cols) and column-side (cols x (d + 1),
  // K = rows * l1) products of a full chunk; gemm_f32 clamps any split to this capacity
  if (pair_mode != GPSIG_PAIRS_DIAG) {
    const size_t pr = gemm_splitk_bytes((int)(rows * l1), d + 1, (int)cols);
    const size_t pc = gemm_splitk_bytes((int)cols, d + 1, (int)(rows * l1));
    p.part = al256(pr > pc ? pr : pc);
  } else if (dg.W > 0) {
    p.dtile = al256((size_t)rows * diag_tiles_of(l1, dg.W, dg.LP).pair * sizeof(float));
  }
  return p;
}

static size_t plan_bytes(const WidePlan &p) {
  return p.rec_x + p.rec_y + p.aug_x + p.aug_y + p.gx + p.gc + p.tile + p.part + p.dtile;
}

// workspace of any pair mode (the query does not name one)
size_t sig_bwd_wide_workspace(int n1, int l1, int n2, int l2, int d) {
  size_t best = 0;
  for (int pm : {GPSIG_PAIRS_RECT, GPSIG_PAIRS_UPPER, GPSIG_PAIRS_DIAG}) {
    if (pm != GPSIG_PAIRS_RECT && (n1 != n2 || l1 != l2)) continue;
    const size_t b = plan_bytes(wide_plan(n1, l1, n2, l2, d, pm));
    best = b > best ? b : best;
  }
  return best;
}

// The wide-channel VJP (order 1) and the higher-order VJP (order > 1, sig_ho_bwd.h: one pair per wave, the
// same tiles and GEMMs).  a: filled by the caller as for the fixed kernels (pair mode, rows, gout, rs,
// scale, jitter, gX/gY/grs, gscale slots, state); X, Y the raw (n, l, d) inputs.
int sig_bwd_wide(BwdArgs a, const float *X, const float *Y, int seed, void *workspace, size_t workspace_bytes,
                 hipStream_t s, int order) {
  const int n1 = a.n1, l1 = a.l1, n2 = a.n2, l2 = a.l2, d = a.d, pm = a.pair_mode;
  if (order > 1 ? !ho_bwd_supported(l2, order, a.M, seed) || a.state : l2 > 512) return GPSIG_EUNSUPPORTED;
  const BwdGeo geo = order > 1 ? BwdGeo{4, 64} : bwd_geometry_wide(l2);
  const WidePlan pl = wide_plan(n1, l1, n2, l2, d, pm);
  if (!workspace || workspace_bytes < plan_bytes(pl)) return GPSIG_EWORKSPACE;
  char *w = static_cast<char *>(workspace);
  float *FX = reinterpret_cast<float *>(w); w += pl.rec_x;
  float *FY = pl.rec_y ? reinterpret_cast<float *>(w) : FX; w += pl.rec_y;
  float *Xa = reinterpret_cast<float *>(w); w += pl.aug_x;
  float *Ya = pl.aug_y ? reinterpret_cast<float *>(w) : Xa; w += pl.aug_y;
  float *Gx = reinterpret_cast<float *>(w); w += pl.gx;
  float *Gc = pl.gc ? reinterpret_cast<float *>(w) : nullptr; w += pl.gc;
  float *T = reinterpret_cast<float *>(w); w += pl.tile;
  float *part = pl.part ? reinterpret_cast<float *>(w) : nullptr; w += pl.part;
  float *DT = pl.dtile ? reinterpret_cast<float *>(w) : nullptr;
  int rc = wide_records(X, n1, l1, d, FX, s);
  if (rc) return rc;
  if (pl.rec_y && (rc = wide_records(Y, n2, l2, d, FY, s))) return rc;
  const long long rx = (long long)n1 * l1, ry = (long long)n2 * l2;
  hipLaunchKernelGGL(aug_ones_kernel, dim3((unsigned)((rx * (d + 1) + 255) / 256)), dim3(256), 0, s, X, rx, d, Xa);
  if (pl.aug_y)
    hipLaunchKernelGGL(aug_ones_kernel, dim3((unsigned)((ry * (d + 1) + 255) / 256)), dim3(256), 0, s, Y, ry, d, Ya);
  if (Gc && hipMemsetAsync(Gc, 0, (size_t)ry * (d + 1) * sizeof(float), s) != hipSuccess) return GPSIG_ELAUNCH;
  if (hipGetLastError() != hipSuccess) return GPSIG_ELAUNCH;

  a.FX = FX;
  a.FY = FY;
  a.wd = d;
  a.lw1 = wide_lw(l1);
  a.lw2 = wide_lw(l2);
  a.sx = wide_rec_floats(d, l1);
  a.sy = wide_rec_floats(d, l2);
  a.tile = T;
  a.nblk = 1;
  if (order == 1) a.scratch = nullptr;  // order > 1: the caller's slab region of the 8-wave split VJP (or null)
  a.scr_stride = 0;
  const int G = 64 / geo.LP;
  const int ntb = (n2 + G - 1) / G;
  const int rb0 = a.row_begin, rb1 = a.row_end;
  const bool rbf = seed == SEED_RBF_DIFF || seed == SEED_RBF_POINT;
  for (int r0 = (rb0 / 4) * 4; r0 < rb1; r0 += pl.rows) {
    const int r1 = r0 + pl.rows < rb1 ? r0 + pl.rows : rb1;
    const int c0 = r0 > rb0 ? r0 : rb0;  // rows of this chunk: [c0, r1)
    const int nr = r1 - r0;              // tile rows from r0 (the chunk's first 4-aligned row)
    BwdArgs c = a;
    c.row_begin = c0;
    c.row_end = r1;
    c.blk0 = 0;
    c.tile_a0 = r0;
    long long nblocks;
    long long tcols;  // tile row length (floats)
    if (pm == GPSIG_PAIRS_DIAG) {
      c.row_begin = c0;
      nblocks = (r1 - c0 + 3) / 4;
      // DIAG enumerates a = row_begin + 4 blk + wave: keep the tile rows relative to c0
      c.tile_a0 = c0;
      c.tile_b0 = 0;
      c.tile_as = (long long)l1 * l1;
      c.tile_ld = l1;
      tcols = l1;
      if (DT && r1 > c0 && diag_tiles_apply(l1, d, geo.W, geo.LP, seed, order)) {
        const DiagTiles dt = diag_tiles_of(l1, geo.W, geo.LP);
        if ((rc = wide_diag_tiles(FX, a.sx, d, a.lw1, c0, r1 - c0, dt, DT, s))) return rc;
        c.dtile = DT;
        c.dt_a0 = c0;
        c.dt_pair = dt.pair;
        c.dt_rows = dt.rows;
        c.dt_ld = dt.ld;
      }
    } else {
      const int ta0 = r0 / 4, ta1 = (r1 + 3) / 4;
      c.tiles_a0 = ta0;
      c.ntb = ntb;
      c.tile_b0 = pm == GPSIG_PAIRS_UPPER ? r0 : 0;
      tcols = (long long)(n2 - c.tile_b0) * l2;
      c.tile_as = (long long)l1 * tcols;
      c.tile_ld = tcols;
      if (pm == GPSIG_PAIRS_RECT) {
        nblocks = (long long)(ta1 - ta0) * ntb;
      } else {
        const int k = 4 / G;
        c.tile_base = up_prefix(ta0, ntb, k);
        nblocks = up_prefix(ta1, ntb, k) - c.tile_base;
      }
      // pairs b < a of the chunk's own rows (UPPER) and rows before the window (c0 > r0) are not
      // evaluated: their weights are zeros
      if ((pm == GPSIG_PAIRS_UPPER || c0 > r0) && hipMemsetAsync(T, 0, (size_t)nr * l1 * tcols * sizeof(float), s) != hipSuccess)
        return GPSIG_ELAUNCH;
    }
    if (nblocks > 0x7fffffffLL) return GPSIG_EUNSUPPORTED;
    if (nblocks > 0 && order > 1) {
      if ((rc = sig_ho_bwd_launch(c, order, seed, nblocks, s))) return rc;
    } else if (nblocks > 0) {
      switch (a.M) {
        case 1: rc = sig_bwd_wide_launch_m<1>(c, seed, nblocks, s); break;
        case 2: rc = sig_bwd_wide_launch_m<2>(c, seed, nblocks, s); break;
        case 3: rc = sig_bwd_wide_launch_m<3>(c, seed, nblocks, s); break;
        case 4: rc = sig_bwd_wide_launch_m<4>(c, seed, nblocks, s); break;
        case 5: rc = sig_bwd_wide_launch_m<5>(c, seed, nblocks, s); break;
        case 6: rc = sig_bwd_wide_launch_m<6>(c, seed, nblocks, s); break;
        case 7: rc = sig_bwd_wide_launch_m<7>(c, seed, nblocks, s); break;
        case 8: rc = sig_bwd_wide_launch_m<8>(c, seed, nblocks, s); break;
        default: return GPSIG_EUNSUPPORTED;
      }
      if (rc) return rc;
    }
    const int D1 = d + 1;
    if (pm == GPSIG_PAIRS_DIAG) {
      const int na = r1 - c0;
      float *Gxc = Gx + (long long)c0 * l1 * D1;
      const float *Xac = Xa + (long long)c0 * l1 * D1;
      // both sides of the pair (a, a): W X and W^T X, batched over the chunk's pairs
      if ((rc = gemm_f32(s, false, false, l1, D1, l1, 1.0f, T, l1, (long long)l1 * l1, Xac, D1, (long long)l1 * D1,
                         0.0f, Gxc, D1, (long long)l1 * D1, na, 0, 0, nullptr, 0)))
        return rc;
      if ((rc = gemm_f32(s, true, false, l1, D1, l1, 1.0f, T, l1, (long long)l1 * l1, Xac, D1, (long long)l1 * D1,
                         1.0f, Gxc, D1, (long long)l1 * D1, na, 0, 0, nullptr, 0)))
        return rc;
    } else {
      const int rows = nr * l1;
      const float *Bcols = (pm == GPSIG_PAIRS_UPPER ? Xa : Ya) + (long long)c.tile_b0 * l2 * D1;
      // row side: the chunk's rows of Gx
      if ((rc = gemm_f32(s, false, false, rows, D1, (int)tcols, 1.0f, T, tcols, 0, Bcols, D1, 0, 0.0f,
                         Gx + (long long)r0 * l1 * D1, D1, 0, 1, 0, 0, part, pl.part)))
        return rc;
      // column side: accumulated over the chunks
      if ((rc = gemm_f32(s, true, false, (int)tcols, D1, rows, 1.0f, T, tcols, 0, Xa + (long long)r0 * l1 * D1, D1,
                         0, 1.0f, Gc + (long long)c.tile_b0 * l2 * D1, D1, 0, 1, 0, 0, part, pl.part)))
        return rc;
    }
  }
  // point gradients: rows [rb0, rb1) of x from Gx; all of y (or x again) from Gc
  {
    const long long r0 = (long long)rb0 * l1, nrw = (long long)(rb1 - rb0) * l1;
    hipLaunchKernelGGL(emit_correct_kernel, dim3((unsigned)((nrw * d + 255) / 256)), dim3(256), 0, s,
                       Gx + r0 * (d + 1), X + r0 * d, nrw, d, rbf ? 1 : 0, a.gX + r0 * d);
    if (Gc) {
      float *gy = pm == GPSIG_PAIRS_RECT ? a.gY : a.gX;
      hipLaunchKernelGGL(emit_correct_kernel, dim3((unsigned)((ry * d + 255) / 256)), dim3(256), 0, s, Gc,
                         pm == GPSIG_PAIRS_RECT ? Y : X, ry, d, rbf ? 1 : 0, gy);
    }
  }
  return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
}

}  // namespace gpsig
