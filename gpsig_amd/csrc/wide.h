// gpsig_amd -- wide channel counts: the truncated-signature kernels with a runtime channel loop.
//
// The fixed-channel kernels keep a lane's column data (y_j, dy_j for W columns) in registers and are
// instantiated per channel count (DP <= 8).  Past that the reference's own training runs feed 26 to
// 1928 channels (benchmarks/run_gpsig_benchmarks.py:32 with add_time and num_lags = 1;
// benchmarks/models/train_gpsigrnn.py:81-83), where per-channel instantiations neither fit the
// register file nor scale.  Here the channel count is a runtime value:
//
//   * the sequence records are channel-major (wide_records_kernel): x[k][j], dx[k][j] with the point
//     index contiguous, so the W columns of a lane are one or two 16-byte loads per channel and the
//     rows of the wave's sequence are one scalar load per channel;
//   * the seed's inner products (the reference's _square_dist GEMM, kernels.py:946-957, restricted to
//     what the recursion consumes: c_ij = <dx_i, dy_j> for every cell and p_ij = <y_j, dx_i> - g_i for
//     one column pair per lane) are computed for R rows at once in a channel loop, so every column
//     value loaded is used R times;
//   * the rows then run through the fixed kernels' recursion unchanged (sig_fo.h), with the same
//     exp-free row and column recurrences and the same exact re-anchoring as RbfSeedPk (sig_common.h).
//
// The register footprint no longer depends on the channel count, so one instantiation per (W, LP, M,
// seed) serves every d.
#pragma once
#include "sig_common.h"

namespace gpsig {

typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));  // dword-aligned 16-byte loads
typedef float f2u __attribute__((ext_vector_type(2), aligned(4)));  // dword-aligned 8-byte loads

// W consecutive floats from q (dword-aligned): 16-byte loads, or 8-byte loads for W = 2 (the split higher-order
// VJP, sig_ho_bwd_split.h)
template <int W>
GPSIG_DEV void ld_cols(const float *q, float (&v)[W]) {
  if constexpr (W % 4 == 0) {
#pragma unroll
    for (int h = 0; h < W / 4; ++h) {
      const f4u t = *reinterpret_cast<const f4u *>(q + 4 * h);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[4 * h + e] = t[e];
    }
  } else {
    static_assert(W == 2, "columns per lane");
    const f2u t = *reinterpret_cast<const f2u *>(q);
    v[0] = t[0];
    v[1] = t[1];
  }
}

// Padded record length: every column a lane group reads (up to 512 past a column block's start) and
// every row a chunk of R <= 8 rows reads stays inside the sequence's record; columns past the sequence
// repeat its last point with a zero increment, so their cells are exact zeros.
__host__ __device__ inline int wide_lw(int l) {
  if (l > 504) return ((l + 7) & ~7) + 520;
  int c = 64;
  while (c < l) c *= 2;
  const int r = ((l + 8) + 7) & ~7;
  return c > r ? c : r;
}
__host__ __device__ inline long long wide_rec_floats(int d, int l) { return (long long)(2 * d + 2) * wide_lw(l); }

// Record of sequence s: [x: d x lw][dx: d x lw][hdx: lw][g: lw]
//   hdx_j = |dx_j|^2 / 2, g_j = <x_j, dx_j> + |dx_j|^2 / 2 (fp64 accumulation, rounded once) -- the same
//   fp32 values as the fixed-channel feature records (sig_fo.hip features_kernel).
__global__ __launch_bounds__(256) void wide_records_kernel(const float *__restrict__ X, int n, int l, int d,
                                                           float *__restrict__ R);
int wide_records(const float *X, int n, int l, int d, float *R, hipStream_t s);

// ---------------------------------------------------------------------------------------------
// Seed tiles of the diagonal's self-pairs (RBF difference seed, order 1; sig_bwd_wide.hip): per pair a,
// over the lane columns j < NC = LP W,
//   [c_ij = <dx_i, dx_j>  (RP x NC)][<dx_i, x_j>  (RP x NC)][anchor rows i = 4 t: k(x_i, x_j), expm1(q_ij) (2 x NC)]
// RP = the cell rows rounded up to 8 (the forward's and the VJP's row chunks), q_ij = <x_i - x_j, dx_j> -
// |dx_j|^2 / 2.  Two batched GEMMs off the wide records and one direct kernel for the anchors replace the
// per-pair channel loops (the chunk dots and the anchors) of the diagonal's N pairs, which run as N waves.
constexpr int DIAG_TILE_ANCHOR = 4;
struct DiagTiles {
  long long rows, ld, pair;  // RP, NC, floats per pair
};
DiagTiles diag_tiles_of(int l, int W, int LP);
bool diag_tiles_apply(int l, int d, int W, int LP, int seed, int order);
int wide_diag_tiles(const float *FX, long long sx, int d, int lw, int a0, int npairs, DiagTiles dt, float *T,
                    hipStream_t s);
// pairs per tile chunk (DIAG_TILE_BYTES of tiles)
constexpr size_t DIAG_TILE_BYTES = (size_t)512 << 20;
inline int diag_tile_pairs(const DiagTiles &dt, int n) {
  long long p = (long long)(DIAG_TILE_BYTES / ((size_t)dt.pair * sizeof(float)));
  if (p < 4) p = 4;
  if (p > 65535) p = 65535;  // the anchor launch's grid z (wide_diag_tiles)
  return (int)(p < n ? p : n);
}

// ---------------------------------------------------------------------------------------------
// RBF difference seed on column pairs, wide channels.  Same cells and recurrences as RbfSeedPk
// (sig_common.h); the dots of R rows come from one channel loop (chunk), the exact rows (anchor and
// slow rows) from another.
template <int W, int R>
struct RbfSeedWide {
  static_assert(W == 2 || W == 4 || W == 8, "columns per lane");
  static constexpr int W2 = W / 2;
  static constexpr int ANCHOR = GPSIG_PK_ANCHOR;
  static constexpr float NHL2E = -0.72134752044448170f;
  static constexpr float L2E = 1.4426950408889634f;
  int d, lw, lwx;  // channel count, record stride of the y (column) and x (row) sequences
  cfloat *fx;         // row side: the x-sequence's record (wave-uniform, scalar loads)
  const float *fyc;   // column side: the y-sequence's record at this lane's first column
  float mlast;        // 0 when the lane's column W-1 is a column block's halo point (no cell)
  f2 hdy[W2];
  f2 Eq[W2], kc[W2];
  float kcR;
  bool valid_last;
  bool clo = false;
  f2 cc[R][W2], pc[R];  // the chunk's c_ij and the pair-0 p_ij
  // seed tiles of the pair (optional, DIAG VJP: wide_diag_tiles): this lane's columns of
  // c_ij = <dx_i, dy_j> (tcc), <dx_i, y_j> (tpp), and per anchor row i = R t the exact k / expm1(q) (tke)
  const float *tcc = nullptr, *tpp = nullptr, *tke = nullptr;
  long long tld = 0;
  int tka = 1, tna = 0;  // anchor rows of the tile: i = tka t, t < tna

  struct Row {
    int i;
    f2 c[W2], p;
  };

  GPSIG_DEV void lcols(const float *base, int k, float (&v)[W]) const { ld_cols<W>(base + (long long)k * lw, v); }

  GPSIG_DEV void init(int d_, int lwx_, int lw_, const float *__restrict__ fxr, const float *__restrict__ fyblk, int gl,
                      int npts) {
    d = d_;
    lw = lw_;
    lwx = lwx_;
    fx = as_const(fxr);
    fyc = fyblk + gl * W;
    const int ncols = npts - 1;
    valid_last = gl * W + W - 1 < ncols;
    mlast = valid_last ? 1.0f : 0.0f;
    const float *h = fyc + (long long)2 * d * lw;
#pragma unroll
    for (int w2 = 0; w2 < W2; ++w2) hdy[w2] = (f2){h[w2], h[w2 + W2] * (w2 == W2 - 1 ? mlast : 1.0f)};
    exact(fx, Eq, kc);
    kcR = lane_next(kc[0][0]);
  }

  GPSIG_DEV void bound_c(int nrows) {
    float hx = 0.0f, hy = 0.0f;
    cfloat *hr = fx + (long long)2 * d * lwx;
    for (int i = (int)__lane_id(); i < nrows; i += 64) hx = __builtin_fmaxf(hx, hr[i]);
#pragma unroll
    for (int w2 = 0; w2 < W2; ++w2) hy = __builtin_fmaxf(hy, __builtin_fmaxf(hdy[w2][0], hdy[w2][1]));
    hx = wave_max(hx);
    hy = wave_max(hy);
    clo = wave_uniform(4.0f * hx * hy < 0.98f * EM1_LO_TAU * EM1_LO_TAU ? 1 : 0) != 0;
  }

  // expm1(q) and k(x, y) of the row whose point is xr[k * lwx] (channel k), from x - y
  GPSIG_DEV void exact(cfloat *xr, f2 (&Eqo)[W2], f2 (&ko)[W2]) const {
    f2 s[W2], qq[W2];
#pragma unroll
    for (int w2 = 0; w2 < W2; ++w2) {
      s[w2] = splat2(0.0f);
      qq[w2] = -hdy[w2];
    }
    const float *yb = fyc, *dyb = fyc + (long long)d * lw;
#pragma unroll 2
    for (int k = 0; k < d; ++k) {
      const float xv = xr[(long long)k * lwx];
      float yv[W], dv[W];
      lcols(yb, k, yv);
      lcols(dyb, k, dv);
      dv[W - 1] *= mlast;
#pragma unroll
      for (int w2 = 0; w2 < W2; ++w2) {
        const f2 df = splat2(xv) - (f2){yv[w2], yv[w2 + W2]};
        s[w2] = fma2(df, df, s[w2]);
        qq[w2] = fma2(df, (f2){dv[w2], dv[w2 + W2]}, qq[w2]);
      }
    }
#pragma unroll
    for (int w2 = 0; w2 < W2; ++w2) {
      const f2 e = s[w2] * splat2(NHL2E);
      Eqo[w2] = em1_small2(qq[w2]);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        ko[w2][h] = __builtin_amdgcn_exp2f(e[h]);
        if (!(__builtin_fabsf(qq[w2][h]) < EM1_TAU)) Eqo[w2][h] = __builtin_amdgcn_exp2f(qq[w2][h] * L2E) - 1.0f;
      }
    }
  }

  GPSIG_DEV void set_tiles(const float *cc, const float *pp, const float *ke, long long ld, int gl, int ka, int na) {
    tcc = cc + gl * W;
    tpp = pp + gl * W;
    tke = ke + gl * W;
    tld = ld;
    tka = ka;
    tna = na;
  }

  // exact k and expm1(q) of anchor row R t from the tile (as exact(fx + R t))
  GPSIG_DEV void exact_tile(int t, f2 (&Eqo)[W2], f2 (&ko)[W2]) const {
    const float *kr = tke + (long long)(2 * t) * tld, *er = kr + tld;
    float kv[W], ev[W];
    ld_cols<W>(kr, kv);
    ld_cols<W>(er, ev);
#pragma unroll
    for (int w2 = 0; w2 < W2; ++w2) {
      ko[w2] = (f2){kv[w2], kv[w2 + W2]};
      Eqo[w2] = (f2){ev[w2], ev[w2 + W2]};
    }
  }

  // chunk() from the tiles
  GPSIG_DEV void chunk_tile(int i0) {
    cfloat *gr = fx + (long long)(2 * d + 1) * lwx + i0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const float *cr = tcc + (long long)(i0 + r) * tld, *pr = tpp + (long long)(i0 + r) * tld;
      float cv[W];
      ld_cols<W>(cr, cv);
      cv[W - 1] *= mlast;
#pragma unroll
      for (int w2 = 0; w2 < W2; ++w2) cc[r][w2] = (f2){cv[w2], cv[w2 + W2]};
      pc[r] = (f2){pr[0], pr[W2]} - splat2(gr[r]);
    }
  }

  // c_ij and the pair-0 p_ij of rows i0 .. i0+R-1 (rows past the sequence read its zero padding)
  GPSIG_DEV void chunk(int i0) {
    cfloat *dxr = fx + (long long)d * lwx + i0;
    cfloat *gr = fx + (long long)(2 * d + 1) * lwx + i0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      pc[r] = splat2(-gr[r]);
#pragma unroll
      for (int w2 = 0; w2 < W2; ++w2) cc[r][w2] = splat2(0.0f);
    }
    const float *yb = fyc, *dyb = fyc + (long long)d * lw;
    for (int k = 0; k < d; ++k) {
      float xr[R];
#pragma unroll
      for (int r = 0; r < R; ++r) xr[r] = dxr[(long long)k * lwx + r];
      float dv[W];
      lcols(dyb, k, dv);
      dv[W - 1] *= mlast;
      const float *yk = yb + (long long)k * lw;
      const f2 y0 = (f2){yk[0], yk[W2]};
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const f2 xs = splat2(xr[r]);
        pc[r] = fma2(y0, xs, pc[r]);
#pragma unroll
        for (int w2 = 0; w2 < W2; ++w2) cc[r][w2] = fma2((f2){dv[w2], dv[w2 + W2]}, xs, cc[r][w2]);
      }
    }
  }

  template <int RR>
  GPSIG_DEV Row row_of(int i) const {
    Row rd;
    rd.i = i;
    rd.p = pc[RR];
#pragma unroll
    for (int w2 = 0; w2 < W2; ++w2) rd.c[w2] = cc[RR][w2];
    return rd;
  }

  GPSIG_DEV void next_exact(const Row &rd, f2 (&Eqo)[W2], f2 (&ko)[W2]) const {
    const int r = rd.i + 1;
    if (tke && r % tka == 0 && r / tka < tna)
      exact_tile(r / tka, Eqo, ko);
    else
      exact(fx + r, Eqo, ko);
  }

  // Cells of row rd.i into dM (RbfSeedPk::row with the chunk's dots).
  template <bool CLO = false>
  GPSIG_DEV void row(const Row &rd, bool anch, f2 (&dM)[W2]) {
    f2 p[W2], c[W2];
#pragma unroll
    for (int w2 = 0; w2 < W2; ++w2) c[w2] = rd.c[w2];
    p[0] = rd.p;
#pragma unroll
    for (int w2 = 1; w2 < W2; ++w2) p[w2] = p[w2 - 1] + c[w2 - 1];
    f2 Ec[W2], Ep[W2];
    if constexpr (CLO)
      em1_lo2_n<W2>(c, Ec);
    else
      em1_small2_n<W2>(c, Ec);
    Ep[0] = em1_small2(p[0]);
    float mx = 0.0f;
#pragma unroll
    for (int w2 = 0; w2 < W2; ++w2) {
      const f2 t = fma2(Ep[w2], Ec[w2], Ec[w2]);
      if (w2 + 1 < W2) Ep[w2 + 1] = Ep[w2] + t;
      const f2 t2 = fma2(Eq[w2], t, t);
      dM[w2] = kc[w2] * fma2(Ep[w2], Eq[w2], t2);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if constexpr (CLO)
          mx = __builtin_fmaxf(mx, __builtin_fabsf(p[w2][h]));
        else
          mx = __builtin_fmaxf(__builtin_fmaxf(mx, __builtin_fabsf(p[w2][h])), __builtin_fabsf(c[w2][h]));
      }
    }
    const bool slow = __builtin_amdgcn_ballot_w64(mx >= EM1_TAU) != 0;
    if (anch || slow) {
      f2 Eqn[W2], kn[W2];
      next_exact(rd, Eqn, kn);
      const float knR = lane_next(kn[0][0]);
      if (slow) {
        f2 Epd[W2], Ecd[W2];
        em1_small2_n<W2>(p, Epd);
        em1_small2_n<W2>(c, Ecd);
#pragma unroll
        for (int w = 0; w < W; ++w) {
          const int w2 = w % W2, h = w / W2;
          const float kn1 = (w + 1 < W) ? kn[(w + 1) % W2][(w + 1) / W2] : knR;
          const float kc1 = (w + 1 < W) ? kc[(w + 1) % W2][(w + 1) / W2] : kcR;
          const float naive = (kn1 - kn[w2][h]) - (kc1 - kc[w2][h]);
          const float m = __builtin_fmaxf(__builtin_fabsf(p[w2][h]), __builtin_fabsf(c[w2][h]));
          float t = __builtin_fmaf(Epd[w2][h], Ecd[w2][h], Ecd[w2][h]);
          t = __builtin_fmaf(Eq[w2][h], t, t);
          const float prod = kc[w2][h] * __builtin_fmaf(Epd[w2][h], Eq[w2][h], t);
          float v = m < EM1_TAU ? prod : naive;
          if (w + 1 == W && !valid_last) v = 0.0f;
          dM[w2][h] = v;
        }
      }
#pragma unroll
      for (int w2 = 0; w2 < W2; ++w2) {
        Eq[w2] = Eqn[w2];
        kc[w2] = kn[w2];
      }
      kcR = knR;
    } else {
#pragma unroll
      for (int w2 = 0; w2 < W2; ++w2) {
        kc[w2] = fma2(kc[w2], Ep[w2], kc[w2]);
        Eq[w2] = fma2(Eq[w2], Ec[w2], Eq[w2] + Ec[w2]);
      }
      kcR = lane_next(kc[0][0]);
    }
  }
};

// ---------------------------------------------------------------------------------------------
// The other seeds, wide channels (one dot per cell, no row state):
//   LIN_DIFF  <dx_i, dy_j>           LIN_POINT  <x_i, y_j>           RBF_POINT  exp(-|x_i - y_j|^2 / 2)
template <int W, int R, int SEED>
struct WideSeedGen {
  static_assert(SEED != SEED_RBF_DIFF, "RbfSeedWide");
  static constexpr int W2 = W / 2;
  static constexpr int ANCHOR = 1 << 30;
  static constexpr bool DIFF = SEED == SEED_LIN_DIFF;
  static constexpr float NHL2E = -0.72134752044448170f;
  int d, lw, lwx;  // channel count, record stride of the y (column) and x (row) sequences
  cfloat *fx;
  const float *fyc;
  f2 msk[W2];   // 1 for the lane's columns that are cells of the grid, 0 otherwise
  f2 cc[R][W2];
  bool clo = false;

  struct Row {
    int i;
    f2 c[W2];
  };

  GPSIG_DEV void lcols(const float *base, int k, float (&v)[W]) const { ld_cols<W>(base + (long long)k * lw, v); }

  GPSIG_DEV void init(int d_, int lwx_, int lw_, const float *__restrict__ fxr, const float *__restrict__ fyblk, int gl,
                      int npts) {
    d = d_;
    lw = lw_;
    lwx = lwx_;
    fx = as_const(fxr);
    fyc = fyblk + gl * W;
    const int ncols = DIFF ? npts - 1 : npts;
#pragma unroll
    for (int w2 = 0; w2 < W2; ++w2)
#pragma unroll
      for (int h = 0; h < 2; ++h) msk[w2][h] = (gl * W + w2 + h * W2 < ncols) ? 1.0f : 0.0f;
  }
  GPSIG_DEV void bound_c(int) {}

  GPSIG_DEV void chunk(int i0) {
    // rows: dx (LIN_DIFF) or x (POINT seeds); columns: dy or y
    cfloat *xr0 = fx + (DIFF ? (long long)d * lwx : 0) + i0;
    const float *yb = fyc + (DIFF ? (long long)d * lw : 0);
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int w2 = 0; w2 < W2; ++w2) cc[r][w2] = splat2(0.0f);
    for (int k = 0; k < d; ++k) {
      float xr[R];
#pragma unroll
      for (int r = 0; r < R; ++r) xr[r] = xr0[(long long)k * lwx + r];
      float yv[W];
      lcols(yb, k, yv);
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int w2 = 0; w2 < W2; ++w2) {
          const f2 yy = (f2){yv[w2], yv[w2 + W2]};
          if constexpr (SEED == SEED_RBF_POINT) {
            const f2 df = splat2(xr[r]) - yy;
            cc[r][w2] = fma2(df, df, cc[r][w2]);
          } else {
            cc[r][w2] = fma2(yy, splat2(xr[r]), cc[r][w2]);
          }
        }
    }
  }

  template <int RR>
  GPSIG_DEV Row row_of(int i) const {
    Row rd;
    rd.i = i;
#pragma unroll
    for (int w2 = 0; w2 < W2; ++w2) rd.c[w2] = cc[RR][w2];
    return rd;
  }

  template <bool CLO = false>
  GPSIG_DEV void row(const Row &rd, bool, f2 (&dM)[W2]) {
#pragma unroll
    for (int w2 = 0; w2 < W2; ++w2) {
      f2 v = rd.c[w2];
      if constexpr (SEED == SEED_RBF_POINT) {
        const f2 e = v * splat2(NHL2E);
        v = (f2){__builtin_amdgcn_exp2f(e[0]), __builtin_amdgcn_exp2f(e[1])};
      }
      dM[w2] = v * msk[w2];
    }
  }
};

template <int W, int R, int SEED>
using WideSeed = std::conditional_t<SEED == SEED_RBF_DIFF, RbfSeedWide<W, R>, WideSeedGen<W, R, SEED>>;

// Level 1 in closed form (level1_closed, sig_common.h) on the wide records.
template <int SEED>
GPSIG_DEV float level1_closed_wide(const float *__restrict__ fx, const float *__restrict__ fy, int d, int lw1,
                                   int lw2, int l1, int l2) {
  double s00 = 0.0, s0l = 0.0, sl0 = 0.0, sll = 0.0, lin = 0.0;
  for (int k = 0; k < d; ++k) {
    const double x0 = fx[(long long)k * lw1], xl = fx[(long long)k * lw1 + l1 - 1];
    const double y0 = fy[(long long)k * lw2], yl = fy[(long long)k * lw2 + l2 - 1];
    if constexpr (SEED == SEED_RBF_DIFF) {
      s00 = __builtin_fma(x0 - y0, x0 - y0, s00);
      s0l = __builtin_fma(x0 - yl, x0 - yl, s0l);
      sl0 = __builtin_fma(xl - y0, xl - y0, sl0);
      sll = __builtin_fma(xl - yl, xl - yl, sll);
    } else {
      lin = __builtin_fma(xl - x0, yl - y0, lin);
    }
  }
  if constexpr (SEED == SEED_RBF_DIFF)
    return (float)((exp(-0.5 * sll) - exp(-0.5 * sl0)) - (exp(-0.5 * s0l) - exp(-0.5 * s00)));
  else
    return (float)lin;
}

}  // namespace gpsig
