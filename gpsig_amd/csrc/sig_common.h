// gpsig_amd -- pieces shared by the truncated-signature kernels (first order, higher order):
// the per-point feature layout, the pair-tile scheduler, the fused normalisation epilogue and the
// per-row seed (base-kernel second difference).
#pragma once
#include "common.h"

namespace gpsig {

// Per-point feature record, FS floats (16-byte aligned): [x (DP) | dx (DP) | |dx|^2/2 | g | pad...]
// dx_i = x_{i+1} - x_i (zero for the last point), g_i = <x_i, dx_i> + |dx_i|^2/2 (2*DP+1 is odd, so
// the record always has this slot).  DP = padded channel count of the instantiation.
__host__ __device__ constexpr int feat_stride(int DP) { return ((2 * DP + 1) + 3) & ~3; }

enum Seed : int {
  SEED_RBF_DIFF = 0,    // stable/naive hybrid second difference of exp(-|x-y|^2/2)
  SEED_LIN_DIFF = 1,    // <dx_i, dy_j>
  SEED_RBF_POINT = 2,   // exp(-|x_i-y_j|^2/2)  (difference=False)
  SEED_LIN_POINT = 3    // <x_i, y_j>           (difference=False)
};

struct SigArgs {
  const float *FX, *FY;  // feature records (n1,l1,FS), (n2,l2,FS)
  int n1, l1, n2, l2;
  int fs;                // feature stride in floats
  int M;                 // num_levels
  int order;
  int pair_mode, row_begin, row_end;
  int tiles_a0;          // first A-tile row of this launch (UPPER/RECT)
  int ntb;               // number of B tiles (RECT) / B-tile count per full row (UPPER)
  long long tile_base;   // UPPER: prefix count of tiles before tiles_a0
  const float *rs1, *rs2, *scale;
  float jitter;
  int out_mode;
  float *out;
  int out_row0, out_rows;
  long long out_ld, out_lvl;  // row stride, level stride (elements)
  float *state;               // optional saved forward state for the VJP (gpsig_sig_gram_state)
  int mfma;                   // RBF difference seed: increment dots on the matrix cores (GPSIG_BASE_SEED_MFMA)
  int nblk;                   // column blocks per pair (first order, LP = 64; 1 = unblocked)
  // split diagnostic (GPSIG_GRAM_SPLIT): a producer launch writes each pair's cells dM to
  // dmbuf, a consumer launch streams them through the recursion; blk0 = first logical workgroup of a
  // chunked launch, dmbuf slot of a pair = its workgroup-local index
  float *dmbuf;
  long long blk0;
  // wide channel counts (DP == 0 instantiations, wide.h): channel count, padded record lengths and
  // record strides (floats) of X and Y
  int wd, lw1, lw2;
  long long sx, sy;
  // higher order past the fixed channel counts (linear base kernel, sig_ho.hip): the cells of pair
  // (a, b), row i, column j at tile + (a - tile_a0) tile_as + (b - tile_b0) (l2 - 1) + i tile_ld + j (DIAG:
  // without the b term), a GEMM of the increments; RX / RY the raw (n, l, wd) inputs (level 1 closed form)
  const float *tile;
  long long tile_as, tile_ld;
  int tile_a0, tile_b0;
  const float *RX, *RY;
  int tile_rbf;  // the tile holds RBF difference-seed cells (level 1 closed form of the RBF kernel)
  // DIAG seed tiles of the wide forward (wide.h DiagTiles): pair a at dtile + (a - dt_a0) dt_pair
  const float *dtile;
  int dt_a0;
  long long dt_pair, dt_rows, dt_ld;
};

// Saved forward state of a first-order pair (gpsig_sig_gram_state): column sums of levels 1..M-1
// after the last row ((M-1) x (l2-1) floats, level-major), then the raw levels K_1..K_M.
__host__ __device__ inline long long state_stride(int M, int l2) { return (long long)(M - 1) * (l2 - 1) + M; }
__host__ __device__ inline long long state_slot(int a, int b, int n2, bool upper) {
  return upper ? (long long)a * n2 - (long long)a * (a - 1) / 2 + (b - a) : (long long)a * n2 + b;
}

// Wave-uniform record of row i: x_{i+1} (RBF DIFF) or x_i (POINT seeds), dx_i, |dx_i|^2/2.
template <int DP>
struct RowData {
  float x[DP], dx[DP], hdx, g;
  GPSIG_DEV void load(const float *__restrict__ fx, int i, int seed) {
    constexpr int FS = feat_stride(DP);
    const float *__restrict__ fr = fx + (long long)i * FS;
    const float *__restrict__ fp = (seed == SEED_RBF_DIFF) ? fr + FS : fr;
#pragma unroll
    for (int k = 0; k < DP; ++k) {
      x[k] = fp[k];
      dx[k] = fr[DP + k];
    }
    hdx = fr[2 * DP];
    g = fr[2 * DP + 1];
  }
};

// ---------------------------------------------------------------------------------------------
// Per-row seed of the recursion: the W cells dM(i, j), j = gl*W + w, of row i of the grid the
// recursion consumes (signature_algs.py:26 for the DIFF seeds, the raw base-kernel grid otherwise).
// The lane's column data (y_j, dy_j, |dy_j|^2/2) is loaded once per pair; the row data (x_i, dx_i,
// |dx_i|^2/2, x_{i+1}) is wave-uniform and read through the scalar cache.
//
// RBF DIFF: dM = k11 - k10 - k01 + k00 with k = exp(-|x-y|^2/2).  That difference cancels
// catastrophically in fp32 for small increments, so it is evaluated as
//     dM = k00 (em1(p) em1(q) + e^p e^q em1(c)),
//     p = -<x_i - y_j, dx_i> - |dx_i|^2/2,  q = <x_i - y_j, dy_j> - |dy_j|^2/2,  c = <dx_i, dy_j>
// when |p|,|q|,|c| < EM1_TAU (em1 = minimax polynomial), and as the plain corner difference of the
// directly evaluated k grid otherwise (large increments: corners far apart, the product form would
// lose more through exponent-space rounding).  k on row i+1 is evaluated once and reused as the
// next row's k00 / k01 (right neighbour through DPP), so the grid costs one exp per cell.
template <int DP, int W, int SEED>
struct RowSeed {
  static constexpr int FS = feat_stride(DP);
  static constexpr bool DIFF = (SEED == SEED_RBF_DIFF || SEED == SEED_LIN_DIFF);
#ifndef GPSIG_D2_RECUR
#define GPSIG_D2_RECUR 1
#endif
  static constexpr int ANCHOR = 8;  // exact |x_i - y_j|^2 every ANCHOR rows (d^2 row recurrence between)
  static constexpr float NHL2E = -0.72134752044448170f;  // -log2(e)/2: exp(-d2/2) = exp2(d2 * NHL2E)
  float y[W][DP], dy[W][DP], hdy[W];
  bool valid_last;  // column W-1 of this lane is a real cell (others: exact zeros by construction)
  bool valid[W];    // POINT seeds
  // RBF_DIFF row state: diff = x_i - y_j, d2 = |diff|^2, kc = k(x_i, y_j), kcR = next lane's kc[0]
  float diff[W][DP], d2[W], kc[W], kcR;

  GPSIG_DEV void init(const float *__restrict__ fx, const float *__restrict__ fy, int gl, int l2) {
    const int ncols = DIFF ? l2 - 1 : l2;
    // Points beyond the sequence are clamped to its last point, whose increment record is zero, so
    // every DIFF-seed cell of a padded column evaluates to exactly 0 (both the stable and the corner
    // form); only the lane's last column can see a foreign right neighbour and is masked.
#pragma unroll
    for (int w = 0; w < W; ++w) {
      const int j = gl * W + w;
      valid[w] = j < ncols;
      const int jj = j < l2 ? j : l2 - 1;
      const float *f = fy + (long long)jj * FS;
#pragma unroll
      for (int k = 0; k < DP; ++k) {
        y[w][k] = f[k];
        dy[w][k] = f[DP + k];
      }
      hdy[w] = f[2 * DP];
    }
    valid_last = valid[W - 1];
    if constexpr (SEED == SEED_RBF_DIFF) {
#pragma unroll
      for (int w = 0; w < W; ++w) {
        float s = 0.0f;
#pragma unroll
        for (int k = 0; k < DP; ++k) {
          diff[w][k] = fx[k] - y[w][k];
          s = __builtin_fmaf(diff[w][k], diff[w][k], s);
        }
        d2[w] = s;
        kc[w] = __builtin_amdgcn_exp2f(s * NHL2E);
      }
      kcR = lane_next(kc[0]);
    }
  }

  // Cells of row i.  rd = wave-uniform record of row i (x_{i+1} for RBF DIFF, x_i for POINT seeds).
  // ANCH: re-evaluate |x_{i+1} - y_j|^2 exactly instead of the d2 - 2p recurrence.
  template <bool ANCH>
  GPSIG_DEV void row(const RowData<DP> &rd, float (&dM)[W]) {
    if constexpr (SEED == SEED_RBF_DIFF) {
      // 1) p, q, c from the current diff = x_i - y_j (consumed before diff is overwritten)
      float pp[W], q[W], c[W];
#pragma unroll
      for (int w = 0; w < W; ++w) {
        float a = -rd.hdx, bq = -hdy[w], cc = 0.0f;
#pragma unroll
        for (int k = 0; k < DP; ++k) {
          a = __builtin_fmaf(-diff[w][k], rd.dx[k], a);
          bq = __builtin_fmaf(diff[w][k], dy[w][k], bq);
          cc = __builtin_fmaf(rd.dx[k], dy[w][k], cc);
        }
        pp[w] = a;
        q[w] = bq;
        c[w] = cc;
      }
      // 2) next row: diff = x_{i+1} - y_j, |diff|^2 = d2 - 2p (exact re-anchor every ANCHOR rows)
      float kn[W];
#pragma unroll
      for (int w = 0; w < W; ++w) {
        float s = 0.0f;
#pragma unroll
        for (int k = 0; k < DP; ++k) {
          diff[w][k] = rd.x[k] - y[w][k];
          if constexpr (ANCH || !GPSIG_D2_RECUR) s = __builtin_fmaf(diff[w][k], diff[w][k], s);
        }
        d2[w] = (ANCH || !GPSIG_D2_RECUR) ? s : __builtin_fmaf(-2.0f, pp[w], d2[w]);
        kn[w] = __builtin_amdgcn_exp2f(d2[w] * NHL2E);
      }
      const float knR = lane_next(kn[0]);
      // 3) the cells
#pragma unroll
      for (int w = 0; w < W; ++w) {
        const float kn1 = (w + 1 < W) ? kn[w + 1] : knR;
        const float kc1 = (w + 1 < W) ? kc[w + 1] : kcR;
        const float naive = (kn1 - kn[w]) - (kc1 - kc[w]);
        const float Ep = em1_small(pp[w]), Eq = em1_small(q[w]), Ec = em1_small(c[w]);
        const float stable = kc[w] * __builtin_fmaf(Ep, Eq, (1.0f + Ep) * (1.0f + Eq) * Ec);
        const float mx = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(pp[w]), __builtin_fabsf(q[w])),
                                         __builtin_fabsf(c[w]));
        const float v = mx < EM1_TAU ? stable : naive;
        dM[w] = (w + 1 < W || valid_last) ? v : 0.0f;
      }
#pragma unroll
      for (int w = 0; w < W; ++w) kc[w] = kn[w];
      kcR = knR;
    } else if constexpr (SEED == SEED_LIN_DIFF) {
#pragma unroll
      for (int w = 0; w < W; ++w) {
        float c = 0.0f;
#pragma unroll
        for (int k = 0; k < DP; ++k) c = __builtin_fmaf(rd.dx[k], dy[w][k], c);
        dM[w] = (w + 1 < W || valid_last) ? c : 0.0f;  // padded columns have dy == 0; the halo cell of a block is masked
      }
    } else if constexpr (SEED == SEED_RBF_POINT) {
#pragma unroll
      for (int w = 0; w < W; ++w) {
        float s = 0.0f;
#pragma unroll
        for (int k = 0; k < DP; ++k) {
          const float t = rd.x[k] - y[w][k];
          s = __builtin_fmaf(t, t, s);
        }
        dM[w] = valid[w] ? __builtin_amdgcn_exp2f(s * NHL2E) : 0.0f;
      }
    } else {
#pragma unroll
      for (int w = 0; w < W; ++w) {
        float c = 0.0f;
#pragma unroll
        for (int k = 0; k < DP; ++k) c = __builtin_fmaf(rd.x[k], y[w][k], c);
        dM[w] = valid[w] ? c : 0.0f;
      }
    }
  }
};

// ---------------------------------------------------------------------------------------------
// RBF DIFF seed on column pairs (first-order kernel; W even).  Same cells as RowSeed<.., RBF_DIFF>,
// with the per-row work cut to what the recursion needs and laid out for v_pk_* instructions.
// With p_ij = <y_j, dx_i> - g_i (g_i from the feature record), c_ij = <dx_i, dy_j> and
// q_ij = <x_i - y_j, dy_j> - |dy_j|^2/2, the cell is k(x_i,y_j) (Ep Eq + (1 + Ep)(1 + Eq) Ec),
// E* = expm1(*), and both row-to-row quantities follow from what the cell already computed:
//   k(x_{i+1}, y_j) = k(x_i, y_j) (1 + Ep_ij)          q_{i+1,j} = q_ij + c_ij
//   Eq_{i+1,j} = Eq_ij + Ec_ij + Eq_ij Ec_ij           (= expm1(q_ij + c_ij), no cancellation)
// so a row costs two packed dots, two polynomial expm1 (p, c) and a few FMAs per column pair: no
// exp.  k and Eq are re-evaluated exactly from x_{i+1} - y_j on anchor rows (every ANCHOR rows), so
// rounding drift is bounded by ANCHOR steps.  When |p| or |c| of some cell of the wave reaches
// EM1_TAU (a wave-uniform branch), the next row is evaluated exactly and those cells take the plain
// corner difference of the k grid.
#ifndef GPSIG_NAIVE
#define GPSIG_NAIVE 1
#endif
#ifndef GPSIG_P0CHECK
#define GPSIG_P0CHECK 1
#endif
template <int DP, int W>
struct RbfSeedPk {
  static_assert(W % 2 == 0, "column pairs");
  static constexpr int W2 = W / 2;
  static constexpr int FS = feat_stride(DP);
#ifndef GPSIG_PK_ANCHOR
#define GPSIG_PK_ANCHOR 128
#endif
  static constexpr int ANCHOR = GPSIG_PK_ANCHOR;
  static constexpr float NHL2E = -0.72134752044448170f;  // exp(-d2/2) = exp2(d2 * NHL2E)
  static constexpr float L2E = 1.4426950408889634f;
  // Wide channels (DP >= GPSIG_YG_DP): only column pair 0's points stay in registers (the rows' p dots
  // need them, the other pairs' p follow by the column recurrence); the others are needed only on
  // anchor and slow rows (exact) and are re-read from the records there.  This keeps W = 8 columns per
  // lane within 256 VGPRs at D = 6..8.
#ifndef GPSIG_YG_DP
#define GPSIG_YG_DP 6
#endif
  // (W = 10, the 10-lane groups: also at any DP, to stay within 256 VGPRs)
  static constexpr bool YG = DP >= GPSIG_YG_DP || W > 8;
  static constexpr int YR = YG ? 1 : W2;
  f2 y[YR][DP], dy[W2][DP], hdy[W2];
  f2 Eq[W2], kc[W2];  // expm1(q_ij), k(x_i, y_j)
  float kcR;          // next lane's kc of its first column
  bool valid_last;
  bool clo = false;   // every |c_ij| of the wave < EM1_LO_TAU: Ec by the cubic (bound_c)
  const float *fyb;   // YG: the block's point records, this lane's first column, the last point
  int jl0, jlast;

  // point y_j of column pair w2 (both halves), channel k
  GPSIG_DEV f2 yv(int w2, int k) const {
    if (!YG || w2 < YR) return y[w2 < YR ? w2 : 0][k];
    f2 v;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int j = jl0 + w2 + h * W2;
      v[h] = fyb[(long long)(j < jlast ? j : jlast) * FS + k];
    }
    return v;
  }
  GPSIG_DEV void init(const float *__restrict__ fx, const float *__restrict__ fy, int gl, int l2) {
    const int ncols = l2 - 1;
    fyb = fy;
    jl0 = gl * W;
    jlast = l2 - 1;
    // columns past the sequence clamp to its last point (zero increment): their cells are exact
    // zeros in the product form; only the lane's last column can see a foreign right neighbour.
    // l2 = points of this column block (its last one the halo point when the block is not the last)
#pragma unroll
    for (int w2 = 0; w2 < W2; ++w2)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int j = gl * W + w2 + h * W2;  // pair w2 = columns (w2, w2 + W/2) of the lane
        const int jj = j < l2 ? j : l2 - 1;
        const float *f = fy + (long long)jj * FS;
        // a column with no cell (past the sequence, or the right halo point of a column block) gets a
        // zero increment, so its product-form cell is exactly 0
        const bool cell = j < ncols;
#pragma unroll
        for (int k = 0; k < DP; ++k) {
          if (w2 < YR) y[w2 < YR ? w2 : 0][k][h] = f[k];
          dy[w2][k][h] = cell ? f[DP + k] : 0.0f;
        }
        hdy[w2][h] = cell ? f[2 * DP] : 0.0f;
        if (w2 == W2 - 1 && h == 1) valid_last = j < ncols;
      }
    float x0[DP];
#pragma unroll
    for (int k = 0; k < DP; ++k) x0[k] = fx[k];
    exact(x0, Eq, kc);
    kcR = lane_next(kc[0][0]);
  }

  // |c_ij| = |<dx_i, dy_j>| <= 2 sqrt(hdx_i hdy_j) (Cauchy-Schwarz on the records' |d|^2/2): when the
  // bound over all rows of x and all columns of the wave stays below EM1_LO_TAU (with margin for the
  // records' rounding), every Ec of the pair block takes the cubic (wave-uniform, once per block).
  GPSIG_DEV void bound_c(const float *__restrict__ fx, int nrows) {
    float hx = 0.0f, hy = 0.0f;
    for (int i = (int)__lane_id(); i < nrows; i += 64) hx = __builtin_fmaxf(hx, fx[(long long)i * FS + 2 * DP]);
#pragma unroll
    for (int w2 = 0; w2 < W2; ++w2) hy = __builtin_fmaxf(hy, __builtin_fmaxf(hdy[w2][0], hdy[w2][1]));
    hx = wave_max(hx);
    hy = wave_max(hy);
    clo = wave_uniform(4.0f * hx * hy < 0.98f * EM1_LO_TAU * EM1_LO_TAU ? 1 : 0) != 0;
  }

  // expm1(q) and k(x, y) of the row with point x, evaluated from x - y
  GPSIG_DEV void exact(const float (&x)[DP], f2 (&Eqo)[W2], f2 (&ko)[W2]) const {
#pragma unroll
    for (int w2 = 0; w2 < W2; ++w2) {
      f2 s = splat2(0.0f), qq = -hdy[w2];
#pragma unroll
      for (int k = 0; k < DP; ++k) {
        const f2 df = splat2(x[k]) - yv(w2, k);
        s = fma2(df, df, s);
        qq = fma2(df, dy[w2][k], qq);
      }
      s = s * splat2(NHL2E);
      Eqo[w2] = em1_small2(qq);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        ko[w2][h] = __builtin_amdgcn_exp2f(s[h]);
        // outside the polynomial range expm1(q) = e^q - 1 loses nothing that matters
        if (!(__builtin_fabsf(qq[h]) < EM1_TAU)) Eqo[w2][h] = __builtin_amdgcn_exp2f(qq[h] * L2E) - 1.0f;
      }
    }
  }

  // Wave-uniform part of row i's record the recurrences need (x_{i+1} is read only on anchor rows
  // and slow rows, straight from the record).
  struct Row {
    float dx[DP], g;
    const float *fr;  // record of row i; x_{i+1} = fr[FS .. FS + DP)
    GPSIG_DEV void load(const float *__restrict__ fx, int i) {
      fr = fx + (long long)i * FS;
#pragma unroll
      for (int k = 0; k < DP; ++k) dx[k] = fr[DP + k];
      g = fr[2 * DP + 1];
    }
  };

  GPSIG_DEV void next_exact(const Row &rd, f2 (&Eqo)[W2], f2 (&ko)[W2]) const {
    float x1[DP];
#pragma unroll
    for (int k = 0; k < DP; ++k) x1[k] = rd.fr[FS + k];
    exact(x1, Eqo, ko);
  }

  // Cells of row i into dM.  anch (wave-uniform): the next row's state is re-evaluated exactly
  // instead of by the recurrences.
  //
  // Column recurrence of the p side: p_{i,j+1} - p_ij = <y_{j+1} - y_j, dx_i> = c_ij, so
  //   p_{i,j+1} = p_ij + c_ij,   Ep_{i,j+1} = expm1(p_ij + c_ij) = Ep_ij + (1 + Ep_ij) Ec_ij
  // and (1 + Ep) Ec is a term the cell needs anyway.  Only column pair 0 (the lane's columns 0 and
  // W/2) takes the dot and the polynomial; pairs 1 .. W/2-1 follow in-lane (two operations each instead
  // of D + 6).  Rows with a cell outside the polynomial range re-evaluate every Ep directly (slow path).
#ifndef GPSIG_PCHAIN
#define GPSIG_PCHAIN 1
#endif
  // CLO: the pair block's |c| bound holds (bound_c): Ec by the cubic, and only |p| is range-checked.
  template <bool CLO = false>
  GPSIG_DEV void row(const Row &rd, bool anch, f2 (&dM)[W2]) {
    f2 p[W2], c[W2];
    if constexpr (!GPSIG_PCHAIN) {  // A/B arm: every pair's dots and polynomials evaluated directly
#pragma unroll
      for (int w2 = 0; w2 < W2; ++w2) {
        f2 a = splat2(-rd.g), cc = splat2(0.0f);
#pragma unroll
        for (int k = 0; k < DP; ++k) {
          a = fma2(yv(w2, k), splat2(rd.dx[k]), a);
          cc = fma2(dy[w2][k], splat2(rd.dx[k]), cc);
        }
        p[w2] = a;
        c[w2] = cc;
      }
      row_pc(rd, anch, p, c, dM);
      return;
    }
#pragma unroll
    for (int w2 = 0; w2 < W2; ++w2) {
      f2 cc = dy[w2][0] * splat2(rd.dx[0]);
#pragma unroll
      for (int k = 1; k < DP; ++k) cc = fma2(dy[w2][k], splat2(rd.dx[k]), cc);
      c[w2] = cc;
    }
    {
      f2 a = splat2(-rd.g);
#pragma unroll
      for (int k = 0; k < DP; ++k) a = fma2(y[0][k], splat2(rd.dx[k]), a);
      p[0] = a;
    }
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
      const f2 t = fma2(Ep[w2], Ec[w2], Ec[w2]);  // (1 + Ep) Ec
      if (w2 + 1 < W2) Ep[w2 + 1] = Ep[w2] + t;
      const f2 t2 = fma2(Eq[w2], t, t);
      dM[w2] = kc[w2] * fma2(Ep[w2], Eq[w2], t2);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        // CLO: every Ec is in the cubic's range a priori, and the pairs after the first take Ep by the exact
        // chain Ep' = Ep + (1 + Ep) Ec, so only the first pair's p meets a polynomial
        if constexpr (CLO) {
          if (w2 == 0 || !GPSIG_P0CHECK) mx = __builtin_fmaxf(mx, __builtin_fabsf(p[w2][h]));
        } else {
          mx = __builtin_fmaxf(__builtin_fmaxf(mx, __builtin_fabsf(p[w2][h])), __builtin_fabsf(c[w2][h]));
        }
      }
    }
    const bool slow = GPSIG_NAIVE && __builtin_amdgcn_ballot_w64(mx >= EM1_TAU) != 0;
    if (anch || slow) {
      f2 Eqn[W2], kn[W2];
      next_exact(rd, Eqn, kn);
      const float knR = lane_next(kn[0][0]);
      if (slow) {
        // a cell outside the polynomial range may have spoilt the chained Ep of the pairs after it:
        // every in-range cell is re-evaluated from its own p, the others take the corner difference
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
      // row-to-row recurrences in place (the cells above were the last readers of kc and Eq)
#pragma unroll
      for (int w2 = 0; w2 < W2; ++w2) {
        kc[w2] = fma2(kc[w2], Ep[w2], kc[w2]);
        Eq[w2] = fma2(Eq[w2], Ec[w2], Eq[w2] + Ec[w2]);
      }
      kcR = lane_next(kc[0][0]);
    }
  }

  // The increment inner products of 4 consecutive rows i0 .. i0+3 on the matrix cores
  // (v_mfma_f32_4x4x1_16b_f32: 16 blocks of 4 x 4 outer products, one k per instruction).  Block b of
  // the wave is lanes 4b .. 4b+3; the A operand of lane l is row i0 + (l & 3), the B operand is the
  // lane's own column, and accumulator register r of lane l receives row i0 + r of column l:
  //   P[w][r] = <y_j, dx_{i0+r}> - g_{i0+r},   Q[w][r] = <dy_j, dx_{i0+r}>,   j = column w of the lane
  // (k-ordered fp32 fma chains, as the VALU dots).  The seed GEMM of the reference (kernels.py:946-957
  // _square_dist -> tf.matmul) restricted to what the recursion consumes.
  GPSIG_DEV void mfma_pc(const float *__restrict__ fx, int i0, f4 (&P)[W], f4 (&Q)[W]) const {
    const float *__restrict__ fa = fx + (long long)(i0 + (int)(__lane_id() & 3)) * FS;
    float ax[DP];
#pragma unroll
    for (int k = 0; k < DP; ++k) ax[k] = fa[DP + k];
    const float ng = -fa[2 * DP + 1];
    const f4 zero = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int w = 0; w < W; ++w) {
      const int w2 = w % W2, h = w / W2;
      f4 accp = __builtin_amdgcn_mfma_f32_4x4x1f32(ng, 1.0f, zero, 0, 0, 0);
      f4 accq = __builtin_amdgcn_mfma_f32_4x4x1f32(ax[0], dy[w2][0][h], zero, 0, 0, 0);
#pragma unroll
      for (int k = 0; k < DP; ++k) accp = __builtin_amdgcn_mfma_f32_4x4x1f32(ax[k], yv(w2, k)[h], accp, 0, 0, 0);
#pragma unroll
      for (int k = 1; k < DP; ++k) accq = __builtin_amdgcn_mfma_f32_4x4x1f32(ax[k], dy[w2][k][h], accq, 0, 0, 0);
      P[w] = accp;
      Q[w] = accq;
    }
  }

  // Cells of row i from its precomputed p, c (column pairs).
  GPSIG_DEV void row_pc(const Row &rd, bool anch, const f2 (&p)[W2], const f2 (&c)[W2], f2 (&dM)[W2]) {
    f2 Eqn[W2], kn[W2];
    f2 Ep[W2], Ec[W2];
    em1_small2_n<W2>(p, Ep);
    em1_small2_n<W2>(c, Ec);
    float mx = 0.0f;
#pragma unroll
    for (int w2 = 0; w2 < W2; ++w2) {
      f2 t = fma2(Ep[w2], Ec[w2], Ec[w2]);
      t = fma2(Eq[w2], t, t);
      dM[w2] = kc[w2] * fma2(Ep[w2], Eq[w2], t);
      kn[w2] = fma2(kc[w2], Ep[w2], kc[w2]);
      Eqn[w2] = fma2(Eq[w2], Ec[w2], Eq[w2] + Ec[w2]);
#pragma unroll
      for (int h = 0; h < 2; ++h) mx = __builtin_fmaxf(__builtin_fmaxf(mx, __builtin_fabsf(p[w2][h])), __builtin_fabsf(c[w2][h]));
    }
    const bool slow = GPSIG_NAIVE && __builtin_amdgcn_ballot_w64(mx >= EM1_TAU) != 0;
    if (anch || slow) next_exact(rd, Eqn, kn);
    const float knR = lane_next(kn[0][0]);
    if (slow) {
      // corner difference k11 - k10 - k01 + k00 for the cells outside the polynomial range
#pragma unroll
      for (int w = 0; w < W; ++w) {
        const int w2 = w % W2, h = w / W2;
        const float kn1 = (w + 1 < W) ? kn[(w + 1) % W2][(w + 1) / W2] : knR;
        const float kc1 = (w + 1 < W) ? kc[(w + 1) % W2][(w + 1) / W2] : kcR;
        const float naive = (kn1 - kn[w2][h]) - (kc1 - kc[w2][h]);
        const float m = __builtin_fmaxf(__builtin_fabsf(p[w2][h]), __builtin_fabsf(c[w2][h]));
        float v = m < EM1_TAU ? dM[w2][h] : naive;
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
  }
};

// ---------------------------------------------------------------------------------------------
// Level 1 of a DIFF seed in closed form.  K_1 = sum_ij dM_ij telescopes to the corner difference
// k(x_L, y_L) - k(x_L, y_0) - k(x_0, y_L) + k(x_0, y_0) (linear: <x_L - x_0, y_L - y_0>), evaluated
// once per pair in fp64.  The fp32 row sums of dM cancel down to K_1 and lose ~1e-7 of sum|dM|,
// which is the whole error budget when K_1 is small against the cells (K_1 feeds only level 1).
template <int DP, int SEED>
GPSIG_DEV float level1_closed(const float *__restrict__ fx, const float *__restrict__ fy, int l1, int l2) {
  constexpr int FS = feat_stride(DP);
  const float *x0 = fx, *xl = fx + (long long)(l1 - 1) * FS;
  const float *y0 = fy, *yl = fy + (long long)(l2 - 1) * FS;
  if constexpr (SEED == SEED_RBF_DIFF) {
    auto k = [](const float *a, const float *b) {
      double s = 0.0;
#pragma unroll
      for (int c = 0; c < DP; ++c) {
        const double d = (double)a[c] - (double)b[c];
        s = __builtin_fma(d, d, s);
      }
      return exp(-0.5 * s);
    };
    return (float)((k(xl, yl) - k(xl, y0)) - (k(x0, yl) - k(x0, y0)));
  } else {
    double s = 0.0;
#pragma unroll
    for (int c = 0; c < DP; ++c) s = __builtin_fma((double)xl[c] - (double)x0[c], (double)yl[c] - (double)y0[c], s);
    return (float)s;
  }
}

// ---------------------------------------------------------------------------------------------
// Tile scheduler.  A workgroup = 4 waves; wave w takes sequence a = 4*ta + w; the wave's G = 64/LP
// lane groups take b = G*tb + g.  UPPER enumerates only tiles with some b >= a: with k = 4/G,
// tile row ta has ntb - k*ta tiles, prefix P(r) = r*ntb - k*r*(r-1)/2, inverted in closed form.
struct Tile { int ta, tb; };

// sum_{i < n} floor((a i + b) / m), n, m > 0, a, b >= 0 (Euclid-like reduction, O(log m) steps)
__host__ __device__ inline long long floor_sum(long long n, long long m, long long a, long long b) {
  long long ans = 0;
  while (true) {
    if (a >= m) {
      ans += (n - 1) * n / 2 * (a / m);
      a %= m;
    }
    if (b >= m) {
      ans += n * (b / m);
      b %= m;
    }
    const long long y = a * n + b;
    if (y < m) break;
    n = y / m;
    b = y % m;
    const long long t = m;
    m = a;
    a = t;
  }
  return ans;
}
// Tiles of the upper triangle when a tile row (4 sequences a) is not a whole number of B tiles (G = 6
// sequences b per wave, LP = 10): tile row r begins at B tile floor(4 r / G) (the first holding some
// b >= 4 r), so P(r) = r ntb - sum_{t < r} floor(4 t / G).
__host__ __device__ inline long long upper_prefix_g(long long r, long long ntb, int G) {
  return r * ntb - floor_sum(r, G, 4, 0);
}
// The same prefix with G a compile-time constant (the kernel's tile decoder: no runtime division).
// With p / q = 4 / G in lowest terms and r = q Q + R, floor(p (q u + v) / q) = p u + floor(p v / q), so
// sum_{t<r} floor(4t/G) = p q Q (Q-1)/2 + Q S + p Q R + sum_{v<R} floor(p v / q), S = sum_{v<q} floor(p v / q).
template <int G>
__host__ __device__ inline long long upper_prefix_c(long long r, long long ntb) {
  constexpr int gg = G % 4 == 0 ? 4 : (G % 2 == 0 ? 2 : 1);
  constexpr long long p = 4 / gg, q = G / gg;
  long long S = 0;
  for (long long v = 0; v < q; ++v) S += p * v / q;
  const long long Q = r / q, R = r % q;
  long long part = 0;
  for (long long v = 0; v < R; ++v) part += p * v / q;
  return r * ntb - (p * q * Q * (Q - 1) / 2 + Q * S + p * Q * R + part);
}
template <int G>
GPSIG_DEV Tile upper_tile_g(long long t, int ntb) {
  // continuous estimate: sum_{t<r} floor(4t/G) ~ (2/G) r (r - 1) - r (q - 1) / (2q), q = G / gcd(4, G)
  // (the fractional parts average (q-1)/(2q)), so the exact prefixes correct it by a step or two
  constexpr int q = G / (G % 4 == 0 ? 4 : (G % 2 == 0 ? 2 : 1));
  const double A = 2.0 / G, B = ntb + 2.0 / G + (q - 1) / (2.0 * q);
  double disc = B * B - 4.0 * A * (double)t;
  disc = disc < 0 ? 0 : disc;
  long long r = (long long)((B - __builtin_sqrt(disc)) / (2.0 * A));
  if (r < 0) r = 0;
  while (r > 0 && upper_prefix_c<G>(r, ntb) > t) --r;
  while (upper_prefix_c<G>(r + 1, ntb) <= t) ++r;
  Tile tl;
  tl.ta = (int)r;
  tl.tb = (int)(4 * r / G + (t - upper_prefix_c<G>(r, ntb)));
  return tl;
}

GPSIG_DEV Tile upper_tile(long long t, int ntb, int k) {
  // largest r with P(r) <= t
  const double A = 0.5 * k, B = ntb + 0.5 * k;
  double disc = B * B - 4.0 * A * (double)t;
  disc = disc < 0 ? 0 : disc;
  long long r = (long long)((B - __builtin_sqrt(disc)) / (2.0 * A));
  if (r < 0) r = 0;
  auto P = [&](long long rr) { return rr * (long long)ntb - (long long)k * rr * (rr - 1) / 2; };
  while (r > 0 && P(r) > t) --r;
  while (P(r + 1) <= t) ++r;
  Tile tl;
  tl.ta = (int)r;
  tl.tb = (int)(k * r + (t - P(r)));
  return tl;
}

// ---------------------------------------------------------------------------------------------
// Epilogue: levels K_1..K_M (K_0 = 1) of pair (a, b) are in lane 0 of the pair's lane group.
template <int MMAX>
GPSIG_DEV void store_pair(const SigArgs &p, int a, int b, const float (&K)[MMAX + 1]) {
  const int M = p.M;
  const bool diag_mode = p.pair_mode == GPSIG_PAIRS_DIAG;
  if (diag_mode) {
    for (int m = 0; m <= M; ++m) {
      const float v = K[m];
      p.out[(long long)m * p.out_lvl + a] = (p.out_mode == GPSIG_OUT_RSQRT) ? 1.0f / __builtin_sqrtf(v + p.jitter) : v;
    }
    return;
  }
  const bool upper = p.pair_mode == GPSIG_PAIRS_UPPER;
  const bool own = a >= p.out_row0 && a < p.out_row0 + p.out_rows;
  const bool mir = upper && a != b && b >= p.out_row0 && b < p.out_row0 + p.out_rows;
  const long long o1 = (long long)(a - p.out_row0) * p.out_ld + b;
  const long long o2 = (long long)(b - p.out_row0) * p.out_ld + a;
  if (p.out_mode == GPSIG_OUT_LEVELS) {
    for (int m = 0; m <= M; ++m) {
      if (own) p.out[m * p.out_lvl + o1] = K[m];
      if (mir) p.out[m * p.out_lvl + o2] = K[m];
    }
    return;
  }
  const float jit = (upper && a == b) ? p.jitter : 0.0f;
  float sum = 0.0f;
  for (int m = 0; m <= M; ++m) {
    float v = K[m] + jit;
    if (p.rs1) v *= p.rs1[(long long)m * p.n1 + a] * p.rs2[(long long)m * p.n2 + b];
    if (p.scale) v *= p.scale[m];
    if (p.out_mode == GPSIG_OUT_NORM_LEVELS) {
      if (own) p.out[m * p.out_lvl + o1] = v;
      if (mir) p.out[m * p.out_lvl + o2] = v;
    }
    sum += v;
  }
  if (p.out_mode == GPSIG_OUT_NORM_SUM) {
    if (own) p.out[o1] = sum;
    if (mir) p.out[o2] = sum;
  }
}

}  // namespace gpsig
