// gpsig_amd -- pieces shared by the truncated-signature kernels (first order, higher order):
// the per-point feature layout, the pair-tile scheduler, the fused normalisation epilogue and the
// per-row seed (base-kernel second difference).
#pragma once
#include "common.h"

namespace gpsig {

// Per-point feature record, FS floats (16-byte aligned): [x (DP) | dx (DP) | |dx|^2/2 | pad...]
// dx_i = x_{i+1} - x_i (zero for the last point).  DP = padded channel count of the instantiation.
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
};

// Wave-uniform record of row i: x_{i+1} (RBF DIFF) or x_i (POINT seeds), dx_i, |dx_i|^2/2.
template <int DP>
struct RowData {
  float x[DP], dx[DP], hdx;
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
        dM[w] = c;  // padded columns have dy == 0
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
// Tile scheduler.  A workgroup = 4 waves; wave w takes sequence a = 4*ta + w; the wave's G = 64/LP
// lane groups take b = G*tb + g.  UPPER enumerates only tiles with some b >= a: with k = 4/G,
// tile row ta has ntb - k*ta tiles, prefix P(r) = r*ntb - k*r*(r-1)/2, inverted in closed form.
struct Tile { int ta, tb; };

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
