// gpsig_amd -- first-order Gram VJP at wide channel counts (runtime channel loop, wide.h).
//
// The recursion's adjoint is the one of sig_bwd.h (forward state recovered by inverting the update,
// adjoint column sums by reverse exclusive scans, dLoss/d dM = sum_m Ch_m S_{m-1}, the adjoint of the
// second difference).  What changes with the channel count is where the point gradients are formed:
// the fixed-channel kernel contracts every point weight with y_j (x_i) in registers (3 W DP floats per
// lane), which does not scale past a few channels.  Here the kernel writes the point weights
//     W_ab[i][j] = dLoss/dk(x_ai, y_bj) * k(x_ai, y_bj)        (RBF; linear: dLoss/dk)
// of a chunk of pairs to a tile in HBM, and the host side turns them into gradients with two GEMMs on
// the matrix cores (gemm.hip) -- the transpose of the reference's _square_dist GEMM
// (kernels.py:946-957), whose TF autodiff produces exactly these products:
//     dLoss/dx_ai = sum_bj W_ab[i][j] (y_bj - x_ai),   dLoss/dy_bj = sum_ai W_ab[i][j] (x_ai - y_bj)
// (linear: without the -x, -y terms), i.e. [W Y | rowsum W] and [W^T X | colsum W].
// The cells are regenerated, forward and in reverse, by the forward kernel's own seed (RbfSeedWide /
// WideSeedGen: the chunk's dots, the exp-free recurrences, exact rows), WIDE_R rows at a time, into the
// lane's LDS slots.
#pragma once
#include "bwd_pair.h"
#include "wide.h"

namespace gpsig {

// rows per regenerated chunk of the VJPs (LDS: 4 waves x RC x 64 lanes x 2W floats)
#ifndef GPSIG_WIDE_BWD_R
#define GPSIG_WIDE_BWD_R 4
#endif

template <int W, int LP, int M, int SEED>
__global__ __launch_bounds__(256) void sig_bwd_wide_kernel(BwdArgs p) {
  constexpr int G = 64 / LP;
  constexpr int W2 = W / 2;
  constexpr int RC = GPSIG_WIDE_BWD_R;
  constexpr bool DIFF = (SEED == SEED_RBF_DIFF || SEED == SEED_LIN_DIFF);
  constexpr bool RBF = (SEED == SEED_RBF_DIFF || SEED == SEED_RBF_POINT);
  constexpr int ML = M > 1 ? M - 1 : 1;
  using Seed = WideSeed<W, RC, SEED>;
  __shared__ __attribute__((aligned(16))) float cbuf[4][RC][64][2 * W];

  const int lane = threadIdx.x & 63;
  const int wave = wave_uniform(threadIdx.x >> 6);
  const int g = lane / LP;
  const int gl = lane % LP;
  const bool diag = p.pair_mode == GPSIG_PAIRS_DIAG;
  const long long lblk = p.blk0 + (long long)blockIdx.x;

  int a, b;
  if (diag) {
    a = p.row_begin + (int)lblk * 4 + wave;
    b = a;
    if (a >= p.row_end) return;
  } else {
    int ta, tb;
    if (p.pair_mode == GPSIG_PAIRS_UPPER) {
      const Tile t = upper_tile(p.tile_base + lblk, p.ntb, 4 / G);
      ta = t.ta;
      tb = t.tb;
    } else {
      ta = p.tiles_a0 + (int)(lblk / p.ntb);
      tb = (int)(lblk % p.ntb);
    }
    a = ta * 4 + wave;
    b = tb * G + g;
    if (a < p.row_begin || a >= p.row_end) return;  // wave-uniform
  }
  bool pair_ok = b < p.n2;
  if (p.pair_mode == GPSIG_PAIRS_UPPER) pair_ok = pair_ok && b >= a;
  if (diag) pair_ok = (g == 0);
  const int bl = b < p.n2 ? b : p.n2 - 1;
  const int l1 = p.l1, l2 = p.l2;
  const float *__restrict__ fx = p.FX + (long long)a * p.sx;
  const float *__restrict__ fy = p.FY + (long long)bl * p.sy;
  cfloat *fxc = as_const(fx);
  const int nrows = DIFF ? l1 - 1 : l1;

  Seed seed;
  seed.init(p.wd, p.lw1, p.lw2, fx, fy, gl, l2);
  if constexpr (SEED == SEED_RBF_DIFF) seed.bound_c(nrows);
  // DIAG: the pair's seed tiles (wide_diag_tiles) replace the channel loops of chunk() and the chunk anchors
  bool tiled = false;
  if constexpr (SEED == SEED_RBF_DIFF) {
    if (diag && p.dtile) {
      const float *base = p.dtile + (long long)(a - p.dt_a0) * p.dt_pair;
      static_assert(DIAG_TILE_ANCHOR == RC, "the regeneration chunks start on the tile's anchor rows");
      seed.set_tiles(base, base + p.dt_rows * p.dt_ld, base + 2 * p.dt_rows * p.dt_ld, p.dt_ld, gl, DIAG_TILE_ANCHOR,
                     (int)(p.dt_rows / DIAG_TILE_ANCHOR));
      tiled = true;
    }
  }
  bool colv[W], ptv[W];
#pragma unroll
  for (int w = 0; w < W; ++w) {
    const int j = gl * W + w;
    colv[w] = j < (DIFF ? l2 - 1 : l2);
    ptv[w] = j < l2;
  }

  // cells dM (slots 0..W-1) and the k values of the row's point (slots W..2W-1, RBF) of rows
  // i0 .. i0 + RC - 1, natural column order, into this lane's LDS slots
  float(*cb)[64][2 * W] = cbuf[wave];
  auto regen = [&](int i0) {
    if constexpr (SEED == SEED_RBF_DIFF) {
      if (tiled)
        seed.exact_tile(i0 / RC, seed.Eq, seed.kc);
      else
        seed.exact(fxc + i0, seed.Eq, seed.kc);
      seed.kcR = lane_next(seed.kc[0][0]);
      if (tiled)
        seed.chunk_tile(i0);
      else
        seed.chunk(i0);
    } else {
      seed.chunk(i0);
    }
    auto one = [&](auto rr) {
      constexpr int r = decltype(rr)::value;
      if (i0 + r >= nrows) return;
      const typename Seed::Row rd = seed.template row_of<r>(i0 + r);
      f2 dM[W2];
      if constexpr (SEED == SEED_RBF_DIFF) {
#pragma unroll
        for (int w = 0; w < W; ++w) cb[r][lane][W + w] = seed.kc[w % W2][w / W2];
        if (seed.clo)
          seed.template row<true>(rd, false, dM);
        else
          seed.template row<false>(rd, false, dM);
      } else {
        seed.template row<false>(rd, false, dM);
      }
#pragma unroll
      for (int w = 0; w < W; ++w) {
        const float v = dM[w % W2][w / W2];
        cb[r][lane][w] = colv[w] ? v : 0.0f;
        if constexpr (SEED == SEED_RBF_POINT) cb[r][lane][W + w] = v;  // the cell is k(x_i, y_j)
      }
    };
    one(std::integral_constant<int, 0>{});
    if constexpr (RC > 1) one(std::integral_constant<int, 1>{});
    if constexpr (RC > 2) one(std::integral_constant<int, 2>{});
    if constexpr (RC > 3) one(std::integral_constant<int, 3>{});
    if constexpr (RC > 4) one(std::integral_constant<int, 4>{});
    if constexpr (RC > 5) one(std::integral_constant<int, 5>{});
    if constexpr (RC > 6) one(std::integral_constant<int, 6>{});
    if constexpr (RC > 7) one(std::integral_constant<int, 7>{});
  };

  // ---- forward state: the end-of-sweep column sums (saved by the forward launch, or by a sweep here)
  float C[M][W];
#pragma unroll
  for (int m = 0; m < M; ++m)
#pragma unroll
    for (int w = 0; w < W; ++w) C[m][w] = 0.0f;
  float K[M + 1];
  K[0] = 1.0f;
  const bool saved = DIFF && p.state != nullptr;
  if (saved) {
    const float *__restrict__ st =
        p.state + (pair_ok ? state_slot(a, bl, p.n2, p.pair_mode == GPSIG_PAIRS_UPPER) * state_stride(M, l2) : 0);
    const int nc = l2 - 1;
#pragma unroll
    for (int m = 0; m + 1 < M; ++m)
#pragma unroll
      for (int w = 0; w < W; ++w) {
        const int j = gl * W + w;
        C[m][w] = (pair_ok && j < nc) ? st[(long long)m * nc + j] : 0.0f;
      }
#pragma unroll
    for (int m = 1; m <= M; ++m) K[m] = pair_ok ? st[(long long)(M - 1) * nc + m - 1] : 0.0f;
  } else {
    for (int i0 = 0; i0 < nrows; i0 += RC) {
      regen(i0);
      const int nr = nrows - i0 < RC ? nrows - i0 : RC;
      for (int r = 0; r < nr; ++r) {
        float dM[W];
#pragma unroll
        for (int w = 0; w < W; ++w) dM[w] = cb[r][lane][w];
        if constexpr (M > 1) {
          float Cs[ML][W], S[ML][W];
#pragma unroll
          for (int m = 0; m < ML; ++m)
#pragma unroll
            for (int w = 0; w < W; ++w) Cs[m][w] = C[m][w];
          group_excl_cols_n<LP, W, ML>(Cs, S);
#pragma unroll
          for (int m = 1; m < M; ++m)
#pragma unroll
            for (int w = 0; w < W; ++w) C[m][w] = __builtin_fmaf(dM[w], S[m - 1][w], C[m][w]);
        }
#pragma unroll
        for (int w = 0; w < W; ++w) C[0][w] += dM[w];
      }
    }
#pragma unroll
    for (int m = 0; m < M; ++m) {
      float s = 0.0f;
#pragma unroll
      for (int w = 0; w < W; ++w) s += C[m][w];
      K[m + 1] = group_sum<LP>(s);
    }
    if constexpr (DIFF) K[1] = level1_closed_wide<SEED>(fx, fy, p.wd, p.lw1, p.lw2, l1, l2);
  }

  // ---- per-level weights g_m = dLoss/dK_m(a, b) and the normalisation / scale terms (bwd_pair.h)
  const PairTerms<M> pt(p, a, bl, gl, pair_ok, lblk);
  float gw[M + 1];
  pt.weights(gw);

  // ---- point weights of this pair into the tile: row pi of the pair's l1 x l2 block
  float *__restrict__ tpair = p.tile + (long long)(a - p.tile_a0) * p.tile_as +
                              (diag ? 0 : (long long)(bl - p.tile_b0) * l2) + gl * W;
  const bool full_cols = gl * W + W <= l2;
  auto emit = [&](int pi, const float (&Kh)[W], const float (&kr)[W]) {
    if (!pair_ok) return;
    float *__restrict__ o = tpair + (long long)pi * p.tile_ld;
    float v[W];
#pragma unroll
    for (int w = 0; w < W; ++w) v[w] = RBF ? Kh[w] * kr[w] : Kh[w];
    if (full_cols) {
#pragma unroll
      for (int h = 0; h < W / 4; ++h) *reinterpret_cast<f4u *>(o + 4 * h) = (f4u){v[4 * h], v[4 * h + 1], v[4 * h + 2], v[4 * h + 3]};
    } else {
#pragma unroll
      for (int w = 0; w < W; ++w)
        if (ptv[w]) o[w] = v[w];
    }
  };

  // ---- reverse sweep
  float Ch[ML][W];
#pragma unroll
  for (int m = 0; m < ML; ++m)
#pragma unroll
    for (int w = 0; w < W; ++w) Ch[m][w] = gw[m + 1];
  const float gM = gw[M];
  float Ep[W], kr1[W];
#pragma unroll
  for (int w = 0; w < W; ++w) {
    Ep[w] = 0.0f;
    kr1[w] = 1.0f;
  }
  if constexpr (SEED == SEED_RBF_DIFF) {  // k row of the last point
    f2 Eq0[W2], k0[W2];
    seed.exact(fxc + nrows, Eq0, k0);
#pragma unroll
    for (int w = 0; w < W; ++w) kr1[w] = k0[w % W2][w / W2];
  }

  auto rev_row = [&](int i, const float (&dM)[W], const float (&k0)[W]) {
    float Dh[W];
#pragma unroll
    for (int w = 0; w < W; ++w) {
      C[0][w] -= dM[w];
      Dh[w] = (M > 1) ? Ch[0][w] : gM;
    }
#pragma unroll
    for (int s = 1; s < M; ++s) {
      float Cm[1][W], Sm[1][W];
#pragma unroll
      for (int w = 0; w < W; ++w) Cm[0][w] = C[s - 1][w];
      group_excl_cols_n<LP, W, 1>(Cm, Sm);
#pragma unroll
      for (int w = 0; w < W; ++w) {
        if (s + 1 < M) C[s][w] = __builtin_fmaf(-dM[w], Sm[0][w], C[s][w]);
        const float chn = (s + 1 < M) ? Ch[s < ML ? s : 0][w] : gM;
        Dh[w] = __builtin_fmaf(chn, Sm[0][w], Dh[w]);
      }
    }
#pragma unroll
    for (int w = 0; w < W; ++w) Dh[w] = colv[w] ? Dh[w] : 0.0f;
    if constexpr (M > 1) {
      float v[ML][W], r[ML][W];
#pragma unroll
      for (int m = 0; m < ML; ++m)
#pragma unroll
        for (int w = 0; w < W; ++w) v[m][w] = dM[w] * ((m + 1 < ML) ? Ch[m + 1][w] : gM);
      group_rexcl_cols_n<LP, W, ML>(v, r);
#pragma unroll
      for (int m = 0; m < ML; ++m)
#pragma unroll
        for (int w = 0; w < W; ++w) Ch[m][w] += r[m][w];
    }
    if constexpr (DIFF) {
      float left = lane_prev(Dh[W - 1]);
      if (gl == 0) left = 0.0f;
      float Kh[W];
#pragma unroll
      for (int w = 0; w < W; ++w) {
        const float e = ((w == 0) ? left : Dh[w - 1]) - Dh[w];
        Kh[w] = e - Ep[w];
        Ep[w] = e;
      }
      emit(i + 1, Kh, kr1);
#pragma unroll
      for (int w = 0; w < W; ++w) kr1[w] = k0[w];
    } else {
      emit(i, Dh, k0);
    }
  };

  for (int i0 = ((nrows - 1) / RC) * RC; i0 >= 0; i0 -= RC) {
    const int nr = nrows - i0 < RC ? nrows - i0 : RC;
    regen(i0);
    for (int r = nr - 1; r >= 0; --r) {
      float dM[W], k0[W];
#pragma unroll
      for (int w = 0; w < W; ++w) {
        dM[w] = cb[r][lane][w];
        k0[w] = RBF ? cb[r][lane][W + w] : 1.0f;
      }
      rev_row(i0 + r, dM, k0);
    }
  }
  if constexpr (DIFF) {
    float Kh[W];
#pragma unroll
    for (int w = 0; w < W; ++w) Kh[w] = -Ep[w];
    emit(0, Kh, kr1);
  }
  pt.norm(K);
}

// Geometry of the wide VJP: the forward's (W = 8, LP = 16/32/64), one column block (l2 <= 512).
inline BwdGeo bwd_geometry_wide(int l2) {
  for (int LP : {16, 32, 64})
    if (LP * 8 >= l2) return {8, LP};
  return {0, 0};
}

}  // namespace gpsig
