// gpsig_amd -- VJP of the higher-order truncated signature kernel Gram (order > 1) on gfx950.
//
// The reference differentiates signature_kern_higher_order (gpsig/signature_algs.py:37-74) through TF
// autodiff of the materialised (N1, L1, N2, L2) block tensors.  Here one wave owns one pair (64 lanes x
// W = 4 columns, l2 <= 256) and streams the rows as the forward kernel (sig_ho.hip):
//
//   level m+1 from level m at row i, with P the multiplier of dM (R_{m+1} = dM * P_{m+1}):
//     P[0][0] = excl_j(sum_x CB_m[x]),   P[0][y] = CB_m[y-1] / (y+1),
//     P[x][0] = excl_j(sum_y R_m[x-1][y]) / (x+1),   P[x][y] = R_m[x-1][y-1] / ((x+1)(y+1))
//   CB_m[y] (rows < i) += sum_x R_m[x][y];   K_m = sum_j sum_y CB_m[y] at the end.
//
// Reverse sweep, rows i = L1-2 .. 0:
//   * inversion (ascending m): CB_m(i) = CB_m(i+1) - colsum(R_m(i)) recovers the forward state, and the
//     multipliers P_m(i) of the row are kept in this lane's LDS slab;
//   * adjoint (descending m), Bh_m[y] = dLoss/dCB_m[y] of the state after the row (Bh_M = g_M):
//       Rh_m[x][y] = Bh_m[y] + rexcl_j(dM Rh_{m+1}[x+1][0]) / (x+2) + dM Rh_{m+1}[x+1][y+1] / ((x+2)(y+2)),
//       Bh_m[y] += rexcl_j(dM Rh_{m+1}[0][0]) + dM Rh_{m+1}[0][y+1] / (y+2),
//       dLoss/d dM += sum_xy Rh_m[x][y] P_m[x][y]   (Rh_1 for level 1: R_1 = dM);
//   * the adjoint of the second difference and the point-weight tile as in the first-order wide VJP
//     (sig_bwd_wide.h): the host turns the tile into gradients with the matrix-core GEMMs.
// Cells come from the wide-channel seed (wide.h), so any channel count is accepted.
#pragma once
#include <type_traits>

#include "bwd_pair.h"
#include "wide.h"

namespace gpsig {

#ifndef GPSIG_WIDE_BWD_R
#define GPSIG_WIDE_BWD_R 4
#endif

// f(std::integral_constant<int, k>) for k = B .. E-1 (ascending) / E-1 .. B (descending)
template <int B, int E, class F>
GPSIG_DEV void static_for(F &&f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}
template <int B, int E, class F>
GPSIG_DEV void static_for_desc(F &&f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, E - 1>{});
    static_for_desc<B, E - 1>(f);
  }
}

template <int ORD, int M>
struct HoBwdLayout {
  static constexpr int dm(int m) { return m < ORD ? m : ORD; }
  static constexpr int cbo(int m) {  // CB slot of level m (1-based), levels 1..M
    int o = 0;
    for (int k = 1; k < m; ++k) o += dm(k);
    return o;
  }
  static constexpr int ncb = cbo(M + 1);  // forward state (level M only for K_M)
  static constexpr int nbh = cbo(M);      // adjoint state, levels 1..M-1
  static constexpr int po(int m) {  // P slot of level m >= 2
    int o = 0;
    for (int k = 2; k < m; ++k) o += dm(k) * dm(k);
    return o;
  }
  static constexpr int np = po(M + 1);
};

// LDS of the multipliers P of one 4-wave workgroup (W = 4 columns per lane)
template <int ORD, int M>
constexpr size_t ho_bwd_lds_bytes() {
  return (size_t)4 * HoBwdLayout<ORD, M>::np * 64 * 4 * sizeof(float);
}

template <int ORD, int M, int SEED>
__global__ __launch_bounds__(256) void sig_ho_bwd_kernel(BwdArgs p) {
  constexpr int W = 4, W2 = 2;
  constexpr int RC = GPSIG_WIDE_BWD_R;
  constexpr bool RBF = SEED == SEED_RBF_DIFF;
  static_assert(SEED == SEED_RBF_DIFF || SEED == SEED_LIN_DIFF, "higher order: difference seeds");
  static_assert(M >= 2 && ORD >= 2 && ORD <= M, "higher order");
  using Lay = HoBwdLayout<ORD, M>;
  using Seed = WideSeed<W, RC, SEED>;
  __shared__ __attribute__((aligned(16))) float cbuf[4][RC][64][2 * W];
  extern __shared__ __attribute__((aligned(16))) float pslab[];

  const int lane = threadIdx.x & 63;
  const int wave = wave_uniform(threadIdx.x >> 6);
  const bool diag = p.pair_mode == GPSIG_PAIRS_DIAG;
  const long long lblk = p.blk0 + (long long)blockIdx.x;

  // ---- which pair: one per wave (the enumeration of the LP = 64 launches)
  int a, b;
  if (diag) {
    a = p.row_begin + (int)lblk * 4 + wave;
    b = a;
    if (a >= p.row_end) return;
  } else {
    int ta, tb;
    if (p.pair_mode == GPSIG_PAIRS_UPPER) {
      const Tile t = upper_tile(p.tile_base + lblk, p.ntb, 4);
      ta = t.ta;
      tb = t.tb;
    } else {
      ta = p.tiles_a0 + (int)(lblk / p.ntb);
      tb = (int)(lblk % p.ntb);
    }
    a = ta * 4 + wave;
    b = tb;
    if (a < p.row_begin || a >= p.row_end) return;  // wave-uniform
  }
  bool pair_ok = b < p.n2;
  if (p.pair_mode == GPSIG_PAIRS_UPPER) pair_ok = pair_ok && b >= a;
  if (!pair_ok) return;  // one pair per wave: wave-uniform (its tile rows stay as the host zeroed them)
  const int bl = b;
  const int l1 = p.l1, l2 = p.l2;
  const float *__restrict__ fx = p.FX + (long long)a * p.sx;
  const float *__restrict__ fy = p.FY + (long long)bl * p.sy;
  cfloat *fxc = as_const(fx);
  const int nrows = l1 - 1;

  Seed seed;
  seed.init(p.wd, p.lw1, p.lw2, fx, fy, lane, l2);
  if constexpr (RBF) seed.bound_c(nrows);
  bool colv[W], ptv[W];
#pragma unroll
  for (int w = 0; w < W; ++w) {
    const int j = lane * W + w;
    colv[w] = j < l2 - 1;
    ptv[w] = j < l2;
  }

  // cells dM (slots 0..W-1) and k of the row's point (W..2W-1, RBF) of rows i0 .. i0 + RC - 1
  float(*cb)[64][2 * W] = cbuf[wave];
  auto regen = [&](int i0) {
    if constexpr (RBF) {
      seed.exact(fxc + i0, seed.Eq, seed.kc);
      seed.kcR = lane_next(seed.kc[0][0]);
    }
    seed.chunk(i0);
    auto one = [&](auto rr) {
      constexpr int r = decltype(rr)::value;
      if (i0 + r >= nrows) return;
      const typename Seed::Row rd = seed.template row_of<r>(i0 + r);
      f2 dM[W2];
      if constexpr (RBF) {
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
      for (int w = 0; w < W; ++w) cb[r][lane][w] = colv[w] ? dM[w % W2][w / W2] : 0.0f;
    };
    one(std::integral_constant<int, 0>{});
    if constexpr (RC > 1) one(std::integral_constant<int, 1>{});
    if constexpr (RC > 2) one(std::integral_constant<int, 2>{});
    if constexpr (RC > 3) one(std::integral_constant<int, 3>{});
  };

  // level m+1's multipliers P (row i) from CB_m (rows < i) and the row's level-m blocks R (all lanes of
  // the wave: the scans run over the pair's columns)
  auto level_up = [&](auto mt, const float (&CB)[Lay::ncb][W], const float (&R)[ORD][ORD][W],
                      float (&P)[ORD][ORD][W]) {
    constexpr int m = decltype(mt)::value;
    constexpr int dmv = Lay::dm(m), dn = Lay::dm(m + 1);
    float in[dn][W], ex[dn][W];
#pragma unroll
    for (int w = 0; w < W; ++w) {
      float t = 0.0f;
#pragma unroll
      for (int x = 0; x < dmv; ++x) t += CB[Lay::cbo(m) + x][w];
      in[0][w] = t;
#pragma unroll
      for (int x = 1; x < dn; ++x) {
        float rs = 0.0f;
#pragma unroll
        for (int y = 0; y < dmv; ++y) rs += R[x - 1][y][w];
        in[x][w] = rs;
      }
    }
    group_excl_cols_n<64, W, dn>(in, ex);
#pragma unroll
    for (int w = 0; w < W; ++w) {
      P[0][0][w] = ex[0][w];
#pragma unroll
      for (int y = 1; y < dn; ++y) P[0][y][w] = CB[Lay::cbo(m) + y - 1][w] * (1.0f / (float)(y + 1));
#pragma unroll
      for (int x = 1; x < dn; ++x) {
        P[x][0][w] = ex[x][w] * (1.0f / (float)(x + 1));
#pragma unroll
        for (int y = 1; y < dn; ++y) P[x][y][w] = R[x - 1][y - 1][w] * (1.0f / (float)((x + 1) * (y + 1)));
      }
    }
  };

  // ---- forward sweep: the end-of-sweep column sums and the raw levels K_m
  float CB[Lay::ncb][W];
#pragma unroll
  for (int k = 0; k < Lay::ncb; ++k)
#pragma unroll
    for (int w = 0; w < W; ++w) CB[k][w] = 0.0f;
  for (int i0 = 0; i0 < nrows; i0 += RC) {
    regen(i0);
    const int nr = nrows - i0 < RC ? nrows - i0 : RC;
    for (int r = 0; r < nr; ++r) {
      float dM[W];
#pragma unroll
      for (int w = 0; w < W; ++w) dM[w] = cb[r][lane][w];
      float R[ORD][ORD][W];
#pragma unroll
      for (int w = 0; w < W; ++w) R[0][0][w] = dM[w];
      auto step = [&](auto mt) {
        constexpr int m = decltype(mt)::value;
        constexpr int dmv = Lay::dm(m), dn = Lay::dm(m + 1);
        float Rn[ORD][ORD][W];
        if constexpr (m < M) {
          level_up(mt, CB, R, Rn);
#pragma unroll
          for (int x = 0; x < dn; ++x)
#pragma unroll
            for (int y = 0; y < dn; ++y)
#pragma unroll
              for (int w = 0; w < W; ++w) Rn[x][y][w] *= dM[w];
        }
        // CB_m += the row's level-m column sums (after level m+1 used the rows before)
#pragma unroll
        for (int y = 0; y < dmv; ++y)
#pragma unroll
          for (int w = 0; w < W; ++w) {
            float cs = 0.0f;
#pragma unroll
            for (int x = 0; x < dmv; ++x) cs += R[x][y][w];
            CB[Lay::cbo(m) + y][w] += cs;
          }
        if constexpr (m < M) {
#pragma unroll
          for (int x = 0; x < dn; ++x)
#pragma unroll
            for (int y = 0; y < dn; ++y)
#pragma unroll
              for (int w = 0; w < W; ++w) R[x][y][w] = Rn[x][y][w];
        }
      };
      static_for<1, M + 1>(step);
    }
  }
  float K[M + 1];
  K[0] = 1.0f;
  static_for<1, M + 1>([&](auto mt) {
    constexpr int m = decltype(mt)::value;
    float s = 0.0f;
#pragma unroll
    for (int y = 0; y < Lay::dm(m); ++y)
#pragma unroll
      for (int w = 0; w < W; ++w) s += CB[Lay::cbo(m) + y][w];
    K[m] = group_sum<64>(s);
  });
  K[1] = level1_closed_wide<SEED>(fx, fy, p.wd, p.lw1, p.lw2, l1, l2);

  const PairTerms<M> pt(p, a, bl, lane, pair_ok, lblk);
  float gw[M + 1];
  pt.weights(gw);

  // ---- point weights of this pair into the tile (as sig_bwd_wide.h)
  float *__restrict__ tpair = p.tile + (long long)(a - p.tile_a0) * p.tile_as +
                              (diag ? 0 : (long long)(bl - p.tile_b0) * l2) + lane * W;
  const bool full_cols = lane * W + W <= l2;
  auto emit = [&](int pi, const float (&Kh)[W], const float (&kr)[W]) {
    float *__restrict__ o = tpair + (long long)pi * p.tile_ld;
    float v[W];
#pragma unroll
    for (int w = 0; w < W; ++w) v[w] = RBF ? Kh[w] * kr[w] : Kh[w];
    if (full_cols) {
      *reinterpret_cast<f4u *>(o) = (f4u){v[0], v[1], v[2], v[3]};
    } else {
#pragma unroll
      for (int w = 0; w < W; ++w)
        if (ptv[w]) o[w] = v[w];
    }
  };

  // ---- reverse sweep
  float Bh[Lay::nbh][W];  // dLoss/dCB_m of levels 1..M-1 (level M: the constant g_M)
#pragma unroll
  for (int k = 0; k < Lay::nbh; ++k)
#pragma unroll
    for (int w = 0; w < W; ++w) Bh[k][w] = 0.0f;
  static_for<1, M>([&](auto mt) {
    constexpr int m = decltype(mt)::value;
#pragma unroll
    for (int y = 0; y < Lay::dm(m); ++y)
#pragma unroll
      for (int w = 0; w < W; ++w) Bh[Lay::cbo(m) + y][w] = gw[m];
  });
  const float gM = gw[M];
  float *__restrict__ ps = pslab + (long long)wave * Lay::np * 64 * W + lane * W;  // [slot][lane][w]
  auto pput = [&](int slot, const float (&v)[W]) {
    *reinterpret_cast<f4 *>(ps + (long long)slot * 64 * W) = (f4){v[0], v[1], v[2], v[3]};
  };
  auto pget = [&](int slot, float (&v)[W]) {
    const f4 t = *reinterpret_cast<const f4 *>(ps + (long long)slot * 64 * W);
#pragma unroll
    for (int w = 0; w < W; ++w) v[w] = t[w];
  };

  float Ep[W], kr1[W];
#pragma unroll
  for (int w = 0; w < W; ++w) {
    Ep[w] = 0.0f;
    kr1[w] = 1.0f;
  }
  if constexpr (RBF) {  // k row of the last point
    f2 Eq0[W2], k0[W2];
    seed.exact(fxc + nrows, Eq0, k0);
#pragma unroll
    for (int w = 0; w < W; ++w) kr1[w] = k0[w % W2][w / W2];
  }

  auto rev_row = [&](int i, const float (&dM)[W], const float (&k0)[W]) {
    // inversion, ascending levels: CB_m(i) and the multipliers P_m(i) of the row
    {
      float R[ORD][ORD][W];
#pragma unroll
      for (int w = 0; w < W; ++w) {
        R[0][0][w] = dM[w];
        CB[Lay::cbo(1)][w] -= dM[w];
      }
      static_for<1, M>([&](auto mt) {
        constexpr int m = decltype(mt)::value;
        constexpr int dn = Lay::dm(m + 1);
        float P[ORD][ORD][W];
        level_up(mt, CB, R, P);
#pragma unroll
        for (int x = 0; x < dn; ++x)
#pragma unroll
          for (int y = 0; y < dn; ++y) {
            pput(Lay::po(m + 1) + x * dn + y, P[x][y]);
#pragma unroll
            for (int w = 0; w < W; ++w) R[x][y][w] = dM[w] * P[x][y][w];
          }
        if constexpr (m + 1 < M) {  // CB_{m+1}(i) = CB_{m+1}(i+1) - colsum(R_{m+1}(i))
#pragma unroll
          for (int y = 0; y < dn; ++y)
#pragma unroll
            for (int w = 0; w < W; ++w) {
              float cs = 0.0f;
#pragma unroll
              for (int x = 0; x < dn; ++x) cs += R[x][y][w];
              CB[Lay::cbo(m + 1) + y][w] -= cs;
            }
        }
      });
    }
    // adjoint, descending levels
    float Dh[W];
    float Rh[ORD][ORD][W];  // Rh_{m+1} entering level m
    {
      constexpr int dM_ = Lay::dm(M);
      float P[W];
#pragma unroll
      for (int w = 0; w < W; ++w) Dh[w] = 0.0f;
#pragma unroll
      for (int x = 0; x < dM_; ++x)
#pragma unroll
        for (int y = 0; y < dM_; ++y) {
          pget(Lay::po(M) + x * dM_ + y, P);
#pragma unroll
          for (int w = 0; w < W; ++w) {
            Rh[x][y][w] = gM;
            Dh[w] = __builtin_fmaf(gM, P[w], Dh[w]);
          }
        }
    }
    static_for_desc<1, M>([&](auto mt) {
      constexpr int m = decltype(mt)::value;
      constexpr int dmv = Lay::dm(m), dn = Lay::dm(m + 1);
      float Q[dn][W], rx[dn][W];
#pragma unroll
      for (int w = 0; w < W; ++w) {
        Q[0][w] = dM[w] * Rh[0][0][w];
#pragma unroll
        for (int x = 1; x < dn; ++x) Q[x][w] = dM[w] * Rh[x][0][w] * (1.0f / (float)(x + 1));
      }
      group_rexcl_cols_n<64, W, dn>(Q, rx);
      float Rm[ORD][ORD][W];
#pragma unroll
      for (int x = 0; x < dmv; ++x)
#pragma unroll
        for (int y = 0; y < dmv; ++y)
#pragma unroll
          for (int w = 0; w < W; ++w) {
            float v = Bh[Lay::cbo(m) + y][w];
            if (x + 1 < dn) v += rx[x + 1][w];
            if (x + 1 < dn && y + 1 < dn)
              v = __builtin_fmaf(dM[w] * Rh[x + 1][y + 1][w], 1.0f / (float)((x + 2) * (y + 2)), v);
            Rm[x][y][w] = v;
          }
#pragma unroll
      for (int y = 0; y < dmv; ++y)
#pragma unroll
        for (int w = 0; w < W; ++w) {
          float v = Bh[Lay::cbo(m) + y][w] + rx[0][w];
          if (y + 1 < dn) v = __builtin_fmaf(dM[w] * Rh[0][y + 1][w], 1.0f / (float)(y + 2), v);
          Bh[Lay::cbo(m) + y][w] = v;
        }
      if constexpr (m >= 2) {
        float P[W];
#pragma unroll
        for (int x = 0; x < dmv; ++x)
#pragma unroll
          for (int y = 0; y < dmv; ++y) {
            pget(Lay::po(m) + x * dmv + y, P);
#pragma unroll
            for (int w = 0; w < W; ++w) Dh[w] = __builtin_fmaf(Rm[x][y][w], P[w], Dh[w]);
          }
      } else {
#pragma unroll
        for (int w = 0; w < W; ++w) Dh[w] += Rm[0][0][w];
      }
#pragma unroll
      for (int x = 0; x < dmv; ++x)
#pragma unroll
        for (int y = 0; y < dmv; ++y)
#pragma unroll
          for (int w = 0; w < W; ++w) Rh[x][y][w] = Rm[x][y][w];
    });
#pragma unroll
    for (int w = 0; w < W; ++w) Dh[w] = colv[w] ? Dh[w] : 0.0f;
    // adjoint of the second difference (signature_algs.py:26): E(i, j) = Dh(i, j-1) - Dh(i, j)
    float left = lane_prev(Dh[W - 1]);
    if (lane == 0) left = 0.0f;
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
  {
    float Kh[W];
#pragma unroll
    for (int w = 0; w < W; ++w) Kh[w] = -Ep[w];
    emit(0, Kh, kr1);
  }
  pt.norm(K);
}

}  // namespace gpsig
