// gpsig_amd -- VJP of the higher-order truncated signature kernel Gram for the orders and lengths past the
// register kernel (sig_ho_bwd.h: min(order, M) <= 3, l2 <= 256).
//
// Same recursion, adjoint and emission as sig_ho_bwd.h (see there for the formulas), reorganised so that the
// per-row state of a pair does not have to live in registers:
//   * one wave per pair and per workgroup, W = 4 or 8 columns per lane (l2 <= 256 / 512);
//   * the row's multipliers P_m[x][y] of every level live in LDS (np slots of 64 W floats), written by the
//     ascending pass (forward sweep and the inversion of the reverse sweep) and read back by level: R_m =
//     dM P_m is never stored, it is formed on the fly from P_m;
//   * the adjoint runs in place: the level-m adjoint blocks Rh_m overwrite P_m slot by slot once P_m[x][y]
//     has been used (Dh += Rh_m[x][y] P_m[x][y]), so the descending pass needs no second slab; Rh_M is the
//     constant g_M;
//   * the column sums CB_m (levels 1..M) follow the multipliers in the slab; their adjoints Bh_m (1..M-1)
//     stay in registers (the kernel runs one wave per SIMD and may use the whole 512-entry register file),
//     accumulated over the rows in fp64 (round 5): summed in fp32, the rounding of these running sums was
//     the dominant error of the gradient (4e-6 unnormalised, 1.1e-5 normalised at the VOSF trainer's
//     L = 500, against 9e-7 / 1.6e-6 in fp64).
// This is what the VOSF-truncated trainer differentiates (benchmarks/models/train_gpsig_vosf.py:102:
// SignatureLinear(num_levels=5, order=5), max_len 500): orders 4-5 at up to 512 points.
#pragma once
#include "sig_ho_bwd.h"

namespace gpsig {

template <int ORD, int M>
constexpr int ho_lds_np() { return HoBwdLayout<ORD, M>::np; }
// LDS of one pair (multiplier slab + the regenerated cells of a chunk of rows)
template <int ORD, int M, int W>
constexpr size_t ho_bwd_lds_slab_bytes() {
  return (size_t)(ho_lds_np<ORD, M>() + HoBwdLayout<ORD, M>::ncb) * 64 * W * sizeof(float);
}
constexpr size_t ho_bwd_lds_cbuf_bytes(int W) { return (size_t)GPSIG_WIDE_BWD_R * 64 * 2 * W * sizeof(float); }

#ifndef HO_LDS_NOFENCE_SLOTS
#define HO_LDS_NOFENCE_SLOTS 100  // 99 slots (order 5 at 6 levels, 4 at 7) run unfenced without spills; 111 (order 6) spill
#endif
template <int ORD, int M, int W, int SEED>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1))) void sig_ho_bwd_lds_kernel(BwdArgs p) {
  constexpr int W2 = W / 2;
  constexpr int RC = GPSIG_WIDE_BWD_R;
  constexpr bool RBF = SEED == SEED_RBF_DIFF;
  static_assert(SEED == SEED_RBF_DIFF || SEED == SEED_LIN_DIFF, "higher order: difference seeds");
  static_assert(M >= 2 && ORD >= 2 && ORD <= M, "higher order");
  using Lay = HoBwdLayout<ORD, M>;
  using Seed = WideSeed<W, RC, SEED>;
  __shared__ __attribute__((aligned(16))) float cbuf[RC][64][2 * W];
  extern __shared__ __attribute__((aligned(16))) float pslab[];

  const int lane = threadIdx.x & 63;
  const bool diag = p.pair_mode == GPSIG_PAIRS_DIAG;
  const long long lblk = p.blk0 + (long long)blockIdx.x;

  // ---- which pair: one per workgroup
  int a, b;
  if (diag) {
    a = p.row_begin + (int)lblk;
    b = a;
  } else if (p.pair_mode == GPSIG_PAIRS_UPPER) {
    const Tile t = upper_tile(p.tile_base + lblk, p.n2, 1);  // row a holds b = a .. n2-1
    a = t.ta;
    b = t.tb;
  } else {
    a = p.row_begin + (int)(lblk / p.n2);
    b = (int)(lblk % p.n2);
  }
  if (a < p.row_begin || a >= p.row_end || b >= p.n2) return;  // the whole workgroup
  const bool pair_ok = true;
  if (p.pair_mode == GPSIG_PAIRS_UPPER && !p.rs1 && !p.gscale) {
    // a pair without upstream gradient adds nothing (its tile rows are zeros already, sig_bwd_wide.hip): the
    // block-structured weights of a folded cross Gram (autograd.SigGram) leave most pairs empty
    const PairTerms<M> pt0(p, a, b, lane, true, lblk);
    float g0[M + 1];
    pt0.weights(g0);
    bool any = false;
#pragma unroll
    for (int m = 1; m <= M; ++m) any = any || g0[m] != 0.0f;
    if (!any) return;
  }
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
        for (int w = 0; w < W; ++w) cbuf[r][lane][W + w] = seed.kc[w % W2][w / W2];
        if (seed.clo)
          seed.template row<true>(rd, false, dM);
        else
          seed.template row<false>(rd, false, dM);
      } else {
        seed.template row<false>(rd, false, dM);
      }
#pragma unroll
      for (int w = 0; w < W; ++w) cbuf[r][lane][w] = colv[w] ? dM[w % W2][w / W2] : 0.0f;
    };
    one(std::integral_constant<int, 0>{});
    if constexpr (RC > 1) one(std::integral_constant<int, 1>{});
    if constexpr (RC > 2) one(std::integral_constant<int, 2>{});
    if constexpr (RC > 3) one(std::integral_constant<int, 3>{});
  };

  // Compiler barriers around the slab accesses bound the register use where the slab is large (W = 8, or many
  // slots): without them a level's reads are hoisted and the kernel spills (W = 4 at 7 levels).  Small slabs
  // go without: the reads of a level batch ahead of their use (each lane touches only its own columns).
  constexpr bool FENCE = W > 4 || Lay::np + Lay::ncb > HO_LDS_NOFENCE_SLOTS;
  // an empty volatile statement on v: orders the computation of v with the slab accesses around it (with the
  // barriers, and for slabs past 60 slots; otherwise the accumulation is scheduled freely)
  constexpr bool PIN = FENCE || Lay::np + Lay::ncb > 60;  // unpinned past 60 slots the W = 4 kernel spills
  auto pin = [&](float (&v)[W]) {
    if constexpr (PIN) {
#pragma unroll
      for (int w = 0; w < W; ++w) asm volatile("" : "+v"(v[w]));
    }
  };
  // the multiplier slab: slot s of this lane's W columns
  float *__restrict__ ps = pslab + lane * W;
  auto pget = [&](int slot, float (&v)[W]) {
    if constexpr (FENCE) asm volatile("" ::: "memory");
#pragma unroll
    for (int h = 0; h < W / 4; ++h) {
      const f4 t = *reinterpret_cast<const f4 *>(ps + (long long)slot * 64 * W + 4 * h);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[4 * h + e] = t[e];
    }
  };
  auto pput = [&](int slot, const float (&v)[W]) {
#pragma unroll
    for (int h = 0; h < W / 4; ++h)
      *reinterpret_cast<f4 *>(ps + (long long)slot * 64 * W + 4 * h) = (f4){v[4 * h], v[4 * h + 1], v[4 * h + 2], v[4 * h + 3]};
    if constexpr (FENCE) asm volatile("" ::: "memory");
  };
  // the column sums CB_m[y] follow the multipliers in the slab
  constexpr int CBS = Lay::np;
  auto cadd = [&](int k, const float (&v)[W], float sgn) {
    float c[W];
    pget(CBS + k, c);
#pragma unroll
    for (int w = 0; w < W; ++w) c[w] = __builtin_fmaf(sgn, v[w], c[w]);
    pput(CBS + k, c);
  };
  // R_m[x][y] of the row (level 1: dM itself)
  auto rget = [&](auto mt, int x, int y, const float (&dM)[W], float (&v)[W]) {
    constexpr int m = decltype(mt)::value;
    if constexpr (m == 1) {
#pragma unroll
      for (int w = 0; w < W; ++w) v[w] = dM[w];
    } else {
      pget(Lay::po(m) + x * Lay::dm(m) + y, v);
#pragma unroll
      for (int w = 0; w < W; ++w) v[w] *= dM[w];
    }
  };

  // level m+1's multipliers P (row i) into the slab, from CB_m (rows < i) and the row's R_m (the scans run
  // over the pair's columns, all lanes of the wave); one column x of P at a time, so that no level-wide
  // temporaries stay live
  auto level_up = [&](auto mt, const float (&dM)[W]) {
    constexpr int m = decltype(mt)::value;
    constexpr int dmv = Lay::dm(m), dn = Lay::dm(m + 1);
    constexpr int base = Lay::po(m + 1);
#pragma unroll
    for (int x = 0; x < dn; ++x) {
      float in[1][W], ex[1][W];
#pragma unroll
      for (int w = 0; w < W; ++w) in[0][w] = 0.0f;
#pragma unroll
      for (int y = 0; y < dmv; ++y) {
        float r[W];
        if (x == 0) {
          pget(CBS + Lay::cbo(m) + y, r);
        } else {
          rget(mt, x - 1, y, dM, r);
        }
#pragma unroll
        for (int w = 0; w < W; ++w) in[0][w] += r[w];
        if (y + 1 < dn) {  // P[x][y+1] = (x ? R[x-1][y] : CB[y]) / ((x+1)(y+2))
#pragma unroll
          for (int w = 0; w < W; ++w) r[w] *= 1.0f / (float)((x + 1) * (y + 2));
          pput(base + x * dn + y + 1, r);
        }
      }
      group_excl_cols_n<64, W, 1>(in, ex);
#pragma unroll
      for (int w = 0; w < W; ++w) ex[0][w] *= 1.0f / (float)(x + 1);
      pput(base + x * dn, ex[0]);
    }
  };
  // colsum_x R_m[x][y] of the row
  auto colsum = [&](auto mt, int y, const float (&dM)[W], float (&cs)[W]) {
    constexpr int m = decltype(mt)::value;
#pragma unroll
    for (int w = 0; w < W; ++w) cs[w] = 0.0f;
#pragma unroll
    for (int x = 0; x < Lay::dm(m); ++x) {
      float r[W];
      rget(mt, x, y, dM, r);
#pragma unroll
      for (int w = 0; w < W; ++w) cs[w] += r[w];
    }
  };

  // ---- forward sweep: the end-of-sweep column sums and the raw levels K_m
  {
    float z[W];
#pragma unroll
    for (int w = 0; w < W; ++w) z[w] = 0.0f;
#pragma unroll
    for (int k = 0; k < Lay::ncb; ++k) pput(CBS + k, z);
  }
  for (int i0 = 0; i0 < nrows; i0 += RC) {
    regen(i0);
    const int nr = nrows - i0 < RC ? nrows - i0 : RC;
    for (int r = 0; r < nr; ++r) {
      float dM[W];
#pragma unroll
      for (int w = 0; w < W; ++w) dM[w] = cbuf[r][lane][w];
      static_for<1, M + 1>([&](auto mt) {
        constexpr int m = decltype(mt)::value;
        if constexpr (m < M) level_up(mt, dM);  // uses CB_m before this row's update
        // CB_m += the row's level-m column sums
#pragma unroll
        for (int y = 0; y < Lay::dm(m); ++y) {
          float cs[W];
          colsum(mt, y, dM, cs);
          cadd(Lay::cbo(m) + y, cs, 1.0f);
        }
      });
    }
  }
  float K[M + 1];
  K[0] = 1.0f;
  static_for<1, M + 1>([&](auto mt) {
    constexpr int m = decltype(mt)::value;
    float s = 0.0f;
#pragma unroll
    for (int y = 0; y < Lay::dm(m); ++y)
    {
      float c[W];
      pget(CBS + Lay::cbo(m) + y, c);
#pragma unroll
      for (int w = 0; w < W; ++w) s += c[w];
    }
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
#pragma unroll
      for (int h = 0; h < W / 4; ++h) *reinterpret_cast<f4u *>(o + 4 * h) = (f4u){v[4 * h], v[4 * h + 1], v[4 * h + 2], v[4 * h + 3]};
    } else {
#pragma unroll
      for (int w = 0; w < W; ++w)
        if (ptv[w]) o[w] = v[w];
    }
  };

  // ---- reverse sweep
  // dLoss/dCB_m of levels 1..M-1 (level M: the constant g_M), accumulated over the rows in fp64
  double Bh[Lay::nbh > 0 ? Lay::nbh : 1][W];
  static_for<1, M>([&](auto mt) {
    constexpr int m = decltype(mt)::value;
#pragma unroll
    for (int y = 0; y < Lay::dm(m); ++y)
#pragma unroll
      for (int w = 0; w < W; ++w) Bh[Lay::cbo(m) + y][w] = gw[m];
  });
  const float gM = gw[M];

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
    // inversion, ascending levels: CB_m(i) (the state before the row) and the multipliers P_m(i) in the slab
    cadd(Lay::cbo(1), dM, -1.0f);
    static_for<1, M>([&](auto mt) {
      constexpr int m = decltype(mt)::value;
      level_up(mt, dM);
      if constexpr (m + 1 < M) {  // CB_{m+1}(i) = CB_{m+1}(i+1) - colsum(R_{m+1}(i))
#pragma unroll
        for (int y = 0; y < Lay::dm(m + 1); ++y) {
          float cs[W];
          colsum(std::integral_constant<int, m + 1>{}, y, dM, cs);
          cadd(Lay::cbo(m + 1) + y, cs, -1.0f);
        }
      }
    });
    // adjoint, descending levels; Rh_m replaces P_m in the slab once used
    float Dh[W];
    {
      constexpr int dM_ = Lay::dm(M);
#pragma unroll
      for (int w = 0; w < W; ++w) Dh[w] = 0.0f;
#pragma unroll
      for (int x = 0; x < dM_; ++x)
#pragma unroll
        for (int y = 0; y < dM_; ++y) {
          float P[W];
          pget(Lay::po(M) + x * dM_ + y, P);
#pragma unroll
          for (int w = 0; w < W; ++w) Dh[w] = __builtin_fmaf(gM, P[w], Dh[w]);
          pin(Dh);
        }
    }
    static_for_desc<1, M>([&](auto mt) {
      constexpr int m = decltype(mt)::value;
      constexpr int dmv = Lay::dm(m), dn = Lay::dm(m + 1);
      // Rh_{m+1}[x][y] (level M: the constant g_M)
      auto rh = [&](int x, int y, float (&v)[W]) {
        if constexpr (m + 1 == M) {
#pragma unroll
          for (int w = 0; w < W; ++w) v[w] = gM;
        } else {
          pget(Lay::po(m + 1) + x * dn + y, v);
        }
      };
      // reverse exclusive scan over the columns of dM Rh_{m+1}[x][0] / (x+1) (x = 0: no factor)
      auto rscan = [&](int x, float (&out)[W]) {
        float q[1][W], r[1][W];
        rh(x, 0, q[0]);
#pragma unroll
        for (int w = 0; w < W; ++w) q[0][w] *= dM[w] * (x == 0 ? 1.0f : 1.0f / (float)(x + 1));
        group_rexcl_cols_n<64, W, 1>(q, r);
#pragma unroll
        for (int w = 0; w < W; ++w) out[w] = r[0][w];
      };
#pragma unroll
      for (int x = 0; x < dmv; ++x) {
        float rx1[W];
        if (x + 1 < dn) rscan(x + 1, rx1);
#pragma unroll
        for (int y = 0; y < dmv; ++y) {
          float v[W];
#pragma unroll
          for (int w = 0; w < W; ++w) v[w] = (float)Bh[Lay::cbo(m) + y][w];
          if (x + 1 < dn) {
#pragma unroll
            for (int w = 0; w < W; ++w) v[w] += rx1[w];
          }
          if (x + 1 < dn && y + 1 < dn) {
            float r[W];
            rh(x + 1, y + 1, r);
#pragma unroll
            for (int w = 0; w < W; ++w) v[w] = __builtin_fmaf(dM[w] * r[w], 1.0f / (float)((x + 2) * (y + 2)), v[w]);
          }
          if constexpr (m >= 2) {
            float P[W];
            pget(Lay::po(m) + x * dmv + y, P);
#pragma unroll
            for (int w = 0; w < W; ++w) Dh[w] = __builtin_fmaf(v[w], P[w], Dh[w]);
            pin(Dh);  // keeps the accumulation in program order (else v and P of every element stay live)
            pput(Lay::po(m) + x * dmv + y, v);  // Rh_m[x][y] for the level below
          } else {
#pragma unroll
            for (int w = 0; w < W; ++w) Dh[w] += v[w];
          }
        }
      }
      {
        float rx0[W];
        rscan(0, rx0);
#pragma unroll
        for (int y = 0; y < dmv; ++y) {
          float v[W];
#pragma unroll
          for (int w = 0; w < W; ++w) v[w] = rx0[w];
          if (y + 1 < dn) {
            float r[W];
            rh(0, y + 1, r);
#pragma unroll
            for (int w = 0; w < W; ++w) v[w] = __builtin_fmaf(dM[w] * r[w], 1.0f / (float)(y + 2), v[w]);
          }
#pragma unroll
          for (int w = 0; w < W; ++w) Bh[Lay::cbo(m) + y][w] += (double)v[w];
        }
      }
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
        dM[w] = cbuf[r][lane][w];
        k0[w] = RBF ? cbuf[r][lane][W + w] : 1.0f;
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

// one translation unit per effective order (sig_ho_bwd_lds_inst.hip)
template <int ORD>
int sig_ho_bwd_lds_launch_o(const BwdArgs &a, int seed, long long nblocks, hipStream_t s);

// (effective order, levels, points) the LDS kernel covers: the multiplier slab of W = 4 / 8 columns fits
constexpr int HO_LDS_MAX_ORD = 6;  // order 6: 6 levels at up to 256 points (W = 4: 111 slab slots, 122 KB)
inline bool ho_bwd_lds_fits(int o, int M, int l2) {
  int np = 0;
  for (int k = 1; k <= M; ++k) {
    const int d = k < o ? k : o;
    np += (k >= 2 ? d * d : 0) + d;  // multipliers of levels 2..M, column sums of levels 1..M
  }
  const int W = l2 <= 256 ? 4 : 8;
  return (size_t)np * 64 * W * sizeof(float) + ho_bwd_lds_cbuf_bytes(W) <= 160 * 1024;
}

}  // namespace gpsig
