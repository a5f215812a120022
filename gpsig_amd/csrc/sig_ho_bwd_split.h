// gpsig_amd -- the LDS-state higher-order Gram VJP (sig_ho_bwd_lds.h) with one pair split over the 4 SIMDs of a
// CU (round 5).
//
// The LDS-state kernel runs one wave per pair and per CU: its multiplier slab fills the CU's LDS, so a call with
// few pairs -- the VOSF trainer's Kff diagonal is 50 pairs of 500 points (benchmarks/models/train_gpsig_vosf.py:
// 102) -- leaves 3 of every 4 SIMDs of its CUs and most CUs idle.  Here a workgroup of NW = 4 waves owns one pair
// and wave v owns the column block j0 = 127 v .. j0 + 126 (64 lanes x W = 2 columns, the block's last column
// its halo point: the next block's first point), so the same slab is split four ways and the four SIMDs work
// on one row together.  What crosses the blocks, per row:
//   * the exclusive / reverse-exclusive column scans (the multipliers P[x][0] of level_up, the adjoint's rscans):
//     each wave scans its block and adds the totals of the blocks to its left / right, exchanged through LDS
//     with one workgroup barrier per level (all scans of a level at once);
//   * the adjoint of the second difference at a block's first point: the left neighbour's last cell;
// and once per pair the level sums K_m.  Rows, levels, formulas and numerics are those of sig_ho_bwd_lds.h
// (adjoint column sums accumulated in fp64).
#pragma once
#include "sig_ho_bwd_lds.h"

namespace gpsig {

constexpr int HO_SPLIT_NW = 4;                                // waves (column blocks) per pair
constexpr int HO_SPLIT_W = 2;                                 // columns per lane
constexpr int HO_SPLIT_CPB = 64 * HO_SPLIT_W - 1;             // cells per block
constexpr int HO_SPLIT_XN = 8;                                // values per wave and exchange (>= max order)
// Past 4 blocks (510 .. 8 x 127 + 1 points): NW = 8 waves, 2 per SIMD, and the slab (twice the LDS) in a
// per-workgroup region of global memory (BwdArgs::scratch, scr_stride floats per workgroup: L2-resident per
// CU); launches are split into at most HO_SPLIT8_BLOCKS workgroups (blk0) to bound that region.
constexpr int HO_SPLIT8_NW = 8;
constexpr long long HO_SPLIT8_BLOCKS = 1024;
template <int ORD, int M>
constexpr long long ho_split_slab_floats(int nw) {
  return (long long)nw * (HoBwdLayout<ORD, M>::np + HoBwdLayout<ORD, M>::ncb) * 64 * HO_SPLIT_W;
}
inline long long ho_split_slab_floats_rt(int o, int M, int nw) {
  int np = 0;
  for (int k = 1; k <= M; ++k) {
    const int d = k < o ? k : o;
    np += (k >= 2 ? d * d : 0) + d;
  }
  return (long long)nw * np * 64 * HO_SPLIT_W;
}
// the 8-wave form covers 510 .. 1017 points where its per-lane state fits 256 VGPRs (2 waves per SIMD) without
// spilling: levels up to 7 / 6 / 5 / 5 at effective order 2 / 3 / 4 / 5 (order 5 with the RBF seed: 20 bytes)
constexpr bool ho_split8_ok(int o, int M) { return (o == 2 && M <= 7) || (o == 3 && M <= 6) || ((o == 4 || o == 5) && M <= 5); }
inline bool ho_bwd_split8_fits(int o, int M, int l2) {
  return l2 > HO_SPLIT_NW * HO_SPLIT_CPB + 1 && l2 <= HO_SPLIT8_NW * HO_SPLIT_CPB + 1 && ho_split8_ok(o, M);
}

// (effective order, levels, points) the split kernel covers: 257 .. 4 x 127 + 1 points (wide records padded
// to 512 columns, so every block's 128 columns lie in the record) and the slab of W = 8 fits
inline bool ho_bwd_split_fits(int o, int M, int l2) {
  int np = 0;
  for (int k = 1; k <= M; ++k) {
    const int d = k < o ? k : o;
    np += (k >= 2 ? d * d : 0) + d;
  }
  const size_t lds = (size_t)np * 64 * 8 * sizeof(float) + ho_bwd_lds_cbuf_bytes(8) + 2 * HO_SPLIT_NW * HO_SPLIT_XN * 4;
  return l2 > 256 && l2 <= HO_SPLIT_NW * HO_SPLIT_CPB + 1 && lds <= 160 * 1024;
}
template <int ORD, int M>
constexpr size_t ho_bwd_split_slab_bytes() {
  return (size_t)HO_SPLIT_NW * (ho_lds_np<ORD, M>() + HoBwdLayout<ORD, M>::ncb) * 64 * HO_SPLIT_W * sizeof(float);
}

template <int ORD, int M, int SEED, int NW = HO_SPLIT_NW>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(NW / 4))) void sig_ho_bwd_split_kernel(
    BwdArgs p) {
  constexpr int W = HO_SPLIT_W, W2 = W / 2, CPB = HO_SPLIT_CPB, XN = HO_SPLIT_XN;
  constexpr bool GLB = NW > HO_SPLIT_NW;  // the slab in global memory
  constexpr int RC = GPSIG_WIDE_BWD_R;
  constexpr bool RBF = SEED == SEED_RBF_DIFF;
  static_assert(SEED == SEED_RBF_DIFF || SEED == SEED_LIN_DIFF, "higher order: difference seeds");
  static_assert(M >= 2 && ORD >= 2 && ORD <= M, "higher order");
  using Lay = HoBwdLayout<ORD, M>;
  static_assert(Lay::dm(M) <= XN, "exchange width");
  using Seed = WideSeed<W, RC, SEED>;
  __shared__ __attribute__((aligned(16))) float cbuf[NW][RC][64][2 * W];
  __shared__ float xbuf[2][NW][XN];  // per-wave totals of the current exchange (double-buffered)
  extern __shared__ __attribute__((aligned(16))) float pslab[];

  const int lane = threadIdx.x & 63;
  const int wave = wave_uniform((int)threadIdx.x >> 6);
  const bool diag = p.pair_mode == GPSIG_PAIRS_DIAG;
  const long long lblk = p.blk0 + (long long)blockIdx.x;

  // ---- which pair: one per workgroup
  int a, b;
  if (diag) {
    a = p.row_begin + (int)lblk;
    b = a;
  } else if (p.pair_mode == GPSIG_PAIRS_UPPER) {
    const Tile t = upper_tile(p.tile_base + lblk, p.n2, 1);
    a = t.ta;
    b = t.tb;
  } else {
    a = p.row_begin + (int)(lblk / p.n2);
    b = (int)(lblk % p.n2);
  }
  if (a < p.row_begin || a >= p.row_end || b >= p.n2) return;  // the whole workgroup
  if (p.pair_mode == GPSIG_PAIRS_UPPER && !p.rs1 && !p.gscale) {  // no upstream gradient (sig_ho_bwd_lds.h)
    const PairTerms<M> pt0(p, a, b, lane, true, lblk);
    float g0[M + 1];
    pt0.weights(g0);
    bool any = false;
#pragma unroll
    for (int m = 1; m <= M; ++m) any = any || g0[m] != 0.0f;
    if (!any) return;
  }
  const int l1 = p.l1, l2 = p.l2;
  const int j0 = wave * CPB;  // this wave's column block
  const float *__restrict__ fx = p.FX + (long long)a * p.sx;
  const float *__restrict__ fy = p.FY + (long long)b * p.sy;
  cfloat *fxc = as_const(fx);
  const int nrows = l1 - 1;
  const int bpts = l2 - j0 < CPB + 1 ? (l2 - j0 > 1 ? l2 - j0 : 1) : CPB + 1;  // the block's points (halo incl.)

  Seed seed;
  seed.init(p.wd, p.lw1, p.lw2, fx, fy + j0, lane, bpts);
  if constexpr (RBF) {
    // the |dx||dy| bound over the whole pair: every block takes the same polynomial (wave max, then blocks)
    seed.bound_c(nrows);
    if (lane == 0) xbuf[1][wave][0] = seed.clo ? 1.0f : 0.0f;
    __syncthreads();
    bool all = true;
#pragma unroll
    for (int u = 0; u < NW; ++u) all = all && xbuf[1][u][0] != 0.0f;
    seed.clo = all;
    __syncthreads();
  }
  bool colv[W], ptv[W];
#pragma unroll
  for (int w = 0; w < W; ++w) {
    const int jj = lane * W + w;
    colv[w] = jj < CPB && j0 + jj < l2 - 1;
    ptv[w] = j0 + jj < l2 && (jj < CPB || wave == NW - 1);  // a block's halo point is the next block's first
  }

  // cross-block exchange: N per-wave values (uniform in the wave) -> every wave's values; one barrier.  The
  // values stay in LDS (broadcast reads, xget) rather than NW x N registers.
  int ph = 0;
  auto exchange = [&](auto nt, const float *mine) {
    constexpr int N = decltype(nt)::value;
    if (lane == 0)
#pragma unroll
      for (int n = 0; n < N; ++n) xbuf[ph][wave][n] = mine[n];
    __syncthreads();
    const int cur = ph;
    ph ^= 1;
    return cur;
  };
  auto xget = [&](int buf, int u, int n) { return xbuf[buf][u][n]; };
  // exclusive (REV: reverse exclusive) scans over the pair's columns of N arrays: in-lane, over the wave, then
  // the totals of the blocks to the left (right)
  auto scan_cols = [&](auto nt, auto rev, const float (*v)[W], float (*out)[W]) {
    constexpr int N = decltype(nt)::value;
    constexpr bool REV = decltype(rev)::value;
    float t[N], incl[N], tot[N];
#pragma unroll
    for (int n = 0; n < N; ++n) {
      float s = 0.0f;
#pragma unroll
      for (int w = 0; w < W; ++w) s += v[n][w];
      t[n] = s;
      incl[n] = s;
    }
    group_incl_scan_n<64, N>(incl);
#pragma unroll
    for (int n = 0; n < N; ++n) tot[n] = __shfl(incl[n], 63, 64);
    const int xb = exchange(nt, tot);
#pragma unroll
    for (int n = 0; n < N; ++n) {
      float off = 0.0f;
#pragma unroll
      for (int u = 0; u < NW; ++u) {
        if constexpr (!GLB) {  // unconditional reads (batched after the barrier), predicated adds
          const float t = xget(xb, u, n);
          off += (REV ? u > wave : u < wave) ? t : 0.0f;
        } else {  // the 8-wave form: reads under the branch (fewer live values at its 256-VGPR cap)
          if (REV ? u > wave : u < wave) off += xget(xb, u, n);
        }
      }
      if constexpr (!REV) {
        float run = off + (incl[n] - t[n]);
#pragma unroll
        for (int w = 0; w < W; ++w) {
          out[n][w] = run;
          run += v[n][w];
        }
      } else {
        float run = off + (tot[n] - incl[n]);
#pragma unroll
        for (int w = W - 1; w >= 0; --w) {
          out[n][w] = run;
          run += v[n][w];
        }
      }
    }
  };

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
        for (int w = 0; w < W; ++w) cbuf[wave][r][lane][W + w] = seed.kc[w % W2][w / W2];
        if (seed.clo)
          seed.template row<true>(rd, false, dM);
        else
          seed.template row<false>(rd, false, dM);
      } else {
        seed.template row<false>(rd, false, dM);
      }
#pragma unroll
      for (int w = 0; w < W; ++w) cbuf[wave][r][lane][w] = colv[w] ? dM[w % W2][w / W2] : 0.0f;
    };
    one(std::integral_constant<int, 0>{});
    if constexpr (RC > 1) one(std::integral_constant<int, 1>{});
    if constexpr (RC > 2) one(std::integral_constant<int, 2>{});
    if constexpr (RC > 3) one(std::integral_constant<int, 3>{});
  };


  // the 8-wave form pins the adjoint accumulator between slab accesses (bounds its registers at 256); the 4-wave
  // form, at one wave per SIMD, lets the compiler schedule it freely (VJP 4.94 -> 4.59 ms at the VOSF shape)
  auto pin = [&](float (&v)[W]) {
    if constexpr (GLB) {
#pragma unroll
      for (int w = 0; w < W; ++w) asm volatile("" : "+v"(v[w]));
    }
  };
  // this wave's part of the multiplier slab: slot s of this lane's W columns
  float *__restrict__ slab = GLB ? p.scratch + (long long)blockIdx.x * p.scr_stride : pslab;
  float *__restrict__ ps = slab + (long long)wave * (Lay::np + Lay::ncb) * 64 * W + lane * W;
  // no compiler barriers around the slab accesses here (the one-wave kernel needs them to bound its register
  // use at W = 8): each lane touches only its own columns, so the compiler may batch a level's LDS reads
  // ahead of their use instead of paying each read's latency in turn
  // (the 8-wave form, 2 waves per SIMD at <= 256 VGPRs, keeps the barriers: unfenced, its global slab reads are
  // hoisted past the register file)
  auto pget = [&](int slot, float (&v)[W]) {
    if constexpr (GLB) asm volatile("" ::: "memory");
    const f2 t = *reinterpret_cast<const f2 *>(ps + (long long)slot * 64 * W);
    v[0] = t[0];
    v[1] = t[1];
  };
  auto pput = [&](int slot, const float (&v)[W]) {
    *reinterpret_cast<f2 *>(ps + (long long)slot * 64 * W) = (f2){v[0], v[1]};
    if constexpr (GLB) asm volatile("" ::: "memory");
  };
  constexpr int CBS = Lay::np;
  auto cadd = [&](int k, const float (&v)[W], float sgn) {
    float c[W];
    pget(CBS + k, c);
#pragma unroll
    for (int w = 0; w < W; ++w) c[w] = __builtin_fmaf(sgn, v[w], c[w]);
    pput(CBS + k, c);
  };
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

  // level m+1's multipliers P (row i) into the slab, from CB_m (rows < i) and the row's R_m; the dn column
  // scans of the level run together (one exchange)
  auto level_up = [&](auto mt, const float (&dM)[W]) {
    constexpr int m = decltype(mt)::value;
    constexpr int dmv = Lay::dm(m), dn = Lay::dm(m + 1);
    constexpr int base = Lay::po(m + 1);
    float in[dn][W], ex[dn][W];
#pragma unroll
    for (int x = 0; x < dn; ++x) {
#pragma unroll
      for (int w = 0; w < W; ++w) in[x][w] = 0.0f;
#pragma unroll
      for (int y = 0; y < dmv; ++y) {
        float r[W];
        if (x == 0) {
          pget(CBS + Lay::cbo(m) + y, r);
        } else {
          rget(mt, x - 1, y, dM, r);
        }
#pragma unroll
        for (int w = 0; w < W; ++w) in[x][w] += r[w];
        if (y + 1 < dn) {  // P[x][y+1] = (x ? R[x-1][y] : CB[y]) / ((x+1)(y+2))
#pragma unroll
          for (int w = 0; w < W; ++w) r[w] *= 1.0f / (float)((x + 1) * (y + 2));
          pput(base + x * dn + y + 1, r);
        }
      }
    }
    scan_cols(std::integral_constant<int, dn>{}, std::false_type{}, in, ex);
#pragma unroll
    for (int x = 0; x < dn; ++x) {
#pragma unroll
      for (int w = 0; w < W; ++w) ex[x][w] *= 1.0f / (float)(x + 1);
      pput(base + x * dn, ex[x]);
    }
  };
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
      for (int w = 0; w < W; ++w) dM[w] = cbuf[wave][r][lane][w];
      static_for<1, M + 1>([&](auto mt) {
        constexpr int m = decltype(mt)::value;
        if constexpr (m < M) level_up(mt, dM);
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
  {
    float ks[XN];
    static_for<1, M + 1>([&](auto mt) {
      constexpr int m = decltype(mt)::value;
      float s = 0.0f;
#pragma unroll
      for (int y = 0; y < Lay::dm(m); ++y) {
        float c[W];
        pget(CBS + Lay::cbo(m) + y, c);
#pragma unroll
        for (int w = 0; w < W; ++w) s += c[w];
      }
      ks[(m - 1) % XN] = group_sum<64>(s);
      if constexpr (m % XN == 0 || m == M) {  // the blocks' sums, XN levels per exchange
        constexpr int n0 = ((m - 1) / XN) * XN, cnt = m - n0;
        const int xb = exchange(std::integral_constant<int, cnt>{}, ks);
#pragma unroll
        for (int n = 0; n < cnt; ++n) {
          float t = 0.0f;
#pragma unroll
          for (int u = 0; u < NW; ++u) t += xget(xb, u, n);
          K[n0 + n + 1] = t;
        }
      }
    });
  }
  K[1] = level1_closed_wide<SEED>(fx, fy, p.wd, p.lw1, p.lw2, l1, l2);

  const PairTerms<M> pt(p, a, b, lane, true, lblk);
  float gw[M + 1];
  pt.weights(gw);

  // ---- point weights of this pair into the tile: this block's points j0 .. j0 + 126
  float *__restrict__ tpair = p.tile + (long long)(a - p.tile_a0) * p.tile_as +
                              (diag ? 0 : (long long)(b - p.tile_b0) * l2) + j0 + lane * W;
  auto emit = [&](int pi, const float (&Kh)[W], const float (&kr)[W]) {
    float *__restrict__ o = tpair + (long long)pi * p.tile_ld;
#pragma unroll
    for (int w = 0; w < W; ++w)
      if (ptv[w]) o[w] = RBF ? Kh[w] * kr[w] : Kh[w];
  };

  // ---- reverse sweep
  double Bh[Lay::nbh > 0 ? Lay::nbh : 1][W];  // dLoss/dCB_m of levels 1..M-1, accumulated in fp64
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
    // inversion, ascending levels
    cadd(Lay::cbo(1), dM, -1.0f);
    static_for<1, M>([&](auto mt) {
      constexpr int m = decltype(mt)::value;
      level_up(mt, dM);
      if constexpr (m + 1 < M) {
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
      auto rh = [&](int x, int y, float (&v)[W]) {
        if constexpr (m + 1 == M) {
#pragma unroll
          for (int w = 0; w < W; ++w) v[w] = gM;
        } else {
          pget(Lay::po(m + 1) + x * dn + y, v);
        }
      };
      // every reverse exclusive scan of the level at once: rs[x] = rexcl_j(dM Rh_{m+1}[x][0] / (x ? x+1 : 1))
      float q[dn][W], rs[dn][W];
#pragma unroll
      for (int x = 0; x < dn; ++x) {
        rh(x, 0, q[x]);
#pragma unroll
        for (int w = 0; w < W; ++w) q[x][w] *= dM[w] * (x == 0 ? 1.0f : 1.0f / (float)(x + 1));
      }
      scan_cols(std::integral_constant<int, dn>{}, std::true_type{}, q, rs);
#pragma unroll
      for (int x = 0; x < dmv; ++x) {
#pragma unroll
        for (int y = 0; y < dmv; ++y) {
          float v[W];
#pragma unroll
          for (int w = 0; w < W; ++w) v[w] = (float)Bh[Lay::cbo(m) + y][w];
          if (x + 1 < dn) {
#pragma unroll
            for (int w = 0; w < W; ++w) v[w] += rs[x + 1][w];
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
            pin(Dh);
            pput(Lay::po(m) + x * dmv + y, v);
          } else {
#pragma unroll
            for (int w = 0; w < W; ++w) Dh[w] += v[w];
          }
        }
      }
#pragma unroll
      for (int y = 0; y < dmv; ++y) {
        float v[W];
#pragma unroll
        for (int w = 0; w < W; ++w) v[w] = rs[0][w];
        if (y + 1 < dn) {
          float r[W];
          rh(0, y + 1, r);
#pragma unroll
          for (int w = 0; w < W; ++w) v[w] = __builtin_fmaf(dM[w] * r[w], 1.0f / (float)(y + 2), v[w]);
        }
#pragma unroll
        for (int w = 0; w < W; ++w) Bh[Lay::cbo(m) + y][w] += (double)v[w];
      }
    });
#pragma unroll
    for (int w = 0; w < W; ++w) Dh[w] = colv[w] ? Dh[w] : 0.0f;
    // adjoint of the second difference (signature_algs.py:26): E(i, j) = Dh(i, j-1) - Dh(i, j); at the block's
    // first point Dh(i, j0 - 1) is the left block's last cell (lane 63, column 0)
    float mine[1] = {__shfl(Dh[0], 63, 64)};
    const int xb = exchange(std::integral_constant<int, 1>{}, mine);
    float left = lane_prev(Dh[W - 1]);
    if (lane == 0) left = wave > 0 ? xget(xb, wave > 0 ? wave - 1 : 0, 0) : 0.0f;
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
        dM[w] = cbuf[wave][r][lane][w];
        k0[w] = RBF ? cbuf[wave][r][lane][W + w] : 1.0f;
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
  if (wave == 0) pt.norm(K);
}

}  // namespace gpsig
