// gpsig_amd -- first-order truncated signature kernel Gram on gfx950 (kernel template).
//
// Replaces, for order == 1, the dataflow of gpsig/kernels.py:209-238 (_K_seq) +
// gpsig/signature_algs.py:8-35 (signature_kern_first_order):
//     dM = second difference of the base-kernel grid M(x_i, y_j)        (signature_algs.py:26)
//     K_1 = sum dM,  R_m = dM * cumsum_x(cumsum_x(R_{m-1})), K_m = sum R_m   (:28-33)
// without materialising M or R: a group of LP lanes owns one pair (a, b) and streams the rows i of
// the dM grid; each lane keeps W columns j.  Per row and level, the exclusive 2-D prefix
// S_m(i, j) = sum_{i'<i, j'<j} R_m(i', j') is the exclusive scan over j of the running column sums
// C_m(j) = sum_{i'<i} R_m(i', j): per pair the state is M x W registers per lane and the only
// cross-lane traffic is one DPP scan per level per row (the M-1 scans of a row are independent, so
// they interleave).  K_m = sum_j C_m(j) at the end.  The seed (base-kernel second difference,
// including the fp32-stable RBF form) is RowSeed in sig_common.h.
#pragma once
#include <type_traits>

#include "sig_common.h"
#include "wide.h"

namespace gpsig {

// Rows per channel-loop chunk of the wide-channel seeds (DP == 0, wide.h): each channel's y columns are
// loaded once per chunk, so the loop's loads per FMA fall as 1/R.  Measured (N = 1024, L = 128, M = 4,
// tools/ab_wide_r.sh): R = 4 -> 8 takes D = 46 from 56.9 to 32.5 ms and D = 126 from 153.6 to 83.6 ms
// (251 VGPRs, 2 waves/SIMD; the loop was load-bound, VALU busy 0.21 at R = 4).
#ifndef GPSIG_WIDE_R
#define GPSIG_WIDE_R 8
#endif
constexpr int WIDE_R = GPSIG_WIDE_R;

// DIAGK: the diagonal pass (pairs (a, a)) is the same body under its own symbol, so profiler
// statistics of the Gram launch are not mixed with it.  SAVE: also write the VJP's saved state
// (gpsig_sig_gram_state) -- a separate instantiation, so the plain Gram keeps its register budget.
// MF: the increment inner products of the RBF seed on the matrix cores (RbfSeedPk::mfma_pc), 4 rows
// per batch, instead of packed VALU dots.
// SPLIT (diagnostic, SURVEY.md 8d "split design"): 1 = producer (cells dM of every row to p.dmbuf, no
// recursion, no output), 2 = consumer (cells streamed from p.dmbuf through the recursion and epilogue).
// Waves per SIMD the register allocation must leave room for: 2 (256 VGPRs) where W = 8 columns per lane
// only just fit at D = 7..8 (the allocator would otherwise take 260 and run one wave per SIMD, 1.6x
// slower; at 256 it spills a few registers outside the row loop).
// per-row record type of the row loop: the seed's own (wide, packed RBF) or the generic RowData
template <bool WIDE, bool PK, class PS, int DP, int W>
struct FoRec { using type = RowData<DP>; };
template <bool PK, class PS, int DP, int W>
struct FoRec<true, PK, PS, DP, W> { using type = typename PS::Row; };
template <class PS, int DP, int W>
struct FoRec<false, true, PS, DP, W> { using type = typename RbfSeedPk<DP, W>::Row; };

__host__ __device__ constexpr int fo_waves(int DP, int W, int M) { return ((W == 8 && DP > 6 && M <= 6) || W == 10) ? 2 : 1; }

template <int DP, int W, int LP, int M, int SEED, bool DIAGK, bool SAVE = false, bool MF = false, int SPLIT = 0>
#ifdef GPSIG_FO_LB
#define GPSIG_FO_BOUNDS __launch_bounds__(256, GPSIG_FO_LB)
#else
#define GPSIG_FO_BOUNDS __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(fo_waves(DP, W, M))))
#endif
__global__ GPSIG_FO_BOUNDS void sig_fo_kernel(SigArgs p) {
  // DP == 0: wide channel counts (runtime p.wd, channel-major records, wide.h)
  constexpr bool WIDE = DP == 0;
  constexpr bool DIFF = SEED == SEED_RBF_DIFF || SEED == SEED_LIN_DIFF;
  constexpr int FS = feat_stride(DP);
  constexpr int G = 64 / LP;
  // SEG: lane groups not aligned to DPP rows (LP = 10: G = 6 pairs per wave, lanes 60..63 idle)
  constexpr bool SEG = (64 % LP) != 0;

  const int lane = threadIdx.x & 63;
  const int wave = wave_uniform(threadIdx.x >> 6);
  const int g = lane / LP;
  const int gl = lane % LP;

  // ---- which pair
  int a, b;
  if (DIAGK) {
    a = p.row_begin + (int)blockIdx.x * 4 + wave;
    b = a;
    if (a >= p.row_end) return;
  } else {
    int ta, tb;
    const long long lblk = p.blk0 + (long long)blockIdx.x;
    if (p.pair_mode == GPSIG_PAIRS_UPPER) {
      Tile t;
      if constexpr (SEG)
        t = upper_tile_g<G>(p.tile_base + lblk, p.ntb);
      else
        t = upper_tile(p.tile_base + lblk, p.ntb, 4 / G);
      ta = t.ta;
      tb = t.tb;
    } else {
      ta = p.tiles_a0 + (int)(lblk / p.ntb);
      tb = (int)(lblk % p.ntb);
    }
    a = ta * 4 + wave;
    b = tb * G + (SEG && g >= G ? G - 1 : g);  // the idle lanes shadow the last group's pair
    if (a < p.row_begin || a >= p.row_end) return;  // wave-uniform
  }
  static_assert(SPLIT == 0 || (!DIAGK && !SAVE && !MF && SEED == SEED_RBF_DIFF), "split: RBF Gram pairs only");
  static_assert(!WIDE || (SPLIT == 0 && !MF), "wide channels: fused VALU seed");
  // split: this pair's cell slab, [row][lane of the group][W] (each lane's W cells contiguous)
  float *__restrict__ dms = nullptr;
  if constexpr (SPLIT != 0)
    dms = p.dmbuf + (((long long)blockIdx.x * 4 + wave) * G + g) * (long long)(p.l1 - 1) * (LP * W) + (long long)gl * W;
  bool pair_ok = b < p.n2;
  if (p.pair_mode == GPSIG_PAIRS_UPPER) pair_ok = pair_ok && b >= a;
  if (SEG) pair_ok = pair_ok && g < G;
  if (DIAGK) pair_ok = (g == 0);
  const int bl = b < p.n2 ? b : p.n2 - 1;

  const float *__restrict__ fx = p.FX + (WIDE ? (long long)a * p.sx : (long long)a * p.l1 * FS);
  const float *__restrict__ fy = p.FY + (WIDE ? (long long)bl * p.sy : (long long)bl * p.l2 * FS);

  constexpr bool PK = (SEED == SEED_RBF_DIFF) && !WIDE;
  using PSeed = std::conditional_t<WIDE, WideSeed<W, WIDE_R, SEED>,
                                   std::conditional_t<PK, RbfSeedPk<DP, W>, RowSeed<DP, W, SEED>>>;
  constexpr int W2 = W / 2;
  constexpr int ML = M > 1 ? M - 1 : 1;
  const int nrows = DIFF ? p.l1 - 1 : p.l1;

  // Column blocks (sequences longer than one lane group covers, LP = 64 only): block k holds the
  // cells j0 .. j0 + CPB - 1 (j0 = k CPB) on the points j0 .. j0 + CPB (the last lane's last column is
  // the block's right halo point, its cell is masked), streamed over all rows before the next block.
  // The exclusive column prefix of block k adds the carry c_m(i) = sum_{j < j0} C_m(i, j) of the blocks
  // to its left, one float per row and level kept in this wave's LDS slab (written by block k-1,
  // read and advanced by block k).
  constexpr int CPB = LP * W - 1;
  const int nblk = (LP == 64) ? p.nblk : 1;
  extern __shared__ float fo_carry[];
  float *__restrict__ carry = fo_carry + (long long)wave * nrows * ML;

  float Kacc[M];
#pragma unroll
  for (int m = 0; m < M; ++m) Kacc[m] = 0.0f;
  using SegF = std::conditional_t<SEG, SegFactors<SEG ? LP : 10>, char>;
  const SegF segf{};

  for (int blk = 0; blk < nblk; ++blk) {
    const int j0 = blk * CPB;
    // points of this block: the DIFF seeds see the halo point, the point seeds do not
    const int npts = nblk == 1 ? p.l2 : min(p.l2 - j0, DIFF ? CPB + 1 : CPB);
    PSeed seed;
    if constexpr (WIDE)
      seed.init(p.wd, p.lw1, p.lw2, fx, fy + j0, gl, npts);
    else
      seed.init(fx, fy + (long long)j0 * FS, gl, npts);
#ifndef GPSIG_CLO
#define GPSIG_CLO 1
#endif
    if constexpr (PK && !MF && SPLIT != 2 && GPSIG_CLO) seed.bound_c(fx, nrows);
    if constexpr (WIDE && SEED == SEED_RBF_DIFF && GPSIG_CLO) seed.bound_c(nrows);
    // DIAG: the pair's seed tiles (wide.h DiagTiles) replace the chunk dots' and the anchors' channel loops
    bool tiled = false;
    if constexpr (WIDE && SEED == SEED_RBF_DIFF && DIAGK) {
      if (p.dtile && nblk == 1) {
        const float *base = p.dtile + (long long)(a - p.dt_a0) * p.dt_pair;
        seed.set_tiles(base, base + p.dt_rows * p.dt_ld, base + 2 * p.dt_rows * p.dt_ld, p.dt_ld, gl, DIAG_TILE_ANCHOR,
                       (int)(p.dt_rows / DIAG_TILE_ANCHOR));
        tiled = true;
      }
    }

    f2 C[M][W2];
#pragma unroll
    for (int m = 0; m < M; ++m)
#pragma unroll
      for (int w2 = 0; w2 < W2; ++w2) C[m][w2] = splat2(0.0f);

    // One row: seed cells, then the level recursion.  S_m = exclusive prefix over (rows < i, cols < j)
    // of R_m = exclusive scan over j of C_m; the M-1 scans are independent and interleave.
    using Rec = typename FoRec<WIDE, PK, PSeed, DP, W>::type;
    auto do_row = [&](auto clo_t, int i, const Rec &rd, bool anch, const f2 *pc = nullptr) {
      f2 dM[W2];
      if constexpr (SPLIT == 2) {
        const f4 *src = reinterpret_cast<const f4 *>(dms + (long long)i * (LP * W));
#pragma unroll
        for (int w4 = 0; w4 < W / 4; ++w4) {
          const f4 v = __builtin_nontemporal_load(src + w4);
          dM[2 * w4] = (f2){v[0], v[1]};
          dM[2 * w4 + 1] = (f2){v[2], v[3]};
        }
      } else if constexpr (WIDE) {
        seed.template row<decltype(clo_t)::value>(rd, anch, dM);
      } else if constexpr (PK) {
        if (MF && pc) {
          f2 pp[W2], cc[W2];
#pragma unroll
          for (int w2 = 0; w2 < W2; ++w2) {
            pp[w2] = pc[w2];
            cc[w2] = pc[W2 + w2];
          }
          seed.row_pc(rd, anch, pp, cc, dM);
        } else {
          seed.template row<decltype(clo_t)::value>(rd, anch, dM);
        }
      } else {
        float d1[W];
        seed.template row<true>(rd, d1);
#pragma unroll
        for (int w2 = 0; w2 < W2; ++w2) dM[w2] = (f2){d1[w2], d1[w2 + W2]};
      }
      if constexpr (SPLIT == 1) {
        f4 *dst = reinterpret_cast<f4 *>(dms + (long long)i * (LP * W));
#pragma unroll
        for (int w4 = 0; w4 < W / 4; ++w4)
          __builtin_nontemporal_store((f4){dM[2 * w4][0], dM[2 * w4][1], dM[2 * w4 + 1][0], dM[2 * w4 + 1][1]}, dst + w4);
        return;
      }
      // Column pair k of a lane holds columns (k, k + W/2), so the in-lane exclusive prefix runs on both
      // halves at once: E_k = P_0 + ... + P_{k-1} (packed), E_{W/2} = (H_lo, H_hi) the half totals, and
      // S_m(column) = E_k + (b, b + H_lo) with b the exclusive cross-lane prefix of T = H_lo + H_hi.
      // The lane totals of the M-1 levels are scanned across the group together.
      f2 E[ML][W2 + 1];
      float T[ML], base[ML];
#pragma unroll
      for (int m = 0; m + 1 < M; ++m) {
        E[m][1] = C[m][0];
#pragma unroll
        for (int k = 2; k <= W2; ++k) E[m][k] = E[m][k - 1] + C[m][k - 1];
        T[m] = E[m][W2][0] + E[m][W2][1];
        base[m] = T[m];
      }
      if constexpr (M > 1) {
        if constexpr (SEG)
          seg_incl_scan_n<LP, ML>(base, segf);
        else
          group_incl_scan_n<LP, ML>(base);
      }
      if constexpr (LP == 64 && M > 1) {
        if (nblk > 1) {  // wave-uniform: carry in from the blocks to the left, carry out to the right
          float *__restrict__ cr = carry + (long long)i * ML;
#pragma unroll
          for (int m = 0; m < ML; ++m) {
            const float cin = blk > 0 ? cr[m] : 0.0f;
            const float tot = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, base[m]), 63));
            if (blk + 1 < nblk && lane == 0) cr[m] = cin + tot;
            base[m] += cin;
          }
        }
      }
      // descending m: level m reads C_m (through E) before level m-1's update writes it
#pragma unroll
      for (int m = M - 2; m >= 0; --m) {
        f2 off;
        off[0] = base[m] - T[m];
        off[1] = off[0] + E[m][W2][0];
        C[m + 1][0] = fma2(dM[0], off, C[m + 1][0]);
#pragma unroll
        for (int k = 1; k < W2; ++k) C[m + 1][k] = fma2(dM[k], E[m][k] + off, C[m + 1][k]);
      }
#pragma unroll
      for (int w2 = 0; w2 < W2; ++w2) C[0][w2] += dM[w2];
    };
    // Row loop.  For the packed RBF seed the row recurrences are re-anchored every ANCH rows (a
    // wave-uniform branch); the other seeds evaluate every row directly.  The saved-state launch of a
    // training step uses the same period, so it writes the inference launch's Gram bit for bit (the
    // VJP, which regenerates its cells from an exact row every 4 rows, inverts the saved sums with
    // cells that differ from these by the recurrences' rounding drift, ~1e-7 relative).
    constexpr int ANCH = PSeed::ANCHOR;
#ifndef GPSIG_FO_UNROLL2
#define GPSIG_FO_UNROLL2 (W <= 4)
#endif
    int i = 0;
    if constexpr (PK && MF) {
      static_assert(ANCH % 4 == 0, "anchor period");
      for (; i + 4 <= nrows; i += 4) {
        f4 P[W], Q[W];
        seed.mfma_pc(fx, i, P, Q);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          Rec rd;
          rd.load(fx, i + r);
          f2 pc[2 * W2];
#pragma unroll
          for (int w2 = 0; w2 < W2; ++w2) {
            pc[w2] = (f2){P[w2][r], P[w2 + W2][r]};
            pc[W2 + w2] = (f2){Q[w2][r], Q[w2 + W2][r]};
          }
          do_row(std::false_type{}, i + r, rd, r == 3 && ((i + 3) % ANCH) == ANCH - 1, pc);
        }
      }
    }
    // the rest of the rows, in a copy per Ec polynomial (the pair block's |c| bound, bound_c)
    auto run_rows = [&](auto clo_t) {
      if constexpr (WIDE) {
        // chunks of WIDE_R rows: one channel loop for their dots, then the rows (compile-time slots)
        for (; i < nrows; i += WIDE_R) {
          if constexpr (SEED == SEED_RBF_DIFF) {
            if (tiled)
              seed.chunk_tile(i);
            else
              seed.chunk(i);
          } else {
            seed.chunk(i);
          }
          auto one = [&](auto rr) {
            constexpr int r = decltype(rr)::value;
            if (i + r < nrows) {
              const Rec rd = seed.template row_of<r>(i + r);
              do_row(clo_t, i + r, rd, ((i + r) % ANCH) == ANCH - 1);
            }
          };
          one(std::integral_constant<int, 0>{});
          if constexpr (WIDE_R > 1) one(std::integral_constant<int, 1>{});
          if constexpr (WIDE_R > 2) one(std::integral_constant<int, 2>{});
          if constexpr (WIDE_R > 3) one(std::integral_constant<int, 3>{});
          if constexpr (WIDE_R > 4) one(std::integral_constant<int, 4>{});
          if constexpr (WIDE_R > 5) one(std::integral_constant<int, 5>{});
          if constexpr (WIDE_R > 6) one(std::integral_constant<int, 6>{});
          if constexpr (WIDE_R > 7) one(std::integral_constant<int, 7>{});
        }
      } else {
      if constexpr (PK && GPSIG_FO_UNROLL2 && !MF) {
        // row pairs: ANCHOR is even, so the first row of a pair never anchors (compile-time)
        static_assert(ANCH % 2 == 0, "anchor period");
        for (; i + 2 <= nrows; i += 2) {
          Rec r0, r1;
          r0.load(fx, i);
          r1.load(fx, i + 1);
          do_row(clo_t, i, r0, false);
          do_row(clo_t, i + 1, r1, ((i + 1) % ANCH) == ANCH - 1);
        }
      }
      for (; i < nrows; ++i) {
        Rec rd;
        bool anch = true;
        if constexpr (PK) {
          rd.load(fx, i);
          anch = (i % ANCH) == ANCH - 1;
        } else {
          rd.load(fx, i, SEED);
        }
        do_row(clo_t, i, rd, anch);
      }
      }
    };
    if constexpr ((PK && !MF && SPLIT != 2) || (WIDE && SEED == SEED_RBF_DIFF)) {
      if (seed.clo)
        run_rows(std::true_type{});
      else
        run_rows(std::false_type{});
    } else {
      run_rows(std::false_type{});
    }

    // ---- saved VJP state (gpsig_sig_gram_state): column sums of levels 1..M-1 (column pair k holds
    // columns k, k + W/2), before the epilogue so it adds no live registers there
    static_assert(!SAVE || (!DIAGK && DIFF), "saved state: Gram pairs of a DIFF seed");
    if constexpr (SAVE) {
      if (pair_ok) {
        const int nc = p.l2 - 1;
        float *__restrict__ st = p.state + state_slot(a, b, p.n2, p.pair_mode == GPSIG_PAIRS_UPPER) * state_stride(M, p.l2);
#pragma unroll
        for (int m = 0; m + 1 < M; ++m)
#pragma unroll
          for (int w2 = 0; w2 < W2; ++w2)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const int jl = gl * W + w2 + h * W2;
              const int j = j0 + jl;
              if (j < nc && jl < CPB) st[(long long)m * nc + j] = C[m][w2][h];
            }
      }
    }

    // ---- this block's share of K_m = sum_j C_m(j)
#pragma unroll
    for (int m = 0; m < M; ++m) {
      f2 s2 = C[m][0];
#pragma unroll
      for (int w2 = 1; w2 < W2; ++w2) s2 += C[m][w2];
      if constexpr (SEG)
        Kacc[m] += seg_group_sum<LP>(s2[0] + s2[1], segf);
      else
        Kacc[m] += group_sum<LP>(s2[0] + s2[1]);
    }
  }

  if constexpr (SPLIT == 1) return;  // the producer stores no output
  // ---- epilogue
  float K[M + 1];
  K[0] = 1.0f;
#pragma unroll
  for (int m = 0; m < M; ++m) K[m + 1] = Kacc[m];
  if (gl == 0 && pair_ok) {
    if constexpr (DIFF) {
      if constexpr (WIDE)
        K[1] = level1_closed_wide<SEED>(fx, fy, p.wd, p.lw1, p.lw2, p.l1, p.l2);
      else
        K[1] = level1_closed<DP, SEED>(fx, fy, p.l1, p.l2);
    }
    store_pair<M>(p, a, b, K);
    if constexpr (SAVE) {  // raw levels K_1..K_M after the column sums
      float *__restrict__ st = p.state + state_slot(a, b, p.n2, p.pair_mode == GPSIG_PAIRS_UPPER) * state_stride(M, p.l2) +
                               (long long)(M - 1) * (p.l2 - 1);
#pragma unroll
      for (int m = 1; m <= M; ++m) st[m - 1] = K[m];
    }
  }
}

// Column geometry: W columns per lane, LP lanes per pair; capacity LP*W >= points per sequence.
// The lane keeps 2*W*DP column floats (y, dy) in VGPRs, so wide channel counts take fewer columns per
// lane (more lanes per pair): W*DP <= 64 keeps the kernel within 256 VGPRs.
struct Geo { int W, LP; };
// W = 8 only while the kernel stays within 256 VGPRs (no AGPR spill): measured on MI355X with
// tools/kbench.hip, W = 8 / LP = 16 beats W = 4 / LP = 32 by 8-18 % when it fits and loses 30-50 % when
// it does not.  With the points of column pairs >= 1 re-read on anchor rows (RbfSeedPk::YG, D >= 6) it
// fits at D = 6 for every M (244-252 VGPRs) and at D = 7..8 for M <= 6 with fo_waves = 2 (D = 8, M = 6,
// N = 4096: 145.4 -> 130.9 ms).
__host__ __device__ constexpr int fo_wmax(int DP, int M) {
  return DP <= 6 ? 8 : (DP <= 8 ? (M <= 6 ? 8 : 4) : (DP <= 16 ? 4 : 2));
}
// Sequences longer than 64 * fo_wmax points run at LP = 64, W = fo_wmax in column blocks
// (sig_fo_kernel, `nblk`), with one float per row and level of carry in LDS per wave.
// Wide channels (DP == 0): no column data in registers, W = 8 from 65 points on (W = 4 below, RBF only).
inline Geo fo_geometry_wide(int l2, int seed) {
  if (l2 <= 64 && seed == SEED_RBF_DIFF) return {4, 16};
  for (int LP : {16, 32, 64})
    if (LP * 8 >= l2) return {8, LP};
  return {8, 64};
}
// 10-lane groups of 10 columns (6 pairs per wave, SEG scans): sequences of 65..100 points take 100 of
// a group's columns instead of LP = 16 x W = 8 = 128 (C2, L = 100: 99 cells per row on 100 columns
// instead of 128).  RBF difference seed only, where W = 10 fits 256 VGPRs (DP <= 5, M <= 5).
constexpr bool fo_seg_ok(int DP, int M, int seed) { return seed == SEED_RBF_DIFF && DP >= 1 && DP <= 5 && M <= 5; }
inline Geo fo_geometry(int l2, int DP, int M, bool mf = false, int seed = -1) {
  if (mf) {  // matrix-core seed (RBF difference seed only): W = 4 columns per lane, no column blocks
    for (int LP : {16, 32, 64})
      if (LP * 4 >= l2) return {4, LP};
    return {0, 0};
  }
#ifndef GPSIG_FO_SEG
#define GPSIG_FO_SEG 1
#endif
  if (GPSIG_FO_SEG && fo_seg_ok(DP, M, seed) && l2 > 64 && l2 <= 100) return {10, 10};
  // smallest LP (shortest scans) at which some W <= fo_wmax covers the sequence, smallest such W
  for (int LP : {16, 32, 64})
    for (int W = 2; W <= fo_wmax(DP, M); W *= 2)
      if (LP * W >= l2) return {W, LP};
  return {fo_wmax(DP, M), 64};
}
// Column blocks of a launch: cells per block LP*W - 1 (the last column of the last lane is the halo point)
inline int fo_blocks(int l2, bool diff, Geo g) {
  if (g.LP * g.W >= l2) return 1;
  const int cells = diff ? l2 - 1 : l2, cpb = g.LP * g.W - 1;
  return (cells + cpb - 1) / cpb;
}
// LDS bytes per 4-wave workgroup for the carries of a blocked launch (0 when unblocked)
inline size_t fo_carry_bytes(int l1, bool diff, int M, int nblk) {
  if (nblk <= 1 || M <= 1) return 0;
  return (size_t)4 * (diff ? l1 - 1 : l1) * (M - 1) * sizeof(float);
}
constexpr size_t FO_MAX_CARRY_BYTES = 160 * 1024;
constexpr int FO_MAX_LEVELS = 8;

template <int DP, int W, int LP, int M, int SEED, bool MF = false>
int launch_fo(const SigArgs &a, long long nblocks, hipStream_t s) {
  if (nblocks <= 0) return GPSIG_OK;
  constexpr bool DIFF = SEED == SEED_RBF_DIFF || SEED == SEED_LIN_DIFF;
  const size_t lds = LP == 64 ? fo_carry_bytes(a.l1, DIFF, M, a.nblk) : 0;
  if (lds > FO_MAX_CARRY_BYTES) return GPSIG_EUNSUPPORTED;
  if (a.pair_mode == GPSIG_PAIRS_DIAG) {
    hipLaunchKernelGGL((sig_fo_kernel<DP, W, LP, M, SEED, true, false, MF>), dim3((unsigned)nblocks), dim3(256), lds, s, a);
  } else if (a.state) {
    if constexpr (DIFF && !MF)
      hipLaunchKernelGGL((sig_fo_kernel<DP, W, LP, M, SEED, false, true>), dim3((unsigned)nblocks), dim3(256), lds, s, a);
    else
      return GPSIG_EUNSUPPORTED;
  } else {
    hipLaunchKernelGGL((sig_fo_kernel<DP, W, LP, M, SEED, false, false, MF>), dim3((unsigned)nblocks), dim3(256), lds, s, a);
  }
  return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
}

// Workgroups per launch chunk of the split diagnostic: dmbuf holds FO_SPLIT_BLOCKS * 4 * G pairs'
// cells, (l1 - 1) x LP * W floats each.
constexpr long long FO_SPLIT_BLOCKS = 4096;

template <int DP, int W, int LP, int M, int SEED>
int launch_fo_split(const SigArgs &a0, long long nblocks, hipStream_t s) {
  if constexpr (SEED != SEED_RBF_DIFF || W % 4 != 0) {
    return GPSIG_EUNSUPPORTED;
  } else {
    if (a0.nblk != 1 || a0.pair_mode == GPSIG_PAIRS_DIAG || a0.state || !a0.dmbuf) return GPSIG_EUNSUPPORTED;
    SigArgs a = a0;
    for (long long c = 0; c < nblocks; c += FO_SPLIT_BLOCKS) {
      a.blk0 = c;
      const long long nb = nblocks - c < FO_SPLIT_BLOCKS ? nblocks - c : FO_SPLIT_BLOCKS;
      hipLaunchKernelGGL((sig_fo_kernel<DP, W, LP, M, SEED, false, false, false, 1>), dim3((unsigned)nb), dim3(256), 0, s, a);
      hipLaunchKernelGGL((sig_fo_kernel<DP, W, LP, M, SEED, false, false, false, 2>), dim3((unsigned)nb), dim3(256), 0, s, a);
    }
    return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
  }
}

template <int M, int SEED>
int fo_geo_wide(const SigArgs &a, long long nblocks, hipStream_t s) {
  if (a.mfma || a.dmbuf) return GPSIG_EUNSUPPORTED;
  const Geo geo = fo_geometry_wide(a.l2, SEED);
  if constexpr (SEED == SEED_RBF_DIFF)
    if (geo.W == 4) return launch_fo<0, 4, 16, M, SEED>(a, nblocks, s);
  if (geo.LP == 16) return launch_fo<0, 8, 16, M, SEED>(a, nblocks, s);
  if (geo.LP == 32) return launch_fo<0, 8, 32, M, SEED>(a, nblocks, s);
  return launch_fo<0, 8, 64, M, SEED>(a, nblocks, s);
}

template <int DP, int M, int SEED>
int fo_geo(const SigArgs &a, long long nblocks, hipStream_t s) {
  if constexpr (DP == 0) {  // wide channel counts
    return fo_geo_wide<M, SEED>(a, nblocks, s);
  } else {
  const Geo geo = fo_geometry(a.l2, DP, M, a.mfma != 0, a.dmbuf ? -1 : SEED);  // split diagnostic: aligned groups
  if constexpr (SEED == SEED_RBF_DIFF) {
    if (a.mfma) {  // A/B variant: seed dots on the matrix cores (not for the saved-state launch)
      if (a.state) return GPSIG_EUNSUPPORTED;
      if (geo.W == 4 && geo.LP == 16) return launch_fo<DP, 4, 16, M, SEED, true>(a, nblocks, s);
      if (geo.W == 4 && geo.LP == 32) return launch_fo<DP, 4, 32, M, SEED, true>(a, nblocks, s);
      if (geo.W == 4 && geo.LP == 64) return launch_fo<DP, 4, 64, M, SEED, true>(a, nblocks, s);
      return GPSIG_EUNSUPPORTED;
    }
  }
  if (a.mfma) return GPSIG_EUNSUPPORTED;
  constexpr int WM = fo_wmax(DP, M);
  if (a.dmbuf) {  // split diagnostic
    if constexpr (SEED == SEED_RBF_DIFF && WM >= 4) {
#define GPSIG_GEO(w, lp) \
  if (geo.W == w && geo.LP == lp) return launch_fo_split<DP, w, lp, M, SEED>(a, nblocks, s);
      GPSIG_GEO(4, 16) GPSIG_GEO(4, 32) GPSIG_GEO(4, 64)
      if constexpr (WM >= 8) { GPSIG_GEO(8, 16) GPSIG_GEO(8, 32) GPSIG_GEO(8, 64) }
#undef GPSIG_GEO
    }
    return GPSIG_EUNSUPPORTED;
  }
#define GPSIG_GEO(w, lp) \
  if (geo.W == w && geo.LP == lp) return launch_fo<DP, w, lp, M, SEED>(a, nblocks, s);
  GPSIG_GEO(2, 16) GPSIG_GEO(2, 32) GPSIG_GEO(2, 64)
  if constexpr (WM >= 4) { GPSIG_GEO(4, 16) GPSIG_GEO(4, 32) GPSIG_GEO(4, 64) }
  if constexpr (WM >= 8) { GPSIG_GEO(8, 16) GPSIG_GEO(8, 32) GPSIG_GEO(8, 64) }
  if constexpr (fo_seg_ok(DP, M, SEED)) { GPSIG_GEO(10, 10) }
#undef GPSIG_GEO
  return GPSIG_EUNSUPPORTED;
  }
}

// sig_fo_launch_dpm<DP, M> (the per-seed dispatch) is defined only in sig_fo_inst.hip, one translation
// unit per (channel count, level count): a definition visible here would make every includer instantiate
// (and embed device code for) all of them.
template <int DP, int M>
int sig_fo_launch_dpm(const SigArgs &a, int seed, long long nblocks, hipStream_t s);

}  // namespace gpsig
