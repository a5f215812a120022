// gpsig_amd -- gradient (vector-Jacobian product) of the first-order signature-kernel Gram on gfx950.
//
// The reference differentiates K through TF autodiff of the materialised graph (kernels.py:209-238
// base-kernel tensor -> signature_algs.py:8-35 recursion -> kernels.py:431-477 normalisation), keeping
// every (N1, L1, N2, L2) intermediate alive for the backward pass.  Here one lane group owns one pair
// (a, b) as in the forward kernel (sig_fo.h) and nothing grid-sized touches memory:
//
//   forward sweep  rows i = 0 .. L1-2:  C_m(j) += dM(i,j) S_{m-1}(i,j),  S_m = exclusive scan_j C_m
//                  (the forward recursion; its end state gives K_m(a,b) for the normalisation term)
//   reverse sweep  rows i = L1-2 .. 0:
//     * the forward state of row i is recovered by inverting the update (C_m -= dM S_{m-1}, levels in
//       ascending order), so no per-row state is stored;
//     * adjoint of the column sums: Ch_m(i) = Ch_m(i+1) + reverse-exclusive-scan_j(dM(i,.) Ch_{m+1}(i+1,.)),
//       Ch_m(L1-1) = g_m = dLoss/dK_m(a,b);
//     * dLoss/d dM(i,j) = sum_m Ch_m(i+1,j) S_{m-1}(i,j);
//     * the adjoint of the second difference (signature_algs.py:26) turns it into dLoss/dk(x_i, y_j) on
//       the point grid, and the base kernel's derivative (RBF: k (y - x); linear: y) gives the point
//       gradients: x-rows are reduced across the wave and added to gX, y-columns accumulate in lane
//       registers and are added to gY at the end.
//
// The cells the reverse sweep inverts with are not bitwise those its forward state came from: the RBF
// difference seed regenerates them in chunks of RC rows with exp-free recurrences (chain over the lane's
// W columns, exact row every RC rows), while the forward sweep here evaluates k directly and the forward
// launch that saves the state (sig_fo.h, RbfSeedPk) chains column pairs (w, w + W/2) and re-anchors
// every 32 rows.  The cells agree to ~1e-7 relative, so the recovered state carries that plus the fp32
// rounding of the sums (gradient error <= 6e-6 norm-relative vs fp64 autodiff).
#pragma once
#include "sig_common.h"

namespace gpsig {

// dLoss/dscale is accumulated into this many partial sums (workspace) and reduced after the launch: one
// address per level for every wave of the grid serialised the atomics (+7.7 ms at N = 1024, L = 100).
constexpr int GSCALE_SLOTS = 64;

struct BwdArgs {
  const float *FX, *FY;  // feature records (n1,l1,FS), (n2,l2,FS)
  int n1, l1, n2, l2, d;
  int M;
  int pair_mode, row_begin, row_end;
  int tiles_a0, ntb;
  long long tile_base;
  const float *gout;  // upstream gradient: (n1, n2) summed [levels == 0] or (M+1, n1, n2) per level;
                      // DIAG: (M+1, n1)
  int gout_levels;
  long long g_ld, g_lvl;
  const float *rs1, *rs2, *scale;
  float jitter;
  float *gX, *gY, *grs1, *grs2;
  float *gscale;  // GSCALE_SLOTS x (M + 1) partial sums (workspace), see gpsig_sig_gram_vjp
  const float *state;  // optional saved forward state (RECT / UPPER), see gpsig_sig_gram_state
  // column blocks (LP = 64, sequences longer than one lane group covers): per-pair scratch of
  // scr_stride floats at scratch + (blockIdx.x * 4 + wave) * scr_stride, see bwd_scratch_floats
  int nblk;
  long long blk0;  // first logical workgroup of this launch (the host splits blocked launches)
  float *scratch;
  long long scr_stride;
  // wide channel counts (sig_bwd_wide.h): channel count, padded record lengths, record strides, and the
  // point-weight tile of the launch: pair (a, b), point row i at tile + (a - tile_a0) tile_as +
  // (b - tile_b0) l2 + i tile_ld (DIAG: + i tile_ld only)
  int wd, lw1, lw2;
  long long sx, sy;
  float *tile;
  int tile_a0, tile_b0;
  long long tile_as, tile_ld;
  // DIAG seed tiles of the wide VJP (sig_bwd_wide.hip wide_diag_tiles): pair a at dtile + (a - dt_a0) dt_pair,
  // [c_ij (dt_rows x dt_ld)][<dx_i, y_j> (dt_rows x dt_ld)][per anchor row: k, expm1(q) (2 x dt_ld each)]
  const float *dtile;
  int dt_a0;
  long long dt_pair, dt_rows, dt_ld;
};

// Load of a carry another lane of this wave stored earlier in the launch: served by L2 (agent scope),
// never by a possibly stale vector L1 line.
GPSIG_DEV float ld_l2(const float *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// Scratch of one pair in column-block mode (floats): the forward carries into blocks 1..nblk-1
// (nrows x (M-1) each), the adjoint carry slab (nrows x (M-1)), the end-of-sweep column sums of every
// block ((M-1) x W x 64, lane-minor).
__host__ __device__ inline long long bwd_scratch_floats(int nrows, int M, int W, int nblk) {
  if (nblk <= 1 || M <= 1) return 0;
  return (long long)nblk * nrows * (M - 1) + (long long)nblk * (M - 1) * W * 64;
}

// Exclusive scan over the group's columns of per-lane column arrays v[W] (W columns of lane gl hold
// columns gl*W .. gl*W+W-1), N independent arrays, scans step-interleaved.
template <int LP, int W, int N>
GPSIG_DEV void group_excl_cols_n(const float (&v)[N][W], float (&out)[N][W]) {
  float t[N], incl[N];
#pragma unroll
  for (int n = 0; n < N; ++n) {
    float s = 0.0f;
#pragma unroll
    for (int w = 0; w < W; ++w) s += v[n][w];
    t[n] = s;
    incl[n] = s;
  }
  if constexpr (64 % LP != 0)
    seg_incl_scan_n<LP, N>(incl, SegFactors<LP>{});
  else
    group_incl_scan_n<LP, N>(incl);
#pragma unroll
  for (int n = 0; n < N; ++n) {
    float run = incl[n] - t[n];
#pragma unroll
    for (int w = 0; w < W; ++w) {
      out[n][w] = run;
      run += v[n][w];
    }
  }
}

// Reverse exclusive scan (sum over columns j' > j of the group) of N arrays.
template <int LP, int W, int N>
GPSIG_DEV void group_rexcl_cols_n(const float (&v)[N][W], float (&out)[N][W]) {
  float t[N], incl[N];
#pragma unroll
  for (int n = 0; n < N; ++n) {
    float s = 0.0f;
#pragma unroll
    for (int w = 0; w < W; ++w) s += v[n][w];
    t[n] = s;
    incl[n] = s;
  }
  int last;
  if constexpr (64 % LP != 0) {  // segmented groups (LP = 20): the group's last lane, the idle tail clamped
    seg_incl_scan_n<LP, N>(incl, SegFactors<LP>{});
    const int l0 = (int)__lane_id() - (int)__lane_id() % LP + LP - 1;
    last = l0 < 64 ? l0 : 63;
  } else {
    group_incl_scan_n<LP, N>(incl);
    last = (int)(__lane_id() | (LP - 1));
  }
#pragma unroll
  for (int n = 0; n < N; ++n) {
    const float tot = __shfl(incl[n], last, 64);
    float run = tot - incl[n];  // sum over the lanes after this one
#pragma unroll
    for (int w = W - 1; w >= 0; --w) {
      out[n][w] = run;
      run += v[n][w];
    }
  }
}

// Column-block variants (LP = 64): add a wave-uniform carry cin[n] to every exclusive prefix and return
// the group total of v in tot[n] (wave-uniform), for the next block's carry.
template <int W, int N>
GPSIG_DEV void wave_excl_cols_carry_n(const float (&v)[N][W], float (&out)[N][W], const float (&cin)[N],
                                      float (&tot)[N]) {
  float t[N], incl[N];
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
  for (int n = 0; n < N; ++n) {
    tot[n] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, incl[n]), 63));
    float run = incl[n] - t[n] + cin[n];
#pragma unroll
    for (int w = 0; w < W; ++w) {
      out[n][w] = run;
      run += v[n][w];
    }
  }
}
template <int W, int N>
GPSIG_DEV void wave_rexcl_cols_carry_n(const float (&v)[N][W], float (&out)[N][W], const float (&cin)[N],
                                       float (&tot)[N]) {
  float t[N], incl[N];
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
  for (int n = 0; n < N; ++n) {
    tot[n] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, incl[n]), 63));
    float run = tot[n] - incl[n] + cin[n];  // sum over the lanes after this one, plus the blocks to the right
#pragma unroll
    for (int w = W - 1; w >= 0; --w) {
      out[n][w] = run;
      run += v[n][w];
    }
  }
}

// Sum over the whole wave of N values; the result is valid in lane 63.
template <int N>
GPSIG_DEV void wave_sum_last_n(float (&v)[N]) {
  group_incl_scan_n<64, N>(v);
}

#ifndef GPSIG_BWD_WPE
#define GPSIG_BWD_WPE 1
#endif
// Timing ablations for tools/kbench_vjp.hip only (wrong results): bit 1 drops the per-row x-gradient
// wave reduction and atomics, bit 2 the inversion scans, bit 4 the adjoint scans.
#ifndef GPSIG_BWD_ABL
#define GPSIG_BWD_ABL 0
#endif
template <int DP, int W, int LP, int M, int SEED>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(GPSIG_BWD_WPE))) void sig_bwd_kernel(BwdArgs p) {
  constexpr int FS = feat_stride(DP);
  constexpr int G = 64 / LP;
  constexpr bool SEG = (64 % LP) != 0;  // LP = 20: 3 pairs per wave, lanes 60..63 idle (common.h)
  constexpr bool DIFF = (SEED == SEED_RBF_DIFF || SEED == SEED_LIN_DIFF);  // else difference=False
  constexpr bool RBF = (SEED == SEED_RBF_DIFF || SEED == SEED_RBF_POINT);   // base kernel
  constexpr float NHL2E = -0.72134752044448170f;  // exp(-d2/2) = exp2(d2 * NHL2E)
  constexpr float L2E = 1.4426950408889634f;
#ifndef GPSIG_BWD_RC
#define GPSIG_BWD_RC 4
#endif
  // rows per chunk of the reverse sweep (LDS: 4 waves x RC x 64 lanes x 2W floats per workgroup); the 20-lane
  // geometry (C2's 65-100 points) regenerates 6 rows per exact row: 21.73 -> 21.45 ms on tools/kbench_vjp.hip
  // (profiles/r6_vjp_rc_ab.txt), the other geometries keep 4 (round 3: 6 within noise there)
  constexpr int RC = W >= 4 ? (LP == 20 ? 6 : GPSIG_BWD_RC) : 8;
  __shared__ __attribute__((aligned(16))) float cbuf[RBF && DIFF ? 4 : 1][RBF && DIFF ? RC : 1][64][2 * W];
  __shared__ float tbuf[DP <= 8 ? 4 : 1][DP <= 8 ? 4 : 1][DP <= 8 ? DP : 1][64];  // x-gradient row batches
  constexpr int ML = M > 1 ? M - 1 : 1;
  constexpr int CPB = LP * W - 1;  // cells of a column block (the last lane's last column is its halo point)

  const int lane = threadIdx.x & 63;
  const int wave = wave_uniform(threadIdx.x >> 6);
  const int g = lane / LP;
  const int gl = lane % LP;
  const bool diag = p.pair_mode == GPSIG_PAIRS_DIAG;
  const long long lblk = p.blk0 + (long long)blockIdx.x;  // logical workgroup

  // ---- which pair (same enumeration as sig_fo_kernel)
  int a, b;
  if (diag) {
    a = p.row_begin + (int)lblk * 4 + wave;
    b = a;
    if (a >= p.row_end) return;
  } else {
    int ta, tb;
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
  bool pair_ok = b < p.n2;
  if (p.pair_mode == GPSIG_PAIRS_UPPER) pair_ok = pair_ok && b >= a;
  if (SEG) pair_ok = pair_ok && g < G;
  if (diag) pair_ok = (g == 0);
  const int bl = b < p.n2 ? b : p.n2 - 1;
  const int l1 = p.l1, l2 = p.l2;

  const float *__restrict__ fx = p.FX + (long long)a * l1 * FS;
  cfloat *fxc = as_const(fx);  // row records: scalar loads, independent of the atomics below
  const float *__restrict__ fy = p.FY + (long long)bl * l2 * FS;
  const int nrows = DIFF ? l1 - 1 : l1;

  // ---- column blocks: block k holds the cells j0 .. j0 + CPB - 1 on the points j0 .. j0 + CPB (j0 = k CPB)
  const int nblk = (LP == 64) ? p.nblk : 1;
  const bool blocked = LP == 64 && nblk > 1 && M > 1;
  float *__restrict__ scr = blocked ? p.scratch + ((long long)blockIdx.x * 4 + wave) * p.scr_stride : nullptr;
  // forward carry into block k (k >= 1): [i][m] = sum_{j < j0} C_{m+1}(i, j) before row i
  auto tcar = [&](int k) { return scr + (long long)(k - 1) * nrows * ML; };
  float *__restrict__ ucar = blocked ? scr + (long long)(nblk - 1) * nrows * ML : nullptr;  // adjoint carry slab
  auto endst = [&](int k) { return ucar + (long long)nrows * ML + (long long)k * ML * W * 64; };

  // ---- column data of this lane in block k
  float y[W][DP], dy[W][DP], hdy[W];
  bool colv[W], ptv[W];
  int j0 = 0;
  auto load_cols = [&](int blk) {
    j0 = blk * CPB;
    // points of this block: the DIFF seeds see the halo point, the point seeds do not
    const int npts = nblk == 1 ? l2 : min(l2 - j0, DIFF ? CPB + 1 : CPB);
#pragma unroll
    for (int w = 0; w < W; ++w) {
      const int j = gl * W + w;
      colv[w] = j < (DIFF ? npts - 1 : npts);  // columns of the grid the recursion consumes
      ptv[w] = j < npts;
      const int jj = j0 + (j < npts ? j : npts - 1);
      const float *f = fy + (long long)jj * FS;
#pragma unroll
      for (int k = 0; k < DP; ++k) {
        y[w][k] = f[k];
        dy[w][k] = f[DP + k];
      }
      hdy[w] = f[2 * DP];
    }
  };

  // k(x_i, y_j) of one point row (RBF); identical instructions in both sweeps
  auto krow = [&](cfloat *xr, float (&k)[W]) {
#pragma unroll
    for (int w = 0; w < W; ++w) {
      float s = 0.0f;
#pragma unroll
      for (int c = 0; c < DP; ++c) {
        const float t = xr[c] - y[w][c];
        s = __builtin_fmaf(t, t, s);
      }
      k[w] = __builtin_amdgcn_exp2f(s * NHL2E);
    }
  };
  // cells dM(i, j) of row i from k rows i (kc) and i+1 (kn); kcR/knR = right neighbour of column W-1
  auto cells = [&](cfloat *fr, const float (&kc)[W], const float (&kn)[W], float kcR, float knR,
                   float (&dM)[W]) {
    if constexpr (RBF) {
      const float hdx = fr[2 * DP];
#pragma unroll
      for (int w = 0; w < W; ++w) {
        float pp = -hdx, q = -hdy[w], c = 0.0f;
#pragma unroll
        for (int k = 0; k < DP; ++k) {
          const float df = fr[k] - y[w][k];
          const float dxk = fr[DP + k];
          pp = __builtin_fmaf(-df, dxk, pp);
          q = __builtin_fmaf(df, dy[w][k], q);
          c = __builtin_fmaf(dxk, dy[w][k], c);
        }
        const float kn1 = (w + 1 < W) ? kn[w + 1] : knR;
        const float kc1 = (w + 1 < W) ? kc[w + 1] : kcR;
        const float naive = (kn1 - kn[w]) - (kc1 - kc[w]);
        const float Ep = em1_small(pp), Eq = em1_small(q), Ec = em1_small(c);
        const float stable = kc[w] * __builtin_fmaf(Ep, Eq, (1.0f + Ep) * (1.0f + Eq) * Ec);
        const float mx = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(pp), __builtin_fabsf(q)), __builtin_fabsf(c));
        const float v = mx < EM1_TAU ? stable : naive;
        dM[w] = colv[w] ? v : 0.0f;
      }
    } else {
#pragma unroll
      for (int w = 0; w < W; ++w) {
        float c = 0.0f;
#pragma unroll
        for (int k = 0; k < DP; ++k) c = __builtin_fmaf(fr[DP + k], dy[w][k], c);
        dM[w] = colv[w] ? c : 0.0f;
      }
    }
  };
  // difference=False: the cells are the point grid itself, k(x_i, y_j) (signature_algs.py:26 skipped)
  auto point_cells = [&](int i, float (&dM)[W], float (&k0)[W]) {
    cfloat *xr = fxc + (long long)i * FS;
    if constexpr (RBF) {
      krow(xr, k0);
#pragma unroll
      for (int w = 0; w < W; ++w) dM[w] = colv[w] ? k0[w] : 0.0f;
    } else {
      float xv[DP];
#pragma unroll
      for (int k = 0; k < DP; ++k) xv[k] = xr[k];
#pragma unroll
      for (int w = 0; w < W; ++w) {
        float c = 0.0f;
#pragma unroll
        for (int k = 0; k < DP; ++k) c = __builtin_fmaf(xv[k], y[w][k], c);
        dM[w] = colv[w] ? c : 0.0f;
        k0[w] = 1.0f;
      }
    }
  };

  // ---- forward sweep(s), or the end state saved by the forward launch (gpsig_sig_gram_state)
  float C[M][W];
  float kc[W], kcR = 0.0f;
  float K[M + 1];
  K[0] = 1.0f;
  const bool saved = DIFF && p.state != nullptr;  // kernel-uniform (the host passes state for DIFF only)
  auto zeroC = [&]() {
#pragma unroll
    for (int m = 0; m < M; ++m)
#pragma unroll
      for (int w = 0; w < W; ++w) C[m][w] = 0.0f;
  };
  zeroC();
  // blocks whose forward sweep runs: all (no saved state), or those left of the last (their carries)
  const int nfwd = saved ? (blocked ? nblk - 1 : 0) : nblk;
  float Kacc[M];
#pragma unroll
  for (int m = 0; m < M; ++m) Kacc[m] = 0.0f;
  for (int blk = 0; blk < nfwd; ++blk) {
    load_cols(blk);
    zeroC();
    if constexpr (RBF && DIFF) {
      krow(fxc, kc);
      kcR = lane_next(kc[0]);
    }
    for (int i = 0; i < nrows; ++i) {
      cfloat *fr = fxc + (long long)i * FS;
      float kn[W], knR = 0.0f, dM[W];
      if constexpr (DIFF) {
        if constexpr (RBF) {
          krow(fr + FS, kn);
          knR = lane_next(kn[0]);
        }
        cells(fr, kc, kn, kcR, knR, dM);
      } else {
        point_cells(i, dM, kn);
      }
      if constexpr (M > 1) {
        float Cs[ML][W], S[ML][W];
#pragma unroll
        for (int m = 0; m < ML; ++m)
#pragma unroll
          for (int w = 0; w < W; ++w) Cs[m][w] = C[m][w];
        if (blocked) {
          float cin[ML], tot[ML];
#pragma unroll
          for (int m = 0; m < ML; ++m) cin[m] = blk > 0 ? ld_l2(tcar(blk) + (long long)i * ML + m) : 0.0f;
          wave_excl_cols_carry_n<W, ML>(Cs, S, cin, tot);
          if (blk + 1 < nblk && lane == 0) {
#pragma unroll
            for (int m = 0; m < ML; ++m) tcar(blk + 1)[(long long)i * ML + m] = cin[m] + tot[m];
          }
        } else {
          group_excl_cols_n<LP, W, ML>(Cs, S);
        }
#pragma unroll
        for (int m = 1; m < M; ++m)
#pragma unroll
          for (int w = 0; w < W; ++w) C[m][w] = __builtin_fmaf(dM[w], S[m - 1][w], C[m][w]);
      }
#pragma unroll
      for (int w = 0; w < W; ++w) C[0][w] += dM[w];
      if constexpr (RBF && DIFF) {
#pragma unroll
        for (int w = 0; w < W; ++w) kc[w] = kn[w];
        kcR = knR;
      }
    }
    if (!saved) {
#pragma unroll
      for (int m = 0; m < M; ++m) {
        float s = 0.0f;
#pragma unroll
        for (int w = 0; w < W; ++w) s += C[m][w];
        if constexpr (SEG)
          Kacc[m] += seg_group_sum<LP>(s, SegFactors<LP>{});
        else
          Kacc[m] += group_sum<LP>(s);
      }
      if (blocked) {  // this block's end state, for its reverse sweep
#pragma unroll
        for (int m = 0; m < ML; ++m)
#pragma unroll
          for (int w = 0; w < W; ++w) endst(blk)[((long long)m * W + w) * 64 + lane] = C[m][w];
      }
    }
  }
  if (saved) {
    const float *__restrict__ st =
        p.state + (pair_ok ? state_slot(a, bl, p.n2, p.pair_mode == GPSIG_PAIRS_UPPER) * state_stride(M, l2) : 0);
#pragma unroll
    for (int m = 1; m <= M; ++m) K[m] = pair_ok ? st[(long long)(M - 1) * (l2 - 1) + m - 1] : 0.0f;
  } else {
#pragma unroll
    for (int m = 0; m < M; ++m) K[m + 1] = Kacc[m];
    if constexpr (DIFF) K[1] = level1_closed<DP, SEED>(fx, fy, l1, l2);
  }

  // ---- per-level weights g_m = dLoss/dK_m(a, b) and the normalisation / scale terms

  // per-level weights g_m = dLoss/dK_m(a, b) and the normalisation / scale factors of this pair
  const bool upper_off = p.pair_mode == GPSIG_PAIRS_UPPER && a != bl;
  const float jit = (p.pair_mode == GPSIG_PAIRS_UPPER && a == bl) ? p.jitter : 0.0f;
  auto pair_terms = [&](float (&gs)[M + 1], float (&sc)[M + 1], float (&r1)[M + 1], float (&r2)[M + 1]) {
    float gsum = 0.0f;
    if (!diag && !p.gout_levels) {
      gsum = p.gout[(long long)a * p.g_ld + bl];
      if (upper_off) gsum += p.gout[(long long)bl * p.g_ld + a];
    }
#pragma unroll
    for (int m = 0; m <= M; ++m) {
      float g;
      if (diag) {
        g = p.gout[(long long)m * p.g_lvl + a];
      } else if (p.gout_levels) {
        g = p.gout[(long long)m * p.g_lvl + (long long)a * p.g_ld + bl];
        if (upper_off) g += p.gout[(long long)m * p.g_lvl + (long long)bl * p.g_ld + a];
      } else {
        g = gsum;
      }
      gs[m] = pair_ok ? g : 0.0f;
      sc[m] = p.scale ? p.scale[m] : 1.0f;
      r1[m] = p.rs1 ? p.rs1[(long long)m * p.n1 + a] : 1.0f;
      r2[m] = p.rs2 ? p.rs2[(long long)m * p.n2 + bl] : 1.0f;
    }
  };
  float gw[M + 1];
  {
    float gs[M + 1], sc[M + 1], r1[M + 1], r2[M + 1];
    pair_terms(gs, sc, r1, r2);
#pragma unroll
    for (int m = 0; m <= M; ++m) gw[m] = gs[m] * sc[m] * r1[m] * r2[m];
  }
  // dLoss/drs and dLoss/dscale of this pair, added after the sweep (their atomics would otherwise sit in
  // vmcnt ahead of every load of the sweep; the factors are reloaded there, only K stays live):
  // grs1[m, a] summed over the wave (its pairs all share a), grs2[m, b] per pair, gscale into one of
  // GSCALE_SLOTS partial sums (summed over the wave)
  auto norm_terms = [&]() {
    if (diag || !(p.gscale || (p.rs1 && (p.grs1 || p.grs2)))) return;
    float gs[M + 1], sc[M + 1], r1[M + 1], r2[M + 1];
    pair_terms(gs, sc, r1, r2);
    const bool lead = gl == 0 && pair_ok;  // one contribution per pair
    float g1[M + 1], g2[M + 1], gsc[M + 1];
#pragma unroll
    for (int m = 0; m <= M; ++m) {
      const float t = gs[m] * sc[m] * (K[m] + jit);
      g1[m] = lead ? t * r2[m] : 0.0f;
      g2[m] = t * r1[m];
      gsc[m] = lead ? gs[m] * (K[m] + jit) * r1[m] * r2[m] : 0.0f;
    }
    if (p.rs1 && p.grs1) {
      wave_sum_last_n<M + 1>(g1);
      if (lane == 63)
        for (int m = 0; m <= M; ++m) unsafeAtomicAdd(p.grs1 + (long long)m * p.n1 + a, g1[m]);
    }
    if (p.rs1 && p.grs2 && lead) {
#pragma unroll
      for (int m = 0; m <= M; ++m) unsafeAtomicAdd(p.grs2 + (long long)m * p.n2 + bl, g2[m]);
    }
    if (p.gscale) {
      wave_sum_last_n<M + 1>(gsc);
      if (lane == 63) {
        float *slot = p.gscale + (long long)(lblk & (GSCALE_SLOTS - 1)) * (M + 1);
        for (int m = 0; m <= M; ++m) unsafeAtomicAdd(slot + m, gsc[m]);
      }
    }
  };

  // ---- reverse sweep, blocks right to left
  float *__restrict__ gxa = p.gX + (long long)a * l1 * p.d;
  const int d = p.d;
  const float gM = gw[M];
  for (int blk = nblk - 1; blk >= 0; --blk) {
    const bool cin_left = blocked && blk > 0;          // forward carry from the blocks to the left
    const bool uin_right = blocked && blk + 1 < nblk;  // adjoint carry from the blocks to the right
    const bool uout_left = blocked && blk > 0;
    if (nfwd != 1 || nblk > 1) load_cols(blk);  // (single unsaved block: still loaded from the forward)
    if (saved) {
      const int nc = l2 - 1;
      const float *__restrict__ st =
          p.state + (pair_ok ? state_slot(a, bl, p.n2, p.pair_mode == GPSIG_PAIRS_UPPER) * state_stride(M, l2) : 0);
#pragma unroll
      for (int m = 0; m + 1 < M; ++m)
#pragma unroll
        for (int w = 0; w < W; ++w) {
          const int jl = gl * W + w, j = j0 + jl;
          C[m][w] = (pair_ok && j < nc && jl < CPB) ? st[(long long)m * nc + j] : 0.0f;
        }
    } else if (blocked) {
#pragma unroll
      for (int m = 0; m < ML; ++m)
#pragma unroll
        for (int w = 0; w < W; ++w) C[m][w] = endst(blk)[((long long)m * W + w) * 64 + lane];
    }
    if constexpr (RBF && DIFF) {
      if (saved || nblk > 1) {
        krow(fxc + (long long)nrows * FS, kc);  // k row of the last point, as the sweep would leave it
        kcR = lane_next(kc[0]);
      }
    }

    float Ch[ML][W];
#pragma unroll
    for (int m = 0; m < ML; ++m)
#pragma unroll
      for (int w = 0; w < W; ++w) Ch[m][w] = gw[m + 1];
    float Ep[W], A[W], B[W][DP];
#pragma unroll
    for (int w = 0; w < W; ++w) {
      Ep[w] = 0.0f;
      A[w] = 0.0f;
#pragma unroll
      for (int k = 0; k < DP; ++k) B[w][k] = 0.0f;
    }

    // point row `pi` of the grid receives dLoss/dk(x_pi, y_j) = Kh[w]: x-gradient reduced over the wave
    // (all pairs of a wave share a), y-gradient accumulated per column
    // The x-gradient of point row pi is a sum over all 64 lanes (every pair of the wave shares a).  The
    // reverse sweep emits the point rows in descending order, so for DP <= 8 they are batched by 4: each
    // lane parks its partials of a row in this wave's LDS slab, and every 4th row one
    // wave_reduce_scatter4 plus one atomic per channel from 4 lanes serve the batch (a wave-wide scan per
    // channel and row before: a quarter of the VJP's time at N = 1024, L = 100).
    constexpr bool BATCH = DP <= 8;
    int nslot = 0, pi0 = 0;  // rows in the open batch, its first (highest) row
    auto flush = [&]() {
      if constexpr (BATCH) {
        float v[4 * DP], o[DP];
#pragma unroll
        for (int k = 0; k < DP; ++k)
#pragma unroll
          for (int r = 0; r < 4; ++r) v[4 * k + r] = tbuf[wave][r][k][lane];
        wave_reduce_scatter4<DP>(v, o);
        const int R = lane >> 4;
        const int slot = R == 0 ? 0 : R == 1 ? 2 : R == 2 ? 1 : 3;  // ROW_SLOT
        if ((lane & 15) == 0 && slot < nslot) {
#pragma unroll
          for (int k = 0; k < DP; ++k)
            if (k < d) unsafeAtomicAdd(gxa + (long long)(pi0 - slot) * d + k, o[k]);
        }
        nslot = 0;
      }
    };
    auto emit = [&](int pi, const float (&Kh)[W], const float (&kr)[W]) {
      cfloat *xp = fxc + (long long)pi * FS;
      float xi[DP];
#pragma unroll
      for (int k = 0; k < DP; ++k) xi[k] = xp[k];
      float wg[W];
#pragma unroll
      for (int w = 0; w < W; ++w) {
        const float v = RBF ? Kh[w] * kr[w] : Kh[w];
        wg[w] = ptv[w] ? v : 0.0f;
      }
      float s[DP + 1];
#pragma unroll
      for (int k = 0; k <= DP; ++k) s[k] = 0.0f;
#pragma unroll
      for (int w = 0; w < W; ++w) {
        s[DP] += wg[w];
#pragma unroll
        for (int k = 0; k < DP; ++k) s[k] = __builtin_fmaf(wg[w], y[w][k], s[k]);
        A[w] += wg[w];
#pragma unroll
        for (int k = 0; k < DP; ++k) B[w][k] = __builtin_fmaf(wg[w], xi[k], B[w][k]);
      }
      // this lane's share of dLoss/dx_pi: sum_j wg (y_j - x_pi) (RBF) or sum_j wg y_j (linear)
      float t[DP];
#pragma unroll
      for (int k = 0; k < DP; ++k) t[k] = RBF ? __builtin_fmaf(-s[DP], xi[k], s[k]) : s[k];
      if constexpr (GPSIG_BWD_ABL & 1) {
        if (t[0] == 1234.5f) gxa[pi] = t[1];  // keep the partials alive
      } else if constexpr (BATCH) {
        if (nslot == 0) pi0 = pi;
#pragma unroll
        for (int k = 0; k < DP; ++k) tbuf[wave][nslot][k][lane] = t[k];
        if (++nslot == 4) flush();
      } else {
        wave_sum_last_n<DP>(t);
        if (lane == 63) {
#pragma unroll
          for (int k = 0; k < DP; ++k)  // compile-time indices (a runtime bound would put t in scratch)
            if (k < d) unsafeAtomicAdd(gxa + (long long)pi * d + k, t[k]);
        }
      }
    };

    float kr1[W];  // k row of point i+1 (DIFF)
    if constexpr (RBF && DIFF) {
#pragma unroll
      for (int w = 0; w < W; ++w) kr1[w] = kc[w];
    } else {
#pragma unroll
      for (int w = 0; w < W; ++w) kr1[w] = 1.0f;
    }
    // one row of the reverse sweep from its cells dM(i, .) and the k row of point i
    auto rev_row = [&](int i, const float (&dM)[W], const float (&k0)[W]) {
      // forward state of row i: C_m(i) = C_m(i+1) - dM S_{m-1}(i), ascending levels (C[m] holds level m+1,
      // S_0 = 1), and dLoss/d dM(i, j) = sum_m Ch_m(i+1, j) S_{m-1}(i, j)
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
        if (blocked) {
          float cin[1], tot[1];
          cin[0] = cin_left ? ld_l2(tcar(blk) + (long long)i * ML + s - 1) : 0.0f;
          wave_excl_cols_carry_n<W, 1>(Cm, Sm, cin, tot);
        } else if constexpr (GPSIG_BWD_ABL & 2) {
#pragma unroll
          for (int w = 0; w < W; ++w) Sm[0][w] = Cm[0][w];
        } else {
          group_excl_cols_n<LP, W, 1>(Cm, Sm);  // S_s(i) from the recovered C_s(i)
        }
#pragma unroll
        for (int w = 0; w < W; ++w) {
          if (s + 1 < M) C[s][w] = __builtin_fmaf(-dM[w], Sm[0][w], C[s][w]);
          const float chn = (s + 1 < M) ? Ch[s < ML ? s : 0][w] : gM;  // Ch_{s+1}
          Dh[w] = __builtin_fmaf(chn, Sm[0][w], Dh[w]);
        }
      }
#pragma unroll
      for (int w = 0; w < W; ++w) Dh[w] = colv[w] ? Dh[w] : 0.0f;

      // adjoint column sums: Ch_m(i) = Ch_m(i+1) + rexcl(dM * Ch_{m+1}(i+1)), ascending m (old Ch_{m+1})
      if constexpr (M > 1) {
        float v[ML][W], r[ML][W];
#pragma unroll
        for (int m = 0; m < ML; ++m)
#pragma unroll
          for (int w = 0; w < W; ++w) v[m][w] = dM[w] * ((m + 1 < ML) ? Ch[m + 1][w] : gM);
        if (blocked) {
          float uin[ML], tot[ML];
          float *__restrict__ ur = ucar + (long long)i * ML;
#pragma unroll
          for (int m = 0; m < ML; ++m) uin[m] = uin_right ? ld_l2(ur + m) : 0.0f;
          wave_rexcl_cols_carry_n<W, ML>(v, r, uin, tot);
          if (uout_left && lane == 0) {
#pragma unroll
            for (int m = 0; m < ML; ++m) ur[m] = uin[m] + tot[m];
          }
        } else if constexpr (GPSIG_BWD_ABL & 4) {
#pragma unroll
          for (int m = 0; m < ML; ++m)
#pragma unroll
            for (int w = 0; w < W; ++w) r[m][w] = v[m][w];
        } else {
          group_rexcl_cols_n<LP, W, ML>(v, r);
        }
#pragma unroll
        for (int m = 0; m < ML; ++m)
#pragma unroll
          for (int w = 0; w < W; ++w) Ch[m][w] += r[m][w];
      }

      if constexpr (DIFF) {
        // adjoint of the second difference: E(i, j) = Dh(i, j-1) - Dh(i, j); Kh(i+1, j) = E(i, j) - E(i+1, j)
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
        emit(i, Dh, k0);  // the cell is the point value: dLoss/dk(x_i, y_j) = Dh(i, j)
      }
    };

    if constexpr (RBF && DIFF) {
      // Chunked: the cells of RC rows are regenerated forward from an exact row (k and expm1(q) from
      // x - y) with exp-free recurrences like the forward kernel's (sig_common.h RbfSeedPk: the same
      // cells up to the rounding of the recurrences, whose chain order and anchor rows differ) into
      // this lane's LDS slots, then consumed in reverse.  Cells with |p| or |c| >= EM1_TAU take the
      // corner difference of the k grid with an exact next row (wave-uniform branch).
      float(*cb)[64][2 * W] = cbuf[wave];
      // |c_ij| <= 2 sqrt(hdx_i hdy_j): when the bound over the wave's rows and columns allows, Ec takes the
      // forward's cubic and only the first column's p meets a polynomial (the others follow the exact chain
      // Ep' = Ep + (1 + Ep) Ec), as RbfSeedPk::row's CLO rows
      bool clo = false;
      {
        float hx = 0.0f, hy = 0.0f;
        for (int i = lane; i < nrows; i += 64) hx = __builtin_fmaxf(hx, fxc[(long long)i * FS + 2 * DP]);
#pragma unroll
        for (int w = 0; w < W; ++w) hy = __builtin_fmaxf(hy, hdy[w]);
        hx = wave_max(hx);
        hy = wave_max(hy);
        clo = wave_uniform(4.0f * hx * hy < 0.98f * EM1_LO_TAU * EM1_LO_TAU ? 1 : 0) != 0;
      }
      auto em1_cubic = [](float x) {
        float q = __builtin_fmaf(4.166666667e-02f, x, 1.666992186e-01f);
        q = __builtin_fmaf(q, x, 5.000000132e-01f);
        q = __builtin_fmaf(q, x, 9.999999841e-01f);
        return q * x;
      };
      auto exact_row = [&](cfloat *xr, float (&k)[W], float (&Eq)[W]) {
        float xv[DP];
#pragma unroll
        for (int c = 0; c < DP; ++c) xv[c] = xr[c];
#pragma unroll
        for (int w = 0; w < W; ++w) {
          float s2 = 0.0f, q = -hdy[w];
#pragma unroll
          for (int c = 0; c < DP; ++c) {
            const float df = xv[c] - y[w][c];
            s2 = __builtin_fmaf(df, df, s2);
            q = __builtin_fmaf(df, dy[w][c], q);
          }
          k[w] = __builtin_amdgcn_exp2f(s2 * NHL2E);
          Eq[w] = __builtin_fabsf(q) < EM1_TAU ? em1_small(q) : __builtin_amdgcn_exp2f(q * L2E) - 1.0f;
        }
      };
      auto chunk_fwd = [&](auto clo_t, int i0, int nr) {
        constexpr bool CLO = decltype(clo_t)::value;
        float kc[W], Eq[W];
        exact_row(fxc + (long long)i0 * FS, kc, Eq);
        for (int r = 0; r < nr; ++r) {
          cfloat *fr = fxc + (long long)(i0 + r) * FS;
          float dxv[DP];
#pragma unroll
          for (int c = 0; c < DP; ++c) dxv[c] = fr[DP + c];
          const float g = fr[2 * DP + 1];
          float dM[W], kn[W], Eqn[W], mx[W], pp[W], cv[W];
          bool slow = false;
          // p along the lane's columns by p_{j+1} = p_j + c_j and Ep_{j+1} = Ep_j + (1 + Ep_j) Ec_j from
          // the exact first column (the forward seed's column recurrence, RbfSeedPk::row: the chain
          // anchors fall on the same columns, multiples of 4)
#pragma unroll
          for (int w = 0; w < W; ++w) {
            float c = dy[w][0] * dxv[0];
#pragma unroll
            for (int k = 1; k < DP; ++k) c = __builtin_fmaf(dy[w][k], dxv[k], c);
            cv[w] = c;
          }
          pp[0] = -g;
#pragma unroll
          for (int k = 0; k < DP; ++k) pp[0] = __builtin_fmaf(y[0][k], dxv[k], pp[0]);
#pragma unroll
          for (int w = 1; w < W; ++w) pp[w] = pp[w - 1] + cv[w - 1];
          float Ep = em1_small(pp[0]);
#pragma unroll
          for (int w = 0; w < W; ++w) {
            const float c = cv[w], Ec = CLO ? em1_cubic(c) : em1_small(c);
            float t = __builtin_fmaf(Ep, Ec, Ec);
            const float Epw = Ep;
            Ep += t;
            t = __builtin_fmaf(Eq[w], t, t);
            dM[w] = kc[w] * __builtin_fmaf(Epw, Eq[w], t);
            kn[w] = __builtin_fmaf(kc[w], Epw, kc[w]);
            Eqn[w] = __builtin_fmaf(Eq[w], Ec, Eq[w] + Ec);
            mx[w] = CLO ? __builtin_fabsf(pp[w]) : __builtin_fmaxf(__builtin_fabsf(pp[w]), __builtin_fabsf(c));
            if (!CLO || w == 0) slow = slow || !(mx[w] < EM1_TAU);
          }
          if (__builtin_amdgcn_ballot_w64(slow) != 0) {
            // out-of-range cells may have spoilt the chained Ep: in-range cells from their own p
            exact_row(fr + FS, kn, Eqn);
            const float knR = lane_next(kn[0]), kcR2 = lane_next(kc[0]);
#pragma unroll
            for (int w = 0; w < W; ++w) {
              const float kn1 = (w + 1 < W) ? kn[w + 1] : knR;
              const float kc1 = (w + 1 < W) ? kc[w + 1] : kcR2;
              const float Epd = em1_small(pp[w]), Ecd = em1_small(cv[w]);
              float t = __builtin_fmaf(Epd, Ecd, Ecd);
              t = __builtin_fmaf(Eq[w], t, t);
              dM[w] = (mx[w] < EM1_TAU) ? kc[w] * __builtin_fmaf(Epd, Eq[w], t) : (kn1 - kn[w]) - (kc1 - kc[w]);
            }
          }
#pragma unroll
          for (int w = 0; w < W; ++w) {
            cb[r][lane][w] = colv[w] ? dM[w] : 0.0f;
            cb[r][lane][W + w] = kc[w];
            kc[w] = kn[w];
            Eq[w] = Eqn[w];
          }
        }
      };
      for (int i0 = ((nrows - 1) / RC) * RC; i0 >= 0; i0 -= RC) {
        const int nr = nrows - i0 < RC ? nrows - i0 : RC;
        if (clo)
          chunk_fwd(std::true_type{}, i0, nr);
        else
          chunk_fwd(std::false_type{}, i0, nr);
        for (int r = nr - 1; r >= 0; --r) {
          float dM[W], k0[W];
#pragma unroll
          for (int w = 0; w < W; ++w) {
            dM[w] = cb[r][lane][w];
            k0[w] = cb[r][lane][W + w];
          }
          rev_row(i0 + r, dM, k0);
        }
      }
    } else if constexpr (DIFF) {
      for (int i = nrows - 1; i >= 0; --i) {
        float k0[W], dM[W];
#pragma unroll
        for (int w = 0; w < W; ++w) k0[w] = 1.0f;
        cells(fxc + (long long)i * FS, k0, kr1, 0.0f, 0.0f, dM);
        rev_row(i, dM, k0);
      }
    } else {
      for (int i = nrows - 1; i >= 0; --i) {
        float k0[W], dM[W];
        point_cells(i, dM, k0);
        rev_row(i, dM, k0);
      }
    }
    if constexpr (DIFF) {
      float Kh[W];
#pragma unroll
      for (int w = 0; w < W; ++w) Kh[w] = -Ep[w];
      emit(0, Kh, kr1);
    }
    if (nslot > 0) flush();  // the last, partial batch

    // ---- y-gradient of the block's points
    if (pair_ok) {
      float *__restrict__ gyb = (diag ? p.gX : p.gY) + (long long)bl * l2 * d;
#pragma unroll
      for (int w = 0; w < W; ++w) {
        const int j = j0 + gl * W + w;
        if (!ptv[w]) continue;
#pragma unroll
        for (int k = 0; k < DP; ++k) {
          const float v = RBF ? __builtin_fmaf(-A[w], y[w][k], B[w][k]) : B[w][k];
          if (k < d) unsafeAtomicAdd(gyb + (long long)j * d + k, v);
        }
      }
    }
  }
  norm_terms();
}

// Column geometry of the backward kernel: W columns per lane, LP lanes per pair.  The lane keeps
// y, dy and the y-gradient accumulator (3 W DP floats) plus 2 (M-1) W level states.  Longer sequences
// run at LP = 64 in column blocks of 64 W - 1 cells (BwdArgs::nblk).
struct BwdGeo { int W, LP; };
// 20-lane groups of 5 columns (3 pairs per wave, segmented scans, common.h) for 65..100 points: 100
// columns per pair instead of LP = 32 x W = 4 = 128, and 5 DPP steps per scan instead of 6 (N = 1024,
// L = 100, D = 5, M = 5, tools/kbench_vjp.hip: 29.9 -> 23.6 ms).  Within 256 VGPRs at 2 waves/SIMD for
// DP <= 5, M <= 6.
constexpr bool bwd_seg_ok(int DP, int M) { return DP >= 1 && DP <= 5 && M <= 6; }
inline BwdGeo bwd_geometry(int l2, int DP, int M = 0) {
#ifndef GPSIG_BWD_SEG
#define GPSIG_BWD_SEG 1
#endif
  if (GPSIG_BWD_SEG && M > 0 && bwd_seg_ok(DP, M) && l2 > 64 && l2 <= 100) return {5, 20};
  const int W = DP <= 8 ? 4 : 2;
  for (int LP : {16, 32, 64})
    if (LP * W >= l2) return {W, LP};
  return {W, 64};
}
inline int bwd_blocks(int l2, bool diff, BwdGeo g) {
  if (g.LP * g.W >= l2) return 1;
  const int cells = diff ? l2 - 1 : l2, cpb = g.LP * g.W - 1;
  return (cells + cpb - 1) / cpb;
}
// workgroups per launch of a column-block VJP (4 pairs each): bounds the per-pair scratch
constexpr long long BWD_CHUNK_BLOCKS = 2048;

}  // namespace gpsig
