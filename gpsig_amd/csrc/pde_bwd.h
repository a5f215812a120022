// gpsig_amd -- gradient of the Goursat-PDE signature kernel on gfx950.
//
// The reference's only hand-written gradient is for the PDE kernel (kernels_pde.py:465-509,
// _KdiagGrad, over the grids K and K_rev returned by sigKer_fast.pyx:15-62; the same formula for the
// CUDA op in covariance_op/_untrunc_cov_grad.py:25-77):
//   KK[s, t] = K[s, t] * K_rev_rev[s+1, t+1],   K_rev_rev = K_rev flipped in both axes,
//   K_rev    = the solution on the time-reversed paths with the first-order scheme (solver 0),
//   G[i]     = 4^-n sum_{s in coarse row i} sum_t KK[s, t] dy_{t >> n}
//   dK/dx_i  = G[i-1] - G[i]   (times 2 for k(x, x), times the upstream gradient of K[-1, -1]).
// For a cross pair (x, y) the same adjoint gives dK/dy_j from the column sums.
//
// One wave per pair, the coarse-row skewed sweep of pde.hip (pde_rep_kernel: lane l owns W fine
// columns = W/REP coarse columns, one step = one coarse row of REP = 2^n fine rows), fp64 solution as
// the reference, and nothing grid-sized in memory:
//   * R(i, c) := K_rev[I-i][J-c] solves the same scheme from the corner (I, J) towards (0, 0)
//     (R(p, q) = R(p+1, q) + R(p, q+1) + R(p+1, q+1) (inc(p, q) - 1), solver 0), so KK[i][c] =
//     K(i, c) R(i+1, c+1).  Swept with the mirrored skew (lane l takes its right boundary from lane
//     l+1; coarse row ic at R step IC + U - 2 - ic - l, U = lanes used), lane l meets coarse row ic at
//     the R step IC + U - 2 - s where s = ic + l is the forward step of the same row: walking the
//     forward steps backwards visits, in every lane, exactly the cells the R sweep needs.
//   * pass A sweeps K forward and stores its front (the lane's last fine row, W values, plus the
//     REP - 1 other right-column values and the corner it hands on) every H steps to the workspace;
//   * pass B walks the chunks of H steps backwards: restore the chunk's front, re-run its H forward
//     steps keeping the K corner of every fine cell in registers, then run H steps of the R sweep,
//     which consume them in reverse.  The fronts and the kept corners are fp32: they enter only the
//     products KK (relative error ~1e-7 on the gradient), never the fp64 recurrences of the R sweep.
//   * per coarse cell the REP x REP products are summed first; the increments are constant over it,
//     so the row (dK/dx) and column (dK/dy) contractions cost 2 DP FMAs per coarse cell.  Row partials
//     go to the wave's LDS row accumulators (ds_add_f64; lanes hold distinct coarse rows at a step),
//     column partials stay in registers.
// Three sweeps of the grid instead of the previous two sweeps plus an fp64 K_rev grid stored and
// re-read through HBM (~0.3 MB per pair at L = 100, dyadic 1).
#pragma once
#include <type_traits>

#include "sig_common.h"

namespace gpsig {

struct PdeBwdArgs {
  const float *X, *Y;
  int n1, l1, n2, l2, d;
  int dyadic, solver;
  int pair_mode, row_begin, row_end;
  int ntb, tiles_a0;
  int wpb;            // waves (pairs) per workgroup: 4, or 2 / 1 when the per-wave LDS of long x needs it
  const float *gout;  // DIAG: (n1,); RECT: (n1, n2)
  float *gX, *gY;     // accumulated (n1, l1, d), (n2, l2, d)
  float *fronts;      // workspace: per evaluated pair, nfronts x (W + REP) x 64 floats (pde_front_floats)
  float *out;         // MODE 1 (forward with fronts): K per pair, DIAG out[a - row_begin], RECT
                      // out[(a - row_begin) * n2 + b]
  // DP == 0 (any channel count; dyadic > 3): increments from the tile of the pair (as PdeArgs: inc +
  // (a - inc_a0) inc_as + (b - inc_b0) (l2 - 1) + i inc_ld + j, kernel cells 2^sub finer than the tile),
  // and the adjoint's coarse-cell sums go to the tile gt of the same layout, scaled to dLoss/d<dx_i, dy_j>
  // (the host contracts them with the increments in two GEMMs)
  const float *inc;
  float *gt;
  long long inc_as, inc_ld;
  int inc_a0, inc_b0, sub;
};

GPSIG_DEV double lane_next_d(double v) { return dpp_d<0x130>(v); }

// increment of kernel cell (ci, cj) from the pair's tile (tile cells 2^sub times coarser, value / 4^sub)
GPSIG_DEV float tile_inc_b(const float *__restrict__ base, long long ld, int sub, int ci, int cj) {
  const float v = base[(long long)(ci >> sub) * ld + (cj >> sub)];
  return sub ? v * __builtin_ldexpf(1.0f, -2 * sub) : v;
}

// coarse steps per stored front: the chunk's K corners (H x REP x W <= GPSIG_PDE_HF floats per lane) live in registers
#ifndef GPSIG_PDE_HF
#define GPSIG_PDE_HF 32
#endif
template <int W, int REP>
constexpr int pde_chunk() { return REP * W >= GPSIG_PDE_HF ? 1 : GPSIG_PDE_HF / (REP * W); }

// Columns per lane of the adjoint kernel: the smallest power of two >= REP with ceil(J / W) <= 64 lanes,
// else the widest the registers take (REP * W <= 64, W <= 16) and the grid is swept in column blocks of
// 64 W fine columns; 0 when unsupported (REP > 8).
__host__ __device__ inline int pde_bwd_cols(int J, int rep) {
  if (rep > 8) return 0;
  const int wmax = rep * 16 <= 64 ? 16 : 64 / rep;
  for (int W = rep; W <= wmax; W *= 2)
    if ((long long)64 * W >= J) return W;
  return wmax;
}

// Per-pair workspace of the adjoint: the K fronts of every column block, then (several blocks only)
// fp64 boundary columns [nblk][I + 1]: slot b >= 1 the K values entering block b from the left, slot 0
// the R values entering a block from the right (reused in place, block by block).
struct PdeLayout {
  int W, H, nblk, nfr;     // nfr: fronts per block
  long long kb_off;        // float offset of the boundary columns
  long long pair_floats;   // fp32 words per pair (a multiple of 2)
};
__host__ __device__ inline PdeLayout pde_layout(int l1, int l2, int dyadic) {
  PdeLayout L{};
  if (dyadic < 0 || dyadic > 3 || l1 < 2 || l2 < 2) return L;
  const int rep = 1 << dyadic;
  const long long IC = l1 - 1, JL = (long long)(l2 - 1) * rep;
  if (JL > (1LL << 30)) return L;
  const int J = (int)JL, W = pde_bwd_cols(J, rep);
  if (W == 0) return L;
  L.W = W;
  L.H = rep * W >= GPSIG_PDE_HF ? 1 : GPSIG_PDE_HF / (rep * W);
  const long long CB = 64LL * W;
  L.nblk = (int)((J + CB - 1) / CB);
  const long long U = L.nblk == 1 ? (J + W - 1) / W : 64;
  L.nfr = (int)((IC + U - 1 + L.H - 1) / L.H);
  L.kb_off = (long long)L.nblk * L.nfr * (W + rep) * 64;
  L.pair_floats = L.kb_off + (L.nblk > 1 ? 2LL * L.nblk * (IC * rep + 1) : 0);
  return L;
}
// Past dyadic 3 the adjoint runs on the increment tiles with kernel cells 2^(dyadic - 3) finer than the
// coarse grid (pde_bwd_sub): the layout of that grid.
__host__ __device__ inline int pde_bwd_sub(int dyadic) { return dyadic > 3 ? dyadic - 3 : 0; }
__host__ __device__ inline PdeLayout pde_layout_eff(int l1, int l2, int dyadic) {
  const int sub = pde_bwd_sub(dyadic);
  if (sub == 0) return pde_layout(l1, l2, dyadic);
  if (((long long)(l1 - 1) << sub) > (1 << 24) || ((long long)(l2 - 1) << sub) > (1 << 24)) return PdeLayout{};
  return pde_layout(((l1 - 1) << sub) + 1, ((l2 - 1) << sub) + 1, 3);
}
// fp32 words of the adjoint's workspace for one pair (0: unsupported)
inline long long pde_front_floats(int l1, int l2, int dyadic) { return pde_layout_eff(l1, l2, dyadic).pair_floats; }

// LDS of one wave (pair) of the adjoint kernel, in doubles
// (cross pairs: plus the lanes' column sums, 64 x WC x DP doubles: in LDS, not registers, for occupancy)
__host__ __device__ inline size_t pde_lds_wave_doubles(int IC, int DP, int WC = 0) {
  return ((size_t)IC * DP * 12 + 7) / 8 + (size_t)64 * WC * DP;
}

GPSIG_DEV double ld_l2_d(const double *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// MODE 0: both passes (gpsig_pde_vjp); 1: pass A only, plus the kernel value K[I][J] of every pair (the
// forward of a training step, gpsig_pde_fronts); 2: pass B only, from the fronts a MODE 1 launch left
// (gpsig_pde_vjp_fronts).
// Column blocks (J > 64 W): pass A sweeps the blocks left to right, the wave's lane 63 handing its right
// column of K to the next block through the workspace (lane 0 of that block reads it as its left
// boundary: pde_rep_kernel's slab, in HBM since pass B re-reads it); pass B sweeps them right to left,
// lane 0 handing its left column of R to the next block the same way (lane 63's right boundary).  The
// cells, recurrences and summation order within a cell are those of one block, so the result does not
// depend on the blocking beyond the order of the per-row atomics.
// V: the K scheme, a compile-time variant of the body (a runtime select per cell cost two v_cndmask per
// fp64 value): 0 the first-order scheme, 1 the second-order scheme (solver 1), 2 first order with the
// second-order formula on the diagonal cells (k(x, x) with solver 0, as the forward's hybrid).
template <int DP, int W, int REP, bool COLS, int MODE, int V>
__device__ __forceinline__ void pde_adj_body(const PdeBwdArgs &p, double *ldsd) {
  static_assert(W % REP == 0, "a lane owns whole coarse columns");
  constexpr bool TILE = DP == 0;
  constexpr int DPA = TILE ? 1 : DP;
  constexpr int WC = W / REP;
  constexpr int WC2 = (WC + 1) / 2;  // coarse columns in packed fp32 pairs (the contractions)
  constexpr int H = pde_chunk<W, REP>();
  // the chunk's K corners: fp64 up to 32 values per lane (the narrow geometries, where 32 more VGPRs keep the
  // occupancy), fp32 beyond
  using KC = typename std::conditional<(H * REP * W <= 32 && W <= 4), double, float>::type;
  constexpr int FW = W + REP;  // front words per lane: up[W], last[0 .. REP-2], corner_prev
  constexpr int CB = 64 * W;   // fine columns per block
  const int lane = threadIdx.x & 63;
  const int wave = wave_uniform(threadIdx.x >> 6);
  const bool diag = p.pair_mode == GPSIG_PAIRS_DIAG;
  int a, b;
  if (diag) {
    a = p.row_begin + (int)blockIdx.x * p.wpb + wave;
    b = a;
  } else {
    a = (p.tiles_a0 + (int)blockIdx.x / p.ntb) * p.wpb + wave;
    b = (int)blockIdx.x % p.ntb;
  }
  const bool ok = a >= p.row_begin && a < p.row_end && b < p.n2;  // wave-uniform
  if (!ok) { a = p.row_begin; b = diag ? a : 0; }

  const double inv_factor = 1.0 / (double)(REP * REP);
  const int sub = TILE ? p.sub : 0;
  const int IC = (p.l1 - 1) << sub, JC = (p.l2 - 1) << sub;
  const int J = JC * REP, I = IC * REP;
  const int d = p.d;
  const float *x = p.X + (long long)a * p.l1 * d;
  const float *y = p.Y + (long long)b * p.l2 * d;
  const long long pidx = diag ? (long long)(a - p.row_begin) : (long long)(a - p.row_begin) * p.n2 + b;
  const PdeLayout lay = pde_layout_eff(p.l1, p.l2, p.dyadic);
  const long long toff = TILE ? (long long)(a - p.inc_a0) * p.inc_as + (diag ? 0 : (long long)(b - p.inc_b0) * (p.l2 - 1)) : 0;
  const float *__restrict__ itile = TILE ? p.inc + toff : nullptr;
  float *__restrict__ gtile = TILE ? p.gt + toff : nullptr;
  const int nblk = lay.nblk;
  float *__restrict__ fr = p.fronts + pidx * lay.pair_floats;
  double *kbr = reinterpret_cast<double *>(fr + lay.kb_off);

  // LDS: [wave] { coarse-row accumulators (IC x DP doubles) | dx (IC x DP floats) }
  // LDS: [wave] { coarse-row accumulators (IC x DP doubles) | (COLS) column sums [WC x DP][64] doubles |
  //               dx (IC x DP floats) }
  constexpr int GCW = (COLS && !TILE) ? WC : 0;
  double *gacc = ldsd + (size_t)wave * pde_lds_wave_doubles(IC, DP, GCW);
  double *gcl = gacc + (size_t)IC * DP;
  float *dxs = reinterpret_cast<float *>(gcl + (size_t)64 * GCW * DP);
  if constexpr (!TILE) {
    for (int r = lane; r < IC; r += 64) {
#pragma unroll
      for (int k = 0; k < DP; ++k) {
        dxs[r * DP + k] = k < d ? x[(r + 1) * d + k] - x[r * d + k] : 0.0f;
        gacc[r * DP + k] = 0.0;
      }
    }
  }
  __syncthreads();

  // the current column block: first fine column, lanes used, y increments of the lane's coarse columns
  int c0 = 0, U = 0;
  f2 dyp[WC2][DPA];  // y increments of the lane's coarse columns as packed pairs (2 w2, 2 w2 + 1)
  auto load_block = [&](int blk) {
    c0 = blk * CB;
    U = (J - c0 + W - 1) / W;
    U = U < 64 ? U : 64;
    if constexpr (!TILE) {
      // columns past the sequence (the lane straddling J, lanes past it) take increment 0: their R stays
      // the boundary value 1 exactly (1 + 1 - 1), no per-cell guard, and they contract with dy = 0
#pragma unroll
      for (int w = 0; w < 2 * WC2; ++w) {
        const int cj = c0 / REP + lane * WC + w;
        const bool in = w < WC && cj < JC;
        const int cjc = cj < JC ? cj : JC - 1;
#pragma unroll
        for (int k = 0; k < DP; ++k) dyp[w / 2][k][w % 2] = (k < d && in) ? y[(cjc + 1) * d + k] - y[cjc * d + k] : 0.0f;
      }
    }
  };

  constexpr bool s1 = V == 1, hybrid = V == 2;
  auto incs = [&](int ci, double (&inc)[WC]) {
    if constexpr (TILE) {
#pragma unroll
      for (int w = 0; w < WC; ++w) {
        const int cj = c0 / REP + lane * WC + w;
        inc[w] = cj < JC ? (double)tile_inc_b(itile, p.inc_ld, sub, ci, cj) * inv_factor : 0.0;
      }
    } else {
      float dxv[DP];
      const float *dxr = dxs + ci * DP;
#pragma unroll
      for (int k = 0; k < DP; ++k) dxv[k] = dxr[k];
#pragma unroll
      for (int w = 0; w < WC; ++w) {
        float incf = 0.0f;
#pragma unroll
        for (int k = 0; k < DP; ++k) incf = __builtin_fmaf(dxv[k], dyp[w / 2][k][w % 2], incf);
        inc[w] = (double)incf * inv_factor;
      }
    }
  };

  // ---- K sweep state and one forward step (pde_rep_kernel's scheme); kc[r][w] = K(i, c) of cell (i, c)
  double up[W], last[REP], corner_prev;
  const double *kin = nullptr;  // the block's left boundary column K(., c0) (null: the boundary 1)
  auto kinit = [&]() {
#pragma unroll
    for (int w = 0; w < W; ++w) up[w] = 1.0;
#pragma unroll
    for (int r = 0; r < REP; ++r) last[r] = 1.0;
    corner_prev = 1.0;
  };
  // inco: the step's coarse increments (pass B's R sweep of the same step reuses them)
  // kc: KC (fp32 where the registers are short, fp64 otherwise: no conversions per cell)
  auto kstep = [&](int s, KC (&kc)[REP][W], double (&inco)[WC]) {
    double left[REP];
#pragma unroll
    for (int r = 0; r < REP; ++r) left[r] = lane_prev(last[r]);
    if (lane == 0) {
#pragma unroll
      for (int r = 0; r < REP; ++r) {
        const int i1 = s * REP + r + 1;
        left[r] = kin ? ld_l2_d(kin + (i1 < I ? i1 : I)) : 1.0;
      }
    }
    const int ci = s - lane;
    if (ci >= 0 && ci < IC && lane < U) {
      double inc[WC], A[WC], B[WC];
      incs(ci, inc);
#pragma unroll
      for (int w = 0; w < WC; ++w) {
        inco[w] = inc[w];
        const double inc2 = inc[w] * inc[w];
        A[w] = s1 ? 1.0 + 0.5 * inc[w] + (1.0 / 12) * inc2 : inc[w];
        B[w] = s1 ? 1.0 - (1.0 / 12) * inc2 : inc[w] - 1.0;  // (compile-time selects)
      }
#pragma unroll
      for (int r = 0; r < REP; ++r) {
        const int i = ci * REP + r;
        double lft = left[r];
        double cor = r == 0 ? corner_prev : left[r - 1];
        // columns c >= J are updated too (as pde_rep_kernel): they never reach a real cell
#pragma unroll
        for (int w = 0; w < W; ++w) {
          const double upw = up[w];
          double kn;
          if constexpr (s1) {
            kn = (upw + lft) * A[w / REP] - cor * B[w / REP];
          } else {
            kn = (upw + lft) + cor * B[w / REP];
            if (hybrid && c0 + lane * W + w == i) {
              const double t = A[w / REP], t2 = t * t;
              kn = (upw + lft) * (1.0 + 0.5 * t + (1.0 / 12) * t2) - cor * (1.0 - (1.0 / 12) * t2);
            }
          }
          kc[r][w] = (KC)cor;
          cor = upw;
          lft = kn;
          up[w] = kn;
        }
        last[r] = lft;
      }
    }
    corner_prev = left[REP - 1];
  };

  // ---- pass A: K forward block by block, a front every H steps (last[REP-1] is up[W-1] after any step)
  for (int blk = 0; MODE != 2 && ok && blk < nblk; ++blk) {
    load_block(blk);
    kin = blk > 0 ? kbr + (long long)blk * (I + 1) : nullptr;
    double *kout = blk + 1 < nblk ? kbr + (long long)(blk + 1) * (I + 1) : nullptr;
    float *fb = fr + (long long)blk * lay.nfr * FW * 64;
    kinit();
    const int nsteps = IC + U - 1;
    for (int s0 = 0; s0 < nsteps; s0 += H) {
      float *f = fb + (long long)(s0 / H) * FW * 64;
#pragma unroll
      for (int w = 0; w < W; ++w) f[w * 64 + lane] = (float)up[w];
#pragma unroll
      for (int r = 0; r + 1 < REP; ++r) f[(W + r) * 64 + lane] = (float)last[r];
      f[(W + REP - 1) * 64 + lane] = (float)corner_prev;
#pragma unroll
      for (int h = 0; h < H; ++h) {
        // steps past nsteps (the last chunk's tail) touch no cell: ci >= IC in every lane used
        KC kc[REP][W];
        double incd[WC];
        const int s = s0 + h;
        kstep(s, kc, incd);
        const int ci = s - 63;  // lane 63 (a full block) hands its right column on
        if (kout && lane == 63 && ci >= 0 && ci < IC) {
#pragma unroll
          for (int r = 0; r < REP; ++r) kout[ci * REP + r + 1] = last[r];
        }
      }
    }
  }

  if constexpr (MODE == 1) {
    // K[I][J] = the last row's value in fine column J - 1 (the forward op's value: same cells)
    const int owner = (J - 1 - c0) / W, slot = (J - 1 - c0) % W;
    double res = 0.0;
#pragma unroll
    for (int w = 0; w < W; ++w)
      if (w == slot) res = up[w];
    if (ok && lane == owner) {
      if (diag) p.out[a - p.row_begin] = (float)res;
      else p.out[(long long)(a - p.row_begin) * p.n2 + b] = (float)res;
    }
    return;
  }
  const float g = diag ? p.gout[a] : p.gout[(long long)a * p.n2 + b];
  // TILE: the coarse-cell sums scaled to dLoss/d<dx_i, dy_j> of the tile cell: 4^-n g (x2 for k(x, x)),
  // and 4^-sub for the kernel cells a tile cell covers (inc = tile / 4^sub)
  const double gts = TILE ? (diag ? 2.0 : 1.0) * inv_factor * (double)g / (double)(1 << (2 * sub)) : 0.0;
  // ---- pass B: blocks right to left, chunks backwards; the R sweep runs in its own step order
  double ru[W], rlast[REP], rcorner;
  f2 gcp[WC2][DPA];  // column sums S dx: fp32 pairs within a chunk, then fp64 in the lane's LDS slots (gcl)
  for (int blk = nblk - 1; ok && blk >= 0; --blk) {
    load_block(blk);
    kin = blk > 0 ? kbr + (long long)blk * (I + 1) : nullptr;
    const double *rin = blk + 1 < nblk ? kbr : nullptr;  // R(., c0 + CB), left by the block on the right
    double *rout = blk > 0 ? kbr : nullptr;                // R(., c0), for the block on the left
    const float *fb = fr + (long long)blk * lay.nfr * FW * 64;
#pragma unroll
    for (int w = 0; w < W; ++w) ru[w] = 1.0;
#pragma unroll
    for (int r = 0; r < REP; ++r) rlast[r] = 1.0;
    rcorner = 1.0;
    if constexpr (GCW > 0) {
#pragma unroll
      for (int e = 0; e < GCW * DP; ++e) gcl[e * 64 + lane] = 0.0;
    }
    const int nsteps = IC + U - 1;
    // the chunk's front, loaded one chunk ahead (the restore would otherwise wait on HBM at every chunk)
    float fv[FW];
    auto ldfront = [&](int c0s) {
      const float *f = fb + (long long)(c0s / H) * FW * 64;
#pragma unroll
      for (int e = 0; e < FW; ++e) fv[e] = f[e * 64 + lane];
    };
    ldfront(((nsteps - 1) / H) * H);
    for (int s0 = ((nsteps - 1) / H) * H; s0 >= 0; s0 -= H) {
#pragma unroll
      for (int w = 0; w < W; ++w) up[w] = (double)fv[w];
#pragma unroll
      for (int r = 0; r + 1 < REP; ++r) last[r] = (double)fv[W + r];
      last[REP - 1] = up[W - 1];
      corner_prev = (double)fv[W + REP - 1];
      if (s0 >= H) ldfront(s0 - H);
      KC kc[H][REP][W];
      double incH[H][WC];
#pragma unroll
      for (int w2 = 0; w2 < WC2; ++w2)
#pragma unroll
        for (int k = 0; k < DPA; ++k) gcp[w2][k] = splat2(0.0f);
      // steps past nsteps touch no cell (ci >= IC in every lane used), and in the R sweep they come first,
      // on the boundary values 1: no guards
#pragma unroll
      for (int h = 0; h < H; ++h) kstep(s0 + h, kc[h], incH[h]);
#pragma unroll
      for (int h = H - 1; h >= 0; --h) {
        double right[REP];
#pragma unroll
        for (int r = 0; r < REP; ++r) right[r] = lane_next_d(rlast[r]);
        if (lane == 63) {
#pragma unroll
          for (int r = 0; r < REP; ++r) {  // rows at or past I: the boundary 1
            const int pr = (s0 + h - 63) * REP + r;
            right[r] = rin && pr < I ? ld_l2_d(rin + (pr > 0 ? pr : 0)) : 1.0;
          }
        }
        const int ci = s0 + h - lane;
        if (ci >= 0 && ci < IC && lane < U) {
          double inc[WC], S[WC];
#pragma unroll
          for (int w = 0; w < WC; ++w) {
            inc[w] = incH[h][w] - 1.0;  // the K step's increments (same row ci)
            S[w] = 0.0;
          }
#pragma unroll
          for (int r = REP - 1; r >= 0; --r) {
            double rgt = right[r];
            double cor = r == REP - 1 ? rcorner : right[r + 1];
#pragma unroll
            for (int w = W - 1; w >= 0; --w) {
              const double upw = ru[w];
              const double rn = (upw + rgt) + cor * inc[w / REP];
              // KK[i][c] = K(i, c) * R(i+1, c+1) = K[i][c] * K_rev[I-1-i][J-1-c] (columns >= J: R = 1,
              // their sums meet dy = 0 and are not stored)
              S[w / REP] = __builtin_fma((double)kc[h][r][w], cor, S[w / REP]);  // (no-op cast for fp64 KC)
              cor = upw;
              rgt = rn;
              ru[w] = rn;
            }
            rlast[r] = rgt;
          }
          if (rout && lane == 0) {
#pragma unroll
            for (int r = 0; r < REP; ++r) rout[ci * REP + r] = rlast[r];
          }
          if constexpr (TILE) {
            // the lane's coarse cells of row ci (columns of the sequence only); several kernel cells share a
            // tile cell when sub > 0 (atomics), one writer otherwise
#pragma unroll
            for (int w = 0; w < WC; ++w) {
              const int cj = c0 / REP + lane * WC + w;
              if (cj < JC) {
                float *gp = gtile + (long long)(ci >> sub) * p.inc_ld + (cj >> sub);
                const float v = (float)(gts * S[w]);
                if (sub) unsafeAtomicAdd(gp, v);
                else *gp = v;
              }
            }
          } else {
            // contractions on packed fp32 pairs of coarse columns: the row sums (over the lane's WC columns,
            // then fp64 in the LDS row accumulators) and the column sums (fp32 over a chunk's H rows, then fp64)
            f2 Sp[WC2], gr[DP];
#pragma unroll
            for (int w2 = 0; w2 < WC2; ++w2)
              Sp[w2] = (f2){(float)S[2 * w2], 2 * w2 + 1 < WC ? (float)S[(2 * w2 + 1) % WC] : 0.0f};
#pragma unroll
            for (int k = 0; k < DP; ++k) {
              gr[k] = Sp[0] * dyp[0][k];
#pragma unroll
              for (int w2 = 1; w2 < WC2; ++w2) gr[k] = fma2(Sp[w2], dyp[w2][k], gr[k]);
            }
#pragma unroll
            for (int k = 0; k < DP; ++k)
              if (k < d) atomicAdd(gacc + ci * DP + k, (double)(gr[k][0] + gr[k][1]));
            if constexpr (COLS) {
              const float *dxr = dxs + ci * DP;
#pragma unroll
              for (int k = 0; k < DP; ++k) {
                const f2 dxk = splat2(dxr[k]);
#pragma unroll
                for (int w2 = 0; w2 < WC2; ++w2) gcp[w2][k] = fma2(Sp[w2], dxk, gcp[w2][k]);
              }
            }
          }
        }
        rcorner = right[0];
      }
      if constexpr (GCW > 0) {
#pragma unroll
        for (int w = 0; w < WC; ++w)
#pragma unroll
          for (int k = 0; k < DP; ++k) gcl[(w * DP + k) * 64 + lane] += (double)gcp[w / 2][k][w % 2];
      }
    }
    if constexpr (COLS && !TILE) {
      if (!diag) {
        // columns: H[j] = 4^-n sum over coarse column j; dK/dy_j = H[j-1] - H[j]
        const double sy = inv_factor * (double)g;
        float *gyb = p.gY + (long long)b * p.l2 * d;
#pragma unroll
        for (int w = 0; w < WC; ++w) {
          const int jc = c0 / REP + lane * WC + w;
          if (jc >= JC) continue;
#pragma unroll
          for (int k = 0; k < DP; ++k) {  // compile-time indices: a runtime bound would put gcol in scratch
            if (k >= d) continue;
            const float v = (float)(sy * gcl[(w * DP + k) * 64 + lane]);
            unsafeAtomicAdd(gyb + (long long)(jc + 1) * d + k, v);
            unsafeAtomicAdd(gyb + (long long)jc * d + k, -v);
          }
        }
      }
    }
  }
  __syncthreads();  // the row accumulators are complete
  if (!ok) return;
  if constexpr (TILE) return;  // the host contracts the tile with the increments

  // dK/dx_i = G[i-1] - G[i] with G[r] = 4^-n gacc[r] (x2 for k(x, x)), times the upstream gradient
  const double sx = (diag ? 2.0 : 1.0) * inv_factor * (double)g;
  float *gxa = p.gX + (long long)a * p.l1 * d;
  for (int r = lane; r <= IC; r += 64)
    for (int k = 0; k < d; ++k) {
      const double gp = r > 0 ? gacc[(r - 1) * DP + k] : 0.0;
      const double gc = r < IC ? gacc[r * DP + k] : 0.0;
      unsafeAtomicAdd(gxa + (long long)r * d + k, (float)(sx * (gp - gc)));
    }
}

template <int DP, int W, int REP, bool COLS, int MODE = 0>
__global__ __launch_bounds__(256) void pde_adj_kernel(PdeBwdArgs p) {
  extern __shared__ __attribute__((aligned(16))) double ldsd[];
  if (p.solver == 1) pde_adj_body<DP, W, REP, COLS, MODE, 1>(p, ldsd);
  else if (p.pair_mode == GPSIG_PAIRS_DIAG) pde_adj_body<DP, W, REP, COLS, MODE, 2>(p, ldsd);
  else pde_adj_body<DP, W, REP, COLS, MODE, 0>(p, ldsd);
}

template <int DP, int W, int REP, int MODE>
static int launch_pde_adj(const PdeBwdArgs &a, long long nblocks, hipStream_t s) {
  if constexpr (W < REP || REP * W > 64) {
    return GPSIG_EUNSUPPORTED;
  } else {
    // the column (dK/dy) accumulators only for cross pairs; k(x, x) takes twice the row part
    const bool cols = !(a.pair_mode == GPSIG_PAIRS_DIAG || MODE == 1);
    const size_t lds =
        DP == 0 ? 0 : (size_t)a.wpb * pde_lds_wave_doubles(a.l1 - 1, DP, cols ? W / REP : 0) * sizeof(double);
    if (lds > 160 * 1024) return GPSIG_EUNSUPPORTED;
    if (!cols)
      hipLaunchKernelGGL((pde_adj_kernel<DP, W, REP, false, MODE>), dim3((unsigned)nblocks), dim3(64 * a.wpb), lds, s, a);
    else
      hipLaunchKernelGGL((pde_adj_kernel<DP, W, REP, true, MODE>), dim3((unsigned)nblocks), dim3(64 * a.wpb), lds, s, a);
    return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
  }
}

template <int DP, int REP, int MODE>
static int pde_adj_w(const PdeBwdArgs &a, long long nblocks, int W, hipStream_t s) {
  switch (W) {
    case 1: return launch_pde_adj<DP, 1, REP, MODE>(a, nblocks, s);
    case 2: return launch_pde_adj<DP, 2, REP, MODE>(a, nblocks, s);
    case 4: return launch_pde_adj<DP, 4, REP, MODE>(a, nblocks, s);
    case 8: return launch_pde_adj<DP, 8, REP, MODE>(a, nblocks, s);
    case 16: return launch_pde_adj<DP, 16, REP, MODE>(a, nblocks, s);
    default: return GPSIG_EUNSUPPORTED;
  }
}

template <int DP, int MODE>
static int pde_adj_rep(const PdeBwdArgs &a, long long nblocks, hipStream_t s) {
  const int kd = a.dyadic - (DP == 0 ? a.sub : 0);  // the kernel's refinement (TILE: past the tile's cells)
  const int rep = 1 << kd;
  const int W = pde_bwd_cols(rep * ((a.l2 - 1) << (DP == 0 ? a.sub : 0)), rep);
  switch (kd) {
    case 0: return pde_adj_w<DP, 1, MODE>(a, nblocks, W, s);
    case 1: return pde_adj_w<DP, 2, MODE>(a, nblocks, W, s);
    case 2: return pde_adj_w<DP, 4, MODE>(a, nblocks, W, s);
    case 3: return pde_adj_w<DP, 8, MODE>(a, nblocks, W, s);
    default: return GPSIG_EUNSUPPORTED;
  }
}

// one channel count (pde_bwd_inst.hip, one unit per DP); mode as pde_adj_kernel's MODE
template <int DP>
int pde_bwd_launch_dp(const PdeBwdArgs &a, long long nblocks, int mode, hipStream_t s) {
  switch (mode) {
    case 0: return pde_adj_rep<DP, 0>(a, nblocks, s);
    case 1: return pde_adj_rep<DP, 1>(a, nblocks, s);
    case 2: return pde_adj_rep<DP, 2>(a, nblocks, s);
    default: return GPSIG_EINVAL;
  }
}

}  // namespace gpsig
