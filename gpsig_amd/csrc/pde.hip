// gpsig_amd -- Goursat-PDE (untruncated) signature kernel on gfx950.
//
// Replaces gpsig/sigKer_fast.pyx:15-62 (CPU, k(x,x) only) and the CUDA op
// gpsig/covariance_op/untrunc_cov_op_gpu.cu:5-94 (one 1024-thread block per pair, one thread per
// grid row, a __syncthreads per anti-diagonal, every cell through global memory).
//
// Here one wave64 solves one pair entirely in registers.  Lane l owns W consecutive fine columns and
// sweeps the rows with a one-step skew: at step s it updates row i = s - l, taking the left boundary
// K[i+1][lW] from lane l-1 (computed one step earlier) through a single DPP wave_shr:1, and the
// corner K[i][lW] from the previous step's left boundary.  No LDS traffic for the solution, no
// barriers, no 1024-row cap (kernels_pde.py:53); the coarse increments of x (the only lane-varying
// input) sit in LDS, y's increments for the lane's columns in registers.
//   inc(i, j) = <dx_{i>>n}, dy_{j>>n}> / 4^n                         (sigKer_fast.pyx:35-43)
//   solver 1: K[i+1][j+1] = (K[i][j+1] + K[i+1][j]) (1 + inc/2 + inc^2/12) - K[i][j] (1 - inc^2/12)
//   solver 0: K[i+1][j+1] = K[i][j+1] + K[i+1][j] + K[i][j] (inc - 1)
// In DIAG mode with solver 0 the diagonal cells take the solver-1 update, as sigKer_fast.pyx:59 does.
#include "sig_common.h"
#include "gemm.h"

namespace gpsig {

struct PdeArgs {
  const float *X, *Y;
  int n1, l1, n2, l2, d;
  int dyadic, solver;
  int pair_mode, row_begin, row_end;
  int ntb, tiles_a0;
  long long tile_base;
  float *out;
  int out_row0, out_rows;
  long long out_ld;
  // DP == 0 (increment tiles, any channel count): the coarse increment Gram <dx_i, dy_j> of pair (a, b)
  // at inc + (a - inc_a0) inc_as + (b - inc_b0) (l2 - 1) + i inc_ld + j (DIAG: + i inc_ld + j), computed
  // by the matrix-core GEMM (gemm.hip) -- the reference's own split (kernels_pde.py:176 tf.matmul, then
  // the solver).  sub > 0: the kernel's grid is 2^sub times finer than the tile (each tile cell covers
  // 2^sub x 2^sub kernel cells, value / 4^sub).
  const float *inc;
  long long inc_as, inc_ld;
  int inc_a0, inc_b0, sub;
};

// increment of kernel cell (ci, cj) from the tile (DP == 0 kernels)
GPSIG_DEV float tile_inc(const float *__restrict__ base, long long ld, int sub, int ci, int cj) {
  const float v = base[(long long)(ci >> sub) * ld + (cj >> sub)];
  return sub ? v * __builtin_ldexpf(1.0f, -2 * sub) : v;
}

template <typename T, int DP, int W>
__global__ __launch_bounds__(256) void pde_kernel(PdeArgs p) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int lane = threadIdx.x & 63;
  const int wave = wave_uniform(threadIdx.x >> 6);

  int a, b;
  if (p.pair_mode == GPSIG_PAIRS_DIAG) {
    a = p.row_begin + (int)blockIdx.x * 4 + wave;
    b = a;
  } else {
    int ta, tb;
    if (p.pair_mode == GPSIG_PAIRS_UPPER) {
      const Tile t = upper_tile(p.tile_base + (long long)blockIdx.x, p.ntb, 4);
      ta = t.ta;
      tb = t.tb;
    } else {
      ta = p.tiles_a0 + (int)blockIdx.x / p.ntb;
      tb = (int)blockIdx.x % p.ntb;
    }
    a = ta * 4 + wave;
    b = tb;
  }
  // wave-uniform validity; every wave still reaches the LDS barrier below
  bool ok = a >= p.row_begin && a < p.row_end && b < p.n2;
  if (p.pair_mode == GPSIG_PAIRS_UPPER && b < a) ok = false;
  if (!ok) { a = p.row_begin; b = p.pair_mode == GPSIG_PAIRS_RECT ? 0 : a; }

  const int n = p.dyadic;
  const int rep = 1 << n;
  const T inv_factor = (T)1.0 / (T)(1 << (2 * n));
  const int I = rep * (p.l1 - 1), J = rep * (p.l2 - 1);
  const int d = p.d;
  const float *x = p.X + (long long)a * p.l1 * d;
  const float *y = p.Y + (long long)b * p.l2 * d;

  // coarse increments of x in this wave's LDS slice: (l1-1) x DP
  float *dxs = lds + (size_t)wave * (p.l1 - 1) * DP;
  for (int r = lane; r < p.l1 - 1; r += 64)
#pragma unroll
    for (int k = 0; k < DP; ++k) dxs[r * DP + k] = k < d ? x[(r + 1) * d + k] - x[r * d + k] : 0.0f;

  // y increments for this lane's fine columns c = lane*W + w (coarse column c >> n)
  float dy[W][DP];
#pragma unroll
  for (int w = 0; w < W; ++w) {
    int cj = (lane * W + w) >> n;
    cj = cj < p.l2 - 2 ? cj : p.l2 - 2;
#pragma unroll
    for (int k = 0; k < DP; ++k) dy[w][k] = k < d ? y[(cj + 1) * d + k] - y[cj * d + k] : 0.0f;
  }
  __syncthreads();
  if (!ok) return;

  const bool hybrid = (p.pair_mode == GPSIG_PAIRS_DIAG) && p.solver == 0;
  T up[W];
#pragma unroll
  for (int w = 0; w < W; ++w) up[w] = (T)1;
  T last = (T)1;   // K[i+1][lW+W] of this lane's most recent row (boundary 1 before it starts)
  T left_prev = (T)1;
  const int lanes_used = (J + W - 1) / W;
  const int nsteps = I + lanes_used - 1;
  for (int s = 0; s < nsteps; ++s) {
    T left = lane_prev(last);
    if (lane == 0) left = (T)1;
    const T corner0 = left_prev;
    left_prev = left;
    const int i = s - lane;
    if (i >= 0 && i < I && lane < lanes_used) {
      const float *dxr = dxs + (i >> n) * DP;
      float dxv[DP];
#pragma unroll
      for (int k = 0; k < DP; ++k) dxv[k] = dxr[k];
      T lft = left, cor = corner0;
#pragma unroll
      for (int w = 0; w < W; ++w) {
        const int c = lane * W + w;
        float incf = 0.0f;
#pragma unroll
        for (int k = 0; k < DP; ++k) incf = __builtin_fmaf(dxv[k], dy[w][k], incf);
        const T inc = (T)incf * inv_factor;
        const T upw = up[w];
        T kn;
        if (p.solver == 1 || (hybrid && c == i)) {
          const T inc2 = inc * inc;
          const T A = (T)1 + (T)0.5 * inc + (T)(1.0 / 12) * inc2;
          const T B = (T)1 - (T)(1.0 / 12) * inc2;
          kn = (upw + lft) * A - cor * B;
        } else {
          kn = (upw + lft) + cor * (inc - (T)1);
        }
        if (c < J) {
          cor = upw;
          lft = kn;
          up[w] = kn;
        }
      }
      last = lft;
    }
  }
  // final corner K[I][J]: fine column J-1 -> lane (J-1)/W, slot (J-1)%W
  const int owner = (J - 1) / W, slot = (J - 1) % W;
  T res = (T)0;
#pragma unroll
  for (int w = 0; w < W; ++w)
    if (w == slot) res = up[w];
  if (lane == owner) {
    const float v = (float)res;
    if (p.pair_mode == GPSIG_PAIRS_DIAG) {
      p.out[a] = v;
    } else {
      if (a >= p.out_row0 && a < p.out_row0 + p.out_rows) p.out[(long long)(a - p.out_row0) * p.out_ld + b] = v;
      if (p.pair_mode == GPSIG_PAIRS_UPPER && a != b && b >= p.out_row0 && b < p.out_row0 + p.out_rows)
        p.out[(long long)(b - p.out_row0) * p.out_ld + a] = v;
    }
  }
}

// Coarse-row stepping (REP = 2^dyadic fine rows per step).  The increment of a coarse cell is shared
// by its REP x REP fine cells (sigKer_fast.pyx:35-43 recomputes it per fine cell), so each step
// evaluates the lane's W/REP coarse increments and update coefficients once and then sweeps REP fine
// rows x W fine columns; the skew is one step per coarse row, the left boundary of the REP rows comes
// from lane l-1 (REP DPP moves per step).
//
// Column blocks (more than 64 W fine columns): the wave sweeps the grid in blocks of 64 W columns,
// left to right.  The last lane of a block hands its right column K[i][c0 + 64 W - 1] (all rows i) to
// the next block through this wave's LDS slab `bnd` (I + 1 doubles), where lane 0 reads it as its left
// boundary; lane 0 reads row i at step i and the last lane overwrites it at step i + 63, so one slab
// serves every block in place.
//
// LP < 64 (Gram pairs, grids of at most LP W fine columns): G = 64 / LP pairs (a, b..b+G-1) per wave, one
// lane group of LP lanes each, sharing x's increments.  Fewer lanes per pair shorten the skew (IC + U - 1
// steps for U lanes) and leave fewer lanes idle, at W columns per lane.
template <typename T, int DP, int W, int REP, int SOLVER, int LP = 64>
__global__ __launch_bounds__(256) void pde_rep_kernel(PdeArgs p) {
  static_assert(W % REP == 0, "a lane owns whole coarse columns");
  static_assert(LP == 16 || LP == 32 || LP == 64, "lane group");
  constexpr bool TILE = DP == 0;  // increments from the tile (any channel count)
  constexpr int DPA = TILE ? 1 : DP;
  constexpr int WC = W / REP;
  constexpr int G = 64 / LP;
  constexpr int CB = LP * W;  // fine columns per block (G > 1: one block)
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int lane = threadIdx.x & 63;
  const int wave = wave_uniform(threadIdx.x >> 6);
  const int g = lane / LP, gl = lane % LP;

  int a, b;
  if (p.pair_mode == GPSIG_PAIRS_DIAG) {
    a = p.row_begin + (int)blockIdx.x * 4 + wave;
    b = a;
  } else {
    int ta, tb;
    if (p.pair_mode == GPSIG_PAIRS_UPPER) {
      const Tile t = upper_tile(p.tile_base + (long long)blockIdx.x, p.ntb, 4 / G);
      ta = t.ta;
      tb = t.tb;
    } else {
      ta = p.tiles_a0 + (int)blockIdx.x / p.ntb;
      tb = (int)blockIdx.x % p.ntb;
    }
    a = ta * 4 + wave;
    b = tb * G + g;
  }
  // a is wave-uniform; b per lane group (G > 1: an invalid group computes on a clamped pair, stores nothing)
  const bool aok = a >= p.row_begin && a < p.row_end;
  bool bok = b < p.n2;
  if (p.pair_mode == GPSIG_PAIRS_UPPER && b < a) bok = false;
  const bool ok = aok && bok;  // wave-uniform when G == 1
  if (!aok) a = p.row_begin;
  if (!bok) b = p.pair_mode == GPSIG_PAIRS_RECT ? 0 : a;

  const T inv_factor = (T)1.0 / (T)(REP * REP);
  // coarse rows / columns (TILE with sub > 0: the tile's cells split 2^sub ways per direction)
  const int IC = (p.l1 - 1) << (TILE ? p.sub : 0), JC = (p.l2 - 1) << (TILE ? p.sub : 0);
  const int I = REP * IC, J = REP * JC;
  const int nblk = (J + CB - 1) / CB;
  const int d = p.d;
  const float *x = p.X + (long long)a * p.l1 * d;
  const float *y = p.Y + (long long)b * p.l2 * d;

  float *dxs = lds + (size_t)wave * IC * DP;
  if constexpr (!TILE) {
    for (int r = lane; r < IC; r += 64)
#pragma unroll
      for (int k = 0; k < DP; ++k) dxs[r * DP + k] = k < d ? x[(r + 1) * d + k] - x[r * d + k] : 0.0f;
  }
  T *bnd = reinterpret_cast<T *>(lds + (((size_t)4 * IC * DP + 3) & ~(size_t)3)) + (size_t)wave * (I + 1);
  __syncthreads();
  if (!aok || (G == 1 && !ok)) return;
  // this pair's increment tile (TILE)
  const float *__restrict__ itile =
      TILE ? p.inc + (long long)(a - p.inc_a0) * p.inc_as +
                 (p.pair_mode == GPSIG_PAIRS_DIAG ? 0 : (long long)(b - p.inc_b0) * (p.l2 - 1))
           : nullptr;

  const bool hybrid = (p.pair_mode == GPSIG_PAIRS_DIAG) && SOLVER == 0;
  constexpr bool s1 = SOLVER == 1;
  // coarse increments of a lane's columns as packed fp32 pairs (2w, 2w + 1): the dots of a step are
  // v_pk_fma_f32 with x's increment broadcast
  constexpr int WC2 = (WC + 1) / 2;
  T up[W];
  for (int blk = 0; blk < nblk; ++blk) {
    const int c0 = blk * CB;  // first fine column of the block (a multiple of REP)
    const bool from_left = blk > 0, to_right = blk + 1 < nblk;
    // y increments of this lane's coarse columns
    f2 dy[WC2][DPA];
    if constexpr (!TILE) {
#pragma unroll
      for (int w = 0; w < 2 * WC2; ++w) {
        int cj = c0 / REP + gl * WC + w;
        cj = cj < JC - 1 ? cj : JC - 1;
#pragma unroll
        for (int k = 0; k < DP; ++k) dy[w / 2][k][w % 2] = (k < d && w < WC) ? y[(cj + 1) * d + k] - y[cj * d + k] : 0.0f;
      }
    }
#pragma unroll
    for (int w = 0; w < W; ++w) up[w] = (T)1;
    T last[REP];  // K[row][c0 + lane*W + W - 1] of this lane's REP rows of the previous step
#pragma unroll
    for (int r = 0; r < REP; ++r) last[r] = (T)1;
    T corner_prev = (T)1;  // left boundary of the previous step's last row
    const int lanes_used = min(LP, (J - c0 + W - 1) / W);
    const int nsteps = IC + lanes_used - 1;
    for (int s = 0; s < nsteps; ++s) {
      T left[REP];
#pragma unroll
      for (int r = 0; r < REP; ++r) {
        left[r] = lane_prev(last[r]);
        if (gl == 0) left[r] = (G == 1 && from_left) ? bnd[min(s * REP + r + 1, I)] : (T)1;
      }
      const int ci = s - gl;
      if (ci >= 0 && ci < IC && gl < lanes_used) {
        f2 incp[WC2];
        if constexpr (TILE) {
          // the tile's coarse increments (columns past the sequence read its last column: never a real cell)
#pragma unroll
          for (int w = 0; w < 2 * WC2; ++w) {
            int cj = c0 / REP + gl * WC + w;
            cj = cj < JC - 1 ? cj : JC - 1;
            incp[w / 2][w % 2] = w < WC ? tile_inc(itile, p.inc_ld, p.sub, ci, cj) : 0.0f;
          }
        } else {
        const float *dxr = dxs + ci * DP;
        float dxv[DP];
#pragma unroll
        for (int k = 0; k < DP; ++k) dxv[k] = dxr[k];
#pragma unroll
        for (int w2 = 0; w2 < WC2; ++w2) {
          f2 acc = dy[w2][0] * splat2(dxv[0]);
#pragma unroll
          for (int k = 1; k < DP; ++k) acc = fma2(dy[w2][k], splat2(dxv[k]), acc);
          incp[w2] = acc;
        }
        }
        // coefficients of the lane's coarse cells: solver 1 uses (A, B), solver 0 uses inc - 1 (as B)
        T A[WC], B[WC];
#pragma unroll
        for (int w = 0; w < WC; ++w) {
          const float incf = incp[w / 2][w % 2];
          const T inc = (T)incf * inv_factor;
          const T inc2 = inc * inc;
          if constexpr (s1) {
            A[w] = (T)1 + (T)0.5 * inc + (T)(1.0 / 12) * inc2;
            B[w] = (T)1 - (T)(1.0 / 12) * inc2;
          } else {
            A[w] = inc;  // hybrid diagonal cells need inc
            B[w] = inc - (T)1;
          }
        }
#pragma unroll
        for (int r = 0; r < REP; ++r) {
          const int i = ci * REP + r;
          T lft = left[r];
          T cor = r == 0 ? corner_prev : left[r - 1];
          // Columns c >= J (padding of the lane straddling J, and lanes past it) are updated too: the
          // solution only flows right and down, so they never reach a real cell, and the lane's last
          // column hands its value only to lanes that are all padding.
#pragma unroll
          for (int w = 0; w < W; ++w) {
            const T upw = up[w];
            T kn;
            if constexpr (s1) {
              kn = (upw + lft) * A[w / REP] - cor * B[w / REP];
            } else {
              kn = (upw + lft) + cor * B[w / REP];
              if (hybrid && c0 + lane * W + w == i) {
                const T inc = A[w / REP], inc2 = inc * inc;
                kn = (upw + lft) * ((T)1 + (T)0.5 * inc + (T)(1.0 / 12) * inc2) - cor * ((T)1 - (T)(1.0 / 12) * inc2);
              }
            }
            cor = upw;
            lft = kn;
            up[w] = kn;
          }
          last[r] = lft;
        }
        if (G == 1 && to_right && lane == 63) {
#pragma unroll
          for (int r = 0; r < REP; ++r) bnd[ci * REP + r + 1] = last[r];
        }
      }
      corner_prev = left[REP - 1];
    }
  }
  const int c0 = (nblk - 1) * CB;
  const int owner = (J - 1 - c0) / W, slot = (J - 1 - c0) % W;
  T res = (T)0;
#pragma unroll
  for (int w = 0; w < W; ++w)
    if (w == slot) res = up[w];
  if (gl == owner && ok) {
    const float v = (float)res;
    if (p.pair_mode == GPSIG_PAIRS_DIAG) {
      p.out[a] = v;
    } else {
      if (a >= p.out_row0 && a < p.out_row0 + p.out_rows) p.out[(long long)(a - p.out_row0) * p.out_ld + b] = v;
      if (p.pair_mode == GPSIG_PAIRS_UPPER && a != b && b >= p.out_row0 && b < p.out_row0 + p.out_rows)
        p.out[(long long)(b - p.out_row0) * p.out_ld + a] = v;
    }
  }
}

// LDS of a pde_rep_kernel launch: the 4 waves' coarse x increments, then (column blocks only) their
// boundary-column slabs
template <typename T, int DP, int W, int REP>
static size_t pde_rep_lds(int l1, int l2, int sub) {
  // sub > 0 (tile mode): the kernel's coarse cells are the tile's split 2^sub ways
  const long long IC = (long long)(l1 - 1) << sub, JC = (long long)(l2 - 1) << sub;
  const size_t dx = ((size_t)4 * IC * DP + 3) & ~(size_t)3;
  const long long J = REP * JC;
  const size_t bnd = J > 64 * W ? (size_t)4 * (REP * IC + 1) * sizeof(T) : 0;
  return dx * sizeof(float) + bnd;
}

template <typename T, int DP, int W, int REP>
static int launch_pde_rep(const PdeArgs &a, long long nblocks, hipStream_t s) {
  if constexpr ((W / REP) * DP > 64) {
    return -1;  // the per-row kernel keeps fewer increments in registers
  } else {
    const size_t lds = pde_rep_lds<T, DP, W, REP>(a.l1, a.l2, a.inc ? a.sub : 0);
    if (lds > 160 * 1024) return GPSIG_EUNSUPPORTED;
    if (a.solver == 1)
      hipLaunchKernelGGL((pde_rep_kernel<T, DP, W, REP, 1>), dim3((unsigned)nblocks), dim3(256), lds, s, a);
    else
      hipLaunchKernelGGL((pde_rep_kernel<T, DP, W, REP, 0>), dim3((unsigned)nblocks), dim3(256), lds, s, a);
    return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
  }
}

// Lane-group geometry for Gram pairs (solver 1, the reference's default): G = 64 / LP pairs per wave,
// W fine columns per lane with LP W >= J (no column blocks).  Per pair the wave issues about
// steps (3 REP W + (DP/2 + 7) W/REP + 2 REP + 12) / G instructions, steps = IC + ceil(J/W) - 1
// (the skew); the smallest estimate among LP = 16, 32 (W = 8, 14, 16, 24; 14 fits grids of 2^n (L-1) a
// little under 32 x 14 = 448 columns, e.g. C3's 398, at 89 % of the lanes' columns instead of 78 %) and
// the one-pair-per-wave
// geometry of pde_rep_w wins.  GPSIG_PDE_LP = 16 / 32 / 64 pins the lane group (A/B).
struct PdeLp { int LP, W; };
// register budget of a lane group's coarse increments: (W / REP) * DP floats; W = 26 (C3: 16 x 26 = 416
// columns for 398, four pairs per wave) fits 13 x 5 at 194 VGPRs
constexpr int pde_lp_regs(int W) { return W == 26 ? 65 : 64; }
inline double pde_cost(int IC, int J, int REP, int DP, int W, int G) {
  const int U = (J + W - 1) / W;
  return (double)(IC + U - 1) * (3.0 * REP * W + (DP / 2.0 + 7.0) * W / REP + 2.0 * REP + 12.0) / G;
}
inline int pde_w64(int J, int REP) {  // W of pde_rep_w's one-pair-per-wave geometry
  if (J <= 64 * REP) return REP;
  if (J <= 128 * REP && 2 * REP <= 16) return 2 * REP;
  if (REP <= 4 && J <= 192 * REP) return 3 * REP;
  return 4 * REP;
}
inline PdeLp pde_pick_lp(int IC, int J, int REP, int DP) {
  static const int force = [] { const char *e = getenv("GPSIG_PDE_LP"); return e ? atoi(e) : 0; }();
  PdeLp best{64, 0};
  if (force == 64) return best;
  double bc = pde_cost(IC, J, REP, DP, pde_w64(J, REP), 1);
  for (int LP : {16, 32})
    for (int W : {8, 14, 16, 24, 26}) {
      if (W % REP || LP * W < J || (W / REP) * DP > pde_lp_regs(W)) continue;
      if (W == 26 && LP != 16) continue;
      if (force && force != LP) continue;
      const double c = pde_cost(IC, J, REP, DP, W, 64 / LP);
      if (force ? (best.LP == 64 || c < bc) : c < bc) { bc = c; best = {LP, W}; }
    }
  return best;
}

template <typename T, int DP, int W, int REP, int LP>
static int launch_pde_lp(const PdeArgs &a, long long nblocks, hipStream_t s) {
  if constexpr (W % REP != 0 || (W / REP) * DP > pde_lp_regs(W)) {
    return GPSIG_EUNSUPPORTED;
  } else {
    const size_t lds = ((size_t)4 * (a.l1 - 1) * DP + 3) / 4 * 4 * sizeof(float);
    if (lds > 160 * 1024) return GPSIG_EUNSUPPORTED;
    hipLaunchKernelGGL((pde_rep_kernel<T, DP, W, REP, 1, LP>), dim3((unsigned)nblocks), dim3(256), lds, s, a);
    return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
  }
}

template <typename T, int DP, int REP>
static int pde_lp_dispatch(const PdeArgs &a, long long nblocks, PdeLp g, hipStream_t s) {
#define GPSIG_LPW(lp, w) \
  if (g.LP == lp && g.W == w) return launch_pde_lp<T, DP, w, REP, lp>(a, nblocks, s);
  GPSIG_LPW(16, 8) GPSIG_LPW(16, 14) GPSIG_LPW(16, 16) GPSIG_LPW(16, 24) GPSIG_LPW(16, 26)
  GPSIG_LPW(32, 8) GPSIG_LPW(32, 14) GPSIG_LPW(32, 16) GPSIG_LPW(32, 24)
#undef GPSIG_LPW
  return GPSIG_EUNSUPPORTED;
}

// W = the smallest multiple of REP with J / W <= 64 lanes (-1: use the per-row kernel).  Longer grids run
// in column blocks of 64 W fine columns: W = 4 REP for REP <= 4, 16 for REP = 8 and 16 (dyadic 3 and 4).
template <typename T, int DP, int REP>
static int pde_rep_w(const PdeArgs &a, long long nblocks, int J, hipStream_t s) {
  if (J <= 64 * REP) return launch_pde_rep<T, DP, REP, REP>(a, nblocks, s);
  if (J <= 128 * REP && 2 * REP <= 16) return launch_pde_rep<T, DP, (2 * REP <= 16 ? 2 * REP : REP), REP>(a, nblocks, s);
  if (REP <= 4 && J <= 192 * REP) return launch_pde_rep<T, DP, (REP <= 4 ? 3 * REP : REP), REP>(a, nblocks, s);
  if (REP <= 4 && J <= 256 * REP) return launch_pde_rep<T, DP, (REP <= 4 ? 4 * REP : REP), REP>(a, nblocks, s);
  // longer: column blocks of 256 * REP fine columns (REP <= 4) or 1024 (REP 8, 16)
  if (REP <= 4) return launch_pde_rep<T, DP, (REP <= 4 ? 4 * REP : REP), REP>(a, nblocks, s);
  if (REP <= 16) return launch_pde_rep<T, DP, 16, (REP <= 16 ? REP : 16)>(a, nblocks, s);
  return -1;
}

template <typename T, int DP, int W>
static int launch_pde(const PdeArgs &a, long long nblocks, hipStream_t s) {
  if constexpr (W * DP > 128) {
    return GPSIG_EUNSUPPORTED;
  } else {
    const size_t lds = (size_t)4 * (a.l1 - 1) * DP * sizeof(float);
    if (lds > 64 * 1024) return GPSIG_EUNSUPPORTED;
    hipLaunchKernelGGL((pde_kernel<T, DP, W>), dim3((unsigned)nblocks), dim3(256), lds, s, a);
    return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
  }
}

template <typename T, int DP>
static int pde_w(const PdeArgs &a, long long nblocks, int J, PdeLp g, hipStream_t s) {
  if constexpr (DP > 0) {
    if (g.LP != 64) {
      if (a.dyadic == 0) return pde_lp_dispatch<T, DP, 1>(a, nblocks, g, s);
      if (a.dyadic == 1) return pde_lp_dispatch<T, DP, 2>(a, nblocks, g, s);
      if (a.dyadic == 2) return pde_lp_dispatch<T, DP, 4>(a, nblocks, g, s);
      return GPSIG_EUNSUPPORTED;
    }
  }
  {
    // kernel grid 2^(dyadic - sub) (TILE with sub > 0: the tile is 2^sub coarser than the kernel's cells)
    const int kd = a.dyadic - a.sub;
    int rc = -1;
    if (kd == 0) rc = pde_rep_w<T, DP, 1>(a, nblocks, J, s);
    if (kd == 1) rc = pde_rep_w<T, DP, 2>(a, nblocks, J, s);
    if (kd == 2) rc = pde_rep_w<T, DP, 4>(a, nblocks, J, s);
    if (kd == 3) rc = pde_rep_w<T, DP, 8>(a, nblocks, J, s);
    if (kd == 4) rc = pde_rep_w<T, DP, 16>(a, nblocks, J, s);
    if (rc != -1) return rc;
  }
  if constexpr (DP == 0) {
    return GPSIG_EUNSUPPORTED;
  } else {
    if (J <= 64) return launch_pde<T, DP, 1>(a, nblocks, s);
    if (J <= 128) return launch_pde<T, DP, 2>(a, nblocks, s);
    if (J <= 256) return launch_pde<T, DP, 4>(a, nblocks, s);
    if (J <= 512) return launch_pde<T, DP, 8>(a, nblocks, s);
    if (J <= 1024) return launch_pde<T, DP, 16>(a, nblocks, s);
    return GPSIG_EUNSUPPORTED;
  }
}

// a: inputs, mode, rows and output filled; a.inc != nullptr selects the increment-tile kernels (DP == 0)
static int pde_launch_args(PdeArgs a, hipStream_t s) {
  const int n2 = a.n2, l1 = a.l1, l2 = a.l2, d = a.d, dyadic = a.dyadic, solver = a.solver;
  const int pair_mode = a.pair_mode, row_begin = a.row_begin, row_end = a.row_end;
  const bool tile = a.inc != nullptr;
  const int J = (1 << dyadic) * (l2 - 1);
  const int DPI = d <= 8 ? d : 16;
  // lane groups of Gram pairs: solver 1, dyadic <= 2, d <= 8 (pde_pick_lp)
  PdeLp lpg{64, 0};
  if (!tile && pair_mode != GPSIG_PAIRS_DIAG && solver == 1 && dyadic <= 2 && d <= 8 && l1 >= 2 && l2 >= 2)
    lpg = pde_pick_lp(l1 - 1, J, 1 << dyadic, DPI);
  const int G = 64 / lpg.LP;
  long long nblocks;
  if (pair_mode == GPSIG_PAIRS_DIAG) {
    nblocks = (row_end - row_begin + 3) / 4;
  } else {
    const int ta0 = row_begin / 4, ta1 = (row_end + 3) / 4;
    const int ntb = (n2 + G - 1) / G;
    a.ntb = ntb;
    a.tiles_a0 = ta0;
    if (pair_mode == GPSIG_PAIRS_RECT) {
      nblocks = (long long)(ta1 - ta0) * ntb;
    } else {
      const long long k = 4 / G;
      auto P = [&](long long r) { return r * (long long)ntb - k * r * (r - 1) / 2; };
      a.tile_base = P(ta0);
      nblocks = P(ta1) - a.tile_base;
    }
  }
  if (nblocks <= 0) return GPSIG_OK;
  if (nblocks > 0x7fffffffLL) return GPSIG_EUNSUPPORTED;
  using T = double;  // fp64 solution grid (the reference's float64), fp32 increments (as the CUDA op, .cu:27)
  if (tile) return pde_w<T, 0>(a, nblocks, J, lpg, s);
  switch (d <= 8 ? d : (d <= 16 ? 16 : 0)) {
#define CASE(v) \
  case v: return pde_w<T, v>(a, nblocks, J, lpg, s);
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8) CASE(16)
#undef CASE
    default: return GPSIG_EUNSUPPORTED;
  }
}

int pde_launch(const float *X, int n1, int l1, const float *Y, int n2, int l2, int d, int dyadic, int solver,
               int pair_mode, int row_begin, int row_end, float *out, int out_row0, int out_rows,
               long long out_ld, hipStream_t s) {
  PdeArgs a{};
  a.X = X; a.Y = Y;
  a.n1 = n1; a.l1 = l1; a.n2 = n2; a.l2 = l2; a.d = d;
  a.dyadic = dyadic; a.solver = solver;
  a.pair_mode = pair_mode; a.row_begin = row_begin; a.row_end = row_end;
  a.out = out; a.out_row0 = out_row0; a.out_rows = out_rows; a.out_ld = out_ld;
  return pde_launch_args(a, s);
}

// ------------------------------------------------------------------------------------ increment tiles

// dX[a][i][k] = x[a][i+1][k] - x[a][i][k]: the coarse increments, (n, l-1, d) row-major
__global__ __launch_bounds__(256) void increments_kernel(const float *__restrict__ X, int n, int l, int d,
                                                         float *__restrict__ dX) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long long)n * (l - 1) * d) return;
  const int k = (int)(idx % d);
  const long long r = idx / d;
  const long long a = r / (l - 1), i = r % (l - 1);
  const float *x = X + (a * l + i) * d + k;
  dX[idx] = x[d] - x[0];
}
int increments_launch(const float *X, int n, int l, int d, float *dX, hipStream_t s) {
  const long long tot = (long long)n * (l - 1) * d;
  hipLaunchKernelGGL(increments_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, X, n, l, d, dX);
  return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
}

static size_t al256p(size_t b) { return (b + 255) & ~(size_t)255; }
constexpr size_t PDE_TILE_BYTES = (size_t)1 << 30;  // increment tile of one chunk of x-rows

// x-rows per chunk of the tiled paths (a multiple of 4) and the tile's row length (also the higher-order
// Gram's tile mode, sig_ho.hip)
void pde_tile_chunk(int n1, int l1, int n2, int l2, int pair_mode, int &rows, long long &cols) {
  cols = pair_mode == GPSIG_PAIRS_DIAG ? (long long)(l1 - 1) : (long long)n2 * (l2 - 1);
  long long r = (long long)(PDE_TILE_BYTES / ((size_t)(l1 - 1) * cols * sizeof(float)));
  r = r < 4 ? 4 : (r / 4) * 4;
  if (r > ((n1 + 3) / 4) * 4) r = ((n1 + 3) / 4) * 4;
  rows = (int)r;
}

// The increment-tile path needs a scratch buffer; 0 when the fixed-channel kernels apply.
bool pde_tiled(int d, int dyadic) { return d > 16 || dyadic > 4; }
size_t pde_tile_scratch_bytes(int n1, int l1, int n2, int l2, int d, int pair_mode) {
  if (n1 <= 0 || n2 <= 0 || l1 < 2 || l2 < 2 || d <= 0) return 0;
  int rows;
  long long cols;
  pde_tile_chunk(n1, l1, n2, l2, pair_mode, rows, cols);
  const bool same = pair_mode != GPSIG_PAIRS_RECT;
  return al256p((size_t)n1 * (l1 - 1) * d * sizeof(float)) +
         (same ? 0 : al256p((size_t)n2 * (l2 - 1) * d * sizeof(float))) +
         al256p((size_t)rows * (l1 - 1) * cols * sizeof(float));
}

// Increment tiles of chunks of x-rows (one matrix-core GEMM each: dX_chunk dY^T, or per pair for DIAG),
// each followed by the tile-fed solver launch.  prep(a, c0, r1) fills the launch's rows and mode fields.
int pde_tiled_run(PdeArgs a, void *scratch, size_t scratch_bytes, hipStream_t s,
                  int (*launch)(PdeArgs, hipStream_t, void *), void *ctx) {
  const int n1 = a.n1, l1 = a.l1, n2 = a.n2, l2 = a.l2, d = a.d, pm = a.pair_mode;
  const int IC = l1 - 1, JC = l2 - 1;
  if (!scratch || scratch_bytes < pde_tile_scratch_bytes(n1, l1, n2, l2, d, pm)) return GPSIG_EWORKSPACE;
  int rows;
  long long cols;
  pde_tile_chunk(n1, l1, n2, l2, pm, rows, cols);
  char *w = static_cast<char *>(scratch);
  float *dX = reinterpret_cast<float *>(w);
  w += al256p((size_t)n1 * IC * d * sizeof(float));
  float *dY = dX;
  if (pm == GPSIG_PAIRS_RECT) {
    dY = reinterpret_cast<float *>(w);
    w += al256p((size_t)n2 * JC * d * sizeof(float));
  }
  float *T = reinterpret_cast<float *>(w);
  int rc = increments_launch(a.X, n1, l1, d, dX, s);
  if (rc) return rc;
  if (pm == GPSIG_PAIRS_RECT && (rc = increments_launch(a.Y, n2, l2, d, dY, s))) return rc;
  // kernel grid: 2^(dyadic - sub) fine cells per tile cell and direction (pde_rep_w takes up to 16)
  a.sub = a.dyadic > 4 ? a.dyadic - 4 : 0;
  a.inc = T;
  const int rb0 = a.row_begin, rb1 = a.row_end;
  for (int r0 = (rb0 / 4) * 4; r0 < rb1; r0 += rows) {
    const int r1 = r0 + rows < rb1 ? r0 + rows : rb1;
    const int c0 = r0 > rb0 ? r0 : rb0;
    PdeArgs c = a;
    c.row_begin = c0;
    c.row_end = r1;
    if (pm == GPSIG_PAIRS_DIAG) {
      c.inc_a0 = c0;
      c.inc_b0 = 0;
      c.inc_as = (long long)IC * IC;
      c.inc_ld = IC;
      rc = gemm_f32(s, false, true, IC, IC, d, 1.0f, dX + (long long)c0 * IC * d, d, (long long)IC * d,
                    dX + (long long)c0 * IC * d, d, (long long)IC * d, 0.0f, T, IC, (long long)IC * IC, r1 - c0, 0, 0,
                    nullptr, 0);
    } else {
      const int b0 = pm == GPSIG_PAIRS_UPPER ? r0 : 0;
      const long long tc = (long long)(n2 - b0) * JC;
      c.inc_a0 = r0;
      c.inc_b0 = b0;
      c.inc_as = (long long)IC * tc;
      c.inc_ld = tc;
      // UPPER: tiles whose x-rows all lie past their y-columns are never read (b >= a)
      rc = gemm_f32(s, false, true, (r1 - r0) * IC, (int)tc, d, 1.0f, dX + (long long)r0 * IC * d, d, 0,
                    dY + (long long)b0 * JC * d, d, 0, 0.0f, T, tc, 0, 1, pm == GPSIG_PAIRS_UPPER ? IC : 0,
                    pm == GPSIG_PAIRS_UPPER ? JC : 0, nullptr, 0);
    }
    if (rc) return rc;
    if ((rc = launch(c, s, ctx))) return rc;
  }
  return GPSIG_OK;
}

static int pde_fwd_launch_cb(PdeArgs a, hipStream_t s, void *) { return pde_launch_args(a, s); }

// gpsig_pde_gram through the increment tiles (any channel count, any dyadic order)
int pde_launch_tiled(const float *X, int n1, int l1, const float *Y, int n2, int l2, int d, int dyadic, int solver,
                     int pair_mode, int row_begin, int row_end, float *out, int out_row0, int out_rows,
                     long long out_ld, void *scratch, size_t scratch_bytes, hipStream_t s) {
  PdeArgs a{};
  a.X = X; a.Y = Y;
  a.n1 = n1; a.l1 = l1; a.n2 = n2; a.l2 = l2; a.d = d;
  a.dyadic = dyadic; a.solver = solver;
  a.pair_mode = pair_mode; a.row_begin = row_begin; a.row_end = row_end;
  a.out = out; a.out_row0 = out_row0; a.out_rows = out_rows; a.out_ld = out_ld;
  return pde_tiled_run(a, scratch, scratch_bytes, s, pde_fwd_launch_cb, nullptr);
}

// ------------------------------------------------------------------------------------ assembly
// dst[l][a][b] = row a's value at column b for b >= a, else row b's value at column a (the mirror).
// 32x32 tiles; the mirrored (lower) tiles go through LDS so both the read and the write are coalesced.
__global__ __launch_bounds__(256) void sym_assemble_kernel(const float *__restrict__ src,
                                                           const long long *__restrict__ row_off,
                                                           long long level_stride, int n, float *__restrict__ dst) {
  __shared__ float tile[32][33];
  const int lvl = blockIdx.z;
  const int bi = blockIdx.y, bj = blockIdx.x;  // dst tile rows bi*32.., cols bj*32..
  const float *S = src + (long long)lvl * level_stride;
  float *Dd = dst + (long long)lvl * n * n;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  if (bj >= bi) {
    for (int r = ty; r < 32; r += 8) {
      const int a = bi * 32 + r, b = bj * 32 + tx;
      if (a < n && b < n) Dd[(long long)a * n + b] = (b >= a) ? S[row_off[a] + b] : S[row_off[b] + a];
    }
  } else {
    // lower tile: dst[a][b] = row b's column a; read rows b (tile columns) coalesced along a
    for (int r = ty; r < 32; r += 8) {
      const int brow = bj * 32 + r, acol = bi * 32 + tx;
      tile[r][tx] = (brow < n && acol < n) ? S[row_off[brow] + acol] : 0.0f;
    }
    __syncthreads();
    for (int r = ty; r < 32; r += 8) {
      const int a = bi * 32 + r, b = bj * 32 + tx;
      if (a < n && b < n) Dd[(long long)a * n + b] = tile[tx][r];
    }
  }
}

int sym_assemble_launch(const float *src, const long long *row_off, long long level_stride, int n, int levels,
                        float *dst, hipStream_t s) {
  const int nt = (n + 31) / 32;
  hipLaunchKernelGGL(sym_assemble_kernel, dim3(nt, nt, levels), dim3(256), 0, s, src, row_off, level_stride, n, dst);
  return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
}

}  // namespace gpsig
