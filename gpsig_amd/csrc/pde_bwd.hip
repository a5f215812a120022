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
// Two passes, one wave per pair, the skewed-wavefront sweep of pde.hip (lane l owns W fine columns,
// row i = step - l), fp64 solution as the reference:
//   pass REV : K_rev on the reversed increments, every cell stored to the caller's scratch grid;
//   pass GRAD: K on the forward increments (the forward op's scheme), and at each cell
//              KK = K[i][c] * K_rev[I-1-i][J-1-c]; row partials go to the wave's LDS row accumulators
//              (ds_add_f64; lanes hold distinct fine rows at a step), column partials stay in registers.
#include "sig_common.h"

namespace gpsig {

struct PdeBwdArgs {
  const float *X, *Y;
  int n1, l1, n2, l2, d;
  int dyadic, solver;
  int pair_mode, row_begin, row_end;
  int ntb, tiles_a0;
  const float *gout;  // DIAG: (n1,); RECT: (n1, n2)
  float *gX, *gY;     // accumulated (n1, l1, d), (n2, l2, d)
  double *grid;       // scratch: per evaluated pair, the interior K_rev cells in wavefront-step order
                      // (pde_grid_cells: steps x lanes x W doubles)
};

template <int DP, int W, bool REV, bool COLS>
__global__ __launch_bounds__(256) void pde_bwd_kernel(PdeBwdArgs p) {
  extern __shared__ __attribute__((aligned(16))) double ldsd[];
  const int lane = threadIdx.x & 63;
  const int wave = wave_uniform(threadIdx.x >> 6);
  const bool diag = p.pair_mode == GPSIG_PAIRS_DIAG;
  int a, b;
  if (diag) {
    a = p.row_begin + (int)blockIdx.x * 4 + wave;
    b = a;
  } else {
    a = (p.tiles_a0 + (int)blockIdx.x / p.ntb) * 4 + wave;
    b = (int)blockIdx.x % p.ntb;
  }
  const bool ok = a >= p.row_begin && a < p.row_end && b < p.n2;  // wave-uniform
  if (!ok) { a = p.row_begin; b = diag ? a : 0; }

  const int n = p.dyadic, rep = 1 << n;
  const double inv_factor = 1.0 / (double)(1 << (2 * n));
  const int IC = p.l1 - 1, JC = p.l2 - 1;
  const int I = rep * IC, J = rep * JC;
  const int d = p.d;
  const float *x = p.X + (long long)a * p.l1 * d;
  const float *y = p.Y + (long long)b * p.l2 * d;
  const long long pidx = diag ? (long long)(a - p.row_begin) : (long long)(a - p.row_begin) * p.n2 + b;
  const int lanes_used = (J + W - 1) / W;
  // STEP (W < 8): K_rev cell (i, c) (interior, 0-based) was produced at wavefront step i + c / W by
  // lane c / W: stored at [(i + c/W) * lanes_used + c/W] * W + c % W, so each step's cells are one
  // contiguous block (coalesced stores) and the reversed read of the GRAD pass touches one or two
  // blocks per step.  W >= 8: the (I+1) x (J+1) row-major grid with its boundary row / column (each
  // lane's run is already 64 bytes, and it has no step padding).
  constexpr bool STEP = W < 8;
  double *grid = p.grid + pidx * (STEP ? (long long)(I + lanes_used - 1) * lanes_used * W : (long long)(I + 1) * (J + 1));

  // LDS: [wave] { dx (IC x DP floats, as doubles' storage) | row accumulators (IC x DP doubles) }
  double *wl = ldsd + (size_t)wave * IC * DP * 2;
  float *dxs = reinterpret_cast<float *>(wl);
  double *gacc = wl + (size_t)IC * DP;
  for (int r = lane; r < IC; r += 64) {
    const int rr = REV ? IC - 1 - r : r;  // reversed path: dx~_r = -dx_{IC-1-r} (the sign cancels in inc)
#pragma unroll
    for (int k = 0; k < DP; ++k) {
      dxs[r * DP + k] = k < d ? x[(rr + 1) * d + k] - x[rr * d + k] : 0.0f;
      gacc[r * DP + k] = 0.0;
    }
  }
  float dy[W][DP];
#pragma unroll
  for (int w = 0; w < W; ++w) {
    int cj = (lane * W + w) >> n;
    cj = cj < JC - 1 ? cj : JC - 1;
    if (REV) cj = JC - 1 - cj;
#pragma unroll
    for (int k = 0; k < DP; ++k) dy[w][k] = k < d ? y[(cj + 1) * d + k] - y[cj * d + k] : 0.0f;
  }
  if (REV && !STEP) {
    // boundaries of the stored grid
    for (int c = lane; c <= J; c += 64) grid[c] = 1.0;
    for (int r = lane; r <= I; r += 64) grid[(long long)r * (J + 1)] = 1.0;
  }
  __syncthreads();

  const int solver = REV ? 0 : p.solver;
  const bool hybrid = !REV && diag && p.solver == 0;
  double up[W];
  double gcol[W][DP];
#pragma unroll
  for (int w = 0; w < W; ++w) {
    up[w] = 1.0;
#pragma unroll
    for (int k = 0; k < DP; ++k) gcol[w][k] = 0.0;
  }
  double last = 1.0, left_prev = 1.0;
  const int nsteps = ok ? I + lanes_used - 1 : 0;  // invalid waves still reach the barrier below
  for (int s = 0; s < nsteps; ++s) {
    double left = lane_prev(last);
    if (lane == 0) left = 1.0;
    const double corner0 = left_prev;
    left_prev = left;
    const int i = s - lane;
    if (i >= 0 && i < I && lane < lanes_used) {
      const float *dxr = dxs + (i >> n) * DP;
      float dxv[DP];
#pragma unroll
      for (int k = 0; k < DP; ++k) dxv[k] = dxr[k];
      double lft = left, cor = corner0;
      double grow[DP];
#pragma unroll
      for (int k = 0; k < DP; ++k) grow[k] = 0.0;
      // K_rev[I-1-i][J-1-c] (grid indices, boundary row / column = 1) of the lane's columns, loaded
      // before the column loop: interior cell (I-2-i, J-2-c)
      double kr[W];
      if constexpr (!REV) {
        if constexpr (STEP) {
          const int ir = I - 2 - i;
#pragma unroll
          for (int w = 0; w < W; ++w) {
            const int c = lane * W + w;
            const int cr = J - 2 - c;
            double v = 1.0;
            if (ir >= 0 && cr >= 0) {
              const int lr = cr / W;
              v = grid[((long long)(ir + lr) * lanes_used + lr) * W + (cr - lr * W)];
            }
            kr[w] = c < J ? v : 0.0;
          }
        } else {
          const double *krr = grid + (long long)(I - 1 - i) * (J + 1) + (J - 1);
#pragma unroll
          for (int w = 0; w < W; ++w) {
            const int c = lane * W + w;
            kr[w] = c < J ? krr[-c] : 0.0;
          }
        }
      }
#pragma unroll
      for (int w = 0; w < W; ++w) {
        const int c = lane * W + w;
        float incf = 0.0f;
#pragma unroll
        for (int k = 0; k < DP; ++k) incf = __builtin_fmaf(dxv[k], dy[w][k], incf);
        const double inc = (double)incf * inv_factor;
        const double upw = up[w];
        double kn;
        if (solver == 1 || (hybrid && c == i)) {
          const double inc2 = inc * inc;
          kn = (upw + lft) * (1.0 + 0.5 * inc + (1.0 / 12) * inc2) - cor * (1.0 - (1.0 / 12) * inc2);
        } else {
          kn = (upw + lft) + cor * (inc - 1.0);
        }
        if (c < J) {
          if (REV) {
            if constexpr (STEP)
              grid[((long long)s * lanes_used + lane) * W + w] = kn;  // cell (i, c), step s = i + lane
            else
              grid[(long long)(i + 1) * (J + 1) + c + 1] = kn;
          } else {
            // KK[i][c] = K[i][c] * K_rev[I-1-i][J-1-c]
            const double kk = cor * kr[w];
#pragma unroll
            for (int k = 0; k < DP; ++k) {
              grow[k] = __builtin_fma(kk, (double)dy[w][k], grow[k]);
              if constexpr (COLS) gcol[w][k] = __builtin_fma(kk, (double)dxv[k], gcol[w][k]);
            }
          }
          cor = upw;
          lft = kn;
          up[w] = kn;
        }
      }
      last = lft;
      if (!REV) {
#pragma unroll
        for (int k = 0; k < DP; ++k)
          if (k < d) atomicAdd(gacc + (i >> n) * DP + k, grow[k]);
      }
    }
  }
  if (REV) return;
  __syncthreads();  // the row accumulators are complete
  if (!ok) return;

  // dK/dx_i = G[i-1] - G[i] with G[r] = 4^-n gacc[r] (x2 for k(x, x)), times the upstream gradient
  const float g = diag ? p.gout[a] : p.gout[(long long)a * p.n2 + b];
  const double sx = (diag ? 2.0 : 1.0) * inv_factor * (double)g;
  float *gxa = p.gX + (long long)a * p.l1 * d;
  for (int r = lane; r <= IC; r += 64)
    for (int k = 0; k < d; ++k) {
      const double gp = r > 0 ? gacc[(r - 1) * DP + k] : 0.0;
      const double gc = r < IC ? gacc[r * DP + k] : 0.0;
      unsafeAtomicAdd(gxa + (long long)r * d + k, (float)(sx * (gp - gc)));
    }
  if (diag || !COLS) return;
  // columns: H[j] = 4^-n sum over the fine columns of coarse column j; dK/dy_j = H[j-1] - H[j]
  const double sy = inv_factor * (double)g;
  float *gyb = p.gY + (long long)b * p.l2 * d;
#pragma unroll
  for (int w = 0; w < W; ++w) {
    const int c = lane * W + w;
    if (c >= J) continue;
    const int jc = c >> n;
    for (int k = 0; k < d; ++k) {
      const float v = (float)(sy * gcol[w][k]);
      unsafeAtomicAdd(gyb + (long long)(jc + 1) * d + k, v);
      unsafeAtomicAdd(gyb + (long long)jc * d + k, -v);
    }
  }
}

template <int DP, int W>
static int launch_pde_bwd(const PdeBwdArgs &a, long long nblocks, hipStream_t s) {
  if constexpr (W * DP > 128) {
    return GPSIG_EUNSUPPORTED;
  } else {
    const size_t lds = (size_t)4 * (a.l1 - 1) * DP * 2 * sizeof(double);
    if (lds > 160 * 1024) return GPSIG_EUNSUPPORTED;
    hipLaunchKernelGGL((pde_bwd_kernel<DP, W, true, false>), dim3((unsigned)nblocks), dim3(256), lds, s, a);
    // the column (dK/dy) accumulators only for cross pairs; k(x, x) takes twice the row part
    if (a.pair_mode == GPSIG_PAIRS_DIAG)
      hipLaunchKernelGGL((pde_bwd_kernel<DP, W, false, false>), dim3((unsigned)nblocks), dim3(256), lds, s, a);
    else
      hipLaunchKernelGGL((pde_bwd_kernel<DP, W, false, true>), dim3((unsigned)nblocks), dim3(256), lds, s, a);
    return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
  }
}

template <int DP>
static int pde_bwd_w(const PdeBwdArgs &a, long long nblocks, int J, hipStream_t s) {
  if (J <= 64) return launch_pde_bwd<DP, 1>(a, nblocks, s);
  if (J <= 128) return launch_pde_bwd<DP, 2>(a, nblocks, s);
  if (J <= 256) return launch_pde_bwd<DP, 4>(a, nblocks, s);
  if (J <= 512) return launch_pde_bwd<DP, 8>(a, nblocks, s);
  if (J <= 1024) return launch_pde_bwd<DP, 16>(a, nblocks, s);
  return GPSIG_EUNSUPPORTED;
}

}  // namespace gpsig

using namespace gpsig;

// K_rev cells of one pair (pde_bwd_kernel): W < 8 (W = the launch's columns per lane, pde_bwd_w) the
// wavefront-step order, (I + lanes - 1) steps x lanes x W with lanes = ceil(J / W); else the
// (I+1) x (J+1) grid.
static long long pde_grid_cells(int l1, int l2, int dyadic) {
  const long long I = (long long)(1 << dyadic) * (l1 - 1), J = (long long)(1 << dyadic) * (l2 - 1);
  const long long W = J <= 64 ? 1 : J <= 128 ? 2 : J <= 256 ? 4 : J <= 512 ? 8 : 16;
  if (W >= 8) return (I + 1) * (J + 1);
  const long long lanes = (J + W - 1) / W;
  return (I + lanes - 1) * lanes * W;
}

extern "C" size_t gpsig_pde_vjp_workspace_bytes(int npairs, int l1, int l2, int dyadic) {
  if (npairs <= 0 || l1 < 2 || l2 < 2 || dyadic < 0 || dyadic > 6) return 0;
  return (size_t)npairs * (size_t)pde_grid_cells(l1, l2, dyadic) * sizeof(double);
}

extern "C" int gpsig_pde_vjp(const float *X, int n1, int l1, const float *Y, int n2, int l2, int d, int dyadic,
                             int solver, int pair_mode, int row_begin, int row_end, const float *gout, float *gX,
                             float *gY, void *workspace, size_t workspace_bytes, gpsig_stream_t stream) {
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (!X || !Y || !gout || !gX || n1 <= 0 || n2 <= 0 || d <= 0 || l1 < 2 || l2 < 2) return GPSIG_EINVAL;
  if (dyadic < 0 || dyadic > 6 || (solver != 0 && solver != 1)) return GPSIG_EINVAL;
  if (pair_mode != GPSIG_PAIRS_RECT && pair_mode != GPSIG_PAIRS_DIAG) return GPSIG_EINVAL;
  if (row_begin < 0 || row_end > n1 || row_begin > row_end) return GPSIG_EINVAL;
  if (pair_mode == GPSIG_PAIRS_DIAG && (n1 != n2 || l1 != l2 || X != Y)) return GPSIG_EINVAL;
  if (pair_mode == GPSIG_PAIRS_RECT && !gY) return GPSIG_EINVAL;
  if (row_end == row_begin) return GPSIG_OK;
  const int rows = row_end - row_begin;
  const int npairs = pair_mode == GPSIG_PAIRS_DIAG ? rows : rows * n2;
  if (!workspace || workspace_bytes < gpsig_pde_vjp_workspace_bytes(npairs, l1, l2, dyadic)) return GPSIG_EWORKSPACE;
  PdeBwdArgs a{};
  a.X = X; a.Y = Y;
  a.n1 = n1; a.l1 = l1; a.n2 = n2; a.l2 = l2; a.d = d;
  a.dyadic = dyadic; a.solver = solver;
  a.pair_mode = pair_mode; a.row_begin = row_begin; a.row_end = row_end;
  a.gout = gout; a.gX = gX; a.gY = gY;
  a.grid = static_cast<double *>(workspace);
  long long nblocks;
  if (pair_mode == GPSIG_PAIRS_DIAG) {
    nblocks = (rows + 3) / 4;
  } else {
    const int ta0 = row_begin / 4, ta1 = (row_end + 3) / 4;
    a.ntb = n2;
    a.tiles_a0 = ta0;
    nblocks = (long long)(ta1 - ta0) * n2;
  }
  if (nblocks > 0x7fffffffLL) return GPSIG_EUNSUPPORTED;
  const int J = (1 << dyadic) * (l2 - 1);
  switch (d <= 8 ? d : (d <= 16 ? 16 : 0)) {
#define CASE(v) \
  case v: return pde_bwd_w<v>(a, nblocks, J, s);
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8) CASE(16)
#undef CASE
    default: return GPSIG_EUNSUPPORTED;
  }
}
