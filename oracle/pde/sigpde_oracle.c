/*
 * CPU oracle: C restatement of the Goursat-PDE signature-kernel solver.
 *
 * TEST INFRASTRUCTURE ONLY -- used by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py as the checker / CPU baseline; never linked
 * into or called by gpsig_amd/.
 *
 * Restates (file:line relative to /root/reference):
 *   gpsig/sigKer_fast.pyx:15-62   sig_kern_diag(x, n, solver) -> (K, K_rev)
 *     - grid (2^n (L-1) + 1)^2, boundary K[i][0] = 1            (:29-31)
 *     - increment = sum_k dx_{ii,k} * dx_{jj,k} / 4^n, ii = i>>n (:35-43)
 *     - solver 0: K[i+1][j+1] = K[i][j+1] + K[i+1][j] + K[i][j]*(inc-1)        (:46)
 *     - solver 1: (K[i][j+1]+K[i+1][j])*(1+inc/2+inc^2/12) - K[i][j]*(1-inc^2/12) (:48)
 *     - K_rev: solver-0 scheme on the time-reversed increments            (:43,50,61)
 *   gpsig/covariance_op/untrunc_cov_op_gpu.cu:29 (same explicit scheme as solver 1)
 *
 * Generalisation (documented in DESIGN.md): the reference only solves x == y
 * (lower triangle + diagonal by symmetry).  sigpde_pair() solves the full
 * (2^n(L1-1)+1) x (2^n(L2-1)+1) grid for x != y with K[0][j] = K[i][0] = 1;
 * for x == y it is bitwise the reference's lower triangle (the update is
 * symmetric in its two neighbours and the increment products commute).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

static double incr_at(const double *x, int lx, const double *y, int ly, int d,
                      int ii, int jj, double factor, int reverse) {
  double inc = 0.0;
  for (int k = 0; k < d; ++k) {
    double dx, dy;
    if (!reverse) {
      dx = x[(ii + 1) * d + k] - x[ii * d + k];
      dy = y[(jj + 1) * d + k] - y[jj * d + k];
    } else { /* sigKer_fast.pyx:43 */
      dx = x[((lx - 1) - (ii + 1)) * d + k] - x[((lx - 1) - ii) * d + k];
      dy = y[((ly - 1) - (jj + 1)) * d + k] - y[((ly - 1) - jj) * d + k];
    }
    inc = inc + dx * dy / factor;
  }
  return inc;
}

/* Solve one pair.  grid (optional): (I+1)*(J+1) doubles, row-major.  Returns K[I][J]. */
double sigpde_pair(const double *x, int lx, const double *y, int ly, int d, int n, int solver,
                   int reverse, int hybrid_diag, double *grid) {
  const int rep = 1 << n;
  const double factor = (double)(1 << (2 * n));
  const int I = rep * (lx - 1), J = rep * (ly - 1);
  double *prev = (double *)malloc(sizeof(double) * (J + 1));
  double *cur = (double *)malloc(sizeof(double) * (J + 1));
  for (int j = 0; j <= J; ++j) prev[j] = 1.0;
  if (grid) for (int j = 0; j <= J; ++j) grid[j] = 1.0;
  for (int i = 0; i < I; ++i) {
    cur[0] = 1.0;
    const int ii = i / rep;
    for (int j = 0; j < J; ++j) {
      const int jj = j / rep;
      const double inc = incr_at(x, lx, y, ly, d, ii, jj, factor, reverse);
      /* sigKer_fast.pyx:59 applies the solver-1 update on the diagonal even when solver == 0
       * (K only; K_rev at :61 stays solver 0).  hybrid_diag reproduces that for x == y. */
      if (solver == 0 && !(hybrid_diag && i == j))
        cur[j + 1] = (prev[j + 1] + cur[j]) + prev[j] * (inc - 1.);
      else
        cur[j + 1] = (prev[j + 1] + cur[j]) * (1. + 0.5 * inc + (1. / 12) * (inc * inc)) -
                     prev[j] * (1. - (1. / 12) * (inc * inc));
    }
    if (grid) memcpy(grid + (size_t)(i + 1) * (J + 1), cur, sizeof(double) * (J + 1));
    double *t = prev; prev = cur; cur = t;
  }
  const double r = prev[J];
  free(prev);
  free(cur);
  return r;
}

/* Gram of final corners.  X (n1,l1,d), Y (n2,l2,d).  symmetric: Y==X, fill both triangles. */
void sigpde_gram(const double *X, int n1, int l1, const double *Y, int n2, int l2, int d, int n,
                 int solver, int symmetric, double *out) {
#pragma omp parallel for schedule(dynamic, 1)
  for (long t = 0; t < (long)n1 * n2; ++t) {
    const int a = (int)(t / n2), b = (int)(t % n2);
    if (symmetric && b < a) continue;
    const double v = sigpde_pair(X + (size_t)a * l1 * d, l1, Y + (size_t)b * l2 * d, l2, d, n, solver, 0, 0, NULL);
    out[(size_t)a * n2 + b] = v;
    if (symmetric) out[(size_t)b * n2 + a] = v;
  }
}

/* Diagonal k(x_a, x_a) for a in [0, A). */
void sigpde_diag(const double *X, int A, int L, int d, int n, int solver, double *out) {
#pragma omp parallel for schedule(dynamic, 1)
  for (int a = 0; a < A; ++a) {
    const double *x = X + (size_t)a * L * d;
    out[a] = sigpde_pair(x, L, x, L, d, n, solver, 0, 1, NULL);
  }
}

/* Full grids as sig_kern_diag returns them: K (solver as given) and K_rev (solver 0, reversed). */
void sigpde_diag_grids(const double *X, int A, int L, int d, int n, int solver, double *K, double *Krev) {
  const int G = (1 << n) * (L - 1) + 1;
#pragma omp parallel for schedule(dynamic, 1)
  for (int a = 0; a < A; ++a) {
    const double *x = X + (size_t)a * L * d;
    sigpde_pair(x, L, x, L, d, n, solver, 0, 1, K + (size_t)a * G * G);
    sigpde_pair(x, L, x, L, d, n, 0, 1, 0, Krev + (size_t)a * G * G);
  }
}

/* The reference's adjoint (kernels_pde.py:465-509 restated in oracle/pde_grad.py pair_grad) for one cross
 * pair: KK[i][j] = K[i][j] K_rev[I-1-i][J-1-j] (K_rev: solver 0 on the reversed paths), coarse-row / column
 * sums contracted with the other path's increments, / 4^n; gx[p] = Gx[p-1] - Gx[p], gy likewise. */
void sigpde_pair_grad(const double *x, int lx, const double *y, int ly, int d, int n, int solver, double *gx,
                      double *gy) {
  const int rep = 1 << n;
  const int I = rep * (lx - 1), J = rep * (ly - 1);
  double *K = (double *)malloc(sizeof(double) * (size_t)(I + 1) * (J + 1));
  double *Kr = (double *)malloc(sizeof(double) * (size_t)(I + 1) * (J + 1));
  double *Gx = (double *)calloc((size_t)(lx - 1) * d, sizeof(double));
  double *Gy = (double *)calloc((size_t)(ly - 1) * d, sizeof(double));
  sigpde_pair(x, lx, y, ly, d, n, solver, 0, 0, K);
  sigpde_pair(x, lx, y, ly, d, n, 0, 1, 0, Kr);
  for (int i = 0; i < I; ++i)
    for (int j = 0; j < J; ++j) {
      const double kk = K[(size_t)i * (J + 1) + j] * Kr[(size_t)(I - 1 - i) * (J + 1) + (J - 1 - j)];
      const int ii = i >> n, jj = j >> n;
      for (int k = 0; k < d; ++k) {
        Gx[(size_t)ii * d + k] += kk * (y[(jj + 1) * d + k] - y[jj * d + k]);
        Gy[(size_t)jj * d + k] += kk * (x[(ii + 1) * d + k] - x[ii * d + k]);
      }
    }
  const double f = 1.0 / (double)(1 << (2 * n));
  for (int p = 0; p < lx; ++p)
    for (int k = 0; k < d; ++k)
      gx[(size_t)p * d + k] = f * ((p > 0 ? Gx[(size_t)(p - 1) * d + k] : 0.0) - (p < lx - 1 ? Gx[(size_t)p * d + k] : 0.0));
  for (int p = 0; p < ly; ++p)
    for (int k = 0; k < d; ++k)
      gy[(size_t)p * d + k] = f * ((p > 0 ? Gy[(size_t)(p - 1) * d + k] : 0.0) - (p < ly - 1 ? Gy[(size_t)p * d + k] : 0.0));
  free(K);
  free(Kr);
  free(Gx);
  free(Gy);
}

/* sum over pairs of w[a][b] * (dK(x_a, y_b)/dX, dK/dY), pairs in parallel (per-pair buffers, summed in order) */
void sigpde_gram_grad(const double *X, int n1, int l1, const double *Y, int n2, int l2, int d, int n, int solver,
                      const double *w, double *gX, double *gY) {
  double *px = (double *)calloc((size_t)n1 * n2 * l1 * d, sizeof(double));
  double *py = (double *)calloc((size_t)n1 * n2 * l2 * d, sizeof(double));
#pragma omp parallel for schedule(dynamic, 1)
  for (long t = 0; t < (long)n1 * n2; ++t) {
    const int a = (int)(t / n2), b = (int)(t % n2);
    sigpde_pair_grad(X + (size_t)a * l1 * d, l1, Y + (size_t)b * l2 * d, l2, d, n, solver, px + (size_t)t * l1 * d,
                     py + (size_t)t * l2 * d);
  }
  for (long t = 0; t < (long)n1 * n2; ++t) {
    const int a = (int)(t / n2), b = (int)(t % n2);
    for (long e = 0; e < (long)l1 * d; ++e) gX[(size_t)a * l1 * d + e] += w[t] * px[(size_t)t * l1 * d + e];
    for (long e = 0; e < (long)l2 * d; ++e) gY[(size_t)b * l2 * d + e] += w[t] * py[(size_t)t * l2 * d + e];
  }
  free(px);
  free(py);
}
