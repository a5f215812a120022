// gpsig_amd -- the inducing-tensor vs sequence VJP at wide channel counts (runtime channel loop).
//
// The recursion and its adjoint are those of sig_tvs_bwd.h (forward end state from the forward launch or a
// sweep, inverted reverse sweep, adjoint running sums Q_j, dLoss/dP_k at the points).  The fixed-channel
// kernel contracts every point weight with z (for the sequence gradient) and x (for the tensor gradient)
// in registers; here the kernel writes the point weights of a chunk of sequences
//     W0[(k, t)][(s, n)] = dLoss/dP_k(s) * k(z0_k, x_s)    (RBF; increments: -..., and W1 with k(z1_k, x_s))
//                          dLoss/dP_k(s)                   (linear)
// and two GEMMs on the matrix cores (gemm.hip) contract them -- the transposes of the reference's
// tensor-vs-point base-kernel products (kernels.py:314-341 over kernels.py:946-957):
//     [gX | rowsum] (s, n) += W0^T [Z0 | 1] + W1^T [Z1 | 1],    [gZ0 | colsum] += W0 [X | 1]
// then gX -= rowsum x, gZ0 -= colsum z0 (RBF).  Linear: gX += W^T Zw (w = z, or z1 - z0), gZ = W X
// (increments: gZ1 += W X, gZ0 -= W X).
#include "sig_common.h"
#include "gemm.h"

namespace gpsig {

size_t tvs_features_bytes(int n, int l, int d);
int tvs_features_launch(const float *X, int n, int l, int d, float *Ft, hipStream_t s);

struct TvsBwdWideArgs {
  const float *Zw;   // (T, [2,] d, LT) + (T, LT) |dz|^2/2: tvs_wide_prep_kernel layout
  const float *Ft;   // time-major features of all n sequences
  int t, n, l, d, lt;
  const float *gout;   // (M+1, T, n)
  const float *state;  // optional (T, n, LT)
  int n0, nc;          // this launch's sequences [n0, n0 + nc)
  float *W0, *W1;      // point weights [(k T + t)][(s nc + n - n0)]
};

__host__ __device__ inline long long tvsw_zs(int d, int lt, bool incr) { return (long long)(incr ? 2 * d + 1 : d) * lt; }

// Zw[tt][h][q][k] (h = 0: z0 or z, h = 1: dz), then Zw[tt][2d][k] = |dz_k|^2/2 (same as sig_tvs_pk.hip)
__global__ __launch_bounds__(256) void tvsw_prep_kernel(const float *__restrict__ Z, int lt, int t, int d, int incr,
                                                        float *__restrict__ Zw) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long long)lt * t) return;
  const int k = (int)(idx % lt), tt = (int)(idx / lt);
  float *o = Zw + (long long)tt * tvsw_zs(d, lt, incr != 0);
  if (!incr) {
    const float *z = Z + ((long long)k * t + tt) * d;
    for (int q = 0; q < d; ++q) o[(long long)q * lt + k] = z[q];
  } else {
    const float *z = Z + (((long long)k * t + tt) * 2) * d;
    float h = 0.f;
    for (int q = 0; q < d; ++q) {
      const float dz = z[d + q] - z[q];
      o[(long long)q * lt + k] = z[q];
      o[((long long)d + q) * lt + k] = dz;
      h = __builtin_fmaf(dz, dz, h);
    }
    o[(long long)2 * d * lt + k] = 0.5f * h;
  }
}

template <int I, int MMAX, bool INCR, bool RBF, bool DIFF>
__device__ __forceinline__ void tvsw_level(const TvsBwdWideArgs &a) {
  constexpr int KB = I * (I - 1) / 2;
  constexpr int LTM = MMAX * (MMAX + 1) / 2;
  constexpr float NHL2E = -0.72134752044448170f, L2E = 1.4426950408889634f;
  const int lane = threadIdx.x;
  const int tt = blockIdx.y;
  const int n = a.n, d = a.d, FC = 2 * d + 3, T = a.t, L = a.l, LT = a.lt;
  const int sl = blockIdx.x * 64 + lane;  // sequence within the launch's chunk
  const bool valid = sl < a.nc;
  const int sq = a.n0 + (valid ? sl : a.nc - 1);
  cfloat *z0 = as_const(a.Zw) + (long long)tt * tvsw_zs(d, LT, INCR) + KB;  // channel q, component c: z0[q LT + c]
  cfloat *dz = z0 + (long long)d * LT;
  cfloat *hdz = z0 + (long long)2 * d * LT;
  auto ft = [&](int s, int c) { return a.Ft[((long long)s * FC + c) * n + sq]; };
  auto em1 = [](float v) { return __builtin_fabsf(v) < EM1_TAU ? em1_small(v) : __builtin_amdgcn_exp2f(v * L2E) - 1.0f; };

  // point values of the level's components at x_s: RBF k(z0, x_s) [and k(z1, x_s)]; linear <w, x_s>
  auto pvals = [&](int s, float (&v0)[I], float (&v1)[I]) {
    float e0[I], e1[I];
#pragma unroll
    for (int c = 0; c < I; ++c) e0[c] = e1[c] = 0.f;
    for (int q = 0; q < d; ++q) {
      const float xv = ft(s, q);
#pragma unroll
      for (int c = 0; c < I; ++c) {
        if constexpr (RBF) {
          const float d0 = z0[(long long)q * LT + c] - xv;
          e0[c] = __builtin_fmaf(d0, d0, e0[c]);
          if constexpr (INCR) {
            const float d1 = d0 + dz[(long long)q * LT + c];
            e1[c] = __builtin_fmaf(d1, d1, e1[c]);
          }
        } else {
          e0[c] = __builtin_fmaf(INCR ? dz[(long long)q * LT + c] : z0[(long long)q * LT + c], xv, e0[c]);
        }
      }
    }
#pragma unroll
    for (int c = 0; c < I; ++c) {
      if constexpr (RBF) {
        v0[c] = __builtin_amdgcn_exp2f(e0[c] * NHL2E);
        v1[c] = INCR ? __builtin_amdgcn_exp2f(e1[c] * NHL2E) : 0.f;
      } else {
        v0[c] = e0[c];  // the linear point value itself
        v1[c] = 0.f;
      }
    }
  };
  // cells M_c(s) of the level (difference): from x_s, dx_s, g_s and the point values at s (c0, c1) and
  // s + 1 (n0, n1), as sig_tvs_bwd.h cell()
  auto cells = [&](int s, const float (&c0)[I], const float (&c1)[I], const float (&n0)[I], const float (&n1)[I],
                   float (&m)[I]) {
    if constexpr (!RBF) {
      float v[I];
#pragma unroll
      for (int c = 0; c < I; ++c) v[c] = 0.f;
      for (int q = 0; q < d; ++q) {
        const float dxv = ft(s, d + q);
#pragma unroll
        for (int c = 0; c < I; ++c)
          v[c] = __builtin_fmaf(INCR ? dz[(long long)q * LT + c] : z0[(long long)q * LT + c], dxv, v[c]);
      }
#pragma unroll
      for (int c = 0; c < I; ++c) m[c] = v[c];
    } else {
      const float gs = ft(s, 2 * d + 1);
      float qv[I], pv[I], cv[I];
#pragma unroll
      for (int c = 0; c < I; ++c) {
        qv[c] = -gs;
        pv[c] = cv[c] = 0.f;
      }
      for (int q = 0; q < d; ++q) {
        const float dxv = ft(s, d + q);
        const float xv = INCR ? ft(s, q) : 0.f;
#pragma unroll
        for (int c = 0; c < I; ++c) {
          const float zq = z0[(long long)q * LT + c];
          qv[c] = __builtin_fmaf(zq, dxv, qv[c]);
          if constexpr (INCR) {
            const float dzq = dz[(long long)q * LT + c];
            pv[c] = __builtin_fmaf(xv - zq, dzq, pv[c]);
            cv[c] = __builtin_fmaf(dzq, dxv, cv[c]);
          }
        }
      }
#pragma unroll
      for (int c = 0; c < I; ++c) {
        if constexpr (!INCR) {
          m[c] = c0[c] * em1(qv[c]);  // k(z, x_{s+1}) - k(z, x_s), any q
        } else {
          const float p = pv[c] - hdz[c];
          const float mx = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(p), __builtin_fabsf(qv[c])), __builtin_fabsf(cv[c]));
          if (mx < EM1_TAU) {
            const float Ep = em1_small(p), Eq = em1_small(qv[c]), Ec = em1_small(cv[c]);
            m[c] = c0[c] * __builtin_fmaf(Ep, Eq, (1.0f + Ep) * (1.0f + Eq) * Ec);
          } else {
            m[c] = (n1[c] - n0[c]) - (c1[c] - c0[c]);
          }
        }
      }
    }
  };
  // point values as cells (difference=False): RBF k(z0, x) [k(z1, x) - k(z0, x)], linear <w, x>
  auto pcells = [&](const float (&v0)[I], const float (&v1)[I], float (&m)[I]) {
#pragma unroll
    for (int c = 0; c < I; ++c) m[c] = RBF ? (INCR ? v1[c] - v0[c] : v0[c]) : v0[c];
  };

  const float gI = valid ? a.gout[((long long)I * T + tt) * n + sq] : 0.f;
  float A[I];
#pragma unroll
  for (int c = 0; c < I; ++c) A[c] = 0.f;
  float pv0[I], pv1[I];
  const int nsteps = DIFF ? L - 1 : L;
  if (a.state) {
    const float *st = a.state + ((long long)tt * n + sq) * LTM + KB;
#pragma unroll
    for (int c = 0; c + 1 < I; ++c) A[c] = st[c];
  } else {
    if constexpr (DIFF) pvals(0, pv0, pv1);
    for (int s = 0; s < nsteps; ++s) {
      float m[I];
      if constexpr (DIFF) {
        float nv0[I], nv1[I];
        pvals(s + 1, nv0, nv1);
        cells(s, pv0, pv1, nv0, nv1, m);
#pragma unroll
        for (int c = 0; c < I; ++c) {
          pv0[c] = nv0[c];
          pv1[c] = nv1[c];
        }
      } else {
        float v0[I], v1[I];
        pvals(s, v0, v1);
        pcells(v0, v1, m);
      }
      float prev = m[0];
#pragma unroll
      for (int c = 1; c < I; ++c) {
        const float as = A[c - 1];
        A[c - 1] = as + prev;
        prev = m[c] * as;
      }
    }
  }

  // reverse sweep
  float Acc[I], Mh[I];
#pragma unroll
  for (int c = 0; c < I; ++c) Acc[c] = Mh[c] = 0.f;
  const long long wld = (long long)L * a.nc;  // row length of the weight tiles
  auto emit = [&](int sp, const float (&Ph)[I], const float (&v0)[I], const float (&v1)[I]) {
    if (!valid) return;
#pragma unroll
    for (int c = 0; c < I; ++c) {
      const long long o = ((long long)(KB + c) * T + tt) * wld + (long long)sp * a.nc + sl;
      if constexpr (RBF) {
        a.W0[o] = INCR ? -Ph[c] * v0[c] : Ph[c] * v0[c];
        if constexpr (INCR) a.W1[o] = Ph[c] * v1[c];
      } else {
        a.W0[o] = Ph[c];
      }
    }
  };
  const int stop = nsteps - 1;
  if constexpr (DIFF) pvals(stop + 1, pv0, pv1);  // point values at the last point
  for (int s = stop; s >= 0; --s) {
    float c0v[I], c1v[I], m[I], Ph[I], Av[I];
    pvals(s, c0v, c1v);
    if constexpr (DIFF)
      cells(s, c0v, c1v, pv0, pv1, m);
    else
      pcells(c0v, c1v, m);
    Av[0] = 1.0f;
#pragma unroll
    for (int j = 1; j < I; ++j) {
      A[j - 1] = __builtin_fmaf(-m[j - 1], Av[j - 1], A[j - 1]);
      Av[j] = A[j - 1];
    }
#pragma unroll
    for (int j = 1; j <= I; ++j) {
      const float Q = (j < I) ? Acc[j - 1] : gI;
      const float mh = Q * Av[j - 1];
      Ph[j - 1] = DIFF ? mh - Mh[j - 1] : mh;
      Mh[j - 1] = mh;
    }
#pragma unroll
    for (int j = 1; j < I; ++j) {
      const float Qn = (j + 1 < I) ? Acc[j] : gI;
      Acc[j - 1] = __builtin_fmaf(m[j], Qn, Acc[j - 1]);
    }
    if constexpr (DIFF)
      emit(s + 1, Ph, pv0, pv1);
    else
      emit(s, Ph, c0v, c1v);
#pragma unroll
    for (int c = 0; c < I; ++c) {
      pv0[c] = c0v[c];
      pv1[c] = c1v[c];
    }
  }
  if constexpr (DIFF) {
    float Ph[I];
#pragma unroll
    for (int c = 0; c < I; ++c) Ph[c] = -Mh[c];
    emit(0, Ph, pv0, pv1);
  }
}

template <int M, bool INCR, bool RBF, bool DIFF>
__global__ __launch_bounds__(64) void tvs_bwd_wide_kernel(TvsBwdWideArgs a) {
  switch (blockIdx.z) {
    case 0: tvsw_level<1, M, INCR, RBF, DIFF>(a); break;
    case 1: if constexpr (M >= 2) tvsw_level<2, M, INCR, RBF, DIFF>(a); break;
    case 2: if constexpr (M >= 3) tvsw_level<3, M, INCR, RBF, DIFF>(a); break;
    case 3: if constexpr (M >= 4) tvsw_level<4, M, INCR, RBF, DIFF>(a); break;
    case 4: if constexpr (M >= 5) tvsw_level<5, M, INCR, RBF, DIFF>(a); break;
    case 5: if constexpr (M >= 6) tvsw_level<6, M, INCR, RBF, DIFF>(a); break;
    case 6: if constexpr (M >= 7) tvsw_level<7, M, INCR, RBF, DIFF>(a); break;
    case 7: if constexpr (M >= 8) tvsw_level<8, M, INCR, RBF, DIFF>(a); break;
    default: break;
  }
}

// Xc[(s nc + j)][q] = x_{n0 + j, s, q} (q < d), 1 (q = d): the chunk's points, time-major, augmented
__global__ __launch_bounds__(256) void tvsw_points_kernel(const float *__restrict__ X, int l, int d, int n0, int nc,
                                                          float *__restrict__ Xc) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long long)l * nc * (d + 1)) return;
  const int q = (int)(idx % (d + 1));
  const long long r = idx / (d + 1);
  const int j = (int)(r % nc), s = (int)(r / nc);
  Xc[idx] = q < d ? X[(((long long)(n0 + j)) * l + s) * d + q] : 1.0f;
}

// Za[(k T + t)][q] = z_h (q < d; h = 0: z0 / z, h = 1: z1, h = 2: z1 - z0), 1 (q = d)
__global__ __launch_bounds__(256) void tvsw_zaug_kernel(const float *__restrict__ Z, int lt, int t, int d, int incr,
                                                        int h, float *__restrict__ Za) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long long)lt * t * (d + 1)) return;
  const int q = (int)(idx % (d + 1));
  const long long r = idx / (d + 1);
  if (q == d) {
    Za[idx] = 1.0f;
    return;
  }
  const float *z = Z + r * (incr ? 2 * d : d);
  Za[idx] = !incr ? z[q] : (h == 0 ? z[q] : h == 1 ? z[d + q] : z[d + q] - z[q]);
}

// gX[n0 + j][s][q] += G[(s nc + j)][q] - rbf * G[..][d] x  (G from the chunk's sequence-side GEMM)
__global__ __launch_bounds__(256) void tvsw_gx_kernel(const float *__restrict__ G, const float *__restrict__ X, int l,
                                                      int d, int n0, int nc, int rbf, float *__restrict__ gX) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long long)l * nc * d) return;
  const int q = (int)(idx % d);
  const long long r = idx / d;
  const int j = (int)(r % nc), s = (int)(r / nc);
  const float *Gr = G + r * (d + 1);
  const long long o = (((long long)(n0 + j)) * l + s) * d + q;
  gX[o] += rbf ? __builtin_fmaf(-Gr[d], X[o], Gr[q]) : Gr[q];
}

// gZ[k][t][h][q] += sgn (G[(k T + t)][q] - rbf * G[..][d] z_h)
__global__ __launch_bounds__(256) void tvsw_gz_kernel(const float *__restrict__ G, const float *__restrict__ Z, int lt,
                                                      int t, int d, int incr, int h, float sgn, int rbf,
                                                      float *__restrict__ gZ) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long long)lt * t * d) return;
  const int q = (int)(idx % d);
  const long long r = idx / d;
  const float *Gr = G + r * (d + 1);
  const long long o = r * (incr ? 2 * d : d) + (long long)h * d + q;
  gZ[o] += sgn * (rbf ? __builtin_fmaf(-Gr[d], Z[o], Gr[q]) : Gr[q]);
}

static size_t a256(size_t b) { return (b + 255) & ~(size_t)255; }
constexpr size_t TVSW_TILE_BYTES = (size_t)1 << 30;

struct TvswPlan {
  int nc;
  size_t ft, zw, za0, za1, xc, gxc, gz, w0, w1, part;
};
static TvswPlan tvsw_plan(int n, int l, int d, int lt, int t, bool incr) {
  TvswPlan p{};
  long long nc = (long long)(TVSW_TILE_BYTES / ((size_t)lt * t * l * sizeof(float)));
  nc = nc < 64 ? 64 : (nc / 64) * 64;
  if (nc > ((n + 63) / 64) * 64) nc = ((n + 63) / 64) * 64;
  p.nc = (int)nc;
  p.ft = a256(tvs_features_bytes(n, l, d));
  p.zw = a256((size_t)t * tvsw_zs(d, lt, true) * sizeof(float));
  p.za0 = a256((size_t)lt * t * (d + 1) * sizeof(float));
  p.za1 = incr ? p.za0 : 0;
  p.xc = a256((size_t)l * nc * (d + 1) * sizeof(float));
  p.gxc = p.xc;
  p.gz = a256((size_t)lt * t * (d + 1) * sizeof(float) * (incr ? 2 : 1));
  p.w0 = a256((size_t)lt * t * l * nc * sizeof(float));
  p.w1 = incr ? p.w0 : 0;
  const size_t pa = gemm_splitk_bytes((int)(l * nc), d + 1, lt * t);
  const size_t pb = gemm_splitk_bytes(lt * t, d + 1, (int)(l * nc));
  // gemm_f32 clamps the split of every chunk (the last, shorter one included) to this capacity
  p.part = a256(pa > pb ? pa : pb);
  return p;
}
static size_t tvsw_bytes(const TvswPlan &p) { return p.ft + p.zw + p.za0 + p.za1 + p.xc + p.gxc + p.gz + p.w0 + p.w1 + p.part; }

size_t tvs_bwd_wide_workspace(int n, int l, int d, int lt, int t) { return tvsw_bytes(tvsw_plan(n, l, d, lt, t, true)); }

template <int M>
static int launch_tvsw(const TvsBwdWideArgs &a, bool incr, bool rbf, bool diff, hipStream_t s) {
  dim3 grid((unsigned)((a.nc + 63) / 64), (unsigned)a.t, (unsigned)M);
#define GPSIG_TVSW(i, r, df)                                                                          \
  if (incr == i && rbf == r && diff == df) {                                                          \
    hipLaunchKernelGGL((tvs_bwd_wide_kernel<M, i, r, df>), grid, dim3(64), 0, s, a);                  \
    return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;                                \
  }
  GPSIG_TVSW(false, true, true) GPSIG_TVSW(true, true, true) GPSIG_TVSW(false, false, true) GPSIG_TVSW(true, false, true)
  GPSIG_TVSW(false, true, false) GPSIG_TVSW(true, true, false) GPSIG_TVSW(false, false, false) GPSIG_TVSW(true, false, false)
#undef GPSIG_TVSW
  return GPSIG_EUNSUPPORTED;
}

int tvs_bwd_wide(const float *Z, int lt, int t, int incr, int d, const float *X, int n, int l, int M, bool rbf,
                 bool diff, const float *gout, float *gZ, float *gX, const float *state, void *workspace,
                 size_t workspace_bytes, hipStream_t s) {
  if (M < 1 || M > 8 || t > 65535) return GPSIG_EUNSUPPORTED;
  const TvswPlan pl = tvsw_plan(n, l, d, lt, t, incr != 0);
  if (!workspace || workspace_bytes < tvsw_bytes(pl)) return GPSIG_EWORKSPACE;
  char *w = static_cast<char *>(workspace);
  float *Ft = reinterpret_cast<float *>(w); w += pl.ft;
  float *Zw = reinterpret_cast<float *>(w); w += pl.zw;
  float *Za0 = reinterpret_cast<float *>(w); w += pl.za0;
  float *Za1 = pl.za1 ? reinterpret_cast<float *>(w) : nullptr; w += pl.za1;
  float *Xc = reinterpret_cast<float *>(w); w += pl.xc;
  float *Gxc = reinterpret_cast<float *>(w); w += pl.gxc;
  float *Gz = reinterpret_cast<float *>(w); w += pl.gz;
  float *W0 = reinterpret_cast<float *>(w); w += pl.w0;
  float *W1 = pl.w1 ? reinterpret_cast<float *>(w) : nullptr; w += pl.w1;
  float *part = pl.part ? reinterpret_cast<float *>(w) : nullptr;
  int rc = tvs_features_launch(X, n, l, d, Ft, s);
  if (rc) return rc;
  const long long zr = (long long)lt * t;
  hipLaunchKernelGGL(tvsw_prep_kernel, dim3((unsigned)((zr + 255) / 256)), dim3(256), 0, s, Z, lt, t, d, incr, Zw);
  // sequence side: [Z0 | 1] and [Z1 | 1] (RBF), or the linear seed's w = z / z1 - z0
  const int h0 = (!rbf && incr) ? 2 : 0;
  hipLaunchKernelGGL(tvsw_zaug_kernel, dim3((unsigned)((zr * (d + 1) + 255) / 256)), dim3(256), 0, s, Z, lt, t, d, incr,
                     h0, Za0);
  if (rbf && incr)
    hipLaunchKernelGGL(tvsw_zaug_kernel, dim3((unsigned)((zr * (d + 1) + 255) / 256)), dim3(256), 0, s, Z, lt, t, d,
                       incr, 1, Za1);
  float *Gz0 = Gz, *Gz1 = (rbf && incr) ? Gz + zr * (d + 1) : nullptr;
  if (hipMemsetAsync(Gz, 0, (size_t)zr * (d + 1) * sizeof(float) * (Gz1 ? 2 : 1), s) != hipSuccess) return GPSIG_ELAUNCH;
  const int D1 = d + 1;
  for (int n0 = 0; n0 < n; n0 += pl.nc) {
    const int nc = n - n0 < pl.nc ? n - n0 : pl.nc;
    TvsBwdWideArgs a{Zw, Ft, t, n, l, d, lt, gout, state, n0, nc, W0, W1 ? W1 : W0};
    switch (M) {
      case 1: rc = launch_tvsw<1>(a, incr, rbf, diff, s); break;
      case 2: rc = launch_tvsw<2>(a, incr, rbf, diff, s); break;
      case 3: rc = launch_tvsw<3>(a, incr, rbf, diff, s); break;
      case 4: rc = launch_tvsw<4>(a, incr, rbf, diff, s); break;
      case 5: rc = launch_tvsw<5>(a, incr, rbf, diff, s); break;
      case 6: rc = launch_tvsw<6>(a, incr, rbf, diff, s); break;
      case 7: rc = launch_tvsw<7>(a, incr, rbf, diff, s); break;
      case 8: rc = launch_tvsw<8>(a, incr, rbf, diff, s); break;
      default: return GPSIG_EUNSUPPORTED;
    }
    if (rc) return rc;
    const int R = l * nc;
    // sequence side: the chunk's point gradients, rows (s, j)
    if ((rc = gemm_f32(s, true, false, R, D1, (int)zr, 1.0f, W0, R, 0, Za0, D1, 0, 0.0f, Gxc, D1, 0, 1, 0, 0, part, pl.part)))
      return rc;
    if (Gz1 && (rc = gemm_f32(s, true, false, R, D1, (int)zr, 1.0f, W1, R, 0, Za1, D1, 0, 1.0f, Gxc, D1, 0, 1, 0, 0, part, pl.part)))
      return rc;
    hipLaunchKernelGGL(tvsw_gx_kernel, dim3((unsigned)(((long long)R * d + 255) / 256)), dim3(256), 0, s, Gxc, X, l, d,
                       n0, nc, rbf ? 1 : 0, gX);
    // tensor side: [gZ | colsum] += W [X | 1] over the chunk's points
    hipLaunchKernelGGL(tvsw_points_kernel, dim3((unsigned)(((long long)R * D1 + 255) / 256)), dim3(256), 0, s, X, l, d,
                       n0, nc, Xc);
    if ((rc = gemm_f32(s, false, false, (int)zr, D1, R, 1.0f, W0, R, 0, Xc, D1, 0, 1.0f, Gz0, D1, 0, 1, 0, 0, part, pl.part)))
      return rc;
    if (Gz1 && (rc = gemm_f32(s, false, false, (int)zr, D1, R, 1.0f, W1, R, 0, Xc, D1, 0, 1.0f, Gz1, D1, 0, 1, 0, 0, part, pl.part)))
      return rc;
  }
  // gZ: RBF z0 (and z1) with the colsum correction; linear: w = z (or z1 - z0: +z1, -z0)
  const long long ge = zr * d;
  const dim3 gg((unsigned)((ge + 255) / 256));
  if (rbf) {
    hipLaunchKernelGGL(tvsw_gz_kernel, gg, dim3(256), 0, s, Gz0, Z, lt, t, d, incr, 0, 1.0f, 1, gZ);
    if (Gz1) hipLaunchKernelGGL(tvsw_gz_kernel, gg, dim3(256), 0, s, Gz1, Z, lt, t, d, incr, 1, 1.0f, 1, gZ);
  } else if (incr) {
    hipLaunchKernelGGL(tvsw_gz_kernel, gg, dim3(256), 0, s, Gz0, Z, lt, t, d, incr, 1, 1.0f, 0, gZ);
    hipLaunchKernelGGL(tvsw_gz_kernel, gg, dim3(256), 0, s, Gz0, Z, lt, t, d, incr, 0, -1.0f, 0, gZ);
  } else {
    hipLaunchKernelGGL(tvsw_gz_kernel, gg, dim3(256), 0, s, Gz0, Z, lt, t, d, incr, 0, 1.0f, 0, gZ);
  }
  return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
}

}  // namespace gpsig
