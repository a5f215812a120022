// gpsig_amd -- gradient of the inducing-tensor Gram (tensor_kern, signature_algs.py:76-99, over the
// component Grams of _K_tens, kernels.py:264-284) for wide channel counts, as pair tiles + matrix-core GEMMs.
//
// K_i(t, t') = prod_{c in level i} m_c(t, t'), m_c the component kernel of tensor component c; with
// G_i(t, t') = dLoss/dK_i and Gs = G_i(t, t') + G_i(t', t) (t as either argument), the weight of component c
// at the pair is w_c = Gs prod_{c' != c} m_c'.  The gradient is a weighted sum over t' of the derivative of
// m_c, which for the difference-of-RBF / linear components is linear in the points of t':
//   RBF, increments   m = k(a1,b1) + k(a0,b0) - k(a1,b0) - k(a0,b1),  dk(a,b)/da = k(a,b) (b - a):
//       dL/da1 = sum_t' w k11 b1 - w k10 b0 - a1 sum_t' (w k11 - w k10)      (and a0 alike)
//   RBF            m = k(a,b):  dL/da = sum_t' w m b - a sum_t' w m
//   linear, incr.  m = <da, db>: dL/da1 = -dL/da0 = sum_t' w db
//   linear         m = <a, b>:   dL/da = sum_t' w b
// So the work splits into (A) a pair-tile kernel: the component kernels of every pair (distances over
// all channels staged through LDS, the cancellation-safe second difference of the forward kernel),
// (B) the per-pair weights w_c and coefficient matrices C (T x T per component and term), (C) batched
// GEMMs C x [Z | 1] on the matrix cores (gemm.hip; the ones column carries the row sums), (D) the
// rank-one correction and accumulation into dLoss/dZ.  Every step is O(T^2 d) or less; the runtime
// channel-window kernel it replaces (sig_tens.hip, tens_gram_vjp_kernel<16, true>) recomputed the
// component kernels once per 16-channel window of the gradient.
#include "gemm.h"
#include "sig_common.h"

namespace gpsig {

namespace {

constexpr int TG_TS = 32;  // pair tile (t rows x t' columns)
constexpr int TG_QS = 32;  // channel slice staged per step
constexpr int TG_MMAX = 8;

struct TgvArgs {
  const float *Z;  // (LT, T, zs), zs = d (points) or 2 d (point pairs)
  int T, d, zs, lt;
  float *m;        // (LT, T, T) component kernels
  float *kv;       // RBF increments: (LT, 4, T, T) = k11, k10, k00, k01
};

// mode: bit 0 = increments, bit 1 = RBF
template <int MODE>
__global__ __launch_bounds__(256) void tgv_pair_kernel(TgvArgs a) {
  constexpr bool INC = MODE & 1, RBF = (MODE & 2) != 0;
  __shared__ float sa0[TG_QS][TG_TS + 1], sad[INC ? TG_QS : 1][TG_TS + 1];
  __shared__ float sb0[TG_QS][TG_TS + 1], sbd[INC ? TG_QS : 1][TG_TS + 1];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int k = blockIdx.z;
  const int r0 = blockIdx.y * TG_TS, c0 = blockIdx.x * TG_TS;
  const int T = a.T, d = a.d;
  const float *Zk = a.Z + (long long)k * T * a.zs;

  // per output (i, j), rows r0 + ty + 16 i, columns c0 + tx + 16 j
  float s2[2][2] = {}, pp[2][2] = {}, qq[2][2] = {}, cc[2][2] = {}, e11[2][2] = {}, e10[2][2] = {}, e01[2][2] = {};
  float hda[2] = {}, hdb[2] = {};
  for (int q0 = 0; q0 < d; q0 += TG_QS) {
    __syncthreads();
    // stage a slice: rows (tid >> 5) + 8 e, channel tid & 31
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int r = (tid >> 5) + 8 * e, q = tid & 31;
      const bool qok = q0 + q < d;
      const int ta = r0 + r, tb = c0 + r;
      const float *za = Zk + (long long)ta * a.zs + q0 + q, *zb = Zk + (long long)tb * a.zs + q0 + q;
      const bool aok = qok && ta < T, bok = qok && tb < T;
      const float a0 = aok ? za[0] : 0.0f, b0 = bok ? zb[0] : 0.0f;
      sa0[q][r] = a0;
      sb0[q][r] = b0;
      if constexpr (INC) {
        sad[q][r] = aok ? za[d] - a0 : 0.0f;
        sbd[q][r] = bok ? zb[d] - b0 : 0.0f;
      }
    }
    __syncthreads();
#pragma unroll 4
    for (int q = 0; q < TG_QS; ++q) {
      float av[2], bv[2], adv[2], bdv[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        av[i] = sa0[q][ty + 16 * i];
        bv[i] = sb0[q][tx + 16 * i];
        if constexpr (INC) {
          adv[i] = sad[q][ty + 16 * i];
          bdv[i] = sbd[q][tx + 16 * i];
        }
      }
      if constexpr (RBF && INC) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          hda[i] = __builtin_fmaf(adv[i], adv[i], hda[i]);
          hdb[i] = __builtin_fmaf(bdv[i], bdv[i], hdb[i]);
        }
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          if constexpr (RBF) {
            const float df = av[i] - bv[j];
            s2[i][j] = __builtin_fmaf(df, df, s2[i][j]);
            if constexpr (INC) {
              pp[i][j] = __builtin_fmaf(-df, adv[i], pp[i][j]);
              qq[i][j] = __builtin_fmaf(df, bdv[j], qq[i][j]);
              cc[i][j] = __builtin_fmaf(adv[i], bdv[j], cc[i][j]);
              const float f11 = df + adv[i] - bdv[j], f10 = df + adv[i], f01 = df - bdv[j];
              e11[i][j] = __builtin_fmaf(f11, f11, e11[i][j]);
              e10[i][j] = __builtin_fmaf(f10, f10, e10[i][j]);
              e01[i][j] = __builtin_fmaf(f01, f01, e01[i][j]);
            }
          } else if constexpr (INC) {
            cc[i][j] = __builtin_fmaf(adv[i], bdv[j], cc[i][j]);
          } else {
            cc[i][j] = __builtin_fmaf(av[i], bv[j], cc[i][j]);
          }
        }
    }
  }
  const long long T2 = (long long)T * T;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int t1 = r0 + ty + 16 * i, t2 = c0 + tx + 16 * j;
      if (t1 >= T || t2 >= T) continue;
      const long long o = (long long)t1 * T + t2;
      float mv;
      if constexpr (RBF && INC) {
        // the forward's cancellation-safe second difference (sig_tens.hip rbf_second_diff)
        const float p = pp[i][j] - 0.5f * hda[i], q = qq[i][j] - 0.5f * hdb[j], c = cc[i][j];
        const float k00 = fast_exp(-0.5f * s2[i][j]);
        const float k11 = fast_exp(-0.5f * e11[i][j]), k10 = fast_exp(-0.5f * e10[i][j]);
        const float k01 = fast_exp(-0.5f * e01[i][j]);
        const float mx = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(p), __builtin_fabsf(q)), __builtin_fabsf(c));
        if (mx < EM1_TAU) {
          const float Ep = em1_small(p), Eq = em1_small(q), Ec = em1_small(c);
          mv = k00 * __builtin_fmaf(Ep, Eq, (1.0f + Ep) * (1.0f + Eq) * Ec);
        } else {
          mv = (k11 - k10) - (k01 - k00);
        }
        if (a.kv) {  // the VJP's corner kernels (the forward Gram needs m only)
          float *kv = a.kv + (long long)k * 4 * T2 + o;
          kv[0] = k11;
          kv[T2] = k10;
          kv[2 * T2] = k00;
          kv[3 * T2] = k01;
        }
      } else if constexpr (RBF) {
        mv = fast_exp(-0.5f * s2[i][j]);
      } else {
        mv = cc[i][j];
      }
      a.m[(long long)k * T2 + o] = mv;
    }
}

struct TgwArgs {
  const float *m, *gout;  // m (LT, T, T); gout (M+1, T, T)
  float *C;               // RBF increments: (LT, 4, T, T) in place over kv; else (LT, T, T)
  int T, M;
};

// (B) the pair weights of level blockIdx.y + 1 and the coefficient matrices of its components; C:
// RBF increments [w k11, -w k10, w k00, -w k01], RBF w m, linear w
template <int MODE>
__global__ __launch_bounds__(256) void tgv_weight_kernel(TgwArgs a) {
  constexpr bool INC = MODE & 1, RBF = (MODE & 2) != 0;
  const long long T2 = (long long)a.T * a.T;
  const long long o = (long long)blockIdx.x * 256 + threadIdx.x;
  if (o >= T2) return;
  const int i = blockIdx.y + 1, k0 = i * (i - 1) / 2;
  const int t1 = (int)(o / a.T), t2 = (int)(o % a.T);
  const float Gs = a.gout[(long long)i * T2 + o] + a.gout[(long long)i * T2 + (long long)t2 * a.T + t1];
  float m[TG_MMAX];
#pragma unroll
  for (int c = 0; c < TG_MMAX; ++c)
    if (c < i) m[c] = a.m[(long long)(k0 + c) * T2 + o];
  float pre[TG_MMAX], suf = 1.0f;
  pre[0] = 1.0f;
#pragma unroll
  for (int c = 1; c < TG_MMAX; ++c) pre[c] = c < i ? pre[c - 1] * m[c - 1] : 0.0f;
#pragma unroll
  for (int c = TG_MMAX - 1; c >= 0; --c) {
    if (c >= i) continue;
    const float w = Gs * pre[c] * suf;
    suf *= m[c];
    const int k = k0 + c;
    if constexpr (RBF && INC) {
      float *C = a.C + (long long)k * 4 * T2 + o;
      C[0] = w * C[0];
      C[T2] = -w * C[T2];
      C[2 * T2] = w * C[2 * T2];
      C[3 * T2] = -w * C[3 * T2];
    } else if constexpr (RBF) {
      a.C[(long long)k * T2 + o] = w * m[c];
    } else {
      a.C[(long long)k * T2 + o] = w;
    }
  }
}

// [Z_h | 1] (RBF), dZ (linear increments), Z (linear): P (LT, H, T, d + 1)
__global__ __launch_bounds__(256) void tgv_points_kernel(const float *__restrict__ Z, int lt, int T, int d, int zs,
                                                         int H, int mode, float *__restrict__ P) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long n = (long long)lt * H * T * (d + 1);
  if (idx >= n) return;
  const int q = (int)(idx % (d + 1));
  long long r = idx / (d + 1);
  const int t = (int)(r % T);
  r /= T;
  const int h = (int)(r % H);
  const int k = (int)(r / H);
  const float *z = Z + ((long long)k * T + t) * zs;
  float v;
  if (q == d) v = (mode & 2) ? 1.0f : 0.0f;
  else if (mode == 1) v = z[d + q] - z[q];  // linear increments: db
  else v = z[h * d + q];
  P[idx] = v;
}

// (D) gZ[k, t, h, q] += G[k, h, t, q] - G[k, h, t, d] z (RBF); linear increments: gZ[.., 1, q] += G,
// gZ[.., 0, q] -= G; linear: gZ += G
__global__ __launch_bounds__(256) void tgv_emit_kernel(const float *__restrict__ G, const float *__restrict__ Z,
                                                       int lt, int T, int d, int zs, int mode, float *__restrict__ gZ) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long n = (long long)lt * T * zs;
  if (idx >= n) return;
  const int e = (int)(idx % zs);
  const long long kt = idx / zs;  // k * T + t
  const int h = e >= d ? 1 : 0, q = e - h * d;
  const int k = (int)(kt / T), t = (int)(kt % T);
  const int H = (mode == 3) ? 2 : 1;
  const float *g = G + (((long long)k * H + (mode == 3 ? h : 0)) * T + t) * (d + 1);
  float v;
  if (mode & 2) v = __builtin_fmaf(-g[d], Z[idx], g[q]);
  else if (mode == 1) v = h ? g[q] : -g[q];
  else v = g[q];
  gZ[idx] += v;
}

// out[i][t][t'] = prod of the level's component kernels (out[0] = 1): the forward Gram from the pair tiles
__global__ __launch_bounds__(256) void tgv_levels_kernel(const float *__restrict__ m, int T, int M,
                                                         float *__restrict__ out) {
  const long long T2 = (long long)T * T;
  const long long o = (long long)blockIdx.x * 256 + threadIdx.x;
  if (o >= T2) return;
  out[o] = 1.0f;
  int k = 0;
  for (int i = 1; i <= M; ++i) {
    float prod = 1.0f;
    for (int st = 0; st < i; ++st, ++k) prod = st == 0 ? m[(long long)k * T2 + o] : m[(long long)k * T2 + o] * prod;
    out[(long long)i * T2 + o] = prod;
  }
}

size_t al256(size_t b) { return (b + 255) & ~(size_t)255; }

struct TgvPlan {
  size_t m, kv, P, G;
};

TgvPlan tgv_plan(int lt, int t, int incr, int d, int rbf) {
  const long long T2 = (long long)t * t;
  const int H = (rbf && incr) ? 2 : 1;
  TgvPlan p;
  p.m = al256((size_t)lt * T2 * sizeof(float));
  p.kv = al256((size_t)lt * (rbf && incr ? 4 : 1) * T2 * sizeof(float));
  p.P = al256((size_t)lt * H * t * (d + 1) * sizeof(float));
  p.G = p.P;
  return p;
}

}  // namespace

size_t tens_gram_vjp_mm_bytes(int lt, int t, int incr, int d, int rbf) {
  const TgvPlan p = tgv_plan(lt, t, incr, d, rbf);
  return p.m + p.kv + p.P + p.G;
}

size_t tens_gram_mm_bytes(int lt, int t) { return al256((size_t)lt * t * t * sizeof(float)); }

// The forward tensor Gram past 32 channels: the VJP's pair-tile kernel (component kernels over all channels
// staged through LDS) and the level products
int tens_gram_mm(const float *Z, int lt, int t, int incr, int d, int M, int rbf, float *out, void *workspace,
                 size_t workspace_bytes, hipStream_t s) {
  if (M > TG_MMAX) return GPSIG_EUNSUPPORTED;
  if (!workspace || workspace_bytes < tens_gram_mm_bytes(lt, t)) return GPSIG_EWORKSPACE;
  if ((t + TG_TS - 1) / TG_TS > 65535 || lt > 65535) return GPSIG_EUNSUPPORTED;
  float *m = static_cast<float *>(workspace);
  const int mode = (incr ? 1 : 0) | (rbf ? 2 : 0);
  TgvArgs pa{Z, t, d, incr ? 2 * d : d, lt, m, nullptr};
  const dim3 tg((t + TG_TS - 1) / TG_TS, (t + TG_TS - 1) / TG_TS, lt);
  switch (mode) {
    case 0: hipLaunchKernelGGL(tgv_pair_kernel<0>, tg, dim3(256), 0, s, pa); break;
    case 1: hipLaunchKernelGGL(tgv_pair_kernel<1>, tg, dim3(256), 0, s, pa); break;
    case 2: hipLaunchKernelGGL(tgv_pair_kernel<2>, tg, dim3(256), 0, s, pa); break;
    default: hipLaunchKernelGGL(tgv_pair_kernel<3>, tg, dim3(256), 0, s, pa); break;
  }
  const long long T2 = (long long)t * t;
  hipLaunchKernelGGL(tgv_levels_kernel, dim3((unsigned)((T2 + 255) / 256)), dim3(256), 0, s, m, t, M, out);
  return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
}

int tens_gram_vjp_mm(const float *Z, int lt, int t, int incr, int d, int M, int rbf, const float *gout, float *gZ,
                     void *workspace, size_t workspace_bytes, hipStream_t s) {
  if (M > TG_MMAX) return GPSIG_EUNSUPPORTED;
  const TgvPlan pl = tgv_plan(lt, t, incr, d, rbf);
  if (!workspace || workspace_bytes < pl.m + pl.kv + pl.P + pl.G) return GPSIG_EWORKSPACE;
  char *w = static_cast<char *>(workspace);
  float *m = reinterpret_cast<float *>(w); w += pl.m;
  float *C = reinterpret_cast<float *>(w); w += pl.kv;
  float *P = reinterpret_cast<float *>(w); w += pl.P;
  float *G = reinterpret_cast<float *>(w);
  const int mode = (incr ? 1 : 0) | (rbf ? 2 : 0);
  const int zs = incr ? 2 * d : d, H = mode == 3 ? 2 : 1;
  const long long T2 = (long long)t * t;
  if ((t + TG_TS - 1) / TG_TS > 65535 || lt > 65535 || (T2 + 255) / 256 > 0x7fffffffLL) return GPSIG_EUNSUPPORTED;

  // (A) component kernels of every pair
  TgvArgs pa{Z, t, d, zs, lt, m, C};
  const dim3 tg((t + TG_TS - 1) / TG_TS, (t + TG_TS - 1) / TG_TS, lt);
  switch (mode) {
    case 0: hipLaunchKernelGGL(tgv_pair_kernel<0>, tg, dim3(256), 0, s, pa); break;
    case 1: hipLaunchKernelGGL(tgv_pair_kernel<1>, tg, dim3(256), 0, s, pa); break;
    case 2: hipLaunchKernelGGL(tgv_pair_kernel<2>, tg, dim3(256), 0, s, pa); break;
    default: hipLaunchKernelGGL(tgv_pair_kernel<3>, tg, dim3(256), 0, s, pa); break;
  }
  // (B) weights and coefficient matrices, one grid row per level
  TgwArgs wa{m, gout, C, t, M};
  const dim3 wg((unsigned)((T2 + 255) / 256), M);
  switch (mode) {
    case 0: hipLaunchKernelGGL(tgv_weight_kernel<0>, wg, dim3(256), 0, s, wa); break;
    case 1: hipLaunchKernelGGL(tgv_weight_kernel<1>, wg, dim3(256), 0, s, wa); break;
    case 2: hipLaunchKernelGGL(tgv_weight_kernel<2>, wg, dim3(256), 0, s, wa); break;
    default: hipLaunchKernelGGL(tgv_weight_kernel<3>, wg, dim3(256), 0, s, wa); break;
  }
  const long long np = (long long)lt * H * t * (d + 1);
  hipLaunchKernelGGL(tgv_points_kernel, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, s, Z, lt, t, d, zs, H, mode, P);
  if (hipGetLastError() != hipSuccess) return GPSIG_ELAUNCH;

  // (C) G[k][h] = sum of C[k][term] x P[k][h'] over the terms of point side h, batched over the components
  const int D1 = d + 1;
  const long long sP = (long long)H * t * D1;
  int rc;
  auto mm = [&](int term, int hin, int hout, float beta) {
    const long long sC = (long long)(mode == 3 ? 4 : 1) * T2;
    return gemm_f32(s, false, false, t, D1, t, 1.0f, C + term * T2, t, sC, P + (long long)hin * t * D1, D1, sP, beta,
                    G + (long long)hout * t * D1, D1, sP, lt, 0, 0, nullptr, 0);
  };
  if (mode == 3) {
    // a1 side: w k11 [b1 | 1] - w k10 [b0 | 1];  a0 side: w k00 [b0 | 1] - w k01 [b1 | 1]
    if ((rc = mm(0, 1, 1, 0.0f)) || (rc = mm(1, 0, 1, 1.0f)) || (rc = mm(2, 0, 0, 0.0f)) || (rc = mm(3, 1, 0, 1.0f)))
      return rc;
  } else if ((rc = mm(0, 0, 0, 0.0f))) {
    return rc;
  }
  // (D) correction and accumulation
  const long long nz = (long long)lt * t * zs;
  hipLaunchKernelGGL(tgv_emit_kernel, dim3((unsigned)((nz + 255) / 256)), dim3(256), 0, s, G, Z, lt, t, d, zs, mode, gZ);
  return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
}

}  // namespace gpsig
