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
  // seed tiles of the chunk (matrix-core GEMMs): rows ((k T + t) H + h), w_{k,t,0} = z0 (RBF) or the linear
  // seed's w, w_{k,t,1} = dz (RBF increments, H = 2);  SD[row][s nc + j] = <w, dx_{n0+j,s}>, and one row
  // (k T + t) of SX[.][s nc + j] = <w', x_{n0+j,s}> with w' = dz (RBF increments) or w (linear; RBF without
  // increments needs none)
  const float *SD, *SX;
  long long sdl, sxl;
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
  constexpr int H = (RBF && INCR) ? 2 : 1;
  constexpr int ANCHOR = 32;
  constexpr float NHL2E = -0.72134752044448170f, L2E = 1.4426950408889634f;
  const int lane = threadIdx.x;
  const int tt = blockIdx.y;
  const int n = a.n, d = a.d, FC = 2 * d + 3, T = a.t, L = a.l, LT = a.lt;
  const int sl = blockIdx.x * 64 + lane;  // sequence within the launch's chunk
  const bool valid = sl < a.nc;
  const int slc = valid ? sl : a.nc - 1;
  const int sq = a.n0 + slc;
  cfloat *z0 = as_const(a.Zw) + (long long)tt * tvsw_zs(d, LT, INCR) + KB;  // channel q, component c: z0[q LT + c]
  cfloat *dz = z0 + (long long)d * LT;
  cfloat *hdz = z0 + (long long)2 * d * LT;
  auto ft = [&](int s, int c) { return a.Ft[((long long)s * FC + c) * n + sq]; };
  auto em1 = [](float v) { return __builtin_fabsf(v) < EM1_TAU ? em1_small(v) : __builtin_amdgcn_exp2f(v * L2E) - 1.0f; };
  // the step dots from the seed tiles: <w_{c,h}, dx_s> (SD) and <w_{c,h}, x_s> (SX)
  const float *sd = a.SD + ((long long)KB * T + tt) * H * a.sdl + slc;
  const float *sx = a.SX + ((long long)KB * T + tt) * a.sxl + slc;
  auto dxdot = [&](int c, int h, int s) { return sd[((long long)c * T * H + h) * a.sdl + (long long)s * a.nc]; };
  auto xdot = [&](int c, int s) { return sx[(long long)c * T * a.sxl + (long long)s * a.nc]; };
  float zdz[I];  // <z0, dz> of each component (RBF increments)
#pragma unroll
  for (int c = 0; c < I; ++c) zdz[c] = 0.f;
  if constexpr (RBF && INCR) {
    for (int q = 0; q < d; ++q)
#pragma unroll
      for (int c = 0; c < I; ++c) zdz[c] = __builtin_fmaf(z0[(long long)q * LT + c], dz[(long long)q * LT + c], zdz[c]);
  }

  // exact point values of the level's components at x_s: RBF k(z0, x_s) [and k(z1, x_s)] (the anchors)
  auto pexact = [&](int s, float (&v0)[I], float (&v1)[I]) {
    float e0[I], e1[I];
#pragma unroll
    for (int c = 0; c < I; ++c) e0[c] = e1[c] = 0.f;
    for (int q = 0; q < d; ++q) {
      const float xv = ft(s, q);
#pragma unroll
      for (int c = 0; c < I; ++c) {
        const float d0 = z0[(long long)q * LT + c] - xv;
        e0[c] = __builtin_fmaf(d0, d0, e0[c]);
        if constexpr (INCR) {
          const float d1 = d0 + dz[(long long)q * LT + c];
          e1[c] = __builtin_fmaf(d1, d1, e1[c]);
        }
      }
    }
#pragma unroll
    for (int c = 0; c < I; ++c) {
      v0[c] = __builtin_amdgcn_exp2f(e0[c] * NHL2E);
      v1[c] = INCR ? __builtin_amdgcn_exp2f(e1[c] * NHL2E) : 0.f;
    }
  };
  // p_s = <x_s - z0, dz> - |dz|^2 / 2 of each component (RBF increments): k(z1, x_s) = k(z0, x_s) e^p
  auto pstep = [&](int s, float (&p)[I]) {
#pragma unroll
    for (int c = 0; c < I; ++c) p[c] = (RBF && INCR) ? xdot(c, s) - zdz[c] - hdz[c] : 0.f;
  };
  // q_s = <z0, dx_s> - g_s (RBF: k(z0, x_{s+1}) = k(z0, x_s) e^q), c_s = <dz, dx_s>; linear: the cell itself
  auto qstep = [&](int s, float (&qv)[I], float (&cv)[I]) {
    const float gs = RBF ? ft(s, 2 * d + 1) : 0.f;
#pragma unroll
    for (int c = 0; c < I; ++c) {
      qv[c] = dxdot(c, 0, s) - gs;
      cv[c] = (RBF && INCR) ? dxdot(c, 1, s) : 0.f;
    }
  };
  // point values from k(z0, x_s) (RBF; k(z1, x_s) = k(z0, x_s) e^p, evaluated exactly -- k(z0, x_s) refreshed
  // too -- where some |p| > 20) or the linear point value <w, x_s>
  auto points = [&](int s, float (&k0)[I], const float (&p)[I], float (&v0)[I], float (&v1)[I]) {
    if constexpr (RBF && INCR) {
      float mx = 0.f;
#pragma unroll
      for (int c = 0; c < I; ++c) mx = __builtin_fmaxf(mx, __builtin_fabsf(p[c]));
      if (__builtin_amdgcn_ballot_w64(mx > 20.0f) != 0) {
        pexact(s, k0, v1);
#pragma unroll
        for (int c = 0; c < I; ++c) v0[c] = k0[c];
        return;
      }
    }
#pragma unroll
    for (int c = 0; c < I; ++c) {
      if constexpr (RBF) {
        v0[c] = k0[c];
        v1[c] = INCR ? k0[c] * __builtin_amdgcn_exp2f(p[c] * L2E) : 0.f;
      } else {
        v0[c] = xdot(c, s);
        v1[c] = 0.f;
      }
    }
  };
  // cells M_c(s) (difference) from the step's q, c, p and the point values at s (c0, c1) and s + 1 (n0, n1)
  auto cells = [&](const float (&qv)[I], const float (&cv)[I], const float (&p)[I], const float (&c0)[I],
                   const float (&c1)[I], const float (&n0)[I], const float (&n1)[I], float (&m)[I]) {
#pragma unroll
    for (int c = 0; c < I; ++c) {
      if constexpr (!RBF) {
        m[c] = qv[c];
      } else if constexpr (!INCR) {
        m[c] = c0[c] * em1(qv[c]);  // k(z, x_{s+1}) - k(z, x_s), any q
      } else {
        const float mx = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(p[c]), __builtin_fabsf(qv[c])), __builtin_fabsf(cv[c]));
        if (mx < EM1_TAU) {
          const float Ep = em1_small(p[c]), Eq = em1_small(qv[c]), Ec = em1_small(cv[c]);
          m[c] = c0[c] * __builtin_fmaf(Ep, Eq, (1.0f + Ep) * (1.0f + Eq) * Ec);
        } else {
          m[c] = (n1[c] - n0[c]) - (c1[c] - c0[c]);
        }
      }
    }
  };
  // point cells (difference=False): RBF k(z0, x) [k(z1, x) - k(z0, x)], linear <w, x>
  auto pcells = [&](const float (&v0)[I], const float (&v1)[I], float (&m)[I]) {
#pragma unroll
    for (int c = 0; c < I; ++c) m[c] = RBF ? (INCR ? v1[c] - v0[c] : v0[c]) : v0[c];
  };
  // k(z0, x) carried along the sweep by e^{+-q} (sgn q: the exponent of this step), re-evaluated exactly every
  // ANCHOR points, wherever |q| >= 2 (the rounding of q costs |q| eps of the exponent per carried step: the
  // forward kernel's TVS_CORNER), and wherever a carried value below 1e-30 is about to grow: once it has
  // underflowed to 0 (or a denormal) the product cannot bring it back, while the exact value may have climbed
  // to O(1) by the next anchor (wave-uniform)
  auto far = [](const float (&qv)[I], const float (&kv)[I], float sgn) {
    float mx = 0.f;
    bool tiny = false;
#pragma unroll
    for (int c = 0; c < I; ++c) {
      mx = __builtin_fmaxf(mx, __builtin_fabsf(qv[c]));
      tiny = tiny || (kv[c] < 1e-30f && sgn * qv[c] > 0.f);
    }
    return __builtin_amdgcn_ballot_w64(mx >= 2.0f || tiny) != 0;
  };

  const float gI = valid ? a.gout[((long long)I * T + tt) * n + sq] : 0.f;
  float A[I];
#pragma unroll
  for (int c = 0; c < I; ++c) A[c] = 0.f;
  const int nsteps = DIFF ? L - 1 : L;
  float k0[I], e1u[I];
  if (a.state) {
    const float *st = a.state + ((long long)tt * n + sq) * LTM + KB;
#pragma unroll
    for (int c = 0; c + 1 < I; ++c) A[c] = st[c];
  } else {
    // forward sweep to the end state
    if constexpr (RBF) pexact(0, k0, e1u);
    for (int s = 0; s < nsteps; ++s) {
      float m[I], qv[I], cv[I], p[I], c0v[I], c1v[I];
      const bool step = s + 1 < L;  // a cell to the next point (always for DIFF)
      if (step) qstep(s, qv, cv);
      pstep(s, p);
      points(s, k0, p, c0v, c1v);
      float k0n[I];
      if constexpr (RBF) {
        if (step) {
          if ((s + 1) % ANCHOR == 0 || far(qv, k0, 1.0f)) {
            pexact(s + 1, k0n, e1u);
          } else {
#pragma unroll
            for (int c = 0; c < I; ++c) k0n[c] = k0[c] * __builtin_amdgcn_exp2f(qv[c] * L2E);
          }
        }
      }
      if constexpr (DIFF) {
        float pn[I], n0v[I], n1v[I];
        pstep(s + 1, pn);
        points(s + 1, k0n, pn, n0v, n1v);
        cells(qv, cv, p, c0v, c1v, n0v, n1v, m);
      } else {
        pcells(c0v, c1v, m);
      }
      if constexpr (RBF) {
        if (step)
#pragma unroll
          for (int c = 0; c < I; ++c) k0[c] = k0n[c];
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
  float pv0[I], pv1[I];  // point values at s + 1 (DIFF) / the previous point
  int since = 0;         // points since the last exact k(z0, x)
  {
    const int s1 = DIFF ? stop + 1 : stop;  // the last point
    float p[I];
    if constexpr (RBF) pexact(s1, k0, e1u);
    pstep(s1, p);
    points(s1, k0, p, pv0, pv1);
  }
  for (int s = stop; s >= 0; --s) {
    float c0v[I], c1v[I], m[I], Ph[I], Av[I], qv[I], cv[I], p[I];
    const bool step = DIFF || s + 1 < L;  // the cell s -> s + 1 exists
    if (step) qstep(s, qv, cv);
    pstep(s, p);
    if constexpr (DIFF) {
      // k(z0, x_s) = k(z0, x_{s+1}) e^{-q_s}
      if constexpr (RBF) {
        if (++since >= ANCHOR || far(qv, k0, -1.0f)) {
          pexact(s, k0, e1u);
          since = 0;
        } else {
#pragma unroll
          for (int c = 0; c < I; ++c) k0[c] *= __builtin_amdgcn_exp2f(-qv[c] * L2E);
        }
      }
      points(s, k0, p, c0v, c1v);
      cells(qv, cv, p, c0v, c1v, pv0, pv1, m);
    } else {
      if constexpr (RBF) {
        if (s < stop) {  // point s from point s + 1
          if (++since >= ANCHOR || far(qv, k0, -1.0f)) {
            pexact(s, k0, e1u);
            since = 0;
          } else {
#pragma unroll
            for (int c = 0; c < I; ++c) k0[c] *= __builtin_amdgcn_exp2f(-qv[c] * L2E);
          }
        }
      }
      points(s, k0, p, c0v, c1v);
      pcells(c0v, c1v, m);
    }
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

// seed-GEMM operands: A[((k T + t) H + h)][q] = z0 / the linear seed's w (h = 0), dz (h = 1)
__global__ __launch_bounds__(256) void tvsw_seed_a_kernel(const float *__restrict__ Z, int lt, int t, int d, int incr,
                                                          int H, int lin, float *__restrict__ A) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long long)lt * t * H * d) return;
  const int q = (int)(idx % d);
  const long long r = idx / d;
  const int h = (int)(r % H);
  const float *z = Z + (r / H) * (incr ? 2 * d : d);
  A[idx] = !incr ? z[q] : ((lin || h == 1) ? z[d + q] - z[q] : z[q]);
}

// DX[(s nc + j)][q] = x_{n0 + j, s + 1, q} - x_{n0 + j, s, q}
__global__ __launch_bounds__(256) void tvsw_seed_dx_kernel(const float *__restrict__ X, int l, int d, int n0, int nc,
                                                           float *__restrict__ DX) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long long)(l - 1) * nc * d) return;
  const int q = (int)(idx % d);
  const long long r = idx / d;
  const int j = (int)(r % nc), s = (int)(r / nc);
  const float *x = X + ((long long)(n0 + j) * l + s) * d + q;
  DX[idx] = x[d] - x[0];
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
size_t tvs_tile_budget();  // sig_tvs_pk.hip (GPSIG_TVS_TILE_BYTES)

struct TvswPlan {
  int nc;
  size_t ft, zw, za0, za1, xc, gxc, gz, w0, w1, part, sa, sdx, sd, sx;
};
static TvswPlan tvsw_plan(int n, int l, int d, int lt, int t, bool incr) {
  TvswPlan p{};
  // a chunk's tiles: the weights (W0, W1) and the seeds (SD, SX with H = 2), ~6 (lt t l) floats per sequence
  long long nc = (long long)(tvs_tile_budget() / ((size_t)lt * t * l * sizeof(float) * 6));
  nc = nc < 64 ? 64 : (nc / 64) * 64;  // whole waves of sequences per chunk, or all of them in one
  if (nc > n) nc = n;
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
  p.sa = a256((size_t)lt * t * 2 * d * sizeof(float));
  p.sdx = a256((size_t)(l - 1) * nc * d * sizeof(float));
  p.sd = a256((size_t)lt * t * 2 * (l - 1) * nc * sizeof(float));
  p.sx = a256((size_t)lt * t * l * nc * sizeof(float));
  return p;
}
static size_t tvsw_bytes(const TvswPlan &p) {
  return p.ft + p.zw + p.za0 + p.za1 + p.xc + p.gxc + p.gz + p.w0 + p.w1 + p.part + p.sa + p.sdx + p.sd + p.sx;
}

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
  float *part = pl.part ? reinterpret_cast<float *>(w) : nullptr; w += pl.part;
  float *SA = reinterpret_cast<float *>(w); w += pl.sa;
  float *DXs = reinterpret_cast<float *>(w); w += pl.sdx;
  float *SD = reinterpret_cast<float *>(w); w += pl.sd;
  float *SX = reinterpret_cast<float *>(w);
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
  const int H = (rbf && incr) ? 2 : 1;
  hipLaunchKernelGGL(tvsw_seed_a_kernel, dim3((unsigned)((zr * H * d + 255) / 256)), dim3(256), 0, s, Z, lt, t, d, incr,
                     H, rbf ? 0 : 1, SA);
  float *Gz0 = Gz, *Gz1 = (rbf && incr) ? Gz + zr * (d + 1) : nullptr;
  if (hipMemsetAsync(Gz, 0, (size_t)zr * (d + 1) * sizeof(float) * (Gz1 ? 2 : 1), s) != hipSuccess) return GPSIG_ELAUNCH;
  const int D1 = d + 1;
  for (int n0 = 0; n0 < n; n0 += pl.nc) {
    const int nc = n - n0 < pl.nc ? n - n0 : pl.nc;
    // the chunk's seeds: <w, dx_s> and <w, x_s> of every component row, one GEMM each
    const long long cd = (long long)(l - 1) * nc, cx = (long long)l * nc;
    hipLaunchKernelGGL(tvsw_seed_dx_kernel, dim3((unsigned)((cd * d + 255) / 256)), dim3(256), 0, s, X, l, d, n0, nc, DXs);
    hipLaunchKernelGGL(tvsw_points_kernel, dim3((unsigned)((cx * (d + 1) + 255) / 256)), dim3(256), 0, s, X, l, d, n0,
                       nc, Xc);
    if ((rc = gemm_f32(s, false, true, (int)(zr * H), (int)cd, d, 1.0f, SA, d, 0, DXs, d, 0, 0.0f, SD, cd, 0, 1, 0, 0,
                       nullptr, 0)))
      return rc;
    // the x-dots of the dz rows (RBF increments: every other row of SA) or of the linear seed's w
    if ((rbf && incr) || !rbf) {
      const float *Aw = (rbf && incr) ? SA + d : SA;
      if ((rc = gemm_f32(s, false, true, (int)zr, (int)cx, d, 1.0f, Aw, (long long)H * d, 0, Xc, d + 1, 0, 0.0f, SX, cx,
                         0, 1, 0, 0, nullptr, 0)))
        return rc;
    }
    TvsBwdWideArgs a{Zw, Ft, t, n, l, d, lt, gout, state, n0, nc, W0, W1 ? W1 : W0, SD, SX, cd, cx};
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
    // tensor side: [gZ | colsum] += W [X | 1] over the chunk's points (Xc, built for the seeds)
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
