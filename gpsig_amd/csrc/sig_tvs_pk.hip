// gpsig_amd -- fast path of gpsig_tens_vs_seq on gfx950: RBF base kernel, difference=True, order 1,
// d <= 8, num_levels <= 6 (signature_algs.py:101-127 with the seeds of kernels.py:314-341).
//
// One wave per (tensor t, 128 sequences): each lane carries TWO sequences as the halves of packed
// fp32 pairs (v_pk_* instructions), the tensor's components are wave-uniform SGPR operands.  Each
// lane streams its sequences in time; per component k and time cell the seed is the time difference
// of the base kernel, evaluated without cancellation and without an exp:
//   M = k(z, x_{s+1}) - k(z, x_s) = k(z, x_s) expm1(q),  q = <z, dx_s> - g_s   (g_s = <x_s,dx_s> + |dx_s|^2/2)
//   k(z, x_{s+1}) = k(z, x_s) + M                                              (row recurrence)
// and with increments (component = (z0, z1), seed = time difference of k(z1, x) - k(z0, x)):
//   M = k(z0, x_s) (Ep Eq + (1 + Ep)(1 + Eq) Ec),  p = -<z0 - x_s, dz> - |dz|^2/2,  q = <z0, dx_s> - g_s,
//   c = <dz, dx_s>;   k(z0, x_{s+1}) = k(z0, x_s)(1 + Eq),  Ep_{s+1} = Ep + Ec + Ep Ec.
// k (and Ep) are re-evaluated exactly every ANCHOR (32) cells.  Arguments past the polynomial range take
// expm1 = e^x - 1 (a wave-uniform branch); with increments, |q| or |c| >= 2 (far-apart corners) takes
// the plain corner difference of directly evaluated base-kernel values.
#include <stdlib.h>

#include "gemm.h"
#include "sig_common.h"

namespace gpsig {

struct TvsPkArgs {
  const float *Zp;  // (T, LT, ZS) prepared components: z (DP) | or z0 (DP), dz (DP), |dz|^2/2
  const float *Ft;  // time-major features Ft[(s * FC + c) * n + seq], FC = 2d + 3 (sig_tens.hip)
  int t, n, l, d;
  float *out;       // (M+1, T, n)
  float *state;     // optional (T, n, LT): end-of-sweep running sums of every component (the VJP's
                    // saved state, gpsig_tens_vs_seq_state)
};

template <int DP, bool INCR>
__host__ __device__ constexpr int tvs_zs() { return INCR ? ((2 * DP + 1 + 1) & ~1) : DP; }

// Zp[(tt * LT + k) * ZS + .] from Z (LT, T, d) or (LT, T, 2, d)
template <int DP, bool INCR>
__global__ __launch_bounds__(256) void tvs_prep_kernel(const float *__restrict__ Z, int lt, int t, int d,
                                                       float *__restrict__ Zp) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= lt * t) return;
  const int k = idx % lt, tt = idx / lt;
  constexpr int ZS = tvs_zs<DP, INCR>();
  float *o = Zp + (long long)(tt * lt + k) * ZS;
  if (!INCR) {
    const float *z = Z + ((long long)k * t + tt) * d;
    for (int q = 0; q < DP; ++q) o[q] = q < d ? z[q] : 0.f;
  } else {
    const float *z = Z + (((long long)k * t + tt) * 2) * d;
    float h = 0.f;
    for (int q = 0; q < DP; ++q) {
      const float z0 = q < d ? z[q] : 0.f, dz = q < d ? z[d + q] - z[q] : 0.f;
      o[q] = z0;
      o[DP + q] = dz;
      h = __builtin_fmaf(dz, dz, h);
    }
    o[2 * DP] = 0.5f * h;
    for (int q = 2 * DP + 1; q < ZS; ++q) o[q] = 0.f;
  }
}

template <int DP, int M, bool INCR>
#ifndef GPSIG_TVS_WPE
#define GPSIG_TVS_WPE 2
#endif
#ifndef GPSIG_TVS_WPE0
#define GPSIG_TVS_WPE0 1
#endif
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(INCR ? GPSIG_TVS_WPE : GPSIG_TVS_WPE0))) void tvs_pk_kernel(TvsPkArgs a) {
  constexpr int LT = M * (M + 1) / 2;
  constexpr int ZS = tvs_zs<DP, INCR>();
#ifndef GPSIG_TVS_ANCHOR
#define GPSIG_TVS_ANCHOR 32
#endif
  constexpr int ANCHOR = GPSIG_TVS_ANCHOR;
  constexpr float TVS_CORNER = 2.0f;  // |q| or |c| past this: corner form (increments)
  constexpr float NHL2E = -0.72134752044448170f, L2E = 1.4426950408889634f;
  const int lane = threadIdx.x;
  const int tt = blockIdx.y;
  // instantiated per exact channel count (DP == a.d): no per-channel guards in the time loop
  constexpr int d = DP;
  const int n = a.n, FC = 2 * d + 3;
  const int s0 = blockIdx.x * 128 + lane, s1 = s0 + 64;
  const int c0 = s0 < n ? s0 : n - 1, c1 = s1 < n ? s1 : n - 1;
  // The tensor's components are wave-uniform: staged once in LDS (broadcast reads, ~100-cycle
  // latency) instead of the L2-latency global loads the compiler emits for them (it cannot prove the
  // prepared buffer invariant against the output stores, so it does not use scalar loads).
  __shared__ __attribute__((aligned(16))) float zl[LT * ZS];
  for (int e = lane; e < LT * ZS; e += 64) zl[e] = a.Zp[(long long)tt * LT * ZS + e];
  __syncthreads();
  const float *zp = zl;

  // loads of channel c of cell s for both sequences of the lane
  auto ld = [&](int s, int c) {
    const float *f = a.Ft + ((long long)s * FC + c) * n;
    return (f2){f[c0], f[c1]};
  };
  auto ldx = [&](int s, f2 (&x)[DP]) {
#pragma unroll
    for (int q = 0; q < DP; ++q) x[q] = q < d ? ld(s, q) : splat2(0.f);
  };
  // exact k(z0_k, x) and (INCR) expm1(p_k) for the point x
  auto exact = [&](int k, const f2 (&x)[DP], f2 &kck, f2 &Epk) {
    const float *z = zp + k * ZS;
    f2 s2 = splat2(0.f), pp = splat2(0.f);
#pragma unroll
    for (int q = 0; q < DP; ++q) {
      const f2 df = splat2(z[q]) - x[q];
      s2 = fma2(df, df, s2);
      if constexpr (INCR) pp = fma2(df, splat2(-z[DP + q]), pp);
    }
    s2 = s2 * splat2(NHL2E);
    kck[0] = __builtin_amdgcn_exp2f(s2[0]);
    kck[1] = __builtin_amdgcn_exp2f(s2[1]);
    if constexpr (INCR) {
      pp = pp - splat2(z[2 * DP]);
      Epk = em1_small2(pp);
#pragma unroll
      for (int h = 0; h < 2; ++h)
        if (!(__builtin_fabsf(pp[h]) < EM1_TAU)) Epk[h] = __builtin_amdgcn_exp2f(pp[h] * L2E) - 1.0f;
    }
  };

  f2 kc[LT], Ep[LT], Ss[LT], K[M + 1];
#pragma unroll
  for (int k = 0; k < LT; ++k) Ss[k] = splat2(0.f);
#pragma unroll
  for (int i = 0; i <= M; ++i) K[i] = splat2(0.f);
  {
    f2 x0[DP];
    ldx(0, x0);
#pragma unroll
    for (int k = 0; k < LT; ++k) exact(k, x0, kc[k], Ep[k]);
  }

  const int ncell = a.l - 1;
  bool far = false;  // wave-uniform: the previous step had some |q| >= TVS_CORNER (no increments)
  for (int s = 0; s < ncell; ++s) {
    // keeps the component reads inside the loop (hoisted, LT x ZS of them would not fit in registers)
    asm volatile("" ::: "memory");
    f2 dx[DP];
#pragma unroll
    for (int q = 0; q < DP; ++q) dx[q] = q < d ? ld(s, d + q) : splat2(0.f);
    const f2 g = ld(s, 2 * d + 1);
    const bool anch = (s % ANCHOR) == ANCHOR - 1 || far;
    f2 x1[DP];
    if (anch) ldx(s + 1, x1);
    uint64_t farm = 0;  // lanes with some |q| >= TVS_CORNER this step (no increments; a scalar mask)
    // components in (level, stage) order; the order-1 recursion (signature_algs.py:115-127) is folded
    // in as each seed is produced
#pragma unroll
    for (int i = 1; i <= M; ++i) {
      const int k0 = i * (i - 1) / 2;
      f2 prev = splat2(0.f);
#pragma unroll
      for (int st = 0; st < i; ++st) {
        const int k = k0 + st;
        // one component's LDS reads at a time: scheduled all up front they would keep LT x ZS values
        // live (the increments kernel then spilled to AGPRs)
        if constexpr (INCR) asm volatile("" ::: "memory");
        const float *z = zp + k * ZS;
        f2 qv = -g, cv = splat2(0.f);
#pragma unroll
        for (int q = 0; q < DP; ++q) {
          qv = fma2(dx[q], splat2(z[q]), qv);
          if constexpr (INCR) cv = fma2(dx[q], splat2(z[DP + q]), cv);
        }
        float mx = __builtin_fmaxf(__builtin_fabsf(qv[0]), __builtin_fabsf(qv[1]));
        if constexpr (INCR) mx = __builtin_fmaxf(mx, __builtin_fmaxf(__builtin_fabsf(cv[0]), __builtin_fabsf(cv[1])));
        f2 Eq = em1_small2(qv), Ec = splat2(0.f);
        if constexpr (INCR) Ec = em1_small2(cv);
        const bool wide = __builtin_amdgcn_ballot_w64(mx >= EM1_TAU) != 0;
        if (wide) {
          // arguments past the polynomial range: expm1 = e^x - 1 (no cancellation there)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            // (finite: e^q past FLT_MAX only multiplies an underflowed carry, where 0 * inf would be NaN)
            if (!(__builtin_fabsf(qv[h]) < EM1_TAU)) Eq[h] = __builtin_fminf(__builtin_amdgcn_exp2f(qv[h] * L2E) - 1.0f, 3.0e38f);
            if constexpr (INCR)
              if (!(__builtin_fabsf(cv[h]) < EM1_TAU)) Ec[h] = __builtin_amdgcn_exp2f(cv[h] * L2E) - 1.0f;
          }
        }
        f2 m;
        if constexpr (INCR) {
          f2 t = fma2(Ep[k], Ec, Ec);
          t = fma2(Eq, t, t);
          m = kc[k] * fma2(Ep[k], Eq, t);
        } else {
          m = kc[k] * Eq;  // = k(z, x_{s+1}) - k(z, x_s) exactly, any q
        }
        if (INCR && wide && __builtin_amdgcn_ballot_w64(mx >= TVS_CORNER) != 0) {
          // increments far apart: corner differences of directly evaluated base-kernel values
          f2 xs[DP], xn[DP], kn, Epn;
          ldx(s, xs);
          ldx(s + 1, xn);
          exact(k, xn, kn, Epn);
          const float *z = zp + k * ZS;
          f2 e1 = splat2(0.f), e0 = splat2(0.f);  // |z1 - x_{s+1}|^2, |z1 - x_s|^2
#pragma unroll
          for (int q = 0; q < DP; ++q) {
            const f2 z1 = splat2(z[q] + z[DP + q]);
            const f2 d1 = z1 - xn[q], d0 = z1 - xs[q];
            e1 = fma2(d1, d1, e1);
            e0 = fma2(d0, d0, e0);
          }
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const bool ok = __builtin_fabsf(qv[h]) < TVS_CORNER && __builtin_fabsf(cv[h]) < TVS_CORNER;
            const float k11 = __builtin_amdgcn_exp2f(e1[h] * NHL2E), k10 = __builtin_amdgcn_exp2f(e0[h] * NHL2E);
            m[h] = ok ? m[h] : (k11 - k10) - (kn[h] - kc[k][h]);
          }
          kc[k] = kn;
          Ep[k] = Epn;
        } else if (anch) {
          exact(k, x1, kc[k], Ep[k]);  // re-anchor the recurrences every ANCHOR cells
        } else if constexpr (INCR) {
          kc[k] = fma2(kc[k], Eq, kc[k]);
          Ep[k] = fma2(Ep[k], Ec, Ep[k] + Ec);
        } else {
          kc[k] = kc[k] + m;
          farm |= __builtin_amdgcn_ballot_w64(mx >= TVS_CORNER);
        }
        if (st == 0) {
          prev = m;
        } else {
          const f2 ss = Ss[k - 1];
          Ss[k - 1] = ss + prev;
          prev = m * ss;
        }
      }
      K[i] += prev;
    }
    // (no increments) a step with some |q| >= TVS_CORNER re-anchors the next one: the rounding of q costs
    // |q| eps of the exponent per carried step, and a carry grown from an underflowed 0 would stay 0 (a path
    // walking towards a far inducing point).  One carried step of that error is at the fp32 noise level,
    // and below TVS_CORNER a carry can grow at most e^(2 x 31) between anchors, so one that underflowed
    // stays below 1e-11: negligible.  The anchor's own path: a second exact evaluation in or after the
    // component loop cost the kernel its third wave per SIMD (168 -> 188 VGPRs at D = 5, M = 5).
    if constexpr (!INCR) far = farm != 0;
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int sq = h ? s1 : s0;
    if (sq < n) {
      a.out[(long long)tt * n + sq] = 1.0f;
#pragma unroll
      for (int i = 1; i <= M; ++i) a.out[((long long)i * a.t + tt) * n + sq] = K[i][h];
    }
  }
  if (a.state) {  // the end-of-sweep running sums: the VJP starts at its reverse sweep
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int sq = h ? s1 : s0;
      if (sq < n) {
#pragma unroll
        for (int k = 0; k < LT; ++k) a.state[((long long)tt * n + sq) * LT + k] = Ss[k][h];
      }
    }
  }
}

// Linear base kernel (kernels.py:979-986), difference=True: the seed of component k at time cell s is
// <w_k, dx_s> with w_k = z_k (or z1_k - z0_k with increments), no state besides the running sums.
template <int DP, int M, bool INCR>
__global__ __launch_bounds__(64) void tvs_lin_kernel(TvsPkArgs a) {
  constexpr int LT = M * (M + 1) / 2;
  constexpr int ZS = tvs_zs<DP, INCR>();
  constexpr int d = DP;
  const int lane = threadIdx.x;
  const int tt = blockIdx.y;
  const int n = a.n, FC = 2 * d + 3;
  const int s0 = blockIdx.x * 128 + lane, s1 = s0 + 64;
  const int c0 = s0 < n ? s0 : n - 1, c1 = s1 < n ? s1 : n - 1;
  __shared__ __attribute__((aligned(16))) float zl[LT * ZS];
  for (int e = lane; e < LT * ZS; e += 64) zl[e] = a.Zp[(long long)tt * LT * ZS + e];
  __syncthreads();
  f2 Ss[LT], K[M + 1];
#pragma unroll
  for (int k = 0; k < LT; ++k) Ss[k] = splat2(0.f);
#pragma unroll
  for (int i = 0; i <= M; ++i) K[i] = splat2(0.f);
  for (int s = 0; s + 1 < a.l; ++s) {
    asm volatile("" ::: "memory");
    f2 dx[DP];
#pragma unroll
    for (int q = 0; q < DP; ++q) {
      const float *f = a.Ft + ((long long)s * FC + d + q) * n;
      dx[q] = (f2){f[c0], f[c1]};
    }
#pragma unroll
    for (int i = 1; i <= M; ++i) {
      const int k0 = i * (i - 1) / 2;
      f2 prev = splat2(0.f);
#pragma unroll
      for (int st = 0; st < i; ++st) {
        const int k = k0 + st;
        const float *w = zl + k * ZS + (INCR ? DP : 0);
        f2 m = splat2(0.f);
#pragma unroll
        for (int q = 0; q < DP; ++q) m = fma2(dx[q], splat2(w[q]), m);
        if (st == 0) {
          prev = m;
        } else {
          const f2 ss = Ss[k - 1];
          Ss[k - 1] = ss + prev;
          prev = m * ss;
        }
      }
      K[i] += prev;
    }
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int sq = h ? s1 : s0;
    if (sq < n) {
      a.out[(long long)tt * n + sq] = 1.0f;
#pragma unroll
      for (int i = 1; i <= M; ++i) a.out[((long long)i * a.t + tt) * n + sq] = K[i][h];
    }
  }
  if (a.state) {  // the end-of-sweep running sums: the VJP starts at its reverse sweep
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int sq = h ? s1 : s0;
      if (sq < n) {
#pragma unroll
        for (int k = 0; k < LT; ++k) a.state[((long long)tt * n + sq) * LT + k] = Ss[k][h];
      }
    }
  }
}

// ------------------------------------------------------------------------------------ wide channels
// The same recursion and seeds (tvs_pk_kernel, tvs_lin_kernel) for any channel count.  The per-step dots
// <z_k, dx_s> (and <dz_k, dx_s>) of all LT components, every tensor and every step of a chunk of sequences
// are ONE matrix-core GEMM (gemm.hip) into a seed tile
//     S[(t LT + k) H + h][s nc + j] = <w_{t,k,h}, dx_{n0 + j, s}>,   w = z0 | dz (RBF, increments; H = 2),
//                                                                    z (RBF) or the linear seed's z / dz
// which the recursion kernel streams (coalesced across its lanes = sequences, next step prefetched).  The
// exact base-kernel values at the anchors (every ANCHOR cells) and the far-apart corners keep the runtime
// channel loop over the prepared [tensor][channel][component] buffer.  One sequence per lane.
struct TvsWideArgs {
  const float *Zw;  // (T, [2,] d, LT) then (T, LT) |dz|^2 / 2: tvs_wide_prep_kernel
  const float *Ft;  // time-major features (sig_tens.hip)
  int t, n, l, d;
  float *out;
  float *state;
  const float *S;   // seed tile of the chunk [n0, n0 + nc): rows (t LT + k) H + h, row length sld
  long long sld;
  int n0, nc;
};

// seed-tile budget of one chunk of sequences (GPSIG_TVS_TILE_BYTES overrides it: the tests force several
// chunks; read per call, so the workspace query and the launch agree)
size_t tvs_tile_budget() {
  const char *e = getenv("GPSIG_TVS_TILE_BYTES");
  const long long v = e ? atoll(e) : 0;
  return v > 0 ? (size_t)v : (size_t)1 << 30;
}

struct TvsSeedPlan {
  int nc;
  size_t a, dx, s;
};

inline TvsSeedPlan tvs_seed_plan(int n, int l, int d, int lt, int t) {
  TvsSeedPlan p{};
  const size_t per_seq = (size_t)(l - 1) * t * lt * 2 * sizeof(float);  // H = 2: the largest tile
  long long nc = per_seq ? (long long)(tvs_tile_budget() / per_seq) : n;
  nc = nc < 64 ? 64 : (nc / 64) * 64;  // whole waves of sequences per chunk ...
  if (nc > n) nc = n;                   // ... or every sequence in one chunk (fewer than 64 only then)
  p.nc = (int)nc;
  p.a = (((size_t)t * lt * 2 * d * sizeof(float)) + 255) & ~(size_t)255;
  p.dx = (((size_t)nc * (l - 1) * d * sizeof(float)) + 255) & ~(size_t)255;
  p.s = (((size_t)nc * (l - 1) * t * lt * 2 * sizeof(float)) + 255) & ~(size_t)255;
  return p;
}

// workspace of the wide path's GEMM seeds (0: d <= 8 runs the packed kernels)
size_t tvs_seed_bytes(int n, int l, int d, int lt, int t) {
  if (d <= 8 || l < 2) return 0;
  const TvsSeedPlan p = tvs_seed_plan(n, l, d, lt, t);
  return p.a + p.dx + p.s;
}

// A[(t LT + k) H + h][q]: the GEMM's component rows
__global__ __launch_bounds__(256) void tvs_seed_a_kernel(const float *__restrict__ Z, int lt, int t, int d, int incr,
                                                         int H, int lin, float *__restrict__ A) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long long)t * lt * H * d) return;
  const int q = (int)(idx % d);
  long long r = idx / d;
  const int h = (int)(r % H);
  r /= H;
  const int k = (int)(r % lt), tt = (int)(r / lt);
  const float *z = Z + ((long long)k * t + tt) * (incr ? 2 * d : d);
  float v;
  if (!incr) v = z[q];
  else if (lin || h == 1) v = z[d + q] - z[q];  // the linear seed's w = z1 - z0, or dz
  else v = z[q];
  A[idx] = v;
}

// DX[(s nc + j)][q] = x_{n0 + j, s + 1, q} - x_{n0 + j, s, q}
__global__ __launch_bounds__(256) void tvs_seed_dx_kernel(const float *__restrict__ X, int l, int d, int n0, int nc,
                                                          float *__restrict__ DX) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long long)(l - 1) * nc * d) return;
  const int q = (int)(idx % d);
  const long long r = idx / d;
  const int j = (int)(r % nc), s = (int)(r / nc);
  const float *x = X + ((long long)(n0 + j) * l + s) * d + q;
  DX[idx] = x[d] - x[0];
}

__host__ __device__ inline long long tvs_wide_zs(int d, int lt, bool incr) { return (long long)(incr ? 2 * d + 1 : d) * lt; }

// Zw[tt][h][q][k] (h = 0: z0 or z, h = 1: dz = z1 - z0), then Zw[tt][2d][k] = |dz_k|^2 / 2 (increments)
__global__ __launch_bounds__(256) void tvs_wide_prep_kernel(const float *__restrict__ Z, int lt, int t, int d, int incr,
                                                            float *__restrict__ Zw) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long long)lt * t) return;
  const int k = (int)(idx % lt), tt = (int)(idx / lt);
  float *o = Zw + (long long)tt * tvs_wide_zs(d, lt, incr != 0);
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

template <int M, bool INCR, bool RBF>
__global__ __launch_bounds__(64) void tvs_wide_kernel(TvsWideArgs a) {
  constexpr int LT = M * (M + 1) / 2;
  constexpr float TVS_CORNER = 2.0f;
  constexpr float NHL2E = -0.72134752044448170f, L2E = 1.4426950408889634f;
  constexpr int ANCHOR = GPSIG_TVS_ANCHOR;
  constexpr int H = (RBF && INCR) ? 2 : 1;
  const int lane = threadIdx.x;
  const int tt = blockIdx.y;
  const int n = a.n, d = a.d, FC = 2 * d + 3;
  const int sl0 = blockIdx.x * 64 + lane;  // sequence within the chunk
  const int sl = sl0 < a.nc ? sl0 : a.nc - 1;
  const int s0 = a.n0 + sl0;
  const int c0 = a.n0 + sl;
  cfloat *z0 = as_const(a.Zw) + (long long)tt * tvs_wide_zs(d, LT, INCR);  // [q][k]
  cfloat *dz = z0 + (long long)d * LT;
  cfloat *hdz = z0 + (long long)2 * d * LT;
  auto ft = [&](int s, int c) { return a.Ft[((long long)s * FC + c) * n + c0]; };

  // exact k(z0_k, x_s) and (INCR) expm1(p_k), p = -<z0 - x, dz> - |dz|^2/2, for every component; e1 (INCR):
  // |z1 - x_s|^2 = |z0 - x_s|^2 + 2 <z0 - x_s, dz> + |dz|^2
  auto exact_all = [&](int s, float (&kc)[LT], float (&Ep)[LT], float *e1 = nullptr, float *s2o = nullptr,
                       float *ppo = nullptr) {
    float s2[LT], pp[LT];
#pragma unroll
    for (int k = 0; k < LT; ++k) s2[k] = pp[k] = 0.f;
    for (int q = 0; q < d; ++q) {
      const float xv = ft(s, q);
#pragma unroll
      for (int k = 0; k < LT; ++k) {
        const float df = z0[(long long)q * LT + k] - xv;
        s2[k] = __builtin_fmaf(df, df, s2[k]);
        if constexpr (INCR) pp[k] = __builtin_fmaf(-df, dz[(long long)q * LT + k], pp[k]);
      }
    }
#pragma unroll
    for (int k = 0; k < LT; ++k) {
      kc[k] = __builtin_amdgcn_exp2f(s2[k] * NHL2E);
      if constexpr (INCR) {
        const float p = pp[k] - hdz[k];
        Ep[k] = __builtin_fabsf(p) < EM1_TAU ? em1_small(p) : __builtin_amdgcn_exp2f(p * L2E) - 1.0f;
        if (e1) e1[k] = __builtin_fmaf(-2.0f, p, s2[k]);
        if (s2o) {
          s2o[k] = s2[k];
          ppo[k] = pp[k];
        }
      }
    }
  };

  float kc[LT], Ep[LT], Ss[LT], K[M + 1];
  // (RBF, INCR) the exponents behind kc and Ep, carried additively between exact passes: s2c = |z0 - x_s|^2
  // (-2 q per step), ppc = -<z0 - x_s, dz> (+ c per step); the corner cells evaluate from them
  float s2c[LT], ppc[LT];
#pragma unroll
  for (int k = 0; k < LT; ++k) Ss[k] = Ep[k] = kc[k] = s2c[k] = ppc[k] = 0.f;
#pragma unroll
  for (int i = 0; i <= M; ++i) K[i] = 0.f;
  if constexpr (RBF) exact_all(0, kc, Ep, nullptr, s2c, ppc);

  const int ncell = a.l - 1;
  // the step's dots from the seed tile; the next step's are in flight while this one is processed
  const float *srow = a.S + (long long)tt * LT * H * a.sld + sl;
  auto seeds = [&](int s, float (&sq)[LT], float (&sc)[LT]) {
#pragma unroll
    for (int k = 0; k < LT; ++k) {
      sq[k] = srow[(long long)(k * H) * a.sld + (long long)s * a.nc];
      if constexpr (H == 2) sc[k] = srow[(long long)(k * H + 1) * a.sld + (long long)s * a.nc];
      else sc[k] = 0.f;
    }
  };
  float sq[LT], sc[LT];
  seeds(0, sq, sc);
  for (int s = 0; s < ncell; ++s) {
    float qv[LT], cv[LT], nq[LT], ncv[LT];
    if (s + 1 < ncell) seeds(s + 1, nq, ncv);
    const float g = RBF ? ft(s, 2 * d + 1) : 0.f;
#pragma unroll
    for (int k = 0; k < LT; ++k) {
      qv[k] = sq[k] - g;
      cv[k] = sc[k];
      sq[k] = nq[k];
      sc[k] = ncv[k];
    }
    float m[LT];
    if constexpr (!RBF) {
#pragma unroll
      for (int k = 0; k < LT; ++k) m[k] = qv[k];
    } else {
      float mx = 0.f;
#pragma unroll
      for (int k = 0; k < LT; ++k) {
        mx = __builtin_fmaxf(mx, __builtin_fabsf(qv[k]));
        if constexpr (INCR) mx = __builtin_fmaxf(mx, __builtin_fabsf(cv[k]));
      }
      const bool wide = __builtin_amdgcn_ballot_w64(mx >= EM1_TAU) != 0;
      const bool corner = INCR && wide && __builtin_amdgcn_ballot_w64(mx >= TVS_CORNER) != 0;
      const bool anch = (s % ANCHOR) == ANCHOR - 1;
      float Eq[LT], Ec[LT];
#pragma unroll
      for (int k = 0; k < LT; ++k) {
        Eq[k] = em1_small(qv[k]);
        Ec[k] = INCR ? em1_small(cv[k]) : 0.f;
        if (wide) {
          if (!(__builtin_fabsf(qv[k]) < EM1_TAU)) Eq[k] = __builtin_amdgcn_exp2f(qv[k] * L2E) - 1.0f;
          if constexpr (INCR)
            if (!(__builtin_fabsf(cv[k]) < EM1_TAU)) Ec[k] = __builtin_amdgcn_exp2f(cv[k] * L2E) - 1.0f;
        }
        if constexpr (INCR) {
          float t = __builtin_fmaf(Ep[k], Ec[k], Ec[k]);
          t = __builtin_fmaf(Eq[k], t, t);
          m[k] = kc[k] * __builtin_fmaf(Ep[k], Eq[k], t);
        } else {
          m[k] = kc[k] * Eq[k];
        }
      }
      if (corner) {
        // increments far apart: corner differences of directly evaluated base-kernel values for the cells
        // with |q| or |c| >= TVS_CORNER (z1 = z0 + dz)
        // e1 = |z1 - x_{s+1}|^2 from the exact pass (s2 - 2 p with p = -<z0 - x, dz> - |dz|^2/2), and
        // e0 = |z1 - x_s|^2 = e1 + 2 <z1 - x_s, dx_s> - |dx_s|^2 = e1 + 2 (q + c) off the step's seeds
        // (q = <z0 - x_s, dx_s> - |dx_s|^2/2, c = <dz, dx_s>): no second pass over the channels
        // off an anchor row the next point's exponents come from the additive carry: no channel pass
        float kn[LT], Epn[LT], e1[LT], e0[LT];
        if (anch) {
          exact_all(s + 1, kn, Epn, e1, s2c, ppc);
        } else {
#pragma unroll
          for (int k = 0; k < LT; ++k) {
            s2c[k] = __builtin_fmaf(-2.0f, qv[k], s2c[k]);
            ppc[k] += cv[k];
            const float p = ppc[k] - hdz[k];
            kn[k] = __builtin_amdgcn_exp2f(s2c[k] * NHL2E);
            Epn[k] = __builtin_fabsf(p) < EM1_TAU ? em1_small(p) : __builtin_amdgcn_exp2f(p * L2E) - 1.0f;
            e1[k] = __builtin_fmaf(-2.0f, p, s2c[k]);
          }
        }
#pragma unroll
        for (int k = 0; k < LT; ++k) e0[k] = __builtin_fmaf(2.0f, qv[k] + cv[k], e1[k]);
#pragma unroll
        for (int k = 0; k < LT; ++k) {
          const bool ok = __builtin_fabsf(qv[k]) < TVS_CORNER && __builtin_fabsf(cv[k]) < TVS_CORNER;
          const float k11 = __builtin_amdgcn_exp2f(e1[k] * NHL2E), k10 = __builtin_amdgcn_exp2f(e0[k] * NHL2E);
          m[k] = ok ? m[k] : (k11 - k10) - (kn[k] - kc[k]);
          kc[k] = kn[k];
          Ep[k] = Epn[k];
        }
      } else if (anch) {
        exact_all(s + 1, kc, Ep, nullptr, s2c, ppc);  // re-anchor the recurrences every ANCHOR cells
      } else if (!INCR && wide && __builtin_amdgcn_ballot_w64(mx >= TVS_CORNER) != 0) {
        // exact point values instead of the carry k (1 + expm1(q)) on steps with |q| >= TVS_CORNER: the
        // rounding of q costs |q| eps of the exponent per carried step, and a carry grown from an underflowed
        // 0 would stay 0 (a path walking towards a far inducing point).  Below TVS_CORNER a carry can grow at
        // most e^(2 x 31) between anchors, so one that underflowed stays below 1e-11: negligible.  (INCR: the
        // corner regime above takes every step with |q| >= TVS_CORNER.)
        exact_all(s + 1, kc, Ep, nullptr, s2c, ppc);
      } else {
#pragma unroll
        for (int k = 0; k < LT; ++k) {
          if constexpr (INCR) {
            kc[k] = __builtin_fmaf(kc[k], Eq[k], kc[k]);
            Ep[k] = __builtin_fmaf(Ep[k], Ec[k], Ep[k] + Ec[k]);
            s2c[k] = __builtin_fmaf(-2.0f, qv[k], s2c[k]);
            ppc[k] += cv[k];
          } else {
            kc[k] = kc[k] + m[k];
          }
        }
      }
    }
    // the order-1 recursion (signature_algs.py:115-127), components in (level, stage) order
#pragma unroll
    for (int i = 1; i <= M; ++i) {
      const int k0 = i * (i - 1) / 2;
      float prev = m[k0];
#pragma unroll
      for (int st = 1; st < i; ++st) {
        const float ss = Ss[k0 + st - 1];
        Ss[k0 + st - 1] = ss + prev;
        prev = m[k0 + st] * ss;
      }
      K[i] += prev;
    }
  }
  if (s0 < n) {
    a.out[(long long)tt * n + s0] = 1.0f;
#pragma unroll
    for (int i = 1; i <= M; ++i) a.out[((long long)i * a.t + tt) * n + s0] = K[i];
    if (a.state) {
#pragma unroll
      for (int k = 0; k < LT; ++k) a.state[((long long)tt * n + s0) * LT + k] = Ss[k];
    }
  }
}

template <int M>
static int launch_tvs_wide(const TvsWideArgs &a, int incr, bool rbf, hipStream_t s) {
  dim3 grid((unsigned)((a.nc + 63) / 64), (unsigned)a.t);
  if (rbf) {
    if (incr) hipLaunchKernelGGL((tvs_wide_kernel<M, true, true>), grid, dim3(64), 0, s, a);
    else hipLaunchKernelGGL((tvs_wide_kernel<M, false, true>), grid, dim3(64), 0, s, a);
  } else {
    if (incr) hipLaunchKernelGGL((tvs_wide_kernel<M, true, false>), grid, dim3(64), 0, s, a);
    else hipLaunchKernelGGL((tvs_wide_kernel<M, false, false>), grid, dim3(64), 0, s, a);
  }
  return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
}

// X: the raw (n, l, d) sequences (the seed GEMM's increments); seedws: tvs_seed_bytes(n, l, d, lt, t)
int tvs_wide_launch(const float *Z, int lt, int t, int increments, int d, const float *X, const float *Ft, int n,
                    int l, int M, float *out, float *Zw, bool rbf, float *state, void *seedws, hipStream_t s) {
  if (l < 2 || M < 1 || M > 8 || !seedws) return -1;
  const TvsSeedPlan pl = tvs_seed_plan(n, l, d, lt, t);
  char *w = static_cast<char *>(seedws);
  float *A = reinterpret_cast<float *>(w); w += pl.a;
  float *DX = reinterpret_cast<float *>(w); w += pl.dx;
  float *S = reinterpret_cast<float *>(w);
  const int H = (rbf && increments) ? 2 : 1;
  const long long rows = (long long)t * lt * H;
  if (rows > 0x7fffffffLL) return GPSIG_EUNSUPPORTED;
  hipLaunchKernelGGL(tvs_wide_prep_kernel, dim3((unsigned)(((long long)lt * t + 255) / 256)), dim3(256), 0, s, Z, lt, t,
                     d, increments, Zw);
  hipLaunchKernelGGL(tvs_seed_a_kernel, dim3((unsigned)((rows * d + 255) / 256)), dim3(256), 0, s, Z, lt, t, d,
                     increments, H, rbf ? 0 : 1, A);
  for (int n0 = 0; n0 < n; n0 += pl.nc) {
    const int nc = n - n0 < pl.nc ? n - n0 : pl.nc;
    const long long cols = (long long)(l - 1) * nc;
    if (cols > 0x7fffffffLL) return GPSIG_EUNSUPPORTED;
    hipLaunchKernelGGL(tvs_seed_dx_kernel, dim3((unsigned)((cols * d + 255) / 256)), dim3(256), 0, s, X, l, d, n0, nc, DX);
    int rc = gemm_f32(s, false, true, (int)rows, (int)cols, d, 1.0f, A, d, 0, DX, d, 0, 0.0f, S, cols, 0, 1, 0, 0,
                      nullptr, 0);
    if (rc) return rc;
    TvsWideArgs a{Zw, Ft, t, n, l, d, out, state, S, cols, n0, nc};
    switch (M) {
      case 1: rc = launch_tvs_wide<1>(a, increments, rbf, s); break;
      case 2: rc = launch_tvs_wide<2>(a, increments, rbf, s); break;
      case 3: rc = launch_tvs_wide<3>(a, increments, rbf, s); break;
      case 4: rc = launch_tvs_wide<4>(a, increments, rbf, s); break;
      case 5: rc = launch_tvs_wide<5>(a, increments, rbf, s); break;
      case 6: rc = launch_tvs_wide<6>(a, increments, rbf, s); break;
      case 7: rc = launch_tvs_wide<7>(a, increments, rbf, s); break;
      default: rc = launch_tvs_wide<8>(a, increments, rbf, s); break;
    }
    if (rc) return rc;
  }
  return GPSIG_OK;
}

template <int DP, int M, bool INCR>
static int launch_tvs_pk(const float *Z, int lt, int t, int d, const float *Ft, int n, int l, float *out, float *Zp,
                         bool rbf, float *state, hipStream_t s) {
  hipLaunchKernelGGL((tvs_prep_kernel<DP, INCR>), dim3((unsigned)((lt * t + 255) / 256)), dim3(256), 0, s, Z, lt, t, d,
                     Zp);
  TvsPkArgs a{Zp, Ft, t, n, l, d, out, state};
  if (rbf)
    hipLaunchKernelGGL((tvs_pk_kernel<DP, M, INCR>), dim3((unsigned)((n + 127) / 128), (unsigned)t), dim3(64), 0, s, a);
  else
    hipLaunchKernelGGL((tvs_lin_kernel<DP, M, INCR>), dim3((unsigned)((n + 127) / 128), (unsigned)t), dim3(64), 0, s, a);
  return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
}

template <int DP, bool INCR>
static int tvs_pk_m(int M, const float *Z, int lt, int t, int d, const float *Ft, int n, int l, float *out, float *Zp,
                    bool rbf, float *state, hipStream_t s) {
  switch (M) {
    case 1: return launch_tvs_pk<DP, 1, INCR>(Z, lt, t, d, Ft, n, l, out, Zp, rbf, state, s);
    case 2: return launch_tvs_pk<DP, 2, INCR>(Z, lt, t, d, Ft, n, l, out, Zp, rbf, state, s);
    case 3: return launch_tvs_pk<DP, 3, INCR>(Z, lt, t, d, Ft, n, l, out, Zp, rbf, state, s);
    case 4: return launch_tvs_pk<DP, 4, INCR>(Z, lt, t, d, Ft, n, l, out, Zp, rbf, state, s);
    case 5: return launch_tvs_pk<DP, 5, INCR>(Z, lt, t, d, Ft, n, l, out, Zp, rbf, state, s);
    case 6: return launch_tvs_pk<DP, 6, INCR>(Z, lt, t, d, Ft, n, l, out, Zp, rbf, state, s);
    default: return -1;
  }
}

// -1: not covered by the fast path (the caller runs the general kernel)
int tvs_pk_launch(const float *Z, int lt, int t, int increments, int d, const float *Ft, int n, int l, int M,
                  float *out, float *Zp, bool rbf, float *state, hipStream_t s) {
  if (M > 6 || d > 8 || l < 2) return -1;
  const int DP = d;
#define GPSIG_TVS(dp)                                                               \
  case dp:                                                                          \
    return increments ? tvs_pk_m<dp, true>(M, Z, lt, t, d, Ft, n, l, out, Zp, rbf, state, s)    \
                      : tvs_pk_m<dp, false>(M, Z, lt, t, d, Ft, n, l, out, Zp, rbf, state, s);
  switch (DP) {
    GPSIG_TVS(1) GPSIG_TVS(2) GPSIG_TVS(3) GPSIG_TVS(4) GPSIG_TVS(5) GPSIG_TVS(6) GPSIG_TVS(7) GPSIG_TVS(8)
    default: return -1;
  }
#undef GPSIG_TVS
}

size_t tvs_pk_zp_bytes(int lt, int t, int d) {
  // the packed paths' (T, LT, ZS) buffer (d <= 8) or the wide kernels' (T, 2d + 1, LT) one
  const int DP = d <= 2 ? 2 : d <= 4 ? 4 : d <= 6 ? 6 : d <= 8 ? 8 : d;
  return ((size_t)lt * t * ((2 * DP + 2)) * sizeof(float) + 255) & ~(size_t)255;
}

}  // namespace gpsig
