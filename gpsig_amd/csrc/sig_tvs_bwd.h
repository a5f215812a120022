// gpsig_amd -- gradient (vector-Jacobian product) of the inducing-tensor vs sequence kernel on gfx950.
//
// Forward (restated from signature_algs.py:101-127 with the seeds of kernels.py:314-341): for tensor
// t, sequence n and level i with components c_1..c_i = k0 .. k0+i-1 (k0 = i(i-1)/2),
//   M_k(s) = P_k(s+1) - P_k(s),  P_k(s) = k(z_k, x_s)  [increments: k(z1_k, x_s) - k(z0_k, x_s)]
//   R_1 = M_{c_1},  R_j(s) = M_{c_j}(s) A_{j-1}(s),  A_j(s) = sum_{s'<s} R_j(s'),  K_i = sum_s R_i(s).
// The reference gets dK/dZ, dK/dX from TF autodiff of the materialised (LT, T, N, L) tensor.  Here one
// lane owns one (t, n) pair (64 sequences per wave, the tensor wave-uniform as in the forward kernels):
//   * a forward sweep over time gives the end state A_j(L-1);
//   * a reverse sweep recovers A_j(s) by inverting the update (A_j -= M A_{j-1}, ascending j) and carries
//     the adjoints Q_j(s) = sum_{s'>s} M_{c_{j+1}}(s') Q_{j+1}(s'), Q_i = g_i = dLoss/dK_i, so that
//     dLoss/dM_{c_j}(s) = Q_j(s) A_{j-1}(s);
//   * the adjoint of the time difference gives dLoss/dP_k(s), and the base kernel's derivative
//     (RBF: k (x - z) for z, k (z - x) for x; linear: x, z) the point gradients: the sequence's are
//     added per time step (time-major, coalesced across lanes), the tensor's accumulate in registers
//     and are reduced over the wave at the end.
// A workgroup is NW waves = NW tensors on the same 64 sequences: the per-step sequence gradients of
// the NW tensors are summed through LDS and added with one atomic per (time, channel, sequence).  One
// atomic per tensor before: T * N * L * d * M of them (1.3e9 at T = 512, N = 1024, L = 100, d = 5,
// M = 5), which at the chip's ~1.3 TB/s of atomic adds was most of the VJP's time.
// Cells use one exp per component and time step (both sweeps evaluate the same instructions, so the
// inversion only carries the fp32 rounding of the forward sums).
#pragma once
#include "sig_common.h"

namespace gpsig {

struct TvsBwdArgs {
  const float *Z;     // (LT, T, d) or (LT, T, 2, d)
  const float *Ft;    // time-major features Ft[(s * FC + c) * n + seq], FC = 2d + 3: x | dx | hdx | g | hx
  int t, n, l, d;
  const float *gout;  // (M+1, T, n) dLoss/dK_m (raw levels)
  float *gZ;          // like Z, accumulated
  float *gXt;         // (l, d, n) time-major, accumulated
  const float *state; // optional (T, n, LT) end-of-sweep running sums of the forward (gpsig_tens_vs_seq_state):
                      // the forward sweep is skipped
};

// waves (tensors) per workgroup of the VJP
template <int DP, bool INCR>
constexpr int tvs_bwd_waves() { return (DP <= 6 && !INCR) ? 8 : 4; }
// time steps per staged chunk of the sequence records (x, dx, g of the workgroup's 64 sequences): 4 keeps
// the 8-wave workgroups at two per CU (4 waves/SIMD); the register-bound increments variants (one wave
// per SIMD) take 8 steps of prefetch distance
template <int DP, bool INCR>
constexpr int tvs_bwd_chunk() { return DP > 8 ? 2 : (INCR ? 8 : 4); }

// reverse-sweep steps between exact point values of the RBF difference cells (backward recurrence)
constexpr int TVSB_ANCHOR = 32;

// Level I only (levels are independent chains; blockIdx.z selects the level, so the per-lane state is
// O(I * DP) and not O(M^2 * DP)).  LT below is the number of components of this level.
// DIFF = false (difference=False): the cells are the point values P_k(s) themselves, s = 0..L-1.
template <int DP, int I, int MMAX, bool INCR, bool RBF, bool DIFF>
__device__ __forceinline__ void tvs_bwd_level(const TvsBwdArgs &a,
                                              float (&zl_all)[tvs_bwd_waves<DP, INCR>()][MMAX * 2 * DP],
                                              float (&red)[2][tvs_bwd_waves<DP, INCR>()][DP][64],
                                              float (&stg)[2][tvs_bwd_chunk<DP, INCR>() + 1][2 * DP + 1][64]) {
  constexpr int LT = I;
  constexpr int NW = tvs_bwd_waves<DP, INCR>();
  constexpr int KB = I * (I - 1) / 2;  // first component of the level
  constexpr float NHL2E = -0.72134752044448170f;  // exp(-d2/2) = exp2(d2 * NHL2E)
  constexpr float L2E = 1.4426950408889634f;
  const int lane = threadIdx.x & 63;
  const int wave = wave_uniform(threadIdx.x >> 6);
  const int n = a.n, d = a.d, FC = 2 * d + 3, T = a.t, L = a.l;
  const int tt0 = blockIdx.y * NW + wave;
  const bool tvalid = tt0 < T;  // wave-uniform; an idle wave still takes part in every barrier
  const int tt = tvalid ? tt0 : T - 1;
  const int s0 = blockIdx.x * 64 + lane;
  const bool valid = s0 < n;
  const int sq = valid ? s0 : n - 1;
  const int zs = INCR ? 2 * d : d;
  // the level's components of this wave's tensor, staged in LDS: broadcast reads instead of the
  // serialised L2-latency vector loads the compiler emits for uniform global data it cannot prove
  // invariant
  float *zl = zl_all[wave];
  for (int e = lane; e < I * 2 * DP; e += 64) {
    const int c = e / (2 * DP), h = (e / DP) % 2, q = e % DP;
    zl[e] = (q < d && (INCR || h == 0)) ? a.Z[((long long)(KB + c) * T + tt) * zs + h * d + q] : 0.f;
  }
  // red: per-step sequence gradients of the NW tensors, summed over the workgroup (double buffered:
  // one barrier per step)
  int rbuf = 0;
  __syncthreads();
  // component c of the level (global component KB + c)
  auto z0c = [&](int c, int q) -> float { return zl[(c * 2) * DP + q]; };
  auto z1c = [&](int c, int q) -> float { return zl[(c * 2 + 1) * DP + q]; };
  // Sequence records staged through LDS: the workgroup's NW waves share the same 64 sequences, so
  // each (step, channel) row of 64 floats is fetched once per workgroup by one global_load_lds (an
  // LDS-DMA, no registers), a chunk of CS steps ahead of its use.  stg[buf][step - c0][slot][lane]:
  // slots 0..DP-1 = x, DP..2DP-1 = dx, 2DP = g (padded channels are zeroed once, never loaded).
  constexpr int CS = tvs_bwd_chunk<DP, INCR>();
  const int NCH = 2 * d + 1;
  for (int e = (int)threadIdx.x; e < 2 * (CS + 1) * 2 * DP * 64; e += NW * 64) {
    const int l = e & 63, r = e >> 6, slot = r % (2 * DP), si = (r / (2 * DP)) % (CS + 1), b = r / (2 * DP * (CS + 1));
    if (slot % DP >= d) stg[b][si][slot][l] = 0.f;
  }
  // stage steps c0 .. c0 + CS (clamped to the sequence) into stg[buf]
  auto stage = [&](int buf, int c0) {
    for (int r = wave; r < (CS + 1) * NCH; r += NW) {
      const int si = r / NCH, ch = r % NCH;
      int st = c0 + si;
      st = st < 0 ? 0 : (st < L ? st : L - 1);
      const int slot = ch < d ? ch : (ch < 2 * d ? DP + ch - d : 2 * DP);
      const int gch = ch < 2 * d ? ch : 2 * d + 1;
      __builtin_amdgcn_global_load_lds(a.Ft + ((long long)st * FC + gch) * n + sq,
                                       (__attribute__((address_space(3))) void *)&stg[buf][si][slot][0], 4, 0, 0);
    }
  };
  auto ldx = [&](const float (*row)[64], float (&x)[DP]) {
#pragma unroll
    for (int q = 0; q < DP; ++q) x[q] = row[q][lane];
  };
  auto lddx = [&](const float (*row)[64], float (&dx)[DP]) {
#pragma unroll
    for (int q = 0; q < DP; ++q) dx[q] = row[DP + q][lane];
  };
  auto em1 = [&](float v) -> float {
    return __builtin_fabsf(v) < EM1_TAU ? em1_small(v) : __builtin_amdgcn_exp2f(v * L2E) - 1.0f;
  };
  // point values of component k at x: RBF k(z0, x) [and k(z1, x)]
  auto pvals = [&](int k, const float (&x)[DP], float &v0, float &v1) {
    if constexpr (RBF) {
      float e0 = 0.f, e1 = 0.f;
#pragma unroll
      for (int q = 0; q < DP; ++q) {
        const float d0 = z0c(k, q) - x[q];
        e0 = __builtin_fmaf(d0, d0, e0);
        if constexpr (INCR) {
          const float d1 = z1c(k, q) - x[q];
          e1 = __builtin_fmaf(d1, d1, e1);
        }
      }
      v0 = __builtin_amdgcn_exp2f(e0 * NHL2E);
      v1 = INCR ? __builtin_amdgcn_exp2f(e1 * NHL2E) : 0.f;
    } else {
      v0 = v1 = 0.f;
    }
  };
  // cell M_k(s) from x_s, dx_s, g_s and the point values at s (c0, c1) and s+1 (n0, n1)
  auto cell = [&](int k, const float (&x)[DP], const float (&dx)[DP], float gs, float c0, float c1, float n0,
                  float n1) -> float {
    if constexpr (!RBF) {
      float v = 0.f;
#pragma unroll
      for (int q = 0; q < DP; ++q) v = __builtin_fmaf(INCR ? z1c(k, q) - z0c(k, q) : z0c(k, q), dx[q], v);
      return v;
    } else if constexpr (!INCR) {
      // k(z, x_{s+1}) - k(z, x_s) = k(z, x_s) expm1(<z, dx> - g)
      float qv = -gs;
#pragma unroll
      for (int q = 0; q < DP; ++q) qv = __builtin_fmaf(z0c(k, q), dx[q], qv);
      (void)n0;
      return c0 * em1(qv);
    } else {
      float p = 0.f, qv = -gs, c = 0.f, hdz = 0.f;
#pragma unroll
      for (int q = 0; q < DP; ++q) {
        const float z0 = z0c(k, q), dz = z1c(k, q) - z0;
        p = __builtin_fmaf(x[q] - z0, dz, p);
        qv = __builtin_fmaf(z0, dx[q], qv);
        c = __builtin_fmaf(dz, dx[q], c);
        hdz = __builtin_fmaf(dz, dz, hdz);
      }
      p = __builtin_fmaf(-0.5f, hdz, p);
      const float mx = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(p), __builtin_fabsf(qv)), __builtin_fabsf(c));
      if (mx < EM1_TAU) {
        const float Ep = em1_small(p), Eq = em1_small(qv), Ec = em1_small(c);
        return c0 * __builtin_fmaf(Ep, Eq, (1.0f + Ep) * (1.0f + Eq) * Ec);
      }
      return (n1 - n0) - (c1 - c0);
    }
  };

  const float gI = (valid && tvalid) ? a.gout[((long long)I * T + tt) * n + sq] : 0.f;

  // ---- forward sweep: end state of the running sums A (index k0 + j - 1 for A_j of level i)
  float A[LT], pv0[LT], pv1[LT];
#pragma unroll
  for (int k = 0; k < LT; ++k) A[k] = 0.f;
  // point value P_k at x (difference=False cell): RBF k(z0, x) [k(z1, x) - k(z0, x)], linear <z, x>
  auto pcell = [&](int k, const float (&x)[DP], float v0, float v1) -> float {
    if constexpr (RBF) {
      return INCR ? v1 - v0 : v0;
    } else {
      float v = 0.f;
#pragma unroll
      for (int q = 0; q < DP; ++q) v = __builtin_fmaf(INCR ? z1c(k, q) - z0c(k, q) : z0c(k, q), x[q], v);
      return v;
    }
  };
  const int nfs = a.state ? 0 : (DIFF ? L - 1 : L);  // forward steps (none from the saved state)
  int buf = 0;
  if (a.state) {
    // the forward launch's end state: A_j(L-1) of this level's stages (global components KB + j - 1)
    const float *st = a.state + ((long long)tt * n + sq) * (MMAX * (MMAX + 1) / 2) + KB;
#pragma unroll
    for (int k = 0; k + 1 < LT; ++k) A[k] = st[k];
  } else {
    stage(0, 0);
  }
  for (int c0 = 0; c0 < nfs; c0 += CS) {
    __syncthreads();  // this chunk has landed (vmcnt(0)); the other buffer is free
    if (c0 + CS < nfs) stage(buf ^ 1, c0 + CS);
    const int ce = c0 + CS < nfs ? c0 + CS : nfs;
    if constexpr (DIFF) {
      if (c0 == 0) {
        float x0[DP];
        ldx(stg[buf][0], x0);
#pragma unroll
        for (int k = 0; k < LT; ++k) pvals(k, x0, pv0[k], pv1[k]);
      }
      for (int s = c0; s < ce; ++s) {
        float x[DP], dx[DP], xn[DP];
        ldx(stg[buf][s - c0], x);
        lddx(stg[buf][s - c0], dx);
        ldx(stg[buf][s - c0 + 1], xn);
        const float gs = stg[buf][s - c0][2 * DP][lane];
        float prev = 0.f;
#pragma unroll
        for (int k = 0; k < I; ++k) {
          float n0, n1;
          pvals(k, xn, n0, n1);
          const float m = cell(k, x, dx, gs, pv0[k], pv1[k], n0, n1);
          pv0[k] = n0;
          pv1[k] = n1;
          if (k == 0) {
            prev = m;
          } else {
            const float as = A[k - 1];
            A[k - 1] = as + prev;
            prev = m * as;
          }
        }
      }
    } else {
      for (int s = c0; s < ce; ++s) {
        float x[DP];
        ldx(stg[buf][s - c0], x);
        float prev = 0.f;
#pragma unroll
        for (int k = 0; k < I; ++k) {
          float v0, v1;
          pvals(k, x, v0, v1);
          const float m = pcell(k, x, v0, v1);
          if (k == 0) {
            prev = m;
          } else {
            const float as = A[k - 1];
            A[k - 1] = as + prev;
            prev = m * as;
          }
        }
      }
    }
    buf ^= 1;
  }

  // ---- reverse sweep
  float Acc[LT], Mh[LT];  // adjoint running sums (same indexing as A), dLoss/dM_k at the previous step
  float S0[LT], S1[LT], V0[LT][DP], V1[LT][DP];
#pragma unroll
  for (int k = 0; k < LT; ++k) {
    Acc[k] = 0.f;
    Mh[k] = 0.f;
    S0[k] = S1[k] = 0.f;
#pragma unroll
    for (int q = 0; q < DP; ++q) V0[k][q] = V1[k][q] = 0.f;
  }
  // point s' receives dLoss/dP_k(s') = Ph for every component k (point values v0, v1 at s')
  // (xp = x at s', kept from the sweep: no load here, so the atomics below never sit in front of a
  // load the next step waits for)
  auto emit = [&](int sp, const float (&Ph)[LT], const float (&v0)[LT], const float (&v1)[LT],
                  const float (&xp)[DP]) {
    float gxa[DP], gxs = 0.f;
#pragma unroll
    for (int q = 0; q < DP; ++q) gxa[q] = 0.f;
#pragma unroll
    for (int k = 0; k < LT; ++k) {
      if constexpr (RBF) {
        const float w0 = INCR ? -Ph[k] * v0[k] : Ph[k] * v0[k];
        S0[k] += w0;
        gxs += w0;
#pragma unroll
        for (int q = 0; q < DP; ++q) {
          V0[k][q] = __builtin_fmaf(w0, xp[q], V0[k][q]);
          gxa[q] = __builtin_fmaf(w0, z0c(k, q), gxa[q]);
        }
        if constexpr (INCR) {
          const float w1 = Ph[k] * v1[k];
          S1[k] += w1;
          gxs += w1;
#pragma unroll
          for (int q = 0; q < DP; ++q) {
            V1[k][q] = __builtin_fmaf(w1, xp[q], V1[k][q]);
            gxa[q] = __builtin_fmaf(w1, z1c(k, q), gxa[q]);
          }
        }
      } else {
#pragma unroll
        for (int q = 0; q < DP; ++q) {
          V0[k][q] = __builtin_fmaf(Ph[k], xp[q], V0[k][q]);
          gxa[q] = __builtin_fmaf(Ph[k], INCR ? z1c(k, q) - z0c(k, q) : z0c(k, q), gxa[q]);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < DP; ++q) red[rbuf][wave][q][lane] = RBF ? __builtin_fmaf(-gxs, xp[q], gxa[q]) : gxa[q];
    // LDS writes done, then the barrier; no vmcnt wait, so the staged chunk's LDS-DMA stays in flight
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    // the workgroup's sum for (point sp, channel q, sequence) from one thread each
    for (int e = (int)threadIdx.x; e < DP * 64; e += NW * 64) {
      const int q = e >> 6, l = e & 63, sqn = (int)blockIdx.x * 64 + l;
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) v += red[rbuf][w][q][l];
      if (q < d && sqn < n) unsafeAtomicAdd(a.gXt + ((long long)sp * d + q) * n + sqn, v);
    }
    rbuf ^= 1;
  };

  // reverse sweep in chunks of CS steps (descending), each staged one chunk ahead: the chunk with top
  // step hi holds steps hi - CS + 1 .. hi + 1 (x at s + 1 for the difference cells)
  const int stop = DIFF ? L - 2 : L - 1;  // last row of the grid the recursion consumes
  float xs1[DP];  // x at s + 1
  __syncthreads();  // every wave is done with the forward sweep's buffers
  stage(buf, stop - CS + 1);
  for (int hi = stop; hi >= 0; hi -= CS) {
    __syncthreads();  // this chunk has landed; the other buffer is free
    const int c0 = hi - CS + 1;
    if (hi - CS >= 0) stage(buf ^ 1, c0 - CS);
    const int lo = c0 > 0 ? c0 : 0;
    if (hi == stop) {
      ldx(stg[buf][stop + 1 - c0], xs1);
      if constexpr (DIFF) {
        // point values at the last point (left there by the forward sweep, evaluated here from the state)
        if (a.state) {
#pragma unroll
          for (int k = 0; k < LT; ++k) pvals(k, xs1, pv0[k], pv1[k]);
        }
      }
    }
    for (int s = hi; s >= lo; --s) {
    float x[DP], dx[DP];
    ldx(stg[buf][s - c0], x);
    lddx(stg[buf][s - c0], dx);
    const float gs = stg[buf][s - c0][2 * DP][lane];
    float c0v[LT], c1v[LT], Ph[LT];
    {
      constexpr int i = I, k0 = 0;
      float m[I], Av[I];
      // RBF difference cells without increments: k(z, x_s) = k(z, x_{s+1}) / (1 + expm1(q_s)) from the cell's
      // own expm1 (no exp, no distance), re-anchored exactly every TVSB_ANCHOR steps (wave-uniform)
      constexpr bool BACKREC = RBF && DIFF && !INCR;
      const bool anchor = !BACKREC || (s % TVSB_ANCHOR) == 0 || s == stop;
#pragma unroll
      for (int st = 0; st < i; ++st) {
        const int k = k0 + st;
        if constexpr (BACKREC) {
          float qv = -gs;
#pragma unroll
          for (int q = 0; q < DP; ++q) qv = __builtin_fmaf(z0c(k, q), dx[q], qv);
          const float E = em1(qv);
          // far from the polynomial range (|q| >= EM1_TAU in some lane) 1 + expm1(q) loses digits or
          // underflows to 0 (q < -17.3): the step takes the exact point values instead (wave-uniform)
          if (anchor || __builtin_amdgcn_ballot_w64(!(__builtin_fabsf(qv) < EM1_TAU)) != 0) pvals(k, x, c0v[k], c1v[k]);
          else c0v[k] = pv0[k] * __builtin_amdgcn_rcpf(1.0f + E);
          c1v[k] = 0.f;
          m[st] = c0v[k] * E;
        } else {
          pvals(k, x, c0v[k], c1v[k]);
          m[st] = DIFF ? cell(k, x, dx, gs, c0v[k], c1v[k], pv0[k], pv1[k]) : pcell(k, x, c0v[k], c1v[k]);
        }
      }
      // A_j(s) = A_j(s+1) - M_{c_j}(s) A_{j-1}(s), ascending j (A_0 = 1)
      Av[0] = 1.0f;
#pragma unroll
      for (int j = 1; j < i; ++j) {
        A[k0 + j - 1] = __builtin_fmaf(-m[j - 1], Av[j - 1], A[k0 + j - 1]);
        Av[j] = A[k0 + j - 1];
      }
      // dLoss/dM_{c_j}(s) = Q_j(s) A_{j-1}(s), Q_i = g_i, Q_j = Acc (sum over s' > s)
#pragma unroll
      for (int j = 1; j <= i; ++j) {
        const float Q = (j < i) ? Acc[k0 + j - 1] : gI;
        const float mh = Q * Av[j - 1];
        const int k = k0 + j - 1;
        Ph[k] = DIFF ? mh - Mh[k] : mh;  // dLoss/dP_k(s+1) = dM_k(s) - dM_k(s+1) [P_k(s) = M_k(s)]
        Mh[k] = mh;
      }
      // Q_j(s-1) = Q_j(s) + M_{c_{j+1}}(s) Q_{j+1}(s), ascending j (old Q_{j+1})
#pragma unroll
      for (int j = 1; j < i; ++j) {
        const float Qn = (j + 1 < i) ? Acc[k0 + j] : gI;
        Acc[k0 + j - 1] = __builtin_fmaf(m[j], Qn, Acc[k0 + j - 1]);
      }
    }
    if constexpr (DIFF)
      emit(s + 1, Ph, pv0, pv1, xs1);
    else
      emit(s, Ph, c0v, c1v, x);
#pragma unroll
    for (int k = 0; k < LT; ++k) {
      pv0[k] = c0v[k];
      pv1[k] = c1v[k];
    }
#pragma unroll
    for (int q = 0; q < DP; ++q) xs1[q] = x[q];
    }
    buf ^= 1;
  }
  if constexpr (DIFF) {
    float Ph[LT];
#pragma unroll
    for (int k = 0; k < LT; ++k) Ph[k] = -Mh[k];
    emit(0, Ph, pv0, pv1, xs1);
  }

  // ---- tensor gradients: reduce over the wave's sequences, one atomic per component channel
  const int zoff1 = INCR ? d : 0;
#pragma unroll
  for (int k = 0; k < LT; ++k) {
    float r[2 * DP + 2];
#pragma unroll
    for (int q = 0; q < DP; ++q) {
      r[q] = V0[k][q];
      r[DP + q] = V1[k][q];
    }
    r[2 * DP] = S0[k];
    r[2 * DP + 1] = S1[k];
    group_incl_scan_n<64, 2 * DP + 2>(r);
    if (lane == 63 && tvalid) {
      float *gz = a.gZ + ((long long)(KB + k) * T + tt) * zs;
      for (int q = 0; q < d; ++q) {
        if constexpr (RBF) {
          unsafeAtomicAdd(gz + q, __builtin_fmaf(-r[2 * DP], z0c(k, q), r[q]));
          if constexpr (INCR) unsafeAtomicAdd(gz + zoff1 + q, __builtin_fmaf(-r[2 * DP + 1], z1c(k, q), r[DP + q]));
        } else if constexpr (INCR) {
          unsafeAtomicAdd(gz + zoff1 + q, r[q]);
          unsafeAtomicAdd(gz + q, -r[q]);
        } else {
          unsafeAtomicAdd(gz + q, r[q]);
        }
      }
    }
  }
}

template <int DP, int M, bool INCR, bool RBF, bool DIFF>
__global__ __launch_bounds__((64 * tvs_bwd_waves<DP, INCR>())) void tvs_bwd_kernel(TvsBwdArgs a) {
  // one LDS allocation for every level's body (declared per level, they would all be allocated)
  constexpr int NW = tvs_bwd_waves<DP, INCR>();
  __shared__ float zl_all[NW][M * 2 * DP];
  __shared__ float red[2][NW][DP][64];
  __shared__ float stg[2][tvs_bwd_chunk<DP, INCR>() + 1][2 * DP + 1][64];
  switch (blockIdx.z) {
    case 0: tvs_bwd_level<DP, 1, M, INCR, RBF, DIFF>(a, zl_all, red, stg); break;
    case 1: if constexpr (M >= 2) tvs_bwd_level<DP, 2, M, INCR, RBF, DIFF>(a, zl_all, red, stg); break;
    case 2: if constexpr (M >= 3) tvs_bwd_level<DP, 3, M, INCR, RBF, DIFF>(a, zl_all, red, stg); break;
    case 3: if constexpr (M >= 4) tvs_bwd_level<DP, 4, M, INCR, RBF, DIFF>(a, zl_all, red, stg); break;
    case 4: if constexpr (M >= 5) tvs_bwd_level<DP, 5, M, INCR, RBF, DIFF>(a, zl_all, red, stg); break;
    case 5: if constexpr (M >= 6) tvs_bwd_level<DP, 6, M, INCR, RBF, DIFF>(a, zl_all, red, stg); break;
    case 6: if constexpr (M >= 7) tvs_bwd_level<DP, 7, M, INCR, RBF, DIFF>(a, zl_all, red, stg); break;
    case 7: if constexpr (M >= 8) tvs_bwd_level<DP, 8, M, INCR, RBF, DIFF>(a, zl_all, red, stg); break;
    default: break;
  }
}

}  // namespace gpsig
