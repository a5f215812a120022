// gpsig_amd -- inducing-tensor kernels on gfx950:
//   gpsig_tens_vs_seq : _K_tens_vs_seq (gpsig/kernels.py:314-341) + signature_kern_tens_vs_seq_{first,
//                       higher}_order (gpsig/signature_algs.py:101-160)
//   gpsig_tens_gram   : _K_tens (kernels.py:264-284) + tensor_kern (signature_algs.py:76-99)
//   gpsig_rescaled    : _Mahalanobis_term_approx_posterior (kernels.py:800-822, kernels_pde.py:191-222)
//                       + signature_kern_rescaled_higher_order (signature_algs_vosf.py:11-48)
//
// tens_vs_seq: lanes = sequences (64 per wave), the wave's tensor t is uniform, so the tensor
// components stream through the scalar cache while the sequence data is read time-major
// (coalesced across lanes) from a feature buffer built per call.  Each lane streams its sequence in
// time with O(num_levels^2) running sums; nothing (LT, T, N, L)-sized is materialised.
#include "sig_common.h"

namespace gpsig {

constexpr int TV_MMAX = 8;

// time-major sequence features: Ft[(l * FC + c) * n + s], c in [x (d) | dx (d) | |dx|^2/2 | <x,dx>+|dx|^2/2 | |x|^2/2]
__global__ __launch_bounds__(256) void tvs_features_kernel(const float *__restrict__ X, int n, int l, int d,
                                                           float *__restrict__ Ft) {
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long long)n * l) return;
  const int s = (int)(idx / l), i = (int)(idx % l);
  const float *x = X + idx * d;
  const int FC = 2 * d + 3;
  float hdx = 0.f, hx = 0.f;
  double xdx = 0.0;  // g = <x, dx> + |dx|^2/2 accumulated in fp64, rounded once
  for (int k = 0; k < d; ++k) {
    const float xv = x[k];
    const float dv = (i + 1 < l) ? x[d + k] - xv : 0.0f;
    Ft[((long long)i * FC + k) * n + s] = xv;
    Ft[((long long)i * FC + d + k) * n + s] = dv;
    hdx = __builtin_fmaf(dv, dv, hdx);
    xdx = __builtin_fma((double)xv, (double)dv, xdx);
    hx = __builtin_fmaf(xv, xv, hx);
  }
  Ft[((long long)i * FC + 2 * d) * n + s] = 0.5f * hdx;
  Ft[((long long)i * FC + 2 * d + 1) * n + s] = (float)(xdx + 0.5 * (double)hdx);
  Ft[((long long)i * FC + 2 * d + 2) * n + s] = 0.5f * hx;
}

// Second difference k(a+da, b+db) - k(a+da, b) - k(a, b+db) + k(a, b) of the RBF kernel for general
// vectors (fp32-stable form when |p|,|q|,|c| < EM1_TAU, corner form otherwise; see RowSeed).
template <int DP>
GPSIG_DEV float rbf_second_diff(const float (&a)[DP], const float (&da)[DP], const float (&b)[DP],
                                const float (&db)[DP]) {
  // padded channels hold zeros in all four vectors and contribute nothing
  float diff2 = 0.f, p = 0.f, q = 0.f, c = 0.f, hda = 0.f, hdb = 0.f;
  float d11 = 0.f, d10 = 0.f, d01 = 0.f;
#pragma unroll
  for (int k = 0; k < DP; ++k) {
    const float df = a[k] - b[k];
    diff2 = __builtin_fmaf(df, df, diff2);
    p = __builtin_fmaf(-df, da[k], p);
    q = __builtin_fmaf(df, db[k], q);
    c = __builtin_fmaf(da[k], db[k], c);
    hda = __builtin_fmaf(da[k], da[k], hda);
    hdb = __builtin_fmaf(db[k], db[k], hdb);
    const float e11 = df + da[k] - db[k], e10 = df + da[k], e01 = df - db[k];
    d11 = __builtin_fmaf(e11, e11, d11);
    d10 = __builtin_fmaf(e10, e10, d10);
    d01 = __builtin_fmaf(e01, e01, d01);
  }
  p -= 0.5f * hda;
  q -= 0.5f * hdb;
  const float k00 = fast_exp(-0.5f * diff2);
  const float mx = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(p), __builtin_fabsf(q)), __builtin_fabsf(c));
  if (mx < EM1_TAU) {
    const float Ep = em1_small(p), Eq = em1_small(q), Ec = em1_small(c);
    return k00 * __builtin_fmaf(Ep, Eq, (1.0f + Ep) * (1.0f + Eq) * Ec);
  }
  return (fast_exp(-0.5f * d11) - fast_exp(-0.5f * d10)) - (fast_exp(-0.5f * d01) - k00);
}

// The same second difference for a runtime channel count; av/dav/bv/dbv(q) return channel q of a, da, b, db.
template <class FA, class FDA, class FB, class FDB>
GPSIG_DEV float rbf_second_diff_rt(int d, FA av, FDA dav, FB bv, FDB dbv) {
  float diff2 = 0.f, p = 0.f, q = 0.f, c = 0.f, hda = 0.f, hdb = 0.f;
  float d11 = 0.f, d10 = 0.f, d01 = 0.f;
  for (int k = 0; k < d; ++k) {
    const float a = av(k), da = dav(k), b = bv(k), db = dbv(k);
    const float df = a - b;
    diff2 = __builtin_fmaf(df, df, diff2);
    p = __builtin_fmaf(-df, da, p);
    q = __builtin_fmaf(df, db, q);
    c = __builtin_fmaf(da, db, c);
    hda = __builtin_fmaf(da, da, hda);
    hdb = __builtin_fmaf(db, db, hdb);
    const float e11 = df + da - db, e10 = df + da, e01 = df - db;
    d11 = __builtin_fmaf(e11, e11, d11);
    d10 = __builtin_fmaf(e10, e10, d10);
    d01 = __builtin_fmaf(e01, e01, d01);
  }
  p -= 0.5f * hda;
  q -= 0.5f * hdb;
  const float k00 = fast_exp(-0.5f * diff2);
  const float mx = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(p), __builtin_fabsf(q)), __builtin_fabsf(c));
  if (mx < EM1_TAU) {
    const float Ep = em1_small(p), Eq = em1_small(q), Ec = em1_small(c);
    return k00 * __builtin_fmaf(Ep, Eq, (1.0f + Ep) * (1.0f + Eq) * Ec);
  }
  return (fast_exp(-0.5f * d11) - fast_exp(-0.5f * d10)) - (fast_exp(-0.5f * d01) - k00);
}

// ------------------------------------------------------------------------------------ tens vs seq
struct TvsArgs {
  const float *Z;  // (LT, T, [2,] d)
  const float *Ft; // time-major features
  int lt, t, n, l, d, M, order, incr, diff, rbf;
  float *out;      // (M+1, T, n)
};

// Per-time-cell data of this lane's sequence (loaded once per cell, shared by all components).
template <int DP>
struct TvsCell {
  float x[DP], dx[DP], xn[DP], beta;
};

// Seed of component k at time cell pt: the base-kernel value k(z_k, x_pt) (difference=False) or its
// time difference k(z_k, x_{pt+1}) - k(z_k, x_pt) (difference=True, signature_algs.py:114); with
// increments the component is the pair (z0, z1) and M = k(z1, x) - k(z0, x) (kernels.py:328-331).
// kc carries k(z_k, x_pt) across cells for the RBF DIFF seed.
// zs: this tensor's components staged in LDS, component k at zs + k * (incr ? 2d : d).
template <int DP>
GPSIG_DEV float tvs_seed(const TvsArgs &a, const float *zs, int k, const TvsCell<DP> &cl, float &kc) {
  const int d = a.d;
  const float *zt = zs + k * (a.incr ? 2 * d : d);
  if (!a.rbf) {
    float v = 0.f;
#pragma unroll
    for (int q = 0; q < DP; ++q) {
      if (q < d) {
        const float zq = a.incr ? zt[d + q] - zt[q] : zt[q];
        v = __builtin_fmaf(zq, a.diff ? cl.dx[q] : cl.x[q], v);
      }
    }
    return v;
  }
  if (!a.incr) {
    if (!a.diff) {
      float s2 = 0.f;
#pragma unroll
      for (int q = 0; q < DP; ++q)
        if (q < d) {
          const float df = zt[q] - cl.x[q];
          s2 = __builtin_fmaf(df, df, s2);
        }
      return fast_exp(-0.5f * s2);
    }
    // k(z, x_{pt+1}) - k(z, x_pt) = k(z, x_pt) em1(<z - x_pt, dx> - |dx|^2/2) (stable) or corners
    float s2 = 0.f, zdx = 0.f;
#pragma unroll
    for (int q = 0; q < DP; ++q)
      if (q < d) {
        const float df = zt[q] - cl.xn[q];
        s2 = __builtin_fmaf(df, df, s2);
        zdx = __builtin_fmaf(zt[q], cl.dx[q], zdx);
      }
    const float kn = fast_exp(-0.5f * s2);
    const float qv = zdx - cl.beta;
    const float kcur = kc;
    kc = kn;
    return __builtin_fabsf(qv) < EM1_TAU ? kcur * em1_small(qv) : kn - kcur;
  }
  if (!a.diff) {
    float s0 = 0.f, s1 = 0.f;
#pragma unroll
    for (int q = 0; q < DP; ++q)
      if (q < d) {
        const float e0 = zt[q] - cl.x[q], e1 = zt[d + q] - cl.x[q];
        s0 = __builtin_fmaf(e0, e0, s0);
        s1 = __builtin_fmaf(e1, e1, s1);
      }
    return fast_exp(-0.5f * s1) - fast_exp(-0.5f * s0);
  }
  float z0[DP], dz[DP];
#pragma unroll
  for (int q = 0; q < DP; ++q) {
    z0[q] = q < d ? zt[q] : 0.f;
    dz[q] = q < d ? zt[d + q] - zt[q] : 0.f;
  }
  return rbf_second_diff<DP>(z0, dz, cl.x, cl.dx);
}

// tvs_seed for a runtime channel count (DP == 0 instantiation): the cell's channels are read from the
// time-major features, channel q of x_pt at fr[q n], of x_{pt+1} at fn[q n], of dx_pt at fr[(d + q) n].
GPSIG_DEV float tvs_seed_wide(const TvsArgs &a, const float *zs, int k, const float *fr, const float *fn, float beta,
                              float &kc) {
  const int d = a.d;
  const long long n = a.n;
  const float *zt = zs + k * (a.incr ? 2 * d : d);
  auto xq = [&](int q) { return fr[q * n]; };
  auto dxq = [&](int q) { return fr[(d + q) * n]; };
  if (!a.rbf) {
    float v = 0.f;
    for (int q = 0; q < d; ++q) {
      const float zq = a.incr ? zt[d + q] - zt[q] : zt[q];
      v = __builtin_fmaf(zq, a.diff ? dxq(q) : xq(q), v);
    }
    return v;
  }
  if (!a.incr) {
    if (!a.diff) {
      float s2 = 0.f;
      for (int q = 0; q < d; ++q) {
        const float df = zt[q] - xq(q);
        s2 = __builtin_fmaf(df, df, s2);
      }
      return fast_exp(-0.5f * s2);
    }
    float s2 = 0.f, zdx = 0.f;
    for (int q = 0; q < d; ++q) {
      const float df = zt[q] - fn[q * n];
      s2 = __builtin_fmaf(df, df, s2);
      zdx = __builtin_fmaf(zt[q], dxq(q), zdx);
    }
    const float kn = fast_exp(-0.5f * s2);
    const float qv = zdx - beta;
    const float kcur = kc;
    kc = kn;
    return __builtin_fabsf(qv) < EM1_TAU ? kcur * em1_small(qv) : kn - kcur;
  }
  if (!a.diff) {
    float s0 = 0.f, s1 = 0.f;
    for (int q = 0; q < d; ++q) {
      const float e0 = zt[q] - xq(q), e1 = zt[d + q] - xq(q);
      s0 = __builtin_fmaf(e0, e0, s0);
      s1 = __builtin_fmaf(e1, e1, s1);
    }
    return fast_exp(-0.5f * s1) - fast_exp(-0.5f * s0);
  }
  return rbf_second_diff_rt(
      d, [&](int q) { return zt[q]; }, [&](int q) { return zt[d + q] - zt[q]; }, xq, dxq);
}

// One wave per block; the per-(level, stage) running sums and the carried k values live in this
// lane's LDS column (dynamic indices, no register arrays), the levels' stage chains are plain loops.
// DP == 0: any channel count (tvs_seed_wide reads the cell's channels from the features per component).
template <int DP>
__global__ __launch_bounds__(64) void tvs_kernel(TvsArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int lane = threadIdx.x;
  const int tt = blockIdx.y;
  const int s0 = blockIdx.x * 64 + lane;
  const int s = s0 < a.n ? s0 : a.n - 1;
  const int n = a.n, d = a.d, FC = 2 * d + 3, M = a.M, LT = a.lt;
  float *Ssum = lds + lane;            // Ssum[k * 64]: exclusive-in-time running sums per (level, stage)
  float *kc = lds + 64 * LT + lane;    // kc[k * 64]: RBF DIFF carried k(z_k, x_pt)
  // the wave's tensor (uniform): staged in LDS -- broadcast reads instead of the serialised
  // L2-latency vector loads the compiler emits for uniform global data it cannot prove invariant
  float *zl = lds + 2 * 64 * LT;
  {
    const int zstride = a.incr ? 2 * d : d;
    for (int e = lane; e < LT * zstride; e += 64) {
      const int k = e / zstride, r = e % zstride;
      zl[e] = a.Z[((long long)k * a.t + tt) * zstride + r];
    }
    __syncthreads();
  }
  float K[TV_MMAX + 1];
#pragma unroll
  for (int k = 0; k <= TV_MMAX; ++k) K[k] = 0.f;
  const bool carry = a.rbf && !a.incr && a.diff;
  for (int k = 0; k < LT; ++k) {
    Ssum[k * 64] = 0.f;
    if (carry) {
      const float *zt = a.Z + ((long long)k * a.t + tt) * d;
      float s2 = 0.f;
      for (int q = 0; q < d; ++q) {
        const float df = zt[q] - a.Ft[(long long)q * n + s];
        s2 = __builtin_fmaf(df, df, s2);
      }
      kc[k * 64] = fast_exp(-0.5f * s2);
    }
  }
  const int npts = a.diff ? a.l - 1 : a.l;
  for (int pt = 0; pt < npts; ++pt) {
    TvsCell<DP == 0 ? 1 : DP> cl;
    const float *fr = a.Ft + (long long)pt * FC * n + s;
    const float *fn = fr + (long long)FC * n;
    if constexpr (DP > 0) {
#pragma unroll
      for (int q = 0; q < DP; ++q) {
        cl.x[q] = q < d ? fr[(long long)q * n] : 0.f;
        cl.dx[q] = q < d ? fr[(long long)(d + q) * n] : 0.f;
        cl.xn[q] = (carry && q < d) ? fn[(long long)q * n] : 0.f;
      }
    }
    cl.beta = fr[(long long)(2 * d + 1) * n];
    auto seed = [&](int k, float &kk) -> float {
      if constexpr (DP == 0)
        return tvs_seed_wide(a, zl, k, fr, fn, cl.beta, kk);
      else
        return tvs_seed<DP>(a, zl, k, cl, kk);
    };
    // level i uses components k0 .. k0+i-1 (k0 = i(i-1)/2); stage st runs on component k0+st
    for (int i = 1; i <= M; ++i) {
      const int k0 = i * (i - 1) / 2;
      float kk = kc[k0 * 64];
      const float m0 = seed(k0, kk);
      kc[k0 * 64] = kk;
      if (a.order <= 1) {
        float prev = m0;  // R_0(pt)
        for (int st = 1; st < i; ++st) {
          float kq = kc[(k0 + st) * 64];
          const float mk = seed(k0 + st, kq);
          kc[(k0 + st) * 64] = kq;
          const float ss = Ssum[(k0 + st - 1) * 64];
          Ssum[(k0 + st - 1) * 64] = ss + prev;
          prev = mk * ss;
        }
        K[i] += prev;
      } else {
        // higher order (signature_algs.py:129-160): blocks b < min(st+1, order) of stage st
        float blk[TV_MMAX];
        blk[0] = m0;
#pragma unroll
        for (int b = 1; b < TV_MMAX; ++b) blk[b] = 0.f;
        for (int st = 1; st < i; ++st) {
          const int dn = (st + 1 < a.order) ? st + 1 : a.order;
          float tot = 0.f;
#pragma unroll
          for (int b = 0; b < TV_MMAX; ++b) tot += blk[b];
          float kq = kc[(k0 + st) * 64];
          const float mk = seed(k0 + st, kq);
          kc[(k0 + st) * 64] = kq;
#pragma unroll
          for (int b = TV_MMAX - 1; b >= 1; --b) blk[b] = (b < dn) ? mk * blk[b - 1] / (float)(b + 1) : 0.f;
          const float ss = Ssum[(k0 + st - 1) * 64];
          blk[0] = mk * ss;
          Ssum[(k0 + st - 1) * 64] = ss + tot;
        }
        float tot = 0.f;
#pragma unroll
        for (int b = 0; b < TV_MMAX; ++b) tot += blk[b];
        K[i] += tot;
      }
    }
  }
  if (s0 < a.n) {
    a.out[(long long)tt * a.n + s0] = 1.0f;
#pragma unroll
    for (int i = 1; i <= TV_MMAX; ++i)
      if (i <= M) a.out[((long long)i * a.t + tt) * a.n + s0] = K[i];
  }
}

// ------------------------------------------------------------------------------------ tensor Gram
struct TgArgs {
  const float *Z;
  int lt, t, d, M, incr, rbf;
  float *out;  // (M+1, T, T)
};

// Channel counts up to 32 (DP = 4 .. 32); wider ones run as pair tiles (tens_vjp_mm.hip tens_gram_mm).
template <int DP>
__global__ __launch_bounds__(256) void tens_gram_kernel(TgArgs a) {
  const int t1 = blockIdx.y;
  const int t2 = blockIdx.x * 256 + threadIdx.x;
  if (t2 >= a.t) return;
  const int d = a.d;
  float K[TV_MMAX + 1];
  K[0] = 1.f;
  int k = 0;
  for (int i = 1; i <= a.M; ++i) {
    float prod = 1.f;
    for (int st = 0; st < i; ++st, ++k) {
      float v;
      if (!a.incr) {
        const float *z1 = a.Z + ((long long)k * a.t + t1) * d, *z2 = a.Z + ((long long)k * a.t + t2) * d;
        float s2 = 0.f, ip = 0.f;
        for (int q = 0; q < d; ++q) {
          const float df = z1[q] - z2[q];
          s2 = __builtin_fmaf(df, df, s2);
          ip = __builtin_fmaf(z1[q], z2[q], ip);
        }
        v = a.rbf ? fast_exp(-0.5f * s2) : ip;
      } else {
        // kernels.py:278  M[1,1] + M[0,0] - M[1,0] - M[0,1]
        const float *za = a.Z + (((long long)k * a.t + t1) * 2) * d, *zb = a.Z + (((long long)k * a.t + t2) * 2) * d;
        {
        float A0[DP], dA[DP], B0[DP], dB[DP];
#pragma unroll
        for (int q = 0; q < DP; ++q) {
          A0[q] = q < d ? za[q] : 0.f;
          dA[q] = q < d ? za[d + q] - za[q] : 0.f;
          B0[q] = q < d ? zb[q] : 0.f;
          dB[q] = q < d ? zb[d + q] - zb[q] : 0.f;
        }
        if (a.rbf) {
          v = rbf_second_diff<DP>(A0, dA, B0, dB);
        } else {
          v = 0.f;
          for (int q = 0; q < d; ++q) v = __builtin_fmaf(dA[q], dB[q], v);
        }
        }
      }
      prod = (st == 0) ? v : v * prod;
    }
    K[i] = prod;
  }
  for (int i = 0; i <= a.M; ++i) a.out[((long long)i * a.t + t1) * a.t + t2] = K[i];
}

// ------------------------------------------------------------------------------------ VOSF rescaled
// Per (sequence n, tensor t'): the higher-order 2-D recursion of signature_algs_vosf.py:11-48 on the
// self-Gram of x_n, with stage seeds dM_r(p,q) = sum_d lam_{r,t',d} delta_d(p,q):
//   linear embedding: delta_d = dx_{p,d} dx_{q,d}
//   RBF embedding   : delta_d = second difference of exp(-(x_{p,d} - x_{q,d})^2 / 2)   (kernels_pde.py:191-222)
// t' = T is the "ones" tensor of the concatenation (shared by all t); out = -K(t) + K(ones).
struct RsArgs {
  const float *Z;  // (LT, T, d)
  const float *X;  // (n, l, d)
  int lt, t, n, l, d, M, emb;
  float *out;      // (M+1, n, T)
  float *kones;    // workspace (M, n): K of the ones tensor
};

template <int M, int W, int DP>
__global__ __launch_bounds__(64) void rescaled_kernel(RsArgs a) {
  const int lane = threadIdx.x;
  const int nn = blockIdx.y;
  const int tt = blockIdx.x;  // tt == a.t : the ones tensor
  const int d = a.d, L = a.l;
  const float *x = a.X + (long long)nn * L * d;
  constexpr int LT = M * (M + 1) / 2;
  // DP == 0: any channel count; every stage seed of a row comes from one runtime channel loop (sd below)
  constexpr bool WIDE = DP == 0;
  constexpr int DPA = WIDE ? 1 : DP;
  // lambda of component r for this tensor (wave-uniform), staged in LDS once (the compiler would
  // otherwise emit serialised vector loads for it inside the row loop); the ones tensor of the
  // concatenation (kernels.py:812) is tt == T
  __shared__ float lz[LT * DPA];
  if constexpr (!WIDE) {
    for (int e = lane; e < LT * DP; e += 64) {
      const int r = e / DP, q = e % DP;
      lz[e] = (q < d) ? ((tt < a.t) ? a.Z[((long long)r * a.t + tt) * d + q] : 1.0f) : 0.f;
    }
    __syncthreads();
  }
  auto lam = [&](int r, int q) -> float { return lz[r * DPA + q]; };
  // this lane's columns q0 = lane*W + w
  float xc[W][DPA], dxc[W][DPA];
  bool valid[W];
  int jjw[W];
#pragma unroll
  for (int w = 0; w < W; ++w) {
    const int j = lane * W + w;
    valid[w] = j < L - 1;
    const int jj = j < L - 1 ? j : L - 2;
    jjw[w] = jj;
    if constexpr (!WIDE) {
#pragma unroll
      for (int q = 0; q < DP; ++q) {
        xc[w][q] = q < d ? x[jj * d + q] : 0.f;
        dxc[w][q] = q < d ? x[(jj + 1) * d + q] - x[jj * d + q] : 0.f;
      }
    }
  }
  cfloat *xcst = as_const(x);
  cfloat *zcst = as_const(a.Z);
  // CB[level i][stage s][b]: column running sums over previous rows of sum_a R[s][a][b]
  constexpr int NCB = M * (M + 1) * (M + 2) / 6;  // sum_i sum_{s<i} (s+1)
  float CB[NCB][W];
#pragma unroll
  for (int k = 0; k < NCB; ++k)
#pragma unroll
    for (int w = 0; w < W; ++w) CB[k][w] = 0.f;
  float K[M + 1];
#pragma unroll
  for (int i = 0; i <= M; ++i) K[i] = 0.f;

  for (int pr = 0; pr < L - 1; ++pr) {
    float xr[DPA], dxr[DPA];
    // per-coordinate increments delta_d(pr, col)
    float del[W][DPA];
    // WIDE: every component's stage seed of this row, sd[r][w] = sum_q lam_{r,q} delta_q(pr, col w)
    float sd[WIDE ? LT : 1][W];
    if constexpr (WIDE) {
#pragma unroll
      for (int r = 0; r < LT; ++r)
#pragma unroll
        for (int w = 0; w < W; ++w) sd[r][w] = 0.f;
      for (int q = 0; q < d; ++q) {
        const float xq = xcst[pr * d + q], dxq = xcst[(pr + 1) * d + q] - xq;
        float dl[W];
#pragma unroll
        for (int w = 0; w < W; ++w) {
          const float xw = x[jjw[w] * d + q], dxw = x[(jjw[w] + 1) * d + q] - xw;
          if (a.emb == 0) {
            dl[w] = dxq * dxw;
          } else {
            const float av[1] = {xq}, dav[1] = {dxq}, bv[1] = {xw}, dbv[1] = {dxw};
            dl[w] = rbf_second_diff<1>(av, dav, bv, dbv);
          }
        }
#pragma unroll
        for (int r = 0; r < LT; ++r) {
          const float lq = tt < a.t ? zcst[((long long)r * a.t + tt) * d + q] : 1.0f;
#pragma unroll
          for (int w = 0; w < W; ++w) sd[r][w] = __builtin_fmaf(lq, dl[w], sd[r][w]);
        }
      }
    } else {
#pragma unroll
    for (int q = 0; q < DP; ++q) {
      xr[q] = q < d ? x[pr * d + q] : 0.f;
      dxr[q] = q < d ? x[(pr + 1) * d + q] - x[pr * d + q] : 0.f;
    }
#pragma unroll
    for (int w = 0; w < W; ++w)
#pragma unroll
      for (int q = 0; q < DP; ++q) {
        if (a.emb == 0) {
          del[w][q] = dxr[q] * dxc[w][q];
        } else {
          const float av[1] = {xr[q]}, dav[1] = {dxr[q]}, bv[1] = {xc[w][q]}, dbv[1] = {dxc[w][q]};
          del[w][q] = (q < d) ? rbf_second_diff<1>(av, dav, bv, dbv) : 0.f;
        }
      }
    }
    // stage seed of component r for column w
    auto seedv = [&](int r, int w) -> float {
      if constexpr (WIDE) {
        return sd[r][w];
      } else {
        float sv = 0.f;
#pragma unroll
        for (int q = 0; q < DP; ++q) sv = __builtin_fmaf(lam(r, q), del[w][q], sv);
        return sv;
      }
    };
    int cbo = 0;
#pragma unroll
    for (int i = 1; i <= M; ++i) {
      const int r0 = i * (i - 1) / 2;
      // R[a][b] blocks of the current stage (stage 0 = seed of component r0)
      float R[M][M][W];
#pragma unroll
      for (int x1 = 0; x1 < M; ++x1)
#pragma unroll
        for (int y1 = 0; y1 < M; ++y1)
#pragma unroll
          for (int w = 0; w < W; ++w) R[x1][y1][w] = 0.f;
#pragma unroll
      for (int w = 0; w < W; ++w) R[0][0][w] = valid[w] ? seedv(r0, w) : 0.f;
#pragma unroll
      for (int st = 0; st < i; ++st) {
        const int dm = st + 1;  // blocks of stage st (full order: num_levels >= i)
        float colsum[M][W], rowsum[M][W];
#pragma unroll
        for (int x1 = 0; x1 < M; ++x1)
#pragma unroll
          for (int w = 0; w < W; ++w) {
            float cs = 0.f, rs = 0.f;
#pragma unroll
            for (int y1 = 0; y1 < M; ++y1) {
              if (y1 < dm) cs += R[y1][x1][w];
              if (y1 < dm) rs += R[x1][y1][w];
            }
            colsum[x1][w] = cs;
            rowsum[x1][w] = rs;
          }
        if (st + 1 < i) {
          const int dn = st + 2;
          float seed[W];
#pragma unroll
          for (int w = 0; w < W; ++w) seed[w] = valid[w] ? seedv(r0 + st + 1, w) : 0.f;
          float tot[W], S00[W];
#pragma unroll
          for (int w = 0; w < W; ++w) {
            float sv = 0.f;
#pragma unroll
            for (int b = 0; b < M; ++b)
              if (b < dm) sv += CB[cbo + b][w];
            tot[w] = sv;
          }
          // exclusive scans over columns (64 lanes x W)
          auto xscan = [&](const float (&v)[W], float (&o)[W]) {
            float t[W];
            t[0] = v[0];
#pragma unroll
            for (int w = 1; w < W; ++w) t[w] = t[w - 1] + v[w];
            const float incl = group_incl_scan<64>(t[W - 1]);
            const float base = incl - t[W - 1];
            o[0] = base;
#pragma unroll
            for (int w = 1; w < W; ++w) o[w] = base + t[w - 1];
          };
          xscan(tot, S00);
          float Sa[M][W];
#pragma unroll
          for (int x1 = 1; x1 < M; ++x1)
            if (x1 < dn) xscan(rowsum[x1 - 1], Sa[x1]);
#pragma unroll
          for (int x1 = M - 1; x1 >= 1; --x1)
#pragma unroll
            for (int y1 = M - 1; y1 >= 1; --y1)
              if (x1 < dn && y1 < dn) {
                const float f = 1.0f / (float)((x1 + 1) * (y1 + 1));
#pragma unroll
                for (int w = 0; w < W; ++w) R[x1][y1][w] = f * seed[w] * R[x1 - 1][y1 - 1][w];
              }
#pragma unroll
          for (int y1 = 1; y1 < M; ++y1)
            if (y1 < dn) {
              const float f = 1.0f / (float)(y1 + 1);
#pragma unroll
              for (int w = 0; w < W; ++w) R[0][y1][w] = f * seed[w] * CB[cbo + y1 - 1][w];
            }
#pragma unroll
          for (int x1 = 1; x1 < M; ++x1)
            if (x1 < dn) {
              const float f = 1.0f / (float)(x1 + 1);
#pragma unroll
              for (int w = 0; w < W; ++w) R[x1][0][w] = f * seed[w] * Sa[x1][w];
            }
#pragma unroll
          for (int w = 0; w < W; ++w) R[0][0][w] = seed[w] * S00[w];
        } else {
          // last stage of the level: its cells add to K_i
#pragma unroll
          for (int x1 = 0; x1 < M; ++x1)
#pragma unroll
            for (int w = 0; w < W; ++w) K[i] += colsum[x1][w];
        }
        // CB of (level i, stage st) += this row's column sums (after their use)
#pragma unroll
        for (int b = 0; b < M; ++b)
          if (b < dm)
#pragma unroll
            for (int w = 0; w < W; ++w) CB[cbo + b][w] += colsum[b][w];
        cbo += dm;
      }
    }
  }
#pragma unroll
  for (int i = 1; i <= M; ++i) K[i] = group_sum<64>(K[i]);
  if (lane == 0) {
    // tt < T: write -K(t) now; the ones-tensor block (tt == T) adds +K(ones) in a second pass
    for (int i = 0; i <= M; ++i) {
      float *o = a.out + ((long long)i * a.n + nn) * a.t;
      if (tt < a.t) o[tt] = (i == 0) ? 0.f : -K[i];
    }
    if (tt == a.t)
      for (int i = 1; i <= M; ++i) a.kones[(long long)(i - 1) * a.n + nn] = K[i];
  }
}

// out[i][n][t] = -K(t) + K(ones)   (signature_algs_vosf.py:47)
__global__ void rescaled_combine_kernel(float *out, const float *kones, int M, int n, int t) {
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long per = (long long)n * t;
  if (idx >= (long long)M * per) return;
  const int i = 1 + (int)(idx / per);
  const int nn = (int)((idx % per) / t);
  out[(long long)i * per + (idx % per)] += kones[(long long)(i - 1) * n + nn];
}

}  // namespace gpsig

using namespace gpsig;

// channel padding of the fixed instantiations; 0 = the runtime-channel (wide) instantiation
static int dpad4(int d) { return d <= 4 ? 4 : d <= 8 ? 8 : d <= 16 ? 16 : d <= 32 ? 32 : 0; }

namespace gpsig {
int tvs_pk_launch(const float *Z, int lt, int t, int increments, int d, const float *Ft, int n, int l, int M,
                  float *out, float *Zp, bool rbf, float *state, hipStream_t s);
int tvs_wide_launch(const float *Z, int lt, int t, int increments, int d, const float *X, const float *Ft, int n,
                    int l, int M, float *out, float *Zw, bool rbf, float *state, void *seedws, hipStream_t s);
size_t tvs_pk_zp_bytes(int lt, int t, int d);
size_t tvs_seed_bytes(int n, int l, int d, int lt, int t);
}  // namespace gpsig

static size_t tvs_ft_bytes(int n, int l, int d) {
  return ((size_t)n * l * (2 * d + 3) * sizeof(float) + 255) & ~(size_t)255;
}

// time-major sequence features for other translation units (the tens-vs-seq VJP, sig_tvs_bwd.hip)
namespace gpsig {
size_t tvs_features_bytes(int n, int l, int d) { return tvs_ft_bytes(n, l, d); }
int tvs_features_launch(const float *X, int n, int l, int d, float *Ft, hipStream_t s) {
  const long long tot = (long long)n * l;
  hipLaunchKernelGGL(tvs_features_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, X, n, l, d, Ft);
  return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
}
}  // namespace gpsig

// features, prepared components, and (d > 8) the wide path's seed GEMM tile
extern "C" size_t gpsig_tens_workspace_bytes(int n, int l, int d, int lt, int t) {
  return tvs_ft_bytes(n, l, d) + tvs_pk_zp_bytes(lt, t, d) + tvs_seed_bytes(n, l, d, lt, t);
}
static void *tvs_seed_ws(void *workspace, int n, int l, int d, int lt, int t) {
  return static_cast<char *>(workspace) + tvs_ft_bytes(n, l, d) + tvs_pk_zp_bytes(lt, t, d);
}

extern "C" int gpsig_tens_vs_seq(const float *Z, int lt, int t, int increments, int d, const float *X, int n, int l,
                                 int num_levels, int order, int base_kind, int difference, float *out, void *workspace,
                                 size_t workspace_bytes, gpsig_stream_t stream) {
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (!Z || !X || !out || lt <= 0 || t <= 0 || n <= 0 || d <= 0 || num_levels < 1) return GPSIG_EINVAL;
  if (lt != num_levels * (num_levels + 1) / 2 || l < (difference ? 2 : 1)) return GPSIG_EINVAL;
  if (num_levels > TV_MMAX || order < 1 || t > 65535) return GPSIG_EUNSUPPORTED;
  if (base_kind != GPSIG_BASE_RBF && base_kind != GPSIG_BASE_LINEAR) return GPSIG_EUNSUPPORTED;
  const int DP = dpad4(d);
  if (!workspace || workspace_bytes < gpsig_tens_workspace_bytes(n, l, d, lt, t)) return GPSIG_EWORKSPACE;
  float *Ft = static_cast<float *>(workspace);
  const long long tot = (long long)n * l;
  hipLaunchKernelGGL(tvs_features_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, X, n, l, d, Ft);
  if (difference && order == 1) {
    // packed fast paths: RBF (exp-free recurrences) and linear, d <= 8; any channel count: the same
    // recursion with a runtime channel loop
    float *Zp = reinterpret_cast<float *>(static_cast<char *>(workspace) + tvs_ft_bytes(n, l, d));
    int rc = tvs_pk_launch(Z, lt, t, increments, d, Ft, n, l, num_levels, out, Zp, base_kind == GPSIG_BASE_RBF,
                           nullptr, s);
    if (rc == -1 && d > 8)
      rc = tvs_wide_launch(Z, lt, t, increments, d, X, Ft, n, l, num_levels, out, Zp, base_kind == GPSIG_BASE_RBF,
                           nullptr, tvs_seed_ws(workspace, n, l, d, lt, t), s);
    if (rc != -1) return rc;
  }
  TvsArgs a{Z, Ft, lt, t, n, l, d, num_levels, order, increments, difference, base_kind == GPSIG_BASE_RBF, out};
  dim3 grid((n + 63) / 64, t);
  const size_t lds = ((size_t)2 * 64 * lt + (size_t)lt * (increments ? 2 : 1) * d) * sizeof(float);
  if (lds > 160 * 1024) return GPSIG_EUNSUPPORTED;
  switch (DP) {
    case 4: hipLaunchKernelGGL(tvs_kernel<4>, grid, dim3(64), lds, s, a); break;
    case 8: hipLaunchKernelGGL(tvs_kernel<8>, grid, dim3(64), lds, s, a); break;
    case 16: hipLaunchKernelGGL(tvs_kernel<16>, grid, dim3(64), lds, s, a); break;
    case 32: hipLaunchKernelGGL(tvs_kernel<32>, grid, dim3(64), lds, s, a); break;
    default: hipLaunchKernelGGL(tvs_kernel<0>, grid, dim3(64), lds, s, a); break;
  }
  return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
}

// As gpsig_tens_vs_seq (order 1, difference 1, RBF or linear, d <= 8, num_levels <= 6: the packed fast
// paths) and also writes the VJP's saved state: state (T, n, LT) = each component's end-of-sweep running
// sum.  GPSIG_EUNSUPPORTED (nothing launched) outside the fast paths.
extern "C" int gpsig_tens_vs_seq_state(const float *Z, int lt, int t, int increments, int d, const float *X, int n,
                                       int l, int num_levels, int base_kind, float *out, float *state, void *workspace,
                                       size_t workspace_bytes, gpsig_stream_t stream) {
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (!Z || !X || !out || !state || lt <= 0 || t <= 0 || n <= 0 || d <= 0 || num_levels < 1 || l < 2)
    return GPSIG_EINVAL;
  if (lt != num_levels * (num_levels + 1) / 2) return GPSIG_EINVAL;
  if (base_kind != GPSIG_BASE_RBF && base_kind != GPSIG_BASE_LINEAR) return GPSIG_EUNSUPPORTED;
  if (num_levels > TV_MMAX || t > 65535) return GPSIG_EUNSUPPORTED;
  if (d <= 8 && num_levels > 6) return GPSIG_EUNSUPPORTED;  // the packed paths' levels
  if (!workspace || workspace_bytes < gpsig_tens_workspace_bytes(n, l, d, lt, t)) return GPSIG_EWORKSPACE;
  float *Ft = static_cast<float *>(workspace);
  const long long tot = (long long)n * l;
  hipLaunchKernelGGL(tvs_features_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, X, n, l, d, Ft);
  float *Zp = reinterpret_cast<float *>(static_cast<char *>(workspace) + tvs_ft_bytes(n, l, d));
  int rc = tvs_pk_launch(Z, lt, t, increments, d, Ft, n, l, num_levels, out, Zp, base_kind == GPSIG_BASE_RBF, state, s);
  if (rc == -1 && d > 8)
    rc = tvs_wide_launch(Z, lt, t, increments, d, X, Ft, n, l, num_levels, out, Zp, base_kind == GPSIG_BASE_RBF, state,
                         tvs_seed_ws(workspace, n, l, d, lt, t), s);
  return rc == -1 ? GPSIG_EUNSUPPORTED : rc;
}

namespace gpsig {
size_t tens_gram_mm_bytes(int lt, int t);
int tens_gram_mm(const float *Z, int lt, int t, int incr, int d, int M, int rbf, float *out, void *workspace,
                 size_t workspace_bytes, hipStream_t s);
}  // namespace gpsig

// Channel counts past 32 run the pair-tile kernel of the VJP (tens_vjp_mm.hip) and need a workspace.
extern "C" size_t gpsig_tens_gram_workspace_bytes(int lt, int t, int d) {
  if (lt <= 0 || t <= 0 || d <= 0 || dpad4(d) != 0) return 0;
  return gpsig::tens_gram_mm_bytes(lt, t);
}

extern "C" int gpsig_tens_gram(const float *Z, int lt, int t, int increments, int d, int num_levels, int base_kind,
                               float *out, void *workspace, size_t workspace_bytes, gpsig_stream_t stream) {
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (!Z || !out || lt <= 0 || t <= 0 || d <= 0 || num_levels < 1) return GPSIG_EINVAL;
  if (lt != num_levels * (num_levels + 1) / 2) return GPSIG_EINVAL;
  if (num_levels > TV_MMAX) return GPSIG_EUNSUPPORTED;
  if (base_kind != GPSIG_BASE_RBF && base_kind != GPSIG_BASE_LINEAR) return GPSIG_EUNSUPPORTED;
  const int DP = dpad4(d);
  if (DP == 0)
    return gpsig::tens_gram_mm(Z, lt, t, increments ? 1 : 0, d, num_levels, base_kind == GPSIG_BASE_RBF ? 1 : 0, out,
                               workspace, workspace_bytes, s);
  TgArgs a{Z, lt, t, d, num_levels, increments, base_kind == GPSIG_BASE_RBF, out};
  dim3 grid((t + 255) / 256, t);
  switch (DP) {
    case 4: hipLaunchKernelGGL(tens_gram_kernel<4>, grid, dim3(256), 0, s, a); break;
    case 8: hipLaunchKernelGGL(tens_gram_kernel<8>, grid, dim3(256), 0, s, a); break;
    case 16: hipLaunchKernelGGL(tens_gram_kernel<16>, grid, dim3(256), 0, s, a); break;
    case 32: hipLaunchKernelGGL(tens_gram_kernel<32>, grid, dim3(256), 0, s, a); break;
    default: return GPSIG_EUNSUPPORTED;  // past 32 channels: the pair tiles above
  }
  return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
}

// ------------------------------------------------------------------------------------ tensor Gram VJP
// Gradient of tensor_kern (signature_algs.py:76-99) over the component Grams of _K_tens
// (kernels.py:264-284): K_i(t, t') = prod_{c in level i} M_c(t, t'), so
//   dLoss/dz_c^t = sum_t' (G_i(t, t') + G_i(t', t)) prod_{c' != c} M_c'(t, t') d/dz_c^t M_c(t, t')
// (the symmetric sum covers t as the second argument).  Lane = t, block = (level, chunk of t').
struct TgBwdArgs {
  const float *Z;     // (LT, T, d) or (LT, T, 2, d)
  int t, d, incr, rbf, chunk;
  const float *gout;  // (M+1, T, T)
  float *gZ;          // like Z, accumulated
};

// Channel counts up to 32 (DP = 4 .. 32, padded channels read as zeros); wider ones: tens_vjp_mm.hip.
template <int DP>
__global__ __launch_bounds__(64) void tens_gram_vjp_kernel(TgBwdArgs a) {
  const int t1 = blockIdx.x * 64 + threadIdx.x;
  if (t1 >= a.t) return;
  const int i = blockIdx.y + 1, k0 = i * (i - 1) / 2;
  const int tb = blockIdx.z * a.chunk, te = min(a.t, tb + a.chunk);
  const int d = a.d, T = a.t, zs = a.incr ? 2 * d : d;
  auto zv = [&](int k, int tt, int h, int q) -> float {
    return q < d ? a.Z[((long long)k * T + tt) * zs + h * d + q] : 0.f;
  };
  float g0[TV_MMAX][DP], g1[TV_MMAX][DP];
#pragma unroll
  for (int c = 0; c < TV_MMAX; ++c)
#pragma unroll
    for (int q = 0; q < DP; ++q) g0[c][q] = g1[c][q] = 0.f;
  for (int t2 = tb; t2 < te; ++t2) {
    const float Gs = a.gout[((long long)i * T + t1) * T + t2] + a.gout[((long long)i * T + t2) * T + t1];
    float m[TV_MMAX];
#pragma unroll
    for (int c = 0; c < TV_MMAX; ++c) {
      if (c >= i) break;
      const int k = k0 + c;
      if (!a.incr) {
        float s2 = 0.f, ip = 0.f;
#pragma unroll
        for (int q = 0; q < DP; ++q) {
          const float df = zv(k, t1, 0, q) - zv(k, t2, 0, q);
          s2 = __builtin_fmaf(df, df, s2);
          ip = __builtin_fmaf(zv(k, t1, 0, q), zv(k, t2, 0, q), ip);
        }
        m[c] = a.rbf ? fast_exp(-0.5f * s2) : ip;
      } else {
        float A0[DP], dA[DP], B0[DP], dB[DP];
#pragma unroll
        for (int q = 0; q < DP; ++q) {
          A0[q] = zv(k, t1, 0, q);
          dA[q] = zv(k, t1, 1, q) - A0[q];
          B0[q] = zv(k, t2, 0, q);
          dB[q] = zv(k, t2, 1, q) - B0[q];
        }
        if (a.rbf) {
          m[c] = rbf_second_diff<DP>(A0, dA, B0, dB);
        } else {
          float v = 0.f;
#pragma unroll
          for (int q = 0; q < DP; ++q) v = __builtin_fmaf(dA[q], dB[q], v);
          m[c] = v;
        }
      }
    }
    // products of the other components: prefix * suffix
    float pre[TV_MMAX], suf = 1.f;
    pre[0] = 1.f;
#pragma unroll
    for (int c = 1; c < TV_MMAX; ++c) pre[c] = (c < i) ? pre[c - 1] * m[c - 1] : 0.f;
#pragma unroll
    for (int c = TV_MMAX - 1; c >= 0; --c) {
      if (c >= i) continue;
      const float w = Gs * pre[c] * suf;
      suf *= m[c];
      const int k = k0 + c;
      constexpr int nq = DP;
      if (!a.incr) {
        if (a.rbf) {
          float s2 = 0.f;

          for (int q = 0; q < nq; ++q) {
            const float df = zv(k, t2, 0, q) - zv(k, t1, 0, q);
            s2 = __builtin_fmaf(df, df, s2);
          }
          const float wk = w * fast_exp(-0.5f * s2);
#pragma unroll
          for (int q = 0; q < DP; ++q) g0[c][q] = __builtin_fmaf(wk, zv(k, t2, 0, q) - zv(k, t1, 0, q), g0[c][q]);
        } else {
#pragma unroll
          for (int q = 0; q < DP; ++q) g0[c][q] = __builtin_fmaf(w, zv(k, t2, 0, q), g0[c][q]);
        }
      } else if (a.rbf) {
        // dM/dA1 = k(A1,B1)(B1 - A1) - k(A1,B0)(B0 - A1),  dM/dA0 = k(A0,B0)(B0 - A0) - k(A0,B1)(B1 - A0)
        float e11 = 0.f, e10 = 0.f, e00 = 0.f, e01 = 0.f;

        for (int q = 0; q < nq; ++q) {
          const float a0 = zv(k, t1, 0, q), a1 = zv(k, t1, 1, q), b0 = zv(k, t2, 0, q), b1 = zv(k, t2, 1, q);
          e11 = __builtin_fmaf(a1 - b1, a1 - b1, e11);
          e10 = __builtin_fmaf(a1 - b0, a1 - b0, e10);
          e00 = __builtin_fmaf(a0 - b0, a0 - b0, e00);
          e01 = __builtin_fmaf(a0 - b1, a0 - b1, e01);
        }
        const float k11 = w * fast_exp(-0.5f * e11), k10 = w * fast_exp(-0.5f * e10);
        const float k00 = w * fast_exp(-0.5f * e00), k01 = w * fast_exp(-0.5f * e01);
#pragma unroll
        for (int q = 0; q < DP; ++q) {
          const float a0 = zv(k, t1, 0, q), a1 = zv(k, t1, 1, q), b0 = zv(k, t2, 0, q), b1 = zv(k, t2, 1, q);
          g1[c][q] += k11 * (b1 - a1) - k10 * (b0 - a1);
          g0[c][q] += k00 * (b0 - a0) - k01 * (b1 - a0);
        }
      } else {
#pragma unroll
        for (int q = 0; q < DP; ++q) {
          const float dBq = zv(k, t2, 1, q) - zv(k, t2, 0, q);
          g1[c][q] = __builtin_fmaf(w, dBq, g1[c][q]);
          g0[c][q] = __builtin_fmaf(-w, dBq, g0[c][q]);
        }
      }
    }
  }
#pragma unroll
  for (int c = 0; c < TV_MMAX; ++c) {
    if (c >= i) break;
    float *gz = a.gZ + ((long long)(k0 + c) * T + t1) * zs;
#pragma unroll
    for (int q = 0; q < DP; ++q) {
      if (q < d) {
        unsafeAtomicAdd(gz + q, g0[c][q]);
        if (a.incr) unsafeAtomicAdd(gz + d + q, g1[c][q]);
      }
    }
  }
}

template <int M, int W>
static int launch_rs(const RsArgs &a, int DP, hipStream_t s) {
  dim3 grid(a.t + 1, a.n);
  switch (DP) {
    case 4: hipLaunchKernelGGL((rescaled_kernel<M, W, 4>), grid, dim3(64), 0, s, a); break;
    case 8: hipLaunchKernelGGL((rescaled_kernel<M, W, 8>), grid, dim3(64), 0, s, a); break;
    case 0: hipLaunchKernelGGL((rescaled_kernel<M, W, 0>), grid, dim3(64), 0, s, a); break;
    default: return GPSIG_EUNSUPPORTED;
  }
  return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
}

template <int M>
static int rs_w(const RsArgs &a, int DP, hipStream_t s) {
  if (a.l - 1 <= 64) return launch_rs<M, 1>(a, DP, s);
  if (a.l - 1 <= 128) return launch_rs<M, 2>(a, DP, s);
  if constexpr (M <= 4) {
    if (a.l - 1 <= 256) return launch_rs<M, 4>(a, DP, s);
  }
  return GPSIG_EUNSUPPORTED;
}

extern "C" size_t gpsig_rescaled_workspace_bytes(int n, int num_levels) {
  return ((size_t)n * num_levels * sizeof(float) + 255) & ~(size_t)255;
}

extern "C" int gpsig_rescaled(const float *Z, int lt, int t, const float *X, int n, int l, int d, int num_levels,
                              int embedding, float *out, void *workspace, size_t workspace_bytes,
                              gpsig_stream_t stream) {
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (!Z || !X || !out || t <= 0 || n <= 0 || l < 2 || d <= 0 || num_levels < 1) return GPSIG_EINVAL;
  if (lt != num_levels * (num_levels + 1) / 2 || (embedding != 0 && embedding != 1)) return GPSIG_EINVAL;
  const int DP = d <= 8 ? dpad4(d) : 0;  // 0: runtime channel loop
  if (!workspace || workspace_bytes < gpsig_rescaled_workspace_bytes(n, num_levels)) return GPSIG_EWORKSPACE;
  RsArgs a{Z, X, lt, t, n, l, d, num_levels, embedding, out, static_cast<float *>(workspace)};
  int rc;
  switch (num_levels) {
    case 1: rc = rs_w<1>(a, DP, s); break;
    case 2: rc = rs_w<2>(a, DP, s); break;
    case 3: rc = rs_w<3>(a, DP, s); break;
    case 4: rc = rs_w<4>(a, DP, s); break;
    case 5: rc = rs_w<5>(a, DP, s); break;
    case 6: rc = rs_w<6>(a, DP, s); break;
    default: return GPSIG_EUNSUPPORTED;
  }
  if (rc) return rc;
  const long long tot = (long long)num_levels * n * t;
  hipLaunchKernelGGL(rescaled_combine_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, out, a.kones,
                     num_levels, n, t);
  return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
}

namespace gpsig {
size_t tens_gram_vjp_mm_bytes(int lt, int t, int incr, int d, int rbf);
int tens_gram_vjp_mm(const float *Z, int lt, int t, int incr, int d, int M, int rbf, const float *gout, float *gZ,
                     void *workspace, size_t workspace_bytes, hipStream_t s);
}  // namespace gpsig

// Channel counts past 32 take the pair-tile + GEMM path (tens_vjp_mm.hip), which needs a workspace.
extern "C" size_t gpsig_tens_gram_vjp_workspace_bytes(int lt, int t, int increments, int d, int num_levels,
                                                      int base_kind) {
  if (lt <= 0 || t <= 0 || d <= 0 || num_levels < 1 || dpad4(d) != 0) return 0;
  return gpsig::tens_gram_vjp_mm_bytes(lt, t, increments ? 1 : 0, d, base_kind == GPSIG_BASE_RBF ? 1 : 0);
}

extern "C" int gpsig_tens_gram_vjp(const float *Z, int lt, int t, int increments, int d, int num_levels,
                                   int base_kind, const float *gout, float *gZ, void *workspace,
                                   size_t workspace_bytes, gpsig_stream_t stream) {
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (!Z || !gout || !gZ || lt <= 0 || t <= 0 || d <= 0 || num_levels < 1) return GPSIG_EINVAL;
  if (lt != num_levels * (num_levels + 1) / 2) return GPSIG_EINVAL;
  if (num_levels > TV_MMAX) return GPSIG_EUNSUPPORTED;
  if (base_kind != GPSIG_BASE_RBF && base_kind != GPSIG_BASE_LINEAR) return GPSIG_EUNSUPPORTED;
  const int DP = dpad4(d);
  if (DP == 0)
    return gpsig::tens_gram_vjp_mm(Z, lt, t, increments ? 1 : 0, d, num_levels, base_kind == GPSIG_BASE_RBF ? 1 : 0, gout,
                            gZ, workspace, workspace_bytes, s);
  const int chunk = 64;
  TgBwdArgs a{Z, t, d, increments, base_kind == GPSIG_BASE_RBF, chunk, gout, gZ};
  dim3 grid((t + 63) / 64, num_levels, (t + chunk - 1) / chunk);
  switch (DP) {
    case 4: hipLaunchKernelGGL(tens_gram_vjp_kernel<4>, grid, dim3(64), 0, s, a); break;
    case 8: hipLaunchKernelGGL(tens_gram_vjp_kernel<8>, grid, dim3(64), 0, s, a); break;
    case 16: hipLaunchKernelGGL(tens_gram_vjp_kernel<16>, grid, dim3(64), 0, s, a); break;
    case 32: hipLaunchKernelGGL(tens_gram_vjp_kernel<32>, grid, dim3(64), 0, s, a); break;
    default: return GPSIG_EUNSUPPORTED;
  }
  return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
}
