// gpsig_amd -- truncated signatures of piecewise-linear paths on gfx950.
//
// Replaces iisignature.sig (iisignature 0.24, requirements.txt:11) behind the reference's
// iisignature_tensorflow.Sig (gpsig/iisignature_tensorflow.py:87), which the VOSF inducing-feature
// path calls for Kuf (gpsig/inducing_variables_vosf.py:120-146): levels 1..depth of
//   S(x) = exp(dx_1) (x) exp(dx_2) (x) ... (x) exp(dx_{L-1}),   exp(h)_m = h^{(x)m} / m!,
// each level flattened first-index-major (iisignature's layout), concatenated.
//
// One workgroup per path; the level tensors live in LDS, or (GLB, past the 160 KiB of a CU's LDS) in a
// per-path slab of global memory (L2-resident at the sizes it takes over; the workgroup barriers order
// its accesses as they do the LDS ones).  Per increment h the levels are updated in
// place from the top level down (Chen's identity):
//   S_m[i_1..i_m] += sum_{j<m} S_j[i_1..i_j] h[i_{j+1}] ... h[i_m] / (m-j)!
// every entry independently (one thread per entry, the prefix sums read the not-yet-updated lower
// levels), one barrier per level.
#include "sig_common.h"

namespace gpsig {

// 1 / k!, k = 0..16: the exponential's and Chen's coefficients as multiplications (a division per term is a
// ten-instruction sequence); indexed by wave-uniform level counts, so read through the scalar cache
__constant__ float c_invfact[17] = {1.0f, 1.0f, 0.5f, 1.6666667e-1f, 4.1666668e-2f, 8.3333338e-3f, 1.3888889e-3f,
                                    1.9841270e-4f, 2.4801587e-5f, 2.7557319e-6f, 2.7557319e-7f, 2.5052108e-8f,
                                    2.0876757e-9f, 1.6059044e-10f, 1.1470746e-11f, 7.6471637e-13f, 4.7794773e-14f};

struct SigFeatArgs {
  const float *X;  // (n, l, d)
  int n, l, d, depth;
  float *out;      // (n, total)
  int total;       // sum_{m=1}^{depth} d^m
  float *glb;      // GLB: per-path slabs of `stride` floats for the paths [path0, path0 + gridDim.x)
  long long stride;
  int path0;
};

// Digits of a multi-index in base d (indices < 2^32 / d; tensors here are < 2^14 entries): quotient by a multiply-high with
// ceil(2^32 / d) instead of an integer division (a runtime division is a ~20-instruction sequence, and
// the digit loops run per tensor entry, per increment).
struct DivD {
  unsigned m, d;
  __device__ explicit DivD(int dd) : m(0xFFFFFFFFu / (unsigned)dd + 1u), d((unsigned)dd) {}
  __device__ int div(int v) const { return d == 1 ? v : (int)__umulhi((unsigned)v, m); }
};

template <bool GLB>
__global__ __launch_bounds__(256) void sig_features_kernel(SigFeatArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds_s[];  // [h (d) | level 1 | level 2 | ...]
  const int path = a.path0 + (int)blockIdx.x, tid = threadIdx.x, nth = blockDim.x;
  float *S = GLB ? a.glb + (long long)blockIdx.x * a.stride : lds_s;
  const int d = a.d, M = a.depth;
  float *h = S;
  float *lev = S + d;
  for (int e = tid; e < a.total; e += nth) lev[e] = 0.0f;
  int off[17], sz[17];  // level m at lev + off[m], d^m entries
  off[1] = 0;
  sz[0] = 1;
  for (int m = 1; m <= M; ++m) {
    sz[m] = sz[m - 1] * d;
    if (m < M) off[m + 1] = off[m] + sz[m];
  }
  const float *x = a.X + (long long)path * a.l * d;
  const DivD dv(d);
  // (tid < d) the path's points: x_s kept from the previous step, x_{s+1} loaded one step ahead
  float xc = tid < d ? x[tid] : 0.0f, xn = tid < d && a.l > 1 ? x[d + tid] : 0.0f;
  for (int s = 0; s + 1 < a.l; ++s) {
    const float xnn = tid < d && s + 2 < a.l ? x[(s + 2) * d + tid] : 0.0f;
    __syncthreads();
    if (tid < d) h[tid] = xn - xc;
    xc = xn;
    xn = xnn;
    __syncthreads();
    for (int m = M; m >= 1; --m) {
      float *Sm = lev + off[m];
      for (int e = tid; e < sz[m]; e += nth) {
        float acc = 0.0f, P = 1.0f;
        int pre = e;
        for (int j = m - 1; j >= 0; --j) {
          const int q = dv.div(pre), digit = pre - q * d;
          pre = q;
          P *= h[digit];
          const float Sj = (j == 0) ? 1.0f : lev[off[j] + pre];
          acc = __builtin_fmaf(Sj, P * c_invfact[m - j], acc);
        }
        Sm[e] += acc;
      }
      __syncthreads();
    }
  }
  float *o = a.out + (long long)path * a.total;
  for (int e = tid; e < a.total; e += nth) o[e] = lev[e];
}

// ------------------------------------------------------------------------------------ backward
// Gradient of sum_m <G_m, S_m(x)> (iisignature.sigbackprop behind the Sig op's gradient,
// iisignature_tensorflow.py:_sigGrad).  Per path, after a forward pass to S(x), the increments are
// walked backwards; with T = S (x) E(h), E(h) = exp(h):
//   S_before = T (x) E(-h)                                   (exact in the truncated algebra)
//   dE_r[v]  = sum_{m>=r} sum_u dT_m[u v] S_{m-r}[u]
//   dS_j[u]  = sum_{m>=j} sum_v dT_m[u v] E_{m-j}[v]          (in place, ascending j)
//   dh[q]    = sum_r sum_v dE_r[v] dE_r[v]/dh[q],  E_r[v] = h[v_1] ... h[v_r] / r!
// and dx_{k+1} += dh, dx_k -= dh.  LDS: h, dh, S, dS, dE, E.
constexpr int GH_REG = 8;  // channels whose increment gradient is accumulated in registers

// lanes per output when `outputs` sums share a wave: the largest power of two G <= 64 / outputs
__device__ inline int group_lanes(int outputs) {
  int G = 1;
  while (G < 64 && 2 * G * outputs <= 64) G *= 2;
  return G;
}
// sum over aligned groups of G lanes (every lane of the wave takes part)
__device__ inline float group_reduce(float v, int G) {
  for (int o = G / 2; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <bool GLB>
__global__ __launch_bounds__(256) void sig_features_bwd_kernel(SigFeatArgs a, const float *__restrict__ gout,
                                                               float *__restrict__ gX) {
  extern __shared__ __attribute__((aligned(16))) float lds_s[];
  const int path = a.path0 + (int)blockIdx.x, tid = threadIdx.x, nth = blockDim.x;
  float *sh = GLB ? a.glb + (long long)blockIdx.x * a.stride : lds_s;
  const int d = a.d, M = a.depth, tot = a.total;
  float *h = sh, *gh = sh + d;
  float *lev = sh + 2 * d, *adj = lev + tot, *gE = adj + tot;
  int off[17], sz[17];
  off[1] = 0;
  sz[0] = 1;
  for (int m = 1; m <= M; ++m) {
    sz[m] = sz[m - 1] * d;
    if (m < M) off[m + 1] = off[m] + sz[m];
  }
  const float *x = a.X + (long long)path * a.l * d;
  const DivD dv(d);
  float *gx = gX + (long long)path * a.l * d;
  const float *g = gout + (long long)path * tot;
  for (int e = tid; e < tot; e += nth) {
    lev[e] = 0.0f;
    adj[e] = g[e];
  }
  // S (x) E(sgn h), in place from the top level down
  auto chen = [&]() {
    for (int m = M; m >= 1; --m) {
      float *Sm = lev + off[m];
      for (int e = tid; e < sz[m]; e += nth) {
        float acc = 0.0f, P = 1.0f;
        int pre = e;
        for (int j = m - 1; j >= 0; --j) {
          const int q = dv.div(pre), digit = pre - q * d;
          pre = q;
          P *= h[digit];
          const float Sj = (j == 0) ? 1.0f : lev[off[j] + pre];
          acc = __builtin_fmaf(Sj, P * c_invfact[m - j], acc);
        }
        Sm[e] += acc;
      }
      __syncthreads();
    }
  };
  // E_r[v] = prod h[v_p] / r!, tabulated per increment in LDS (Et, same layout as the levels)
  float *Et = gE + tot;
  auto fill_E = [&]() {
    for (int r = 1; r <= M; ++r)
      for (int v = tid; v < sz[r]; v += nth) {
        float P = 1.0f;
        int w = v;
        for (int p = 0; p < r; ++p) {
          const int q = dv.div(w);
          P *= h[w - q * d];
          w = q;
        }
        Et[off[r] + v] = P * c_invfact[r];
      }
  };
  for (int s = 0; s + 1 < a.l; ++s) {
    __syncthreads();
    if (tid < d) h[tid] = x[(s + 1) * d + tid] - x[s * d + tid];
    __syncthreads();
    chen();
  }
  float ghp = 0.0f;  // (tid < d) dh of the step after this one
  for (int s = a.l - 2; s >= 0; --s) {
    if (tid < d) {
      h[tid] = -(x[(s + 1) * d + tid] - x[s * d + tid]);
      gh[tid] = 0.0f;
    }
    __syncthreads();
    chen();  // lev = S before increment s
    if (tid < d) h[tid] = -h[tid];
    __syncthreads();
    fill_E();
    // dE_r[v] for r = 1..M.  The low levels have few outputs with long sums: each output gets a group of
    // G lanes (G = the largest power of two with G * outputs <= the wave) that split its terms and
    // reduce them by xor-shuffles, so the wave stays busy.
    for (int r = 1; r <= M; ++r) {
      const int G = group_lanes(sz[r]), g = tid & (G - 1);
      for (int ob = 0; ob < sz[r]; ob += nth / G) {
        const int v = ob + tid / G;
        float acc = 0.0f;
        if (v < sz[r])
          for (int m = r; m <= M; ++m) {
            const int nu = sz[m - r];
            const float *Tm = adj + off[m];
            for (int u = g; u < nu; u += G) {
              const float Su = (m == r) ? 1.0f : lev[off[m - r] + u];
              acc = __builtin_fmaf(Tm[u * sz[r] + v], Su, acc);
            }
          }
        acc = group_reduce(acc, G);
        if (v < sz[r] && g == 0) gE[off[r] + v] = acc;
      }
    }
    __syncthreads();
    // dh from dE: per-thread partials in registers (d <= GH_REG), reduced over the wave and added
    // to the d LDS slots by one lane per wave; wider paths take LDS atomics
    float ghr[GH_REG];
#pragma unroll
    for (int q = 0; q < GH_REG; ++q) ghr[q] = 0.0f;
    for (int r = 1; r <= M; ++r)
      for (int v = tid; v < sz[r]; v += nth) {
        const float ge = gE[off[r] + v] * c_invfact[r];
        // digits of v (most significant first is irrelevant: the product is symmetric)
        int vv = v;
        for (int p = 0; p < r; ++p) {
          const int vq = dv.div(vv), q = vv - vq * d;
          vv = vq;
          float P = 1.0f;
          int w = v;
          for (int p2 = 0; p2 < r; ++p2) {
            const int wq = dv.div(w);
            if (p2 != p) P *= h[w - wq * d];
            w = wq;
          }
          const float val = ge * P;
          if (d <= GH_REG) {
#pragma unroll
            for (int q2 = 0; q2 < GH_REG; ++q2) ghr[q2] += (q2 == q) ? val : 0.0f;  // no dynamic register index
          } else {
            atomicAdd(gh + q, val);
          }
        }
      }
    if (d <= GH_REG) {
      group_incl_scan_n<64, GH_REG>(ghr);  // wave sums in lane 63
      if ((tid & 63) == 63)
#pragma unroll
        for (int q = 0; q < GH_REG; ++q)
          if (q < d) atomicAdd(gh + q, ghr[q]);
    }
    // dS_j[u] = sum_{m>=j} sum_v dT_m[u v] E_{m-j}[v], ascending j in place (grouped as dE)
    for (int j = 1; j <= M; ++j) {
      const int G = group_lanes(sz[j]), g = tid & (G - 1);
      for (int ob = 0; ob < sz[j]; ob += nth / G) {
        const int u = ob + tid / G;
        float acc = 0.0f;
        if (u < sz[j]) {
          if (g == 0) acc = adj[off[j] + u];
          for (int m = j + 1; m <= M; ++m) {
            const int nv = sz[m - j];
            const float *Tm = adj + off[m];
            const float *E = Et + off[m - j];
            for (int v = g; v < nv; v += G) acc = __builtin_fmaf(Tm[u * nv + v], E[v], acc);
          }
        }
        acc = group_reduce(acc, G);
        if (u < sz[j] && g == 0) adj[off[j] + u] = acc;
      }
      __syncthreads();
    }
    // dx_{s+1} += dh_s, dx_s -= dh_s: point s+1 takes dh_s - dh_{s+1} now (each point's gradient is read and
    // written once, so no step waits on the previous step's store to the same address)
    if (tid < d) {
      gx[(s + 1) * d + tid] += gh[tid] - ghp;
      ghp = gh[tid];
    }
  }
  if (tid < d && a.l > 1) gx[tid] -= ghp;
}

}  // namespace gpsig

using namespace gpsig;

namespace {
constexpr size_t SIG_LDS_MAX = 160 * 1024;               // a CU's LDS
constexpr size_t SIG_GLB_BUDGET = (size_t)1 << 30;       // per launch chunk of paths (GLB slabs)
long long sig_total(int d, int depth) {
  long long t = 0, p = 1;
  for (int m = 1; m <= depth; ++m) {
    p *= d;
    t += p;
  }
  return t;
}
// floats of one path's level storage: forward [h | levels], backward [h | gh | levels | adjoints | dE | E]
long long sig_slab_floats(long long total, int d, bool vjp) {
  const long long f = vjp ? 4 * total + 2 * d : total + d;
  return (f + 63) & ~63LL;  // 256-byte aligned slabs
}
bool sig_in_lds(long long total, int d, bool vjp) { return (size_t)(vjp ? 4 * total + 2 * d : total + d) * 4 <= SIG_LDS_MAX; }
int sig_chunk_paths(long long slab, int n) {
  long long c = (long long)(SIG_GLB_BUDGET / ((size_t)slab * sizeof(float)));
  if (c < 1) c = 1;
  return (int)(c < n ? c : n);
}
bool sig_args_ok(long long total, int d, int depth) {
  // entries are indexed in int, digits by a multiply-high valid below 2^32 / d
  return depth <= 16 && total > 0 && total < (1LL << 31) / 4 && (long long)d * total < (1LL << 32);
}
}  // namespace

extern "C" long long gpsig_signature_channels(int d, int depth) {
  if (d <= 0 || depth <= 0) return 0;
  return sig_total(d, depth);
}

extern "C" size_t gpsig_signature_workspace_bytes(int n, int d, int depth, int vjp) {
  if (n <= 0 || d <= 0 || depth <= 0 || depth > 16) return 0;
  const long long total = sig_total(d, depth);
  if (sig_in_lds(total, d, vjp != 0)) return 0;
  const long long slab = sig_slab_floats(total, d, vjp != 0);
  return (size_t)sig_chunk_paths(slab, n) * (size_t)slab * sizeof(float);
}

extern "C" int gpsig_signature_ex(const float *X, int n, int l, int d, int depth, float *out, void *workspace,
                                  size_t workspace_bytes, gpsig_stream_t stream) {
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (!X || !out || n <= 0 || l < 1 || d <= 0 || depth < 1) return GPSIG_EINVAL;
  if (depth > 16) return GPSIG_EUNSUPPORTED;
  const long long total = sig_total(d, depth);
  if (!sig_args_ok(total, d, depth)) return GPSIG_EUNSUPPORTED;
  SigFeatArgs a{X, n, l, d, depth, out, (int)total, nullptr, 0, 0};
  const int nth = (total - (total - 1) / d) <= 256 ? 64 : 256;  // top level d^depth entries
  if (sig_in_lds(total, d, false)) {
    const size_t lds = (size_t)(total + d) * sizeof(float);
    hipLaunchKernelGGL(sig_features_kernel<false>, dim3((unsigned)n), dim3(nth), lds, s, a);
    return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
  }
  a.stride = sig_slab_floats(total, d, false);
  const int chunk = sig_chunk_paths(a.stride, n);
  if (!workspace || workspace_bytes < (size_t)chunk * (size_t)a.stride * sizeof(float)) return GPSIG_EWORKSPACE;
  a.glb = static_cast<float *>(workspace);
  for (int p0 = 0; p0 < n; p0 += chunk) {
    a.path0 = p0;
    const int np = n - p0 < chunk ? n - p0 : chunk;
    hipLaunchKernelGGL(sig_features_kernel<true>, dim3((unsigned)np), dim3(256), 0, s, a);
  }
  return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
}

extern "C" int gpsig_signature(const float *X, int n, int l, int d, int depth, float *out, gpsig_stream_t stream) {
  return gpsig_signature_ex(X, n, l, d, depth, out, nullptr, 0, stream);
}

extern "C" int gpsig_signature_vjp_ex(const float *X, int n, int l, int d, int depth, const float *gout, float *gX,
                                      void *workspace, size_t workspace_bytes, gpsig_stream_t stream) {
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (!X || !gout || !gX || n <= 0 || l < 1 || d <= 0 || depth < 1) return GPSIG_EINVAL;
  if (depth > 16) return GPSIG_EUNSUPPORTED;
  const long long total = sig_total(d, depth);
  if (!sig_args_ok(total, d, depth)) return GPSIG_EUNSUPPORTED;
  SigFeatArgs a{X, n, l, d, depth, nullptr, (int)total, nullptr, 0, 0};
  // one wave per path while the top level fits a few entries per lane (barriers stay wave-local)
  const int nth = (total - (total - 1) / d) <= 256 ? 64 : 256;
  if (sig_in_lds(total, d, true)) {
    const size_t lds = (size_t)(4 * total + 2 * d) * sizeof(float);
    hipLaunchKernelGGL(sig_features_bwd_kernel<false>, dim3((unsigned)n), dim3(nth), lds, s, a, gout, gX);
    return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
  }
  a.stride = sig_slab_floats(total, d, true);
  const int chunk = sig_chunk_paths(a.stride, n);
  if (!workspace || workspace_bytes < (size_t)chunk * (size_t)a.stride * sizeof(float)) return GPSIG_EWORKSPACE;
  a.glb = static_cast<float *>(workspace);
  for (int p0 = 0; p0 < n; p0 += chunk) {
    a.path0 = p0;
    const int np = n - p0 < chunk ? n - p0 : chunk;
    hipLaunchKernelGGL(sig_features_bwd_kernel<true>, dim3((unsigned)np), dim3(256), 0, s, a, gout, gX);
  }
  return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
}

extern "C" int gpsig_signature_vjp(const float *X, int n, int l, int d, int depth, const float *gout, float *gX,
                                   gpsig_stream_t stream) {
  return gpsig_signature_vjp_ex(X, n, l, d, depth, gout, gX, nullptr, 0, stream);
}
