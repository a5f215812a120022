// gpsig_amd -- host side of the matrix-core wide-channel Gram (sig_fo_mf.h): the GEMM operand records and the
// pair-tile launch.
#include "sig_fo_mf.h"

namespace gpsig {

// Record rows: aug[t][k] = x_0 (t = 0), x_t - x_{t-1} (1 <= t < l); points[t][k] = x_t (t < l); zero past the
// sequence and past d.
__global__ __launch_bounds__(256) void mf_aug_kernel(const float *__restrict__ X, int n, int l, int d,
                                                     float *__restrict__ R) {
  const int rows = mf_rows(l), kp = mf_kp(d);
  const long long rec = mf_rec_floats(d, l);
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long long)n * rows * kp) return;
  const int k = (int)(idx % kp);
  const long long r = idx / kp;
  const int t = (int)(r % rows);
  const int s = (int)(r / rows);
  float v = 0.0f, pt = 0.0f;
  if (k < d && t < l) {
    const float *x = X + ((long long)s * l + t) * d + k;
    pt = x[0];
    v = t == 0 ? x[0] : x[0] - x[-d];
  }
  float *rs = R + (long long)s * rec + (long long)t * kp + k;
  rs[0] = v;
  rs[(long long)rows * kp] = pt;
}

// Per-cell scalars hd_i = |dx_i|^2 / 2, gg_i = <x_i, dx_i> + |dx_i|^2 / 2 (wide_records' arithmetic: fp32
// squares in channel order, fp64 <x, dx>), zero past the cells.
__global__ __launch_bounds__(256) void mf_scalars_kernel(const float *__restrict__ X, int n, int l, int d,
                                                         float *__restrict__ R) {
  const int rows = mf_rows(l), kp = mf_kp(d);
  const long long rec = mf_rec_floats(d, l);
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long long)n * rows) return;
  const int i = (int)(idx % rows);
  const int s = (int)(idx / rows);
  float *base = R + (long long)s * rec + 2LL * rows * kp;
  float h = 0.0f;
  double gx = 0.0;
  if (i + 1 < l) {
    const float *x = X + ((long long)s * l + i) * d;
    for (int k = 0; k < d; ++k) {
      const float xv = x[k], dv = x[d + k] - xv;
      h = __builtin_fmaf(dv, dv, h);
      gx = __builtin_fma((double)xv, (double)dv, gx);
    }
  }
  base[i] = 0.5f * h;
  base[rows + i] = (i + 1 < l) ? (float)(gx + 0.5 * (double)h) : 0.0f;
}

// 2^e with the largest |value| m at 2^e m in [2^14, 2^15) (1 for m = 0), as 2^-e, 2^e
GPSIG_DEV f2 mf_scale_of(float m) {
  int ex = 0;
  if (m > 0.0f && __builtin_isfinite(m)) frexpf(m, &ex);  // m in [2^(ex-1), 2^ex)
  int e = m > 0.0f && __builtin_isfinite(m) ? 15 - ex : 0;
  e = e < -120 ? -120 : (e > 120 ? 120 : e);
  return (f2){ldexpf(1.0f, -e), ldexpf(1.0f, e)};
}

// The B-side scales of a sequence (sig_fo_mf.h): its largest |increment| and its largest |point|; one
// workgroup per sequence.
__global__ __launch_bounds__(256) void mf_scale_kernel(const float *__restrict__ X, int n, int l, int d,
                                                       float *__restrict__ R) {
  const int s = (int)blockIdx.x;
  const float *__restrict__ x = X + (long long)s * l * d;
  float mi = 0.0f, mp = 0.0f;
  for (int e = (int)threadIdx.x; e < l * d; e += 256) {
    const float v = x[e];
    mp = __builtin_fmaxf(mp, __builtin_fabsf(v));
    if (e >= d) mi = __builtin_fmaxf(mi, __builtin_fabsf(v - x[e - d]));
  }
  __shared__ float red[2][4];
  mi = wave_max(mi);
  mp = wave_max(mp);
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = mi;
    red[1][threadIdx.x >> 6] = mp;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    mi = __builtin_fmaxf(__builtin_fmaxf(red[0][0], red[0][1]), __builtin_fmaxf(red[0][2], red[0][3]));
    mp = __builtin_fmaxf(__builtin_fmaxf(red[1][0], red[1][1]), __builtin_fmaxf(red[1][2], red[1][3]));
    float *sc = R + (long long)s * mf_rec_floats(d, l) + mf_scale_off(d, l);
    const f2 a = mf_scale_of(mi), b = mf_scale_of(mp);
    sc[0] = a[0];
    sc[1] = a[1];
    sc[2] = b[0];
    sc[3] = b[1];
  }
}

// The A-side scale of every aug row (x_0, dx_t; 1 past the sequence), after mf_aug_kernel
__global__ __launch_bounds__(256) void mf_rowscale_kernel(int n, int l, int d, float *__restrict__ R) {
  const int rows = mf_rows(l), kp = mf_kp(d);
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long long)n * rows) return;
  const int t = (int)(idx % rows);
  const int s = (int)(idx / rows);
  float *__restrict__ base = R + (long long)s * mf_rec_floats(d, l);
  const float *__restrict__ row = base + (long long)t * kp;
  float m = 0.0f;
  for (int k = 0; k < d; ++k) m = __builtin_fmaxf(m, __builtin_fabsf(row[k]));
  const f2 sc = mf_scale_of(m);
  float *__restrict__ rs = base + mf_rowsc_off(d, l);
  rs[t] = sc[0];
  rs[rows + t] = sc[1];
}

// aug rows as MF_NPMAX halves at their row scale (zero past KP); a kernel with 2 parts reads the first two
__global__ __launch_bounds__(256) void mf_half_kernel(int n, int l, int d, float *__restrict__ R) {
  const int rows = mf_rows(l), kp = mf_kp(d), kh = mf_kh(d);
  const long long rec = mf_rec_floats(d, l);
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long long)n * rows * (kh / 2)) return;
  const int k = 2 * (int)(idx % (kh / 2));
  const long long r = idx / (kh / 2);
  const int t = (int)(r % rows);
  const int s = (int)(r / rows);
  float *__restrict__ base = R + (long long)s * rec;
  const float sc = base[mf_rowsc_off(d, l) + rows + t];
  const f2 v = k < kp ? *reinterpret_cast<const f2 *>(base + (long long)t * kp + k) : (f2){0.0f, 0.0f};
  const MfParts<MF_NPMAX> s0 = mf_split<MF_NPMAX>(v[0], sc), s1 = mf_split<MF_NPMAX>(v[1], sc);
  _Float16 *__restrict__ hh = reinterpret_cast<_Float16 *>(base + mf_half_off(d, l)) + (long long)t * kh + k;
#pragma unroll
  for (int u = 0; u < MF_NPMAX; ++u) *reinterpret_cast<h2 *>(hh + (long long)u * rows * kh) = (h2){s0.h[u], s1.h[u]};
}

int mf_records(const float *X, int n, int l, int d, float *R, hipStream_t s) {
  if (n <= 0) return GPSIG_OK;
  const long long ta = (long long)n * mf_rows(l) * mf_kp(d), ts = (long long)n * mf_rows(l);
  const long long th = (long long)n * mf_rows(l) * (mf_kh(d) / 2);
  hipLaunchKernelGGL(mf_aug_kernel, dim3((unsigned)((ta + 255) / 256)), dim3(256), 0, s, X, n, l, d, R);
  hipLaunchKernelGGL(mf_scalars_kernel, dim3((unsigned)((ts + 255) / 256)), dim3(256), 0, s, X, n, l, d, R);
  hipLaunchKernelGGL(mf_scale_kernel, dim3((unsigned)n), dim3(256), 0, s, X, n, l, d, R);
  hipLaunchKernelGGL(mf_rowscale_kernel, dim3((unsigned)((ts + 255) / 256)), dim3(256), 0, s, n, l, d, R);
  hipLaunchKernelGGL(mf_half_kernel, dim3((unsigned)((th + 255) / 256)), dim3(256), 0, s, n, l, d, R);
  return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
}

size_t mf_records_bytes(int n, int l, int d) { return (size_t)n * (size_t)mf_rec_floats(d, l) * sizeof(float); }
bool mf_gram_applies(int d, int l2) { return mf_applies(d, l2); }
// carry scratch of a column-blocked launch (any level count)
size_t mf_gram_scratch_bytes(int l1, int l2, int d) {
  return mf_gram_applies(d, l2) && mf_nblk(l2) > 1 ? mf_carry_bytes(l1, mf_waves(d, l2)) : 0;
}

// a: the SigArgs of sig_gram_impl (pair mode UPPER / RECT, rows, outputs, state) with FX / FY the mf records;
// scratch: mf_gram_scratch_bytes(l1, l2, d) bytes (column blocks only).
int sig_fo_mf(const SigArgs &a0, int d, int seed, float *scratch, hipStream_t s) {
  if (!mf_applies(d, a0.l2) || a0.pair_mode == GPSIG_PAIRS_DIAG || a0.l1 < 2) return GPSIG_EUNSUPPORTED;
  MfArgs m{};
  m.p = a0;
  m.rx = mf_rec_floats(d, a0.l1);
  m.ry = mf_rec_floats(d, a0.l2);
  m.rowsx = mf_rows(a0.l1);
  m.rowsy = mf_rows(a0.l2);
  m.kp = mf_kp(d);
  m.d = d;
  m.nblk = mf_nblk(a0.l2);
  m.blk0 = 0;
  m.carry = scratch;
  m.cw = mf_cw(a0.M);
  if (m.nblk > 1 && a0.M > 1 && !scratch) return GPSIG_EWORKSPACE;
  const int xb = mf_waves(d, a0.l2) * MF_G;  // x-sequences per workgroup
  const int t0 = a0.row_begin / xb, t1 = (a0.row_end + xb - 1) / xb;
  long long nblocks;
  if (a0.pair_mode == GPSIG_PAIRS_UPPER) {
    auto P = [&](long long r) { return r * a0.n2 - (long long)xb * r * (r - 1) / 2; };
    m.p.tile_base = P(t0);
    nblocks = P(t1) - P(t0);
  } else {
    m.p.tile_base = (long long)t0 * a0.n2;
    nblocks = (long long)(t1 - t0) * a0.n2;
  }
  if (nblocks <= 0) return GPSIG_OK;
  if (nblocks > 0x7fffffffLL) return GPSIG_EUNSUPPORTED;
  switch (a0.M) {
    case 1: return sig_fo_mf_launch_m<1>(m, seed, nblocks, s);
    case 2: return sig_fo_mf_launch_m<2>(m, seed, nblocks, s);
    case 3: return sig_fo_mf_launch_m<3>(m, seed, nblocks, s);
    case 4: return sig_fo_mf_launch_m<4>(m, seed, nblocks, s);
    case 5: return sig_fo_mf_launch_m<5>(m, seed, nblocks, s);
    case 6: return sig_fo_mf_launch_m<6>(m, seed, nblocks, s);
    case 7: return sig_fo_mf_launch_m<7>(m, seed, nblocks, s);
    case 8: return sig_fo_mf_launch_m<8>(m, seed, nblocks, s);
    default: return GPSIG_EUNSUPPORTED;
  }
}

int sig_fo_mf_cells_launch(const MfArgs &a, long long nblocks, hipStream_t s);

// The RBF difference-seed cells of the pairs of rows [row_begin, row_end) (pair_mode RECT / UPPER: against every
// / every later y-sequence; DIAG: (a, a)) into the higher-order recursion's tile: cell (i, j) of pair (a, b) at
// dm + (a - dm_a0) dm_as + (b - dm_b0) dm_bs + i dm_ld + j.  FX / FY: mf records of X and Y (mf_records).
int sig_fo_mf_cells(const float *FX, int n1, int l1, const float *FY, int n2, int l2, int d, int pair_mode,
                    int row_begin, int row_end, float *dm, int dm_a0, int dm_b0, long long dm_as, long long dm_bs,
                    long long dm_ld, hipStream_t s) {
  if (!mf_applies(d, l2) || l1 < 2 || l2 < 2) return GPSIG_EUNSUPPORTED;
  MfArgs m{};
  m.p.FX = FX;
  m.p.FY = FY;
  m.p.n1 = n1; m.p.l1 = l1; m.p.n2 = n2; m.p.l2 = l2;
  m.p.M = 1;
  m.p.pair_mode = pair_mode;
  m.p.row_begin = row_begin;
  m.p.row_end = row_end;
  m.rx = mf_rec_floats(d, l1);
  m.ry = mf_rec_floats(d, l2);
  m.rowsx = mf_rows(l1);
  m.rowsy = mf_rows(l2);
  m.kp = mf_kp(d);
  m.d = d;
  m.nblk = mf_nblk(l2);
  m.dm = dm;
  m.dm_a0 = dm_a0;
  m.dm_b0 = dm_b0;
  m.dm_as = dm_as;
  m.dm_bs = dm_bs;
  m.dm_ld = dm_ld;
  const int xb = mf_waves(d, l2) * MF_G;
  long long nblocks;
  if (pair_mode == GPSIG_PAIRS_DIAG) {
    m.p.tile_base = 0;
    nblocks = row_end - row_begin;
  } else {
    const int t0 = row_begin / xb, t1 = (row_end + xb - 1) / xb;
    if (pair_mode == GPSIG_PAIRS_UPPER) {
      auto P = [&](long long r) { return r * n2 - (long long)xb * r * (r - 1) / 2; };
      m.p.tile_base = P(t0);
      nblocks = P(t1) - P(t0);
    } else {
      m.p.tile_base = (long long)t0 * n2;
      nblocks = (long long)(t1 - t0) * n2;
    }
  }
  if (nblocks <= 0) return GPSIG_OK;
  if (nblocks > 0x7fffffffLL) return GPSIG_EUNSUPPORTED;
  return sig_fo_mf_cells_launch(m, nblocks, s);
}

}  // namespace gpsig
