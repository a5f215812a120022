// gpsig_amd -- first-order Gram at wide channel counts with the increment inner products on the matrix cores.
//
// The reference builds the base-kernel grid of a pair with one GEMM over the channels (_square_dist,
// gpsig/kernels.py:946-957; the linear kernel's tf.matmul, :1042-1044) and then runs the recursion of
// signature_algs.py:8-35 on it.  The runtime-channel-loop kernel (wide.h) keeps that GEMM on the VALU,
// where each channel costs a dependent column load and the waves sit in s_waitcnt.  Here the GEMM is an
// MFMA producer inside the recursion kernel:
//
//   * a workgroup = 8 waves = 32 x-sequences (4 per wave, one per 16-lane group; 4 waves when the LDS is
//     short) against ONE y-sequence b.
//     b's columns are the GEMM's B operand and stay in LDS for the workgroup's whole life;
//   * per chunk of 4 rows, each wave multiplies its 4 x-sequences' rows (16 GEMM rows, A operand straight
//     from HBM/L2) by B with v_mfma_f32_16x16x4_f32 and parks the 16 x LPW result in its own LDS tile;
//   * the wave's lane groups then stream those rows through the fixed kernels' recursion (sig_fo.h), reading
//     their W columns per lane from the tile.
//
// GEMM operands per sequence (mf records, mf_records_kernel): row 0 = x_0, row t = x_t - x_{t-1}.  On the B
// side column j < LPW-1 is row j+1 (the increment dy_j) and column LPW-1 is row 0 (the point y_0), so one
// LP x W tile row of pair (a, b) holds, for x-row t >= 1 (cell row i = t-1),
//     c_ij = <dx_i, dy_j>   (every cell)        and      <dx_i, y_0>   (last column)
// and for t = 0 the values Q_0j = <x_0, dy_j>.  Everything else the RBF cell needs follows by exact
// identities (sig_common.h RbfSeedPk):
//     p_i0 = <dx_i, y_0> - g_i,   p_{i,j+1} = p_ij + c_ij          (a scan of c along the row)
//     q_ij = Q_ij - h_j,          Q_{i+1,j} = Q_ij + c_ij          (h_j = <y_j, dy_j> + |dy_j|^2/2)
//     e_ij = -|x_i - y_j|^2 / 2,  e_{i+1,j} = e_ij + p_ij,  e_{0,j+1} = e_0j + q_0j   (e_00 exact)
// k = exp(e) and expm1(q) by the exp-free recurrences between anchor rows, re-anchored from e and Q.
#pragma once
#include <stdlib.h>
#include "sig_common.h"

namespace gpsig {

constexpr int MF_G = 4;                     // lane groups (x-sequences) per wave
constexpr int MF_LP = 16;                   // lanes per pair (one DPP row)
constexpr size_t MF_LDS_MAX = 160 * 1024;

// fp32 record rows are padded to KP = 4 KQ (KQ = ceil(d / 4) rounded up to even) channels.
__host__ __device__ inline int mf_kq(int d) {
  const int q = (d + 3) / 4;
  return q + (q & 1);
}
__host__ __device__ inline int mf_kp(int d) { return 4 * mf_kq(d); }
// The GEMM runs on v_mfma_f32_16x16x32_f16 with every fp32 operand split into NP halves at a power-of-two
// scale, a = 2^-e (h_0 + h_1 [+ h_2]), h_u = f16 of what the previous parts left: the products h_u h'_v with
// u + v < NP carry 22 (NP = 2) or 33 (NP = 3) bits of every product, exact in the fp32 accumulator (16
// cycles per 16x16x32 against 32 per 16x16x4 for the f32 form: 3 or 6 MFMAs per 32 channels instead of 8).
// The scales keep the low parts above the f16 subnormal range, which the matrix cores flush: the A rows (x_0,
// dx_t) each at their own 2^e (largest |component| in [2^14, 2^15)), the B side at one scale for y's
// increments and one for its points.  K is padded to KH = 32 multiples.
__host__ __device__ inline int mf_kh(int d) { return (d + 31) & ~31; }
constexpr int MF_NPMAX = 3;
// B image in LDS: column j at j LDBH halves, parts u at u KH, + 8 halves of padding (a column stride of
// 4 mod 16 dwords for every KH: the 16 columns of a ds_read_b128 start on distinct 4-bank groups)
__host__ __device__ inline int mf_ldbh(int d, int np) { return np * mf_kh(d) + 8; }
// columns per lane by sequence length: one tile of LP W columns up to 160 points, past that W = 8 in column
// blocks of LPW - 1 = 127 cells (the block's last column is the point of its first cell, below)
__host__ __device__ inline int mf_w(int l) { return l <= 64 ? 4 : (l <= 128 ? 8 : (l <= 160 ? 10 : 8)); }
__host__ __device__ inline int mf_lpw(int l) { return MF_LP * mf_w(l); }
__host__ __device__ inline int mf_nblk(int l) { return l <= 160 ? 1 : (l - 2) / (8 * MF_LP - 1) + 1; }
// record rows: the chunked x side reads rows in fours, the B side LPW rows (a blocked B side up to nblk 127)
__host__ __device__ inline int mf_rows(int l) {
  if (l > 160) return (l + 127 + 3) & ~3;
  const int r = (l + 3) & ~3, w = mf_lpw(l);
  return r > w ? r : w;
}
// record of a sequence (floats): [aug: rows x KP][points: rows x KP][hd: rows][gg: rows]
// [B scales: 2^-e_inc, 2^e_inc, 2^-e_pt, 2^e_pt][A row scales: 2^-e_t (rows), 2^e_t (rows)]
// [aug parts u = 0..2: rows x KH halves each]
//   aug row 0 = x_0, aug row t = x_t - x_{t-1} (1 <= t < l), points row t = x_t; zero past l and past d
//   (every section 16-byte aligned: rows is a multiple of 4, KP of 8, KH of 32)
__host__ __device__ inline long long mf_scale_off(int d, int l) { return 2LL * mf_rows(l) * mf_kp(d) + 2LL * mf_rows(l); }
__host__ __device__ inline long long mf_rowsc_off(int d, int l) { return mf_scale_off(d, l) + 4; }
__host__ __device__ inline long long mf_half_off(int d, int l) { return mf_rowsc_off(d, l) + 2LL * mf_rows(l); }
__host__ __device__ inline long long mf_rec_floats(int d, int l) {
  return mf_half_off(d, l) + (long long)mf_rows(l) * mf_kh(d) * MF_NPMAX / 2;
}
inline size_t mf_lds_bytes(int d, int l2, int nw, int np) {
  const size_t lpw = (size_t)mf_lpw(l2);
  return lpw * (size_t)mf_ldbh(d, np) * 2 + (size_t)nw * 16 * (lpw + 4) * sizeof(float);
}
// Launch geometry by LDS: 8 waves per workgroup (two per SIMD, so one wave's matrix-core phase overlaps
// another's recursion) when the LDS allows, else 4; 0: no tile geometry.  Operand parts: 2 (22 bits); with
// GPSIG_MF_PARTS=3 three (33 bits) where the B image fits.  The third part buys little: the matrix cores align
// a product block to its largest term and truncate below it (tools/mfma_f16_probe.hip: -0.52 ulp mean on
// positive terms spread over 2^8), which the recurrences' running sums then accumulate; per-level error vs
// fp64 1.0-1.2e-6 (2 parts) against 0.9-1.1e-6 (3 parts) at 500 points, 1.2-1.5e-7 for the fp32 channel loop
// (GPSIG_WIDE_MF=0), at 1.2x the time.  GPSIG_MF_NW=4 pins 4 waves (A/B runs).
struct MfGeo {
  int nw, np;
};
inline MfGeo mf_geo(int d, int l2) {
  if (mf_w(l2) == 0) return {0, 0};
  static const int parts = [] { const char *e = getenv("GPSIG_MF_PARTS"); return e ? atoi(e) : 2; }();
  static const bool four = [] { const char *e = getenv("GPSIG_MF_NW"); return e && e[0] == '4'; }();
  for (int nw : {8, 4}) {
    if (nw == 8 && four) continue;
    if (parts == 3 && mf_lds_bytes(d, l2, nw, 3) <= MF_LDS_MAX) return {nw, 3};
    if (mf_lds_bytes(d, l2, nw, 2) <= MF_LDS_MAX) return {nw, 2};
  }
  return {0, 0};
}
inline int mf_waves(int d, int l2) { return mf_geo(d, l2).nw; }
inline bool mf_applies(int d, int l2) { return mf_waves(d, l2) != 0; }

struct MfArgs {
  SigArgs p;          // pair mode, rows, outputs, normalisation, state; FX / FY = mf records
  long long rx, ry;   // record strides (floats)
  int rowsx, rowsy;   // record rows
  int kp, d;
  int nblk;           // column blocks of the y side
  long long blk0;     // first logical workgroup of a chunked launch (column blocks)
  float *carry;       // column blocks, M > 1: per launched workgroup XB pairs x (l1 - 1) rows x cw floats
  int cw;
  // cell producer (DMO instantiations, the higher-order recursion past 32 channels with the RBF base kernel):
  // cell (i, j) of pair (a, b) to dm + (a - dm_a0) dm_as + (b - dm_b0) dm_bs + i dm_ld + j, no recursion
  float *dm;
  long long dm_as, dm_bs, dm_ld;
  int dm_a0, dm_b0;
};
// Column-blocked launches are chunked so that the carry scratch stays bounded
constexpr int MF_BLK_CHUNK = 256;
inline int mf_cw(int M) { return M <= 5 ? 4 : 8; }
inline size_t mf_carry_bytes(int l1, int nw) { return (size_t)MF_BLK_CHUNK * nw * MF_G * (size_t)(l1 > 1 ? l1 - 1 : 1) * 8 * sizeof(float); }

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
// v_mfma_f32_16x16x32_f16: lane l supplies A[l & 15][8 (l >> 4) + e] and B[8 (l >> 4) + e][l & 15], e < 8;
// D row 4 (l >> 4) + r, col l & 15
GPSIG_DEV f4 mfma16h(h8 a, h8 b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0); }
// v = 2^-e (h_0 + ... + h_{NP-1}) at the scale 2^e
template <int NP>
struct MfParts {
  _Float16 h[NP];
};
template <int NP>
GPSIG_DEV MfParts<NP> mf_split(float v, float sc) {
  MfParts<NP> r;
  float b = v * sc;
#pragma unroll
  for (int u = 0; u < NP; ++u) {
    r.h[u] = (_Float16)b;
    b -= (float)r.h[u];
  }
  return r;
}

// Wavefront-scope ordering of the wave's own LDS tile between its lanes (writes by one lane, reads by another)
GPSIG_DEV void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int NW, int W, int M, int SEED, bool SAVE, bool BLK, bool DMO = false, int NP = 3>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(NW / 4))) void sig_fo_mf_kernel(MfArgs q) {
  static_assert(SEED == SEED_RBF_DIFF || SEED == SEED_LIN_DIFF, "difference seeds");
  static_assert(!BLK || W == 8, "column blocks at W = 8");
  static_assert(!DMO || (M == 1 && !SAVE), "cell producer: no recursion");
  constexpr bool RBF = SEED == SEED_RBF_DIFF;
  constexpr int LP = MF_LP, W2 = W / 2, LPW = LP * W, NCB = LPW / 16, ML = M > 1 ? M - 1 : 1;
  constexpr int LDC = LPW + 4;
  constexpr float L2E = 1.4426950408889634f;
  constexpr int ANCH = GPSIG_PK_ANCHOR;
  constexpr int XB = NW * MF_G;  // x-sequences per workgroup
  constexpr int CPB = LPW - 1;   // cells per column block
  const SigArgs &p = q.p;
  extern __shared__ __attribute__((aligned(16))) float mf_lds[];
  const int KP = q.kp, KH = mf_kh(q.d), LDBH = NP * KH + 8;
  _Float16 *__restrict__ Bs = reinterpret_cast<_Float16 *>(mf_lds);
  const int lane = (int)threadIdx.x & 63;
  const int wave = wave_uniform((int)threadIdx.x >> 6);
  float *__restrict__ Cs = mf_lds + LPW * LDBH / 2 + wave * 16 * LDC;
  const int g = lane >> 4, gl = lane & 15;

  // ---- tile: x-block tx (XB sequences) against y-sequence b
  int tx, b;
  {
    const long long t = p.tile_base + q.blk0 + (long long)blockIdx.x;
    if (p.pair_mode == GPSIG_PAIRS_DIAG) {  // pairs (b, b): the x-block holding b, one live group
      b = p.row_begin + (int)t;
      tx = b / XB;
    } else if (p.pair_mode == GPSIG_PAIRS_UPPER) {
      const Tile tl = upper_tile(t, p.n2, XB);
      tx = tl.ta;
      b = tl.tb;
    } else {
      tx = (int)(t / p.n2);
      b = (int)(t % p.n2);
    }
  }
  const float *__restrict__ fyb = p.FY + (long long)b * q.ry;
  const float *__restrict__ pty = fyb + (long long)q.rowsy * KP;  // y's points
  // y's scales: increments (B columns < LPW - 1) and points (the last column)
  const float *__restrict__ ysc = fyb + mf_scale_off(q.d, p.l2);
  const float syi = ysc[1], syp = ysc[3], rsyi = ysc[0], rsyp = ysc[2];
  // B image of column block j0: column jj < LPW - 1 = aug row j0 + jj + 1 (dy_{j0+jj}), column LPW - 1 = the
  // point y_{j0}, split into halves at y's scale: column j at j LDBH, hi at k, lo at KH + k
  auto load_b = [&](int j0) {
    const int k2n = KH / 2;
    for (int e = (int)threadIdx.x; e < LPW * k2n; e += 64 * NW) {
      const int j = e / k2n, k = 2 * (e - j * k2n);
      const float *src = j + 1 == LPW ? pty + (long long)j0 * KP : fyb + (long long)(j0 + j + 1) * KP;
      const f2 v = k < KP ? *reinterpret_cast<const f2 *>(src + k) : (f2){0.0f, 0.0f};
      const float sy = j + 1 == LPW ? syp : syi;
      const MfParts<NP> s0 = mf_split<NP>(v[0], sy), s1 = mf_split<NP>(v[1], sy);
#pragma unroll
      for (int u = 0; u < NP; ++u) *reinterpret_cast<h2 *>(Bs + j * LDBH + u * KH + k) = (h2){s0.h[u], s1.h[u]};
    }
  };
  load_b(0);
  __syncthreads();

  const int a = tx * XB + wave * MF_G + g;
  bool pair_ok = a < p.n1 && a >= p.row_begin && a < p.row_end;
  if (p.pair_mode == GPSIG_PAIRS_UPPER) pair_ok = pair_ok && b >= a;
  if (p.pair_mode == GPSIG_PAIRS_DIAG) pair_ok = pair_ok && b == a;
  const bool live = __builtin_amdgcn_ballot_w64(pair_ok) != 0;  // wave-uniform
  if (!BLK && !live) return;                                     // no barrier follows without column blocks
  const int al = a < p.n1 ? a : p.n1 - 1;
  const float *__restrict__ fx = p.FX + (long long)al * q.rx;
  const float *__restrict__ hdx = fx + 2LL * q.rowsx * KP;
  const float *__restrict__ hdyp = fyb + 2LL * q.rowsy * KP;
  const float *__restrict__ ggyp = hdyp + q.rowsy;
  const int nrows = p.l1 - 1, ncell = p.l2 - 1;
  const int nchunk = (p.l1 + 3) / 4;
  const int nblk = BLK ? q.nblk : 1;
  const bool carries = BLK && M > 1 && nblk > 1;

  // ---- GEMM of one chunk (x-rows 4 ch .. 4 ch + 3 of the wave's four sequences) into the wave's tile
  // A operand of lane l: GEMM row m = l & 15 = 4 (x-sequence) + (chunk row), halves 8 (l >> 4) .. + 7 of
  // every 32-channel step, from the x record's hi / lo rows
  const _Float16 *__restrict__ Asrc;
  {
    const int am = lane & 15;
    const int aa = tx * XB + wave * MF_G + (am >> 2);
    Asrc = reinterpret_cast<const _Float16 *>(p.FX + (long long)(aa < p.n1 ? aa : p.n1 - 1) * q.rx +
                                              mf_half_off(q.d, p.l1)) + (am & 3) * KH + 8 * (lane >> 4);
  }
  const long long ALO = (long long)q.rowsx * KH;  // part u of the rows at u ALO (halves)
  const _Float16 *__restrict__ Bl = Bs + (lane & 15) * LDBH + 8 * (lane >> 4);
  // D rows of lane l are rows 4 ch + r of x-sequence l >> 4: 2^-(e_row + e_col) undoes both scales (exact)
  const float *__restrict__ xrs;
  {
    const int aw = tx * XB + wave * MF_G + (lane >> 4);
    xrs = p.FX + (long long)(aw < p.n1 ? aw : p.n1 - 1) * q.rx + mf_rowsc_off(q.d, p.l1);
  }
  // the last tile column holds <dx_i, y_{j0}>: its writers subtract g_i there, so the tile carries p_{i,j0}
  const float *__restrict__ ggw;
  {
    const int aw = tx * XB + wave * MF_G + (lane >> 4);
    ggw = p.FX + (long long)(aw < p.n1 ? aw : p.n1 - 1) * q.rx + 2LL * q.rowsx * KP + q.rowsx;
  }
  // column-block carries of this workgroup's pairs: [XB][nrows][cw] (written by block k, read by block k + 1)
  float *__restrict__ carry_wg = carries ? q.carry + (long long)blockIdx.x * XB * nrows * q.cw : nullptr;
  float cinr[BLK && M > 1 ? 4 : 1][ML];  // the current chunk's carries (column blocks)
  auto gemm_chunk = [&](int ch, int blk) {
    // the chunk's carries into registers: every lane of group g loads its group's 4 rows x (M - 1) levels,
    // through L2 (agent scope: the previous block's stores landed there)
    if constexpr (BLK && M > 1) {
      if (carries) {
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int i = 4 * ch + rr - 1;
          const bool ok = blk > 0 && i >= 0 && i < nrows;
          const float *src = carry_wg + ((long long)(wave * MF_G + g) * nrows + (ok ? i : 0)) * q.cw;
#pragma unroll
          for (int m = 0; m < ML; ++m)
            cinr[rr][m] = ok ? __hip_atomic_load(src + m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0f;
        }
      }
    }
    f4 acc[NCB];
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) acc[cb] = (f4){0.0f, 0.0f, 0.0f, 0.0f};
    const _Float16 *__restrict__ ap = Asrc + (long long)ch * 4 * KH;
    const f4 rsc = *reinterpret_cast<const f4 *>(xrs + 4 * ch);  // 2^-e of the chunk's 4 rows
    h8 na[NP];
#pragma unroll
    for (int u = 0; u < NP; ++u) na[u] = *reinterpret_cast<const h8 *>(ap + u * ALO);
    for (int s = 0; s < KH; s += 32) {
      h8 av[NP];
#pragma unroll
      for (int u = 0; u < NP; ++u) av[u] = na[u];
      if (s + 32 < KH) {
#pragma unroll
        for (int u = 0; u < NP; ++u) na[u] = *reinterpret_cast<const h8 *>(ap + u * ALO + s + 32);
      }
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        h8 bv[NP];
#pragma unroll
        for (int u = 0; u < NP; ++u) bv[u] = *reinterpret_cast<const h8 *>(Bl + cb * 16 * LDBH + u * KH + s);
        // the products of parts u + v < NP, smallest first: (lo, hi), (hi, lo) [, (mid, mid) ...], (hi, hi)
#pragma unroll
        for (int t = NP - 1; t >= 0; --t)
#pragma unroll
          for (int u = t; u >= 0; --u) acc[cb] = mfma16h(av[u], bv[t - u], acc[cb]);
      }
    }
    wave_lds_sync();  // the previous chunk's rows are read
    // D: lane l holds rows 4 (l >> 4) + r (x-sequence l >> 4, chunk row r), column 16 cb + (l & 15);
    // tile row of (sequence g, chunk row r) = 4 r + g
    const int gq = lane >> 4, col = lane & 15;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int t = 4 * ch + r;  // x-row of the record
      float *__restrict__ crow = Cs + (4 * r + gq) * LDC + col;
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        float v = acc[cb][r] * (rsc[r] * (cb == NCB - 1 && col == 15 ? rsyp : rsyi));
        if (cb == NCB - 1 && col == 15 && t >= 1 && t - 1 < nrows) v -= ggw[t - 1];
        crow[16 * cb] = v;
      }
    }
    wave_lds_sync();
  };

  const bool valid_last = gl != LP - 1;  // the last lane's last column is the block's point column, never a cell
  float Kacc[M];
#pragma unroll
  for (int m = 0; m < M; ++m) Kacc[m] = 0.0f;

  for (int blk = 0; blk < nblk; ++blk) {
    const int j0 = blk * CPB;
    if (BLK && blk > 0) {
      // every wave is done with the previous block's B image; its carry stores are at L2
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      __syncthreads();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      load_b(j0);
      __syncthreads();
    }
    if (BLK && !live) continue;

    // ---- lane state: W columns jj = gl W + w of the block (cell j0 + jj), column pair w2 = (w2, w2 + W/2)
    f2 C[M][W2];
#pragma unroll
    for (int m = 0; m < M; ++m)
#pragma unroll
      for (int w2 = 0; w2 < W2; ++w2) C[m][w2] = splat2(0.0f);
    f2 hh[W2], Eq[W2], kc[W2], ev[W2], Qv[W2];
    float kcR = 0.0f;
    bool clo = false;

    // tile row (sequence g, chunk row r) into column pairs; the point column of the last lane reads as 0
    auto read_row = [&](int r, f2 (&v)[W2], float &last) {
      const float *__restrict__ crow = Cs + (4 * r + g) * LDC;
      float t[W];
      if constexpr (W % 4 == 0) {
#pragma unroll
        for (int h = 0; h < W / 4; ++h) {
          const f4 x = *reinterpret_cast<const f4 *>(crow + gl * W + 4 * h);
#pragma unroll
          for (int e = 0; e < 4; ++e) t[4 * h + e] = x[e];
        }
      } else {
#pragma unroll
        for (int h = 0; h < W / 2; ++h) {
          const f2 x = *reinterpret_cast<const f2 *>(crow + gl * W + 2 * h);
          t[2 * h] = x[0];
          t[2 * h + 1] = x[1];
        }
      }
      if (!valid_last) t[W - 1] = 0.0f;
#pragma unroll
      for (int w2 = 0; w2 < W2; ++w2) v[w2] = (f2){t[w2], t[w2 + W2]};
      last = crow[LPW - 1];
    };

    if constexpr (RBF) {
      // y-side column data: h_j = <y_j, dy_j> + |dy_j|^2/2, |dy_j|^2/2 (0 past the cells)
      float hy = 0.0f;
#pragma unroll
      for (int w2 = 0; w2 < W2; ++w2)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int jj = gl * W + w2 + h * W2;
          const bool cell = j0 + jj < ncell && jj < CPB;
          hh[w2][h] = cell ? ggyp[j0 + jj] : 0.0f;
          hy = __builtin_fmaxf(hy, cell ? hdyp[j0 + jj] : 0.0f);
        }
      // |c_ij| <= 2 sqrt(hdx_i hdy_j): the cubic expm1(c) when the wave's bound allows (RbfSeedPk::bound_c)
      float hx = 0.0f;
      for (int i = gl; i < nrows; i += LP) hx = __builtin_fmaxf(hx, hdx[i]);
      hx = wave_max(hx);
      hy = wave_max(hy);
      clo = wave_uniform(4.0f * hx * hy < 0.98f * EM1_LO_TAU * EM1_LO_TAU ? 1 : 0) != 0;
    }

    // ---- chunk 0: its row 0 (x_0) seeds the state, its rows 1..3 are cell rows 0..2
    gemm_chunk(0, blk);
    if constexpr (RBF) {
      float dummy;
      read_row(0, Qv, dummy);
      // e_{0,j0} = -|x_0 - y_{j0}|^2 / 2 (x_0 = record row 0, y_{j0} = the B image's last column), the group's
      // lanes splitting the channels
      float s00 = 0.0f;
      for (int k = gl; k < q.d; k += LP) {
        const float df = fx[k] - pty[(long long)j0 * KP + k];
        s00 = __builtin_fmaf(df, df, s00);
      }
      const float e00 = -0.5f * group_sum<LP>(s00);
      // e_0j = e_{0,j0} + sum_{j0 <= j' < j} q_0j' (exclusive prefix along the row: in-lane, then across the group)
      f2 qv[W2], pre[W2 + 1];
      pre[0] = splat2(0.0f);
#pragma unroll
      for (int w2 = 0; w2 < W2; ++w2) {
        qv[w2] = Qv[w2] - hh[w2];
        pre[w2 + 1] = pre[w2] + qv[w2];
      }
      float tq[1] = {pre[W2][0] + pre[W2][1]};
      const float tq0 = tq[0];
      group_incl_scan_n<LP, 1>(tq);
      const float bq = e00 + (tq[0] - tq0);
#pragma unroll
      for (int w2 = 0; w2 < W2; ++w2) {
        ev[w2] = splat2(bq) + (f2){pre[w2][0], pre[W2][0] + pre[w2][1]};
        Eq[w2] = em1_small2(qv[w2]);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          kc[w2][h] = __builtin_amdgcn_exp2f(ev[w2][h] * L2E);
          if (!(__builtin_fabsf(qv[w2][h]) < EM1_TAU)) Eq[w2][h] = __builtin_amdgcn_exp2f(qv[w2][h] * L2E) - 1.0f;
        }
      }
      kcR = lane_next(kc[0][0]);
    }

    // ---- one cell row: cells, then the level recursion (sig_fo.h do_row)
    auto do_row = [&](auto clo_t, int i, int r) {
      constexpr bool CLO = decltype(clo_t)::value;
      f2 c[W2];
      float p0;
      read_row(r, c, p0);
      constexpr int NS = (M > 1 ? ML : 0) + (RBF ? 1 : 0);
      f2 E[ML][W2 + 1];
      float T[NS > 0 ? NS : 1], base[NS > 0 ? NS : 1];
#pragma unroll
      for (int m = 0; m + 1 < M; ++m) {
        E[m][1] = C[m][0];
#pragma unroll
        for (int k = 2; k <= W2; ++k) E[m][k] = E[m][k - 1] + C[m][k - 1];
        T[m] = E[m][W2][0] + E[m][W2][1];
        base[m] = T[m];
      }
      f2 slo = splat2(0.0f);
      if constexpr (RBF) {
#pragma unroll
        for (int w2 = 0; w2 < W2; ++w2) slo += c[w2];
        T[NS - 1] = slo[0] + slo[1];
        base[NS - 1] = T[NS - 1];
      }
      if constexpr (NS > 0) group_incl_scan_n<LP, NS>(base);
      if constexpr (BLK && M > 1) {
        if (carries) {
          // the levels' column sums of the blocks to the left: into this block's prefix, and on to the next
          float *__restrict__ cout = carry_wg + ((long long)(wave * MF_G + g) * nrows + i) * q.cw;
#pragma unroll
          for (int m = 0; m < ML; ++m) {
            const float ci = cinr[r][m];
            if (gl == LP - 1 && blk + 1 < nblk)
              __hip_atomic_store(cout + m, ci + base[m], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            base[m] += ci;
          }
        }
      }
      f2 dM[W2];
      if constexpr (RBF) {
        // p at the lane's columns 0 and W/2 from p_{i,j0} and the exclusive prefix of c along the row
        f2 pv[W2];
        const float pl0 = p0 + (base[NS - 1] - T[NS - 1]);
        pv[0] = (f2){pl0, pl0 + slo[0]};
#pragma unroll
        for (int w2 = 1; w2 < W2; ++w2) pv[w2] = pv[w2 - 1] + c[w2 - 1];
        f2 Ec[W2], Ep[W2];
        if constexpr (CLO)
          em1_lo2_n<W2>(c, Ec);
        else
          em1_small2_n<W2>(c, Ec);
        Ep[0] = em1_small2(pv[0]);
        float mx = 0.0f;
#pragma unroll
        for (int w2 = 0; w2 < W2; ++w2) {
          const f2 t = fma2(Ep[w2], Ec[w2], Ec[w2]);
          if (w2 + 1 < W2) Ep[w2 + 1] = Ep[w2] + t;
          const f2 t2 = fma2(Eq[w2], t, t);
          dM[w2] = kc[w2] * fma2(Ep[w2], Eq[w2], t2);
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            if constexpr (CLO) {  // only the first pair's p meets a polynomial (RbfSeedPk::row)
              if (w2 == 0 || !GPSIG_P0CHECK) mx = __builtin_fmaxf(mx, __builtin_fabsf(pv[w2][h]));
            } else {
              mx = __builtin_fmaxf(__builtin_fmaxf(mx, __builtin_fabsf(pv[w2][h])), __builtin_fabsf(c[w2][h]));
            }
          }
        }
        // exact state of the next row: e_{i+1} = e_i + p_i, Q_{i+1} = Q_i + c_i
#pragma unroll
        for (int w2 = 0; w2 < W2; ++w2) {
          ev[w2] += pv[w2];
          Qv[w2] += c[w2];
        }
        const bool slow = __builtin_amdgcn_ballot_w64(mx >= EM1_TAU) != 0;
        const bool anch = (i % ANCH) == ANCH - 1;
        if (anch || slow) {
          f2 Eqn[W2], kn[W2];
#pragma unroll
          for (int w2 = 0; w2 < W2; ++w2) {
            const f2 qn = Qv[w2] - hh[w2];
            Eqn[w2] = em1_small2(qn);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              kn[w2][h] = __builtin_amdgcn_exp2f(ev[w2][h] * L2E);
              if (!(__builtin_fabsf(qn[h]) < EM1_TAU)) Eqn[w2][h] = __builtin_amdgcn_exp2f(qn[h] * L2E) - 1.0f;
            }
          }
          const float knR = lane_next(kn[0][0]);
          if (slow) {
            // every in-range cell from its own p, the others by the corner difference (RbfSeedPk::row)
            f2 Epd[W2], Ecd[W2];
            em1_small2_n<W2>(pv, Epd);
            em1_small2_n<W2>(c, Ecd);
#pragma unroll
            for (int w = 0; w < W; ++w) {
              const int w2 = w % W2, h = w / W2;
              const float kn1 = (w + 1 < W) ? kn[(w + 1) % W2][(w + 1) / W2] : knR;
              const float kc1 = (w + 1 < W) ? kc[(w + 1) % W2][(w + 1) / W2] : kcR;
              const float naive = (kn1 - kn[w2][h]) - (kc1 - kc[w2][h]);
              const float m = __builtin_fmaxf(__builtin_fabsf(pv[w2][h]), __builtin_fabsf(c[w2][h]));
              float t = __builtin_fmaf(Epd[w2][h], Ecd[w2][h], Ecd[w2][h]);
              t = __builtin_fmaf(Eq[w2][h], t, t);
              const float prod = kc[w2][h] * __builtin_fmaf(Epd[w2][h], Eq[w2][h], t);
              float v = m < EM1_TAU ? prod : naive;
              if (w + 1 == W && !valid_last) v = 0.0f;
              dM[w2][h] = v;
            }
          }
#pragma unroll
          for (int w2 = 0; w2 < W2; ++w2) {
            Eq[w2] = Eqn[w2];
            kc[w2] = kn[w2];
          }
          kcR = knR;
        } else {
#pragma unroll
          for (int w2 = 0; w2 < W2; ++w2) {
            kc[w2] = fma2(kc[w2], Ep[w2], kc[w2]);
            Eq[w2] = fma2(Eq[w2], Ec[w2], Eq[w2] + Ec[w2]);
          }
          kcR = lane_next(kc[0][0]);
        }
      } else {
#pragma unroll
        for (int w2 = 0; w2 < W2; ++w2) dM[w2] = c[w2];
      }
      if constexpr (DMO) {  // the cells to the tile of the higher-order recursion, which runs the levels
        if (pair_ok) {
          float *__restrict__ dst = q.dm + (long long)(a - q.dm_a0) * q.dm_as + (long long)(b - q.dm_b0) * q.dm_bs +
                                    (long long)i * q.dm_ld + j0;
#pragma unroll
          for (int w2 = 0; w2 < W2; ++w2)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const int jj = gl * W + w2 + h * W2;
              if (jj < CPB && j0 + jj < ncell) dst[jj] = dM[w2][h];
            }
        }
        return;
      }
      // level recursion, descending m (level m reads C_m through E before level m-1 writes it)
#pragma unroll
      for (int m = M - 2; m >= 0; --m) {
        f2 off;
        off[0] = base[m] - T[m];
        off[1] = off[0] + E[m][W2][0];
        C[m + 1][0] = fma2(dM[0], off, C[m + 1][0]);
#pragma unroll
        for (int k = 1; k < W2; ++k) C[m + 1][k] = fma2(dM[k], E[m][k] + off, C[m + 1][k]);
      }
#pragma unroll
      for (int w2 = 0; w2 < W2; ++w2) C[0][w2] += dM[w2];
    };

    auto run_rows = [&](auto clo_t) {
      // chunk 0: cell rows 0..2 at tile rows 1..3
      for (int r = 1; r < 4 && r - 1 < nrows; ++r) do_row(clo_t, r - 1, r);
      for (int ch = 1; ch < nchunk; ++ch) {
        gemm_chunk(ch, blk);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = 4 * ch + r - 1;
          if (i < nrows) do_row(clo_t, i, r);
        }
      }
    };
    if constexpr (M > 1 || DMO) {  // level 1 alone is the closed form
      if (RBF && clo)
        run_rows(std::true_type{});
      else
        run_rows(std::false_type{});
    }

    // ---- saved VJP state: column sums of levels 1..M-1
    if constexpr (SAVE) {
      if (pair_ok) {
        float *__restrict__ st = p.state + state_slot(a, b, p.n2, p.pair_mode == GPSIG_PAIRS_UPPER) * state_stride(M, p.l2);
#pragma unroll
        for (int m = 0; m + 1 < M; ++m)
#pragma unroll
          for (int w2 = 0; w2 < W2; ++w2)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const int jj = gl * W + w2 + h * W2;
              if (jj < CPB && j0 + jj < ncell) st[(long long)m * ncell + j0 + jj] = C[m][w2][h];
            }
      }
    }
#pragma unroll
    for (int m = 0; m < M; ++m) {
      f2 s2 = C[m][0];
#pragma unroll
      for (int w2 = 1; w2 < W2; ++w2) s2 += C[m][w2];
      Kacc[m] += group_sum<LP>(s2[0] + s2[1]);
    }
  }
  if (DMO || (BLK && !live)) return;

  float K[M + 1];
  K[0] = 1.0f;
#pragma unroll
  for (int m = 0; m < M; ++m) K[m + 1] = Kacc[m];
  // level 1 in closed form (level1_closed, fp64), the group's lanes splitting the channels
  {
    const float *__restrict__ x0 = fx + (long long)q.rowsx * KP, *__restrict__ xl = x0 + (long long)(p.l1 - 1) * KP;
    const float *__restrict__ y0 = pty, *__restrict__ yl = pty + (long long)(p.l2 - 1) * KP;
    double s[4] = {0.0, 0.0, 0.0, 0.0};
    for (int k = gl; k < q.d; k += LP) {
      const double xa = x0[k], xb = xl[k], ya = y0[k], yb = yl[k];
      if constexpr (RBF) {
        s[0] = __builtin_fma(xa - ya, xa - ya, s[0]);
        s[1] = __builtin_fma(xa - yb, xa - yb, s[1]);
        s[2] = __builtin_fma(xb - ya, xb - ya, s[2]);
        s[3] = __builtin_fma(xb - yb, xb - yb, s[3]);
      } else {
        s[0] = __builtin_fma(xb - xa, yb - ya, s[0]);
      }
    }
#pragma unroll
    for (int o = LP / 2; o >= 1; o >>= 1)
#pragma unroll
      for (int u = 0; u < 4; ++u) s[u] += __shfl_xor(s[u], o, 64);
    if constexpr (RBF)
      K[1] = (float)((exp(-0.5 * s[3]) - exp(-0.5 * s[2])) - (exp(-0.5 * s[1]) - exp(-0.5 * s[0])));
    else
      K[1] = (float)s[0];
  }
  if (gl == 0 && pair_ok) {
    store_pair<M>(p, a, b, K);
    if constexpr (SAVE) {
      float *__restrict__ st = p.state + state_slot(a, b, p.n2, p.pair_mode == GPSIG_PAIRS_UPPER) * state_stride(M, p.l2) +
                               (long long)(M - 1) * ncell;
#pragma unroll
      for (int m = 1; m <= M; ++m) st[m - 1] = K[m];
    }
  }
}

template <int M>
int sig_fo_mf_launch_m(const MfArgs &a, int seed, long long nblocks, hipStream_t s);

}  // namespace gpsig
