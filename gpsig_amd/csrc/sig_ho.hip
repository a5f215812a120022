// gpsig_amd -- higher-order truncated signature kernel Gram on gfx950.
//
// Replaces gpsig/signature_algs.py:37-74 (signature_kern_higher_order) for order > 1, row-streamed
// like the first-order kernel (sig_fo.h).  At level m the reference keeps a d x d array of tensors
// R[a][b] (d = min(m, order)); with the grid streamed by rows i and one pair per wave (W columns
// per lane), level m+1 at row i is
//   R'[0][0]   = dM * excl_scan_j( sum_{i'<i} sum_{a,b} R[a][b] )          (:64, both cumsums)
//   R'[0][b']  = dM / (b'+1) * sum_{i'<i} sum_a R[a][b'-1]                  (:66, cumsum over rows)
//   R'[a'][0]  = dM / (a'+1) * excl_scan_j( sum_b R[a'-1][b] at row i )     (:67, cumsum over cols)
//   R'[a'][b'] = dM / ((a'+1)(b'+1)) * R[a'-1][b'-1]                        (:69, same cell)
// so the state per column is the current row's blocks plus the running column sums
// CB_m[b] = sum_{i'<i} sum_a R_m[a][b]; K_m = sum_j sum_b CB_m[b] at the end.
// Sequences longer than the wave's 64 W columns run in column blocks of 64 W - 1 cells (the last
// column is the halo point), left to right over all rows; the exclusive column scans of a block add the
// carry of the blocks to its left: per row, one float per scanned quantity (S00 and Sa[1..dn-1] of each
// level), kept in this wave's LDS slab.
#include <stdlib.h>

#include "sig_common.h"
#include "gemm.h"

namespace gpsig {

template <int ORD, int MMAX>
struct HoLayout {
  static constexpr int dm(int m) { return m < ORD ? m : ORD; }  // blocks at 1-based level m
  static constexpr int off(int m) {                              // CB offset of 1-based level m
    int o = 0;
    for (int k = 1; k < m; ++k) o += dm(k);
    return o;
  }
  static constexpr int total = off(MMAX + 1);
  // column-block carries: the level-m scans of a row (S00 and Sa[1 .. dm(m+1)-1]) start at coff(m)
  static constexpr int coff(int m) {
    int o = 0;
    for (int k = 1; k < m; ++k) o += dm(k + 1);
    return o;
  }
};
// scanned floats per row of a launch at num_levels M (the row stride of the carry slab)
__host__ __device__ inline int ho_carries(int order, int M) {
  int o = 0;
  for (int k = 1; k < M; ++k) o += (k + 1 < order ? k + 1 : order);
  return o;
}

// exclusive scan over the wave's columns; blocked launches (nblk > 1) add the carry cr of the blocks to
// the left (written by lane 0 of the previous block) and leave the running total for the next one
template <int W>
GPSIG_DEV void excl_scan_cols(const float (&v)[W], float (&out)[W], float *cr, int blk, int nblk) {
  float t[W];
  t[0] = v[0];
#pragma unroll
  for (int w = 1; w < W; ++w) t[w] = t[w - 1] + v[w];
  const float incl = group_incl_scan<64>(t[W - 1]);
  float base = incl - t[W - 1];
  if (nblk > 1) {  // wave-uniform
    const float cin = blk > 0 ? *cr : 0.0f;
    const float tot = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, incl), 63));
    if (blk + 1 < nblk && (threadIdx.x & 63) == 0) *cr = cin + tot;
    base += cin;
  }
  out[0] = base;
#pragma unroll
  for (int w = 1; w < W; ++w) out[w] = base + t[w - 1];
}

// TILE (linear base kernel, any channel count): the cells come from the increment-Gram tile of the
// launch (SigArgs::tile, a GEMM of the increments, the reference's own tf.matmul of the linear base
// kernel, kernels.py:1042-1044), DP is unused.
// SPLIT (round 5): one pair per workgroup, its column blocks (2..4) side by side on the 4 waves instead of one
// after another on one wave: every exclusive column scan of a row adds the totals of the blocks to its left,
// exchanged through LDS, one barrier per level and row (the scans of a level at once).  For calls with few
// pairs (the VOSF trainer's Kff diagonal: 50 pairs of 500 points = 50 waves) it puts 4 SIMDs on each pair.
// The workgroups enumerate the pairs in the order of the 4-pair workgroups of the plain kernel (slot =
// blockIdx.x & 3), so the launches share the host's pair counts (x 4).
template <int DP, int W, int ORD, int MMAX, int SEED, bool TILE = false, bool SPLIT = false>
__global__ __launch_bounds__(256) void sig_ho_kernel(SigArgs p) {
  using Seed = RowSeed<DP, W, SEED>;
  using Lay = HoLayout<ORD, MMAX>;
  constexpr int FS = feat_stride(DP);
  static_assert(!TILE || SEED == SEED_LIN_DIFF, "tile cells: linear difference seed");
  const int lane = threadIdx.x & 63;
  const int wave = wave_uniform(threadIdx.x >> 6);
  const int slot = SPLIT ? (int)(blockIdx.x & 3) : wave;                   // the pair's slot in its group of 4
  const long long grp = SPLIT ? (long long)(blockIdx.x >> 2) : (long long)blockIdx.x;

  int a, b;
  if (p.pair_mode == GPSIG_PAIRS_DIAG) {
    a = p.row_begin + (int)grp * 4 + slot;
    b = a;
    if (a >= p.row_end) return;
  } else {
    int ta, tb;
    if (p.pair_mode == GPSIG_PAIRS_UPPER) {
      const Tile t = upper_tile(p.tile_base + grp, p.ntb, 4);
      ta = t.ta;
      tb = t.tb;
    } else {
      ta = p.tiles_a0 + (int)(grp / p.ntb);
      tb = (int)(grp % p.ntb);
    }
    a = ta * 4 + slot;
    b = tb;
    if (a < p.row_begin || a >= p.row_end) return;
  }
  bool pair_ok = b < p.n2;
  if (p.pair_mode == GPSIG_PAIRS_UPPER) pair_ok = pair_ok && b >= a;
  if (!pair_ok) return;  // one pair per wave (SPLIT: per workgroup): uniform
  // SPLIT: per-wave totals of the current exchange (double-buffered), the pair's level sums at the end
  __shared__ float hx[SPLIT ? 2 : 1][SPLIT ? 4 : 1][SPLIT ? ORD : 1];
  int ph = 0;

  const float *__restrict__ fx = TILE ? nullptr : p.FX + (long long)a * p.l1 * FS;
  const float *__restrict__ fy = TILE ? nullptr : p.FY + (long long)b * p.l2 * FS;
  const float *__restrict__ tcells =
      TILE ? p.tile + (long long)(a - p.tile_a0) * p.tile_as +
                 (p.pair_mode == GPSIG_PAIRS_DIAG ? 0 : (long long)(b - p.tile_b0) * (p.l2 - 1))
           : nullptr;
  const int M = p.M;
  const int nrows = Seed::DIFF ? p.l1 - 1 : p.l1;
  constexpr int CPB = 64 * W - 1;
  const int nblk = p.nblk;
  const int ncar = ho_carries(ORD, M);
  extern __shared__ float ho_carry[];
  float *__restrict__ carry = ho_carry + (long long)wave * nrows * ncar;

  float Kacc[MMAX + 1];
#pragma unroll
  for (int m = 0; m <= MMAX; ++m) Kacc[m] = 0.0f;

  for (int blk = SPLIT ? wave : 0; blk < (SPLIT ? wave + 1 : nblk); ++blk) {
  // SPLIT: a wave past the last block keeps a valid record view (block 0) and contributes zero cells
  const bool idle = SPLIT && blk >= nblk;
  const int j0 = idle ? 0 : blk * CPB;
  Seed seed;
  if constexpr (!TILE) seed.init(fx, fy + (long long)j0 * FS, lane, nblk == 1 ? p.l2 : min(p.l2 - j0, CPB + 1));
  // TILE: this lane's cell columns of the block (the halo column of a block is not a cell of it)
  bool tcol[W];
#pragma unroll
  for (int w = 0; w < W; ++w) tcol[w] = !idle && lane * W + w < CPB && j0 + lane * W + w < p.l2 - 1;

  float CB[Lay::total][W];
#pragma unroll
  for (int k = 0; k < Lay::total; ++k)
#pragma unroll
    for (int w = 0; w < W; ++w) CB[k][w] = 0.0f;

  RowData<DP> rd;
  if constexpr (!TILE) rd.load(fx, 0, SEED);
  for (int i = 0; i < nrows; ++i) {
    float *__restrict__ cr = carry + (long long)i * ncar;
    RowData<DP> rn;
    float dM[W];
    if constexpr (TILE) {
      const float *__restrict__ tr = tcells + (long long)i * p.tile_ld + j0 + lane * W;
#pragma unroll
      for (int w = 0; w < W; ++w) dM[w] = tcol[w] ? tr[w] : 0.0f;
    } else {
      rn.load(fx, i + 1 < nrows ? i + 1 : i, SEED);
      seed.template row<true>(rd, dM);
      if (idle)
#pragma unroll
        for (int w = 0; w < W; ++w) dM[w] = 0.0f;
    }

    float R[ORD][ORD][W];
#pragma unroll
    for (int x = 0; x < ORD; ++x)
#pragma unroll
      for (int y = 0; y < ORD; ++y)
#pragma unroll
        for (int w = 0; w < W; ++w) R[x][y][w] = (x == 0 && y == 0) ? dM[w] : 0.0f;

#pragma unroll
    for (int m = 1; m <= MMAX; ++m) {
      if (m <= M) {
        const int dmv = Lay::dm(m);
        // column / row sums of the level-m blocks at this row
        float colsum[ORD][W], rowsum[ORD][W];
#pragma unroll
        for (int x = 0; x < ORD; ++x)
#pragma unroll
          for (int w = 0; w < W; ++w) {
            float cs = 0.0f, rs = 0.0f;
#pragma unroll
            for (int y = 0; y < ORD; ++y) {
              if (y < dmv) cs += R[y][x][w];
              if (y < dmv) rs += R[x][y][w];
            }
            colsum[x][w] = cs;
            rowsum[x][w] = rs;
          }
        if (m < M) {
          const int dn = Lay::dm(m + 1);
          // S00 from the column running sums (rows < i)
          float tot[W], S00[W];
#pragma unroll
          for (int w = 0; w < W; ++w) {
            float s = 0.0f;
#pragma unroll
            for (int x = 0; x < ORD; ++x)
              if (x < dmv) s += CB[Lay::off(m) + x][w];
            tot[w] = s;
          }
          float Sa[ORD][W];
          if constexpr (SPLIT) {
            // the dn scans of the level together: in-lane and over the wave, then the blocks to the left
            float in[ORD][W], t[ORD], incl[ORD];
#pragma unroll
            for (int x = 0; x < ORD; ++x)
              if (x < dn)
#pragma unroll
                for (int w = 0; w < W; ++w) in[x][w] = x == 0 ? tot[w] : rowsum[x - 1][w];
            // the level's scans step-interleaved (one DPP chain per value would wait on each step's result)
#pragma unroll
            for (int x = 0; x < ORD; ++x) {
              float c = 0.0f;
              if (x < dn)
#pragma unroll
                for (int w = 0; w < W; ++w) c += in[x][w];
              t[x] = c;
              incl[x] = c;
            }
            group_incl_scan_n<64, ORD>(incl);
            if (lane == 63)
#pragma unroll
              for (int x = 0; x < ORD; ++x)
                if (x < dn) hx[ph][wave][x] = incl[x];
            __syncthreads();
#pragma unroll
            for (int x = 0; x < ORD; ++x)
              if (x < dn) {
                float base = incl[x] - t[x];
#pragma unroll
                for (int u = 0; u < 4; ++u) {  // unconditional reads (batched after the barrier), predicated adds
                  const float h = hx[ph][u][x];
                  base += u < wave ? h : 0.0f;
                }
                float *o = x == 0 ? S00 : Sa[x];
                o[0] = base;
#pragma unroll
                for (int w = 1; w < W; ++w) o[w] = o[w - 1] + in[x][w - 1];
              }
            ph ^= 1;
          } else {
            // the level's dn exclusive column scans, their DPP steps interleaved (in-lane totals first; the
            // in-lane prefixes are rebuilt when the outputs are written)
            float c[ORD], incl[ORD];
#pragma unroll
            for (int x = 0; x < ORD; ++x) {
              float t = 0.0f;
              if (x < dn)
#pragma unroll
                for (int w = 0; w < W; ++w) t += x == 0 ? tot[w] : rowsum[x > 0 ? x - 1 : 0][w];
              c[x] = t;
              incl[x] = t;
            }
            group_incl_scan_n<64, ORD>(incl);
#pragma unroll
            for (int x = 0; x < ORD; ++x)
              if (x < dn) {
                float base = incl[x] - c[x];
                if (nblk > 1) {  // wave-uniform: the carry of the blocks to the left, this block's total onwards
                  float *crx = cr + Lay::coff(m) + x;
                  const float cin = blk > 0 ? *crx : 0.0f;
                  const float bt = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, incl[x]), 63));
                  if (blk + 1 < nblk && lane == 0) *crx = cin + bt;
                  base += cin;
                }
                float *o = x == 0 ? S00 : Sa[x];
                o[0] = base;
#pragma unroll
                for (int w = 1; w < W; ++w) o[w] = o[w - 1] + (x == 0 ? tot[w - 1] : rowsum[x > 0 ? x - 1 : 0][w - 1]);
              }
          }
          // new blocks, in place: same-cell chain first (descending), then the edges
#pragma unroll
          for (int x = ORD - 1; x >= 1; --x)
#pragma unroll
            for (int y = ORD - 1; y >= 1; --y)
              if (x < dn && y < dn) {
                const float f = 1.0f / (float)((x + 1) * (y + 1));
#pragma unroll
                for (int w = 0; w < W; ++w) R[x][y][w] = f * dM[w] * R[x - 1][y - 1][w];
              }
#pragma unroll
          for (int y = 1; y < ORD; ++y)
            if (y < dn) {
              const float f = 1.0f / (float)(y + 1);
#pragma unroll
              for (int w = 0; w < W; ++w) R[0][y][w] = f * dM[w] * CB[Lay::off(m) + y - 1][w];  // y-1 < dm(m)
            }
#pragma unroll
          for (int x = 1; x < ORD; ++x)
            if (x < dn) {
              const float f = 1.0f / (float)(x + 1);
#pragma unroll
              for (int w = 0; w < W; ++w) R[x][0][w] = f * dM[w] * Sa[x][w];
            }
#pragma unroll
          for (int w = 0; w < W; ++w) R[0][0][w] = dM[w] * S00[w];
        }
        // CB_m += this row's level-m column sums (after their use above)
#pragma unroll
        for (int x = 0; x < ORD; ++x)
          if (x < dmv)
#pragma unroll
            for (int w = 0; w < W; ++w) CB[Lay::off(m) + x][w] += colsum[x][w];
      }
    }
    if constexpr (!TILE) rd = rn;
  }

#pragma unroll
  for (int m = 1; m <= MMAX; ++m) {
    float s = 0.0f;
#pragma unroll
    for (int x = 0; x < Lay::dm(m); ++x)
#pragma unroll
      for (int w = 0; w < W; ++w) s += CB[Lay::off(m) + x][w];
    Kacc[m] += group_sum<64>(s);
  }
  }  // column blocks

  float K[MMAX + 1];
  K[0] = 1.0f;
#pragma unroll
  for (int m = 1; m <= MMAX; ++m) K[m] = Kacc[m];
  if constexpr (SPLIT) {  // the blocks' level sums (every wave holds its block's in every lane)
    __shared__ float ks[4][MMAX + 1];
    if (lane == 0)
#pragma unroll
      for (int m = 1; m <= MMAX; ++m) ks[wave][m] = Kacc[m];
    __syncthreads();
#pragma unroll
    for (int m = 1; m <= MMAX; ++m) K[m] = ((ks[0][m] + ks[1][m]) + ks[2][m]) + ks[3][m];
    if (wave != 0) return;
  }
  if constexpr (TILE) {
    // level 1 in closed form (fp64, channels over the lanes): linear sum_ij <dx_i, dy_j> = <x_L - x_0, y_L - y_0>,
    // RBF cells (tile_rbf) the corner difference k(x_L, y_L) - k(x_L, y_0) - k(x_0, y_L) + k(x_0, y_0)
    const int d = p.wd;
    const float *xa = p.RX + (long long)a * p.l1 * d, *yb = p.RY + (long long)b * p.l2 * d;
    const float *xl = xa + (long long)(p.l1 - 1) * d, *yl = yb + (long long)(p.l2 - 1) * d;
    double s[4] = {0.0, 0.0, 0.0, 0.0};
    for (int k = lane; k < d; k += 64) {
      const double x0 = xa[k], x1 = xl[k], y0 = yb[k], y1 = yl[k];
      if (p.tile_rbf) {
        s[0] += (x0 - y0) * (x0 - y0);
        s[1] += (x0 - y1) * (x0 - y1);
        s[2] += (x1 - y0) * (x1 - y0);
        s[3] += (x1 - y1) * (x1 - y1);
      } else {
        s[0] += (x1 - x0) * (y1 - y0);
      }
    }
    for (int o = 32; o >= 1; o >>= 1)
      for (int u = 0; u < 4; ++u) s[u] += __shfl_xor(s[u], o, 64);
    K[1] = p.tile_rbf ? (float)((exp(-0.5 * s[3]) - exp(-0.5 * s[2])) - (exp(-0.5 * s[1]) - exp(-0.5 * s[0])))
                      : (float)s[0];
  }
  if (lane == 0) {
    if constexpr (!TILE) K[1] = level1_closed<DP, SEED>(fx, fy, p.l1, p.l2);  // ho seeds are the DIFF seeds
    store_pair<MMAX>(p, a, b, K);
  }
}

// Columns per lane for the higher-order kernel (one pair per wave): the fewest that cover the sequence,
// up to the register budget of the order (4 for order <= 4, 2 for order 5, 1 above); longer sequences
// run in column blocks at that width.
static int ho_wmax(int order) { return order <= 4 ? 4 : (order <= 5 ? 2 : 1); }
static int ho_w(int l2, int order) {
  for (int W = 1; W < ho_wmax(order); W *= 2)
    if (64 * W >= l2) return W;
  return ho_wmax(order);
}
static int ho_blocks(int l2, int W) { return 64 * W >= l2 ? 1 : (l2 - 1 + 64 * W - 2) / (64 * W - 1); }
// LDS of a 4-wave workgroup for the carries of a blocked launch
static size_t ho_carry_bytes(int l1, int order, int M, int nblk) {
  return nblk > 1 ? (size_t)4 * (l1 - 1) * ho_carries(order, M) * sizeof(float) : 0;
}
constexpr size_t HO_MAX_CARRY_BYTES = 160 * 1024;

// the split form (one pair per workgroup, column blocks side by side) for calls with few pairs: below about
// two waves per SIMD the plain kernel leaves the chip idle (GPSIG_HO_SPLIT=0 keeps the plain kernel)
constexpr long long HO_SPLIT_PAIRS = 2048;
static bool ho_split_on() {
  const char *e = getenv("GPSIG_HO_SPLIT");
  return !(e && e[0] == '0');
}

template <int DP, int W, int ORD, int SEED, bool TILE = false>
static int launch_ho(const SigArgs &a0, long long nblocks, hipStream_t s) {
  if (nblocks <= 0) return GPSIG_OK;
  SigArgs a = a0;
  a.nblk = ho_blocks(a.l2, W);
  if (a.nblk >= 2 && a.nblk <= 4 && nblocks * 4 <= HO_SPLIT_PAIRS && ho_split_on()) {
    hipLaunchKernelGGL((sig_ho_kernel<DP, W, ORD, 8, SEED, TILE, true>), dim3((unsigned)(nblocks * 4)), dim3(256), 0,
                       s, a);
    return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
  }
  const size_t lds = ho_carry_bytes(a.l1, ORD, a.M, a.nblk);
  if (lds > HO_MAX_CARRY_BYTES) return GPSIG_EUNSUPPORTED;
  hipLaunchKernelGGL((sig_ho_kernel<DP, W, ORD, 8, SEED, TILE>), dim3((unsigned)nblocks), dim3(256), lds, s, a);
  return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
}

int ho_lanes_per_pair(int l2, int order, int M) { return (M <= 8 && order <= 8 && l2 >= 2) ? 64 : 0; }

template <int DP, int SEED, bool TILE = false>
static int ho_dispatch(const SigArgs &a, long long nblocks, hipStream_t s) {
  const int W = ho_w(a.l2, a.order);
  switch (a.order) {
#define ORDCASE(o)                                                          \
  case o:                                                                   \
    if (W == 1) return launch_ho<DP, 1, o, SEED, TILE>(a, nblocks, s);      \
    if constexpr (o <= 5) {                                                 \
      if (W == 2) return launch_ho<DP, 2, o, SEED, TILE>(a, nblocks, s);    \
    }                                                                       \
    if constexpr (o <= 4) {                                                 \
      if (W == 4) return launch_ho<DP, 4, o, SEED, TILE>(a, nblocks, s);    \
    }                                                                       \
    return GPSIG_EUNSUPPORTED;
    ORDCASE(2) ORDCASE(3) ORDCASE(4) ORDCASE(5) ORDCASE(6) ORDCASE(7) ORDCASE(8)
#undef ORDCASE
    default: return GPSIG_EUNSUPPORTED;
  }
}

int sig_ho_launch(const SigArgs &a, int DP, int seed, long long nblocks, hipStream_t s) {
  if (seed != SEED_RBF_DIFF && seed != SEED_LIN_DIFF) return GPSIG_EUNSUPPORTED;
  if (a.M > 8 || a.order > 8 || a.order < 2) return GPSIG_EUNSUPPORTED;
  switch (DP) {
#define DCASE(v)                                                                          \
  case v:                                                                                 \
    return seed == SEED_RBF_DIFF ? ho_dispatch<v, SEED_RBF_DIFF>(a, nblocks, s)          \
                                 : ho_dispatch<v, SEED_LIN_DIFF>(a, nblocks, s);
    DCASE(4) DCASE(8) DCASE(16) DCASE(32)
#undef DCASE
    default: return GPSIG_EUNSUPPORTED;
  }
}

// ---- tile mode: the higher-order Gram past the fixed channel counts (linear base kernel, difference)
void pde_tile_chunk(int n1, int l1, int n2, int l2, int pair_mode, int &rows, long long &cols);
size_t pde_tile_scratch_bytes(int n1, int l1, int n2, int l2, int d, int pair_mode);
int increments_launch(const float *X, int n, int l, int d, float *dX, hipStream_t s);

int mf_records(const float *X, int n, int l, int d, float *R, hipStream_t s);
size_t mf_records_bytes(int n, int l, int d);
bool mf_gram_applies(int d, int l2);
int sig_fo_mf_cells(const float *FX, int n1, int l1, const float *FY, int n2, int l2, int d, int pair_mode,
                    int row_begin, int row_end, float *dm, int dm_a0, int dm_b0, long long dm_as, long long dm_bs,
                    long long dm_ld, hipStream_t s);

bool ho_tiled(int d, int order) { return order > 1 && d > 32; }
static size_t al256h(size_t b) { return (b + 255) & ~(size_t)255; }
// the operands of a chunk's cells (linear: the increments; RBF: the matrix-core seed's records), then the tile
static size_t ho_operand_bytes(int n1, int l1, int n2, int l2, int d, int pair_mode) {
  const bool rect = pair_mode == GPSIG_PAIRS_RECT;
  const size_t inc = al256h((size_t)n1 * (l1 - 1) * d * sizeof(float)) + (rect ? al256h((size_t)n2 * (l2 - 1) * d * sizeof(float)) : 0);
  const size_t rec = al256h(mf_records_bytes(n1, l1, d)) + (rect ? al256h(mf_records_bytes(n2, l2, d)) : 0);
  return inc > rec ? inc : rec;
}
size_t ho_tile_bytes(int n1, int l1, int n2, int l2, int d, int pair_mode) {
  if (n1 <= 0 || n2 <= 0 || l1 < 2 || l2 < 2 || d <= 0) return 0;
  int rows;
  long long cols;
  pde_tile_chunk(n1, l1, n2, l2, pair_mode, rows, cols);
  return ho_operand_bytes(n1, l1, n2, l2, d, pair_mode) + al256h((size_t)rows * (l1 - 1) * cols * sizeof(float));
}
static inline long long ho_upper_prefix(long long r, long long ntb) { return r * ntb - 4 * r * (r - 1) / 2; }

// Chunks of x-rows: the cell tile of the chunk -- linear: the increment Gram (one matrix-core GEMM dX_chunk dY^T,
// batched per pair for DIAG); RBF: the difference-seed cells from the matrix-core wide seed (sig_fo_mf.h, cell
// producer) -- then the tile-fed recursion.  a: filled by the caller (rows, mode, output, M, order).
int sig_ho_tiled(SigArgs a, const float *X, const float *Y, int d, int seed, void *workspace, size_t workspace_bytes,
                 hipStream_t s) {
  const int n1 = a.n1, l1 = a.l1, n2 = a.n2, l2 = a.l2, pm = a.pair_mode;
  const int IC = l1 - 1, JC = l2 - 1;
  if (a.M > 8 || a.order > 8) return GPSIG_EUNSUPPORTED;
  if (!workspace || workspace_bytes < ho_tile_bytes(n1, l1, n2, l2, d, pm)) return GPSIG_EWORKSPACE;
  int rows;
  long long cols;
  pde_tile_chunk(n1, l1, n2, l2, pm, rows, cols);
  const bool rbf = seed == SEED_RBF_DIFF;
  if (rbf ? !mf_gram_applies(d, l2) : seed != SEED_LIN_DIFF) return GPSIG_EUNSUPPORTED;
  char *w = static_cast<char *>(workspace);
  float *dX = reinterpret_cast<float *>(w), *dY = dX;
  const size_t xb = rbf ? al256h(mf_records_bytes(n1, l1, d)) : al256h((size_t)n1 * IC * d * sizeof(float));
  if (pm == GPSIG_PAIRS_RECT) dY = reinterpret_cast<float *>(w + xb);
  float *T = reinterpret_cast<float *>(w + ho_operand_bytes(n1, l1, n2, l2, d, pm));
  int rc = rbf ? mf_records(X, n1, l1, d, dX, s) : increments_launch(X, n1, l1, d, dX, s);
  if (rc) return rc;
  if (pm == GPSIG_PAIRS_RECT && (rc = rbf ? mf_records(Y, n2, l2, d, dY, s) : increments_launch(Y, n2, l2, d, dY, s)))
    return rc;
  a.tile = T;
  a.tile_rbf = rbf ? 1 : 0;
  a.RX = X;
  a.RY = pm == GPSIG_PAIRS_RECT ? Y : X;
  a.wd = d;
  const int rb0 = a.row_begin, rb1 = a.row_end;
  for (int r0 = (rb0 / 4) * 4; r0 < rb1; r0 += rows) {
    const int r1 = r0 + rows < rb1 ? r0 + rows : rb1;
    const int c0 = r0 > rb0 ? r0 : rb0;
    SigArgs c = a;
    c.row_begin = c0;
    c.row_end = r1;
    long long nblocks;
    if (pm == GPSIG_PAIRS_DIAG) {
      c.tile_a0 = c0;
      c.tile_b0 = 0;
      c.tile_as = (long long)IC * IC;
      c.tile_ld = IC;
      nblocks = (r1 - c0 + 3) / 4;
      if (rbf)
        rc = sig_fo_mf_cells(dX, n1, l1, dX, n1, l1, d, pm, c0, r1, T, c0, 0, (long long)IC * IC, 0, IC, s);
      else
        rc = gemm_f32(s, false, true, IC, IC, d, 1.0f, dX + (long long)c0 * IC * d, d, (long long)IC * d,
                      dX + (long long)c0 * IC * d, d, (long long)IC * d, 0.0f, T, IC, (long long)IC * IC, r1 - c0, 0, 0,
                      nullptr, 0);
    } else {
      const int b0 = pm == GPSIG_PAIRS_UPPER ? r0 : 0;
      const long long tc = (long long)(n2 - b0) * JC;
      c.tile_a0 = r0;
      c.tile_b0 = b0;
      c.tile_as = (long long)IC * tc;
      c.tile_ld = tc;
      const int ta0 = r0 / 4, ta1 = (r1 + 3) / 4;
      c.tiles_a0 = ta0;
      c.ntb = n2;  // one pair per wave: b-tiles are single sequences
      if (pm == GPSIG_PAIRS_RECT) {
        nblocks = (long long)(ta1 - ta0) * n2;
      } else {
        c.tile_base = ho_upper_prefix(ta0, n2);
        nblocks = ho_upper_prefix(ta1, n2) - c.tile_base;
      }
      if (rbf)
        rc = sig_fo_mf_cells(dX, n1, l1, dY, n2, l2, d, pm, c0, r1, T, r0, b0, (long long)IC * tc, JC, tc, s);
      else
        rc = gemm_f32(s, false, true, (r1 - r0) * IC, (int)tc, d, 1.0f, dX + (long long)r0 * IC * d, d, 0,
                      dY + (long long)b0 * JC * d, d, 0, 0.0f, T, tc, 0, 1, pm == GPSIG_PAIRS_UPPER ? IC : 0,
                      pm == GPSIG_PAIRS_UPPER ? JC : 0, nullptr, 0);
    }
    if (rc) return rc;
    if (nblocks > 0x7fffffffLL) return GPSIG_EUNSUPPORTED;
    if ((rc = ho_dispatch<1, SEED_LIN_DIFF, true>(c, nblocks, s))) return rc;
  }
  return GPSIG_OK;
}

}  // namespace gpsig
