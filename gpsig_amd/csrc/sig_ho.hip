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
#include "sig_common.h"

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

template <int DP, int W, int ORD, int MMAX, int SEED>
__global__ __launch_bounds__(256) void sig_ho_kernel(SigArgs p) {
  using Seed = RowSeed<DP, W, SEED>;
  using Lay = HoLayout<ORD, MMAX>;
  constexpr int FS = feat_stride(DP);
  const int lane = threadIdx.x & 63;
  const int wave = wave_uniform(threadIdx.x >> 6);

  int a, b;
  if (p.pair_mode == GPSIG_PAIRS_DIAG) {
    a = p.row_begin + (int)blockIdx.x * 4 + wave;
    b = a;
    if (a >= p.row_end) return;
  } else {
    int ta, tb;
    if (p.pair_mode == GPSIG_PAIRS_UPPER) {
      const Tile t = upper_tile(p.tile_base + (long long)blockIdx.x, p.ntb, 4);
      ta = t.ta;
      tb = t.tb;
    } else {
      ta = p.tiles_a0 + (int)blockIdx.x / p.ntb;
      tb = (int)blockIdx.x % p.ntb;
    }
    a = ta * 4 + wave;
    b = tb;
    if (a < p.row_begin || a >= p.row_end) return;
  }
  bool pair_ok = b < p.n2;
  if (p.pair_mode == GPSIG_PAIRS_UPPER) pair_ok = pair_ok && b >= a;
  if (!pair_ok) return;  // one pair per wave: wave-uniform

  const float *__restrict__ fx = p.FX + (long long)a * p.l1 * FS;
  const float *__restrict__ fy = p.FY + (long long)b * p.l2 * FS;
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

  for (int blk = 0; blk < nblk; ++blk) {
  const int j0 = blk * CPB;
  Seed seed;
  seed.init(fx, fy + (long long)j0 * FS, lane, nblk == 1 ? p.l2 : min(p.l2 - j0, CPB + 1));

  float CB[Lay::total][W];
#pragma unroll
  for (int k = 0; k < Lay::total; ++k)
#pragma unroll
    for (int w = 0; w < W; ++w) CB[k][w] = 0.0f;

  RowData<DP> rd;
  rd.load(fx, 0, SEED);
  for (int i = 0; i < nrows; ++i) {
    float *__restrict__ cr = carry + (long long)i * ncar;
    RowData<DP> rn;
    rn.load(fx, i + 1 < nrows ? i + 1 : i, SEED);
    float dM[W];
    seed.template row<true>(rd, dM);

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
          excl_scan_cols<W>(tot, S00, cr + Lay::coff(m), blk, nblk);
          float Sa[ORD][W];
#pragma unroll
          for (int x = 1; x < ORD; ++x)
            if (x < dn) excl_scan_cols<W>(rowsum[x - 1], Sa[x], cr + Lay::coff(m) + x, blk, nblk);
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
    rd = rn;
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
  if (lane == 0) {
    K[1] = level1_closed<DP, SEED>(fx, fy, p.l1, p.l2);  // ho seeds are the DIFF seeds
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

template <int DP, int W, int ORD, int SEED>
static int launch_ho(const SigArgs &a0, long long nblocks, hipStream_t s) {
  if (nblocks <= 0) return GPSIG_OK;
  SigArgs a = a0;
  a.nblk = ho_blocks(a.l2, W);
  const size_t lds = ho_carry_bytes(a.l1, ORD, a.M, a.nblk);
  if (lds > HO_MAX_CARRY_BYTES) return GPSIG_EUNSUPPORTED;
  hipLaunchKernelGGL((sig_ho_kernel<DP, W, ORD, 8, SEED>), dim3((unsigned)nblocks), dim3(256), lds, s, a);
  return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
}

int ho_lanes_per_pair(int l2, int order, int M) { return (M <= 8 && order <= 8 && l2 >= 2) ? 64 : 0; }

template <int DP, int SEED>
static int ho_dispatch(const SigArgs &a, long long nblocks, hipStream_t s) {
  const int W = ho_w(a.l2, a.order);
  switch (a.order) {
#define ORDCASE(o)                                                          \
  case o:                                                                   \
    if (W == 1) return launch_ho<DP, 1, o, SEED>(a, nblocks, s);            \
    if constexpr (o <= 5) {                                                 \
      if (W == 2) return launch_ho<DP, 2, o, SEED>(a, nblocks, s);          \
    }                                                                       \
    if constexpr (o <= 4) {                                                 \
      if (W == 4) return launch_ho<DP, 4, o, SEED>(a, nblocks, s);          \
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

}  // namespace gpsig
