// gpsig_amd -- launches of the higher-order Gram VJP kernel (sig_ho_bwd.h): orders 2 (levels 2..8) and 3
// (levels 3..5), the (order, levels) whose multiplier slab fits the LDS next to the cell buffer.  Orders
// at or above the level count are the exact signature kernel: order min(order, M).
#include "sig_ho_bwd_split.h"

namespace gpsig {

constexpr size_t HO_BWD_STATIC_LDS = (size_t)4 * GPSIG_WIDE_BWD_R * 64 * 8 * sizeof(float);  // cbuf

template <int ORD, int M>
static int launch_ho_bwd(const BwdArgs &a, int seed, long long nblocks, hipStream_t s) {
  constexpr size_t lds = ho_bwd_lds_bytes<ORD, M>();
  static_assert(lds + HO_BWD_STATIC_LDS <= 160 * 1024, "LDS");
  if (seed == SEED_RBF_DIFF)
    hipLaunchKernelGGL((sig_ho_bwd_kernel<ORD, M, SEED_RBF_DIFF>), dim3((unsigned)nblocks), dim3(256), lds, s, a);
  else if (seed == SEED_LIN_DIFF)
    hipLaunchKernelGGL((sig_ho_bwd_kernel<ORD, M, SEED_LIN_DIFF>), dim3((unsigned)nblocks), dim3(256), lds, s, a);
  else
    return GPSIG_EUNSUPPORTED;
  return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
}

static int ho_eff_order(int order, int M) { return order < M ? order : M; }

// the register kernel (sig_ho_bwd.h: one pair per wave, 4 per workgroup)
static bool ho_bwd_reg(int l2, int o, int M) { return l2 <= 256 && (o == 2 || (o == 3 && M <= 5)); }

bool ho_bwd_supported(int l2, int order, int M, int seed) {
  if (seed != SEED_RBF_DIFF && seed != SEED_LIN_DIFF) return false;
  if (l2 < 2 || M < 2 || M > 8 || order < 2) return false;
  const int o = ho_eff_order(order, M);
  if (l2 > HO_SPLIT_NW * HO_SPLIT_CPB + 1 && o <= HO_LDS_MAX_ORD && ho_bwd_split8_fits(o, M, l2)) return true;
  if (l2 > 512) return false;
  return ho_bwd_reg(l2, o, M) || (o <= HO_LDS_MAX_ORD && ho_bwd_lds_fits(o, M, l2));
}

// global slabs of the 8-wave split VJP (510 .. 1017 points): one launch chunk of workgroups
size_t ho_bwd_slab_bytes(int l2, int order, int M) {
  const int o = ho_eff_order(order, M);
  if (!ho_bwd_split8_fits(o, M, l2)) return 0;
  return (size_t)HO_SPLIT8_BLOCKS * (size_t)ho_split_slab_floats_rt(o, M, HO_SPLIT8_NW) * sizeof(float);
}

// The LDS kernel runs one pair per workgroup: its own grid over the launch's rows [row_begin, row_end)
static int ho_bwd_lds_launch(BwdArgs a, int o, int seed, hipStream_t s) {
  const int r0 = a.row_begin, r1 = a.row_end;
  long long nblocks;
  if (a.pair_mode == GPSIG_PAIRS_DIAG) {
    nblocks = r1 - r0;
  } else if (a.pair_mode == GPSIG_PAIRS_UPPER) {
    auto P = [&](long long r) { return r * a.n2 - r * (r - 1) / 2; };
    a.tile_base = P(r0);
    nblocks = P(r1) - P(r0);
  } else {
    nblocks = (long long)(r1 - r0) * a.n2;
  }
  a.blk0 = 0;
  if (nblocks <= 0) return GPSIG_OK;
  if (nblocks > 0x7fffffffLL) return GPSIG_EUNSUPPORTED;
  switch (o) {
    case 2: return sig_ho_bwd_lds_launch_o<2>(a, seed, nblocks, s);
    case 3: return sig_ho_bwd_lds_launch_o<3>(a, seed, nblocks, s);
    case 4: return sig_ho_bwd_lds_launch_o<4>(a, seed, nblocks, s);
    case 5: return sig_ho_bwd_lds_launch_o<5>(a, seed, nblocks, s);
    case 6: return sig_ho_bwd_lds_launch_o<6>(a, seed, nblocks, s);
    default: return GPSIG_EUNSUPPORTED;
  }
}

int sig_ho_bwd_launch(const BwdArgs &a, int order, int seed, long long nblocks, hipStream_t s) {
  const int o = ho_eff_order(order, a.M);
  if (!ho_bwd_reg(a.l2, o, a.M)) return ho_bwd_lds_launch(a, o, seed, s);
  switch (o * 16 + a.M) {
    case 2 * 16 + 2: return launch_ho_bwd<2, 2>(a, seed, nblocks, s);
    case 2 * 16 + 3: return launch_ho_bwd<2, 3>(a, seed, nblocks, s);
    case 2 * 16 + 4: return launch_ho_bwd<2, 4>(a, seed, nblocks, s);
    case 2 * 16 + 5: return launch_ho_bwd<2, 5>(a, seed, nblocks, s);
    case 2 * 16 + 6: return launch_ho_bwd<2, 6>(a, seed, nblocks, s);
    case 2 * 16 + 7: return launch_ho_bwd<2, 7>(a, seed, nblocks, s);
    case 2 * 16 + 8: return launch_ho_bwd<2, 8>(a, seed, nblocks, s);
    case 3 * 16 + 3: return launch_ho_bwd<3, 3>(a, seed, nblocks, s);
    case 3 * 16 + 4: return launch_ho_bwd<3, 4>(a, seed, nblocks, s);
    case 3 * 16 + 5: return launch_ho_bwd<3, 5>(a, seed, nblocks, s);
    default: return GPSIG_EUNSUPPORTED;
  }
}

}  // namespace gpsig
