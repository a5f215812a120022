// gpsig_amd -- launches of the higher-order Gram VJP kernel (sig_ho_bwd.h): orders 2 (levels 2..8) and 3
// (levels 3..5), the (order, levels) whose multiplier slab fits the LDS next to the cell buffer.  Orders
// at or above the level count are the exact signature kernel: order min(order, M).
#include "sig_ho_bwd.h"

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

bool ho_bwd_supported(int l2, int order, int M, int seed) {
  if (seed != SEED_RBF_DIFF && seed != SEED_LIN_DIFF) return false;
  if (l2 < 2 || l2 > 256 || M < 2 || M > 8 || order < 2) return false;
  const int o = ho_eff_order(order, M);
  return o == 2 || (o == 3 && M <= 5);
}

int sig_ho_bwd_launch(const BwdArgs &a, int order, int seed, long long nblocks, hipStream_t s) {
  const int o = ho_eff_order(order, a.M);
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
