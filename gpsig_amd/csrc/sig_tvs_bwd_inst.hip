// One (channel padding, increments) instantiation set of the tens-vs-seq VJP kernel (sig_tvs_bwd.h),
// compiled once per -DGPSIG_DP=.. -DGPSIG_INCR=.. so the sets build in parallel.
#include "sig_tvs_bwd.h"
#if !defined(GPSIG_DP) || !defined(GPSIG_INCR)
#error "GPSIG_DP and GPSIG_INCR must be defined"
#endif

namespace gpsig {

template <int DP, int M, bool INCR>
static int launch_tvs_bwd(const TvsBwdArgs &a, bool rbf, bool diff, hipStream_t s) {
  constexpr int NW = tvs_bwd_waves<DP, INCR>();
  const dim3 grid((unsigned)((a.n + 63) / 64), (unsigned)((a.t + NW - 1) / NW), (unsigned)M);
  const dim3 block(64 * NW);
  if (rbf && diff)
    hipLaunchKernelGGL((tvs_bwd_kernel<DP, M, INCR, true, true>), grid, block, 0, s, a);
  else if (diff)
    hipLaunchKernelGGL((tvs_bwd_kernel<DP, M, INCR, false, true>), grid, block, 0, s, a);
  else if (rbf)
    hipLaunchKernelGGL((tvs_bwd_kernel<DP, M, INCR, true, false>), grid, block, 0, s, a);
  else
    hipLaunchKernelGGL((tvs_bwd_kernel<DP, M, INCR, false, false>), grid, block, 0, s, a);
  return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
}

template <int DP, bool INCR>
int tvs_bwd_launch_dp(const TvsBwdArgs &a, int M, bool rbf, bool diff, hipStream_t s) {
  switch (M) {
    case 1: return launch_tvs_bwd<DP, 1, INCR>(a, rbf, diff, s);
    case 2: return launch_tvs_bwd<DP, 2, INCR>(a, rbf, diff, s);
    case 3: return launch_tvs_bwd<DP, 3, INCR>(a, rbf, diff, s);
    case 4: return launch_tvs_bwd<DP, 4, INCR>(a, rbf, diff, s);
    case 5: return launch_tvs_bwd<DP, 5, INCR>(a, rbf, diff, s);
    case 6: return launch_tvs_bwd<DP, 6, INCR>(a, rbf, diff, s);
    case 7: return launch_tvs_bwd<DP, 7, INCR>(a, rbf, diff, s);
    case 8: return launch_tvs_bwd<DP, 8, INCR>(a, rbf, diff, s);
    default: return GPSIG_EUNSUPPORTED;
  }
}

template int tvs_bwd_launch_dp<GPSIG_DP, (GPSIG_INCR != 0)>(const TvsBwdArgs &, int, bool, bool, hipStream_t);

}  // namespace gpsig
