// One (channel count, level count) instantiation of the first-order Gram VJP kernel (sig_bwd.h);
// compiled once per -DGPSIG_DP=.. -DGPSIG_M=.. so the instantiations build in parallel.
#include "sig_bwd_pk.h"

namespace gpsig {

template <int DP, int W, int LP, int M, int SEED>
static int launch_bwd(const BwdArgs &a, long long nblocks, hipStream_t s) {
  hipLaunchKernelGGL((sig_bwd_kernel<DP, W, LP, M, SEED>), dim3((unsigned)nblocks), dim3(256), 0, s, a);
  return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
}

template <int DP, int M, int SEED>
static int bwd_geo(const BwdArgs &a, long long nblocks, hipStream_t s) {
  const BwdGeo geo = bwd_geometry(a.l2, DP, M);
  if constexpr (bwd_seg_ok(DP, M))
    if (geo.W == 5 && geo.LP == 20) return launch_bwd<DP, 5, 20, M, SEED>(a, nblocks, s);
  constexpr int W = DP <= 8 ? 4 : 2;
  if (geo.W != W) return GPSIG_EUNSUPPORTED;
  switch (geo.LP) {
    case 16: return launch_bwd<DP, W, 16, M, SEED>(a, nblocks, s);
    case 32: return launch_bwd<DP, W, 32, M, SEED>(a, nblocks, s);
    case 64: return launch_bwd<DP, W, 64, M, SEED>(a, nblocks, s);
    default: return GPSIG_EUNSUPPORTED;
  }
}

template <int DP, int M>
int sig_bwd_launch_dpm(const BwdArgs &a, int seed, long long nblocks, hipStream_t s) {
  switch (seed) {
    case SEED_RBF_DIFF: return bwd_geo<DP, M, SEED_RBF_DIFF>(a, nblocks, s);
    case SEED_LIN_DIFF: return bwd_geo<DP, M, SEED_LIN_DIFF>(a, nblocks, s);
    case SEED_RBF_POINT: return bwd_geo<DP, M, SEED_RBF_POINT>(a, nblocks, s);
    case SEED_LIN_POINT: return bwd_geo<DP, M, SEED_LIN_POINT>(a, nblocks, s);
    default: return GPSIG_EUNSUPPORTED;
  }
}

template int sig_bwd_launch_dpm<GPSIG_DP, GPSIG_M>(const BwdArgs &, int, long long, hipStream_t);

// the packed column-pair VJP (sig_bwd_pk.h) at the geometry bwd_pk_geometry picked
template <int DP, int W, int LP, int M, int SEED>
static int launch_bwd_pk(const BwdArgs &a, long long nblocks, hipStream_t s) {
  hipLaunchKernelGGL((sig_bwd_pk_kernel<DP, W, LP, M, SEED>), dim3((unsigned)nblocks), dim3(256), 0, s, a);
  return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
}
template <int DP, int M, int SEED>
static int bwd_pk_geo(const BwdArgs &a, BwdGeo geo, long long nblocks, hipStream_t s) {
  if constexpr (DP > 8) {
    return GPSIG_EUNSUPPORTED;  // (bwd_pk_geometry: DP <= 8)
  } else {
    constexpr bool W6 = SEED == SEED_LIN_DIFF && DP <= 5 && M <= 6;
    if (geo.W == 4) {
      switch (geo.LP) {
        case 16: return launch_bwd_pk<DP, 4, 16, M, SEED>(a, nblocks, s);
        case 32: return launch_bwd_pk<DP, 4, 32, M, SEED>(a, nblocks, s);
        case 64: return launch_bwd_pk<DP, 4, 64, M, SEED>(a, nblocks, s);
        default: return GPSIG_EUNSUPPORTED;
      }
    }
    if constexpr (W6) {
      if (geo.W == 6) {
        switch (geo.LP) {
          case 20: return launch_bwd_pk<DP, 6, 20, M, SEED>(a, nblocks, s);
          case 32: return launch_bwd_pk<DP, 6, 32, M, SEED>(a, nblocks, s);
          default: return GPSIG_EUNSUPPORTED;
        }
      }
    }
    return GPSIG_EUNSUPPORTED;
  }
}

template <int DP, int M>
int sig_bwd_pk_launch_dpm(const BwdArgs &a, int seed, BwdGeo geo, long long nblocks, hipStream_t s) {
  switch (seed) {
    case SEED_RBF_DIFF: return bwd_pk_geo<DP, M, SEED_RBF_DIFF>(a, geo, nblocks, s);
    case SEED_LIN_DIFF: return bwd_pk_geo<DP, M, SEED_LIN_DIFF>(a, geo, nblocks, s);
    default: return GPSIG_EUNSUPPORTED;
  }
}

template int sig_bwd_pk_launch_dpm<GPSIG_DP, GPSIG_M>(const BwdArgs &, int, BwdGeo, long long, hipStream_t);

}  // namespace gpsig
