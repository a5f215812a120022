// One level-count instantiation of the wide-channel Gram VJP kernel (sig_bwd_wide.h); compiled once per
// -DGPSIG_M=.. so the instantiations build in parallel.
#include "sig_bwd_wide.h"
#if !defined(GPSIG_M)
#error "GPSIG_M must be defined"
#endif

namespace gpsig {

template <int LP, int M, int SEED>
static int launch_bwd_wide(const BwdArgs &a, long long nblocks, hipStream_t s) {
  hipLaunchKernelGGL((sig_bwd_wide_kernel<8, LP, M, SEED>), dim3((unsigned)nblocks), dim3(256), 0, s, a);
  return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
}

template <int M, int SEED>
static int bwd_wide_geo(const BwdArgs &a, long long nblocks, hipStream_t s) {
  switch (bwd_geometry_wide(a.l2).LP) {
    case 16: return launch_bwd_wide<16, M, SEED>(a, nblocks, s);
    case 32: return launch_bwd_wide<32, M, SEED>(a, nblocks, s);
    case 64: return launch_bwd_wide<64, M, SEED>(a, nblocks, s);
    default: return GPSIG_EUNSUPPORTED;
  }
}

template <int M>
int sig_bwd_wide_launch_m(const BwdArgs &a, int seed, long long nblocks, hipStream_t s) {
  switch (seed) {
    case SEED_RBF_DIFF: return bwd_wide_geo<M, SEED_RBF_DIFF>(a, nblocks, s);
    case SEED_LIN_DIFF: return bwd_wide_geo<M, SEED_LIN_DIFF>(a, nblocks, s);
    case SEED_RBF_POINT: return bwd_wide_geo<M, SEED_RBF_POINT>(a, nblocks, s);
    case SEED_LIN_POINT: return bwd_wide_geo<M, SEED_LIN_POINT>(a, nblocks, s);
    default: return GPSIG_EUNSUPPORTED;
  }
}

template int sig_bwd_wide_launch_m<GPSIG_M>(const BwdArgs &, int, long long, hipStream_t);

}  // namespace gpsig
