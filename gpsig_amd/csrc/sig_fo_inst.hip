// gpsig_amd -- explicit instantiation unit: the first-order kernels for one (channel count, level
// count).  Compiled once per (GPSIG_DP, GPSIG_M) by gpsig_amd/csrc/Makefile.
#include "sig_fo.h"
#if !defined(GPSIG_DP) || !defined(GPSIG_M)
#error "GPSIG_DP and GPSIG_M must be defined"
#endif
namespace gpsig {
// per-seed dispatch of one (channel count, level count); built in parallel, one unit each
template <int DP, int M>
int sig_fo_launch_dpm(const SigArgs &a, int seed, long long nblocks, hipStream_t s) {
  switch (seed) {
    case SEED_RBF_DIFF: return fo_geo<DP, M, SEED_RBF_DIFF>(a, nblocks, s);
    case SEED_LIN_DIFF: return fo_geo<DP, M, SEED_LIN_DIFF>(a, nblocks, s);
    case SEED_RBF_POINT: return fo_geo<DP, M, SEED_RBF_POINT>(a, nblocks, s);
    case SEED_LIN_POINT: return fo_geo<DP, M, SEED_LIN_POINT>(a, nblocks, s);
    default: return GPSIG_EUNSUPPORTED;
  }
}

template int sig_fo_launch_dpm<GPSIG_DP, GPSIG_M>(const SigArgs &, int, long long, hipStream_t);
}
