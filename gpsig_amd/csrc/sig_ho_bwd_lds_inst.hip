// gpsig_amd -- instantiations of the LDS-state higher-order Gram VJP (sig_ho_bwd_lds.h) for one effective
// order (GPSIG_ORD): every level count whose multiplier slab fits the LDS, W = 4 (l2 <= 256) and 8 (l2 <= 512).
#include "sig_ho_bwd_lds.h"

#ifndef GPSIG_ORD
#error "GPSIG_ORD"
#endif

namespace gpsig {

template <int ORD, int M, int W>
static int launch_lds(const BwdArgs &a, int seed, long long nblocks, hipStream_t s) {
  constexpr size_t lds = ho_bwd_lds_slab_bytes<ORD, M, W>();
  if constexpr (lds + ho_bwd_lds_cbuf_bytes(W) > 160 * 1024) {
    return GPSIG_EUNSUPPORTED;
  } else {
    if (seed == SEED_RBF_DIFF)
      hipLaunchKernelGGL((sig_ho_bwd_lds_kernel<ORD, M, W, SEED_RBF_DIFF>), dim3((unsigned)nblocks), dim3(64), lds, s, a);
    else if (seed == SEED_LIN_DIFF)
      hipLaunchKernelGGL((sig_ho_bwd_lds_kernel<ORD, M, W, SEED_LIN_DIFF>), dim3((unsigned)nblocks), dim3(64), lds, s, a);
    else
      return GPSIG_EUNSUPPORTED;
    return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
  }
}

template <int ORD, int M>
static int launch_lds_w(const BwdArgs &a, int seed, long long nblocks, hipStream_t s) {
  if (a.l2 <= 256) return launch_lds<ORD, M, 4>(a, seed, nblocks, s);
  return launch_lds<ORD, M, 8>(a, seed, nblocks, s);
}

template <>
int sig_ho_bwd_lds_launch_o<GPSIG_ORD>(const BwdArgs &a, int seed, long long nblocks, hipStream_t s) {
  constexpr int O = GPSIG_ORD;
  switch (a.M) {
#define GPSIG_CASE(m) \
  case m:             \
    if constexpr (m >= O) return launch_lds_w<O, m>(a, seed, nblocks, s); else return GPSIG_EUNSUPPORTED;
    GPSIG_CASE(2) GPSIG_CASE(3) GPSIG_CASE(4) GPSIG_CASE(5) GPSIG_CASE(6) GPSIG_CASE(7) GPSIG_CASE(8)
#undef GPSIG_CASE
    default: return GPSIG_EUNSUPPORTED;
  }
}

}  // namespace gpsig
