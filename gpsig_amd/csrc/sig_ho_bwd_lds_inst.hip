// gpsig_amd -- instantiations of the LDS-state higher-order Gram VJP (sig_ho_bwd_lds.h) for one effective
// order (GPSIG_ORD): every level count whose multiplier slab fits the LDS, W = 4 (l2 <= 256) and 8 (l2 <= 512);
// the split kernels (257 .. 509 points on 4 waves, 510 .. 1017 on 8 waves with a global slab).
#include <stdlib.h>

#include "sig_ho_bwd_split.h"

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

// one pair over the 4 SIMDs of a CU (sig_ho_bwd_split.h): 257..509 points; GPSIG_HO_SPLIT=0 keeps the one-wave
// kernel (A/B)
template <int ORD, int M>
static int launch_split(const BwdArgs &a, int seed, long long nblocks, hipStream_t s) {
  constexpr size_t lds = ho_bwd_split_slab_bytes<ORD, M>();
  if constexpr (lds + ho_bwd_lds_cbuf_bytes(8) + 2 * HO_SPLIT_NW * HO_SPLIT_XN * 4 > 160 * 1024) {
    return GPSIG_EUNSUPPORTED;
  } else {
    if (seed == SEED_RBF_DIFF)
      hipLaunchKernelGGL((sig_ho_bwd_split_kernel<ORD, M, SEED_RBF_DIFF>), dim3((unsigned)nblocks),
                         dim3(64 * HO_SPLIT_NW), lds, s, a);
    else if (seed == SEED_LIN_DIFF)
      hipLaunchKernelGGL((sig_ho_bwd_split_kernel<ORD, M, SEED_LIN_DIFF>), dim3((unsigned)nblocks),
                         dim3(64 * HO_SPLIT_NW), lds, s, a);
    else
      return GPSIG_EUNSUPPORTED;
    return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
  }
}

// 510 .. 1017 points: 8 waves per pair, 2 per SIMD, the slab in the caller's global region (a.scratch), at most
// HO_SPLIT8_BLOCKS workgroups per launch (each owns scr_stride floats of the region)
template <int ORD, int M>
static int launch_split8(BwdArgs a, int seed, long long nblocks, hipStream_t s) {
  constexpr int NW = HO_SPLIT8_NW;
  if constexpr (!ho_split8_ok(ORD, M)) {
    return GPSIG_EUNSUPPORTED;
  } else {
  if (!a.scratch) return GPSIG_EWORKSPACE;
  a.scr_stride = ho_split_slab_floats<ORD, M>(NW);
  for (long long b0 = 0; b0 < nblocks; b0 += HO_SPLIT8_BLOCKS) {
    const long long nb = nblocks - b0 < HO_SPLIT8_BLOCKS ? nblocks - b0 : HO_SPLIT8_BLOCKS;
    BwdArgs c = a;
    c.blk0 = a.blk0 + b0;
    if (seed == SEED_RBF_DIFF)
      hipLaunchKernelGGL((sig_ho_bwd_split_kernel<ORD, M, SEED_RBF_DIFF, NW>), dim3((unsigned)nb), dim3(64 * NW), 0, s, c);
    else if (seed == SEED_LIN_DIFF)
      hipLaunchKernelGGL((sig_ho_bwd_split_kernel<ORD, M, SEED_LIN_DIFF, NW>), dim3((unsigned)nb), dim3(64 * NW), 0, s, c);
    else
      return GPSIG_EUNSUPPORTED;
    if (hipGetLastError() != hipSuccess) return GPSIG_ELAUNCH;
  }
  return GPSIG_OK;
  }
}

static bool split_on() {
  const char *e = getenv("GPSIG_HO_SPLIT");
  return !(e && e[0] == '0');
}

template <int ORD, int M>
static int launch_lds_w(const BwdArgs &a, int seed, long long nblocks, hipStream_t s) {
  // 510 .. 512 points at (order, levels) the 8-wave form does not hold keep the one-wave W = 8 kernel
  if (a.l2 > HO_SPLIT_NW * HO_SPLIT_CPB + 1 && ho_split8_ok(ORD, M)) return launch_split8<ORD, M>(a, seed, nblocks, s);
  if (a.l2 <= 256) return launch_lds<ORD, M, 4>(a, seed, nblocks, s);
  if (split_on() && ho_bwd_split_fits(ORD, M, a.l2)) return launch_split<ORD, M>(a, seed, nblocks, s);
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
