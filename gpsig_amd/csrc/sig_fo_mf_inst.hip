// gpsig_amd -- instantiations of the matrix-core wide-channel Gram (sig_fo_mf.h) for one level count
// (GPSIG_M): columns per lane 4 / 8 / 10, RBF and linear difference seeds, with and without saved state.
#include "sig_fo_mf.h"

#ifndef GPSIG_M
#error "GPSIG_M"
#endif

namespace gpsig {

template <int NW, int W, int M, int SEED, bool BLK, int NP>
static int mf_launch_np(const MfArgs &a, long long nblocks, hipStream_t s) {
  const size_t lds = mf_lds_bytes(a.d, a.p.l2, NW, NP);
  if (a.p.state)
    hipLaunchKernelGGL((sig_fo_mf_kernel<NW, W, M, SEED, true, BLK, false, NP>), dim3((unsigned)nblocks), dim3(64 * NW), lds,
                       s, a);
  else
    hipLaunchKernelGGL((sig_fo_mf_kernel<NW, W, M, SEED, false, BLK, false, NP>), dim3((unsigned)nblocks), dim3(64 * NW), lds,
                       s, a);
  return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
}
template <int NW, int W, int M, int SEED, bool BLK>
static int mf_launch_blk(const MfArgs &a, long long nblocks, hipStream_t s) {
  return mf_geo(a.d, a.p.l2).np == 3 ? mf_launch_np<NW, W, M, SEED, BLK, 3>(a, nblocks, s)
                                     : mf_launch_np<NW, W, M, SEED, BLK, 2>(a, nblocks, s);
}
template <int NW, int W, int M, int SEED>
static int mf_launch_nw(const MfArgs &a, long long nblocks, hipStream_t s) {
  if constexpr (W == 8) {
    if (a.nblk > 1) {  // column blocks: chunks of MF_BLK_CHUNK workgroups share the carry scratch
      MfArgs c = a;
      for (long long b0 = 0; b0 < nblocks; b0 += MF_BLK_CHUNK) {
        c.blk0 = b0;
        const long long nb = nblocks - b0 < MF_BLK_CHUNK ? nblocks - b0 : MF_BLK_CHUNK;
        const int rc = mf_launch_blk<NW, W, M, SEED, true>(c, nb, s);
        if (rc) return rc;
      }
      return GPSIG_OK;
    }
  }
  return mf_launch_blk<NW, W, M, SEED, false>(a, nblocks, s);
}
template <int W, int M, int SEED>
static int mf_launch_w(const MfArgs &a, long long nblocks, hipStream_t s) {
  switch (mf_waves(a.d, a.p.l2)) {
    case 8: return mf_launch_nw<8, W, M, SEED>(a, nblocks, s);
    case 4: return mf_launch_nw<4, W, M, SEED>(a, nblocks, s);
    default: return GPSIG_EUNSUPPORTED;
  }
}

template <int M, int SEED>
static int mf_launch_seed(const MfArgs &a, long long nblocks, hipStream_t s) {
  switch (mf_w(a.p.l2)) {
    case 4: return mf_launch_w<4, M, SEED>(a, nblocks, s);
    case 8: return mf_launch_w<8, M, SEED>(a, nblocks, s);
    case 10: return mf_launch_w<10, M, SEED>(a, nblocks, s);
    default: return GPSIG_EUNSUPPORTED;
  }
}

template <>
int sig_fo_mf_launch_m<GPSIG_M>(const MfArgs &a, int seed, long long nblocks, hipStream_t s) {
  if (seed == SEED_RBF_DIFF) return mf_launch_seed<GPSIG_M, SEED_RBF_DIFF>(a, nblocks, s);
  if (seed == SEED_LIN_DIFF) return mf_launch_seed<GPSIG_M, SEED_LIN_DIFF>(a, nblocks, s);
  return GPSIG_EUNSUPPORTED;
}

#if GPSIG_M == 1
// The RBF cells of a chunk of pairs into the higher-order recursion's tile (DMO instantiations).
template <int NW, int W, bool BLK, int NP>
static int mf_cells_np(const MfArgs &a, long long nblocks, hipStream_t s) {
  const size_t lds = mf_lds_bytes(a.d, a.p.l2, NW, NP);
  hipLaunchKernelGGL((sig_fo_mf_kernel<NW, W, 1, SEED_RBF_DIFF, false, BLK, true, NP>), dim3((unsigned)nblocks),
                     dim3(64 * NW), lds, s, a);
  return hipGetLastError() == hipSuccess ? GPSIG_OK : GPSIG_ELAUNCH;
}
template <int NW, int W, bool BLK>
static int mf_cells_launch(const MfArgs &a, long long nblocks, hipStream_t s) {
  return mf_geo(a.d, a.p.l2).np == 3 ? mf_cells_np<NW, W, BLK, 3>(a, nblocks, s) : mf_cells_np<NW, W, BLK, 2>(a, nblocks, s);
}
template <int NW>
static int mf_cells_nw(const MfArgs &a, long long nblocks, hipStream_t s) {
  switch (mf_w(a.p.l2)) {
    case 4: return mf_cells_launch<NW, 4, false>(a, nblocks, s);
    case 8: return a.nblk > 1 ? mf_cells_launch<NW, 8, true>(a, nblocks, s) : mf_cells_launch<NW, 8, false>(a, nblocks, s);
    case 10: return mf_cells_launch<NW, 10, false>(a, nblocks, s);
    default: return GPSIG_EUNSUPPORTED;
  }
}
int sig_fo_mf_cells_launch(const MfArgs &a, long long nblocks, hipStream_t s) {
  switch (mf_waves(a.d, a.p.l2)) {
    case 8: return mf_cells_nw<8>(a, nblocks, s);
    case 4: return mf_cells_nw<4>(a, nblocks, s);
    default: return GPSIG_EUNSUPPORTED;
  }
}
#endif

}  // namespace gpsig
