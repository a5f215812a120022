// gpsig_amd -- explicit instantiation unit: the first-order kernels for one (channel count, level
// count).  Compiled once per (GPSIG_DP, GPSIG_M) by gpsig_amd/csrc/Makefile.
#include "sig_fo.h"
#if !defined(GPSIG_DP) || !defined(GPSIG_M)
#error "GPSIG_DP and GPSIG_M must be defined"
#endif
namespace gpsig {
template int sig_fo_launch_dpm<GPSIG_DP, GPSIG_M>(const SigArgs &, int, long long, hipStream_t);
}
