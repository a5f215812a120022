// gpsig_amd -- explicit instantiation unit: all first-order kernels for one channel count.
// Compiled once per GPSIG_DP value by gpsig_amd/csrc/Makefile.
#include "sig_fo.h"
#ifndef GPSIG_DP
#error "GPSIG_DP must be defined"
#endif
namespace gpsig {
template int sig_fo_launch_dp<GPSIG_DP>(const SigArgs &, int, long long, hipStream_t);
}
