// gpsig_amd -- explicit instantiation unit: the PDE adjoint kernels for one channel count.  Compiled
// once per GPSIG_DP by gpsig_amd/csrc/Makefile.
#include "pde_bwd.h"
#if !defined(GPSIG_DP)
#error "GPSIG_DP must be defined"
#endif
namespace gpsig {
template int pde_bwd_launch_dp<GPSIG_DP>(const PdeBwdArgs &, long long, int, hipStream_t);
}
