// gpsig_amd -- tensor-vs-sequence, tensor Gram and VOSF rescaled kernels (in progress).
#include "sig_common.h"

extern "C" int gpsig_tens_vs_seq(const float *, int, int, int, int, const float *, int, int, int, int, int, int,
                                 float *, void *, size_t, gpsig_stream_t) {
  return GPSIG_EUNSUPPORTED;
}
extern "C" int gpsig_tens_gram(const float *, int, int, int, int, int, int, float *, gpsig_stream_t) {
  return GPSIG_EUNSUPPORTED;
}
extern "C" int gpsig_rescaled(const float *, int, int, const float *, int, int, int, int, int, float *,
                              gpsig_stream_t) {
  return GPSIG_EUNSUPPORTED;
}
extern "C" size_t gpsig_tens_workspace_bytes(int n, int l, int d) { return (size_t)n * l * (2 * d + 4) * 4 + 256; }
