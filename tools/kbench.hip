// A/B timing harness for the first-order Gram kernel (one instantiation), independent of the ABI.
// Build variants with -D flags (GPSIG_FO_BLOCKED, GPSIG_D2_RECUR, GPSIG_FO_LB) and compare in one
// gpurun call:  ./kbench N reps  ->  prints "variant ms_per_launch entries_per_s"
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../gpsig_amd/csrc/sig_fo.h"

#ifndef VARIANT
#define VARIANT "default"
#endif
#ifndef KD
#define KD 5
#endif
#ifndef KM
#define KM 5
#endif
#ifndef KL
#define KL 128
#endif
#ifndef KW
#define KW 4
#endif
#ifndef KLP
#define KLP 32
#endif
#ifndef KMF
#define KMF 0
#endif

using namespace gpsig;

#define CK(x)                                                                                 \
  do {                                                                                        \
    hipError_t e = (x);                                                                       \
    if (e != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } \
  } while (0)

int main(int argc, char **argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 2048;
  const int reps = argc > 2 ? atoi(argv[2]) : 5;
  const int l = KL, d = KD, M = KM;
  constexpr int DP = KD;
  const int FS = feat_stride(DP);
  // random walks, features on the host (layout of features_kernel)
  std::vector<float> X((size_t)n * l * d), F((size_t)n * l * FS, 0.f);
  unsigned long long st = 12345;
  auto rnd = [&]() {
    st = st * 6364136223846793005ULL + 1442695040888963407ULL;
    return ((st >> 11) * (1.0 / 9007199254740992.0));
  };
  for (int a = 0; a < n; ++a)
    for (int k = 0; k < d; ++k) {
      double acc = 0;
      for (int i = 0; i < l; ++i) {
        const double u1 = rnd() + 1e-12, u2 = rnd();
        acc += std::sqrt(-2 * std::log(u1)) * std::cos(6.283185307179586 * u2);
        X[((size_t)a * l + i) * d + k] = (float)(acc / std::sqrt((double)l * d));
      }
    }
  for (int a = 0; a < n; ++a)
    for (int i = 0; i < l; ++i) {
      float h = 0;
      for (int k = 0; k < DP; ++k) {
        const float xv = X[((size_t)a * l + i) * d + k];
        const float dv = i + 1 < l ? X[((size_t)a * l + i + 1) * d + k] - xv : 0.f;
        F[((size_t)a * l + i) * FS + k] = xv;
        F[((size_t)a * l + i) * FS + DP + k] = dv;
        h += dv * dv;
      }
      F[((size_t)a * l + i) * FS + 2 * DP] = 0.5f * h;
      double gx = 0;
      for (int k = 0; k < DP; ++k) gx += (double)F[((size_t)a * l + i) * FS + k] * F[((size_t)a * l + i) * FS + DP + k];
      F[((size_t)a * l + i) * FS + 2 * DP + 1] = (float)(gx + 0.5 * h);
    }
  float *dF, *dOut;
  CK(hipMalloc(&dF, F.size() * 4));
  CK(hipMalloc(&dOut, (size_t)n * n * 4));
  CK(hipMemcpy(dF, F.data(), F.size() * 4, hipMemcpyHostToDevice));
  SigArgs p{};
  p.FX = p.FY = dF;
  p.n1 = p.n2 = n;
  p.l1 = p.l2 = l;
  p.fs = FS;
  p.M = M;
  p.order = 1;
  p.pair_mode = GPSIG_PAIRS_UPPER;
  p.row_begin = 0;
  p.row_end = n;
  p.out_mode = GPSIG_OUT_NORM_SUM;
  p.out = dOut;
  p.out_row0 = 0;
  p.out_rows = n;
  p.out_ld = n;
  p.out_lvl = (long long)n * n;
  const Geo geo{KW, KLP};
  const int G = 64 / geo.LP;
  const long long ntb = (n + G - 1) / G, nta = (n + 3) / 4;
  p.ntb = (int)ntb;
  p.tile_base = 0;
  const long long nblocks = upper_prefix_g(nta, ntb, G);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto launch = [&]() {
    hipLaunchKernelGGL((sig_fo_kernel<DP, KW, KLP, KM, SEED_RBF_DIFF, false, false, (KMF != 0)>),
                       dim3((unsigned)nblocks), dim3(256), 0, 0, p);
  };
  launch();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) launch();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  // checksum of the upper triangle (the launch stores both triangles; compare variants by it)
  std::vector<float> out((size_t)n * n);
  CK(hipMemcpy(out.data(), dOut, out.size() * 4, hipMemcpyDeviceToHost));
  double cs = 0, ca = 0;
  for (int a = 0; a < n; ++a)
    for (int b = a; b < n; ++b) {
      cs += out[(size_t)a * n + b] * (1.0 + 1e-3 * ((a * 7 + b) % 13));
      ca += std::fabs(out[(size_t)a * n + b]);
    }
  printf("%s n=%d L=%d D=%d M=%d ms=%.3f entries/s=%.4g chk=%.9e abs=%.9e\n", VARIANT, n, l, d, M, ms / reps,
         (double)n * n / (ms / reps / 1e3), cs, ca);
  return 0;
}
