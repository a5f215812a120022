// A/B timing harness for the first-order Gram VJP kernel (sig_bwd.h), one instantiation, no ABI:
// K(X) upper-triangle pairs, RBF difference seed, unit upstream gradient, no saved state.
//   ./kbench_vjp N reps  ->  "variant ms_per_launch checksum"
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../gpsig_amd/csrc/sig_bwd_pk.h"

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
#define KL 100
#endif
#ifndef KW
#define KW 4
#endif
#ifndef KLP
#define KLP 32
#endif
#ifndef KPK  // 1: the packed column-pair kernel (sig_bwd_pk.h)
#define KPK 0
#endif
#ifndef KSTATE  // 1: a (zero) saved forward state, as the training step's VJP launch
#define KSTATE 0
#endif

using namespace gpsig;

#define CK(x)                                                                                 \
  do {                                                                                        \
    hipError_t e = (x);                                                                       \
    if (e != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } \
  } while (0)

int main(int argc, char **argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 1024;
  const int reps = argc > 2 ? atoi(argv[2]) : 5;
  const int l = KL, d = KD, M = KM;
  constexpr int DP = KD;
  const int FS = feat_stride(DP);
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
  float *dF, *dG, *dGX;
  CK(hipMalloc(&dF, F.size() * 4));
  CK(hipMalloc(&dG, (size_t)(M + 1) * n * n * 4));
  CK(hipMalloc(&dGX, (size_t)n * l * d * 4));
  CK(hipMemcpy(dF, F.data(), F.size() * 4, hipMemcpyHostToDevice));
  std::vector<float> G((size_t)(M + 1) * n * n);
  for (auto &v : G) v = (float)(rnd() - 0.5);
  CK(hipMemcpy(dG, G.data(), G.size() * 4, hipMemcpyHostToDevice));
  BwdArgs p{};
  p.FX = p.FY = dF;
  p.n1 = p.n2 = n;
  p.l1 = p.l2 = l;
  p.d = d;
  p.M = M;
  p.pair_mode = GPSIG_PAIRS_UPPER;
  p.row_begin = 0;
  p.row_end = n;
  p.gout = dG;
  p.gout_levels = 1;
  p.g_ld = n;
  p.g_lvl = (long long)n * n;
  p.gX = p.gY = dGX;
  p.nblk = 1;
  if (KSTATE) {
    float *dS;
    const size_t sb = (size_t)n * (n + 1) / 2 * state_stride(M, l) * 4;
    CK(hipMalloc(&dS, sb));
    CK(hipMemset(dS, 0, sb));
    p.state = dS;
  }
  const int G_ = 64 / KLP;
  const long long ntb = (n + G_ - 1) / G_, nta = (n + 3) / 4;
  p.ntb = (int)ntb;
  const long long nblocks = upper_prefix_g(nta, ntb, G_);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto launch = [&]() {
    if constexpr (KPK)
      hipLaunchKernelGGL((sig_bwd_pk_kernel<DP, KW, KLP, KM, SEED_RBF_DIFF>), dim3((unsigned)nblocks), dim3(256), 0, 0, p);
    else
      hipLaunchKernelGGL((sig_bwd_kernel<DP, KW, KLP, KM, SEED_RBF_DIFF>), dim3((unsigned)nblocks), dim3(256), 0, 0, p);
  };
  CK(hipMemset(dGX, 0, (size_t)n * l * d * 4));
  launch();
  CK(hipDeviceSynchronize());
  std::vector<float> gx((size_t)n * l * d);
  CK(hipMemcpy(gx.data(), dGX, gx.size() * 4, hipMemcpyDeviceToHost));
  double cs = 0;
  for (size_t i = 0; i < gx.size(); ++i) cs += gx[i] * (1.0 + 1e-3 * (i % 13));
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) launch();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("%s n=%d L=%d D=%d M=%d W=%d LP=%d pk=%d state=%d ms=%.3f chk=%.9e\n", VARIANT, n, l, d, M, KW, KLP, KPK, KSTATE,
         ms / reps, cs);
  return 0;
}
