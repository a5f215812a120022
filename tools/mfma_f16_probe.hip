// Rounding probe of v_mfma_f32_16x16x32_f16 (and, for comparison, v_mfma_f32_16x16x4_f32): random operands with
// a spread of magnitudes; per output |err| / sum |products| (max) and the mean SIGNED error in units of the
// output's fp32 ulp (a rounding bias shows as a mean far from 0), with the C input 0 or a large offset.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
__global__ void k16(const _Float16 *A, const _Float16 *B, const float *C, float *D) {
  const int l = threadIdx.x;
  h8 a, b;
  for (int e = 0; e < 8; ++e) {
    a[e] = A[(l & 15) * 32 + 8 * (l >> 4) + e];
    b[e] = B[(8 * (l >> 4) + e) * 16 + (l & 15)];
  }
  f4 c;
  for (int r = 0; r < 4; ++r) c[r] = C[(4 * (l >> 4) + r) * 16 + (l & 15)];
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[(4 * (l >> 4) + r) * 16 + (l & 15)] = c[r];
}
int main(int argc, char **argv) {
  const float spread = argc > 1 ? atof(argv[1]) : 8.0f;
  const float coff = argc > 2 ? atof(argv[2]) : 0.0f;  // C = coff * sum|p|
  const int allpos = argc > 3 ? atoi(argv[3]) : 0;
  _Float16 hA[16 * 32], hB[32 * 16];
  float hC[256], hD[256];
  srand(7);
  double worst = 0, bias = 0;
  long cnt = 0;
  _Float16 *dA, *dB;
  float *dC, *dD;
  (void)hipMalloc(&dA, sizeof hA); (void)hipMalloc(&dB, sizeof hB); (void)hipMalloc(&dC, sizeof hC); (void)hipMalloc(&dD, sizeof hD);
  for (int trial = 0; trial < 400; ++trial) {
    for (int i = 0; i < 512; ++i) {
      float u = (rand() / (float)RAND_MAX - 0.5f) * 2.0f, v = (rand() / (float)RAND_MAX - 0.5f) * 2.0f;
      if (allpos) { u = fabsf(u); v = fabsf(v); }
      hA[i] = (_Float16)(u * exp2f(spread * (rand() / (float)RAND_MAX)));
      hB[i] = (_Float16)(v * exp2f(spread * (rand() / (float)RAND_MAX)));
    }
    double ex[256], ab[256];
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        double e = 0, a = 0;
        for (int kk = 0; kk < 32; ++kk) {
          const double p = (double)(float)hA[i * 32 + kk] * (double)(float)hB[kk * 16 + j];
          e += p;
          a += fabs(p);
        }
        hC[i * 16 + j] = (float)(coff * a);
        ex[i * 16 + j] = e + (double)hC[i * 16 + j];
        ab[i * 16 + j] = a;
      }
    (void)hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
    (void)hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
    (void)hipMemcpy(dC, hC, sizeof hC, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k16, dim3(1), dim3(64), 0, 0, dA, dB, dC, dD);
    (void)hipMemcpy(hD, dD, sizeof hD, hipMemcpyDeviceToHost);
    for (int e = 0; e < 256; ++e) {
      if (ab[e] <= 0) continue;
      const double err = (double)hD[e] - ex[e];
      worst = fmax(worst, fabs(err) / ab[e]);
      int ee;
      frexp(ex[e], &ee);
      const double ulp = ldexp(1.0, ee - 24);
      bias += err / ulp;
      ++cnt;
    }
  }
  printf("f16 mfma spread 2^%.0f C=%.1f*sum|p| allpos=%d: max |err|/sum|p| %.3e  mean signed err %.3f ulp\n", spread, coff,
         allpos, worst, bias / cnt);
  return 0;
}
