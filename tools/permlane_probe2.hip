// Stage dump of the wave reduce-scatter (for debugging against a host simulation).
#include <cstdio>
#include <vector>
#include "../gpsig_amd/csrc/common.h"
constexpr int K = 5;
__global__ void probe(const float *in, float *o1, float *o2, float *o3) {
  const int l = threadIdx.x;
  float v[4 * K];
#pragma unroll
  for (int i = 0; i < 4 * K; ++i) v[i] = in[i * 64 + l];
  float s1[2 * K], out[K];
#pragma unroll
  for (int i = 0; i < 2 * K; ++i) {
    const auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, v[2 * i]),
                                                    __builtin_bit_cast(unsigned, v[2 * i + 1]), false, false);
    s1[i] = __builtin_bit_cast(float, r[0]) + __builtin_bit_cast(float, r[1]);
    o1[i * 64 + l] = s1[i];
  }
#pragma unroll
  for (int i = 0; i < K; ++i) {
    const auto r = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, s1[2 * i]),
                                                    __builtin_bit_cast(unsigned, s1[2 * i + 1]), false, false);
    out[i] = __builtin_bit_cast(float, r[0]) + __builtin_bit_cast(float, r[1]);
    o2[i * 64 + l] = out[i];
  }
#pragma unroll
  for (int i = 0; i < K; ++i) out[i] += gpsig::dpp_f<0x128>(out[i]);
#pragma unroll
  for (int i = 0; i < K; ++i) o3[i * 64 + l] = out[i];
}
int main() {
  std::vector<float> h(4 * K * 64), a(2 * K * 64), b(K * 64), c(K * 64);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 37) % 101) - 50.0f;
  float *di, *d1, *d2, *d3;
  (void)hipMalloc(&di, h.size() * 4); (void)hipMalloc(&d1, a.size() * 4); (void)hipMalloc(&d2, b.size() * 4); (void)hipMalloc(&d3, c.size() * 4);
  (void)hipMemcpy(di, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, di, d1, d2, d3);
  (void)hipMemcpy(a.data(), d1, a.size() * 4, hipMemcpyDeviceToHost);
  (void)hipMemcpy(b.data(), d2, b.size() * 4, hipMemcpyDeviceToHost);
  (void)hipMemcpy(c.data(), d3, c.size() * 4, hipMemcpyDeviceToHost);
  for (float x : a) printf("%g ", x); printf("\n");
  for (float x : b) printf("%g ", x); printf("\n");
  for (float x : c) printf("%g ", x); printf("\n");
  return 0;
}
