// Check of wave_reduce_scatter4 (common.h) against a host reduction: 64 lanes x 4K values.
#include <cstdio>
#include <vector>

#include "../gpsig_amd/csrc/common.h"

constexpr int K = 5;
__global__ void probe(const float *in, float *out) {
  const int l = threadIdx.x;
  float v[4 * K], o[K];
#pragma unroll
  for (int i = 0; i < 4 * K; ++i) v[i] = in[i * 64 + l];
  gpsig::wave_reduce_scatter4<K>(v, o);
#pragma unroll
  for (int i = 0; i < K; ++i) out[i * 64 + l] = o[i];
}

int main() {
  std::vector<float> h(4 * K * 64), r(K * 64);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 37) % 101) - 50.0f;
  float *di, *dout;
  (void)hipMalloc(&di, h.size() * 4);
  (void)hipMalloc(&dout, r.size() * 4);
  (void)hipMemcpy(di, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, di, dout);
  (void)hipMemcpy(r.data(), dout, r.size() * 4, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < K; ++i)
    for (int l = 0; l < 64; ++l) {
      const int idx = 4 * i + gpsig::ROW_SLOT[l / 16];
      double s = 0;
      for (int t = 0; t < 64; ++t) s += h[idx * 64 + t];
      if (r[i * 64 + l] != (float)s) {
        if (bad < 10) printf("out[%d] lane %d: got %g want %g\n", i, l, r[i * 64 + l], s);
        ++bad;
      }
    }
  printf("wave_reduce_scatter4 mismatches: %d\n", bad);
  return bad != 0;
}
