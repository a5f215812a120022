// Micro-benchmark: fp32 FMA throughput of v_fma_f32 (scalar) vs v_pk_fma_f32 (packed pairs) on gfx950, at
// 1, 2 and 4 waves per SIMD, independent chains.  Decides whether a packed rewrite of a VALU-bound kernel can
// buy cycles.  Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_pk.hip -o tools/bin/ubench_pk
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int ITERS = 8192;

template <int CH>
__global__ __launch_bounds__(256) void scalar_fma(float *out, float a, float b) {
  float v[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) v[c] = threadIdx.x * 1e-3f + c;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) v[c] = __builtin_fmaf(v[c], a, b);
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) s += v[c];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int CH>
__global__ __launch_bounds__(256) void packed_fma(float *out, float a, float b) {
  f2 v[CH / 2];
#pragma unroll
  for (int c = 0; c < CH / 2; ++c) v[c] = (f2){threadIdx.x * 1e-3f + 2 * c, threadIdx.x * 1e-3f + 2 * c + 1};
  const f2 aa = (f2){a, a}, bb = (f2){b, b};
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH / 2; ++c) v[c] = __builtin_elementwise_fma(v[c], aa, bb);
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CH / 2; ++c) s += v[c][0] + v[c][1];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <typename K>
static double run(K kern, int blocks, float *out) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 0.999f, 1e-3f);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 0.999f, 1e-3f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main() {
  float *out;
  hipMalloc(&out, 256 * 4096 * sizeof(float));
  for (int wps : {1, 2, 4}) {  // waves per SIMD: 256 CUs x 4 SIMDs x wps waves, 4 waves per block
    const int blocks = 256 * wps;
    const double fl = (double)blocks * 256 * 16 * ITERS * 2;  // 16 values per thread, one FMA each per iter
    const double ts = run(scalar_fma<16>, blocks, out), tp = run(packed_fma<16>, blocks, out);
    printf("{\"waves_per_simd\": %d, \"scalar_ms\": %.4f, \"packed_ms\": %.4f, \"scalar_tflops\": %.1f, "
           "\"packed_tflops\": %.1f}\n", wps, ts, tp, fl / ts / 1e9, fl / tp / 1e9);
  }
  return 0;
}
