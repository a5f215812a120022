// Semantics probe of v_permlane32_swap_b32 / v_permlane16_swap_b32 on gfx950: a = lane, b = 100 + lane.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int *o) {
  const unsigned l = threadIdx.x;
  const auto r = __builtin_amdgcn_permlane32_swap(l, 100u + l, false, false);
  const auto q = __builtin_amdgcn_permlane16_swap(l, 100u + l, false, false);
  o[l] = r[0]; o[64 + l] = r[1]; o[128 + l] = q[0]; o[192 + l] = q[1];
}
int main() {
  int *d, h[256];
  (void)hipMalloc(&d, sizeof h);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  (void)hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  const char *nm[4] = {"p32.r0", "p32.r1", "p16.r0", "p16.r1"};
  for (int t = 0; t < 4; ++t) {
    printf("%s:", nm[t]);
    for (int l = 0; l < 64; l += 4) printf(" %d", h[t * 64 + l]);
    printf("\n");
  }
  return 0;
}
