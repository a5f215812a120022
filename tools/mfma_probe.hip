// Layout probe for v_mfma_f32_4x4x1_16b_f32 on gfx950: prints, for every lane and accumulator
// register, which (A lane, B lane) product it received.  A = 1000 + lane, B = lane + 1 (exact in f32), so
// D = A*B identifies both lanes.  Also checks the CBSZ/ABID broadcast of A from block 0.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void probe(float *out, float *outb) {
  const int l = threadIdx.x;
  const float a = 1000.0f + l, b = (float)(l + 1);
  f4 c = {0, 0, 0, 0};
  f4 d = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
  f4 e = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 4, 0, 0);  // CBSZ=4: broadcast A of block ABID=0
  for (int r = 0; r < 4; ++r) {
    out[l * 4 + r] = d[r];
    outb[l * 4 + r] = e[r];
  }
}

int main() {
  float *o, *ob;
  hipMalloc(&o, 256 * 4);
  hipMalloc(&ob, 256 * 4);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, o, ob);
  float h[256], hb[256];
  hipMemcpy(h, o, sizeof h, hipMemcpyDeviceToHost);
  hipMemcpy(hb, ob, sizeof hb, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int l = 0; l < 64; ++l)
    for (int r = 0; r < 4; ++r) {
      // decode: D = (1000 + la) * lb
      auto dec = [](float v, int &la, int &lb) {
        la = -1, lb = -1;
        for (int x = 0; x < 64; ++x) {
          const float q = v / (1000.0f + x);
          const int qi = (int)(q + 0.5f);
          if (qi >= 1 && qi <= 64 && (1000.0f + x) * qi == v) { la = x; lb = qi - 1; return; }
        }
      };
      int la, lb, lab, lbb;
      dec(h[l * 4 + r], la, lb);
      dec(hb[l * 4 + r], lab, lbb);
      if (l < 8 || l % 16 == 0) printf("lane %2d reg %d: A lane %2d B lane %2d | bcast A lane %2d B lane %2d\n", l, r, la, lb, lab, lbb);
      // expected (hypothesis): block = l/4, col = l%4, row = r: A lane 4*block + r, B lane l
      if (la != 4 * (l / 4) + r || lb != l) ++bad;
      if (lab != r || lbb != l) ++bad;
    }
  printf("hypothesis mismatches: %d\n", bad);
  return 0;
}
