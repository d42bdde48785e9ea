// Probe: operand lane layout of v_mfma_scale_f32_16x16x128_f8f6f4 with e4m3 A/B (exact small-integer data).
// Build+run on the GPU box: hipcc --offload-arch=gfx950 scripts/probes/fp8_mfma_layout.hip -o gpurun_out/p && gpurun_out/p
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
__global__ void k(const unsigned char* A, const unsigned char* B, float* C) {
  int l = threadIdx.x;
  i32x8 a, b;
  const int* pa = (const int*)(A + l * 32);
  const int* pb = (const int*)(B + l * 32);
  for (int i = 0; i < 8; ++i) { a[i] = pa[i]; b[i] = pb[i]; }
  f32x4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 127, 0, 127);
  for (int r = 0; r < 4; ++r) C[l * 4 + r] = c[r];
}
static unsigned char enc(int v) { switch (v) { case 0: return 0; case 1: return 0x38; case 2: return 0x40; case -1: return 0xB8; default: return 0xC0; } }
int main() {
  srand(7);
  std::vector<int> av(64 * 32), bv(64 * 32);
  std::vector<unsigned char> ab(64 * 32), bb(64 * 32);
  for (int i = 0; i < 64 * 32; ++i) { av[i] = rand() % 5 - 2; bv[i] = rand() % 5 - 2; ab[i] = enc(av[i]); bb[i] = enc(bv[i]); }
  unsigned char *dA, *dB; float* dC;
  hipMalloc(&dA, 2048); hipMalloc(&dB, 2048); hipMalloc(&dC, 64 * 4 * 4);
  hipMemcpy(dA, ab.data(), 2048, hipMemcpyHostToDevice);
  hipMemcpy(dB, bb.data(), 2048, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dC);
  std::vector<float> C(256);
  hipMemcpy(C.data(), dC, 1024, hipMemcpyDeviceToHost);
  // hypotheses for k index of (lane, byte j)
  for (int h = 0; h < 3; ++h) {
    float Am[16][128] = {}, Bm[128][16] = {};
    for (int l = 0; l < 64; ++l)
      for (int j = 0; j < 32; ++j) {
        int kk;
        if (h == 0) kk = 32 * (l >> 4) + j;                        // contiguous 32 per lane group
        else if (h == 1) kk = 16 * (l >> 4) + (j & 15) + 64 * (j >> 4);  // two 16-wide halves
        else kk = 8 * (l >> 4) + (j & 7) + 32 * (j >> 3);            // four 8-wide quarters
        Am[l & 15][kk] = av[l * 32 + j];
        Bm[kk][l & 15] = bv[l * 32 + j];
      }
    int bad = 0;
    for (int l = 0; l < 64; ++l)
      for (int r = 0; r < 4; ++r) {
        int row = (l >> 4) * 4 + r, col = l & 15;
        float s = 0;
        for (int kk = 0; kk < 128; ++kk) s += Am[row][kk] * Bm[kk][col];
        if (s != C[l * 4 + r]) ++bad;
      }
    printf("hypothesis %d: %d mismatches of 256\n", h, bad);
  }
  printf("C[0..3] = %f %f %f %f\n", C[0], C[1], C[2], C[3]);
  return 0;
}
