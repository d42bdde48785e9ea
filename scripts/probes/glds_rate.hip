// Probe: LDS-DMA (global_load_lds_dwordx4) throughput per CU, alone and with
// concurrent ds_read_b128 traffic.  One 512-thread workgroup per CU streams
// 1-KB pieces from an L2-resident 2 MB buffer into a 2 x 72 KB LDS double
// buffer (the shape of the 384-pixel conv tile's staging), NSTEP steps.
// Build: hipcc --offload-arch=gfx950 -O3 glds_rate.hip -o glds_rate
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>

#define AG_LDS(p) ((__attribute__((address_space(3))) void*)(p))
typedef __attribute__((ext_vector_type(4))) float f4;

template <int READS>
__global__ __launch_bounds__(512, 1) void probe(const char* src, float* out, int nstep, int pieces_per_wave) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int STAGE = 72 * 1024;
  f4 acc = {0, 0, 0, 0};
  const char* base = src + ((blockIdx.x * 8 + wave) % 64) * 32768;
  for (int s = 0; s < nstep; ++s) {
    char* lb = smem + (s & 1) * STAGE;
    for (int i = 0; i < pieces_per_wave; ++i) {
      const char* g = base + ((s * pieces_per_wave + i) & 31) * 1024 + lane * 16;
      __builtin_amdgcn_global_load_lds((const void*)g, AG_LDS(lb + (wave * pieces_per_wave + i) * 1024), 16, 0, 0);
    }
    if (READS) {
      const char* rb = smem + ((s + 1) & 1) * STAGE;
#pragma unroll
      for (int r = 0; r < READS; ++r) acc += *(const f4*)(rb + ((r * 8 + wave) * 1024 + lane * 16) % STAGE);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (acc[0] == 12345.f) out[0] = acc[1];
}

int main() {
  int ncu = 256;
  char* src; float* out;
  hipMalloc(&src, 4 << 20); hipMalloc(&out, 64);
  hipMemset(src, 1, 4 << 20);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const int nstep = 2000, ppw = 9;  // 9 x 1 KB per wave per step = 72 KB per CU per step
  auto run = [&](auto kern, const char* name) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * 72 * 1024);
    for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(kern, dim3(ncu), dim3(512), 2 * 72 * 1024, 0, src, out, 200, ppw);
    hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(ncu), dim3(512), 2 * 72 * 1024, 0, src, out, nstep, ppw);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    double bytes = (double)ncu * nstep * 72 * 1024;
    printf("%-28s %8.3f ms  %7.1f GB/s/CU  %6.1f TB/s chip  %6.0f ns/step\n", name, ms, bytes / ncu / (ms * 1e-3) / 1e9,
           bytes / (ms * 1e-3) / 1e12, ms * 1e6 / nstep);
  };
  run(probe<0>, "glds only");
  run(probe<24>, "glds + 24 ds_read_b128/wave");
  run(probe<48>, "glds + 48 ds_read_b128/wave");
  return 0;
}
