// Kernel-lab ISA probes (built into _hip_kernels_lab.so only).
// tr8_probe: pins the lane mapping of ds_read_b64_tr_b8 (the 8-bit transpose read the fp8 wgrad
// needs; the guides document only the 16-bit form).  LDS holds byte o = lds_init[o]; lane l reads
// 8 bytes with ds_read_b64_tr_b8 at byte address addr[l]; out[l] = the 8 bytes it received.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "common.h"
#include "kernels.h"

namespace agk {

namespace {

__global__ __launch_bounds__(64) void tr8_probe_kernel(const uint8_t* lds_init, int nbytes, const int* addr,
                                                      unsigned long long* out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[4096];
  for (int i = threadIdx.x; i < nbytes && i < 4096; i += 64) lds[i] = lds_init[i];
  __syncthreads();
  const int a = addr[threadIdx.x];
  typedef __attribute__((ext_vector_type(2))) unsigned u2;
  u2 v;
  asm volatile("ds_read_b64_tr_b8 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"((unsigned)(uintptr_t)(lds + a)));
  out[threadIdx.x] = ((unsigned long long)v.y << 32) | v.x;
}

}  // namespace

void launch_tr8_probe(const uint8_t* lds_init, int nbytes, const int* addr, unsigned long long* out, hipStream_t st) {
  hipLaunchKernelGGL(tr8_probe_kernel, dim3(1), dim3(64), 0, st, lds_init, nbytes, addr, out);
}

}  // namespace agk
