// One-GPU stand-in for an RCCL ring all-reduce running beside the backward:
// `channels` workgroups (RCCL runs one workgroup per channel) stream the
// bucket's bytes through the CUs they occupy -- a read of the bucket and a
// write to a scratch buffer, about the 2 (W-1)/W x bucket bytes a ring moves
// through each rank -- and hold their CUs until the wire time of the transfer
// has passed (bytes / bus bandwidth, measured on the 100 MHz real-time
// counter).  Launched on a side stream at every bucket point of the backward
// it reproduces the CU contention that the overlapped all-reduce costs the
// dgrad / wgrad kernels, which a world-1 RCCL group (a no-op ring) does not.
// Never touches the gradient (reads only).
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace agk {

__global__ __launch_bounds__(256) void comm_proxy_kernel(const float4* __restrict__ src, float4* __restrict__ dst,
                                                         long n4, long long ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x)
    dst[i] = src[i];
  while ((long long)(__builtin_amdgcn_s_memrealtime() - t0) < ticks) __builtin_amdgcn_s_sleep(8);
}

void launch_comm_proxy(const float* src, float* dst, long n, int channels, double wire_us, hipStream_t st) {
  const long n4 = n / 4;
  const long long ticks = (long long)(wire_us * 100.0);  // s_memrealtime: 100 MHz
  hipLaunchKernelGGL(comm_proxy_kernel, dim3(channels < 1 ? 1 : channels), dim3(256), 0, st,
                     reinterpret_cast<const float4*>(src), reinterpret_cast<float4*>(dst), n4, ticks);
}

}  // namespace agk
