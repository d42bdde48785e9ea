// Shared helpers for the gfx950 (CDNA4) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <stdexcept>
#include <string>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(2))) float f32x2;

#define AG_LDS(p) ((__attribute__((address_space(3))) void*)(p))

namespace agk {

// Host: throw on a HIP error (checked hipFuncSetAttribute etc.); surfaces in
// Python as a RuntimeError through the op wrappers.
inline void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

// Exact unsigned division by a runtime constant d (x < 2^32, d < 2^16):
// q = (x * m) >> 40 with m = ceil(2^40 / d), computed once on the host.
struct FastDiv {
  uint32_t d;
  uint64_t m;
};
inline FastDiv make_fastdiv(uint32_t d) { return FastDiv{d, ((1ull << 40) + d - 1) / d}; }
__device__ __forceinline__ uint32_t fdiv(uint32_t x, const FastDiv& f) {
  return (uint32_t)(((uint64_t)x * f.m) >> 40);
}

// 16-byte global -> LDS DMA (global_load_lds_dwordx4).  `lds_wave_base` must be
// wave-uniform: the hardware writes lane i's 16 bytes at base + 16*i.
__device__ __forceinline__ void glds16(const void* gsrc, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(gsrc, AG_LDS(lds_wave_base), 16, 0, 0);
}

__device__ __forceinline__ void wait_vmcnt0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ f32x4 mfma16x16x32(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float bf2f(__bf16 v) { return (float)v; }
__device__ __forceinline__ __bf16 f2bf(float v) { return (__bf16)v; }

__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

}  // namespace agk
