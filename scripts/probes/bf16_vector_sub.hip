#include <hip/hip_runtime.h>
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
__global__ void k(bf16x8* a, const bf16x8* b, const bf16x8* c) {
  int i = threadIdx.x;
  a[i] = b[i] - c[i];
}
__global__ void k2(float* a, const float* b) {
  int i = threadIdx.x;
  a[i] = __builtin_amdgcn_ds_bpermute(i*4, (int)b[i]);
}
