// fp32 dense layers of the value head (reference AlphaGo/models/value.py:26-28:
// Flatten -> Dense(256) -> Dense(1, tanh)) on gfx950, replacing the library
// GEMMs (hipBLASLt addmm / mm) of round 1.
//
//   forward     h  = z W1 + b1        M = boards, N = 256, K = S*S (361)
//   weight grad dW1 = z^T dh          M = S*S,    N = 256, K = boards
//   input grad  dz = dh W1^T          M = boards, N = S*S, K = 256
//
// One kernel, C[M][N] = beta*C + sum_k A[m][k] B[k][n] (+ bias[n]), with A
// and B read either row-major or transposed (TA/TB) so no operand is ever
// copied.  Exact fp32 on the f32-input MFMA v_mfma_f32_32x32x2_f32 (the
// result is a k-ordered fp32 fma chain -- same rate as the fp32 vector FMA,
// but one VGPR per operand per lane and the VALU left for staging).
// Workgroup tile 64x64, four waves each owning one 32x32 quadrant, K staged
// through LDS in steps of 32 ([k][m] / [k][n] images, +1 padding).  Few
// output tiles and a long K (dW1 = z^T dh: 24 tiles, K = boards) are split
// over K (grid.z) into fp32 partial slabs that dense_reduce_kernel sums in
// split order.  Fixed summation order everywhere: deterministic.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdexcept>

#include "common.h"
#include "kernels.h"

namespace agk {

namespace {
constexpr int DBM = 64, DBN = 64, DBK = 32;
}

template <bool TA, bool TB>
__global__ __launch_bounds__(256) void dense_f32_kernel(DenseArgs a) {
  __shared__ float As[DBK][DBM + 1];
  __shared__ float Bs[DBK][DBN + 1];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int m0 = blockIdx.y * DBM, n0 = blockIdx.x * DBN;
  const int kbeg = blockIdx.z * a.kchunk;
  const int kend = min(a.K, kbeg + a.kchunk);
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  f32x16 acc;
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] = 0.f;
  for (int k0 = kbeg; k0 < kend; k0 += DBK) {
    // stage A[m0:+64][k0:+32] as As[k][m] and B[k0:+32][n0:+64] as Bs[k][n]
#pragma unroll
    for (int r = 0; r < (DBM * DBK) / 256; ++r) {
      const int idx = r * 256 + tid;
      int m, k;
      if (TA) {  // A stored [k][m]: consecutive threads walk m
        m = idx & (DBM - 1);
        k = idx >> 6;
      } else {   // A stored [m][k]: consecutive threads walk k
        k = idx & (DBK - 1);
        m = idx >> 5;
      }
      const int gm = m0 + m, gk = k0 + k;
      float v = 0.f;
      if (gm < a.M && gk < kend) v = TA ? a.A[(size_t)gk * a.lda + gm] : a.A[(size_t)gm * a.lda + gk];
      As[k][m] = v;
    }
#pragma unroll
    for (int r = 0; r < (DBN * DBK) / 256; ++r) {
      const int idx = r * 256 + tid;
      int n, k;
      if (TB) {  // B stored [n][k]
        k = idx & (DBK - 1);
        n = idx >> 5;
      } else {   // B stored [k][n]
        n = idx & (DBN - 1);
        k = idx >> 6;
      }
      const int gn = n0 + n, gk = k0 + k;
      float v = 0.f;
      if (gn < a.N && gk < kend) v = TB ? a.B[(size_t)gn * a.ldb + gk] : a.B[(size_t)gk * a.ldb + gn];
      Bs[k][n] = v;
    }
    __syncthreads();
    // v_mfma_f32_32x32x2_f32: lane l holds A[i = l&31][k = l>>5] and B[k = l>>5][j = l&31]
    const int i = lane & 31, kk = lane >> 5;
#pragma unroll
    for (int ks = 0; ks < DBK; ks += 2)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(As[ks + kk][wm + i], Bs[ks + kk][wn + i], acc, 0, 0, 0);
    __syncthreads();
  }
  // C/D layout: col = lane & 31, row = (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5)
  const int col = n0 + wn + (lane & 31);
  if (col >= a.N) return;
  if (a.splits > 1) {  // partial slab [split][M][N]; dense_reduce_kernel finishes
    float* ws = a.ws + (size_t)blockIdx.z * a.M * a.N;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int row = m0 + wm + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
      if (row < a.M) ws[(size_t)row * a.N + col] = acc[e];
    }
    return;
  }
  const float bv = a.bias ? a.bias[col] : 0.f;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int row = m0 + wm + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
    if (row < a.M) {
      float* c = a.C + (size_t)row * a.ldc + col;
      const float v = acc[e] + bv;
      *c = a.beta != 0.f ? a.beta * *c + v : v;
    }
  }
}

// C = beta*C + sum_split ws[split] (+ bias), splits summed in order
__global__ __launch_bounds__(256) void dense_reduce_kernel(DenseArgs a) {
  const size_t mn = (size_t)a.M * a.N;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < mn; i += (size_t)gridDim.x * blockDim.x) {
    float v = 0.f;
    for (int z = 0; z < a.splits; ++z) v += a.ws[(size_t)z * mn + i];
    const int row = (int)(i / a.N), col = (int)(i - (size_t)row * a.N);
    if (a.bias) v += a.bias[col];
    float* c = a.C + (size_t)row * a.ldc + col;
    *c = a.beta != 0.f ? a.beta * *c + v : v;
  }
}

int dense_splits(int M, int N, int K) {
  const int tiles = ((M + DBM - 1) / DBM) * ((N + DBN - 1) / DBN);
  int s = (256 + tiles - 1) / tiles;         // about one workgroup per CU
  const int kmax = (K + 4 * DBK - 1) / (4 * DBK);  // each split keeps >= 4 K-steps
  if (s > kmax) s = kmax;
  return s < 1 ? 1 : s;
}

void launch_dense_f32(const DenseArgs& a_in, bool ta, bool tb, hipStream_t st) {
  DenseArgs a = a_in;
  if (a.splits < 1) a.splits = 1;
  a.kchunk = ((a.K + a.splits - 1) / a.splits + DBK - 1) / DBK * DBK;
  a.splits = (a.K + a.kchunk - 1) / a.kchunk;
  if (a.splits > 1 && !a.ws) throw std::invalid_argument("dense_f32: split-K needs a workspace");
  dim3 grid((a.N + DBN - 1) / DBN, (a.M + DBM - 1) / DBM, a.splits);
  if (!ta && !tb) hipLaunchKernelGGL((dense_f32_kernel<false, false>), grid, dim3(256), 0, st, a);
  else if (ta && !tb) hipLaunchKernelGGL((dense_f32_kernel<true, false>), grid, dim3(256), 0, st, a);
  else if (!ta && tb) hipLaunchKernelGGL((dense_f32_kernel<false, true>), grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((dense_f32_kernel<true, true>), grid, dim3(256), 0, st, a);
  if (a.splits > 1) {
    const size_t mn = (size_t)a.M * a.N;
    const int blocks = (int)std::min<size_t>((mn + 255) / 256, 1024);
    hipLaunchKernelGGL(dense_reduce_kernel, dim3(blocks), dim3(256), 0, st, a);
  }
}

}  // namespace agk
