// Fused move sampling for the batched samplers (search/selfplay.py BatchedSampler.sample_device): one
// workgroup per board draws a move from p**beta (p = the head's legal-masked softmax), -1 where the
// board has no sensible move.  Replaces a chain of ~10 small tensor kernels per ply and set (clamp,
// pow, where, sum, divide, multinomial, where) in the lock-step drivers, where at 10-256 boards per
// forward their launches were a visible part of each ply.  Reference semantics: the probabilistic
// player's sample of the move distribution raised to 1/temperature (AlphaGo/ai.py:37-49).
#include <hip/hip_runtime.h>

#include "common.h"
#include "kernels.h"

namespace agk {

namespace {
__device__ __forceinline__ uint64_t mix64(uint64_t x) {  // splitmix64 finaliser
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
}  // namespace

// NP <= 2 * 256: thread t owns entries 2t, 2t + 1
__global__ __launch_bounds__(256) void sample_moves_kernel(SampleArgs a) {
  __shared__ float wsum[4];
  __shared__ int wpick[4];
  const int b = blockIdx.x;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const float* p = a.probs + (size_t)b * a.NP;
  const int i0 = 2 * t, i1 = 2 * t + 1;
  float w0 = i0 < a.NP ? fmaxf(p[i0], 0.f) : 0.f;
  float w1 = i1 < a.NP ? fmaxf(p[i1], 0.f) : 0.f;
  if (a.beta != 1.f) {
    w0 = w0 > 0.f ? __powf(w0, a.beta) : 0.f;
    w1 = w1 > 0.f ? __powf(w1, a.beta) : 0.f;
  }
  // inclusive prefix sums: within the wave, then across the four waves
  float s = w0 + w1;
  float incl = s;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const float v = __shfl_up(incl, d, 64);
    if (lane >= d) incl += v;
  }
  if (lane == 63) wsum[wv] = incl;
  __syncthreads();
  float before = 0.f, total = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (k < wv) before += wsum[k];
    total += wsum[k];
  }
  const float hi = before + incl, lo = hi - s;  // this thread's cumulative range [lo, hi)
  // any sensible move: the caller's flag, or (legal mask) any nonzero entry of the row -- every
  // thread reaches this barrier
  const bool has = a.has ? a.has[b] != 0
                         : __syncthreads_or((i0 < a.NP && a.legal[(size_t)b * a.NP + i0]) ||
                                            (i1 < a.NP && a.legal[(size_t)b * a.NP + i1])) != 0;
  // u in [0, total): 24 random bits from (seed, board)
  const float u = (float)(mix64(a.seed * 0x100000001B3ull + (uint64_t)b) >> 40) * (1.f / 16777216.f) * total;
  // the thread whose range holds u picks; rounding at the top end falls back to the last positive entry
  int pick = -1;
  if (s > 0.f && u >= lo && u < hi) pick = (u < lo + w0 && w0 > 0.f) ? i0 : (w1 > 0.f ? i1 : i0);
  int last = w1 > 0.f ? i1 : (w0 > 0.f ? i0 : -1);
  // max over the block of pick and of last
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    pick = max(pick, __shfl_xor(pick, d, 64));
    last = max(last, __shfl_xor(last, d, 64));
  }
  __syncthreads();
  if (lane == 0) {
    wsum[wv] = (float)last;
    wpick[wv] = pick;
  }
  __syncthreads();
  if (t == 0) {
    int pk = -1, ls = -1;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      pk = max(pk, wpick[k]);
      ls = max(ls, (int)wsum[k]);
    }
    if (pk < 0) pk = ls;  // u fell on the top edge of the sum (float rounding)
    if (pk < 0) pk = 0;   // an all-zero row with has set: any index (the torch path samples uniformly)
    a.out[b] = has ? (int64_t)pk : (int64_t)-1;
  }
}

void launch_sample_moves(const SampleArgs& a, hipStream_t st) {
  if (a.B <= 0) return;
  hipLaunchKernelGGL(sample_moves_kernel, dim3(a.B), dim3(256), 0, st, a);
}

}  // namespace agk
