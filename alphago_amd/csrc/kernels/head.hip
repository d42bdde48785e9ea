// Fused policy head: 1x1 conv (F -> 1, scalar bias) + flatten + softmax over
// S*S + clipped categorical cross-entropy + top-1 accuracy + the whole backward
// of the head (dlogits, the ReLU-masked gradient into the last trunk layer, and
// per-board partials of the head weight/bias gradients).  One workgroup per
// board: the board's 361 x F activations are read from HBM once into registers
// (BoardRows / BoardRegs), and nothing of the head round-trips through HBM as a
// separate tensor.
//
// Reference ops replaced: policy.py:145-154 (Conv 1x1 / Flatten / Softmax),
// Keras categorical_crossentropy with output clipping (supervised_policy_trainer
// .py:200) and the 'accuracy' metric; inference renormalisation over legal
// moves replaces CNNPolicy._select_moves_and_normalize (policy.py:44-54).
#include <hip/hip_runtime.h>

#include "common.h"
#include "kernels.h"

namespace agk {

// boards below which the per-board head kernels run 1024 threads per workgroup instead of 256
constexpr int kHeadWideBelow = 256;

__device__ __forceinline__ float block_reduce_max(float v, float* red) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float r = red[0];
  for (int i = 1; i < (int)(blockDim.x >> 6); ++i) r = fmaxf(r, red[i]);
  return r;
}
__device__ __forceinline__ float block_reduce_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float r = 0.f;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) r += red[i];
  return r;
}

// z_s[p] = y[p, :] . w for every position of one board, coalesced and
// deterministic: each 32-lane half-wave owns one position at a time, lane c8
// (< C/8) reads 16 B of the position's row (one contiguous row per half-wave)
// and the 8-term partial dot products are summed with a fixed xor-shuffle tree.
__device__ __forceinline__ void head_dots(const __bf16* base, const float* w_s, float* z_s, int S, int C) {
  const int tid = threadIdx.x;
  const int SS = S * S;
  const int HP = S + 2;
  const int C8 = C >> 3;  // <= 32
  const int R = blockDim.x >> 5;
  const int l32 = tid & 31, slot = tid >> 5;
  const int c8 = l32 << 3;
  // HU rows in flight per half-wave: the loop is bound by load latency (one
  // workgroup per board, every workgroup resident at once), not bandwidth
  constexpr int HU = 8;
  for (int p0 = 0; p0 < SS; p0 += HU * R) {
    bf16x8 v[HU];
#pragma unroll
    for (int u = 0; u < HU; ++u) {
      const int p = p0 + u * R + slot;
      if (p < SS && l32 < C8) {
        const int i = p / S, j = p - (p / S) * S;
        v[u] = *(const bf16x8*)(base + (size_t)((i + 1) * HP + j + 1) * C + c8);
      } else {
        v[u] = bf16x8{};
      }
    }
#pragma unroll
    for (int u = 0; u < HU; ++u) {
      const int p = p0 + u * R + slot;
      float d = 0.f;
      if (l32 < C8) {  // w_s holds only the C real slots: lanes past them must not read it
#pragma unroll
        for (int e = 0; e < 8; ++e) d += (float)v[u][e] * w_s[c8 + e];
      }
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) d += __shfl_xor(d, o, 64);
      if (l32 == 0 && p < SS) z_s[p] = d;
    }
  }
  __syncthreads();
}

// Gradient of a 1x1 (F -> 1) head conv given dlogits g (in g_s, length S*S):
// ReLU'-masked dY into the trunk's last activation and per-board partials of
// dW_head (the dbias partial is written by the caller).
template <int NT>
__device__ __forceinline__ void head_input_backward(const PolicyHeadArgs& a, int b, const __bf16* base,
                                                    const float* w_s, const float* g_s) {
  // One pass over the board's activations: thread (r, c8) walks positions
  // p = r, r + R, ... for its 8-channel group, writing the ReLU'-masked dY and
  // accumulating sum_p g[p] * y[p, c] in registers; the R partials per
  // channel are then reduced through LDS.  Consecutive threads cover
  // consecutive 16-B channel groups of one position (coalesced rows).
  __shared__ float part[NT * 8];
  const int tid = threadIdx.x;
  const int SS = a.S * a.S;
  const int HP = a.S + 2;
  const int C8 = a.C >> 3;
  const int R = blockDim.x / C8;  // positions processed concurrently
  const int r = tid / C8, cg = tid - r * C8;
  __bf16* dzb = a.dz + (size_t)b * HP * HP * a.C;
  uint8_t* dz8b = a.dz8 ? a.dz8 + (size_t)b * HP * HP * a.C : nullptr;
  const float sc8 = a.dz8 ? *a.dz8_scale : 0.f;
  float m8 = 0.f;  // max |bf16 dY| (e5m2 output)
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (r < R) {
    const int c8 = cg << 3;
    // BU positions' loads issued before their stores (latency-bound loop)
    constexpr int BU = 8;
    for (int p0 = r; p0 < SS; p0 += BU * R) {
      bf16x8 v[BU];
      size_t off[BU];
#pragma unroll
      for (int u = 0; u < BU; ++u) {
        const int p = p0 + u * R;
        const int pc = p < SS ? p : SS - 1;
        const int i = pc / a.S, j = pc - (pc / a.S) * a.S;
        off[u] = (size_t)((i + 1) * HP + j + 1) * a.C + c8;
        v[u] = *(const bf16x8*)(base + off[u]);
      }
#pragma unroll
      for (int u = 0; u < BU; ++u) {
        const int p = p0 + u * R;
        if (p < SS) {
          const float g = g_s[p];
          bf16x8 o;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float y = (float)v[u][e];
            o[e] = (__bf16)(y > 0.f ? g * w_s[c8 + e] : 0.f);
            acc[e] += g * y;
          }
          if (dz8b) {
            // quantize_bf8_dev_kernel's conversion of the bf16 value: the same bytes and max, and the
            // bf16 dz is never written or re-read
            float f[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              f[e] = (float)o[e];
              m8 = fmaxf(m8, fabsf(f[e]));
              f[e] = fminf(fmaxf(f[e] * sc8, -57344.f), 57344.f);
            }
            int lo = __builtin_amdgcn_cvt_pk_bf8_f32(f[0], f[1], 0, false);
            lo = __builtin_amdgcn_cvt_pk_bf8_f32(f[2], f[3], lo, true);
            int hi = __builtin_amdgcn_cvt_pk_bf8_f32(f[4], f[5], 0, false);
            hi = __builtin_amdgcn_cvt_pk_bf8_f32(f[6], f[7], hi, true);
            *(int2*)(dz8b + off[u]) = make_int2(lo, hi);
          } else {
            *(bf16x8*)(dzb + off[u]) = o;
          }
        }
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) part[tid * 8 + e] = acc[e];
  if (dz8b) {  // one atomic per board into the spread amax slots
    __shared__ float red8[NT / 64];
    m8 = wave_max(m8);
    if ((tid & 63) == 0) red8[tid >> 6] = m8;
    __syncthreads();
    if (tid == 0) {
      for (int w = 1; w < NT / 64; ++w) m8 = fmaxf(m8, red8[w]);
      if (m8 > 0.f) atomicMax(a.dz8_amax + (b & (kFp8AmaxSlots - 1)), __float_as_uint(m8));
    }
  }
  __syncthreads();
  float* dh = a.dhead + (size_t)b * (a.C_real + 1);
  for (int c = tid; c < a.C_real; c += blockDim.x) {
    const int g8 = c >> 3, e = c & 7;
    float s = 0.f;
    for (int rr = 0; rr < R; ++rr) s += part[(rr * C8 + g8) * 8 + e];
    dh[c] = s;
  }
}

// One board's interior activations held in registers between the policy head's forward and
// backward passes, so the board is read from HBM once (head_dots + head_input_backward read it
// twice).  Half-wave `slot` owns positions slot, slot + R, ... (R = NT / 32); lane l32 < C / 8 owns
// the 16-byte channel group l32 of each.  P = ceil(361 / R) covers every board up to 19 x 19.
template <int NT>
struct BoardRegs {
  static constexpr int R = NT / 32;
  static constexpr int P = (361 + R - 1) / R;
  bf16x8 v[P];

  __device__ __forceinline__ static size_t offset(int p, int S, int C, int c8) {
    const int i = p / S, j = p - i * S;
    return (size_t)((i + 1) * (S + 2) + j + 1) * C + c8;
  }

  // every load issued before any is used: P outstanding 16-B loads per lane
  __device__ __forceinline__ void load(const __bf16* base, int S, int C) {
    const int l32 = threadIdx.x & 31, slot = threadIdx.x >> 5;
    const int SS = S * S;
    const bool lane = l32 < (C >> 3);
#pragma unroll
    for (int u = 0; u < P; ++u) {
      const int p = u * R + slot;
      v[u] = (p < SS && lane) ? *(const bf16x8*)(base + offset(p, S, C, l32 << 3)) : bf16x8{};
    }
  }

  // z_s[p] = y[p, :] . w with head_dots' xor-shuffle order (same bits)
  __device__ __forceinline__ void dots(const float* w_s, float* z_s, int S, int C) const {
    const int l32 = threadIdx.x & 31, slot = threadIdx.x >> 5;
    const int SS = S * S;
    const int c8 = l32 << 3;
    const bool lane = l32 < (C >> 3);
#pragma unroll
    for (int u = 0; u < P; ++u) {
      const int p = u * R + slot;
      float d = 0.f;
      if (lane) {
#pragma unroll
        for (int e = 0; e < 8; ++e) d += (float)v[u][e] * w_s[c8 + e];
      }
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) d += __shfl_xor(d, o, 64);
      if (l32 == 0 && p < SS) z_s[p] = d;
    }
    __syncthreads();
  }

  // ReLU'-masked dY = g[p] w into the trunk's last activation gradient and per-board partials of
  // dW_head (sum_p g[p] y[p, c], slot partials summed through LDS in slot order)
  __device__ __forceinline__ void backward(const PolicyHeadArgs& a, int b, const float* w_s,
                                           const float* g_s) const {
    __shared__ float part[NT * 8];
    const int tid = threadIdx.x;
    // laundered so the store addresses are recomputed here instead of kept live from load()
    // (23 x 64-bit addresses would push the 512-thread kernel past 128 VGPRs)
    int lane_id = tid;
    asm volatile("" : "+v"(lane_id));
    const int l32 = lane_id & 31, slot = lane_id >> 5;
    const int SS = a.S * a.S;
    const int c8 = l32 << 3;
    const bool lane = l32 < (a.C >> 3);
    __bf16* dzb = a.dz + (size_t)b * (a.S + 2) * (a.S + 2) * a.C;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    float wl[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) wl[e] = lane ? w_s[c8 + e] : 0.f;
#pragma unroll
    for (int u = 0; u < P; ++u) {
      const int p = u * R + slot;
      if (p < SS && lane) {
        const float g = g_s[p];
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float y = (float)v[u][e];
          o[e] = (__bf16)(y > 0.f ? g * wl[e] : 0.f);
          acc[e] += g * y;
        }
        *(bf16x8*)(dzb + offset(p, a.S, a.C, c8)) = o;
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) part[tid * 8 + e] = acc[e];
    __syncthreads();
    float* dh = a.dhead + (size_t)b * (a.C_real + 1);
    for (int c = tid; c < a.C_real; c += NT) {
      const int g8 = c >> 3, e = c & 7;
      float s = 0.f;
      for (int r = 0; r < R; ++r) s += part[(r * 32 + g8) * 8 + e];
      dh[c] = s;
    }
  }
};

// The same for large batches with fewer registers: thread t < S * C / 8 owns 16-byte chunk t of
// every board row (a row's interior is contiguous in the padded layout), so the 19 loads of a lane
// differ by one uniform row stride and no per-load address stays live.  A position's dot product
// is the fixed-order sum of its C / 8 lanes' partials through LDS.  Needs S * C / 8 <= NT.
template <int NT>
struct BoardRows {
  static constexpr int P = 19;
  bf16x8 v[P];

  __device__ __forceinline__ static size_t offset(int u, int S, int C, int t) {
    return (size_t)((u + 1) * (S + 2) + 1) * C + t * 8;
  }

  __device__ __forceinline__ void load(const __bf16* base, int S, int C) {
    const int t = threadIdx.x;
    const bool lane = t < S * (C >> 3);
#pragma unroll
    for (int u = 0; u < P; ++u) v[u] = (u < S && lane) ? *(const bf16x8*)(base + offset(u, S, C, t)) : bf16x8{};
  }

  __device__ __forceinline__ void dots(const float* w_s, float* z_s, int S, int C) const {
    __shared__ float dpart[P * NT];
    const int t = threadIdx.x;
    const int C8 = C >> 3;
    const int cg = t % C8;
    const bool lane = t < S * C8;
#pragma unroll
    for (int u = 0; u < P; ++u) {
      float d = 0.f;
      if (lane) {
#pragma unroll
        for (int e = 0; e < 8; ++e) d += (float)v[u][e] * w_s[cg * 8 + e];
      }
      dpart[u * NT + t] = d;
    }
    __syncthreads();
    for (int p = t; p < S * S; p += NT) {
      const int u = p / S, j = p - u * S;
      const float* q = dpart + u * NT + j * C8;
      float d = 0.f;
      for (int k = 0; k < C8; ++k) d += q[k];
      z_s[p] = d;
    }
    __syncthreads();
  }

  __device__ __forceinline__ void backward(const PolicyHeadArgs& a, int b, const float* w_s,
                                           const float* g_s) const {
    __shared__ float part[NT * 8];
    const int t = threadIdx.x;
    const int S = a.S, C8 = a.C >> 3;
    const int j = t / C8, cg = t - j * C8;
    const bool lane = t < S * C8;
    __bf16* dzb = a.dz + (size_t)b * (S + 2) * (S + 2) * a.C;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    float wl[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) wl[e] = lane ? w_s[cg * 8 + e] : 0.f;
#pragma unroll
    for (int u = 0; u < P; ++u) {
      if (u < S && lane) {
        const float g = g_s[u * S + j];
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float y = (float)v[u][e];
          o[e] = (__bf16)(y > 0.f ? g * wl[e] : 0.f);
          acc[e] += g * y;
        }
        *(bf16x8*)(dzb + offset(u, S, a.C, t)) = o;
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) part[t * 8 + e] = acc[e];
    __syncthreads();
    float* dh = a.dhead + (size_t)b * (a.C_real + 1);
    for (int c = t; c < a.C_real; c += NT) {
      const int g8 = c >> 3, e = c & 7;
      float s = 0.f;
      for (int jj = 0; jj < S; ++jj) s += part[(jj * C8 + g8) * 8 + e];
      dh[c] = s;
    }
  }
};

// Reference RL loss (reinforcement_policy_trainer.py:109, Keras 1.0
// binary_crossentropy on the softmax output): per board
//   L = -1/SS * sum_j [y_j log pc_j + (1 - y_j) log(1 - pc_j)],  pc = clip(p, 1e-7, 1 - 1e-7)
// with y the one-hot move; clip has zero gradient outside its range (Theano
// clip), and the softmax backward is dz_i = p_i (g_i - sum_j p_j g_j).
template <int NT, class Board>
__device__ void policy_bce_train(const PolicyHeadArgs& a, int b, int t, float wb, float zmax, float inv, int lidx,
                                 const Board& board, const float* w_s, float* z_s, float* red) {
  __shared__ float p_s[368];
  const int tid = threadIdx.x;
  const int SS = a.S * a.S;
  const float eps = 1e-7f;
  float ls = 0.f, pg = 0.f;
  for (int p = tid; p < SS; p += NT) {
    const float pr = (z_s[p] == -INFINITY) ? 0.f : __expf(z_s[p] - zmax) * inv;
    const float pc = fminf(fmaxf(pr, eps), 1.f - eps);
    const bool y = p == t;
    ls += y ? __logf(pc) : __logf(1.f - pc);
    const float g = (pr < eps || pr > 1.f - eps) ? 0.f : -(y ? 1.f / pr : -1.f / (1.f - pr)) / (float)SS;
    p_s[p] = pr;
    z_s[p] = g;
    pg += pr * g;
  }
  ls = block_reduce_sum(ls, red);
  pg = block_reduce_sum(pg, red);
  if (tid == 0) {
    a.loss[b] = t >= 0 ? -ls / (float)SS : 0.f;
    a.correct[b] = (t >= 0 && lidx == t) ? 1.f : 0.f;
  }
  const float sc = t >= 0 ? a.grad_scale * wb : 0.f;
  for (int p = tid; p < SS; p += NT) z_s[p] = p_s[p] * (z_s[p] - pg) * sc;
  __syncthreads();
  board.backward(a, b, w_s, z_s);
  float gs = 0.f;
  for (int p = tid; p < SS; p += NT) gs += z_s[p];
  gs = block_reduce_sum(gs, red);
  if (tid == 0) a.dhead[(size_t)b * (a.C_real + 1) + a.C_real] = gs;
}

// One workgroup per board, its activations read once into registers (Board).  Large batches: 512
// threads with BoardRows (126 VGPRs, two boards per CU).  Below kHeadWideBelow boards, or when a
// row does not fit 512 lanes: 1024 threads with BoardRegs (B = 16 has only 16 workgroups: a board's
// loads get all the lanes).
template <bool TRAIN, int NT, class Board>
__global__ __launch_bounds__(NT) void policy_head_kernel(PolicyHeadArgs a) {
  __shared__ float w_s[256];
  __shared__ float z_s[368];
  __shared__ float red[16];
  __shared__ int redi[16];
  // boards in reverse: the last-written boards of the final forward are the ones still in the
  // Infinity Cache, and they are read before this kernel's own dZ writes evict them
  const int b = (int)gridDim.x - 1 - (int)blockIdx.x;
  const int tid = threadIdx.x;
  const int SS = a.S * a.S;
  const int HP = a.S + 2;
  for (int c = tid; c < a.C; c += NT) w_s[c] = c < a.C_real ? a.w[c] : 0.f;
  Board board;
  board.load(a.y + (size_t)b * HP * HP * a.C, a.S, a.C);
  __syncthreads();
  const float bias = a.b[0];
  const uint8_t* legal = a.legal ? a.legal + (size_t)b * SS : nullptr;

  float lmax = -INFINITY;
  int lidx = 0x7fffffff;
  board.dots(w_s, z_s, a.S, a.C);
  for (int p = tid; p < SS; p += NT) {
    float z = (z_s[p] + bias) * a.inv_temp;
    if (legal && !legal[p]) z = -INFINITY;
    z_s[p] = z;
    if (z > lmax) {  // first max wins (p increases within a thread)
      lmax = z;
      lidx = p;
    }
  }
  // block argmax / max (ties -> smallest index)
  {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      float ov = __shfl_xor(lmax, o, 64);
      int oi = __shfl_xor(lidx, o, 64);
      if (ov > lmax || (ov == lmax && oi < lidx)) {
        lmax = ov;
        lidx = oi;
      }
    }
    if ((tid & 63) == 0) {
      red[tid >> 6] = lmax;
      redi[tid >> 6] = lidx;
    }
    __syncthreads();
    lmax = red[0];
    lidx = redi[0];
    for (int w = 1; w < NT / 64; ++w)
      if (red[w] > lmax || (red[w] == lmax && redi[w] < lidx)) {
        lmax = red[w];
        lidx = redi[w];
      }
  }
  const float zmax = lmax;
  float ls = 0.f;
  for (int p = tid; p < SS; p += NT) ls += (z_s[p] == -INFINITY) ? 0.f : __expf(z_s[p] - zmax);
  const float sum = block_reduce_sum(ls, red);
  const float inv = 1.f / sum;
  if (a.probs) {
    for (int p = tid; p < SS; p += NT)
      a.probs[(size_t)b * SS + p] = (z_s[p] == -INFINITY) ? 0.f : __expf(z_s[p] - zmax) * inv;
  }
  if constexpr (TRAIN) {
    const int t = a.target[b];
    const float wb = a.weight ? a.weight[b] : 1.f;
    if (a.loss_kind == 1) {
      policy_bce_train<NT, Board>(a, b, t, wb, zmax, inv, lidx, board, w_s, z_s, red);
      return;
    }
    if (tid == 0) {
      if (t >= 0) {
        float pt = __expf(z_s[t] - zmax) * inv;
        pt = fminf(fmaxf(pt, 1e-7f), 1.f - 1e-7f);  // Keras clip
        a.loss[b] = -__logf(pt);
        a.correct[b] = (lidx == t) ? 1.f : 0.f;
      } else {
        a.loss[b] = 0.f;
        a.correct[b] = 0.f;
      }
    }
    __syncthreads();  // everyone has read z_s[t]
    for (int p = tid; p < SS; p += NT) {
      float g = 0.f;
      if (t >= 0) g = (__expf(z_s[p] - zmax) * inv - (p == t ? 1.f : 0.f)) * a.grad_scale * wb;
      z_s[p] = g;
    }
    __syncthreads();
    board.backward(a, b, w_s, z_s);
    float gs = 0.f;
    for (int p = tid; p < SS; p += NT) gs += z_s[p];
    gs = block_reduce_sum(gs, red);
    if (tid == 0) a.dhead[(size_t)b * (a.C_real + 1) + a.C_real] = gs;
  }
}

// Head logits only: z[b][p] = y[b,p,:] . w + bias (value-net head input,
// value.py:23-26); the board's activations are read once.
template <int NT>
__global__ __launch_bounds__(NT) void head_logits_kernel(PolicyHeadArgs a) {
  __shared__ float w_s[256];
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int SS = a.S * a.S;
  const int HP = a.S + 2;
  for (int c = tid; c < a.C; c += NT) w_s[c] = c < a.C_real ? a.w[c] : 0.f;
  __syncthreads();
  __shared__ float z_s[368];
  const __bf16* base = a.y + (size_t)b * HP * HP * a.C;
  const float bias = a.b[0];
  head_dots(base, w_s, z_s, a.S, a.C);
  for (int p = tid; p < SS; p += NT) a.probs[(size_t)b * SS + p] = z_s[p] + bias;  // probs slot carries the logits
}

// Head backward from an externally computed dlogits (value net: dz = dh W1^T).
template <int NT>
__global__ __launch_bounds__(NT) void head_backward_kernel(PolicyHeadArgs a, const float* dlogits) {
  __shared__ float w_s[256];
  __shared__ float g_s[368];
  __shared__ float red[16];
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int SS = a.S * a.S;
  const int HP = a.S + 2;
  for (int c = tid; c < a.C; c += NT) w_s[c] = c < a.C_real ? a.w[c] : 0.f;
  float gs = 0.f;
  for (int p = tid; p < SS; p += NT) {
    const float g = dlogits[(size_t)b * SS + p];
    g_s[p] = g;
    gs += g;
  }
  __syncthreads();
  head_input_backward<NT>(a, b, a.y + (size_t)b * HP * HP * a.C, w_s, g_s);
  gs = block_reduce_sum(gs, red);
  if (tid == 0) a.dhead[(size_t)b * (a.C_real + 1) + a.C_real] = gs;
}

// Value output layer: v = tanh(h . w2 + b2) (value.py:28-29) and, with
// targets, MSE loss (v - t)^2, sign agreement, dv = 2 (v - t)(1 - v^2) * scale
// * weight[b], dh = dv w2 and per-board partials [dw2 | db2].  One workgroup
// per board, one thread per dense unit.
__global__ __launch_bounds__(256) void value_out_kernel(ValueOutArgs a) {
  __shared__ float red[8];
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  float s = 0.f;
  for (int j = tid; j < a.D; j += 256) s += a.h[(size_t)b * a.D + j] * a.w2[j];
  s = block_reduce_sum(s, red);
  const float v = tanhf(s + a.b2[0]);
  if (tid == 0) a.v[b] = v;
  if (!a.target) return;
  const float t = a.target[b];
  const float e = v - t;
  if (tid == 0) {
    a.loss[b] = e * e;
    a.correct[b] = (v > 0.f ? 1.f : (v < 0.f ? -1.f : 0.f)) == (t > 0.f ? 1.f : (t < 0.f ? -1.f : 0.f)) ? 1.f : 0.f;
  }
  const float dv = 2.f * e * (1.f - v * v) * a.grad_scale * (a.weight ? a.weight[b] : 1.f);
  float* dp = a.dout + (size_t)b * (a.D + 1);
  for (int j = tid; j < a.D; j += 256) {
    a.dh[(size_t)b * a.D + j] = dv * a.w2[j];
    dp[j] = dv * a.h[(size_t)b * a.D + j];
  }
  if (tid == 0) dp[a.D] = dv;
}

// Column sums of the per-board head partials (dhead [B][N]) into the flat gradient, plus the two
// per-board metric vectors (loss, correct) into sums[0..1]: one launch instead of three library
// reductions.  One workgroup per column; each thread sums rows tid, tid + 256, ... in order, then a
// fixed tree (deterministic).
__global__ __launch_bounds__(256) void head_grad_sums_kernel(const float* dhead, int B, int N, const float* loss,
                                                            const float* correct, float* grad, float* sums) {
  __shared__ float red[4];
  const int col = blockIdx.x;
  const float* src = col < N ? dhead + col : (col == N ? loss : correct);
  const int stride = col < N ? N : 1;
  float s = 0.f;
  for (int r = threadIdx.x; r < B; r += 256) s += src[(size_t)r * stride];
  s = block_reduce_sum(s, red);
  if (threadIdx.x == 0) {
    if (col < N) grad[col] = s;
    else sums[col - N] = s;
  }
}

void launch_head_grad_sums(const float* dhead, int B, int N, const float* loss, const float* correct, float* grad,
                           float* sums, hipStream_t st) {
  hipLaunchKernelGGL(head_grad_sums_kernel, dim3(N + 2), dim3(256), 0, st, dhead, B, N, loss, correct, grad, sums);
}

void launch_head_logits(const PolicyHeadArgs& a, hipStream_t st) {
  if (a.B < kHeadWideBelow) hipLaunchKernelGGL(head_logits_kernel<1024>, dim3(a.B), dim3(1024), 0, st, a);
  else hipLaunchKernelGGL(head_logits_kernel<256>, dim3(a.B), dim3(256), 0, st, a);
}
void launch_head_backward(const PolicyHeadArgs& a, const float* dlogits, hipStream_t st) {
  if (a.B < kHeadWideBelow) hipLaunchKernelGGL(head_backward_kernel<1024>, dim3(a.B), dim3(1024), 0, st, a, dlogits);
  else hipLaunchKernelGGL(head_backward_kernel<256>, dim3(a.B), dim3(256), 0, st, a, dlogits);
}
void launch_value_out(const ValueOutArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(value_out_kernel, dim3(a.B), dim3(256), 0, st, a);
}

template <bool TRAIN>
static void policy_head_go(const PolicyHeadArgs& a, hipStream_t st) {
  if (a.B >= kHeadWideBelow && a.S * (a.C >> 3) <= 512)
    hipLaunchKernelGGL((policy_head_kernel<TRAIN, 512, BoardRows<512>>), dim3(a.B), dim3(512), 0, st, a);
  else
    hipLaunchKernelGGL((policy_head_kernel<TRAIN, 1024, BoardRegs<1024>>), dim3(a.B), dim3(1024), 0, st, a);
}

void launch_policy_head(const PolicyHeadArgs& a, bool train, hipStream_t st) {
  if (train) policy_head_go<true>(a, st);
  else policy_head_go<false>(a, st);
}

}  // namespace agk
