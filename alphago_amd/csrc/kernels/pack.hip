// Data-movement kernels around the conv trunk:
//  * pack_input: uint8 feature planes [B][C][S][S] -> zero-bordered NHWC bf16
//    with a per-board D4 symmetry applied on the fly (the reference does the
//    8-way augmentation on the CPU per sample with numpy, supervised_policy_
//    trainer.py:27-36,71-80) and the move targets transformed consistently.
//  * pack_weights: fp32 OIHW master weights -> bf16 [tap][Cout][Cin] (forward)
//    and the tap-flipped, transposed [tap][Cin][Cout] copy used by dgrad, for
//    every layer in one launch.
//  * sgd: p -= lr * scale * g over the flat fp32 parameter buffer (Keras SGD,
//    momentum 0; the 1/world_size all-reduce average is folded into `scale`).
#include <hip/hip_runtime.h>

#include "common.h"
#include "kernels.h"

namespace agk {

// Symmetry s maps board point (x, y) to (x', y'); numpy semantics of the
// reference BOARD_TRANSFORMATIONS on a [x][y] array.
__device__ __forceinline__ void sym_fwd(int s, int n, int x, int y, int& ox, int& oy) {
  switch (s) {
    case 1: ox = n - 1 - y; oy = x; break;          // rot90
    case 2: ox = n - 1 - x; oy = n - 1 - y; break;  // rot180
    case 3: ox = y; oy = n - 1 - x; break;          // rot270
    case 4: ox = x; oy = n - 1 - y; break;          // fliplr
    case 5: ox = n - 1 - x; oy = y; break;          // flipud
    case 6: ox = y; oy = x; break;                  // transpose
    case 7: ox = n - 1 - y; oy = n - 1 - x; break;  // fliplr(rot90)
    default: ox = x; oy = y; break;
  }
}
__device__ __forceinline__ void sym_inv(int s, int n, int i, int j, int& x, int& y) {
  switch (s) {
    case 1: x = j; y = n - 1 - i; break;
    case 3: x = n - 1 - j; y = i; break;
    default: sym_fwd(s, n, i, j, x, y); break;  // the others are involutions
  }
}

// boards up to this many plane bytes take pack_input_board_kernel (64 planes of 19 x 19 = 23 KB)
constexpr int kPackBoardMaxBytes = 48 * 1024;

__global__ void pack_input_kernel(PackInputArgs a) {
  const int SS = a.S * a.S;
  const int C8 = a.Cp >> 3;
  const int HP = a.S + 2 * a.P;
  const int total = a.B * SS * C8;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += gridDim.x * blockDim.x) {
    const int c8 = idx % C8;
    const int rest = idx / C8;
    const int p = rest % SS;
    const int b = rest / SS;
    const int i = p / a.S, j = p - (p / a.S) * a.S;
    const int s = a.sym ? a.sym[b] : 0;
    int x, y;
    sym_inv(s, a.S, i, j, x, y);
    const int64_t row = a.rows ? a.rows[b] : b;
    const bool valid = row >= 0 && row < a.npool;
    const uint8_t* src = a.planes + (size_t)(valid ? row : 0) * a.Creal * SS + x * a.S + y;
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = c8 * 8 + e;
      o[e] = (__bf16)(c < a.Creal && valid ? (float)src[(size_t)c * SS] : 0.f);
    }
    *(bf16x8*)(a.out + ((size_t)(b * HP + i + a.P) * HP + j + a.P) * a.Cp + c8 * 8) = o;
    if (a.target_out && p == 0 && c8 == 0) {
      const int t = a.target[b];
      int r = -1;
      if (t >= 0) {
        int ox, oy;
        sym_fwd(s, a.S, t / a.S, t % a.S, ox, oy);
        r = ox * a.S + oy;
      }
      a.target_out[b] = r;
    }
  }
}

// One workgroup per board (pool row rows[b] when given: the minibatch gather fused into the pack):
// the board's Creal x S x S bytes come in with coalesced 4-byte loads into
// LDS, then lane (p, c8) gathers its 8 planes at the symmetry's source point from LDS and writes 16
// contiguous bytes of the padded NHWC row (consecutive lanes: consecutive 16-byte chunks).
// pack_input_kernel's per-lane strided byte loads from HBM ran at ~3 TB/s (57 us at B = 2176).
__global__ __launch_bounds__(256) void pack_input_board_kernel(PackInputArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t pl_s[];
  const int b = blockIdx.x;
  const int SS = a.S * a.S;
  const int n = a.Creal * SS;
  const int64_t row = a.rows ? a.rows[b] : b;
  const bool valid = row >= 0 && row < a.npool;
  const uint8_t* src = a.planes + (size_t)(valid ? row : 0) * n;
  if (!valid) {
    for (int i = threadIdx.x; i < n; i += 256) pl_s[i] = 0;
  } else if ((n & 3) == 0) {  // the board's bytes start 4-byte aligned: n is a multiple of 4
    const uint32_t* s4 = (const uint32_t*)src;
    for (int i = threadIdx.x; i < (n >> 2); i += 256) ((uint32_t*)pl_s)[i] = s4[i];
  } else {
    for (int i = threadIdx.x; i < n; i += 256) pl_s[i] = src[i];
  }
  __syncthreads();
  const int C8 = a.Cp >> 3;
  const int HP = a.S + 2 * a.P;
  const int s = a.sym ? a.sym[b] : 0;
  __bf16* ob = a.out + (size_t)b * HP * HP * a.Cp;
  uint8_t* ob8 = a.out8 ? a.out8 + (size_t)b * HP * HP * a.Cp : nullptr;
  for (int idx = threadIdx.x; idx < SS * C8; idx += 256) {
    const int c8 = idx % C8;
    const int p = idx / C8;
    const int i = p / a.S, j = p - i * a.S;
    int x, y;
    sym_inv(s, a.S, i, j, x, y);
    const uint8_t* q = pl_s + x * a.S + y;
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = c8 * 8 + e;
      o[e] = (__bf16)(c < a.Creal ? (float)q[c * SS] : 0.f);
    }
    const size_t off = ((size_t)(i + a.P) * HP + j + a.P) * a.Cp + c8 * 8;
    *(bf16x8*)(ob + off) = o;
    if (ob8) {  // quantize_fp8_kernel's conversion at scale 1 (the fp8 trunk's input; no second pass)
      float f[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = fminf(fmaxf((float)o[e], -448.f), 448.f);
      int lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], 0, false);
      lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], lo, true);
      int hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[4], f[5], 0, false);
      hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[6], f[7], hi, true);
      *(int2*)(ob8 + off) = make_int2(lo, hi);
    }
  }
  if (a.target_out && threadIdx.x == 0) {
    const int t = a.target[b];
    int r = -1;
    if (t >= 0) {
      int ox, oy;
      sym_fwd(s, a.S, t / a.S, t % a.S, ox, oy);
      r = ox * a.S + oy;
    }
    a.target_out[b] = r;
  }
}

void launch_pack_input(const PackInputArgs& a, hipStream_t st) {
  const int bytes = a.Creal * a.S * a.S;
  if (a.out8 && bytes > kPackBoardMaxBytes)
    throw std::invalid_argument("pack_input: the e4m3 output needs boards of at most 48 KB of planes");
  if (bytes <= kPackBoardMaxBytes) {
    hipLaunchKernelGGL(pack_input_board_kernel, dim3(a.B), dim3(256), bytes, st, a);
    return;
  }
  const int total = a.B * a.S * a.S * (a.Cp / 8);
  int blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(pack_input_kernel, dim3(blocks), dim3(256), 0, st, a);
}

__global__ void pack_weights_kernel(PackWeightsArgs a) {
  const PackLayer L = a.layers[blockIdx.y];
  const int T = L.K * L.K;
  if (L.pk_cpt > 0) {  // packed-tap first layer: [step][Cout_p][64], chunk j of step s = q = 8 s + j
    const int nst = (T * L.pk_cpt + 7) >> 3;
    const int tot = nst * L.Cout_p * 64;
    for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < tot; idx += gridDim.x * blockDim.x) {
      const int k = idx & 63;
      const int rest = idx >> 6;
      const int n = rest % L.Cout_p;
      const int q = (rest / L.Cout_p) * 8 + (k >> 3);
      const int t = q / L.pk_cpt;
      const int c = (q - t * L.pk_cpt) * 8 + (k & 7);
      float v = 0.f;
      if (t < T && n < L.Cout_real && c < L.Cin_real) v = L.w[((size_t)n * L.Cin_real + c) * T + t];
      L.wf[idx] = (__bf16)v;
    }
    return;
  }
  const int total = T * L.Cout_p * L.Cin_p;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += gridDim.x * blockDim.x) {
    const int c = idx % L.Cin_p;
    const int rest = idx / L.Cin_p;
    const int n = rest % L.Cout_p;
    const int t = rest / L.Cout_p;
    float v = 0.f;
    if (n < L.Cout_real && c < L.Cin_real) v = L.w[((size_t)n * L.Cin_real + c) * T + t];
    const __bf16 bv = (__bf16)v;
    L.wf[idx] = bv;
    if (L.wd) {
      const int kh = t / L.K, kw = t - (t / L.K) * L.K;
      const int tf = (L.K - 1 - kh) * L.K + (L.K - 1 - kw);
      L.wd[((size_t)tf * L.Cin_p + c) * L.Cout_p + n] = bv;
    }
  }
}

void launch_pack_weights(const PackWeightsArgs& a, hipStream_t st) {
  if (a.nlayers <= 0) return;
  int maxtot = 0;
  for (int i = 0; i < a.nlayers; ++i) {
    const PackLayer& L = a.layers[i];
    const int tot = L.pk_cpt > 0 ? ((L.K * L.K * L.pk_cpt + 7) / 8) * L.Cout_p * 64 : L.K * L.K * L.Cout_p * L.Cin_p;
    if (tot > maxtot) maxtot = tot;
  }
  int blocks = (maxtot + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(pack_weights_kernel, dim3(blocks, a.nlayers), dim3(256), 0, st, a);
}

__global__ void sgd_kernel(float* __restrict__ p, const float* __restrict__ g, int64_t n, float step) {
  const int64_t n4 = n >> 2;
  float4* p4 = (float4*)p;
  const float4* g4 = (const float4*)g;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    float4 pv = p4[i];
    const float4 gv = g4[i];
    pv.x -= step * gv.x;
    pv.y -= step * gv.y;
    pv.z -= step * gv.z;
    pv.w -= step * gv.w;
    p4[i] = pv;
  }
  for (int64_t i = (n4 << 2) + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] -= step * g[i];
}

// Keras-SGD schedule kept on the device so a whole training step can be
// captured in a HIP graph: sched = {lr0, decay, iterations, lr_current} (f64).
// One thread computes lr = lr0 / (1 + decay * iterations) -- the same double
// expression as KerasSGDSchedule.current() -- and advances the counter.
// An 8-entry schedule {lr0, decay, iterations, lr, beta_1, beta_2, opt, 0} adds Keras 1.0 Adam's
// bias correction lr_t = lr sqrt(1 - beta_2^t) / (1 - beta_1^t), t = iterations + 1, when opt == 2.
__global__ void sgd_sched_kernel(double* sched, int n) {
  if (threadIdx.x == 0) {
    double lr = sched[0] / (1.0 + sched[1] * sched[2]);
    if (n >= 8 && sched[6] == 2.0) {
      const double t = sched[2] + 1.0;
      lr = lr * sqrt(1.0 - pow(sched[5], t)) / (1.0 - pow(sched[4], t));
    }
    sched[3] = lr;
    sched[2] = sched[2] + 1.0;
  }
}

__global__ void sgd_dev_kernel(float* __restrict__ p, const float* __restrict__ g, int64_t n,
                               const double* __restrict__ sched, float gscale) {
  const float step = (float)sched[3] * gscale;  // == launch_sgd's (float)lr * gscale
  const int64_t n4 = n >> 2;
  float4* p4 = (float4*)p;
  const float4* g4 = (const float4*)g;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    float4 pv = p4[i];
    const float4 gv = g4[i];
    pv.x -= step * gv.x;
    pv.y -= step * gv.y;
    pv.z -= step * gv.z;
    pv.w -= step * gv.w;
    p4[i] = pv;
  }
  for (int64_t i = (n4 << 2) + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] -= step * g[i];
}

void launch_sgd_sched(float* p, const float* g, int64_t n, double* sched, float gscale, hipStream_t st) {
  hipLaunchKernelGGL(sgd_sched_kernel, dim3(1), dim3(64), 0, st, sched, 4);
  int64_t blocks = ((n >> 2) + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(sgd_dev_kernel, dim3((unsigned)blocks), dim3(256), 0, st, p, g, n, (const double*)sched, gscale);
}

__global__ void invalid_config_probe_kernel(int* p) {
  if (p) p[threadIdx.x] = 0;
}

void launch_invalid_config_probe(hipStream_t st) {
  // 2048 threads per block exceeds the 1024 limit: the runtime refuses the
  // launch (hipErrorInvalidConfiguration); nothing executes on the device
  hipLaunchKernelGGL(invalid_config_probe_kernel, dim3(1), dim3(2048), 0, st, nullptr);
}

void launch_sgd(float* p, const float* g, int64_t n, float lr, float gscale, hipStream_t st) {
  int64_t blocks = ((n >> 2) + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(sgd_kernel, dim3((unsigned)blocks), dim3(256), 0, st, p, g, n, lr * gscale);
}


// ----------------------------------------------------------------- fused SGD + bf16 weight packs
// One launch per step for the whole update (round 4; was sgd_kernel over the flat buffer, then
// pack_weights_kernel, whose strided OIHW reads and transposed writes took ~25 us at every batch
// size).  Job y < nlayers: a 32 (c) x 32 (n) tile of conv layer y -- each thread updates the K*K
// taps of one (n, c) (contiguous in OIHW), writes the forward pack wf[t][n][c] (or the first layer's
// packed-tap layout) directly and stages the transposed dgrad pack through LDS so that wd[t'][c][n]
// is written along n.  Job y == nlayers: plain SGD over the remaining ranges (biases, head).
namespace {
__device__ __forceinline__ size_t wf_index(const SgdPackLayer& L, int t, int n, int c) {
  if (L.pk_cpt > 0) {  // packed-tap first layer (conv_fwd_pk_kernel)
    const int q = t * L.pk_cpt + (c >> 3);
    return ((size_t)(q >> 3) * L.Cout_p + n) * 64 + (q & 7) * 8 + (c & 7);
  }
  return ((size_t)t * L.Cout_p + n) * L.Cin_p + c;
}
}  // namespace

// Phase 1 reads the tile's OIHW span along memory (for each of the 32 n, its 32 c x K*K taps are
// contiguous), 18-20 independent loads in flight per thread, and stages the bf16 result in LDS as
// [t][c][n]; phase 2 writes wf along c and wd along n from LDS.  (The round-4 first cut had each thread
// walk its (n, c)'s taps serially: strided, one load in flight, 79 us per step.)
// One parameter's update under the optimizer OPT (SgdPackArgs::opt); i = its flat index.  OPT 0 is the
// round-4 expression (p - step g, step = lr * gscale), so plain SGD stays bitwise unchanged.
template <int OPT>
__device__ __forceinline__ float opt_update(const SgdPackArgs& a, size_t i, float p, float g, float step, float m1v,
                                            float m2v) {
  if constexpr (OPT == 0) {
    return p - step * g;
  } else if constexpr (OPT == 1) {
    const float v = a.mom * m1v - step * g;
    a.m1[i] = v;
    return a.nesterov ? p + a.mom * v - step * g : p + v;
  } else {
    const float ge = g * a.gscale;
    const float m = a.b1 * m1v + (1.f - a.b1) * ge;
    const float v = a.b2 * m2v + (1.f - a.b2) * ge * ge;
    a.m1[i] = m;
    a.m2[i] = v;
    return p - step * m / (sqrtf(v) + a.eps);
  }
}

template <int K, int OPT>
__device__ __forceinline__ void sgd_pack_layer(const SgdPackArgs& a, const SgdPackLayer& L, float* P, const float* G,
                                               float step, __bf16* tile) {
  constexpr int KK = K;
  constexpr int T = KK * KK;
  constexpr int span = 32 * T;  // one n's slice of the tile, in floats
  const int ctiles = (L.Cin_p + 31) >> 5;
  const int c0 = (blockIdx.x % ctiles) * 32, n0 = (blockIdx.x / ctiles) * 32;
  const int cw = min(32, L.Cin_real - c0), nw = min(32, L.Cout_real - n0);
  const int lim = cw * T;  // real floats of one n's slice
  const size_t rows = (size_t)L.Cin_real * T;
  const size_t base0 = ((size_t)n0 * L.Cin_real + c0) * T;
  constexpr int B = K == 1 ? 4 : K == 3 ? 18 : 20;  // loads in flight: 2 rounds (3x3), 5 (5x5)
#pragma unroll 1
  for (int e0 = 0; e0 < 32 * span; e0 += 256 * B) {
    float pv[B], gv[B], m1v[OPT ? B : 1], m2v[OPT == 2 ? B : 1];
#pragma unroll
    for (int j = 0; j < B; ++j) {
      const int e = e0 + j * 256 + (int)threadIdx.x;
      const int nl = e / span, r = e - nl * span;
      pv[j] = gv[j] = 0.f;
      if constexpr (OPT != 0) m1v[j] = 0.f;
      if constexpr (OPT == 2) m2v[j] = 0.f;
      if (e < 32 * span && nl < nw && r < lim) {
        pv[j] = P[base0 + nl * rows + r];
        gv[j] = G[base0 + nl * rows + r];
        if constexpr (OPT != 0) m1v[j] = a.m1[L.off + base0 + nl * rows + r];
        if constexpr (OPT == 2) m2v[j] = a.m2[L.off + base0 + nl * rows + r];
      }
    }
#pragma unroll
    for (int j = 0; j < B; ++j) {
      const int e = e0 + j * 256 + (int)threadIdx.x;
      if (e >= 32 * span) break;
      const int nl = e / span, r = e - nl * span;
      const int cl = r / T, t = r - cl * T;
      float v = 0.f;
      if (nl < nw && r < lim) {
        v = opt_update<OPT>(a, L.off + base0 + nl * rows + r, pv[j], gv[j], step, m1v[OPT ? j : 0],
                            m2v[OPT == 2 ? j : 0]);
        P[base0 + nl * rows + r] = v;
      }
      tile[(t * 32 + cl) * 33 + nl] = (__bf16)v;
    }
  }
  __syncthreads();
  // forward pack wf[t][n][c] (or the packed-tap layout): along c.  Packed-tap layout: channels past the
  // last chunk of a tap have no slot (their index would alias the next tap's first chunk).
  const int cslots = L.pk_cpt > 0 ? L.pk_cpt * 8 : L.Cin_p;
  {
    const int cl = threadIdx.x & 31, c = c0 + cl;
#pragma unroll 4
    for (int row = threadIdx.x >> 5; row < T * 32; row += 8) {
      const int t = row >> 5, nl = row & 31, n = n0 + nl;
      if (n < L.Cout_p && c < cslots) L.wf[wf_index(L, t, n, c)] = tile[(t * 32 + cl) * 33 + nl];
    }
  }
  if (!L.wd) return;
  // dgrad pack wd[t'][c][n] (t' = the 180-degree-rotated tap): along n
  const int nl = threadIdx.x & 31, n = n0 + nl;
#pragma unroll 4
  for (int row = threadIdx.x >> 5; row < T * 32; row += 8) {
    const int t = row >> 5, cc = row & 31;
    const int kh = t / KK, kw = t - kh * KK;
    const int tf = (KK - 1 - kh) * KK + (KK - 1 - kw);
    if (c0 + cc < L.Cin_p && n < L.Cout_p)
      L.wd[((size_t)tf * L.Cin_p + c0 + cc) * L.Cout_p + n] = tile[(t * 32 + cc) * 33 + nl];
  }
}

template <int OPT>
__device__ __forceinline__ void sgd_pack_job(const SgdPackArgs& a, __bf16* tile) {
  // SGD: step = lr * gscale (the sgd_dev_kernel step); momentum / Adam: step = lr (Adam: lr_t), and
  // Adam scales the gradient itself (its step is invariant to a gradient scale only up to eps)
  float step = OPT == 2 ? a.lr : a.lr * a.gscale;
  if (a.sched) step = OPT == 2 ? (float)a.sched[3] : (float)a.sched[3] * a.gscale;
  if ((int)blockIdx.y == a.nlayers) {  // plain ranges
    for (int r = 0; r < a.nranges; ++r) {
      const int64_t o = a.range_off[r];
      float* p = a.p + o;
      const float* g = a.g + o;
      for (int i = blockIdx.x * 256 + threadIdx.x; i < a.range_len[r]; i += gridDim.x * 256) {
        if constexpr (OPT == 0) {
          p[i] -= step * g[i];
        } else {
          const float m2v = OPT == 2 ? a.m2[o + i] : 0.f;
          p[i] = opt_update<OPT>(a, o + i, p[i], g[i], step, a.m1[o + i], m2v);
        }
      }
    }
    return;
  }
  const SgdPackLayer& L = a.layers[blockIdx.y];
  const int ctiles = (L.Cin_p + 31) >> 5;
  const int ntiles = (L.Cout_p + 31) >> 5;
  if ((int)blockIdx.x >= ctiles * ntiles) return;  // block-uniform: before any barrier
  float* P = a.p + L.off;
  const float* G = a.g + L.off;
  switch (L.K) {  // layer-uniform
    case 1: sgd_pack_layer<1, OPT>(a, L, P, G, step, tile); break;
    case 3: sgd_pack_layer<3, OPT>(a, L, P, G, step, tile); break;
    case 5: sgd_pack_layer<5, OPT>(a, L, P, G, step, tile); break;
    default: break;  // rejected on the host (kSgdPackMaxTaps)
  }
}

// one kernel per optimizer: the Adam body's extra moment registers must not lower the SGD kernel's
// occupancy (one kernel with a runtime switch took 56 us per step instead of 35, round 5)
template <int OPT>
__global__ __launch_bounds__(256) void sgd_pack_kernel(SgdPackArgs a) {
  __shared__ __bf16 tile[kSgdPackMaxTaps * 32 * 33];  // [t][c][n] (n padded to 33: no bank conflicts)
  sgd_pack_job<OPT>(a, tile);
}

void launch_sgd_pack(const SgdPackArgs& a, hipStream_t st) {
  if (a.sched) hipLaunchKernelGGL(sgd_sched_kernel, dim3(1), dim3(64), 0, st, a.sched, a.opt == 2 ? 8 : 4);
  int tiles = 1;
  for (int i = 0; i < a.nlayers; ++i) {
    const SgdPackLayer& L = a.layers[i];
    const int t = ((L.Cin_p + 31) / 32) * ((L.Cout_p + 31) / 32);
    if (t > tiles) tiles = t;
  }
  if (tiles < 64) tiles = 64;  // the plain-range job's blocks
  if (a.opt == 1) hipLaunchKernelGGL(sgd_pack_kernel<1>, dim3(tiles, a.nlayers + 1), dim3(256), 0, st, a);
  else if (a.opt == 2) hipLaunchKernelGGL(sgd_pack_kernel<2>, dim3(tiles, a.nlayers + 1), dim3(256), 0, st, a);
  else hipLaunchKernelGGL(sgd_pack_kernel<0>, dim3(tiles, a.nlayers + 1), dim3(256), 0, st, a);
}

}  // namespace agk
