// Shared pieces of the implicit-GEMM conv kernels (conv.hip: production
// kernels and dispatch; conv_fwd_variants.hip: the forward kernel lab).
#pragma once
#include <hip/hip_runtime.h>

#include "common.h"
#include "kernels.h"

namespace agk {

// Debug build (AGK_DEBUG): device bounds checks.  AGK_DCHECK(cond, code)
// evaluates to cond; when it is false the code is OR-ed into a per-module error
// word (a vector atomic) and the caller skips / redirects the access, so a bad
// offset is reported (debug_error_fetch_and_clear -> Python RuntimeError)
// instead of touching memory outside the tensor.  Release builds: always true.
#ifdef AGK_DEBUG
static __device__ unsigned g_dbg_err;
#define AGK_DCHECK(cond, code) \
  ((cond) ? true : (atomicOr(&::agk::g_dbg_err, (unsigned)(code)), false))
#else
#define AGK_DCHECK(cond, code) true
#endif
enum : unsigned {
  DBG_FWD_X = 1u << 0,   // conv_fwd: activation (pixel operand) staging offset
  DBG_FWD_W = 1u << 1,   // conv_fwd: weight staging offset
  DBG_FWD_Y = 1u << 2,   // conv_fwd: epilogue store offset
  DBG_WG_X = 1u << 3,    // conv_wgrad: activation staging offset
  DBG_WG_DZ = 1u << 4,   // conv_wgrad: gradient staging offset
};

template <int N>
__device__ __forceinline__ void vmcnt_wait() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if constexpr (N == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
  else if constexpr (N == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (N == 7) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else static_assert(N < 0, "unsupported vmcnt");
}

// s_waitcnt vmcnt(N) for any immediate N (gfx950: 0..63)
template <int N>
__device__ __forceinline__ void vmcnt_n() {
  static_assert(N >= 0 && N <= 63, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// LDS-ring wait: at most `later` stages of PW DMA instructions each may still be outstanding
// (later = 0 .. MAXL, wave-uniform); the exact count, not a clamped one, so the ring keeps its depth
template <int PW, int MAXL>
__device__ __forceinline__ void ring_wait(int later) {
  static_assert(MAXL >= 0 && MAXL <= 3 && PW * MAXL <= 63, "ring depth");
  if (MAXL >= 3 && later >= 3) vmcnt_n<PW * (MAXL >= 3 ? 3 : 0)>();
  else if (MAXL >= 2 && later >= 2) vmcnt_n<PW * (MAXL >= 2 ? 2 : 0)>();
  else if (MAXL >= 1 && later >= 1) vmcnt_n<PW * (MAXL >= 1 ? 1 : 0)>();
  else vmcnt_n<0>();
}

__device__ __forceinline__ void vmcnt_wait_dyn(int n) {
  switch (n) {
    case 0: vmcnt_wait<0>(); break;
    case 1: vmcnt_wait<1>(); break;
    case 2: vmcnt_wait<2>(); break;
    case 3: vmcnt_wait<3>(); break;
    case 4: vmcnt_wait<4>(); break;
    case 5: vmcnt_wait<5>(); break;
    case 6: vmcnt_wait<6>(); break;
    case 7: vmcnt_wait<7>(); break;
    default: vmcnt_wait<8>(); break;
  }
}

// ---- wgrad helpers (conv.hip, conv_wgrad_row.hip)
// s_waitcnt lgkmcnt(CNT) tying one read pair: issued for each pair of a group whose reads are all
// older than the CNT most recent ones (the first wait blocks, the rest are already satisfied)
template <int CNT>
__device__ __forceinline__ void lgkm_wait_pair(bf16x4& a, bf16x4& b) {
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(a), "+v"(b) : "n"(CNT));
}

// s_waitcnt lgkmcnt(0) with every listed read result as an in/out operand:
// nothing that uses them can be scheduled above the wait.
template <int N>
__device__ __forceinline__ void lgkm_fence(bf16x4 (&a)[N], bf16x4 (&b)[N]) {
  static_assert(N >= 1 && N <= 15, "lgkm_fence supports 1..15 pairs (30 asm operands)");
  if constexpr (N == 15)
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a[0]), "+v"(b[0]), "+v"(a[1]), "+v"(b[1]), "+v"(a[2]), "+v"(b[2]), "+v"(a[3]), "+v"(b[3]), "+v"(a[4]), "+v"(b[4]), "+v"(a[5]), "+v"(b[5]), "+v"(a[6]), "+v"(b[6]), "+v"(a[7]), "+v"(b[7]), "+v"(a[8]), "+v"(b[8]), "+v"(a[9]), "+v"(b[9]), "+v"(a[10]), "+v"(b[10]), "+v"(a[11]), "+v"(b[11]), "+v"(a[12]), "+v"(b[12]), "+v"(a[13]), "+v"(b[13]), "+v"(a[14]), "+v"(b[14]));
  else if constexpr (N == 14)
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a[0]), "+v"(b[0]), "+v"(a[1]), "+v"(b[1]), "+v"(a[2]), "+v"(b[2]), "+v"(a[3]), "+v"(b[3]), "+v"(a[4]), "+v"(b[4]), "+v"(a[5]), "+v"(b[5]), "+v"(a[6]), "+v"(b[6]), "+v"(a[7]), "+v"(b[7]), "+v"(a[8]), "+v"(b[8]), "+v"(a[9]), "+v"(b[9]), "+v"(a[10]), "+v"(b[10]), "+v"(a[11]), "+v"(b[11]), "+v"(a[12]), "+v"(b[12]), "+v"(a[13]), "+v"(b[13]));
  else if constexpr (N == 13)
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a[0]), "+v"(b[0]), "+v"(a[1]), "+v"(b[1]), "+v"(a[2]), "+v"(b[2]), "+v"(a[3]), "+v"(b[3]), "+v"(a[4]), "+v"(b[4]), "+v"(a[5]), "+v"(b[5]), "+v"(a[6]), "+v"(b[6]), "+v"(a[7]), "+v"(b[7]), "+v"(a[8]), "+v"(b[8]), "+v"(a[9]), "+v"(b[9]), "+v"(a[10]), "+v"(b[10]), "+v"(a[11]), "+v"(b[11]), "+v"(a[12]), "+v"(b[12]));
  else if constexpr (N == 12)
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a[0]), "+v"(b[0]), "+v"(a[1]), "+v"(b[1]), "+v"(a[2]), "+v"(b[2]), "+v"(a[3]), "+v"(b[3]), "+v"(a[4]), "+v"(b[4]), "+v"(a[5]), "+v"(b[5]), "+v"(a[6]), "+v"(b[6]), "+v"(a[7]), "+v"(b[7]), "+v"(a[8]), "+v"(b[8]), "+v"(a[9]), "+v"(b[9]), "+v"(a[10]), "+v"(b[10]), "+v"(a[11]), "+v"(b[11]));
  else if constexpr (N == 11)
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a[0]), "+v"(b[0]), "+v"(a[1]), "+v"(b[1]), "+v"(a[2]), "+v"(b[2]), "+v"(a[3]), "+v"(b[3]), "+v"(a[4]), "+v"(b[4]), "+v"(a[5]), "+v"(b[5]), "+v"(a[6]), "+v"(b[6]), "+v"(a[7]), "+v"(b[7]), "+v"(a[8]), "+v"(b[8]), "+v"(a[9]), "+v"(b[9]), "+v"(a[10]), "+v"(b[10]));
  else if constexpr (N == 10)
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a[0]), "+v"(b[0]), "+v"(a[1]), "+v"(b[1]), "+v"(a[2]), "+v"(b[2]), "+v"(a[3]), "+v"(b[3]), "+v"(a[4]), "+v"(b[4]), "+v"(a[5]), "+v"(b[5]), "+v"(a[6]), "+v"(b[6]), "+v"(a[7]), "+v"(b[7]), "+v"(a[8]), "+v"(b[8]), "+v"(a[9]), "+v"(b[9]));
  else if constexpr (N == 9)
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a[0]), "+v"(b[0]), "+v"(a[1]), "+v"(b[1]), "+v"(a[2]), "+v"(b[2]), "+v"(a[3]), "+v"(b[3]), "+v"(a[4]), "+v"(b[4]), "+v"(a[5]), "+v"(b[5]), "+v"(a[6]), "+v"(b[6]), "+v"(a[7]), "+v"(b[7]), "+v"(a[8]), "+v"(b[8]));
  else if constexpr (N == 8)
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a[0]), "+v"(b[0]), "+v"(a[1]), "+v"(b[1]), "+v"(a[2]), "+v"(b[2]), "+v"(a[3]), "+v"(b[3]), "+v"(a[4]), "+v"(b[4]), "+v"(a[5]), "+v"(b[5]), "+v"(a[6]), "+v"(b[6]), "+v"(a[7]), "+v"(b[7]));
  else if constexpr (N == 7)
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a[0]), "+v"(b[0]), "+v"(a[1]), "+v"(b[1]), "+v"(a[2]), "+v"(b[2]), "+v"(a[3]), "+v"(b[3]), "+v"(a[4]), "+v"(b[4]), "+v"(a[5]), "+v"(b[5]), "+v"(a[6]), "+v"(b[6]));
  else if constexpr (N == 6)
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a[0]), "+v"(b[0]), "+v"(a[1]), "+v"(b[1]), "+v"(a[2]), "+v"(b[2]), "+v"(a[3]), "+v"(b[3]), "+v"(a[4]), "+v"(b[4]), "+v"(a[5]), "+v"(b[5]));
  else if constexpr (N == 5)
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a[0]), "+v"(b[0]), "+v"(a[1]), "+v"(b[1]), "+v"(a[2]), "+v"(b[2]), "+v"(a[3]), "+v"(b[3]), "+v"(a[4]), "+v"(b[4]));
  else if constexpr (N == 4)
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a[0]), "+v"(b[0]), "+v"(a[1]), "+v"(b[1]), "+v"(a[2]), "+v"(b[2]), "+v"(a[3]), "+v"(b[3]));
  else if constexpr (N == 3)
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a[0]), "+v"(b[0]), "+v"(a[1]), "+v"(b[1]), "+v"(a[2]), "+v"(b[2]));
  else if constexpr (N == 2)
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a[0]), "+v"(b[0]), "+v"(a[1]), "+v"(b[1]));
  else if constexpr (N == 1)
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a[0]), "+v"(b[0]));
}

// ds_read_b64_tr_b16 through inline asm.  The builtin form makes hipcc wait
// vmcnt(0) before every such read while any LDS-DMA is outstanding (it cannot
// tell the read from the DMA target), which would drain the ring; the caller
// waits lgkmcnt itself (lgkm_fence below) before touching the results.
__device__ __forceinline__ bf16x4 ds_read_tr16_asm(const char* p) {
  bf16x4 v;
  const uint32_t off = (uint32_t)(uintptr_t)(AG_LDS(p));
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(off));
  return v;
}


// Shared epilogue of the forward/dgrad kernels: lane owns output channels
// nbase + 16 i + [0, 4) of pixel mrow + 16 j.  load() issues every operand
// load (bias, or the ReLU' mask of dgrad) with clamped pixel indices — no
// per-element branches, so the loads overlap instead of forming 24
// load -> wait -> store round trips; the kernels call it a few K-steps before
// the end of the main loop so the mask read hides under the last MFMAs.
template <int NB, int MB, int MODE>
struct ConvEpilogue {
  int ooff[MB];
  int pix[MB];
  f32x4 bb[NB];
  bf16x4 mk[NB][MB];
  uint32_t mw[MB];
  int mslot, mwords;

  // ReLU' bitmask layout: per padded pixel, (Cout/BN)*8 32-bit words; word
  // (blockIdx.y*8 + wn*4 + lane/16) holds bit 4i+r for channel nbase+16i+r —
  // exactly the channels one lane owns, so producer and consumer never
  // exchange data (12x less traffic than re-reading the bf16 activation).
  __device__ __forceinline__ void load(const ConvFwdArgs& a, int mrow, int nbase, int wn = 0) {
    const int SS = a.S * a.S;
    mslot = blockIdx.y * 8 + wn * 4 + ((threadIdx.x & 63) >> 4);
    mwords = gridDim.y * 8;
#pragma unroll
    for (int j = 0; j < MB; ++j) {
      int m = mrow + j * 16;
      m = m < a.M ? m : a.M - 1;
      const int b = fdiv(m, a.divSS);
      const int rem = m - b * SS;
      const int ii = fdiv(rem, a.divS);
      const int jj = rem - ii * a.S;
      pix[j] = (b * a.HPo + ii + a.Po) * a.HPo + jj + a.Po;
      ooff[j] = pix[j] * a.Cout + nbase;
    }
    if constexpr (MODE == MODE_BIAS_RELU) {
#pragma unroll
      for (int i = 0; i < NB; ++i) bb[i] = *(const f32x4*)(a.bias + nbase + i * 16);
    } else if constexpr (MODE == MODE_MASK) {
#pragma unroll
      for (int j = 0; j < MB; ++j)
#pragma unroll
        for (int i = 0; i < NB; ++i) mk[i][j] = *(const bf16x4*)(a.mask + ooff[j] + i * 16);
    } else if constexpr (MODE == MODE_MASKBITS) {
#pragma unroll
      for (int j = 0; j < MB; ++j) mw[j] = a.mbits_in[(size_t)pix[j] * mwords + mslot];
    }
  }

  __device__ __forceinline__ void store(const ConvFwdArgs& a, const f32x4 (&acc)[NB][MB], int mrow) const {
    float gmax = 0.f;  // MODE_MASKBITS with an e5m2 copy: max |dx| of the lane
    const float gsc = (MODE == MODE_MASKBITS && a.y_bf8) ? *a.bf8_scale : 0.f;
#pragma unroll
    for (int j = 0; j < MB; ++j) {
      if (mrow + j * 16 >= a.M) continue;
      uint32_t bits = 0u;
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        f32x4 v = acc[i][j];
        if constexpr (MODE == MODE_BIAS_RELU) {
          v[0] = fmaxf(v[0] + bb[i][0], 0.f);
          v[1] = fmaxf(v[1] + bb[i][1], 0.f);
          v[2] = fmaxf(v[2] + bb[i][2], 0.f);
          v[3] = fmaxf(v[3] + bb[i][3], 0.f);
        } else if constexpr (MODE == MODE_MASK) {
          v[0] = (float)mk[i][j][0] > 0.f ? v[0] : 0.f;
          v[1] = (float)mk[i][j][1] > 0.f ? v[1] : 0.f;
          v[2] = (float)mk[i][j][2] > 0.f ? v[2] : 0.f;
          v[3] = (float)mk[i][j][3] > 0.f ? v[3] : 0.f;
        } else if constexpr (MODE == MODE_MASKBITS) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = ((mw[j] >> (4 * i + r)) & 1u) ? v[r] : 0.f;
        }
        bf16x4 o;
        o[0] = (__bf16)v[0];
        o[1] = (__bf16)v[1];
        o[2] = (__bf16)v[2];
        o[3] = (__bf16)v[3];
        if constexpr (MODE == MODE_BIAS_RELU) {
          // the bit records what the bf16 value the dgrad would re-read says: y > 0
#pragma unroll
          for (int r = 0; r < 4; ++r) bits |= ((float)o[r] > 0.f ? 1u : 0u) << (4 * i + r);
        }
#ifdef AGK_DEBUG
        const long long yo = (long long)ooff[j] + i * 16;
        if (AGK_DCHECK(yo >= 0 && yo + 4 <= a.y_elems, DBG_FWD_Y)) *(bf16x4*)(a.y + yo) = o;
#else
        *(bf16x4*)(a.y + ooff[j] + i * 16) = o;
#endif
        if constexpr (MODE == MODE_MASKBITS) {
          if (a.y_bf8) {  // wave-uniform
            float sv[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              gmax = fmaxf(gmax, fabsf(v[r]));
              sv[r] = fminf(fmaxf(v[r] * gsc, -57344.f), 57344.f);
            }
            int pk = __builtin_amdgcn_cvt_pk_bf8_f32(sv[0], sv[1], 0, false);
            pk = __builtin_amdgcn_cvt_pk_bf8_f32(sv[2], sv[3], pk, true);
            *(int*)(a.y_bf8 + ooff[j] + i * 16) = pk;
          }
        }
      }
      if constexpr (MODE == MODE_BIAS_RELU)
        if (a.mbits_out) a.mbits_out[(size_t)pix[j] * mwords + mslot] = bits;
    }
    if constexpr (MODE == MODE_MASKBITS) {
      if (a.y_bf8 && a.bf8_amax) {
        gmax = wave_max(gmax);
        if ((threadIdx.x & 63) == 0 && gmax > 0.f) atomicMax(a.bf8_amax + (blockIdx.x & 63), __float_as_uint(gmax));
      }
    }
  }
};

template <int NB, int MB, int MODE>
__device__ __forceinline__ void conv_store_tile(const ConvFwdArgs& a, const f32x4 (&acc)[NB][MB], int mrow,
                                                int nbase, int wn) {
  ConvEpilogue<NB, MB, MODE> ep;
  ep.load(a, mrow, nbase, wn);
  ep.store(a, acc, mrow);
}

// ---------------- epilogue for the 32x32x16 MFMA layout (weights as A, pixels as B)
// acc[i][j] (f32x16) of a wave: output channel nbase + 32 i + 8 g + 4 h + r
// (h = lane >> 5, reg = 4 g + r) of pixel mrow + 32 j, mrow = the lane's pixel
// of block 0.  ReLU' bitmask: per padded pixel (Cout/BN)*8 words; the lane's
// 16*NB bits (bit 16 i + 4 g + r) sit in words blockIdx.y*8 + wn*4 + 2h + {0, 1}.
template <int NB, int MB, int MODE>
struct ConvEpilogue32 {
  int ooff[MB];
  int pix[MB];
  f32x4 bb[NB][4];
  bf16x4 mk[NB][MB][4];
  uint2 mw[MB];
  int mslot, mwords;

  __device__ __forceinline__ void load(const ConvFwdArgs& a, int mrow, int nbase, int wn) {
    const int SS = a.S * a.S;
    const int h = (threadIdx.x & 63) >> 5;
    mslot = blockIdx.y * 8 + wn * 4 + 2 * h;
    mwords = gridDim.y * 8;
#pragma unroll
    for (int j = 0; j < MB; ++j) {
      int m = mrow + j * 32;
      m = m < a.M ? m : a.M - 1;
      const int b = fdiv(m, a.divSS);
      const int rem = m - b * SS;
      const int ii = fdiv(rem, a.divS);
      const int jj = rem - ii * a.S;
      pix[j] = (b * a.HPo + ii + a.Po) * a.HPo + jj + a.Po;
      ooff[j] = pix[j] * a.Cout + nbase + 4 * h;
    }
    if constexpr (MODE == MODE_BIAS_RELU) {
#pragma unroll
      for (int i = 0; i < NB; ++i)
#pragma unroll
        for (int g = 0; g < 4; ++g) bb[i][g] = *(const f32x4*)(a.bias + nbase + 4 * h + i * 32 + g * 8);
    } else if constexpr (MODE == MODE_MASK) {
#pragma unroll
      for (int j = 0; j < MB; ++j)
#pragma unroll
        for (int i = 0; i < NB; ++i)
#pragma unroll
          for (int g = 0; g < 4; ++g) mk[i][j][g] = *(const bf16x4*)(a.mask + ooff[j] + i * 32 + g * 8);
    } else if constexpr (MODE == MODE_MASKBITS) {
#pragma unroll
      for (int j = 0; j < MB; ++j) mw[j] = *(const uint2*)(a.mbits_in + (size_t)pix[j] * mwords + mslot);
    }
  }

  __device__ __forceinline__ void store(const ConvFwdArgs& a, const f32x16 (&acc)[NB][MB], int mrow) const {
#pragma unroll
    for (int j = 0; j < MB; ++j) {
      if (mrow + j * 32 >= a.M) continue;
      uint32_t bits[2] = {0u, 0u};
#pragma unroll
      for (int i = 0; i < NB; ++i)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = acc[i][j][4 * g + r];
          const int bit0 = 16 * i + 4 * g;
          if constexpr (MODE == MODE_BIAS_RELU) {
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r] + bb[i][g][r], 0.f);
          } else if constexpr (MODE == MODE_MASK) {
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = (float)mk[i][j][g][r] > 0.f ? v[r] : 0.f;
          } else if constexpr (MODE == MODE_MASKBITS) {
            const uint32_t w = bit0 < 32 ? mw[j].x : mw[j].y;
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = ((w >> ((bit0 & 31) + r)) & 1u) ? v[r] : 0.f;
          }
          bf16x4 o;
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = (__bf16)v[r];
          if constexpr (MODE == MODE_BIAS_RELU) {
#pragma unroll
            for (int r = 0; r < 4; ++r) bits[bit0 >> 5] |= ((float)o[r] > 0.f ? 1u : 0u) << ((bit0 & 31) + r);
          }
          *(bf16x4*)(a.y + ooff[j] + i * 32 + g * 8) = o;
        }
      if constexpr (MODE == MODE_BIAS_RELU)
        if (a.mbits_out) *(uint2*)(a.mbits_out + (size_t)pix[j] * mwords + mslot) = make_uint2(bits[0], bits[1]);
    }
  }
};


// forward variants in conv_fwd_variants.hip (tile codes -1, 2, 4, 5, 6, 32);
// returns false when the variant does not apply to the geometry
bool launch_conv_fwd_variant(int code, const ConvFwdArgs& a, int mode, hipStream_t st);

}  // namespace agk
