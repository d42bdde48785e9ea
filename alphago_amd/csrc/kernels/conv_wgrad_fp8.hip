// fp8 weight gradient: dW_t[n][c] = sum_m dZ[m][n] * X[m + shift_t][c] on the block-scaled MFMA
// (v_mfma_scale_f32_16x16x128_f8f6f4, A = e5m2 gradients, B = e4m3 activations), VERDICT r2 item 4.
// Reference layer: the value net trunk, /root/reference/AlphaGo/models/value.py:14-25 (152 filters,
// padded to 160).
//
// The reduction runs over pixels, so both operands must reach the MFMA pixel-contiguous while they
// are stored channel-contiguous (NHWC).  Each 128-pixel K-step is staged global -> LDS with
// global_load_lds_dwordx4 as whole 160-byte pixel rows ([128 rows][160 B] per operand; a 1-KB piece
// covers 6.4 consecutive rows, ~8 cache lines -- round 3's first build staged 32-byte row pieces,
// 32 partial lines per piece, 171 vs 143 us per layer) and read back with the gfx950 8-bit transpose
// read ds_read_b64_tr_b8 (per 16-lane group: lane 2q+p supplies row q, bytes 8p..8p+7 of an 8-row x
// 16-byte block; lane i receives column i of the 8 rows -- pinned by
// tests/test_fp8_inference.py::test_tr8_transpose_read_mapping), with compile-time offsets from one
// base register per operand.  Four reads give a lane the 32 K-bytes of its 16x16x128 fragment.  The
// pixel order inside a step is permuted identically for both operands: K position k = 32 g + 8 j + q
// (g = lane group, j = read, q = row) lives in LDS row 32 j + 8 g + q, and each row's ten 16-byte
// chunks are rotated by (row >> 3) & 1, so the two lane groups of a 32-lane half (rows R and R + 8,
// which share banks at a 160-byte pitch) read disjoint banks.
//
// Scales: the MFMA's E8M0 block scales dequantise both operands (127 - e, from the device-resident
// delayed scales), so the fp32 partials go to the same per-split slab as the bf16 wgrad and the same
// deterministic conv_wgrad_reduce sums them.  Bias gradient: the tap-0 workgroups multiply their A
// fragments by an all-ones e4m3 operand (one more MFMA per fragment, dequantised by the same block
// scale); they also fold max |dZ| into the delayed-scale amax slots from the e5m2 magnitude bytes (a
// saturated e5m2 value reads 57344 / 2^eg, so a scale that overflows shrinks by the margin every step
// until it fits).
// Borders: pixels past the batch read padded-pixel 0 of dZ (always zero).
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>
#include <utility>

#include "common.h"
#include "conv_common.h"
#include "kernels.h"

namespace agk {

namespace {

typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(2))) unsigned u32x2;

// ds_read_b64_tr_b8 with a compile-time byte offset (the instruction's 16-bit offset field): one base
// VGPR serves every fragment of a step instead of one address register per (block, read)
template <int OFF>
__device__ __forceinline__ u32x2 ds_read_tr8_off(uint32_t base) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset field");
  u32x2 v;
  asm volatile("ds_read_b64_tr_b8 %0, %1 offset:%2" : "=v"(v) : "v"(base), "n"(OFF));
  return v;
}

template <int... I, typename F>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// e5m2 byte -> float (the byte is the high half of an IEEE half)
__device__ __forceinline__ float bf8_to_f32(unsigned byte) {
  return (float)__builtin_bit_cast(_Float16, (unsigned short)(byte << 8));
}

constexpr int kStepPx = 128;               // pixels per K-step (one 16x16x128 MFMA deep)
constexpr int kImgBytes = kStepPx * 160;  // one operand image of a step: 128 pixel rows x 160 B

// WN x WC tile of one tap per workgroup, 4 waves as 2 (n) x 2 (c); each lane stages the same rows
// of both operands, so one pixel decomposition serves a dz piece and an x piece.
// PROBE (kernel-lab timing probes, wrong values): bit 1 no MFMA, 2 no staging loads, 4 no LDS
// fragment reads, 8 no partial-tile stores
template <int WN, int WC, int PROBE = 0>
__global__ __launch_bounds__(256, 2) void conv_wgrad_fp8_kernel(ConvWgradFp8Args a) {
  static_assert(WN == 160 && WC == 160, "line staging: whole 160-channel pixel rows");
  constexpr int NBn = WN / 32;  // 16-blocks per wave (a wave covers WN/2 x WC/2)
  constexpr int NBc = WC / 32;
  constexpr int STAGE = 2 * kImgBytes;  // dz image, then x image
  static_assert(WN % 32 == 0 && WC % 32 == 0, "two waves per dimension, 32-channel blocks");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int lane = threadIdx.x & 63;
  const int wave = wave_id();
  const int wn = wave >> 1, wc = wave & 1;
  const int split = blockIdx.x;
  const int t = blockIdx.y;
  const int ncb = a.Cin / WC;
  const int n0 = (blockIdx.z / ncb) * WN;
  const int c0 = (blockIdx.z % ncb) * WC;
  const int kh = t / a.K, kw = t - (t / a.K) * a.K;
  const int toff = (kh * a.HPi + kw) * a.Cin + c0;
  const int SS = a.S * a.S;
  const int ks_begin = split * a.ksteps_per_split;
  int ks_end = ks_begin + a.ksteps_per_split;
  const int nks_total = (a.M + kStepPx - 1) / kStepPx;
  if (ks_end > nks_total) ks_end = nks_total;
  const int sa = *a.gscale, sb = *a.xscale;  // E8M0 exponents (dZ, X)

  constexpr int NPAIR = kStepPx * WC / 4096;  // 1-KB pieces per operand image per wave
  // Each lane's pixel of piece i advances by exactly 128 pixels per stage() call (consecutive steps),
  // so the (row, column) decomposition and both padded pixel indices are carried from step to step
  // with adds and selects: the per-step divisions and 32-bit multiplies of a fresh decomposition
  // (quarter-rate on CDNA: ~1300 of the SIMD's cycles per wave and step, more than the step's 25
  // MFMAs) are paid once here.  Past the batch: dz pixel 0 (a zero border) and x pixel 0.
  int spx[NPAIR], sii[NPAIR], sjx[NPAIR], spo[NPAIR], spi[NPAIR], sc16[NPAIR];
  const int DB = kStepPx / SS, DI = (kStepPx % SS) / a.S, DJ = kStepPx % a.S;
  const int stepo = (DB * a.HPo + DI) * a.HPo + DJ, stepi = (DB * a.HPi + DI) * a.HPi + DJ;
  const int wjo = a.HPo - a.S, wjo_i = (a.HPo - a.S) * a.HPo;
  const int wji = a.HPi - a.S, wji_i = (a.HPi - a.S) * a.HPi;
#pragma unroll
  for (int i = 0; i < NPAIR; ++i) {
    const int idx = (wave * NPAIR + i) * 64 + lane;  // 16-byte unit of the image
    const int R = idx / 10, pos = idx - R * 10;
    int c = pos - ((R >> 3) & 1);
    c = c < 0 ? c + 10 : c;  // source chunk (16 channels) of this LDS unit
    const int k = 32 * ((R >> 3) & 3) + 8 * (R >> 5) + (R & 7);
    const int px = ks_begin * kStepPx + k;
    const int b = fdiv(px, a.divSS);
    const int rem = px - b * SS;
    const int ii = fdiv(rem, a.divS);
    const int jx = rem - ii * a.S;
    spx[i] = px;
    sii[i] = ii;
    sjx[i] = jx;
    spo[i] = (b * a.HPo + ii + a.Po) * a.HPo + jx + a.Po;
    spi[i] = (b * a.HPi + ii + a.offi) * a.HPi + jx + a.offi;
    sc16[i] = c * 16;
  }
  auto stage = [&](int buf) {
    if constexpr ((PROBE & 2) != 0) return;
    char* base = smem + buf * STAGE;
    int dzo[NPAIR], xo[NPAIR];
#pragma unroll
    for (int i = 0; i < NPAIR; ++i) {
      const bool in = spx[i] < a.M;
      dzo[i] = (in ? (int)__umul24((unsigned)spo[i], (unsigned)a.Cout) : 0) + sc16[i];
      xo[i] = (in ? (int)__umul24((unsigned)spi[i], (unsigned)a.Cin) : 0) + toff + sc16[i];
      // advance to the next step's pixel
      spx[i] += kStepPx;
      int jx = sjx[i] + DJ;
      const bool w1 = jx >= a.S;
      jx = w1 ? jx - a.S : jx;
      int ii = sii[i] + DI + (w1 ? 1 : 0);
      const bool w2 = ii >= a.S;
      ii = w2 ? ii - a.S : ii;
      sjx[i] = jx;
      sii[i] = ii;
      spo[i] += stepo + (w1 ? wjo : 0) + (w2 ? wjo_i : 0);
      spi[i] += stepi + (w1 ? wji : 0) + (w2 ? wji_i : 0);
    }
#pragma unroll
    for (int i = 0; i < NPAIR; ++i) glds16(a.dz8 + dzo[i], base + (wave * NPAIR + i) * 1024);
#pragma unroll
    for (int i = 0; i < NPAIR; ++i) glds16(a.x8 + xo[i], base + kImgBytes + (wave * NPAIR + i) * 1024);
  };

  f32x4 acc[NBn][NBc];
#pragma unroll
  for (int i = 0; i < NBn; ++i)
#pragma unroll
    for (int j = 0; j < NBc; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // tap-0 workgroups (wc == 0 waves): the bias gradient as one more MFMA per A fragment against an
  // all-ones e4m3 operand (every column of the 16 x 16 result is the row sum, dequantised by the
  // block scale), and max |e5m2 dZ| as a packed 16-bit max of the magnitude bytes (e5m2 orders by
  // byte & 0x7f) -- 4 VALU per dword instead of a float conversion per byte (the conversions made
  // the tap-0 workgroups, and with one resident round the whole kernel, ~530 VALU per step longer)
  f32x4 accb[NBn];
#pragma unroll
  for (int i = 0; i < NBn; ++i) accb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  typedef __attribute__((ext_vector_type(2))) unsigned short u16x2;
  u16x2 mlo = {0, 0}, mhi = {0, 0};
  const bool do_bias = (t == 0) && (c0 == 0) && (wc == 0);
  const i32x8 ones = {0x38383838, 0x38383838, 0x38383838, 0x38383838, 0x38383838, 0x38383838, 0x38383838, 0x38383838};

  // transposed reads: lane (g = lane >> 4, li = lane & 15) reads row 32 j + lrow, byte 8 (li & 1) of
  // the rotated 16-byte chunk of its block
  const int g = lane >> 4, li = lane & 15;
  const int lrow = 8 * g + (li >> 1);

  if (ks_begin < ks_end) {
    stage(0);
    wait_vmcnt0();
    __syncthreads();
  }
  for (int ks = ks_begin; ks < ks_end; ++ks) {
    const int cur = (ks - ks_begin) & 1;
    if (ks + 1 < ks_end) stage(cur ^ 1);
    const char* base = smem + cur * STAGE;
    i32x8 af[NBn];
    {
      // lane base (row lrow, the rotated chunk of block 0 of the wave's range) + immediate offsets;
      // the range's last block (index 4 of 5) wraps to chunk 0 on rotated rows of the upper wave.
      // All A fragments are read first; the B fragments of block C + 1 are read under block C's
      // MFMAs (a 2-deep ring of 8 registers instead of all 40: the step otherwise spills).
      const uint32_t b0 = (uint32_t)(uintptr_t)AG_LDS(base) + lrow * 160 + 8 * (li & 1) + (g & 1) * 16;
      const uint32_t bn = b0 + wn * NBn * 16, bc = b0 + kImgBytes + wc * NBc * 16;
      const uint32_t bn4 = bn - ((wn == 1 && (g & 1)) ? 160 : 0), bc4 = bc - ((wc == 1 && (g & 1)) ? 160 : 0);
      u32x2 ra[NBn][4], rb[2][4];
      if constexpr ((PROBE & 4) != 0) {
        static_for<4>([&](auto J) {
          static_for<NBn>([&](auto I) { ra[I][J] = u32x2{bn + I * 7u + J, bn4 ^ (unsigned)ks}; });
          rb[0][J] = u32x2{bc + J, bc4 ^ (unsigned)ks};
          rb[1][J] = rb[0][J];
        });
      } else {
        static_for<4>([&](auto J) {
          static_for<NBn>([&](auto I) { ra[I][J] = ds_read_tr8_off<J * 32 * 160 + I * 16>(I == NBn - 1 ? bn4 : bn); });
        });
        static_for<4>([&](auto J) { rb[0][J] = ds_read_tr8_off<J * 32 * 160>(bc); });
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < NBn; ++i)
        af[i] = i32x8{(int)ra[i][0].x, (int)ra[i][0].y, (int)ra[i][1].x, (int)ra[i][1].y,
                      (int)ra[i][2].x, (int)ra[i][2].y, (int)ra[i][3].x, (int)ra[i][3].y};
      static_for<NBc>([&](auto C) {
        constexpr int cb = C & 1, nb = (C + 1) & 1;
        if constexpr (C + 1 < NBc && (PROBE & 4) == 0)
          static_for<4>([&](auto J) {
            rb[nb][J] = ds_read_tr8_off<J * 32 * 160 + (C + 1) * 16>(C + 1 == NBc - 1 ? bc4 : bc);
          });
        const i32x8 bm = i32x8{(int)rb[cb][0].x, (int)rb[cb][0].y, (int)rb[cb][1].x, (int)rb[cb][1].y,
                               (int)rb[cb][2].x, (int)rb[cb][2].y, (int)rb[cb][3].x, (int)rb[cb][3].y};
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < NBn; ++i) {
          if constexpr ((PROBE & 1) != 0) acc[i][C][0] += (float)(af[i][0] ^ bm[1]);
          else acc[i][C] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[i], bm, acc[i][C], 1, 0, 0, sa, 0, sb);
        }
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (C + 1 < NBc)
          asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(rb[nb][0]), "+v"(rb[nb][1]), "+v"(rb[nb][2]), "+v"(rb[nb][3]));
      });
    }
    // pin the step's MFMAs above the barrier: without a use here, hipcc sinks them (pure builtins)
    // past the barrier into the next iteration, keeping every fragment live across it (spills)
#pragma unroll
    for (int i = 0; i < NBn; ++i)
#pragma unroll
      for (int c = 0; c < NBc; ++c) asm volatile("" : "+v"(acc[i][c]));
    if (do_bias) {
#pragma unroll
      for (int i = 0; i < NBn; ++i) {
        accb[i] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[i], ones, accb[i], 1, 0, 0, sa, 0, 127);
#pragma unroll
        for (int d = 0; d < 8; ++d) {
          const unsigned w = (unsigned)af[i][d];
          mlo = __builtin_elementwise_max(mlo, __builtin_bit_cast(u16x2, w & 0x007f007fu));
          mhi = __builtin_elementwise_max(mhi, __builtin_bit_cast(u16x2, w & 0x7f007f00u));
        }
      }
    }
    wait_vmcnt0();
    __syncthreads();
  }

  // --- the split's partial tile: D[n][c], lane owns n..n+3 at column c
  const int nb0 = n0 + wn * (WN / 2) + ((lane >> 4) << 2);
  const int cbase = c0 + wc * (WC / 2) + (lane & 15);
  float* out = a.slab + ((size_t)split * a.T + t) * (size_t)a.Cout * a.Cin;
#pragma unroll
  for (int i = 0; i < NBn; ++i)
#pragma unroll
    for (int c = 0; c < NBc; ++c) {
      const int n = nb0 + i * 16;
      const int cc = cbase + c * 16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if constexpr ((PROBE & 8) != 0) {
          if (acc[i][c][r] == 12345.f) out[(size_t)(n + r) * a.Cin + cc] = 0.f;  // keeps the sums live
        } else {
          out[(size_t)(n + r) * a.Cin + cc] = acc[i][c][r];
        }
      }
    }
  if (do_bias) {
    // column 0 of the ones-product: lanes 0, 16, 32, 48 hold rows 4 (lane / 16) + r of block i
    if ((lane & 15) == 0) {
#pragma unroll
      for (int i = 0; i < NBn; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          a.dbias_slab[(size_t)split * a.Cout + n0 + wn * (WN / 2) + i * 16 + (lane >> 4) * 4 + r] = accb[i][r];
    }
    if (a.amax) {  // the delayed scale of the next step: max |dZ| = max |e5m2| / 2^eg
      const unsigned mb = max(max((unsigned)mlo.x, (unsigned)mlo.y), max((unsigned)mhi.x, (unsigned)mhi.y) >> 8);
      float vmax = bf8_to_f32(mb);
      vmax = wave_max(vmax) / *a.gmul;
      if (lane == 0 && vmax > 0.f) atomicMax(a.amax + (split & (kFp8AmaxSlots - 1)), __float_as_uint(vmax));
    }
  }
}

}  // namespace

int wgrad_fp8_supported(int Cout, int Cin, int K) { return Cout == 160 && Cin == 160 && K == 3 ? 1 : 0; }

template <int WN, int WC, int PROBE>
static void launch_wgrad_fp8_t(const ConvWgradFp8Args& a, hipStream_t st) {
  constexpr int smem = 2 * 2 * kImgBytes;  // two stages of two images
  static const hipError_t attr = hipFuncSetAttribute((const void*)conv_wgrad_fp8_kernel<WN, WC, PROBE>,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, smem);
  hip_check(attr, "hipFuncSetAttribute(max dynamic LDS)");
  dim3 grid(a.nsplit, a.T, (a.Cout / WN) * (a.Cin / WC));
  hipLaunchKernelGGL((conv_wgrad_fp8_kernel<WN, WC, PROBE>), grid, dim3(256), smem, st, a);
}

void launch_conv_wgrad_fp8(const ConvWgradFp8Args& a_in, hipStream_t st) {
  ConvWgradFp8Args a = a_in;
  a.divSS = make_fastdiv((uint32_t)(a.S * a.S));
  a.divS = make_fastdiv((uint32_t)a.S);
  if (!wgrad_fp8_supported(a.Cout, a.Cin, a.K))
    throw std::invalid_argument("conv_wgrad_fp8: 160 -> 160 3x3 layers only");
  constexpr int WN = 160, WC = 160;
#ifdef AGK_KERNEL_LAB
  switch (a.probe) {
    case 0: launch_wgrad_fp8_t<WN, WC, 0>(a, st); break;
#define AGK_WG8_PROBE(P) \
  case P: launch_wgrad_fp8_t<WN, WC, P>(a, st); break;
    AGK_WG8_PROBE(1) AGK_WG8_PROBE(2) AGK_WG8_PROBE(4) AGK_WG8_PROBE(8) AGK_WG8_PROBE(3) AGK_WG8_PROBE(5)
    AGK_WG8_PROBE(6) AGK_WG8_PROBE(7) AGK_WG8_PROBE(14) AGK_WG8_PROBE(15)
#undef AGK_WG8_PROBE
    default: throw std::invalid_argument("conv_wgrad_fp8: probe " + std::to_string(a.probe));
  }
#else
  if (a.probe != 0) throw std::invalid_argument("conv_wgrad_fp8: timing probes are kernel-lab code");
  launch_wgrad_fp8_t<WN, WC, 0>(a, st);
#endif
}

int wgrad_fp8_stage_pixels() { return kStepPx; }

}  // namespace agk
