// FP8 (OCP e4m3) implicit-GEMM convolution on the gfx950 block-scaled MFMA
// v_mfma_scale_f32_16x16x128_f8f6f4 — twice the bf16 MFMA rate (BASELINE
// config "fp8 MFMA conv path").
//
// Same gather structure as conv_fwd_kernel (conv.hip), re-cut for 1-byte
// operands:
//   * activations: zero-bordered NHWC e4m3, channels padded to 64 (one 64-B
//     "chunk" per pixel per 64 channels); weights packed [chunk q][Cout][64 B]
//     with q = tap * (Cin/64) + c, the chunk count padded to even with zeros;
//   * a K-step is TWO chunks (K = 128, possibly two different taps): each
//     128-B LDS row is assembled from two 64-B source rows by the per-lane
//     source addresses of global_load_lds_dwordx4;
//   * 16-B chunks of a row are XOR-swizzled by fp8_swz(row) (conflict-free
//     for the two ds_read_b128 of a lane's 32-byte fragment);
//   * per-tensor power-of-two scales are passed as the MFMA's E8M0 block
//     scales (read from device memory, so a captured graph picks up new
//     scales), the epilogue adds bias, applies ReLU, tracks the output amax
//     (atomicMax, delayed scaling) and writes bf16 and/or e4m3 outputs.
#include <hip/hip_runtime.h>

#include "common.h"
#include "kernels.h"

namespace agk {

// e4m3 pack of four ReLU outputs (already scaled and clamped to 448): round to nearest even, or with
// sr (training forward, ConvFp8Args::sr_seed) stochastic rounding with per-element random bits from a
// hash of (output element index, seed) -- unbiased activations for the fp8 training step
__device__ __forceinline__ uint32_t fp8_sr_bits(uint32_t idx, uint32_t seed) {
  uint32_t h = idx * 0x9E3779B1u ^ (seed + 0x7F4A7C15u) * 0x85EBCA77u;
  h ^= h >> 16;
  h *= 0x7FEB352Du;
  h ^= h >> 15;
  h *= 0x846CA68Bu;
  h ^= h >> 16;
  return h;
}
__device__ __forceinline__ int fp8_pack4(float s0, float s1, float s2, float s3, bool sr, uint32_t idx,
                                         uint32_t seed) {
  if (sr) {
    int pk = __builtin_amdgcn_cvt_sr_fp8_f32(s0, (int)fp8_sr_bits(idx, seed), 0, 0);
    pk = __builtin_amdgcn_cvt_sr_fp8_f32(s1, (int)fp8_sr_bits(idx + 1, seed), pk, 1);
    pk = __builtin_amdgcn_cvt_sr_fp8_f32(s2, (int)fp8_sr_bits(idx + 2, seed), pk, 2);
    return __builtin_amdgcn_cvt_sr_fp8_f32(s3, (int)fp8_sr_bits(idx + 3, seed), pk, 3);
  }
  int pk = __builtin_amdgcn_cvt_pk_fp8_f32(s0, s1, 0, false);
  return __builtin_amdgcn_cvt_pk_fp8_f32(s2, s3, pk, true);
}


typedef __attribute__((ext_vector_type(8))) int i32x8;

__device__ __forceinline__ int fp8_swz(int row) { return ((row >> 1) & 1) | (((row >> 3) & 1) << 2); }

__device__ __forceinline__ f32x4 mfma_fp8(const i32x8& a, const i32x8& b, const f32x4& c, int sa, int sb) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, sa, 0, sb);
}
// A e4m3 (weights), B e5m2 (gradients): the dgrad operand formats
__device__ __forceinline__ f32x4 mfma_fp8_bf8(const i32x8& a, const i32x8& b, const f32x4& c, int sa, int sb) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 1, 0, sa, 0, sb);
}

template <int BN, bool OUT_BF16, bool OUT_FP8>
__global__ __launch_bounds__(512, 1) void conv_fwd_fp8_kernel(ConvFp8Args a) {
  constexpr int BM = 256;
  constexpr int NB = BN / 32;  // 16-wide n blocks per wave (wave covers BN/2)
  constexpr int MB = 4;        // 16-wide m blocks per wave (64 pixels)
  constexpr int A_BYTES = BM * 128;
  constexpr int B_BYTES = BN * 128;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int B_INSTR = BN / 64;  // 1-KB weight pieces per wave
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int lane = threadIdx.x & 63;
  const int wave = wave_id();
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int SS = a.S * a.S;
  const int CC = (a.Cin + 63) >> 6;  // Cin 160: the third chunk's upper half is the next pixel (zero weights)
  const int nK = a.nch >> 1;
  const int qmax = a.K * a.K * CC - 1;  // last real chunk (padding chunks re-read it; their weights are 0)
  const int sx = a.scales[0], sw = a.scales[1];

  // A staging: 4 pieces per wave; lane -> row 8i + lane/8 of the wave's 32 rows,
  // physical 16-B chunk lane%8 -> logical chunk (which half = which K chunk)
  int abase[4], alc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = wave * 32 + i * 8 + (lane >> 3);
    int m = m0 + r;
    m = m < a.M ? m : a.M - 1;
    const int b = fdiv(m, a.divSS);
    const int rem = m - b * SS;
    const int ii = fdiv(rem, a.divS);
    const int jj = rem - ii * a.S;
    alc[i] = (lane & 7) ^ fp8_swz(r);
    abase[i] = ((b * a.HPi + ii + a.offi) * a.HPi + jj + a.offi) * a.Cin + (alc[i] & 3) * 16;
  }
  int bbase[B_INSTR], blc[B_INSTR];
#pragma unroll
  for (int i = 0; i < B_INSTR; ++i) {
    const int r = wave * (BN / 8) + i * 8 + (lane >> 3);
    blc[i] = (lane & 7) ^ fp8_swz(r);
    bbase[i] = (n0 + r) * 64 + (blc[i] & 3) * 16;
  }

  auto chunk_off = [&](int q) {  // activation offset of chunk q (tap shift + channel block)
    q = q < qmax ? q : qmax;
    const int t = q / CC;
    const int c = q - t * CC;
    const int kh = t / a.K;
    const int kw = t - kh * a.K;
    return (kh * a.HPi + kw) * a.Cin + c * 64;
  };
  auto stage = [&](int ks, int buf) {
    const int q0 = 2 * ks;
    const int off0 = chunk_off(q0), off1 = chunk_off(q0 + 1);
    char* base = smem + buf * STAGE;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      glds16(a.x + abase[i] + ((alc[i] >> 2) ? off1 : off0), base + (wave * 32 + i * 8) * 128);
    const size_t w0 = (size_t)q0 * a.Cout * 64;
    const size_t w1 = w0 + (size_t)a.Cout * 64;
#pragma unroll
    for (int i = 0; i < B_INSTR; ++i)
      glds16(a.w + bbase[i] + ((blc[i] >> 2) ? w1 : w0), base + A_BYTES + (wave * (BN / 8) + i * 8) * 128);
  };

  f32x4 acc[NB][MB];
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int j = 0; j < MB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment: row (lane & 15) of a 16-row block, logical chunks 2g, 2g+1 (g = lane >> 4)
  const int r15 = lane & 15;
  const int g = lane >> 4;
  const int c0 = ((2 * g) ^ fp8_swz(r15)) << 4;
  const int c1 = ((2 * g + 1) ^ fp8_swz(r15)) << 4;
  const int xrow = (wm * 64 + r15) * 128;
  const int wrow = A_BYTES + (wn * (BN / 2) + r15) * 128;
  auto frag = [&](const char* p) {
    const int4 lo = *(const int4*)(p + c0);
    const int4 hi = *(const int4*)(p + c1);
    return i32x8{lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  };

  stage(0, 0);
  wait_vmcnt0();
  __syncthreads();
  for (int ks = 0; ks < nK; ++ks) {
    const int cur = ks & 1;
    const char* base = smem + cur * STAGE;
    if (ks + 1 < nK) stage(ks + 1, cur ^ 1);
    i32x8 xf[MB], wf[NB];
#pragma unroll
    for (int j = 0; j < MB; ++j) xf[j] = frag(base + xrow + j * 16 * 128);
#pragma unroll
    for (int i = 0; i < NB; ++i) wf[i] = frag(base + wrow + i * 16 * 128);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < NB; ++i)
#pragma unroll
      for (int j = 0; j < MB; ++j) acc[i][j] = mfma_fp8(wf[i], xf[j], acc[i][j], sw, sx);
    __builtin_amdgcn_s_setprio(0);
    wait_vmcnt0();
    __syncthreads();
  }

  // --- epilogue: bias + ReLU, amax, bf16 and/or e4m3 stores (lane: 4 channels of one pixel per block)
  const int nbase = n0 + wn * (BN / 2) + ((lane >> 4) << 2);
  f32x4 bb[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) bb[i] = *(const f32x4*)(a.bias + nbase + i * 16);
  const float osc = a.out_scale[0];
  float vmax = 0.f;
#pragma unroll
  for (int j = 0; j < MB; ++j) {
    int m = m0 + wm * 64 + j * 16 + (lane & 15);
    const bool ok = m < a.M;
    m = ok ? m : a.M - 1;
    const int b = fdiv(m, a.divSS);
    const int rem = m - b * SS;
    const int ii = fdiv(rem, a.divS);
    const int jj = rem - ii * a.S;
    const size_t ooff = (size_t)((b * a.HPo + ii + a.Po) * a.HPo + jj + a.Po) * a.Cout;
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      f32x4 v = acc[i][j];
      v[0] = fmaxf(v[0] + bb[i][0], 0.f);
      v[1] = fmaxf(v[1] + bb[i][1], 0.f);
      v[2] = fmaxf(v[2] + bb[i][2], 0.f);
      v[3] = fmaxf(v[3] + bb[i][3], 0.f);
      if (ok) vmax = fmaxf(vmax, fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3])));
      const int n = nbase + i * 16;
      if (!ok) continue;
      if constexpr (OUT_BF16) {
        bf16x4 o;
        o[0] = (__bf16)v[0];
        o[1] = (__bf16)v[1];
        o[2] = (__bf16)v[2];
        o[3] = (__bf16)v[3];
        *(bf16x4*)(a.y_bf16 + ooff + n) = o;
      }
      if constexpr (OUT_FP8) {
        const float s0 = fminf(v[0] * osc, 448.f), s1 = fminf(v[1] * osc, 448.f);
        const float s2 = fminf(v[2] * osc, 448.f), s3 = fminf(v[3] * osc, 448.f);
        const bool sr = a.sr_seed != nullptr;  // uniform
        *(int*)(a.y_fp8 + ooff + n) = fp8_pack4(s0, s1, s2, s3, sr, (uint32_t)(ooff + n), sr ? (uint32_t)*a.sr_seed : 0u);
      }
    }
  }
  if (a.amax) {
    // workgroup max, then one atomic per workgroup into one of kFp8AmaxSlots
    // slots (a single address would serialise ~10k atomics per layer)
    vmax = wave_max(vmax);
    __syncthreads();  // LDS stages are dead; reuse the first bytes
    float* red = reinterpret_cast<float*>(smem);
    if (lane == 0) red[wave] = vmax;
    __syncthreads();
    if (threadIdx.x == 0) {
      float m = red[0];
#pragma unroll
      for (int w = 1; w < 8; ++w) m = fmaxf(m, red[w]);
      atomicMax(a.amax + (blockIdx.x & (kFp8AmaxSlots - 1)), __float_as_uint(m));
    }
  }
}

// ------------------------------------------ pixel operand straight from L2
// PMC on conv_fwd_fp8_kernel (profiles/r1_conv_pmc_fp8.md): the matrix pipe
// is busy 27 % of the time and waves wait on the stage DMA -- each 128-B LDS
// row is assembled from two 64-B activation rows, and a 24-MFMA step is too
// short to cover 56 KB of LDS-DMA.  Here each wave loads its own pixel
// fragments (32 B per lane: half of one 64-B chunk) with buffer loads into
// registers, one step ahead, and only the weights (24 KB per step for BN 192)
// go through LDS, by VGPR + ds_write so the compiler's vmcnt bookkeeping stays
// exact.  Waves own disjoint pixels (8 x 32 = 256 per workgroup) and all BN
// channels.
// DG: dgrad (e5m2 gradient operand, ReLU' mask from a.mask, no bias, max |dx|, e5m2 output)
// DGB: dgrad whose gradient operand is the bf16 dZ itself: each lane loads its 32 bf16 values
// (64 B) per K-step and converts them to e5m2 in registers (v_cvt_scalef32_pk_bf8_bf16, two per
// instruction, multiplier *a.in_scale) -- no quantisation pass, no e5m2 tensor; ReLU' mask from
// the forward's bitmask; bf16 output and max |dx| only
typedef __attribute__((ext_vector_type(2))) short s16x2_t;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
__device__ __forceinline__ int cvt4_bf16_bf8(unsigned lo2, unsigned hi2, float s) {
  // two packed bf16 pairs -> four e5m2 bytes (low pair in bytes 0-1); the instruction DIVIDES by
  // its scale operand (e5m2(x / s), measured by tests/test_fp8_inference.py::
  // test_scalef32_bf8_conversion_semantics), so callers pass the reciprocal of the multiplier
  s16x2_t r = __builtin_amdgcn_cvt_scalef32_pk_bf8_bf16((s16x2_t){0, 0}, __builtin_bit_cast(bf16x2_t, lo2), s, false);
  r = __builtin_amdgcn_cvt_scalef32_pk_bf8_bf16(r, __builtin_bit_cast(bf16x2_t, hi2), s, true);
  return __builtin_bit_cast(int, r);
}

// DGBITS (with DG): the e5m2 gradient operand is the copy the previous dgrad wrote for the fp8 wgrad,
// ReLU' comes from the forward's bitmask (as DGB), outputs e5m2 (for the fp8 wgrad and the next
// fp8 dgrad) and bf16 only where a bf16 consumer exists (the first layer's wgrad)
// CW: bytes of one packed weight chunk = channels per K-chunk.  64 (default): a 128-K step is two
// 64-channel chunks.  32 (the 160-channel value width, round 4): a step is four 32-channel chunks
// and every MFMA K-block is one (tap, 32 channels) pair, so 160 channels are 5 chunks per tap instead
// of 3 x 64 with a 32-channel zero half -- 45 chunks (12 steps) per 3x3 layer instead of 14 steps.
// LDS of conv_fwd_fp8_ga_kernel: two weight slots (BN rows rounded up to whole 512-thread pieces),
// or with the staged epilogue 8 waves x 16*MB pixels x (BN + 16) bytes if larger, then the amax
// reduction's 8 floats
constexpr int fp8_ga_wrows(int BN, int NT) { return (BN * 8) % NT == 0 ? BN : ((BN * 8 + NT - 1) / NT * NT) / 8; }
constexpr int fp8_ga_red_off(int BN, int MB, bool stg, int NW) {
  return stg && NW * 16 * MB * (BN + 16) > 2 * fp8_ga_wrows(BN, 64 * NW) * 128
             ? NW * 16 * MB * (BN + 16)
             : 2 * fp8_ga_wrows(BN, 64 * NW) * 128;
}

template <int BN, int MB, int NPART, bool OUT_BF16, bool OUT_FP8, bool DG = false, bool DGB = false,
          bool DGBITS = false, int CW = 64, int NW = 8, bool STGE = false, int PROBE = 0>
__global__ __launch_bounds__(64 * NW, 8 / NW) void conv_fwd_fp8_ga_kernel(ConvFp8Args a) {
  // PROBE (kernel-lab timing probes, wrong values): bit 1 no MFMA, 2 no pixel loads, 4 no weight
  // staging (load + ds_write), 8 no LDS fragment reads, 16 no epilogue stores;
  // NW: waves per workgroup -- 8 (one workgroup per CU) or 4 (two per CU: one workgroup's
  // prologue, barriers and epilogue overlap the other's MFMA steps).  STGE: byte outputs staged
  // through LDS and stored as 16-B row segments (instead of one 4-B store per lane and block)
  static_assert(NW == 8 || NW == 4, "waves per workgroup");
  constexpr bool STG = STGE && OUT_FP8;
  static_assert(CW == 64 || CW == 32, "chunk width");
  constexpr int CPS = 128 / CW;  // chunks per K-step
  static_assert(!(DG && DGB), "one dgrad form");
  static_assert(!DGBITS || DG, "DGBITS: the e5m2-operand dgrad");
  constexpr bool MASKBITS = DGB || DGBITS;  // ReLU' from the forward epilogue's bitmask
  // MB: 16-pixel blocks per wave; the BN/16 channel blocks are read from LDS in NPART parts
  constexpr int NB = BN / 16;   // 16-channel blocks per wave
  constexpr int NH = NB / NPART;
  static_assert(NB % NPART == 0, "channel blocks must split evenly into parts");
  constexpr int NT = 64 * NW;
  constexpr int BM = NW * 16 * MB;
  // weight slot rows: BN rounded up so that every thread stages the same number
  // of 16-B pieces (BN 160 -> 192 rows; rows >= BN hold copies, never read)
  constexpr int WROWS = fp8_ga_wrows(BN, NT);
  constexpr int W_BYTES = WROWS * 128;
  constexpr int WP = W_BYTES / 16 / NT;  // 16-B weight pieces per thread and step
  constexpr int SROW = BN + 16;           // STG: LDS bytes per staged pixel (16-B aligned, skewed banks)
  constexpr int RED_OFF = fp8_ga_red_off(BN, MB, STG, NW);
  typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int lane = threadIdx.x & 63;
  const int wave = wave_id();
  const int nwg = gridDim.x;
  const int xcd = blockIdx.x & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (blockIdx.x >> 3);
  const int m0 = tile * BM;
  const int n0 = blockIdx.y * BN;
  const int SS = a.S * a.S;
  // CW 64, Cin 160: the third chunk's upper half is the next pixel (zero weights)
  const int CC = (a.Cin + CW - 1) / CW;
  const int nK = a.nch / CPS;
  const int qmax = a.K * a.K * CC - 1;
  const int sx = a.scales[0], sw = a.scales[1];

  const int nimg = a.M / SS;
  constexpr int XB = DGB ? 2 : 1;  // bytes per operand element in memory
  const long long xbytes = (long long)nimg * a.HPi * a.HPi * a.Cin * XB;
  const long long wbytes = (long long)a.nch * a.Cout * 64;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.x, (short)0, (int)(xbytes < 0x7fffffffLL ? xbytes : 0x7fffffffLL), 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.w, (short)0, (int)(wbytes < 0x7fffffffLL ? wbytes : 0x7fffffffLL), 0x00020000);

  // B operand (pixels): lane -> pixel (block j, lane&15), K bytes [32g, 32g+32), g = lane>>4:
  // g < 2 from chunk q0 of the step, g >= 2 from chunk q1
  const int g = lane >> 4;
  int xbase[MB];
#pragma unroll
  for (int j = 0; j < MB; ++j) {
    int m = m0 + wave * 16 * MB + j * 16 + (lane & 15);
    m = m < a.M ? m : a.M - 1;
    const int b = fdiv(m, a.divSS);
    const int rem = m - b * SS;
    const int ii = fdiv(rem, a.divS);
    const int jj = rem - ii * a.S;
    xbase[j] = ((b * a.HPi + ii + a.offi) * a.HPi + jj + a.offi) * a.Cin + (CW == 64 ? (g & 1) * 32 : 0);
  }
  // A operand (weights) staging: piece p = tid + NT i -> LDS row p/8, physical 16-B chunk p%8
  int wsrc[WP], wdst[WP];
#pragma unroll
  for (int i = 0; i < WP; ++i) {
    const int p = threadIdx.x + NT * i;
    const int r = p >> 3, pc = p & 7;
    const int lc = pc ^ fp8_swz(r);
    // logical 16-B chunk lc of the 128-B row: chunk lc / (CW / 16) of the step, bytes (lc % (CW / 16)) * 16
    wsrc[i] = (((lc / (CW / 16)) * a.Cout) + n0 + (r < BN ? r : BN - 1)) * CW + (lc % (CW / 16)) * 16;
    wdst[i] = r * 128 + pc * 16;
  }
  auto chunk_off = [&](int q) {  // wave-uniform; divisions by the launcher's exact fast divisors
    q = q < qmax ? q : qmax;
    const int t = (int)fdiv((uint32_t)q, a.divCC);
    const int c = q - t * CC;
    const int kh = (int)fdiv((uint32_t)t, a.divK);
    const int kw = t - kh * a.K;
    return (kh * a.HPi + kw) * a.Cin + c * CW;
  };
  // the lane's K-block (32 channels = 32 B of e4m3 / e5m2) of step ks: element offset from xbase
  auto lane_off = [&](int ks) {
    if constexpr (CW == 64) {
      const int off0 = chunk_off(2 * ks), off1 = chunk_off(2 * ks + 1);
      return g >= 2 ? off1 : off0;
    } else {
      const int o0 = chunk_off(4 * ks), o1 = chunk_off(4 * ks + 1);
      const int o2 = chunk_off(4 * ks + 2), o3 = chunk_off(4 * ks + 3);
      return g == 0 ? o0 : g == 1 ? o1 : g == 2 ? o2 : o3;
    }
  };
  u32x4 wreg[WP];
  auto load_w = [&](int ks) {
    if constexpr (PROBE & 4) return;
    const int k0 = ks < nK ? ks : nK - 1;  // one step ahead of the last: any in-range step (unused)
#pragma unroll
    for (int i = 0; i < WP; ++i) wreg[i] = __builtin_amdgcn_raw_buffer_load_b128(wr, wsrc[i], k0 * a.Cout * 128, 0);
  };
  auto store_w = [&](int slot) {
    if constexpr (PROBE & 4) return;
#pragma unroll
    for (int i = 0; i < WP; ++i) *(u32x4*)(smem + slot * W_BYTES + wdst[i]) = wreg[i];
  };
  auto load_x = [&](i32x8 (&xf)[MB], int ks) {
    if constexpr (PROBE & 2) {
#pragma unroll
      for (int j = 0; j < MB; ++j) xf[j] = i32x8{ks, j, lane, 0, ks, j, lane, 0};
      return;
    }
    const int off = lane_off(ks);
#pragma unroll
    for (int j = 0; j < MB; ++j) {
      const u32x4 lo = __builtin_amdgcn_raw_buffer_load_b128(xr, xbase[j] + off, 0, 0);
      const u32x4 hi = __builtin_amdgcn_raw_buffer_load_b128(xr, xbase[j] + off + 16, 0, 0);
      xf[j] = i32x8{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
    }
  };
  // DGB: the raw bf16 operand of a step (4 x 16 B per fragment), converted at the top of its step
  u32x4 xraw[DGB ? MB : 1][4];
  const float gin = DGB ? 1.f / *a.in_scale : 1.f;  // power of two: exact
  auto load_xraw = [&](int ks) {
    const int off = lane_off(ks) * 2;
#pragma unroll
    for (int j = 0; j < (DGB ? MB : 0); ++j)
#pragma unroll
      for (int k = 0; k < 4; ++k) xraw[j][k] = __builtin_amdgcn_raw_buffer_load_b128(xr, xbase[j] * 2 + off + 16 * k, 0, 0);
  };
  auto convert_x = [&](i32x8 (&xf)[MB]) {
#pragma unroll
    for (int j = 0; j < (DGB ? MB : 0); ++j) {
      // dword d of the fragment = e5m2 of channels 4d .. 4d+3 = bf16 pairs 2d, 2d+1 of the raw load
#pragma unroll
      for (int d = 0; d < 8; ++d) {
        const u32x4& r = xraw[j][d >> 1];
        const unsigned p0 = (d & 1) ? r.z : r.x, p1 = (d & 1) ? r.w : r.y;
        xf[j][d] = cvt4_bf16_bf8(p0, p1, gin);
      }
    }
  };

  f32x4 acc[NB][MB];
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int j = 0; j < MB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int r15 = lane & 15;
  const int c0 = ((2 * g) ^ fp8_swz(r15)) << 4;
  const int c1 = ((2 * g + 1) ^ fp8_swz(r15)) << 4;
  const int wrow = r15 * 128;

  // issue order per step: W(next) then x(next); every consumer waits for exactly its own loads
  i32x8 xa[MB], xb[MB];
  load_w(0);
  if constexpr (DGB) load_xraw(0);
  else load_x(xa, 0);
  store_w(0);
  __syncthreads();
  auto body = [&](int ks, i32x8 (&xc)[MB], i32x8 (&xn)[MB]) {
    const char* wb = smem + (ks & 1) * W_BYTES;
    if constexpr (DGB) convert_x(xc);  // this step's raw loads -> e5m2 (waits for exactly them)
    load_w(ks + 1);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (DGB) load_xraw(ks + 1);
    else load_x(xn, ks + 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int h = 0; h < NPART; ++h) {
      i32x8 wf[NH];
#pragma unroll
      for (int i = 0; i < NH; ++i) {
        const char* p = wb + wrow + (h * NH + i) * 16 * 128;
        if constexpr (PROBE & 8) {
          wf[i] = i32x8{h, i, ks, lane, h, i, ks, lane};
          continue;
        }
        const int4 lo = *(const int4*)(p + c0);
        const int4 hi = *(const int4*)(p + c1);
        wf[i] = i32x8{lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < NH; ++i)
#pragma unroll
        for (int j = 0; j < MB; ++j)
          if constexpr (PROBE & 1) acc[h * NH + i][j][0] += (float)(wf[i][0] ^ xc[j][1]);
          else acc[h * NH + i][j] = (DG || DGB) ? mfma_fp8_bf8(wf[i], xc[j], acc[h * NH + i][j], sw, sx)
                                           : mfma_fp8(wf[i], xc[j], acc[h * NH + i][j], sw, sx);
      __builtin_amdgcn_s_setprio(0);
    }
    store_w((ks + 1) & 1);
    __syncthreads();
  };
  int ks = 0;
  for (; ks + 1 < nK; ks += 2) {
    body(ks, xa, xb);
    body(ks + 1, xb, xa);
  }
  if (ks < nK) body(ks, xa, xb);
  wait_vmcnt0();

  // --- epilogue: bias + ReLU, amax, bf16 and/or e4m3 stores (lane: 4 channels of one pixel per block)
  // STG: the wave's byte outputs go to its own LDS rows (SROW bytes per pixel) and leave as 16-B
  // row segments after the block loop (the weight slots are free: the loop ended on a barrier)
  char* stg = smem + wave * (16 * MB * SROW);
  const int nbase = n0 + ((lane >> 4) << 2);
  const float osc = a.out_scale[0];
  const bool sr = a.sr_seed != nullptr;  // uniform
  const uint32_t seed = sr ? (uint32_t)*a.sr_seed : 0u;
  float vmax = 0.f;
  // ReLU' bitmask in conv_fwd_kernel's layout: channel block i belongs to its wave half
  // wn = i / (NB/2), bit 4*(i % (NB/2)) + r of word blockIdx.y*8 + wn*4 + lane/16
  const int mwords = gridDim.y * 8;
  // the lane's bias quads, loaded once for all MB pixel blocks and issued back to back: inside the
  // block loop the compiler sank each load under the pixel-range branch and waited on it there, 30
  // serialised L2 round trips per wave at MB 3 x NB 10 (ISA of the 160-wide value forward)
  constexpr bool BIAS = !DG && !MASKBITS;
  f32x4 bias4[BIAS ? NB : 1];
  if constexpr (BIAS) {
#pragma unroll
    for (int i = 0; i < NB; ++i) bias4[i] = *(const f32x4*)(a.bias + nbase + i * 16);
  }
  // pixel of each block and (MASKBITS) its ReLU' words, all issued before the first use
  int pixo[MB];
  bool okj[MB];
  uint32_t mwj[MASKBITS ? MB : 1][2];
#pragma unroll
  for (int j = 0; j < MB; ++j) {
    int m = m0 + wave * 16 * MB + j * 16 + (lane & 15);
    okj[j] = m < a.M;
    m = okj[j] ? m : a.M - 1;
    const int b = fdiv(m, a.divSS);
    const int rem = m - b * SS;
    const int ii = fdiv(rem, a.divS);
    const int jj = rem - ii * a.S;
    pixo[j] = (b * a.HPo + ii + a.Po) * a.HPo + jj + a.Po;
    if constexpr (MASKBITS) {  // ReLU' bits of the lane's channels (the forward epilogue's layout)
      const size_t pw = (size_t)pixo[j] * mwords + blockIdx.y * 8 + ((lane >> 4) & 3);
      mwj[j][0] = a.mbits_in[pw];
      mwj[j][1] = a.mbits_in[pw + 4];
    }
  }
#pragma unroll
  for (int j = 0; j < MB; ++j) {
    uint32_t mb[2] = {0u, 0u};
    const bool ok = okj[j];
    const size_t ooff = (size_t)pixo[j] * a.Cout;
    uint32_t mw[2] = {0u, 0u};
    if constexpr (MASKBITS) {
      mw[0] = mwj[j][0];
      mw[1] = mwj[j][1];
    }
    bf16x4 mk[DG ? NB : 1];  // DG: the block's ReLU' mask quads, issued together (m is clamped in range)
    if constexpr (DG) {
#pragma unroll
      for (int i = 0; i < NB; ++i) mk[i] = *(const bf16x4*)(a.mask + ooff + nbase + i * 16);
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int n = nbase + i * 16;
      f32x4 v = acc[i][j];
      if constexpr (MASKBITS) {
        const uint32_t w = mw[i / (NB / 2)];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = ((w >> (4 * (i % (NB / 2)) + r)) & 1u) ? v[r] : 0.f;
      } else if constexpr (DG) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = (float)mk[i][r] > 0.f ? v[r] : 0.f;
      } else {
        const f32x4 bb = bias4[i];
        v[0] = fmaxf(v[0] + bb[0], 0.f);
        v[1] = fmaxf(v[1] + bb[1], 0.f);
        v[2] = fmaxf(v[2] + bb[2], 0.f);
        v[3] = fmaxf(v[3] + bb[3], 0.f);
      }
      if (!ok) continue;
      if constexpr ((PROBE & 16) != 0) {
        vmax = fmaxf(vmax, v[0] + v[1] + v[2] + v[3]);
        continue;
      }
      if constexpr (DG || DGB)
        vmax = fmaxf(vmax, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
      else
        vmax = fmaxf(vmax, fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3])));
      if constexpr (OUT_BF16) {
        bf16x4 o;
        o[0] = (__bf16)v[0];
        o[1] = (__bf16)v[1];
        o[2] = (__bf16)v[2];
        o[3] = (__bf16)v[3];
        *(bf16x4*)(a.y_bf16 + ooff + n) = o;
        if constexpr (!DG && !DGB && NB % 2 == 0) {
#pragma unroll
          for (int r = 0; r < 4; ++r) mb[i / (NB / 2)] |= ((float)o[r] > 0.f ? 1u : 0u) << (4 * (i % (NB / 2)) + r);
        }
      } else if constexpr (!DG && !DGB && NB % 2 == 0) {
        // e4m3-only forward (the all-fp8 value step: no bf16 consumer below the last layer): the
        // ReLU' bits from the fp32 result (bf16 rounding keeps the sign and fp32's exponent range)
#pragma unroll
        for (int r = 0; r < 4; ++r) mb[i / (NB / 2)] |= (v[r] > 0.f ? 1u : 0u) << (4 * (i % (NB / 2)) + r);
      }
      if constexpr (OUT_FP8) {
        if constexpr (DG) {
          float sv[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) sv[r] = fminf(fmaxf(v[r] * osc, -57344.f), 57344.f);
          int pk = __builtin_amdgcn_cvt_pk_bf8_f32(sv[0], sv[1], 0, false);
          pk = __builtin_amdgcn_cvt_pk_bf8_f32(sv[2], sv[3], pk, true);
          if constexpr (STG) *(int*)(stg + (j * 16 + (lane & 15)) * SROW + (n - n0)) = pk;
          else *(int*)(a.y_fp8 + ooff + n) = pk;
        } else {
          const float s0 = fminf(v[0] * osc, 448.f), s1 = fminf(v[1] * osc, 448.f);
          const float s2 = fminf(v[2] * osc, 448.f), s3 = fminf(v[3] * osc, 448.f);
          const int pk = fp8_pack4(s0, s1, s2, s3, sr, (uint32_t)(ooff + n), seed);
          if constexpr (STG) *(int*)(stg + (j * 16 + (lane & 15)) * SROW + (n - n0)) = pk;
          else *(int*)(a.y_fp8 + ooff + n) = pk;
        }
      }
    }
    if constexpr (!DG && !DGB && NB % 2 == 0) {
      if (a.mbits_out && ok) {
        const size_t pw = (size_t)pixo[j] * mwords + blockIdx.y * 8 + ((lane >> 4) & 3);
        a.mbits_out[pw] = mb[0];
        a.mbits_out[pw + 4] = mb[1];
      }
    }
  }
  if constexpr (STG) {
    __syncthreads();  // the block loop's LDS writes before the row reads (any lane's rows)
    constexpr int SEG = BN / 16;  // 16-B segments per pixel
    constexpr int TOT = 16 * MB * SEG;
#pragma unroll
    for (int it = 0; it < (TOT + 63) / 64; ++it) {
      const int idx = it * 64 + lane;
      const int p = idx / SEG, sg = idx - p * SEG;
      const int m = m0 + wave * 16 * MB + p;
      if (idx < TOT && m < a.M) {
        const int b = fdiv(m, a.divSS);
        const int rem = m - b * SS;
        const int ii = fdiv(rem, a.divS);
        const int jj = rem - ii * a.S;
        const size_t po = (size_t)((b * a.HPo + ii + a.Po) * a.HPo + jj + a.Po);
        *(u32x4*)(a.y_fp8 + po * a.Cout + n0 + sg * 16) = *(const u32x4*)(stg + p * SROW + sg * 16);
      }
    }
  }
  if (a.amax) {
    vmax = wave_max(vmax);
    float* red = reinterpret_cast<float*>(smem + RED_OFF);
    if (lane == 0) red[wave] = vmax;
    __syncthreads();
    if (threadIdx.x == 0) {
      float m = red[0];
#pragma unroll
      for (int w = 1; w < NW; ++w) m = fmaxf(m, red[w]);
      atomicMax(a.amax + (blockIdx.x & (kFp8AmaxSlots - 1)), __float_as_uint(m));
    }
  }
}

// ConvFp8Args::variant: 0 = production (pixel operand from L2, 48 px/wave,
// weights in 4 parts); kernel-lab build only: 1 / 3 / 4 = other L2-operand
// tilings, 5 = LDS-staged conv_fwd_fp8_kernel

template <int BN, int MB, int NPART, bool OB, bool OF, bool DG, bool DGB, bool DGBITS, int CW, int NW, bool STGE,
          int PROBE = 0>
static void launch_fp8_ga_cw(const ConvFp8Args& a, hipStream_t st) {
  constexpr int smem = fp8_ga_red_off(BN, MB, STGE && OF, NW) + 64;  // as in the kernel
  static const hipError_t attr = hipFuncSetAttribute(
      (const void*)conv_fwd_fp8_ga_kernel<BN, MB, NPART, OB, OF, DG, DGB, DGBITS, CW, NW, STGE, PROBE>,
      hipFuncAttributeMaxDynamicSharedMemorySize, smem);  // once per instantiation (thread-safe static)
  hip_check(attr, "hipFuncSetAttribute(max dynamic LDS)");
  constexpr int BM = NW * 16 * MB;
  dim3 grid((a.M + BM - 1) / BM, a.Cout / BN);
  hipLaunchKernelGGL((conv_fwd_fp8_ga_kernel<BN, MB, NPART, OB, OF, DG, DGB, DGBITS, CW, NW, STGE, PROBE>), grid, dim3(64 * NW), smem, st,
                     a);
}

// a.cw: the packed weights' chunk width (32 for the 160-channel value layers packed in 32-channel
// chunks, else 64).  The 160-wide value tile runs 4-wave workgroups, two per CU, with the byte
// outputs staged through LDS: value layer at B = 1024, e4m3 output + ReLU' bitmask (the fp8
// training forward), same-box lab A/B (scripts/r5/fp8_probe2.py): 120.3 us (8 waves, direct
// 4-B stores) -> 116.3 (staged) / 109.4 (4 waves) -> 101.4 (both); bf16 + e4m3 outputs 138.6 -> 115.2
// (4-wave workgroups only with 32-channel chunks: the 64-channel packing's extra weight pieces spill).
// The 192-wide policy tile stages its byte outputs too, with 8-wave workgroups (4 waves spill 23-81
// VGPRs there): B = 1024, same-box lab A/B (lab 7 = the staged tile, scripts/r5/gpu49.sh): e4m3
// output 151.6 -> 146.8 us, e4m3 + bitmask 156.3 -> 148.2, bf16 + e4m3 185.5 -> 161.9; B = 64 34.5 -> 33.2.
// NW = 0 / STGE = -1: this policy; lab variants pass explicit values
template <int BN, int MB, int NPART, bool OB, bool OF, bool DG = false, bool DGB = false, bool DGBITS = false,
          int NW = 0, int STGE = -1>
static void launch_fp8_ga(const ConvFp8Args& a, hipStream_t st) {
  constexpr bool stg = STGE >= 0 ? STGE != 0 : (BN == 160 || BN == 192);
  if (a.cw == 32) launch_fp8_ga_cw<BN, MB, NPART, OB, OF, DG, DGB, DGBITS, 32, NW ? NW : (BN == 160 ? 4 : 8), stg>(a, st);
  else launch_fp8_ga_cw<BN, MB, NPART, OB, OF, DG, DGB, DGBITS, 64, NW ? NW : 8, stg>(a, st);
}

// fp8 dgrad of the fp8-wgrad value step: e5m2 operand (the previous dgrad's copy), bitmask ReLU',
// e5m2 and/or bf16 outputs; the 160-wide value tile only
template <bool OB, bool OF>
static void launch_fp8_dgrad_bits_t(const ConvFp8Args& a, hipStream_t st) {
  launch_fp8_ga<160, 3, 5, OB, OF, true, false, true>(a, st);
}

// fp8 dgrad from the bf16 gradient (in-register e5m2 conversion, bitmask ReLU', bf16 output)
template <int BN>
static void launch_fp8_dgrad_bf16(const ConvFp8Args& a, hipStream_t st) {
  if (a.y_bf16 == nullptr || a.mbits_in == nullptr || a.in_scale == nullptr)
    throw std::invalid_argument("conv_dgrad_fp8 (bf16 operand): needs y_bf16, mbits and the input scale");
  if constexpr (BN == 160) launch_fp8_ga<160, 2, 5, true, false, false, true>(a, st);
  else if constexpr (BN == 192) launch_fp8_ga<192, 2, 4, true, false, false, true>(a, st);
  else launch_fp8_ga<BN, 2, 2, true, false, false, true>(a, st);
}

// fp8 dgrad: production tilings only, bf16 output always (the wgrad reads it)
template <int BN, bool OF>
static void launch_fp8_dgrad_t(const ConvFp8Args& a, hipStream_t st) {
  if (a.variant != 0) throw std::invalid_argument("conv_dgrad_fp8: production kernel only");
  if constexpr (BN == 160) launch_fp8_ga<160, 3, 5, true, OF, true>(a, st);
  else if constexpr (BN == 192) launch_fp8_ga<192, 3, 4, true, OF, true>(a, st);
  else launch_fp8_ga<BN, 2, 2, true, OF, true>(a, st);
}

template <int BN>
static void launch_fp8_dgrad_bn(const ConvFp8Args& a, hipStream_t st) {
  if (a.y_bf16 == nullptr) throw std::invalid_argument("conv_dgrad_fp8: needs the bf16 output");
  if (a.y_fp8 != nullptr) launch_fp8_dgrad_t<BN, true>(a, st);
  else launch_fp8_dgrad_t<BN, false>(a, st);
}

template <int BN, bool OB, bool OF>
static void launch_fp8_t(const ConvFp8Args& a, hipStream_t st) {
  if (a.cw != 64 && a.variant != 0 && a.variant != 6 && a.variant <= 100) throw std::invalid_argument("conv_fwd_fp8: 32-channel chunks: production kernel only");
#ifndef AGK_KERNEL_LAB
  if (a.variant != 0) throw std::invalid_argument("conv_fwd_fp8: variant " + std::to_string(a.variant) +
                                                  " is a kernel-lab variant");
#endif
  if constexpr (BN == 160) {  // value net (152 filters): L2-operand kernel only
    // production: 48 px per wave, weights read in 5 parts (230 VGPRs, no spills).  Value layer,
    // B=1024, round-robin min (scripts/lab/fp8_160_variants.py): 149.5 us; lab 1 (48 px, 2 parts,
    // 254 VGPRs) 146.1; lab 3 (32 px, 5 parts) 158.8; lab 4 (32 px, 2 parts) 157.0 (as the
    // default it cost value fp8 training 144.9k -> 142.9k)
    if (a.variant == 0) launch_fp8_ga<160, 3, 5, OB, OF>(a, st);
#ifdef AGK_KERNEL_LAB
    else if (a.variant == 1) launch_fp8_ga<160, 3, 2, OB, OF>(a, st);
    else if (a.variant == 3) launch_fp8_ga<160, 2, 5, OB, OF>(a, st);
    else if (a.variant == 4) launch_fp8_ga<160, 2, 2, OB, OF>(a, st);
    else if (a.variant == 6) launch_fp8_ga<160, 3, 5, OB, OF, false, false, false, 8, 0>(a, st);  // round 4
    else if (a.variant > 100 && a.variant < 132 && a.cw == 32) {  // timing probes (PROBE = variant - 100)
      switch (a.variant - 100) {
#define AGK_FP8_PROBE(P) \
  case P: launch_fp8_ga_cw<160, 3, 5, OB, OF, false, false, false, 32, 4, true, P>(a, st); break;
        AGK_FP8_PROBE(1) AGK_FP8_PROBE(2) AGK_FP8_PROBE(4) AGK_FP8_PROBE(8) AGK_FP8_PROBE(16)
        AGK_FP8_PROBE(6) AGK_FP8_PROBE(14) AGK_FP8_PROBE(30) AGK_FP8_PROBE(31) AGK_FP8_PROBE(17)
#undef AGK_FP8_PROBE
        default: throw std::invalid_argument("conv_fwd_fp8: probe " + std::to_string(a.variant));
      }
    }
#endif
    else throw std::invalid_argument("conv_fwd_fp8: 160-wide tile variant " + std::to_string(a.variant));
  } else {
    if (a.variant != 5 && (BN * 128) % (16 * 512) == 0) {
      if constexpr (BN == 192) {
        // 0: 48 px/wave, weights read in 4 parts (production); lab: 1: 32 px/wave, 2 parts;
        // 3: 32 px/wave, 3 parts; 4: 48 px/wave, 6 parts
        if (a.variant == 0) launch_fp8_ga<BN, 3, 4, OB, OF>(a, st);
#ifdef AGK_KERNEL_LAB
        else if (a.variant == 3) launch_fp8_ga<BN, 2, 3, OB, OF>(a, st);
        else if (a.variant == 4) launch_fp8_ga<BN, 3, 6, OB, OF>(a, st);
        else if (a.variant == 6) launch_fp8_ga<BN, 3, 4, OB, OF, false, false, false, 4, 1>(a, st);
        else if (a.variant == 7) launch_fp8_ga<BN, 3, 4, OB, OF, false, false, false, 8, 0>(a, st);  // round 4
        else launch_fp8_ga<BN, 2, 2, OB, OF>(a, st);
#endif
      } else {
        launch_fp8_ga<BN, 2, 2, OB, OF>(a, st);
      }
      return;
    }
#ifdef AGK_KERNEL_LAB
    constexpr int smem = 2 * (256 * 128 + BN * 128);
    static const hipError_t attr = hipFuncSetAttribute((const void*)conv_fwd_fp8_kernel<BN, OB, OF>,
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    hip_check(attr, "hipFuncSetAttribute(max dynamic LDS)");
    dim3 grid((a.M + 255) / 256, a.Cout / BN);
    hipLaunchKernelGGL((conv_fwd_fp8_kernel<BN, OB, OF>), grid, dim3(512), smem, st, a);
#endif
  }
}

template <int BN>
static void launch_fp8_bn(const ConvFp8Args& a, hipStream_t st) {
  const bool ob = a.y_bf16 != nullptr, of = a.y_fp8 != nullptr;
  if (ob && of) launch_fp8_t<BN, true, true>(a, st);
  else if (ob) launch_fp8_t<BN, true, false>(a, st);
  else launch_fp8_t<BN, false, true>(a, st);
}

void launch_conv_fwd_fp8(const ConvFp8Args& a_in, hipStream_t st) {
  ConvFp8Args a = a_in;
  a.divSS = make_fastdiv((uint32_t)(a.S * a.S));
  a.divS = make_fastdiv((uint32_t)a.S);
  const int cw = a.cw ? a.cw : 64;
  a.cw = cw;
  a.divCC = make_fastdiv((uint32_t)((a.Cin + cw - 1) / cw));  // chunks per tap
  a.divK = make_fastdiv((uint32_t)a.K);
  if (a.dgrad_bf16) {
    if (a.Cout == 160) launch_fp8_dgrad_bf16<160>(a, st);
    else if (a.Cout % 192 == 0) launch_fp8_dgrad_bf16<192>(a, st);
    else if (a.Cout % 128 == 0) launch_fp8_dgrad_bf16<128>(a, st);
    else launch_fp8_dgrad_bf16<64>(a, st);
    return;
  }
  if (a.dgrad && a.mbits_in) {
    if (a.Cout != 160) throw std::invalid_argument("conv_dgrad_fp8_bits: 160-wide value layers only");
    if (a.y_bf16 && a.y_fp8) launch_fp8_dgrad_bits_t<true, true>(a, st);
    else if (a.y_bf16) launch_fp8_dgrad_bits_t<true, false>(a, st);
    else launch_fp8_dgrad_bits_t<false, true>(a, st);
    return;
  }
  if (a.dgrad) {
    if (a.Cout == 160) launch_fp8_dgrad_bn<160>(a, st);
    else if (a.Cout % 192 == 0) launch_fp8_dgrad_bn<192>(a, st);
    else if (a.Cout % 128 == 0) launch_fp8_dgrad_bn<128>(a, st);
    else launch_fp8_dgrad_bn<64>(a, st);
    return;
  }
  if (a.Cout == 160) launch_fp8_bn<160>(a, st);
  else if (a.Cout % 192 == 0) launch_fp8_bn<192>(a, st);
  else if (a.Cout % 128 == 0) launch_fp8_bn<128>(a, st);
  else launch_fp8_bn<64>(a, st);
}

// ------------------------------------------------------------- packing
// weights: fp32 OIHW [Cout_real][Cin_real][K][K] -> e4m3 [nch][Cout_p][64] * 2^e, chunks over
// the input channels.  transposed (dgrad): rows = input channels, chunks over the output
// channels, taps flipped -- w'[ci][co][kh][kw] = w[co][ci][K-1-kh][K-1-kw]; Cout_p / Cin_p are
// then the padded row / chunked extents.
__global__ void pack_weights_fp8_kernel(const float* w, uint8_t* out, int Cout_real, int Cin_real, int K, int Cout_p,
                                        int Cin_p, int nch, float scale, const float* scale_dev, int transposed,
                                        int cw) {
  const int CC = Cin_p / cw;
  if (scale_dev) scale = *scale_dev;
  const int rows_real = transposed ? Cin_real : Cout_real;
  const int chans_real = transposed ? Cout_real : Cin_real;
  const long total = (long)nch * Cout_p * cw;
  for (long idx = (long)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const int byte = (int)(idx % cw);
    const long qn = idx / cw;
    const int n = (int)(qn % Cout_p);
    const int q = (int)(qn / Cout_p);
    const int t = q / CC;
    const int c = (q - t * CC) * cw + byte;
    float v = 0.f;
    if (t < K * K && n < rows_real && c < chans_real) {
      const int kh = t / K, kw = t - (t / K) * K;
      const size_t src = transposed ? (((size_t)c * Cin_real + n) * K + (K - 1 - kh)) * K + (K - 1 - kw)
                                    : (((size_t)n * Cin_real + c) * K + kh) * K + kw;
      v = w[src] * scale;
      v = fminf(fmaxf(v, -448.f), 448.f);
    }
    out[idx] = (uint8_t)(__builtin_amdgcn_cvt_pk_fp8_f32(v, 0.f, 0, false) & 0xff);
  }
}

void launch_pack_weights_fp8(const float* w, uint8_t* out, int Cout_real, int Cin_real, int K, int Cout_p, int Cin_p,
                             int nch, float scale, const float* scale_dev, int transposed, int cw, hipStream_t st) {
  const long total = (long)nch * Cout_p * cw;
  int blocks = (int)((total + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(pack_weights_fp8_kernel, dim3(blocks), dim3(256), 0, st, w, out, Cout_real, Cin_real, K, Cout_p,
                     Cin_p, nch, scale, scale_dev, transposed, cw);
}

__global__ __launch_bounds__(256) void pack_weights_fp8_multi_kernel(Fp8PackArgs a) {
  const Fp8PackJob& j = a.jobs[blockIdx.y];
  const int cw = j.cw;
  const int CC = j.Cin_p / cw;
  const float scale = *j.scale;
  const int rows_real = j.transposed ? j.Cin_real : j.Cout_real;
  const int chans_real = j.transposed ? j.Cout_real : j.Cin_real;
  const int K = j.K;
  const long total = (long)j.nch * j.Cout_p * (cw / 4);  // 4 bytes per thread
  for (long i4 = (long)blockIdx.x * blockDim.x + threadIdx.x; i4 < total; i4 += (long)gridDim.x * blockDim.x) {
    const long idx = i4 * 4;
    const int byte = (int)(idx % cw);
    const long qn = idx / cw;
    const int n = (int)(qn % j.Cout_p);
    const int q = (int)(qn / j.Cout_p);
    const int t = q / CC;
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = (q - t * CC) * cw + byte + r;
      v[r] = 0.f;
      if (t < K * K && n < rows_real && c < chans_real) {
        const int kh = t / K, kw = t - (t / K) * K;
        const size_t src = j.transposed ? (((size_t)c * j.Cin_real + n) * K + (K - 1 - kh)) * K + (K - 1 - kw)
                                        : (((size_t)n * j.Cin_real + c) * K + kh) * K + kw;
        v[r] = fminf(fmaxf(j.w[src] * scale, -448.f), 448.f);
      }
    }
    int pk = __builtin_amdgcn_cvt_pk_fp8_f32(v[0], v[1], 0, false);
    pk = __builtin_amdgcn_cvt_pk_fp8_f32(v[2], v[3], pk, true);
    *(int*)(j.out + idx) = pk;
  }
}

void launch_pack_weights_fp8_multi(const Fp8PackArgs& a, hipStream_t st) {
  if (a.n <= 0) return;
  hipLaunchKernelGGL(pack_weights_fp8_multi_kernel, dim3(64, a.n), dim3(256), 0, st, a);
}

// Per-layer weight scales, one workgroup per layer: e = floor(log2(448 / amax|w|)),
// wscale[l] = 2^e (for packing) and the MFMA E8M0 exponent scales8[l][1] = 127 - e.
__global__ __launch_bounds__(1024) void fp8_weight_scales_kernel(Fp8WeightScalesArgs a) {
  __shared__ float red[16];
  const int l = blockIdx.x;
  const float* w = a.w[l];
  const int n = a.n[l];
  // eight independent 16-B loads in flight per thread: a layer is a few round trips of one
  // workgroup (a one-load loop was latency-bound at 39.6 us per value-net repack, round 4; eight
  // 4-B loads still took 25 round trips per 208k-weight layer, 56 us per repack in round 5's step)
  float m = 0.f;
  const int n4 = (((uintptr_t)w) & 15) == 0 ? n >> 2 : 0;  // 16-B aligned prefix (the flat
                                                           // parameter buffer's views are)
  const float4* w4 = reinterpret_cast<const float4*>(w);
  for (int i0 = threadIdx.x; i0 < n4; i0 += 8 * 1024) {
    float4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int i = i0 + k * 1024;
      v[k] = i < n4 ? w4[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k)
      m = fmaxf(m, fmaxf(fmaxf(fabsf(v[k].x), fabsf(v[k].y)), fmaxf(fabsf(v[k].z), fabsf(v[k].w))));
  }
  for (int i = 4 * n4 + threadIdx.x; i < n; i += 1024) m = fmaxf(m, fabsf(w[i]));
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < 16; ++i) m = fmaxf(m, red[i]);
    m = fmaxf(m, red[0]);
    int e = (m > 0.f) ? (int)floorf(log2f(448.f / m)) : 0;
    e = e < -60 ? -60 : (e > 60 ? 60 : e);
    a.wscale[l] = exp2f((float)e);
    a.scales8[2 * l + 1] = 127 - e;
  }
}

void launch_fp8_weight_scales(const Fp8WeightScalesArgs& a, int L, hipStream_t st) {
  hipLaunchKernelGGL(fp8_weight_scales_kernel, dim3(L), dim3(1024), 0, st, a);
}

// Delayed activation scaling: from this step's per-layer output amax set the
// next step's e4m3 exponents (input of layer l+1 = output of layer l) with
// `margin` bits of headroom, then clear the amax accumulators.
// Underflow guard (max_drop > 0): the exponent falls by at most max_drop binades per step.  After a
// loss spike the amax of a layer can grow 2^8 within a few steps; following it at once pushed the bulk
// of the e4m3 activations below the format's smallest subnormal, round-to-nearest flushed them to zero
// and the trunk died (SL at lr 0.05, 1 seed of 3, profiles/r5/README.md).  Under the guard the outliers
// saturate at +-448 (a clip) while the scale follows at max_drop binades per step; a falling amax
// (growing exponent) is followed at once.  max_drop 0: the plain one-step delayed scale.
__global__ void fp8_act_scales_kernel(unsigned* amax, int* scales8, float* osc, int L, int margin, int max_drop) {
  const int l = threadIdx.x;
  if (l >= L) return;
  unsigned mu = 0u;
  for (int k = 0; k < kFp8AmaxSlots; ++k) mu = max(mu, amax[l * kFp8AmaxSlots + k]);
  const float m = __uint_as_float(mu);
  int e = (m > 0.f) ? (int)floorf(log2f(448.f / m)) - margin : 0;
  if (max_drop > 0 && l + 1 < L) {
    const int e_prev = 127 - scales8[2 * (l + 1)];
    if (e < e_prev - max_drop) e = e_prev - max_drop;
  }
  e = e < -60 ? -60 : (e > 60 ? 60 : e);
  if (l + 1 < L) {
    osc[l] = exp2f((float)e);
    scales8[2 * (l + 1)] = 127 - e;
  }
  for (int k = 0; k < kFp8AmaxSlots; ++k) amax[l * kFp8AmaxSlots + k] = 0u;
}

void launch_fp8_act_scales(unsigned* amax, int* scales8, float* osc, int L, int margin, int max_drop, hipStream_t st) {
  hipLaunchKernelGGL(fp8_act_scales_kernel, dim3(1), dim3(64), 0, st, amax, scales8, osc, L, margin, max_drop);
}

// Delayed gradient scaling for the fp8 dgrad chain: from this step's amax of dZ_l set the next
// step's e5m2 exponent of dZ_l (gosc[l] = 2^e multiplies before conversion, gscales8[l][0] =
// 127 - e is the MFMA's E8M0 dequantisation), `margin` bits of headroom; clears the amax.
__global__ void fp8_grad_scales_kernel(unsigned* amax, int* gscales8, float* gosc, int L, int margin) {
  const int l = threadIdx.x;
  if (l >= L) return;
  unsigned mu = 0u;
  for (int k = 0; k < kFp8AmaxSlots; ++k) mu = max(mu, amax[l * kFp8AmaxSlots + k]);
  const float m = __uint_as_float(mu);
  int e = (m > 0.f) ? (int)floorf(log2f(57344.f / m)) - margin : 0;
  e = e < -100 ? -100 : (e > 100 ? 100 : e);
  gosc[l] = exp2f((float)e);
  gscales8[2 * l] = 127 - e;
  for (int k = 0; k < kFp8AmaxSlots; ++k) amax[l * kFp8AmaxSlots + k] = 0u;
}

void launch_fp8_grad_scales(unsigned* amax, int* gscales8, float* gosc, int L, int margin, hipStream_t st) {
  hipLaunchKernelGGL(fp8_grad_scales_kernel, dim3(1), dim3(64), 0, st, amax, gscales8, gosc, L, margin);
}

// e5m2 quantisation with a device-resident scale, tracking max |x| (the head's dZ, the first
// input of the fp8 dgrad chain).  16-byte loads (8 bf16), 8-byte stores, one grid round of 4
// workgroups per CU, and the max folded per workgroup before one atomic (round 3: 8-byte loads and
// a per-wave atomic over 4096 workgroups took 99 us for the value head's 72 M elements)
// E4M3 = true: the e4m3 variant (activations: a bf16-precision layer of the mixed-precision fp8 step
// feeding an fp8 layer, with the delayed activation scale and amax of the fp8 kernels)
template <bool E4M3>
__global__ __launch_bounds__(256) void quantize_bf8_dev_kernel(const __bf16* x, uint8_t* y, long n8, const float* scale,
                                                               unsigned* amax) {
  __shared__ float red[4];
  constexpr float kMax = E4M3 ? 448.f : 57344.f;
  const float sc = *scale;
  float m = 0.f;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    const bf16x8 v = *(const bf16x8*)(x + 8 * i);
    float f[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      f[r] = (float)v[r];
      m = fmaxf(m, fabsf(f[r]));
      f[r] = fminf(fmaxf(f[r] * sc, -kMax), kMax);
    }
    if (y) {  // null: max |x| only
      int lo, hi;
      if constexpr (E4M3) {
        lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], 0, false);
        lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], lo, true);
        hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[4], f[5], 0, false);
        hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[6], f[7], hi, true);
      } else {
        lo = __builtin_amdgcn_cvt_pk_bf8_f32(f[0], f[1], 0, false);
        lo = __builtin_amdgcn_cvt_pk_bf8_f32(f[2], f[3], lo, true);
        hi = __builtin_amdgcn_cvt_pk_bf8_f32(f[4], f[5], 0, false);
        hi = __builtin_amdgcn_cvt_pk_bf8_f32(f[6], f[7], hi, true);
      }
      *(int2*)(y + 8 * i) = make_int2(lo, hi);
    }
  }
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    if (m > 0.f) atomicMax(amax + (blockIdx.x & (kFp8AmaxSlots - 1)), __float_as_uint(m));
  }
}

void launch_quantize_bf8_dev(const __bf16* x, uint8_t* y, long n, const float* scale, unsigned* amax, hipStream_t st,
                             bool e4m3) {
  if (n % 8 != 0) throw std::invalid_argument("quantize_bf8: element count must be a multiple of 8");
  const long n8 = n / 8;
  int blocks = (int)((n8 + 255) / 256);
  if (blocks > 1024) blocks = 1024;
  if (blocks < 1) return;
  if (e4m3) hipLaunchKernelGGL(quantize_bf8_dev_kernel<true>, dim3(blocks), dim3(256), 0, st, x, y, n8, scale, amax);
  else hipLaunchKernelGGL(quantize_bf8_dev_kernel<false>, dim3(blocks), dim3(256), 0, st, x, y, n8, scale, amax);
}

#ifdef AGK_KERNEL_LAB
// Probe of v_cvt_scalef32_pk_bf8_bf16 (2 bf16 -> 2 e5m2 with an f32 scale, one instruction):
// mode 0 = f32 multiply + v_cvt_pk_bf8_f32 (the reference), 1 = scalef32 with `scale`,
// 2 = scalef32 with 1 / scale.  tests/test_fp8_inference.py pins which scalef32 form equals x * scale.
typedef __attribute__((ext_vector_type(2))) short agk_s16x2;
typedef __attribute__((ext_vector_type(2))) __bf16 agk_bf16x2;
__global__ void bf8_convert_probe_kernel(const __bf16* x, uint8_t* y, long n2, float scale, int mode) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += (long)gridDim.x * blockDim.x) {
    const agk_bf16x2 v = *(const agk_bf16x2*)(x + 2 * i);
    unsigned short out;
    if (mode == 0) {
      const float f0 = fminf(fmaxf((float)v[0] * scale, -57344.f), 57344.f);
      const float f1 = fminf(fmaxf((float)v[1] * scale, -57344.f), 57344.f);
      out = (unsigned short)__builtin_amdgcn_cvt_pk_bf8_f32(f0, f1, 0, false);
    } else {
      const agk_s16x2 r = __builtin_amdgcn_cvt_scalef32_pk_bf8_bf16((agk_s16x2){0, 0}, v,
                                                                     mode == 1 ? scale : 1.f / scale, false);
      out = (unsigned short)r[0];
    }
    *(unsigned short*)(y + 2 * i) = out;
  }
}
void launch_bf8_convert_probe(const __bf16* x, uint8_t* y, long n, float scale, int mode, hipStream_t st) {
  hipLaunchKernelGGL(bf8_convert_probe_kernel, dim3(256), dim3(256), 0, st, x, y, n / 2, scale, mode);
}
#endif

// e4m3 quantisation of a padded NHWC bf16 tensor (interior and borders alike: borders stay 0)
__global__ void quantize_fp8_kernel(const __bf16* x, uint8_t* y, long n4, float scale) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const bf16x4 v = *(const bf16x4*)(x + 4 * i);
    const float s0 = fminf(fmaxf((float)v[0] * scale, -448.f), 448.f);
    const float s1 = fminf(fmaxf((float)v[1] * scale, -448.f), 448.f);
    const float s2 = fminf(fmaxf((float)v[2] * scale, -448.f), 448.f);
    const float s3 = fminf(fmaxf((float)v[3] * scale, -448.f), 448.f);
    int pk = __builtin_amdgcn_cvt_pk_fp8_f32(s0, s1, 0, false);
    pk = __builtin_amdgcn_cvt_pk_fp8_f32(s2, s3, pk, true);
    *(int*)(y + 4 * i) = pk;
  }
}

void launch_quantize_fp8(const __bf16* x, uint8_t* y, long n, float scale, hipStream_t st) {
  const long n4 = n / 4;
  int blocks = (int)((n4 + 255) / 256);
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(quantize_fp8_kernel, dim3(blocks), dim3(256), 0, st, x, y, n4, scale);
}

}  // namespace agk
