// Weight-stationary small-batch convolution (tile code 40).
//
// At the reference's training batch (B = 16, supervised_policy_trainer.py:93) and the search's leaf
// batches (mcts.py:107-118 calls the policy at batch 1) the implicit-GEMM tiles of conv_fwd_kernel are
// latency bound: every 32-pixel workgroup streams the whole 663 KB weight tensor of a 192 -> 192 3x3
// layer through LDS, 27 dependent K-steps deep (B = 16 forward: ~21 us per layer, MFMA ~5 % busy).
// Here the weights do not move: a workgroup owns a slice of output channels and holds that slice's
// weights in VGPRs for its whole life -- the K dimension is split over the workgroup's waves, wave w
// keeping the A fragments of K-steps [w*KW, (w+1)*KW) of every n-block -- and streams 16-pixel chunks
// of activations past them (direct 16-byte global loads, one chunk prefetched ahead).  Each wave's
// partial 16 x (16*NBLK) tile goes to LDS; after one barrier per chunk the epilogue waves sum the
// NWV partials in wave order (deterministic) and apply bias + ReLU / the ReLU' bitmask.
//
// Channel slices are word-aligned to conv_fwd_kernel's ReLU'-bitmask layout ((Cout/BN)*8 words per
// padded pixel; word w covers channels base(w) + 16 i + r, i < BN/32, r < 4 -- see
// conv_splitk_finish_kernel): a slice holds WS whole words, so its epilogue writes whole bitmask words
// and the dgrad reads whole words; the slice's MFMA rows are those channels in (word, i, r) order.
//
// MFMA: v_mfma_f32_16x16x32_bf16 issued "swapped" as everywhere in this library -- A = 16 weight rows
// x 32 k, B = 32 k x 16 pixels; lane l holds D rows 4 (l/16) .. +3 (4 channels of one group) of pixel
// l % 16.
#include <hip/hip_runtime.h>


#include <algorithm>
#include <stdexcept>
#include <vector>
#include <string>

#include "conv_common.h"
#include "kernels.h"

namespace agk {

namespace {

struct WsParams {
  int cpw;     // 16-pixel chunks per workgroup
  int BN;      // conv_fwd_kernel's n tile of this Cout (bitmask layout)
  int NB;      // groups (of 4 channels) per bitmask word = BN / 32
  int WS;      // bitmask words per slice (WS * NB == 4 * NBLK)
  int WPP;     // bitmask words per padded pixel = (Cout / BN) * 8
  int CS;      // 32-channel K-steps per tap = Cin / 32
  int slices;  // channel slices = WPP / WS
  int ngrp;    // chunk groups = ceil(chunks / cpw)
  int k;       // slices per XCD (a divisor of slices); P = 8 k / slices XCDs share a slice set
  int P;
  int gper;    // chunk groups per XCD = ceil(ngrp / P); grid = 8 * k * gper
  int NR;      // RING: input-row slots (the rows of two consecutive chunks fit)
  int RS;      // RING: bytes per slot = HPi * PST
  int PST;     // RING: bytes per pixel in a slot = Cin * 2 + 16 (the pad spreads a fragment read over
               // all LDS banks)
};

typedef __attribute__((ext_vector_type(4))) unsigned ws_u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned ws_u32x2;

__device__ __forceinline__ int ws_word_base(int w, int BN) {
  const int tn = w >> 3, wn = (w >> 2) & 1, q = w & 3;
  return tn * BN + wn * (BN >> 1) + 4 * q;
}

// a raw buffer over [p, p + bytes): loads past the end return 0, stores past the end are dropped --
// so the epilogue's edge stores need no branch and every wave's vmcnt bookkeeping stays exact
__device__ __forceinline__ __amdgpu_buffer_rsrc_t ws_rsrc(const void* p, long long bytes) {
  if (!p) bytes = 0;
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)(bytes < 0x7fffffffLL ? bytes : 0x7fffffffLL),
                                           0x00020000);
}
constexpr unsigned WS_OOB = 0x80000000u;  // a byte offset past every buffer's end

}  // namespace

// NWV MFMA waves split the K-steps (KW each) and NE epilogue waves finish the chunks (1 workgroup per CU).
// The roles are wave-uniform and run separate loops that meet at one barrier per chunk (plus one after
// the prologue and one at the end), so the MFMA waves' vector-memory queue never holds the epilogue's
// output stores.  RING: activations through an LDS ring of input rows (RM: most new rows per chunk,
// IPR: 16-byte row units per lane); else straight from global memory, two chunks ahead.
// PROBE (kernel lab only, tiles 1000 + PROBE): bit 1 = no MFMA, bit 2 = no epilogue work, bit 3 = no
// weight loads -- which part sets the layer's time (round-5 probes: profiles/r5/README.md)
template <int NBLK, int KW, int NWV, int NE, int MODE, bool RING, int PROBE = 0>
__global__ __launch_bounds__(64 * (NWV + NE), 1) void conv_ws_kernel(ConvFwdArgs a, WsParams p) {
  constexpr int RM = 6, IPR = 1;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = wave_id();
  // XCD placement (blockIdx % 8 labels the workgroups that share an XCD's L2): the 8 XCDs form
  // slices / k sets of P; a set owns k slices -- their weights are what its L2s hold -- and each of its
  // P XCDs runs a contiguous 1 / P of the chunk groups for all k of them, so the k slices reading one
  // chunk's activations (and neighbouring chunks' halo rows) share an L2.  k trades weight bytes
  // (8 k / slices copies) against activation bytes (slices / k copies): launch_conv_ws picks it.
  const int xcd = blockIdx.x & 7, idx = blockIdx.x >> 3;
  const int sset = xcd / p.P, member = xcd - sset * p.P;
  const int gl = idx / p.k;
  const int slice = sset * p.k + (idx - gl * p.k), grp = member * p.gper + gl;
  if (gl >= p.gper || grp >= p.ngrp) return;  // the rounding tail: the whole workgroup leaves
  const int chunks = (a.M + 15) >> 4;
  const int c_begin = grp * p.cpw;
  const int c_end = c_begin + p.cpw < chunks ? c_begin + p.cpw : chunks;
  const int nc = c_end - c_begin;  // >= 1: ngrp = ceil(chunks / cpw)
  const int SS = a.S * a.S;
  constexpr int PART = NWV * NBLK * 64;           // f32x4 partials per chunk buffer
  f32x4* part = (f32x4*)smem;                     // [2][NWV][NBLK][64]
  uint32_t* bitw = (uint32_t*)(part + 2 * PART);  // [2][16 px][WS] bitmask words being assembled

  if (wave < NWV) {
    // ---------------- MFMA waves
    const int row = lane & 15, kq = lane >> 4;
    const int s0 = wave * KW;  // first K-step of this wave
    // the slice's weights, resident for the workgroup's life (A operands): in the weight-stationary
    // order (ws_pack_kernel) each fragment is one contiguous KB, 16 bytes per lane -- from the standard
    // [tap][Cout][Cin] pack each load instruction touched 16 half-used cache lines (round-5 probe: 4.6 us
    // of a 15 us layer at B = 16)
    bf16x8 wa[NBLK][KW];
    const __bf16* wsl = a.w + (size_t)(slice * NWV + wave) * NBLK * KW * 512 + lane * 8;
#pragma unroll
    for (int b = 0; b < NBLK; ++b)
#pragma unroll
      for (int kk = 0; kk < KW; ++kk) {
        if constexpr (PROBE & 8) wa[b][kk] = bf16x8{};
        else wa[b][kk] = *(const bf16x8*)(wsl + (b * KW + kk) * 512);
      }
    const __amdgpu_buffer_rsrc_t xr = ws_rsrc(a.x, (long long)(a.M / SS) * a.HPi * a.HPi * a.Cin * 2);
    auto mfma_chunk = [&](int j, const bf16x8 (&cur)[KW]) {
      f32x4 acc[NBLK];
#pragma unroll
      for (int b = 0; b < NBLK; ++b) acc[b] = f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (PROBE & 2) {
#pragma unroll
        for (int kk = 0; kk < KW; ++kk) acc[0][0] += (float)cur[kk][0] + (float)wa[kk % NBLK][kk][0];
      } else {
#pragma unroll
        for (int kk = 0; kk < KW; ++kk)
#pragma unroll
          for (int b = 0; b < NBLK; ++b) acc[b] = mfma16x16x32(wa[b][kk], cur[kk], acc[b]);
      }
      f32x4* pb = part + (j & 1) * PART;
#pragma unroll
      for (int b = 0; b < NBLK; ++b) pb[(wave * NBLK + b) * 64 + lane] = acc[b];
      __syncthreads();  // chunk j's partials complete (the epilogue waves read them next)
    };

    if constexpr (RING) {
      // Activations through an LDS ring of padded input rows: the waves copy each row the chunks need
      // once, as whole 16-byte runs of the row (a row of the padded NHWC input is contiguous), and every
      // wave then reads its B fragments (16 pixels x 64 bytes per K-step) from LDS.  Reading them from
      // global memory directly, each load instruction touched 16 half-used cache lines.
      uint8_t* ring = (uint8_t*)(bitw + 2 * 16 * p.WS);
      const int rowbytes = a.HPi * a.Cin * 2, upp = a.Cin / 8, U = a.HPi * upp;
      int u_src[IPR], u_dst[IPR];
#pragma unroll
      for (int i = 0; i < IPR; ++i) {  // this lane's 16-byte units of a row load
        const int u = wave * 64 + lane + 64 * NWV * i;
        const int uc = u < U ? u : U - 1;
        u_src[i] = uc * 16;
        u_dst[i] = u < U ? (uc / upp) * p.PST + (uc - (uc / upp) * upp) * 16 : -1;
      }
      // per-K-step tap row and in-row byte offset (tap column, channel chunk): wave-uniform
      int kh_[KW], kofs[KW];
#pragma unroll
      for (int kk = 0; kk < KW; ++kk) {
        const int s = s0 + kk;
        const int t = s / p.CS, c0 = (s - t * p.CS) * 32;
        const int kh = t / a.K, kw = t - kh * a.K;
        kh_[kk] = __builtin_amdgcn_readfirstlane(kh);
        kofs[kk] = __builtin_amdgcn_readfirstlane(kw * p.PST + c0 * 2);
      }
      auto row_of = [&](int m) -> int {  // padded input row of pixel m's first tap row
        const int bb = fdiv(m, a.divSS);
        const int ii = fdiv(m - bb * SS, a.divS);
        return bb * a.HPi + ii + a.offi;
      };
      auto g0 = [&](int c) { return __builtin_amdgcn_readfirstlane(row_of(c * 16)); };
      auto g1 = [&](int c) {
        const int m = c * 16 + 15 < a.M ? c * 16 + 15 : a.M - 1;
        return __builtin_amdgcn_readfirstlane(row_of(m) + a.K - 1);
      };
      auto load_row = [&](int G, ws_u32x4 (&v)[IPR]) {
#pragma unroll
        for (int i = 0; i < IPR; ++i) v[i] = __builtin_amdgcn_raw_buffer_load_b128(xr, u_src[i], G * rowbytes, 0);
      };
      auto write_row = [&](int G, const ws_u32x4 (&v)[IPR]) {
        uint8_t* d = ring + (G % p.NR) * p.RS;
#pragma unroll
        for (int i = 0; i < IPR; ++i)
          if (u_dst[i] >= 0) *(ws_u32x4*)(d + u_dst[i]) = v[i];
      };
      // prologue: the rows of the first two chunks
      int loaded = g1(c_begin + (nc > 1 ? 1 : 0));
      for (int G = g0(c_begin); G <= loaded; ++G) {
        ws_u32x4 v[IPR];
        load_row(G, v);
        write_row(G, v);
      }
      __syncthreads();
      ws_u32x4 stage[RM][IPR];
      int npend = 0, pend_lo = 0;
      for (int j = 0; j < nc; ++j) {
        const int c = c_begin + j;
        // a. the rows loaded during the previous chunk (chunk j + 1's new rows) into their slots: no wave
        // still reads those slots (the ring holds chunk j's and j + 1's rows at once; launch_conv_ws)
#pragma unroll
        for (int r = 0; r < RM; ++r)
          if (r < npend) write_row(pend_lo + r, stage[r]);
        // b. chunk j + 2's new rows into registers: written at the next chunk, read two chunks on
        npend = 0;
        if (j + 2 < nc) {
          const int h = g1(c + 2);
          pend_lo = loaded + 1;
          npend = h - loaded;
          loaded = h;
#pragma unroll
          for (int r = 0; r < RM; ++r)
            if (r < npend) load_row(pend_lo + r, stage[r]);
        }
        // c. this chunk's B fragments from the ring (past the last pixel: any valid pixel)
        const int m = c * 16 + row < a.M ? c * 16 + row : a.M - 1;
        const int bb = fdiv(m, a.divSS);
        const int rem = m - bb * SS;
        const int ii = fdiv(rem, a.divS);
        const int jj = rem - ii * a.S;
        const int gs = (bb * a.HPi + ii + a.offi) % p.NR;
        const uint8_t* cb = ring + (jj + a.offi) * p.PST + kq * 16;
        bf16x8 xb[KW];
#pragma unroll
        for (int kk = 0; kk < KW; ++kk) {
          const int sl = gs + kh_[kk] < p.NR ? gs + kh_[kk] : gs + kh_[kk] - p.NR;
          xb[kk] = *(const bf16x8*)(cb + sl * p.RS + kofs[kk]);
        }
        mfma_chunk(j, xb);
      }
    } else {
      // Activations straight from global memory, two chunks ahead (the 160-wide shape: its partials leave
      // no LDS for a ring)
      int koff[KW];  // per-K-step byte offsets (tap shift + channel chunk): wave-uniform, scalar operands
#pragma unroll
      for (int kk = 0; kk < KW; ++kk) {
        const int s = s0 + kk;
        const int t = s / p.CS, c0 = (s - t * p.CS) * 32;
        const int kh = t / a.K, kw = t - kh * a.K;
        koff[kk] = __builtin_amdgcn_readfirstlane(((kh * a.HPi + kw) * a.Cin + c0) * 2);
      }
      auto load_chunk = [&](int c, bf16x8 (&xb)[KW]) {  // (past the last pixel: any valid pixel)
        int m = c * 16 + row;
        m = m < a.M ? m : a.M - 1;
        const int bb = fdiv(m, a.divSS);
        const int rem = m - bb * SS;
        const int ii = fdiv(rem, a.divS);
        const int jj = rem - ii * a.S;
        const int base = (((bb * a.HPi + ii + a.offi) * a.HPi + jj + a.offi) * a.Cin + 8 * kq) * 2;
#pragma unroll
        for (int kk = 0; kk < KW; ++kk)
          xb[kk] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(xr, base, koff[kk], 0));
      };
      // one chunk: prefetch chunk j + 2 (always issued, clamped, so the wait count is static), MFMA
      auto body = [&](int j, bf16x8 (&cur)[KW], bf16x8 (&fill)[KW]) {
        load_chunk(c_begin + j + 2, fill);
        __builtin_amdgcn_sched_barrier(0);  // the prefetch leaves before this chunk's MFMAs, not after
        mfma_chunk(j, cur);
      };
      bf16x8 x0[KW], x1[KW], x2[KW];  // three chunk buffers in rotation: chunk j lives in x[j % 3]
      load_chunk(c_begin, x0);
      load_chunk(c_begin + 1, x1);
      __syncthreads();  // (the ring variant's prologue barrier: the epilogue waves count it)
      int j = 0;
      for (; j + 3 <= nc; j += 3) {
        body(j, x0, x2);
        body(j + 1, x1, x0);
        body(j + 2, x2, x1);
      }
      if (j < nc) body(j, x0, x2);
      if (j + 1 < nc) body(j + 1, x1, x0);
    }
    __syncthreads();  // the epilogue waves' last-chunk barrier
  } else {
    // ---------------- epilogue waves: item (pixel it % 16, group it / 16) of every chunk, IPT per thread
    constexpr int IPT = (NBLK + NE - 1) / NE, NI = 64 * NBLK;  // items per thread; items per chunk
    const int et = threadIdx.x - 64 * NWV;
    const __amdgpu_buffer_rsrc_t yr = ws_rsrc(a.y, (long long)(a.M / SS) * a.HPo * a.HPo * a.Cout * 2);
    const long long mbytes = (long long)(a.M / SS) * a.HPo * a.HPo * p.WPP * 4;
    const __amdgpu_buffer_rsrc_t mo = ws_rsrc(MODE == MODE_BIAS_RELU ? a.mbits_out : nullptr, mbytes);
    const __amdgpu_buffer_rsrc_t mi = ws_rsrc(MODE == MODE_MASKBITS ? a.mbits_in : nullptr, mbytes);
    auto out_pixel = [&](int m) -> int {
      const int bb = fdiv(m, a.divSS);
      const int rem = m - bb * SS;
      const int ii = fdiv(rem, a.divS);
      const int jj = rem - ii * a.S;
      return (bb * a.HPo + ii + a.Po) * a.HPo + jj + a.Po;
    };
    // per item: channels, bias and bitmask word are fixed for the workgroup's life
    int e_px[IPT], e_gi[IPT], e_wl[IPT], e_i[IPT], e_ch[IPT];
    f32x4 bias4[IPT];
#pragma unroll
    for (int q = 0; q < IPT; ++q) {
      const int it = et + 64 * NE * q < NI ? et + 64 * NE * q : NI - 1;  // (past NI: unused, see below)
      e_px[q] = it & 15;
      e_gi[q] = it >> 4;
      e_wl[q] = e_gi[q] / p.NB;
      e_i[q] = e_gi[q] - e_wl[q] * p.NB;
      e_ch[q] = ws_word_base(slice * p.WS + e_wl[q], p.BN) + 16 * e_i[q];
      bias4[q] = f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (MODE == MODE_BIAS_RELU) bias4[q] = *(const f32x4*)(a.bias + e_ch[q]);
    }
    // the dgrad's mask words, one chunk ahead (past the last pixel: out of range, read as 0)
    auto load_mw = [&](int c, uint32_t (&mw)[IPT]) {
#pragma unroll
      for (int q = 0; q < IPT; ++q) {
        const int m = c * 16 + e_px[q];
        const unsigned off = m < a.M ? (unsigned)(out_pixel(m) * p.WPP + slice * p.WS + e_wl[q]) * 4u : WS_OOB;
        mw[q] = __builtin_amdgcn_raw_buffer_load_b32(mi, off, 0, 0);
      }
    };
    uint32_t mw_cur[IPT], mw_next[IPT];
    if constexpr (MODE == MODE_MASKBITS) load_mw(c_begin, mw_cur);
    if constexpr (MODE == MODE_BIAS_RELU)
      for (int k = et; k < 32 * p.WS; k += 64 * NE) bitw[k] = 0u;
    __syncthreads();  // the MFMA waves' prologue
    // write chunk c's assembled bitmask words (lanes < 16 * WS; others and c < c_begin: dropped), clear them
    auto flush_bits = [&](int c, int buf) {
      const int k = et < 16 * p.WS ? et : 16 * p.WS - 1;
      const int m = c * 16 + (k & 15);
      uint32_t* bw = bitw + buf * 16 * p.WS + k;
      const bool ok = c >= c_begin && et < 16 * p.WS && m < a.M;
      const unsigned off = ok ? (unsigned)(out_pixel(m) * p.WPP + slice * p.WS + (k >> 4)) * 4u : WS_OOB;
      __builtin_amdgcn_raw_buffer_store_b32(*bw, mo, off, 0, 0);
      if (et < 16 * p.WS) *bw = 0u;
    };
    for (int j = 0; j < nc; ++j) {
      const int c = c_begin + j, buf = j & 1;
      if constexpr (MODE == MODE_MASKBITS) load_mw(c + 1, mw_next);
      __syncthreads();  // chunk j's partials are in LDS; chunk j - 1's bitmask ORs are done
      if constexpr (MODE == MODE_BIAS_RELU) flush_bits(c - 1, buf ^ 1);
      if constexpr (PROBE & 4) continue;
      const f32x4* pb = part + buf * PART;
#pragma unroll
      for (int q = 0; q < IPT; ++q) {
        if (IPT * NE > NBLK && et + 64 * NE * q >= NI) break;
        const int px = e_px[q], gi = e_gi[q];
        const int m = c * 16 + px;
        // partials added in wave order (deterministic), loaded 5 at a time
        const f32x4* src = pb + (gi >> 2) * 64 + 16 * (gi & 3) + px;
        f32x4 sum = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int q0 = 0; q0 < NWV; q0 += 5) {
          f32x4 v[5];
#pragma unroll
          for (int u = 0; u < 5; ++u)
            if (q0 + u < NWV) v[u] = src[(q0 + u) * NBLK * 64];
#pragma unroll
          for (int u = 0; u < 5; ++u)
            if (q0 + u < NWV) sum = (q0 + u == 0) ? v[u] : sum + v[u];
        }
        const uint32_t mw = MODE == MODE_MASKBITS ? mw_cur[q] >> (4 * e_i[q]) : 0u;
        bf16x4 o;
        uint32_t bits = 0u;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float x = sum[r];
          if constexpr (MODE == MODE_BIAS_RELU) x = fmaxf(x + bias4[q][r], 0.f);
          if constexpr (MODE == MODE_MASKBITS) x = ((mw >> r) & 1u) ? x : 0.f;
          o[r] = (__bf16)x;
          bits |= ((float)o[r] > 0.f ? 1u : 0u) << r;
        }
        const unsigned off = m < a.M ? (unsigned)(out_pixel(m) * a.Cout + e_ch[q]) * 2u : WS_OOB;
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(ws_u32x2, o), yr, off, 0, 0);
        if constexpr (MODE == MODE_BIAS_RELU)
          if (bits) atomicOr(bitw + buf * 16 * p.WS + e_wl[q] * 16 + px, bits << (4 * e_i[q]));
      }
      if constexpr (MODE == MODE_MASKBITS)
#pragma unroll
        for (int q = 0; q < IPT; ++q) mw_cur[q] = mw_next[q];
    }
    __syncthreads();  // the last chunk's bitmask ORs are done
    if constexpr (MODE == MODE_BIAS_RELU) flush_bits(c_end - 1, (nc - 1) & 1);
  }
}

// (NBLK, KW) of a conv: n-blocks per slice from the bitmask word geometry, K-steps per wave so that the
// waves (nsteps / KW <= 16) and the resident weight fragments (NBLK * KW * 4 VGPRs) fit; 0: not covered
static bool ws_shape(int Cout, int Cin, int K, int& nblk, int& kw, int& bn) {
  bn = Cout == 160 ? 160 : Cout % 192 == 0 ? 192 : Cout % 128 == 0 ? 128 : 64;
  const int nb = bn / 32;
  // words per slice: the fewest whole words whose groups fill whole 16-row n-blocks
  int ws = 1;
  while ((ws * nb) % 4) ++ws;
  nblk = ws * nb / 4;
  if (Cin % 32) return false;
  const int nsteps = K * K * (Cin / 32);
  // the instantiated (NBLK, KW, NWV = nsteps / KW) shapes (launch_conv_ws)
  struct Shape { int nblk, kw, nwv; };
  const Shape shapes[] = {{3, 6, 9}, {3, 5, 10}, {5, 3, 15}, {1, 6, 6}, {1, 6, 3}};
  for (const Shape& sh : shapes)
    if (sh.nblk == nblk && nsteps == sh.kw * sh.nwv) {
      kw = sh.kw;
      return true;
    }
  return false;
}

bool conv_ws_supported(int Cout, int Cin, int K) {
  int nblk, kw, bn;
  return ws_shape(Cout, Cin, K, nblk, kw, bn);
}

// Weight-stationary order of a standard (tap, Cout, Cin) bf16 pack: fragment (slice, wave, n-block, K-step)
// is one KB, lane l's 16 bytes at l * 16 -- rows / K of v_mfma_f32_16x16x32_bf16's A operand as
// conv_ws_kernel's MFMA waves hold it (row channel from the bitmask word geometry, see the kernel).
__global__ __launch_bounds__(256) void ws_pack_kernel(WsPackArgs args) {
  const WsPackJob& j = args.job[blockIdx.y];
  const int nb = j.bn / 32;
  const long units = (long)j.slices * j.nwv * j.nblk * j.kw * 64;
  for (long u = (long)blockIdx.x * 256 + threadIdx.x; u < units; u += (long)gridDim.x * 256) {
    const int lane = (int)(u & 63);
    long blk = u >> 6;
    const int kk = (int)(blk % j.kw);
    blk /= j.kw;
    const int b = (int)(blk % j.nblk);
    blk /= j.nblk;
    const int wave = (int)(blk % j.nwv);
    const int slice = (int)(blk / j.nwv);
    const int row = lane & 15, kq = lane >> 4;
    const int gi = 4 * b + (row >> 2);
    const int w = slice * j.ws + gi / nb;
    const int n = ws_word_base(w, j.bn) + 16 * (gi % nb) + (row & 3);
    const int s = wave * j.kw + kk, cs = j.Cin / 32;
    const int t = s / cs, c0 = (s - t * cs) * 32;
    *(bf16x8*)(j.dst + u * 8) = *(const bf16x8*)(j.src + ((size_t)t * j.Cout + n) * j.Cin + c0 + 8 * kq);
  }
}

void launch_ws_pack(const std::vector<WsPackJob>& jobs_in, hipStream_t st) {
  for (size_t i0 = 0; i0 < jobs_in.size(); i0 += kMaxWsPackJobs) {
    WsPackArgs args{};
    args.n = (int)std::min(jobs_in.size() - i0, (size_t)kMaxWsPackJobs);
    long most = 0;
    for (int i = 0; i < args.n; ++i) {
      WsPackJob j = jobs_in[i0 + i];
      if (!ws_shape(j.Cout, j.Cin, j.K, j.nblk, j.kw, j.bn))
        throw std::invalid_argument("ws_pack: no weight-stationary shape for Cout " + std::to_string(j.Cout) +
                                    " Cin " + std::to_string(j.Cin) + " K " + std::to_string(j.K));
      j.nwv = j.K * j.K * (j.Cin / 32) / j.kw;
      j.ws = 4 * j.nblk / (j.bn / 32);
      j.slices = (j.Cout / j.bn) * 8 / j.ws;
      args.job[i] = j;
      most = std::max(most, (long)j.slices * j.nwv * j.nblk * j.kw * 64);
    }
    const dim3 grid((unsigned)std::min((most + 255) / 256, 1024L), args.n);
    hipLaunchKernelGGL(ws_pack_kernel, grid, dim3(256), 0, st, args);
  }
}

// The input-row window of the ring: slots for the rows two consecutive chunks read (NR) and the most
// new rows one chunk adds (RM), from a scan of one period of the chunk / image pattern (16 c mod S^2)
struct RingGeo {
  int nr, rm;
};
static RingGeo ring_geometry(int S, int HPi, int offi, int K) {
  const int SS = S * S;
  auto row_of = [&](long m) { return (int)((m / SS) * HPi + (m % SS) / S + offi); };
  auto g0 = [&](long c) { return row_of(16 * c); };
  auto g1 = [&](long c) { return row_of(16 * c + 15) + K - 1; };
  RingGeo r{0, 0};
  for (long c = 0; c <= SS + 1; ++c) {
    r.nr = std::max(r.nr, g1(c + 1) - g0(c) + 1);
    r.rm = std::max(r.rm, g1(c + 1) - g1(c));
  }
  return r;
}

template <auto KERN>
static void ws_go(dim3 grid, dim3 block, int smem, hipStream_t st, const ConvFwdArgs& a, const WsParams& p) {
  static const hipError_t e =
      hipFuncSetAttribute((const void*)KERN, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hip_check(e, "hipFuncSetAttribute(max dynamic LDS)");
  hipLaunchKernelGGL(KERN, grid, block, smem, st, a, p);
}

template <int NBLK, int KW, int NWV, int NE, bool RING, int PROBE = 0>
static void launch_ws_t(const ConvFwdArgs& a, int mode, WsParams p, hipStream_t st) {
  // partials of two chunks + the bitmask words being assembled (+ the input-row ring)
  int smem = 2 * NWV * NBLK * 64 * 16 + 2 * 16 * p.WS * 4;
  if constexpr (RING) {
    static thread_local int key[4] = {-1, -1, -1, -1};
    static thread_local RingGeo geo;
    if (key[0] != a.S || key[1] != a.HPi || key[2] != a.offi || key[3] != a.K) {
      geo = ring_geometry(a.S, a.HPi, a.offi, a.K);
      key[0] = a.S, key[1] = a.HPi, key[2] = a.offi, key[3] = a.K;
    }
    p.PST = a.Cin * 2 + 16;
    p.RS = a.HPi * p.PST;
    p.NR = geo.nr;
    smem += p.NR * p.RS;
    if (geo.rm > 6 || a.HPi * a.Cin / 8 > 64 * NWV || smem > 160 * 1024)
      throw std::invalid_argument("conv_fwd tile 40: the input-row ring does not fit this geometry (S " +
                                  std::to_string(a.S) + ", Cin " + std::to_string(a.Cin) + ")");
  }
  const dim3 grid(8 * p.k * p.gper), block(64 * (NWV + NE));
  // one attribute call per kernel instantiation: the kernel is a template argument of ws_go, so every
  // mode has its own static (a generic lambda over the kernel pointer shares ONE instantiation -- and
  // one static -- between all modes, because their pointers have the same type)
  if constexpr (PROBE != 0) {
    if (mode != MODE_BIAS_RELU) throw std::invalid_argument("conv_fwd tiles 1000+: mode 0 only");
    ws_go<conv_ws_kernel<NBLK, KW, NWV, NE, MODE_BIAS_RELU, RING, PROBE>>(grid, block, smem, st, a, p);
    return;
  }
  if (mode == MODE_BIAS_RELU) ws_go<conv_ws_kernel<NBLK, KW, NWV, NE, MODE_BIAS_RELU, RING>>(grid, block, smem, st, a, p);
  else if (mode == MODE_MASKBITS) ws_go<conv_ws_kernel<NBLK, KW, NWV, NE, MODE_MASKBITS, RING>>(grid, block, smem, st, a, p);
  else if (mode == MODE_NONE) ws_go<conv_ws_kernel<NBLK, KW, NWV, NE, MODE_NONE, RING>>(grid, block, smem, st, a, p);
  else throw std::invalid_argument("conv_fwd tile 40: modes 0 (bias + ReLU), 2 (none) and 3 (bitmask dgrad)");
}

void launch_conv_ws(const ConvFwdArgs& a, int mode, int target_wgs, hipStream_t st, int probe) {
  int nblk, kw, bn;
  if (!ws_shape(a.Cout, a.Cin, a.K, nblk, kw, bn))
    throw std::invalid_argument("conv_fwd tile 40: unsupported shape Cout " + std::to_string(a.Cout) + " Cin " +
                                std::to_string(a.Cin) + " K " + std::to_string(a.K));
  if (a.y_bf8 || a.sk_ws) throw std::invalid_argument("conv_fwd tile 40: no e5m2 copy / split-K");
  if (a.M % (a.S * a.S)) throw std::invalid_argument("conv_fwd tile 40: M must be whole boards");
  WsParams p;
  p.BN = bn;
  p.NB = bn / 32;
  p.WS = 4 * nblk / p.NB;
  p.WPP = (a.Cout / bn) * 8;
  p.CS = a.Cin / 32;
  const int nsteps = a.K * a.K * p.CS;
  const int nwv = nsteps / kw;
  p.slices = p.WPP / p.WS;
  const int chunks = (a.M + 15) / 16;
  // ~one workgroup per CU (round-5 sweep, scripts/r5/ws_bench.py: 128 and 512 were slower at B <= 8)
  const int tgt = target_wgs > 0 ? target_wgs : 256;
  p.cpw = (chunks * p.slices + tgt - 1) / tgt;
  if (p.cpw < 1) p.cpw = 1;
  p.ngrp = (chunks + p.cpw - 1) / p.cpw;
  // slices per XCD: the fewest L2 fill bytes, 8 k / slices weight copies + slices / k activation copies
  const double wbytes = (double)a.K * a.K * a.Cin * a.Cout * 2;
  const double xbytes = (double)(a.M / (a.S * a.S)) * a.HPi * a.HPi * a.Cin * 2;
  p.k = 0;
  double best = 0;
  for (int k = 1; k <= p.slices; k *= 2) {
    if (p.slices % k || (8 * k) % p.slices) continue;
    const double cost = 8.0 * k * wbytes / p.slices + (double)p.slices / k * xbytes;
    if (p.k == 0 || cost < best) {
      p.k = k;
      best = cost;
    }
  }
  if (p.k == 0) throw std::invalid_argument("conv_fwd tile 40: no XCD placement for " + std::to_string(p.slices) + " slices");
  p.P = 8 * p.k / p.slices;
  p.gper = (p.ngrp + p.P - 1) / p.P;
  // (NBLK, KW, NWV, NE): 192-wide 3x3 (54 K-steps) and 5x5 over 64 channels (50), 160-wide 3x3 (45),
  // 128-wide 3x3 (36) and 64-wide 3x3 (18); NE epilogue waves (NWV + NE <= 16)
#ifdef AGK_KERNEL_LAB
  if (probe) {
    if (!(nblk == 3 && kw == 6 && nwv == 9)) throw std::invalid_argument("conv_fwd tiles 1000+: 192 x 192 3x3 only");
    switch (probe) {
      case 2: launch_ws_t<3, 6, 9, 3, true, 2>(a, mode, p, st); return;
      case 4: launch_ws_t<3, 6, 9, 3, true, 4>(a, mode, p, st); return;
      case 6: launch_ws_t<3, 6, 9, 3, true, 6>(a, mode, p, st); return;
      case 8: launch_ws_t<3, 6, 9, 3, true, 8>(a, mode, p, st); return;
      case 14: launch_ws_t<3, 6, 9, 3, true, 14>(a, mode, p, st); return;
      default: throw std::invalid_argument("conv_fwd tiles 1000 + probe: probes 2, 4, 6, 8, 14");
    }
  }
#else
  if (probe) throw std::invalid_argument("conv_fwd tiles 1000+: kernel-lab build only");
#endif
  if (nblk == 3 && kw == 6 && nwv == 9) launch_ws_t<3, 6, 9, 3, true>(a, mode, p, st);
  else if (nblk == 3 && kw == 5 && nwv == 10) launch_ws_t<3, 5, 10, 2, true>(a, mode, p, st);
  else if (nblk == 5 && kw == 3 && nwv == 15) launch_ws_t<5, 3, 15, 1, false>(a, mode, p, st);
  else if (nblk == 1 && kw == 6 && nwv == 6) launch_ws_t<1, 6, 6, 1, true>(a, mode, p, st);
  else if (nblk == 1 && kw == 6 && nwv == 3) launch_ws_t<1, 6, 3, 1, true>(a, mode, p, st);
  else throw std::invalid_argument("conv_fwd tile 40: no instantiation for this shape");
}

}  // namespace agk
