// Implicit-GEMM convolution for 19x19 boards on CDNA4 MFMA (gfx950).
//
// Activation layout: zero-bordered ("padded") NHWC bf16.  Element (b, i, j, c)
// of a tensor with padded side HP lives at ((b*HP + i)*HP + j)*C + c, the
// board interior is i, j in [P, P+S).  Borders are zero and never written, so
// every tap of a 'same' convolution is a plain load — no boundary branches.
//
// conv_fwd_kernel   D[n][m] = sum_{t,c} W_t[n][c] * X[m + shift_t][c]
//   M = boards*S*S output pixels, N = Cout, K = taps*Cin.  Workgroup tile
//   128(m) x BN(n), K-step = one tap x 64 channels.  Both operands are staged
//   global->LDS with global_load_lds_dwordx4 (the A rows are a per-lane gather:
//   row address of pixel m + tap offset); the 16-B chunks of each 128-B LDS row
//   are XOR-swizzled on the *source* address so the 16x16x32 bf16 MFMA fragment
//   reads (ds_read_b128) are bank-conflict free.  Double-buffered LDS.
//   The MFMA is issued "swapped" (A = weights, B = pixels) so each lane owns 4
//   consecutive output channels of one pixel: the epilogue (bias + ReLU, or the
//   ReLU-derivative mask for dgrad) stores 8 bytes per lane.
//   The same kernel computes dgrad with flipped/transposed packed weights.
//
// conv_wgrad_kernel dW_t[n][c] = sum_m dZ[m][n] * X[m + shift_t][c]
//   K = pixels (split over workgroups), tile 192(n) x 192(c) per workgroup for
//   one tap.  Tiles are staged as [16-channel block][32 pixels][16 ch] and the
//   pixel-contiguous MFMA operands are read with the gfx950 hardware transpose
//   read ds_read_b64_tr_b16.  The k (pixel) order inside a K-step is permuted
//   identically for both operands so that each 32-lane half reads 8 distinct
//   contiguous rows (conflict free).  Partial sums go to a per-split fp32 slab
//   that conv_wgrad_reduce_kernel sums deterministically into the OIHW fp32
//   gradient (and the bias gradient, accumulated by the tap-0 workgroups).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <numeric>

#include "common.h"
#include "kernels.h"

namespace agk {

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
        *(bf16x4*)(a.y + ooff[j] + i * 16) = o;
      }
      if constexpr (MODE == MODE_BIAS_RELU)
        if (a.mbits_out) a.mbits_out[(size_t)pix[j] * mwords + mslot] = bits;
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

// ----------------------------------------------------------------- forward
template <int NB, int MB, int MODE>
struct ConvEpilogue32;

template <int BN, int MODE, int BM, int MBW, bool EPF = true, bool PIPE = true, bool M32 = false, bool ILV = false>
__global__ __launch_bounds__(BM / MBW * 8, 1) void conv_fwd_kernel(ConvFwdArgs a) {
  // (BM / (16 MBW)) x 2 waves; each wave owns a 16*MBW (m) x BN/2 (n) output tile
  constexpr int NW = BM / (16 * MBW) * 2;  // waves per workgroup
  constexpr int NB = BN / 32;  // 16-wide n blocks per wave (a wave covers BN/2 channels)
  constexpr int MB = MBW;      // 16-wide m blocks per wave
  constexpr int A_BYTES = BM * 128;
  constexpr int B_BYTES = BN * 128;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int A_ROWS_PW = BM / NW;   // pixel rows staged per wave
  constexpr int A_INSTR = A_ROWS_PW / 8;
  constexpr int B_ROWS_PW = BN / NW;   // weight rows staged per wave
  constexpr int B_INSTR = B_ROWS_PW / 8;  // glds instructions per wave for the weight tile
  static_assert(B_ROWS_PW % 8 == 0 && A_ROWS_PW % 8 == 0, "rows per wave must be multiples of 8");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int lane = threadIdx.x & 63;
  const int wave = wave_id();
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int SS = a.S * a.S;
  const int CC = a.Cin >> 6;  // 64-channel chunks
  const int nK = a.K * a.K * CC;

  // --- staging addresses (element offsets)
  int arow[A_INSTR];
#pragma unroll
  for (int i = 0; i < A_INSTR; ++i) {
    const int r = wave * A_ROWS_PW + i * 8 + (lane >> 3);
    int m = m0 + r;
    m = m < a.M ? m : a.M - 1;
    const int b = fdiv(m, a.divSS);
    const int rem = m - b * SS;
    const int ii = fdiv(rem, a.divS);
    const int jj = rem - ii * a.S;
    const int logical = (lane & 7) ^ ((r >> 1) & 7);
    arow[i] = ((b * a.HPi + ii + a.offi) * a.HPi + jj + a.offi) * a.Cin + logical * 8;
  }
  int brow[B_INSTR];
#pragma unroll
  for (int i = 0; i < B_INSTR; ++i) {
    const int r = wave * B_ROWS_PW + i * 8 + (lane >> 3);
    const int logical = (lane & 7) ^ ((r >> 1) & 7);
    brow[i] = (n0 + r) * a.Cin + logical * 8;
  }
  const size_t wtap = (size_t)a.Cout * a.Cin;

  // staging cursor over (tap, 64-channel chunk), advanced incrementally with
  // scalar adds (no per-step integer divisions)
  int st_c0 = 0, st_kw = 0, st_a = 0;
  size_t st_w = 0;
  auto stage = [&](int buf) {
    char* base = smem + buf * STAGE;
#pragma unroll
    for (int i = 0; i < A_INSTR; ++i) glds16(a.x + arow[i] + st_a + st_c0, base + (wave * A_ROWS_PW + i * 8) * 128);
    const __bf16* wt = a.w + st_w + st_c0;
#pragma unroll
    for (int i = 0; i < B_INSTR; ++i) glds16(wt + brow[i], base + A_BYTES + (wave * B_ROWS_PW + i * 8) * 128);
    // branch-free cursor advance (selects), so a caller can interleave the
    // DMA with MFMAs inside one basic block
    st_c0 += 64;
    const bool wrap = st_c0 == a.Cin;
    st_c0 = wrap ? 0 : st_c0;
    st_w += wrap ? wtap : 0;
    st_kw += wrap ? 1 : 0;
    const bool wrap2 = st_kw == a.K;
    st_kw = wrap2 ? 0 : st_kw;
    st_a += (wrap ? a.Cin : 0) + (wrap2 ? (a.HPi - a.K) * a.Cin : 0);
  };

  f32x4 acc[NB][MB];
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int j = 0; j < MB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment read offsets: row*128 + (chunk ^ swz)*16, swz = ((row>>1)&7) = (lane&15)>>1
  const int swz = (lane & 15) >> 1;
  const int xrow0 = (wm * 16 * MB + (lane & 15)) * 128;
  const int wrow0 = A_BYTES + (wn * (BN / 2) + (lane & 15)) * 128;

  auto read_frags = [&](const char* base, int kk, bf16x8 (&xf)[MB], bf16x8 (&wf)[NB]) {
    const int choff = (((kk << 2) + (lane >> 4)) ^ swz) << 4;
#pragma unroll
    for (int j = 0; j < MB; ++j) xf[j] = *(const bf16x8*)(base + xrow0 + j * 16 * 128 + choff);
#pragma unroll
    for (int i = 0; i < NB; ++i) wf[i] = *(const bf16x8*)(base + wrow0 + i * 16 * 128 + choff);
  };
  auto mfmas = [&](const bf16x8 (&xf)[MB], const bf16x8 (&wf)[NB]) {
#pragma unroll
    for (int i = 0; i < NB; ++i)
#pragma unroll
      for (int j = 0; j < MB; ++j) acc[i][j] = mfma16x16x32(wf[i], xf[j], acc[i][j]);
  };

  // software pipeline: the first half (k 0..31) of step ks+1 is read right
  // after the barrier that publishes it, so its LDS latency hides under the
  // staging issue and the second-half reads of the next iteration.
  bf16x8 xa[MB], wa[NB], xb[MB], wb[NB];
  const int ep_mrow = m0 + wm * 16 * MB + (lane & 15);
  const int ep_nbase = n0 + wn * (BN / 2) + ((lane >> 4) << 2);
  ConvEpilogue<NB, MB, MODE> ep;
  const int ep_at = EPF ? (nK > 2 ? nK - 2 : 0) : nK - 1;
  stage(0);
  wait_vmcnt0();
  __syncthreads();
  if constexpr (M32) {
    // v_mfma_f32_32x32x16_bf16: an MFMA holds the SIMD's vector issue for 8 of
    // 32 cycles (8 of 16 for 16x16x32), leaving the co-resident wave more room
    // for its LDS reads and DMA issue.  Wave tile 16*MBW pixels x BN/2 channels
    // as (MBW/2) x (BN/64) 32x32 tiles; epilogue in the 32x32 C/D layout.
    constexpr int NB2 = BN / 64, MB2 = MBW / 2;
    static_assert(MBW % 2 == 0 && BN % 64 == 0, "32x32 tiles");
    f32x16 acc2[NB2][MB2];
#pragma unroll
    for (int i = 0; i < NB2; ++i)
#pragma unroll
      for (int j = 0; j < MB2; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc2[i][j][e] = 0.f;
    const int h = lane >> 5;
    const int l31 = lane & 31;
    const int xr0 = wm * 16 * MB + l31;         // tile row of block 0 (blocks are 32-aligned)
    const int wr0 = wn * (BN / 2) + l31;
    const int sw = (l31 >> 1) & 7;               // (row >> 1) & 7 for every 32-aligned block
    for (int ks = 0; ks < nK; ++ks) {
      const int cur = ks & 1;
      const char* base = smem + cur * STAGE;
      if (ks + 1 < nK) stage(cur ^ 1);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 xf2[2][MB2], wf2[2][NB2];
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const int co = ((((2 * kk + s2) << 1) + h) ^ sw) << 4;
#pragma unroll
          for (int j = 0; j < MB2; ++j) xf2[s2][j] = *(const bf16x8*)(base + (xr0 + j * 32) * 128 + co);
#pragma unroll
          for (int i = 0; i < NB2; ++i) wf2[s2][i] = *(const bf16x8*)(base + A_BYTES + (wr0 + i * 32) * 128 + co);
        }
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
          for (int i = 0; i < NB2; ++i)
#pragma unroll
            for (int j = 0; j < MB2; ++j)
              acc2[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf2[s2][i], xf2[s2][j], acc2[i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      }
      wait_vmcnt0();
      __syncthreads();
    }
    ConvEpilogue32<NB2, MB2, MODE> ep2;
    ep2.load(a, m0 + wm * 16 * MB + l31, n0 + wn * (BN / 2), wn);
    ep2.store(a, acc2, m0 + wm * 16 * MB + l31);
    return;
  }
  if constexpr (!PIPE && ILV) {
    // The 2-buffer loop issues the next stage's LDS-DMA as one burst at the top
    // of every step; with both waves of a SIMD in lockstep the matrix pipe
    // idles while they wait on DMA issue.  Here the burst is spread through
    // the first k-half's MFMAs (one DMA piece per MPD MFMAs, order pinned with
    // sched_barrier) so DMA issue overlaps matrix work.
    constexpr int NDMA = A_INSTR + B_INSTR;
    constexpr int NMF = NB * MB;
    constexpr int MPD = NMF / (NDMA + 1);
    auto mfma_range = [&](int f0, int f1) {
#pragma unroll
      for (int f = 0; f < NMF; ++f)
        if (f >= f0 && f < f1) acc[f / MB][f % MB] = mfma16x16x32(wa[f / MB], xa[f % MB], acc[f / MB][f % MB]);
    };
    for (int ks = 0; ks < nK; ++ks) {
      const int cur = ks & 1;
      const char* base = smem + cur * STAGE;
      const bool more = ks + 1 < nK;
      read_frags(base, 0, xa, wa);
      char* nb = smem + (cur ^ 1) * STAGE;
      const __bf16* wt = a.w + st_w + st_c0;
      const __bf16* xs = a.x + st_a + st_c0;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int d = 0; d < NDMA; ++d) {
        mfma_range(d * MPD, (d + 1) * MPD);
        __builtin_amdgcn_sched_barrier(0);
        if (more) {
          if (d < A_INSTR) glds16(xs + arow[d], nb + (wave * A_ROWS_PW + d * 8) * 128);
          else glds16(wt + brow[d - A_INSTR], nb + A_BYTES + (wave * B_ROWS_PW + (d - A_INSTR) * 8) * 128);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      mfma_range(NDMA * MPD, NMF);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      // advance the staging cursor (branch-free)
      st_c0 += 64;
      const bool wrap = st_c0 == a.Cin;
      st_c0 = wrap ? 0 : st_c0;
      st_w += wrap ? wtap : 0;
      st_kw += wrap ? 1 : 0;
      const bool wrap2 = st_kw == a.K;
      st_kw = wrap2 ? 0 : st_kw;
      st_a += (wrap ? a.Cin : 0) + (wrap2 ? (a.HPi - a.K) * a.Cin : 0);
      read_frags(base, 1, xa, wa);
      __builtin_amdgcn_s_setprio(1);
      mfmas(xa, wa);
      __builtin_amdgcn_s_setprio(0);
      wait_vmcnt0();
      __syncthreads();
    }
    ep.load(a, ep_mrow, ep_nbase, wn);
    ep.store(a, acc, ep_mrow);
    return;
  }
  if constexpr (!PIPE) {  // one fragment set (large wave tiles): read, then MFMA, per k-half
    for (int ks = 0; ks < nK; ++ks) {
      const int cur = ks & 1;
      const char* base = smem + cur * STAGE;
      if (ks + 1 < nK) stage(cur ^ 1);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        read_frags(base, kk, xa, wa);
        __builtin_amdgcn_s_setprio(1);
        mfmas(xa, wa);
        __builtin_amdgcn_s_setprio(0);
      }
      wait_vmcnt0();
      __syncthreads();
    }
    ep.load(a, ep_mrow, ep_nbase, wn);
    ep.store(a, acc, ep_mrow);
    return;
  }
  read_frags(smem, 0, xa, wa);
  for (int ks = 0; ks < nK; ++ks) {
    const int cur = ks & 1;
    const char* base = smem + cur * STAGE;
    if (ks + 1 < nK) stage(cur ^ 1);
    if (ks == ep_at) ep.load(a, ep_mrow, ep_nbase, wn);  // epilogue operands ride along with the last stages
    read_frags(base, 1, xb, wb);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    mfmas(xa, wa);
    mfmas(xb, wb);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    wait_vmcnt0();
    __syncthreads();
    if (ks + 1 < nK) read_frags(base + (cur ^ 1) * STAGE - cur * STAGE, 0, xa, wa);
  }

  // --- epilogue: lane owns channels n..n+3 of pixel m for every (i, j) block
  ep.store(a, acc, ep_mrow);
}

// ------------------------------------------------------ forward, halo variant
// 3x3 convolutions whose input and output share the padded geometry (all
// layers but the first): M runs over *padded* output positions, so tap t reads
// input row q + off_t with a constant off_t = (kh-1)*HP + (kw-1).  A workgroup
// owns 256 consecutive positions; the input rows [q0-HP-1, q0+256+HP+1) of one
// 64-channel chunk are staged ONCE into LDS (the halo) and reused by all 9
// taps, so per K-step only the 24 KB weight tile streams (3-deep ring, counted
// vmcnt, raw s_barrier so the next loads stay in flight across barriers).
// Border positions are computed (18% extra MFMA at S=19) and not stored.
constexpr int HALO_BM = 256;
constexpr int HALO_ROWS = 320;      // >= 256 + 2*(HP+1) for S <= 19, 40 x 1 KB pieces
constexpr int HALO_PW = HALO_ROWS / 8 / 8;  // glds pieces per wave (8 waves)

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

template <int BN, int MODE>
__global__ __launch_bounds__(512, 1) void conv_fwd_halo_kernel(ConvFwdArgs a) {
  constexpr int NB = BN / 32;           // 16-wide n blocks per wave (wave covers BN/2)
  constexpr int MB = 4;                 // wave covers 64 positions
  constexpr int W_BYTES = BN * 128;     // one (tap, 64-ch chunk) weight tile
  constexpr int H_BYTES = HALO_ROWS * 128;
  constexpr int NW_PW = BN / 64;        // weight glds pieces per wave
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const hbuf = smem;                      // 2 x H_BYTES
  char* const wbuf = smem + 2 * H_BYTES;        // 3 x W_BYTES

  const int lane = threadIdx.x & 63;
  const int wave = wave_id();
  const int wm = wave >> 1, wn = wave & 1;
  const int q0 = blockIdx.x * HALO_BM;
  const int n0 = blockIdx.y * BN;
  const int HP = a.HPo;
  const int G = HP + 1;                 // max |tap offset|
  const int Q = a.M;                    // number of padded positions (B * HP * HP)
  const int CC = a.Cin >> 6;
  const int nK = 9 * CC;

  // halo staging addresses: this lane's rows for each of its HALO_PW pieces
  int hrow[HALO_PW];
#pragma unroll
  for (int i = 0; i < HALO_PW; ++i) {
    const int r = (wave * HALO_PW + i) * 8 + (lane >> 3);
    int q = q0 - G + r;
    q = q < 0 ? 0 : (q >= Q ? Q - 1 : q);
    const int logical = (lane & 7) ^ ((r >> 1) & 7);
    hrow[i] = q * a.Cin + logical * 8;
  }
  int wrow[NW_PW];
#pragma unroll
  for (int i = 0; i < NW_PW; ++i) {
    const int r = (wave * NW_PW + i) * 8 + (lane >> 3);
    const int logical = (lane & 7) ^ ((r >> 1) & 7);
    wrow[i] = (n0 + r) * a.Cin + logical * 8;
  }
  const size_t wtap = (size_t)a.Cout * a.Cin;
  auto stage_halo = [&](int c, int buf) {
    char* base = hbuf + buf * H_BYTES;
#pragma unroll
    for (int i = 0; i < HALO_PW; ++i) glds16(a.x + hrow[i] + (c << 6), base + (wave * HALO_PW + i) * 1024);
  };
  auto stage_w = [&](int ks, int slot) {
    const int c = ks / 9;
    const int t = ks - c * 9;
    const __bf16* wt = a.w + (size_t)t * wtap + (c << 6);
    char* base = wbuf + slot * W_BYTES;
#pragma unroll
    for (int i = 0; i < NW_PW; ++i) glds16(wt + wrow[i], base + (wave * NW_PW + i) * 1024);
  };

  f32x4 acc[NB][MB];
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int j = 0; j < MB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int wr0 = (wn * (BN / 2) + (lane & 15)) * 128;
  const int wswz = (lane & 15) >> 1;

  stage_halo(0, 0);
  stage_w(0, 0);
  if (nK > 1) stage_w(1, 1);
  wait_vmcnt0();
  __syncthreads();

  for (int ks = 0; ks < nK; ++ks) {
    const int c = ks / 9;
    const int t = ks - c * 9;
    const bool issue_halo = (t == 4) && (c + 1 < CC);
    const bool issue_w = ks + 2 < nK;
    if (issue_halo) stage_halo(c + 1, (c + 1) & 1);
    if (issue_w) stage_w(ks + 2, (ks + 2) % 3);
    const char* hb = hbuf + (c & 1) * H_BYTES;
    const char* wb = wbuf + (ks % 3) * W_BYTES;
    const int kh = t / 3, kw = t - (t / 3) * 3;
    const int rbase = wm * 64 + (lane & 15) + G + (kh - 1) * HP + (kw - 1);
    const int xswz = (rbase >> 1) & 7;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ch = (kk << 2) + (lane >> 4);
      bf16x8 xf[MB], wf[NB];
#pragma unroll
      for (int j = 0; j < MB; ++j) xf[j] = *(const bf16x8*)(hb + (rbase + j * 16) * 128 + ((ch ^ xswz) << 4));
#pragma unroll
      for (int i = 0; i < NB; ++i) wf[i] = *(const bf16x8*)(wb + wr0 + i * 16 * 128 + ((ch ^ wswz) << 4));
#pragma unroll
      for (int i = 0; i < NB; ++i)
#pragma unroll
        for (int j = 0; j < MB; ++j) acc[i][j] = mfma16x16x32(wf[i], xf[j], acc[i][j]);
    }
    // the next K-step needs W(ks+1) (and the halo if a new chunk starts); the
    // loads issued this iteration may stay in flight across the barrier
    if (issue_w && issue_halo) vmcnt_wait<NW_PW + HALO_PW>();
    else if (issue_w) vmcnt_wait<NW_PW>();
    else if (issue_halo) vmcnt_wait<HALO_PW>();
    else vmcnt_wait<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }

  // --- epilogue: skip border positions (they must stay zero)
  const int nbase = n0 + wn * (BN / 2) + ((lane >> 4) << 2);
#pragma unroll
  for (int j = 0; j < MB; ++j) {
    const int q = q0 + wm * 64 + j * 16 + (lane & 15);
    if (q >= Q) continue;
    const int b = fdiv(q, a.divSS);       // divSS = HP*HP here
    const int rem = q - b * HP * HP;
    const int ii = fdiv(rem, a.divS);     // divS = HP here
    const int jj = rem - ii * HP;
    if (ii < a.Po || ii >= a.Po + a.S || jj < a.Po || jj >= a.Po + a.S) continue;
    const size_t ooff = (size_t)q * a.Cout;
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int n = nbase + i * 16;
      f32x4 v = acc[i][j];
      if constexpr (MODE == MODE_BIAS_RELU) {
        const f32x4 bb = *(const f32x4*)(a.bias + n);
        v[0] = fmaxf(v[0] + bb[0], 0.f);
        v[1] = fmaxf(v[1] + bb[1], 0.f);
        v[2] = fmaxf(v[2] + bb[2], 0.f);
        v[3] = fmaxf(v[3] + bb[3], 0.f);
      } else if constexpr (MODE == MODE_MASK) {
        const bf16x4 mk = *(const bf16x4*)(a.mask + ooff + n);
        v[0] = (float)mk[0] > 0.f ? v[0] : 0.f;
        v[1] = (float)mk[1] > 0.f ? v[1] : 0.f;
        v[2] = (float)mk[2] > 0.f ? v[2] : 0.f;
        v[3] = (float)mk[3] > 0.f ? v[3] : 0.f;
      }
      bf16x4 o;
      o[0] = (__bf16)v[0];
      o[1] = (__bf16)v[1];
      o[2] = (__bf16)v[2];
      o[3] = (__bf16)v[3];
      *(bf16x4*)(a.y + ooff + n) = o;
    }
  }
}


// ------------------------------------------------------ forward, ring variant
// Same gather/implicit-GEMM math as conv_fwd_kernel, restructured so the
// global->LDS DMA stays in flight across barriers (the 2-buffer kernel's
// __syncthreads() drains vmcnt every K-step):
//   * K-step = one tap x 32 channels; A = 256 pixel rows x 64 B (16 KB),
//     B = BN weight rows x 64 B; 4 LDS slots (112 KB at BN = 192);
//   * loads run 3 steps ahead: at step ks the wave waits (counted vmcnt) only
//     for its own pieces of step ks+1, passes a raw s_barrier, issues step
//     ks+3 into the slot freed by step ks-1, reads step ks+1's fragments and
//     only then issues step ks's 24 MFMAs, so the LDS latency hides under them;
//   * 64-B rows swizzled phys = chunk ^ (((row >> 2) & 1) << 1) (conflict-free
//     for the ds_read_b128 lane groups), applied on the DMA source address.
constexpr int RING_BM = 256;
constexpr int RING_SLOTS = 4;

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

template <int BN, int MODE>
__global__ __launch_bounds__(512, 1) void conv_fwd_ring_kernel(ConvFwdArgs a) {
  constexpr int NB = BN / 32;  // 16-wide n blocks per wave (wave covers BN/2 channels)
  constexpr int MB = 4;        // 16-wide m blocks per wave (wave covers 64 pixels)
  constexpr int A_BYTES = RING_BM * 64;
  constexpr int SLOT = A_BYTES + BN * 64;
  constexpr int BPIECES = BN / 16;  // 1 KB DMA pieces of the weight tile
  constexpr int BP_MAX = (BPIECES + 7) / 8;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int lane = threadIdx.x & 63;
  const int wave = wave_id();
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.x * RING_BM;
  const int n0 = blockIdx.y * BN;
  const int SS = a.S * a.S;
  const int CC2 = a.Cin >> 5;  // 32-channel chunks
  const int nK = a.K * a.K * CC2;

  // A pieces: wave w stages rows [16w, 16w+16) and [16(w+8), ...); lane -> row lane/4, 16-B chunk lane%4
  int arow[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = 16 * (wave + 8 * i) + (lane >> 2);
    int m = m0 + r;
    m = m < a.M ? m : a.M - 1;
    const int b = fdiv(m, a.divSS);
    const int rem = m - b * SS;
    const int ii = fdiv(rem, a.divS);
    const int jj = rem - ii * a.S;
    const int logical = (lane & 3) ^ (((r >> 2) & 1) << 1);
    arow[i] = ((b * a.HPi + ii + a.offi) * a.HPi + jj + a.offi) * a.Cin + logical * 8;
  }
  const int nbp = BPIECES / 8 + (wave < (BPIECES % 8) ? 1 : 0);  // wave-uniform
  int brow[BP_MAX];
#pragma unroll
  for (int i = 0; i < BP_MAX; ++i) {
    const int r = 16 * (wave + 8 * i) + (lane >> 2);
    const int logical = (lane & 3) ^ (((r >> 2) & 1) << 1);
    brow[i] = (n0 + (r < BN ? r : 0)) * a.Cin + logical * 8;
  }
  const int P = 2 + nbp;  // DMA pieces this wave issues per K-step
  const size_t wtap = (size_t)a.Cout * a.Cin;

  auto issue = [&](int ks) {
    const int t = ks / CC2;
    const int c = ks - t * CC2;
    const int kh = t / a.K;
    const int kw = t - kh * a.K;
    const int toff = (kh * a.HPi + kw) * a.Cin + (c << 5);
    char* base = smem + (ks % RING_SLOTS) * SLOT;
    glds16(a.x + arow[0] + toff, base + wave * 1024);
    glds16(a.x + arow[1] + toff, base + (wave + 8) * 1024);
    const __bf16* wt = a.w + (size_t)t * wtap + (c << 5);
#pragma unroll
    for (int i = 0; i < BP_MAX; ++i)
      if (i < nbp) glds16(wt + brow[i], base + A_BYTES + (wave + 8 * i) * 1024);
  };

  f32x4 acc[NB][MB];
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int j = 0; j < MB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int r15 = lane & 15;
  const int pch = (lane >> 4) ^ (((r15 >> 2) & 1) << 1);
  const int xoff = (wm * 64 + r15) * 64 + pch * 16;
  const int woff = A_BYTES + (wn * (BN / 2) + r15) * 64 + pch * 16;
  auto read_frags = [&](int ks, bf16x8 (&xf)[MB], bf16x8 (&wf)[NB]) {
    const char* base = smem + (ks % RING_SLOTS) * SLOT;
#pragma unroll
    for (int j = 0; j < MB; ++j) xf[j] = *(const bf16x8*)(base + xoff + j * 16 * 64);
#pragma unroll
    for (int i = 0; i < NB; ++i) wf[i] = *(const bf16x8*)(base + woff + i * 16 * 64);
  };
  auto mfmas = [&](const bf16x8 (&xf)[MB], const bf16x8 (&wf)[NB], int i0, int i1) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = i0; i < i1; ++i)
#pragma unroll
      for (int j = 0; j < MB; ++j) acc[i][j] = mfma16x16x32(wf[i], xf[j], acc[i][j]);
    __builtin_amdgcn_s_setprio(0);
  };
  // one K-step: publish step ks+1 (counted vmcnt + raw barrier), half of
  // step ks's MFMAs, refill the freed slot, read step ks+1's fragments, and
  // the other half of the MFMAs (covering the LDS read latency)
  auto step = [&](int ks, const bf16x8 (&xc)[MB], const bf16x8 (&wc)[NB], bf16x8 (&xn)[MB], bf16x8 (&wn_)[NB]) {
    const bool more = ks + 1 < nK;
    if (more) {
      vmcnt_wait_dyn(ks + 2 < nK ? P : 0);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
    }
    __builtin_amdgcn_sched_barrier(0);
    mfmas(xc, wc, 0, NB / 2);
    __builtin_amdgcn_sched_barrier(0);
    if (more) {
      if (ks + 3 < nK) issue(ks + 3);
      read_frags(ks + 1, xn, wn_);
    }
    __builtin_amdgcn_sched_barrier(0);
    mfmas(xc, wc, NB / 2, NB);
    __builtin_amdgcn_sched_barrier(0);
  };

  issue(0);
  if (nK > 1) issue(1);
  if (nK > 2) issue(2);
  vmcnt_wait_dyn(nK > 2 ? 2 * P : (nK > 1 ? P : 0));
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  bf16x8 xa[MB], wa[NB], xb[MB], wb[NB];
  read_frags(0, xa, wa);
  int ks = 0;
  for (; ks + 1 < nK; ks += 2) {
    step(ks, xa, wa, xb, wb);
    step(ks + 1, xb, wb, xa, wa);
  }
  if (ks < nK) step(ks, xa, wa, xb, wb);

  // --- epilogue
  conv_store_tile<NB, MB, MODE>(a, acc, m0 + wm * 64 + (lane & 15), n0 + wn * (BN / 2) + ((lane >> 4) << 2), wn);
}

// ------------------------------------------------- forward, ping-pong variant
// The 2-buffer kernels run both waves of a SIMD in lockstep: they read LDS
// fragments together, then fight for the one matrix pipe together, and every
// K-step ends in vmcnt(0) + barrier.  Here the 8 waves form two groups
// (waves 0-3 / 4-7, i.e. one wave of each group per SIMD) that run one
// barrier apart: while group 0 issues its 24 MFMAs, group 1 reads its next
// fragments and issues its share of the DMA, and vice versa, so the matrix
// pipe of every SIMD alternates between the two waves.
//   * tile 256 pixels x BN channels, K-step (phase) = one tap x 32 channels,
//     group g owns pixel rows [128g, 128g+128) (2x2 waves of 64 x BN/2);
//   * 4-slot LDS ring of 64-B rows (16 KB pixels + BN*64 B weights per slot),
//     the DMA runs 3 phases ahead; each wave retires its own pieces of phase
//     p+1 with a counted vmcnt during phase p, and the barrier that follows
//     publishes them to the other group (whose next read is >= 1 barrier later);
//   * a group's LDS reads complete (lgkmcnt(0)) before the barrier that ends
//     its read segment, so a slot refilled after that barrier is never read.
// Same packed operands, padded geometry and epilogue (bias + ReLU + ReLU'
// bitmask, or the dgrad mask) as conv_fwd_kernel.
constexpr int PP_BM = 256;
constexpr int PP_SLOTS = 4;

template <int BN, int MODE, bool STAMP = false>
__global__ __launch_bounds__(512, 1) void conv_fwd_pp_kernel(ConvFwdArgs a) {
  constexpr int NB = BN / 32;  // 16-wide n blocks per wave (wave covers BN/2 channels)
  constexpr int MB = 4;        // 16-wide m blocks per wave (64 pixels)
  constexpr int A_BYTES = PP_BM * 64;
  constexpr int SLOT = A_BYTES + BN * 64;
  constexpr int BPIECES = BN / 16;  // 1 KB DMA pieces of the weight tile
  constexpr int BP_MAX = (BPIECES + 7) / 8;
  constexpr int BP_MIN = BPIECES / 8;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int lane = threadIdx.x & 63;
  const int wave = wave_id();
  const int grp = wave >> 2;
  const int wm = grp * 2 + ((wave >> 1) & 1);  // 64-pixel row block of the tile
  const int wn = wave & 1;                     // channel half
  // XCD-aware bijective tile order: the 8 XCDs each get a contiguous tile range
  const int nwg = gridDim.x;
  const int xcd = blockIdx.x & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (blockIdx.x >> 3);
  const int m0 = tile * PP_BM;
  const int n0 = blockIdx.y * BN;
  const int SS = a.S * a.S;
  const int CC2 = a.Cin >> 5;  // 32-channel chunks
  const int nK = a.K * a.K * CC2;

  // A pieces: wave w stages rows [16w, 16w+16) and [16(w+8), ...); lane -> row lane/4, 16-B chunk lane%4
  int arow[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = 16 * (wave + 8 * i) + (lane >> 2);
    int m = m0 + r;
    m = m < a.M ? m : a.M - 1;
    const int b = fdiv(m, a.divSS);
    const int rem = m - b * SS;
    const int ii = fdiv(rem, a.divS);
    const int jj = rem - ii * a.S;
    const int logical = (lane & 3) ^ (((r >> 2) & 1) << 1);
    arow[i] = ((b * a.HPi + ii + a.offi) * a.HPi + jj + a.offi) * a.Cin + logical * 8;
  }
  const bool bfull = wave < (BPIECES & 7);  // this wave stages BP_MAX weight pieces (else BP_MIN)
  int brow[BP_MAX];
#pragma unroll
  for (int i = 0; i < BP_MAX; ++i) {
    const int r = 16 * (wave + 8 * i) + (lane >> 2);
    const int logical = (lane & 3) ^ (((r >> 2) & 1) << 1);
    brow[i] = (n0 + (r < BN ? r : 0)) * a.Cin + logical * 8;
  }
  const size_t wtap = (size_t)a.Cout * a.Cin;

  // staging cursor (tap kh/kw, chunk c) of the next phase to issue, advanced incrementally
  int is_c = 0, is_kw = 0, is_aoff = 0;
  size_t is_w = 0;
  int is_slot = 0;
  auto issue_next = [&]() {
    char* base = smem + is_slot * SLOT;
    glds16(a.x + arow[0] + is_aoff + (is_c << 5), base + wave * 1024);
    glds16(a.x + arow[1] + is_aoff + (is_c << 5), base + (wave + 8) * 1024);
    const __bf16* wt = a.w + is_w + (is_c << 5);
#pragma unroll
    for (int i = 0; i < BP_MAX; ++i)
      if (i < BP_MIN || bfull) glds16(wt + brow[i], base + A_BYTES + (wave + 8 * i) * 1024);
    is_slot = (is_slot + 1) & (PP_SLOTS - 1);
    if (++is_c == CC2) {
      is_c = 0;
      is_w += wtap;
      is_aoff += a.Cin;
      if (++is_kw == a.K) {
        is_kw = 0;
        is_aoff += (a.HPi - a.K) * a.Cin;
      }
    }
  };
  // retire the oldest phase in flight, leaving `ahead` younger phases' pieces outstanding
  auto retire = [&](int ahead) {
    if (BP_MAX == BP_MIN || bfull) {
      if (ahead >= 2) vmcnt_wait<2 * (2 + BP_MAX)>();
      else if (ahead == 1) vmcnt_wait<2 + BP_MAX>();
      else vmcnt_wait<0>();
    } else {
      if (ahead >= 2) vmcnt_wait<2 * (2 + BP_MIN)>();
      else if (ahead == 1) vmcnt_wait<2 + BP_MIN>();
      else vmcnt_wait<0>();
    }
  };

  f32x4 acc[NB][MB];
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int j = 0; j < MB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int r15 = lane & 15;
  const int pch = (lane >> 4) ^ (((r15 >> 2) & 1) << 1);
  const int xoff = (wm * 64 + r15) * 64 + pch * 16;
  const int woff = A_BYTES + (wn * (BN / 2) + r15) * 64 + pch * 16;
  const int ep_mrow = m0 + wm * 64 + r15;
  const int ep_nbase = n0 + wn * (BN / 2) + ((lane >> 4) << 2);
  ConvEpilogue<NB, MB, MODE> ep;
  const int ep_at = nK > 3 ? nK - 3 : 0;

  // prologue: phases 0..2 in flight, phase 0 retired and published
  const int npro = nK < 3 ? nK : 3;
  for (int p = 0; p < npro; ++p) issue_next();
  retire(npro - 1);
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  if (grp == 1) __builtin_amdgcn_s_barrier();  // stagger: group 1 runs one barrier behind
  __builtin_amdgcn_sched_barrier(0);

  bf16x8 xf[MB], wf[NB];
  // diagnostic build only: cycles per segment summed over the phases
  uint64_t st_sum[7] = {0, 0, 0, 0, 0, 0, 0};
  const uint64_t st_begin = STAMP ? __builtin_amdgcn_s_memtime() : 0;
  for (int p = 0; p < nK; ++p) {
    // ---- read segment (the partner group is in its MFMA segment)
    uint64_t ts[8];
    if constexpr (STAMP) ts[0] = __builtin_amdgcn_s_memtime();
    const char* base = smem + (p & (PP_SLOTS - 1)) * SLOT;
#pragma unroll
    for (int j = 0; j < MB; ++j) xf[j] = *(const bf16x8*)(base + xoff + j * 16 * 64);
#pragma unroll
    for (int i = 0; i < NB; ++i) wf[i] = *(const bf16x8*)(base + woff + i * 16 * 64);
    const bool more = p + 3 < nK;
    if constexpr (STAMP) {
      __builtin_amdgcn_sched_barrier(0);
      ts[7] = __builtin_amdgcn_s_memtime();
      __builtin_amdgcn_sched_barrier(0);
    }
    if (more) issue_next();
    if (p == ep_at) ep.load(a, ep_mrow, ep_nbase, wn);
    if constexpr (STAMP) __builtin_amdgcn_sched_barrier(0);
    if constexpr (STAMP) ts[1] = __builtin_amdgcn_s_memtime();
    retire(more ? 2 : (nK - 2 - p > 0 ? nK - 2 - p : 0));  // retire phase p+1
    if constexpr (STAMP) ts[2] = __builtin_amdgcn_s_memtime();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (STAMP) ts[3] = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (STAMP) ts[4] = __builtin_amdgcn_s_memtime();
    // ---- MFMA segment (the partner group reads)
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < NB; ++i)
#pragma unroll
      for (int j = 0; j < MB; ++j) acc[i][j] = mfma16x16x32(wf[i], xf[j], acc[i][j]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (STAMP) ts[5] = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (STAMP) {
      ts[6] = __builtin_amdgcn_s_memtime();
#pragma unroll
      for (int i = 0; i < 6; ++i) st_sum[i] += ts[i + 1] - ts[i];
      st_sum[6] += ts[7] - ts[0];
    }
  }
  if constexpr (STAMP) {
    if (lane == 0) {
      unsigned long long* d = a.dbg + ((size_t)blockIdx.x * 8 + wave) * 8;
#pragma unroll
      for (int i = 0; i < 6; ++i) d[i] = st_sum[i];
      d[6] = __builtin_amdgcn_s_memtime() - st_begin;
      d[7] = nK | (st_sum[6] << 16);
    }
  }
  if (grp == 0) __builtin_amdgcn_s_barrier();  // equal barrier counts
  ep.store(a, acc, ep_mrow);
}

static unsigned long long* g_conv_dbg = nullptr;
void set_conv_debug(unsigned long long* buf) { g_conv_dbg = buf; }

template <int BN, int MODE>
static void launch_fwd_pp(const ConvFwdArgs& a_in, hipStream_t st) {
  constexpr int smem = PP_SLOTS * (PP_BM * 64 + BN * 64);
  if constexpr (BN == 192 && MODE == MODE_BIAS_RELU) {
    if (g_conv_dbg) {  // diagnostic instantiation with segment stamps
      static bool attr_d = false;
      if (!attr_d) {
        hipFuncSetAttribute((const void*)conv_fwd_pp_kernel<BN, MODE, true>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, smem);
        attr_d = true;
      }
      ConvFwdArgs a = a_in;
      a.dbg = g_conv_dbg;
      dim3 grid((a.M + PP_BM - 1) / PP_BM, a.Cout / BN);
      hipLaunchKernelGGL((conv_fwd_pp_kernel<BN, MODE, true>), grid, dim3(512), smem, st, a);
      return;
    }
  }
  const ConvFwdArgs& a = a_in;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)conv_fwd_pp_kernel<BN, MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr = true;
  }
  dim3 grid((a.M + PP_BM - 1) / PP_BM, a.Cout / BN);
  hipLaunchKernelGGL((conv_fwd_pp_kernel<BN, MODE>), grid, dim3(512), smem, st, a);
}

template <int BN, int MODE>
static void launch_fwd_ring(const ConvFwdArgs& a, hipStream_t st) {
  constexpr int smem = RING_SLOTS * (RING_BM * 64 + BN * 64);
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)conv_fwd_ring_kernel<BN, MODE>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        smem);
    attr = true;
  }
  dim3 grid((a.M + RING_BM - 1) / RING_BM, a.Cout / BN);
  hipLaunchKernelGGL((conv_fwd_ring_kernel<BN, MODE>), grid, dim3(512), smem, st, a);
}

template <int BN, int MODE>
static void launch_fwd_halo(const ConvFwdArgs& a_in, hipStream_t st) {
  constexpr int smem = 2 * HALO_ROWS * 128 + 3 * BN * 128;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)conv_fwd_halo_kernel<BN, MODE>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        smem);
    attr = true;
  }
  ConvFwdArgs a = a_in;
  const int B = a.M / (a.S * a.S);
  a.M = B * a.HPo * a.HPo;  // padded positions
  a.divSS = make_fastdiv((uint32_t)(a.HPo * a.HPo));
  a.divS = make_fastdiv((uint32_t)a.HPo);
  dim3 grid((a.M + HALO_BM - 1) / HALO_BM, a.Cout / BN);
  hipLaunchKernelGGL((conv_fwd_halo_kernel<BN, MODE>), grid, dim3(512), smem, st, a);
}

static int g_fwd_bm = 0;  // 0 = auto

template <int BN, int MODE, int BM, int MBW, bool EPF = true, bool PIPE = true, bool M32 = false, bool ILV = false>
static void launch_fwd_bm(const ConvFwdArgs& a, hipStream_t st) {
  constexpr int smem = 2 * (BM * 128 + BN * 128);
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)conv_fwd_kernel<BN, MODE, BM, MBW, EPF, PIPE, M32, ILV>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr = true;
  }
  dim3 grid((a.M + BM - 1) / BM, a.Cout / BN);
  hipLaunchKernelGGL((conv_fwd_kernel<BN, MODE, BM, MBW, EPF, PIPE, M32, ILV>), grid, dim3(BM / MBW * 8), smem, st,
                     a);
}


// ------------------------------------------- forward, interior-halo variant
// The gather kernel re-fetches every input row once per tap (9x for 3x3).
// Here a workgroup stages, per 64-channel chunk, the contiguous range of
// padded input rows that its 256 interior pixels and all taps touch (the
// "halo", <= H2_ROWS rows) ONCE, then runs all K*K taps against it: the A
// fragments are gathered from LDS with per-lane row addresses (row = padded
// position of the pixel + tap offset), so only interior pixels are computed
// (no border waste, unlike conv_fwd_halo_kernel).  Per tap-step only the
// weight tile (24 KB at BN = 192) streams through a double buffer.
constexpr int H2_BM = 256;
constexpr int H2_ROWS = 384;  // 48 KB of 128-B rows per halo buffer
// compact halo of the halo + ping-pong kernel: 256 + 2*(S+1) pixel rows (S <= 23) + 8 zero rows
constexpr int HC_DATA = 320;
constexpr int HC_ROWS = HC_DATA + 8;

template <int BN, int MODE>
__global__ __launch_bounds__(512, 1) void conv_fwd_halo2_kernel(ConvFwdArgs a) {
  constexpr int NB = BN / 32;
  constexpr int MB = 4;
  constexpr int H_BYTES = H2_ROWS * 128;
  constexpr int W_BYTES = BN * 128;
  constexpr int B_INSTR = BN / 64;        // weight pieces per wave
  constexpr int H_PIECES = H2_ROWS / 8;   // 1-KB halo pieces per chunk
  constexpr int H_PW = H_PIECES / 8;      // per wave
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const hbuf = smem;                // 2 x H_BYTES
  char* const wbuf = smem + 2 * H_BYTES;  // 2 x W_BYTES

  const int lane = threadIdx.x & 63;
  const int wave = wave_id();
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.x * H2_BM;
  const int n0 = blockIdx.y * BN;
  const int SS = a.S * a.S;
  const int CC = a.Cin >> 6;
  const int T = a.K * a.K;
  const int HP = a.HPi;
  const int Pc = a.offi + a.K / 2;  // interior offset of the input (its pad)
  const int G = (a.K / 2) * (HP + 1);
  const int Q = a.M / SS * HP * HP;  // padded input positions

  auto qpos = [&](int m) {
    const int b = fdiv(m, a.divSS);
    const int rem = m - b * SS;
    const int ii = fdiv(rem, a.divS);
    const int jj = rem - ii * a.S;
    return (b * HP + ii + Pc) * HP + jj + Pc;
  };
  const int mlast = (m0 + H2_BM - 1 < a.M ? m0 + H2_BM - 1 : a.M - 1);
  const int qfirst = qpos(m0) - G;

  // halo staging: lane -> row 8*piece + lane/8, physical chunk lane%8
  int hsrc[H_PW];
#pragma unroll
  for (int i = 0; i < H_PW; ++i) {
    const int r = (wave * H_PW + i) * 8 + (lane >> 3);
    int q = qfirst + r;
    q = q < 0 ? 0 : (q >= Q ? Q - 1 : q);
    const int logical = (lane & 7) ^ ((r >> 1) & 7);
    hsrc[i] = q * a.Cin + logical * 8;
  }
  int brow[B_INSTR];
#pragma unroll
  for (int i = 0; i < B_INSTR; ++i) {
    const int r = wave * (BN / 8) + i * 8 + (lane >> 3);
    const int logical = (lane & 7) ^ ((r >> 1) & 7);
    brow[i] = (n0 + r) * a.Cin + logical * 8;
  }
  const size_t wtap = (size_t)a.Cout * a.Cin;
  auto stage_halo = [&](int c, int buf) {
    char* base = hbuf + buf * H_BYTES;
#pragma unroll
    for (int i = 0; i < H_PW; ++i) glds16(a.x + hsrc[i] + c * 64, base + (wave * H_PW + i) * 1024);
  };
  auto stage_w = [&](int t, int c, int buf) {
    const __bf16* wt = a.w + (size_t)t * wtap + c * 64;
    char* base = wbuf + buf * W_BYTES;
#pragma unroll
    for (int i = 0; i < B_INSTR; ++i) glds16(wt + brow[i], base + (wave * (BN / 8) + i * 8) * 128);
  };

  // per-lane halo-relative rows of this lane's pixel in each m block
  int qrel[MB];
#pragma unroll
  for (int j = 0; j < MB; ++j) {
    int m = m0 + wm * 64 + j * 16 + (lane & 15);
    m = m < a.M ? m : a.M - 1;
    qrel[j] = qpos(m) - qfirst;
  }
  f32x4 acc[NB][MB];
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int j = 0; j < MB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int swzw = (lane & 15) >> 1;
  const int wrow0 = (wn * (BN / 2) + (lane & 15)) * 128;
  const int ep_mrow = m0 + wm * 64 + (lane & 15);
  const int ep_nbase = n0 + wn * (BN / 2) + ((lane >> 4) << 2);
  ConvEpilogue<NB, MB, MODE> ep;

  const int nK = CC * T;
  stage_halo(0, 0);
  stage_w(0, 0, 0);
  wait_vmcnt0();
  __syncthreads();
  int c = 0, t = 0;
  for (int ks = 0; ks < nK; ++ks) {
    // prefetch the next weight tile (and, on a chunk's first tap, the next chunk's halo)
    const int tn = (t + 1 == T) ? 0 : t + 1;
    const int cn = (t + 1 == T) ? c + 1 : c;
    if (ks + 1 < nK) stage_w(tn, cn, (ks + 1) & 1);
    if (t == 0 && c + 1 < CC) stage_halo(c + 1, (c + 1) & 1);
    if (ks == (nK > 2 ? nK - 2 : 0)) ep.load(a, ep_mrow, ep_nbase, wn);
    const char* hb = hbuf + (c & 1) * H_BYTES;
    const char* wb = wbuf + (ks & 1) * W_BYTES;
    const int kh = t / a.K, kw = t - (t / a.K) * a.K;
    const int toff = (kh - a.K / 2) * HP + (kw - a.K / 2) + G;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ch = (kk << 2) + (lane >> 4);
      bf16x8 xf[MB], wf[NB];
#pragma unroll
      for (int j = 0; j < MB; ++j) {
        const int row = qrel[j] + toff - G;  // halo row of (pixel, tap)
        xf[j] = *(const bf16x8*)(hb + row * 128 + ((ch ^ ((row >> 1) & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < NB; ++i) wf[i] = *(const bf16x8*)(wb + wrow0 + i * 16 * 128 + ((ch ^ swzw) << 4));
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < NB; ++i)
#pragma unroll
        for (int j = 0; j < MB; ++j) acc[i][j] = mfma16x16x32(wf[i], xf[j], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
    }
    wait_vmcnt0();
    __syncthreads();
    t = tn;
    c = cn;
  }
  ep.store(a, acc, ep_mrow);
}

// ------------------------------------ forward, halo + ping-pong variant (3x3)
// The interior-halo staging of conv_fwd_halo2_kernel (per 64-channel chunk the
// padded input rows of the tile's 256 pixels and all 9 taps are staged ONCE,
// A fragments are gathered from LDS per tap) combined with the two-group
// ping-pong of conv_fwd_pp_kernel (waves 0-3 / 4-7 alternate between an LDS
// read segment and a 48-MFMA segment, one barrier apart).  Global traffic per
// MFMA is ~3x lower than the gather kernels: per K-step (tap x 64 channels)
// only the 24 KB weight tile streams, the 48 KB halo once per 9 steps.
// The loads are split by group so that every DMA is retired (own vmcnt)
// before a barrier that precedes its first reader in either group:
//   * group 0 loads the weights: W(p+1) is issued in its read segment of
//     step p into the slot W(p-1) used (both groups finished reading it one
//     barrier earlier) and retired at the end of its MFMA segment of step p;
//   * group 1 loads the next chunk's halo during steps 0..5 of a chunk and
//     retires it in step 7 (the halo buffer it overwrites was last read in
//     the previous chunk).
// LDS: 2 x 48 KB halo + 2 x BN*128 B weights (144 KB at BN = 192).
template <int BN, int MODE, bool STAMP = false>
__global__ __launch_bounds__(512, 1) void conv_fwd_hpp_kernel(ConvFwdArgs a) {
  // STAMP (diagnostic build): per-wave cycle sums of the loop segments into a.dbg
  uint64_t st_sum[8] = {0, 0, 0, 0, 0, 0, 0, 0}, ts[9];
#define HPP_STAMP(i)                          \
  if constexpr (STAMP) {                      \
    __builtin_amdgcn_sched_barrier(0);        \
    ts[i] = __builtin_amdgcn_s_memtime();     \
    __builtin_amdgcn_sched_barrier(0);        \
  }
  constexpr int NB = BN / 32;
  constexpr int MB = 4;
  constexpr int H_BYTES = HC_ROWS * 128;
  constexpr int W_BYTES = BN * 128;
  constexpr int WP = BN / 32;              // weight pieces per group-0 wave (BN/8 1-KB pieces over 4 waves)
  constexpr int H_PIECES = HC_DATA / 8;    // 1-KB halo pieces per chunk (40)
  constexpr int HP1 = H_PIECES / 4;        // per group-1 wave in steady state (10)
  constexpr int HP_STEP = 2;               // halo pieces a group-1 wave issues per step
  constexpr int T = 9;                     // 3x3 only
  static_assert(HP1 == 5 * HP_STEP && H_PIECES % 8 == 0, "halo pieces must be issued within steps 0..4");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const hbuf = smem;
  char* const wbuf = smem + 2 * H_BYTES;

  const int lane = threadIdx.x & 63;
  const int wave = wave_id();
  const int grp = wave >> 2;
  const int wq = wave & 3;
  const int wm = grp * 2 + ((wave >> 1) & 1);
  const int wn = wave & 1;
  const int nwg = gridDim.x;
  const int xcd = blockIdx.x & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (blockIdx.x >> 3);
  const int m0 = tile * H2_BM;
  const int n0 = blockIdx.y * BN;
  const int S = a.S;
  const int SS = S * S;
  const int CC = a.Cin >> 6;
  const int HP = a.HPi;
  const int Pc = a.offi + 1;
  const int G = S + 1;  // largest |tap shift| in the compact (unpadded) pixel index
  const int nK = CC * T;

  // Halo rows are COMPACT pixel indices (no padding): row r holds interior
  // pixel m0 - G + r, so the 16 pixels of an MFMA block read 16 consecutive
  // rows for every tap (the padded layout skips 2 rows at each board-row end,
  // which made 2-way bank conflicts unavoidable).  Taps that leave the board
  // read the zero rows [HC_DATA, HC_ROWS) instead.
  auto halo_piece = [&](int c, int k, int buf) {
    const int r = k * 8 + (lane >> 3);
    int m = m0 - G + r;
    m = m < 0 ? 0 : (m >= a.M ? a.M - 1 : m);
    const int b = fdiv(m, a.divSS);
    const int rem = m - b * SS;
    const int ii = fdiv(rem, a.divS);
    const int q = (b * HP + ii + Pc) * HP + (rem - ii * S) + Pc;
    const int logical = (lane & 7) ^ ((r >> 1) & 7);
    glds16(a.x + (size_t)q * a.Cin + c * 64 + logical * 8, hbuf + buf * H_BYTES + k * 1024);
  };
  // weight tile of step (t, c) into slot: group-0 wave wq stages rows [8(wq*WP+i), +8)
  int wrow[WP];
#pragma unroll
  for (int i = 0; i < WP; ++i) {
    const int r = (wq * WP + i) * 8 + (lane >> 3);
    wrow[i] = (n0 + r) * a.Cin + (((lane & 7) ^ ((r >> 1) & 7)) << 3);
  }
  const size_t wtap = (size_t)a.Cout * a.Cin;
  auto stage_w = [&](int t, int c, int slot) {
    const __bf16* wt = a.w + (size_t)t * wtap + c * 64;
#pragma unroll
    for (int i = 0; i < WP; ++i) glds16(wt + wrow[i], wbuf + slot * W_BYTES + (wq * WP + i) * 1024);
  };

  // Pixel order inside a 16-pixel MFMA block: lanes i = 0-3, 12-15 take the
  // even pixels and i = 4-11 the odd ones.  A ds_read_b128 lane group reads
  // rows i in {0-3, 12-15} at one 16-B chunk and i in {4-11} at the next, so
  // the two chunk sets sit on rows of opposite parity (opposite 128-B bank
  // halves) and the (row >> 1) swizzle keeps each set conflict-free for any
  // row alignment (the per-tap shifts make every alignment occur).
  const int li = lane & 15;
  const int pix16 = li < 4 ? 2 * li : (li < 12 ? 2 * (li - 4) + 1 : 2 * (li - 12) + 8);
  int prel[MB], px[MB], py[MB];
#pragma unroll
  for (int j = 0; j < MB; ++j) {
    int m = m0 + wm * 64 + j * 16 + pix16;
    m = m < a.M ? m : a.M - 1;
    const int b = fdiv(m, a.divSS);
    const int rem = m - b * SS;
    py[j] = fdiv(rem, a.divS);
    px[j] = rem - py[j] * S;
    prel[j] = m - m0 + G;
  }
  f32x4 acc[NB][MB];
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int j = 0; j < MB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int swzw = (lane & 15) >> 1;
  const int wrow0 = (wn * (BN / 2) + (lane & 15)) * 128;
  const int ep_mrow = m0 + wm * 64 + pix16;
  const int ep_nbase = n0 + wn * (BN / 2) + ((lane >> 4) << 2);
  ConvEpilogue<NB, MB, MODE> ep;
  const int ep_at = nK > 3 ? nK - 3 : 0;

  // prologue: zero rows of both halo buffers, chunk 0's halo by all waves, W(0) by group 0
  if (wave < 2) {
    const int zb = (HC_ROWS - HC_DATA) * 128;  // zero-row bytes per buffer
    for (int o = lane * 16; o < zb; o += 64 * 16)
      *(uint4*)(hbuf + wave * H_BYTES + HC_DATA * 128 + o) = make_uint4(0u, 0u, 0u, 0u);
  }
#pragma unroll
  for (int i = 0; i < H_PIECES / 8; ++i) halo_piece(0, wave * (H_PIECES / 8) + i, 0);
  if (grp == 0) stage_w(0, 0, 0);
  wait_vmcnt0();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  if (grp == 1) __builtin_amdgcn_s_barrier();  // stagger
  __builtin_amdgcn_sched_barrier(0);

  int c = 0, t = 0, kh = 0, kw = 0, wslot = 0;
  const uint64_t st_begin = STAMP ? __builtin_amdgcn_s_memtime() : 0;
  for (int p = 0; p < nK; ++p) {
    // ---- read segment
    HPP_STAMP(0);
    const char* hb = hbuf + (c & 1) * H_BYTES;
    const char* wb = wbuf + wslot * W_BYTES;
    const int toff = (kh - 1) * S + (kw - 1);
    int arow[MB];
#pragma unroll
    for (int j = 0; j < MB; ++j) {
      const bool ok = (unsigned)(py[j] + kh - 1) < (unsigned)S && (unsigned)(px[j] + kw - 1) < (unsigned)S;
      arow[j] = ok ? prel[j] + toff : HC_DATA;
    }
    bf16x8 xf[2][MB], wf[2][NB];
    auto read_half = [&](int kk) {
      const int ch = (kk << 2) + (lane >> 4);
#pragma unroll
      for (int j = 0; j < MB; ++j) {
        const int row = arow[j];
        xf[kk][j] = *(const bf16x8*)(hb + row * 128 + ((ch ^ ((row >> 1) & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < NB; ++i) wf[kk][i] = *(const bf16x8*)(wb + wrow0 + i * 16 * 128 + ((ch ^ swzw) << 4));
    };
    read_half(0);  // k 0..31 here; k 32..63 is read under the first half's MFMAs
    HPP_STAMP(1);
    // step cursor of p+1
    int tn = t + 1, cn = c, khn = kh, kwn = kw + 1;
    if (kwn == 3) { kwn = 0; ++khn; }
    if (tn == T) { tn = 0; ++cn; khn = 0; kwn = 0; }
    if (grp == 0) {
      if (p + 1 < nK) stage_w(tn, cn, wslot == 2 ? 0 : wslot + 1);
    } else if (c + 1 < CC) {
      if (t < 5) {
#pragma unroll
        for (int i = 0; i < HP_STEP; ++i) halo_piece(c + 1, wq * HP1 + t * HP_STEP + i, (c + 1) & 1);
      } else if (t == 7) {
        wait_vmcnt0();  // next chunk's halo landed (published by this step's barrier)
      }
    }
    if (p == ep_at) ep.load(a, ep_mrow, ep_nbase, wn);
    HPP_STAMP(2);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    HPP_STAMP(3);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    HPP_STAMP(4);
    // ---- MFMA segment: first half, with the second half's LDS reads interleaved
    __builtin_amdgcn_s_setprio(1);
    read_half(1);
#pragma unroll
    for (int i = 0; i < NB; ++i)
#pragma unroll
      for (int j = 0; j < MB; ++j) acc[i][j] = mfma16x16x32(wf[0][i], xf[0][j], acc[i][j]);
#pragma unroll
    for (int g = 0; g < MB + NB; ++g) {  // 1 ds_read per 2 MFMAs
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, NB * MB - 2 * (MB + NB), 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < NB; ++i)
#pragma unroll
      for (int j = 0; j < MB; ++j) acc[i][j] = mfma16x16x32(wf[1][i], xf[1][j], acc[i][j]);
    __builtin_amdgcn_s_setprio(0);
    HPP_STAMP(5);
    __builtin_amdgcn_sched_barrier(0);
    if (grp == 0) wait_vmcnt0();  // W(p+1) landed before the barrier that precedes its readers
    HPP_STAMP(6);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    HPP_STAMP(7);
    if constexpr (STAMP) {
#pragma unroll
      for (int i = 0; i < 7; ++i) st_sum[i] += ts[i + 1] - ts[i];
    }
    t = tn; c = cn; kh = khn; kw = kwn;
    wslot = wslot == 2 ? 0 : wslot + 1;
  }
  if constexpr (STAMP) {
    if (lane == 0) {
      unsigned long long* d = a.dbg + ((size_t)blockIdx.x * 8 + wave) * 8;
#pragma unroll
      for (int i = 0; i < 7; ++i) d[i] = st_sum[i];
      d[7] = __builtin_amdgcn_s_memtime() - st_begin;
    }
  }
#undef HPP_STAMP
  if (grp == 0) __builtin_amdgcn_s_barrier();
  ep.store(a, acc, ep_mrow);
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

// --------------------- forward, compact halo + ping-pong, 32x32x16 MFMA (3x3 / 5x5)
// Same schedule as conv_fwd_hpp_kernel (two wave groups one barrier apart,
// group 0 streams the weights through 3 slots, group 1 the next chunk's halo,
// half of each step's fragment reads under the previous half's MFMAs), but on
// v_mfma_f32_32x32x16_bf16: an MFMA holds the SIMD's vector issue for 8 of its
// 32 cycles instead of 8 of 16, which leaves the partner wave 3x the issue
// slots for its LDS reads, address math and DMA (the 16x16x32 form saturated
// the issue port: measured with conv_stamps.py).  Per wave 64 pixels x BN/2
// channels = 2 x (BN/64) MFMA tiles, 24 MFMAs per 64-channel step at BN=192.
// The compact halo (rows = unpadded pixel indices, zero rows for taps leaving
// the board) makes the 32 rows of a block contiguous: conflict-free reads.
constexpr int H32_DATA3 = 320;  // K=3: 256 + 2*(S+1) <= 320 rows, 40 one-KB pieces (10 per group-1 wave)
constexpr int H32_DATA5 = 344;  // K=5 (single 64-channel chunk): 256 + 4*(S+1) <= 344 rows

template <int BN, int MODE, int K, bool STAMP = false>
__global__ __launch_bounds__(512, 1) void conv_fwd_h32_kernel(ConvFwdArgs a) {
  uint64_t st_sum[8] = {0, 0, 0, 0, 0, 0, 0, 0}, ts[9];
#define H32_STAMP(i)                          \
  if constexpr (STAMP) {                      \
    __builtin_amdgcn_sched_barrier(0);        \
    ts[i] = __builtin_amdgcn_s_memtime();     \
    __builtin_amdgcn_sched_barrier(0);        \
  }
  constexpr int NB = BN / 64;  // 32-channel MFMA tiles per wave (wave covers BN/2)
  constexpr int MB = 2;        // 32-pixel MFMA tiles per wave
  constexpr int T = K * K;
  constexpr int HDATA = K == 3 ? H32_DATA3 : H32_DATA5;
  constexpr int HROWS = HDATA + 16;  // + 16 zero rows (a redirected lane keeps its bank slot)
  constexpr int NHBUF = K == 3 ? 2 : 1;
  constexpr int H_BYTES = HROWS * 128;
  constexpr int W_BYTES = BN * 128;
  constexpr int WP = BN / 64;          // weight pieces per wave (each group stages half of every tile)
  constexpr int H_PIECES = HDATA / 8;  // 1-KB halo pieces per chunk
  constexpr int HP1 = H_PIECES / 4;
  constexpr int HP_STEP = 2;
  static_assert(K == 5 || HP1 == 5 * HP_STEP, "K=3 halo pieces are issued in steps 0..4");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const hbuf = smem;
  char* const wbuf = smem + NHBUF * H_BYTES;

  const int lane = threadIdx.x & 63;
  const int h = lane >> 5;
  const int wave = wave_id();
  const int grp = wave >> 2;
  const int wq = wave & 3;
  const int wm = grp * 2 + ((wave >> 1) & 1);
  const int wn = wave & 1;
  const int nwg = gridDim.x;
  const int xcd = blockIdx.x & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (blockIdx.x >> 3);
  const int m0 = tile * H2_BM;
  const int n0 = blockIdx.y * BN;
  const int S = a.S;
  const int SS = S * S;
  const int CC = a.Cin >> 6;
  const int HP = a.HPi;
  const int Pc = a.offi + K / 2;
  const int G = (K / 2) * (S + 1);
  const int nK = CC * T;

  auto halo_piece = [&](int c, int k, int buf) {
    const int r = k * 8 + (lane >> 3);
    int m = m0 - G + r;
    m = m < 0 ? 0 : (m >= a.M ? a.M - 1 : m);
    const int b = fdiv(m, a.divSS);
    const int rem = m - b * SS;
    const int ii = fdiv(rem, a.divS);
    const int q = (b * HP + ii + Pc) * HP + (rem - ii * S) + Pc;
    const int logical = (lane & 7) ^ ((r >> 1) & 7);
    glds16(a.x + (size_t)q * a.Cin + c * 64 + logical * 8, hbuf + buf * H_BYTES + k * 1024);
  };
  // weight pieces: group g stages pieces [g*4*WP, (g+1)*4*WP) of every tile, WP per wave
  const int wpiece0 = (grp * 4 + wq) * WP;
  int wrow[WP];
#pragma unroll
  for (int i = 0; i < WP; ++i) {
    const int r = (wpiece0 + i) * 8 + (lane >> 3);
    wrow[i] = (n0 + r) * a.Cin + (((lane & 7) ^ ((r >> 1) & 7)) << 3);
  }
  const size_t wtap = (size_t)a.Cout * a.Cin;
  auto stage_w = [&](int t, int c, int slot) {
    const __bf16* wt = a.w + (size_t)t * wtap + c * 64;
#pragma unroll
    for (int i = 0; i < WP; ++i) glds16(wt + wrow[i], wbuf + slot * W_BYTES + (wpiece0 + i) * 1024);
  };
  // cursor (tap, chunk) of step q
  auto step_tc = [&](int q, int& tq, int& cq) {
    cq = q / T;
    tq = q - cq * T;
  };

  // lane pixel of block j: m0 + 64 wm + 32 j + (lane & 31)
  int prel[MB], px[MB], py[MB];
#pragma unroll
  for (int j = 0; j < MB; ++j) {
    int m = m0 + wm * 64 + j * 32 + (lane & 31);
    m = m < a.M ? m : a.M - 1;
    const int b = fdiv(m, a.divSS);
    const int rem = m - b * SS;
    py[j] = fdiv(rem, a.divS);
    px[j] = rem - py[j] * S;
    prel[j] = m - m0 + G;
  }
  f32x16 acc[NB][MB];
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int j = 0; j < MB; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  const int swzw = ((lane & 31) >> 1) & 7;
  const int wrow0 = (wn * (BN / 2) + (lane & 31)) * 128;
  const int ep_mrow = m0 + wm * 64 + (lane & 31);
  const int ep_nbase = n0 + wn * (BN / 2);
  ConvEpilogue32<NB, MB, MODE> ep;
  const int ep_at = nK > 3 ? nK - 3 : 0;

  // prologue: zero rows, chunk 0's halo by all waves, W(0) by group 0
  if (wave < NHBUF) {
    for (int o = lane * 16; o < 16 * 128; o += 64 * 16)
      *(uint4*)(hbuf + wave * H_BYTES + HDATA * 128 + o) = make_uint4(0u, 0u, 0u, 0u);
  }
  for (int k = wave; k < H_PIECES; k += 8) halo_piece(0, k, 0);
  stage_w(0, 0, 0);
  wait_vmcnt0();
  if (grp == 1 && nK > 1) {  // group 1 runs its weight half two steps ahead
    int t1, c1;
    step_tc(1, t1, c1);
    stage_w(t1, c1, 1);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  if (grp == 1) __builtin_amdgcn_s_barrier();  // stagger
  __builtin_amdgcn_sched_barrier(0);

  int c = 0, t = 0, kh = 0, kw = 0, wslot = 0;
  const uint64_t st_begin = STAMP ? __builtin_amdgcn_s_memtime() : 0;
  for (int p = 0; p < nK; ++p) {
    H32_STAMP(0);
    const char* hb = hbuf + (NHBUF == 2 ? (c & 1) : 0) * H_BYTES;
    const char* wb = wbuf + wslot * W_BYTES;
    const int toff = (kh - K / 2) * S + (kw - K / 2);
    int abase[MB], aswz[MB];
#pragma unroll
    for (int j = 0; j < MB; ++j) {
      const bool ok = (unsigned)(py[j] + kh - K / 2) < (unsigned)S && (unsigned)(px[j] + kw - K / 2) < (unsigned)S;
      const int r = prel[j] + toff;
      const int row = ok ? r : HDATA + (r & 15);  // zero row with the same (parity, swizzle) bank slot
      abase[j] = row * 128;
      aswz[j] = (row >> 1) & 7;
    }
    bf16x8 xf[4][MB], wf[4][NB];
    auto read_slice = [&](int s) {
      const int kc = 2 * s + h;
#pragma unroll
      for (int j = 0; j < MB; ++j) xf[s][j] = *(const bf16x8*)(hb + abase[j] + ((kc ^ aswz[j]) << 4));
      const int wo = wrow0 + ((kc ^ swzw) << 4);
#pragma unroll
      for (int i = 0; i < NB; ++i) wf[s][i] = *(const bf16x8*)(wb + wo + i * 32 * 128);
    };
    read_slice(0);
    read_slice(1);
    H32_STAMP(1);
    int tn = t + 1, cn = c, khn = kh, kwn = kw + 1;
    if (kwn == K) { kwn = 0; ++khn; }
    if (tn == T) { tn = 0; ++cn; khn = 0; kwn = 0; }
    if (p == ep_at) ep.load(a, ep_mrow, ep_nbase, wn);  // (older than this segment's DMA)
    if (grp == 0) {
      if (p + 1 < nK) stage_w(tn, cn, wslot == 2 ? 0 : wslot + 1);  // retired at the end of M0(p)
    } else {
      // group 1: next chunk's halo (steps 0..4 of a chunk), its half of W(p+2), then
      // retire everything issued in earlier segments (W(p+1) half, older halo pieces)
      int nh = 0;
      if (K == 3 && c + 1 < CC && t < 5) {
#pragma unroll
        for (int i = 0; i < HP_STEP; ++i) halo_piece(c + 1, wq * HP1 + t * HP_STEP + i, (c + 1) & 1);
        nh = HP_STEP;
      }
      const bool w2 = p + 2 < nK;
      if (w2) {
        int t2, c2;
        step_tc(p + 2, t2, c2);
        stage_w(t2, c2, wslot == 0 ? 2 : wslot - 1);
      }
      if (w2) {
        if (nh) vmcnt_wait<HP_STEP + WP>();
        else vmcnt_wait<WP>();
      } else {
        if (nh) vmcnt_wait<HP_STEP>();
        else vmcnt_wait<0>();
      }
    }
    H32_STAMP(2);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    H32_STAMP(3);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    H32_STAMP(4);
    // ---- MFMA segment: slices 0-1 with the reads of slices 2-3 interleaved
    __builtin_amdgcn_s_setprio(1);
    read_slice(2);
    read_slice(3);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < NB; ++i)
#pragma unroll
        for (int j = 0; j < MB; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[s][i], xf[s][j], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int g = 0; g < MB + NB; ++g) {  // 2 ds_reads per MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 2 * NB * MB - (MB + NB), 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 2; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < NB; ++i)
#pragma unroll
        for (int j = 0; j < MB; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[s][i], xf[s][j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    H32_STAMP(5);
    __builtin_amdgcn_sched_barrier(0);
    if (grp == 0) wait_vmcnt0();  // W(p+1) landed before the barrier that precedes its readers
    H32_STAMP(6);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    H32_STAMP(7);
    if constexpr (STAMP) {
#pragma unroll
      for (int i = 0; i < 7; ++i) st_sum[i] += ts[i + 1] - ts[i];
    }
    t = tn; c = cn; kh = khn; kw = kwn;
    wslot = wslot == 2 ? 0 : wslot + 1;
  }
  if constexpr (STAMP) {
    if (lane == 0) {
      unsigned long long* d = a.dbg + ((size_t)blockIdx.x * 8 + wave) * 8;
#pragma unroll
      for (int i = 0; i < 7; ++i) d[i] = st_sum[i];
      d[7] = __builtin_amdgcn_s_memtime() - st_begin;
    }
  }
#undef H32_STAMP
  if (grp == 0) __builtin_amdgcn_s_barrier();
  ep.store(a, acc, ep_mrow);
}

// largest halo span (rows) of any 256-pixel tile, cached per geometry
static int halo2_rows_needed(int M, int S, int HPi, int K, int offi) {
  static int cM = -1, cS = -1, cH = -1, cK = -1, cO = -1, cR = 0;
  if (M == cM && S == cS && HPi == cH && K == cK && offi == cO) return cR;
  const int SS = S * S, Pc = offi + K / 2, G = (K / 2) * (HPi + 1);
  auto q = [&](int m) {
    const int b = m / SS, rem = m % SS;
    return (b * HPi + rem / S + Pc) * HPi + rem % S + Pc;
  };
  int worst = 0;
  // tiles start at multiples of 256; their offsets within a board repeat with period lcm(256, SS)
  const int period_tiles = SS / std::__gcd(SS, H2_BM);
  const int ntiles = (M + H2_BM - 1) / H2_BM;
  for (int k = 0; k < ntiles && k < period_tiles + 2; ++k) {
    const int m0 = k * H2_BM, m1 = std::min(m0 + H2_BM - 1, M - 1);
    worst = std::max(worst, q(m1) - q(m0) + 2 * G + 1);
  }
  cM = M; cS = S; cH = HPi; cK = K; cO = offi; cR = worst;
  return worst;
}

template <int BN, int MODE>
static void launch_fwd_halo2(const ConvFwdArgs& a, hipStream_t st) {
  constexpr int smem = 2 * H2_ROWS * 128 + 2 * BN * 128;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)conv_fwd_halo2_kernel<BN, MODE>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        smem);
    attr = true;
  }
  dim3 grid((a.M + H2_BM - 1) / H2_BM, a.Cout / BN);
  hipLaunchKernelGGL((conv_fwd_halo2_kernel<BN, MODE>), grid, dim3(512), smem, st, a);
}

template <int BN, int MODE>
static void launch_fwd_hpp(const ConvFwdArgs& a_in, hipStream_t st) {
  constexpr int smem = 2 * HC_ROWS * 128 + 3 * BN * 128;
  if constexpr (BN == 192 && MODE == MODE_BIAS_RELU) {
    if (g_conv_dbg) {  // diagnostic instantiation with segment stamps
      static bool attr_d = false;
      if (!attr_d) {
        hipFuncSetAttribute((const void*)conv_fwd_hpp_kernel<BN, MODE, true>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, smem);
        attr_d = true;
      }
      ConvFwdArgs a = a_in;
      a.dbg = g_conv_dbg;
      dim3 grid((a.M + H2_BM - 1) / H2_BM, a.Cout / BN);
      hipLaunchKernelGGL((conv_fwd_hpp_kernel<BN, MODE, true>), grid, dim3(512), smem, st, a);
      return;
    }
  }
  const ConvFwdArgs& a = a_in;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)conv_fwd_hpp_kernel<BN, MODE>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        smem);
    attr = true;
  }
  dim3 grid((a.M + H2_BM - 1) / H2_BM, a.Cout / BN);
  hipLaunchKernelGGL((conv_fwd_hpp_kernel<BN, MODE>), grid, dim3(512), smem, st, a);
}

template <int BN, int MODE, int K>
static void launch_fwd_h32(const ConvFwdArgs& a_in, hipStream_t st) {
  constexpr int smem = (K == 3 ? 2 * (H32_DATA3 + 16) : (H32_DATA5 + 16)) * 128 + 3 * BN * 128;
  ConvFwdArgs a = a_in;
  dim3 grid((a.M + H2_BM - 1) / H2_BM, a.Cout / BN);
  if constexpr (BN == 192 && MODE == MODE_BIAS_RELU && K == 3) {
    if (g_conv_dbg) {  // diagnostic instantiation with segment stamps
      static bool attr_d = false;
      if (!attr_d) {
        hipFuncSetAttribute((const void*)conv_fwd_h32_kernel<BN, MODE, K, true>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, smem);
        attr_d = true;
      }
      a.dbg = g_conv_dbg;
      hipLaunchKernelGGL((conv_fwd_h32_kernel<BN, MODE, K, true>), grid, dim3(512), smem, st, a);
      return;
    }
  }
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)conv_fwd_h32_kernel<BN, MODE, K>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        smem);
    attr = true;
  }
  hipLaunchKernelGGL((conv_fwd_h32_kernel<BN, MODE, K>), grid, dim3(512), smem, st, a);
}

// the 32x32 halo kernel applies (3x3 any Cin; 5x5 with one 64-channel chunk)
static bool h32_ok(const ConvFwdArgs& a) {
  if (a.K == 3) return H2_BM + 2 * (a.S + 1) <= H32_DATA3;
  if (a.K == 5) return a.Cin == 64 && H2_BM + 4 * (a.S + 1) <= H32_DATA5;
  return false;
}

template <int BN, int MODE>
static void launch_fwd_t(const ConvFwdArgs& a, hipStream_t st) {
  const bool halo_ok = a.K == 3 && a.HPi == a.HPo && a.offi == 0 && a.Po == 1 && a.HPo + 1 <= 32 &&
                       (a.S + 2) * (a.S + 2) * 0 + 256 + 2 * (a.HPo + 1) <= HALO_ROWS;
  if (halo_ok && g_fwd_bm == -1 && !a.mbits_out && MODE != MODE_MASKBITS) {  // opt-in: slower at S=19 (18% border work), see profiles/
    launch_fwd_halo<BN, MODE>(a, st);
    return;
  }
  int bm = g_fwd_bm;
  if (bm == 6) {  // compact halo + ping-pong on 32x32x16 MFMA
    if (h32_ok(a)) {
      if (a.K == 3) launch_fwd_h32<BN, MODE, 3>(a, st);
      else launch_fwd_h32<BN, MODE, 5>(a, st);
      return;
    }
    bm = 0;
  }
  if (bm == 5) {  // halo + ping-pong kernel (3x3, halo fits)
    if (a.K == 3 && H2_BM + 2 * (a.S + 1) <= HC_DATA) {
      launch_fwd_hpp<BN, MODE>(a, st);
      return;
    }
    bm = 0;
  }
  if (bm == 2) {  // interior-halo kernel when the tile's halo fits
    if (halo2_rows_needed(a.M, a.S, a.HPi, a.K, a.offi) <= H2_ROWS && BN <= 192) {
      launch_fwd_halo2<BN, MODE>(a, st);
      return;
    }
    bm = 0;
  }
  // forward and dgrad: 96x96-per-wave tiles (147 KB LDS).  dgrad used to keep
  // a 112-KB tile so that a wgrad workgroup (48 KB) could share its CU, but the
  // concurrent pair is bound by the same per-CU operand delivery either way;
  // the larger tile moves fewer bytes per MFMA (bench: 106.2k -> 108.5k pos/s,
  // scripts/bench_variants.sh).
  if (bm <= 0) bm = (a.M >= 384 * 512) ? 384 : (a.M >= 256 * 512) ? 256 : 128;
  // tile codes: 128 / 256 (64-pixel waves), 2568 (BM 256, 128-pixel waves: 4 waves, 1 per SIMD)
  if (bm == 4) launch_fwd_pp<BN, MODE>(a, st);
  else if (bm == 32) launch_fwd_ring<BN, MODE>(a, st);
  else if (bm == 256) launch_fwd_bm<BN, MODE, 256, 4>(a, st);
  else if (bm == 2560) launch_fwd_bm<BN, MODE, 256, 4, false>(a, st);  // epilogue loads after the loop
  else if (bm == 2568) launch_fwd_bm<BN, MODE, 256, 8>(a, st);
  else if (bm == 384) launch_fwd_bm<BN, MODE, 384, 6, false, false>(a, st);  // 96x96 per wave, 147 KB LDS
  else if (bm == 9) launch_fwd_bm<BN, MODE, 384, 6, false, false, false, true>(a, st);  // DMA spread through MFMAs
  else if (bm == 10) launch_fwd_bm<BN, MODE, 256, 4, false, false, false, true>(a, st);
  else if (bm == 7) {  // 384-pixel tile on the 32x32x16 MFMA (BN multiple of 64)
    if constexpr (BN % 64 == 0) launch_fwd_bm<BN, MODE, 384, 6, false, false, true>(a, st);
  } else if (bm == 8) {  // 256-pixel tile on the 32x32x16 MFMA
    if constexpr (BN % 64 == 0) launch_fwd_bm<BN, MODE, 256, 4, false, false, true>(a, st);
  }
  else launch_fwd_bm<BN, MODE, 128, 4>(a, st);
}

void set_conv_fwd_tile(int bm) { g_fwd_bm = bm; }

template <int MODE>
static void launch_fwd_mode(const ConvFwdArgs& a, hipStream_t st) {
  if (a.Cout % 192 == 0) launch_fwd_t<192, MODE>(a, st);
  else if (a.Cout % 128 == 0) launch_fwd_t<128, MODE>(a, st);
  else launch_fwd_t<64, MODE>(a, st);
}

void launch_conv_fwd(const ConvFwdArgs& a_in, int mode, hipStream_t st) {
  ConvFwdArgs a = a_in;
  a.divSS = make_fastdiv((uint32_t)(a.S * a.S));
  a.divS = make_fastdiv((uint32_t)a.S);
  if (mode == MODE_BIAS_RELU) launch_fwd_mode<MODE_BIAS_RELU>(a, st);
  else if (mode == MODE_MASK) launch_fwd_mode<MODE_MASK>(a, st);
  else if (mode == MODE_MASKBITS) launch_fwd_mode<MODE_MASKBITS>(a, st);
  else launch_fwd_mode<MODE_NONE>(a, st);
}

// ----------------------------------------------------------------- wgrad
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


// 512 threads = 8 waves as 2 (n) x 4 (c).  One pipeline stage = KSUB sub-steps
// of 32 pixels (one barrier per KSUB*32 pixels); each sub-step region is laid
// out [16-channel block][32 px][16 ch] for the transpose reads.
//
// TAPS > 1 (tap-merged, used when the c tile is 64 wide, i.e. the thin first
// layer): one workgroup owns a whole kernel row (TAPS == K taps, kw = 0..K-1)
// and reuses each staged dz tile for all of them; the x image of tap kw is the
// tap-0 image shifted by kw columns (kw * Cin elements).  This triples (5x5:
// quintuples) the MFMAs per staged dz byte, the limiter of the 64-wide tile.
template <int WN, int WC, int KSUB, int NWC = 4, int TAPS = 1>
__global__ __launch_bounds__(128 * NWC, 1) void conv_wgrad_kernel(ConvWgradArgs a) {
  // 2 (n) x NWC (c) waves; NWC = 2 gives each wave a 96x96 tile at 192x192
  // (a third fewer LDS fragment reads per MFMA than NWC = 4)
  constexpr int NWAVES = 2 * NWC;
  constexpr int NBn = WN / 32;          // n blocks per wave (wave covers WN/2)
  constexpr int NBc = WC / (16 * NWC);  // c blocks per wave (wave covers WC/NWC)
  constexpr int DZ_BYTES = WN * 64;  // [WN/16][32 px][16 ch] bf16
  constexpr int X_BYTES = WC * 64 * TAPS;  // [TAPS][WC/16][32 px][16 ch]
  constexpr int SUB = DZ_BYTES + X_BYTES;
  constexpr int STAGE = SUB * KSUB;
  constexpr int XP = WC / 16;  // x pieces per tap
  constexpr int NINSTR = (WN / 16 + XP * TAPS) * KSUB;  // 1 KB glds pieces per stage
  constexpr int IPW = (NINSTR + NWAVES - 1) / NWAVES;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int lane = threadIdx.x & 63;
  const int wave = wave_id();
  const int wn = wave / NWC, wc = wave % NWC;
  const int split = blockIdx.x;
  const int t = blockIdx.y * TAPS;  // first tap of the group
  const int ncb = a.Cin / WC;
  const int n0 = (blockIdx.z / ncb) * WN;
  const int c0 = (blockIdx.z % ncb) * WC;
  const int kh = t / a.K, kw = t - (t / a.K) * a.K;
  const int toff = (kh * a.HPi + kw) * a.Cin + c0;
  const int SS = a.S * a.S;
  // a.ksteps_per_split is in units of one stage (KSUB*32 pixels)
  const int ks_begin = split * a.ksteps_per_split;
  int ks_end = ks_begin + a.ksteps_per_split;
  const int nks_total = (a.M + 32 * KSUB - 1) / (32 * KSUB);
  if (ks_end > nks_total) ks_end = nks_total;

  auto stage = [&](int ks, int buf) {
    const int half = (lane & 1) * 8;
    char* base = smem + buf * STAGE;
    int dzr[KSUB], xr[KSUB];
#pragma unroll
    for (int sub = 0; sub < KSUB; ++sub) {
      const int px = (ks * KSUB + sub) * 32 + (lane >> 1);
      const int pm = px < a.M ? px : a.M - 1;
      const int b = fdiv(pm, a.divSS);
      const int rem = pm - b * SS;
      const int ii = fdiv(rem, a.divS);
      const int jx = rem - ii * a.S;
      dzr[sub] = px < a.M ? ((b * a.HPo + ii + a.Po) * a.HPo + jx + a.Po) * a.Cout : 0;  // 0 = zero border
      xr[sub] = ((b * a.HPi + ii + a.offi) * a.HPi + jx + a.offi) * a.Cin + toff;
    }
    // dz pieces and x pieces in separate loops: a per-piece select between the
    // two source tensors makes hipcc drain vmcnt(0) before the LDS reads that
    // follow, which would turn the double buffer into a synchronous load
#pragma unroll
    for (int sub = 0; sub < KSUB; ++sub) {
      const __bf16* dsrc = a.dz + dzr[sub] + n0 + half;
      const __bf16* xsrc = a.x + xr[sub] + half;
#pragma unroll
      for (int i = 0; i < IPW; ++i) {
        const int jj = wave * IPW + i - sub * (NINSTR / KSUB);
        if (jj >= 0 && jj < WN / 16) glds16(dsrc + jj * 16, base + sub * SUB + jj * 1024);
      }
#pragma unroll
      for (int i = 0; i < IPW; ++i) {
        const int jj = wave * IPW + i - sub * (NINSTR / KSUB);
        if (jj >= WN / 16 && jj < NINSTR / KSUB) {
          const int xj = jj - WN / 16;  // tap xj / XP, channel piece xj % XP
          glds16(xsrc + (xj / XP) * a.Cin + (xj % XP) * 16, base + sub * SUB + jj * 1024);
        }
      }
    }
  };

  f32x4 acc[TAPS][NBn][NBc];
#pragma unroll
  for (int tp = 0; tp < TAPS; ++tp)
#pragma unroll
    for (int i = 0; i < NBn; ++i)
#pragma unroll
      for (int j = 0; j < NBc; ++j) acc[tp][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float dbs[NBn];
#pragma unroll
  for (int i = 0; i < NBn; ++i) dbs[i] = 0.f;
  const bool do_bias = (t == 0) && (c0 == 0) && (wc == 0);

  // transposed-read addresses: group g = lane>>4, row q = (lane&15)>>2, col 4p, p = lane&3
  const int g = lane >> 4;
  const int q = (lane & 15) >> 2;
  const int p = lane & 3;
  const int tr0 = (4 * g + q) * 32 + p * 8;         // rows 4g..4g+3
  const int tr1 = (16 + 4 * g + q) * 32 + p * 8;    // rows 16+4g..16+4g+3
  constexpr int NF = NBn + TAPS * NBc;  // fragments read per sub-step

  if (ks_begin < ks_end) {
    stage(ks_begin, 0);
    wait_vmcnt0();
    __syncthreads();
  }
  for (int ks = ks_begin; ks < ks_end; ++ks) {
    const int cur = (ks - ks_begin) & 1;
    if (ks + 1 < ks_end) stage(ks + 1, cur ^ 1);
#pragma unroll
    for (int sub = 0; sub < KSUB; ++sub) {
      const char* base = smem + cur * STAGE + sub * SUB;
      bf16x4 tl[NF], th[NF];
#pragma unroll
      for (int i = 0; i < NBn; ++i) {
        const char* cb = base + (wn * NBn + i) * 1024;
        tl[i] = ds_read_tr16_asm(cb + tr0);
        th[i] = ds_read_tr16_asm(cb + tr1);
      }
#pragma unroll
      for (int tp = 0; tp < TAPS; ++tp)
#pragma unroll
        for (int j = 0; j < NBc; ++j) {
          const char* cb = base + DZ_BYTES + (tp * XP + wc * NBc + j) * 1024;
          tl[NBn + tp * NBc + j] = ds_read_tr16_asm(cb + tr0);
          th[NBn + tp * NBc + j] = ds_read_tr16_asm(cb + tr1);
        }
      lgkm_fence<NF>(tl, th);
      bf16x8 af[NBn], bfm[TAPS * NBc];
#pragma unroll
      for (int i = 0; i < NBn; ++i)
        af[i] = bf16x8{tl[i][0], tl[i][1], tl[i][2], tl[i][3], th[i][0], th[i][1], th[i][2], th[i][3]};
#pragma unroll
      for (int j = 0; j < TAPS * NBc; ++j)
        bfm[j] = bf16x8{tl[NBn + j][0], tl[NBn + j][1], tl[NBn + j][2], tl[NBn + j][3],
                        th[NBn + j][0], th[NBn + j][1], th[NBn + j][2], th[NBn + j][3]};
#pragma unroll
      for (int tp = 0; tp < TAPS; ++tp)
#pragma unroll
        for (int i = 0; i < NBn; ++i)
#pragma unroll
          for (int j = 0; j < NBc; ++j)
            acc[tp][i][j] = mfma16x16x32(af[i], bfm[tp * NBc + j], acc[tp][i][j]);
      if (do_bias) {
#pragma unroll
        for (int i = 0; i < NBn; ++i) {
          float s = 0.f;
#pragma unroll
          for (int e = 0; e < 8; ++e) s += (float)af[i][e];
          dbs[i] += s;
        }
      }
    }
    wait_vmcnt0();
    __syncthreads();
  }

  // --- write the split's partial tile: D[n][c], lane owns n..n+3 at column c
  const int nb0 = n0 + wn * (WN / 2) + ((lane >> 4) << 2);
  const int cbase = c0 + wc * (WC / NWC) + (lane & 15);
#pragma unroll
  for (int tp = 0; tp < TAPS; ++tp) {
    float* out = a.slab + ((size_t)split * a.T + t + tp) * (size_t)a.Cout * a.Cin;
#pragma unroll
    for (int i = 0; i < NBn; ++i)
#pragma unroll
      for (int j = 0; j < NBc; ++j) {
        const int n = nb0 + i * 16;
        const int c = cbase + j * 16;
#pragma unroll
        for (int r = 0; r < 4; ++r) out[(size_t)(n + r) * a.Cin + c] = acc[tp][i][j][r];
      }
  }
  if (do_bias) {
#pragma unroll
    for (int i = 0; i < NBn; ++i) {
      float s = dbs[i];
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      if (lane < 16) a.dbias_slab[(size_t)split * a.Cout + n0 + wn * (WN / 2) + i * 16 + lane] = s;
    }
  }
}


// wgrad, ring variant: same tile math and LDS image as conv_wgrad_kernel
// (KSUB = 1, 32-pixel K-steps), but 4 LDS slots with the DMA running 3 steps
// ahead, counted vmcnt for the wave's own pieces of the next step and a raw
// s_barrier, so no barrier ever drains the loads in flight.
template <int WN, int WC, int WRING_SLOTS>
__global__ __launch_bounds__(512, 1) void conv_wgrad_ring_kernel(ConvWgradArgs a) {
  constexpr int AHEAD = WRING_SLOTS - 1;  // steps the DMA runs ahead of the MFMAs
  constexpr int NBn = WN / 32;
  constexpr int NBc = WC / 64;
  constexpr int DZ_BYTES = WN * 64;
  constexpr int X_BYTES = WC * 64;
  constexpr int SLOT = DZ_BYTES + X_BYTES;
  constexpr int NINSTR = (WN + WC) / 16;
  constexpr int IPW = (NINSTR + 7) / 8;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int lane = threadIdx.x & 63;
  const int wave = wave_id();
  const int wn = wave >> 2, wc = wave & 3;
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
  const int nks_total = (a.M + 31) / 32;
  if (ks_end > nks_total) ks_end = nks_total;
  const int jlo = wave * IPW;
  const int P = (NINSTR - jlo) < 0 ? 0 : ((NINSTR - jlo) < IPW ? (NINSTR - jlo) : IPW);  // pieces per step

  auto issue = [&](int ks) {
    const int half = (lane & 1) * 8;
    char* base = smem + (ks % WRING_SLOTS) * SLOT;
    const int px = ks * 32 + (lane >> 1);
    const int pm = px < a.M ? px : a.M - 1;
    const int b = fdiv(pm, a.divSS);
    const int rem = pm - b * SS;
    const int ii = fdiv(rem, a.divS);
    const int jx = rem - ii * a.S;
    const int dzr = px < a.M ? ((b * a.HPo + ii + a.Po) * a.HPo + jx + a.Po) * a.Cout : 0;  // 0 = zero border
    const int xr = ((b * a.HPi + ii + a.offi) * a.HPi + jx + a.offi) * a.Cin + toff;
    // dz pieces and x pieces in separate (wave-uniform) loops: a per-piece
    // select between the two source tensors makes hipcc drain vmcnt before the
    // next LDS reads
    const __bf16* dsrc = a.dz + dzr + n0 + half;
    const __bf16* xsrc = a.x + xr + half;
#pragma unroll
    for (int i = 0; i < IPW; ++i) {
      const int j = jlo + i;
      if (j < WN / 16) glds16(dsrc + j * 16, base + j * 1024);
    }
#pragma unroll
    for (int i = 0; i < IPW; ++i) {
      const int j = jlo + i;
      if (j >= WN / 16 && j < NINSTR) glds16(xsrc + (j - WN / 16) * 16, base + j * 1024);
    }
  };

  f32x4 acc[NBn][NBc];
#pragma unroll
  for (int i = 0; i < NBn; ++i)
#pragma unroll
    for (int j = 0; j < NBc; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float dbs[NBn];
#pragma unroll
  for (int i = 0; i < NBn; ++i) dbs[i] = 0.f;
  const bool do_bias = (t == 0) && (c0 == 0) && (wc == 0);

  const int g = lane >> 4;
  const int q = (lane & 15) >> 2;
  const int p = lane & 3;
  const int tr0 = (4 * g + q) * 32 + p * 8;
  const int tr1 = (16 + 4 * g + q) * 32 + p * 8;

  const int nst = ks_end - ks_begin;
  if (nst > 0) {
#pragma unroll
    for (int d = 0; d < AHEAD; ++d)
      if (d < nst) issue(ks_begin + d);
    vmcnt_wait_dyn(P * (nst > AHEAD ? AHEAD - 1 : nst - 1));
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  }
  for (int ks = ks_begin; ks < ks_end; ++ks) {
    if (ks + AHEAD < ks_end) issue(ks + AHEAD);  // into the slot step ks-1 used (all waves are past its reads)
    const char* base = smem + (ks % WRING_SLOTS) * SLOT;
    bf16x4 tl[NBn + NBc], th[NBn + NBc];
#pragma unroll
    for (int i = 0; i < NBn; ++i) {
      const char* cb = base + (wn * NBn + i) * 1024;
      tl[i] = ds_read_tr16_asm(cb + tr0);
      th[i] = ds_read_tr16_asm(cb + tr1);
    }
#pragma unroll
    for (int j = 0; j < NBc; ++j) {
      const char* cb = base + DZ_BYTES + (wc * NBc + j) * 1024;
      tl[NBn + j] = ds_read_tr16_asm(cb + tr0);
      th[NBn + j] = ds_read_tr16_asm(cb + tr1);
    }
    // lgkmcnt(0) with every read result as an in/out operand: nothing that
    // uses them can be scheduled above the wait
    lgkm_fence<NBn + NBc>(tl, th);
    bf16x8 af[NBn], bfm[NBc];
#pragma unroll
    for (int i = 0; i < NBn; ++i)
      af[i] = bf16x8{tl[i][0], tl[i][1], tl[i][2], tl[i][3], th[i][0], th[i][1], th[i][2], th[i][3]};
#pragma unroll
    for (int j = 0; j < NBc; ++j)
      bfm[j] = bf16x8{tl[NBn + j][0], tl[NBn + j][1], tl[NBn + j][2], tl[NBn + j][3],
                      th[NBn + j][0], th[NBn + j][1], th[NBn + j][2], th[NBn + j][3]};
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < NBn; ++i)
#pragma unroll
      for (int j = 0; j < NBc; ++j) acc[i][j] = mfma16x16x32(af[i], bfm[j], acc[i][j]);
    __builtin_amdgcn_s_setprio(0);
    if (do_bias) {
#pragma unroll
      for (int i = 0; i < NBn; ++i) {
        float s = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) s += (float)af[i][e];
        dbs[i] += s;
      }
    }
    if (ks + 1 < ks_end) {
      const int ahead = ks_end - ks - 2;  // steps issued beyond ks+1 (at most AHEAD-1)
      vmcnt_wait_dyn(P * (ahead > AHEAD - 1 ? AHEAD - 1 : ahead));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  float* out = a.slab + ((size_t)split * a.T + t) * (size_t)a.Cout * a.Cin;
  const int nb0 = n0 + wn * (WN / 2) + ((lane >> 4) << 2);
  const int cbase = c0 + wc * (WC / 4) + (lane & 15);
#pragma unroll
  for (int i = 0; i < NBn; ++i)
#pragma unroll
    for (int j = 0; j < NBc; ++j) {
      const int n = nb0 + i * 16;
      const int c = cbase + j * 16;
#pragma unroll
      for (int r = 0; r < 4; ++r) out[(size_t)(n + r) * a.Cin + c] = acc[i][j][r];
    }
  if (do_bias) {
#pragma unroll
    for (int i = 0; i < NBn; ++i) {
      float s = dbs[i];
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      if (lane < 16) a.dbias_slab[(size_t)split * a.Cout + n0 + wn * (WN / 2) + i * 16 + lane] = s;
    }
  }
}

constexpr int kWgradKsub = 1;
static int g_wgrad_variant = 0;  // 0 = 2-buffer, 3/4 = ring with that many LDS slots

template <int WN, int WC, int NS>
static void launch_wgrad_ring(const ConvWgradArgs& a, dim3 grid, hipStream_t st) {
  constexpr int smem = NS * (WN + WC) * 64;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)conv_wgrad_ring_kernel<WN, WC, NS>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        smem);
    attr = true;
  }
  hipLaunchKernelGGL((conv_wgrad_ring_kernel<WN, WC, NS>), grid, dim3(512), smem, st, a);
}

template <int WN, int TAPS>
static void launch_wgrad_taps(const ConvWgradArgs& a, hipStream_t st) {
  constexpr int smem = 2 * (WN + 64 * TAPS) * 64 * kWgradKsub;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)conv_wgrad_kernel<WN, 64, kWgradKsub, 4, TAPS>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr = true;
  }
  dim3 grid(a.nsplit, a.T / TAPS, (a.Cout / WN) * (a.Cin / 64));
  hipLaunchKernelGGL((conv_wgrad_kernel<WN, 64, kWgradKsub, 4, TAPS>), grid, dim3(512), smem, st, a);
}

int wgrad_tap_group(int Cout, int Cin, int K) {
  const bool c64 = Cin % 192 != 0 && Cin % 128 != 0;
  (void)Cout;
  return (c64 && g_wgrad_variant == 0 && (K == 3 || K == 5)) ? K : 1;
}

template <int WN, int WC>
static void launch_wgrad_t(const ConvWgradArgs& a, hipStream_t st) {
  dim3 grid(a.nsplit, a.T, (a.Cout / WN) * (a.Cin / WC));
  if (g_wgrad_variant == 3 || g_wgrad_variant == 4) {
    if (g_wgrad_variant == 3) launch_wgrad_ring<WN, WC, 3>(a, grid, st);
    else launch_wgrad_ring<WN, WC, 4>(a, grid, st);
    return;
  }
  constexpr int KS = kWgradKsub;
  constexpr int smem = 2 * (WN + WC) * 64 * KS;
  if (g_wgrad_variant == 2 && WC % 32 == 0 && WC >= 64) {
    static bool attr2 = false;
    if (!attr2) {
      hipFuncSetAttribute((const void*)conv_wgrad_kernel<WN, WC, KS, 2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          smem);
      attr2 = true;
    }
    hipLaunchKernelGGL((conv_wgrad_kernel<WN, WC, KS, 2>), grid, dim3(256), smem, st, a);
    return;
  }
  if constexpr (WC == 64) {
    // tap-merged kernel rows (see conv_wgrad_kernel); variant 1 forces one tap per workgroup
    if (g_wgrad_variant != 1 && (a.K == 3 || a.K == 5)) {
      if (a.K == 3) launch_wgrad_taps<WN, 3>(a, st);
      else launch_wgrad_taps<WN, 5>(a, st);
      return;
    }
  }
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)conv_wgrad_kernel<WN, WC, KS>, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr = true;
  }
  hipLaunchKernelGGL((conv_wgrad_kernel<WN, WC, KS>), grid, dim3(512), smem, st, a);
}

void set_wgrad_variant(int v) { g_wgrad_variant = v; }

int wgrad_stage_pixels() { return 32 * kWgradKsub; }

void launch_conv_wgrad(const ConvWgradArgs& a_in, hipStream_t st) {
  ConvWgradArgs a = a_in;
  a.divSS = make_fastdiv((uint32_t)(a.S * a.S));
  a.divS = make_fastdiv((uint32_t)a.S);
  const bool n192 = a.Cout % 192 == 0, c192 = a.Cin % 192 == 0;
  const bool n128 = a.Cout % 128 == 0, c128 = a.Cin % 128 == 0;
  if (n192 && c192) launch_wgrad_t<192, 192>(a, st);
  else if (n192 && c128) launch_wgrad_t<192, 128>(a, st);
  else if (n192) launch_wgrad_t<192, 64>(a, st);
  else if (n128 && c128) launch_wgrad_t<128, 128>(a, st);
  else if (n128 && c192) launch_wgrad_t<128, 192>(a, st);
  else if (n128) launch_wgrad_t<128, 64>(a, st);
  else if (c192) launch_wgrad_t<64, 192>(a, st);
  else if (c128) launch_wgrad_t<64, 128>(a, st);
  else launch_wgrad_t<64, 64>(a, st);
}

// Sum split partials into the fp32 OIHW gradient (real channel counts) + bias.
// Threads walk the slab in its natural [t][n][c] order (c fastest) so every
// split read is coalesced; the OIHW write is strided but only touches the
// (small) gradient once.
__global__ void conv_wgrad_reduce_kernel(WgradReduceArgs a) {
  const int total = a.T * a.Cout_real * a.Cin;
  const size_t tile = (size_t)a.Cout * a.Cin;
  const size_t sstride = (size_t)a.T * tile;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += gridDim.x * blockDim.x) {
    const int c = idx % a.Cin;
    const int tn = idx / a.Cin;
    const int n = tn % a.Cout_real;
    const int t = tn / a.Cout_real;
    if (c >= a.Cin_real) continue;
    const float* s = a.slab + (size_t)t * tile + (size_t)n * a.Cin + c;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    int sp = 0;
    for (; sp + 4 <= a.nsplit; sp += 4) {
      s0 += s[(size_t)sp * sstride];
      s1 += s[(size_t)(sp + 1) * sstride];
      s2 += s[(size_t)(sp + 2) * sstride];
      s3 += s[(size_t)(sp + 3) * sstride];
    }
    for (; sp < a.nsplit; ++sp) s0 += s[(size_t)sp * sstride];
    const float sum = (s0 + s1) + (s2 + s3);
    float* g = a.grad_w + ((size_t)n * a.Cin_real + c) * a.T + t;
    *g = a.beta * *g + a.scale * sum;
  }
  if (blockIdx.x == 0 && a.grad_b) {
    for (int n = threadIdx.x; n < a.Cout_real; n += blockDim.x) {
      float sum = 0.f;
      for (int sp = 0; sp < a.nsplit; ++sp) sum += a.dbias_slab[(size_t)sp * a.Cout + n];
      a.grad_b[n] = a.beta * a.grad_b[n] + a.scale * sum;
    }
  }
}

void launch_wgrad_reduce(const WgradReduceArgs& a, hipStream_t st) {
  const int total = a.T * a.Cout_real * a.Cin;
  int blocks = (total + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(conv_wgrad_reduce_kernel, dim3(blocks), dim3(256), 0, st, a);
}

}  // namespace agk
