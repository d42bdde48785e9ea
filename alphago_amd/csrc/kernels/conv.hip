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
#include <cstdlib>
#include <numeric>

#include "common.h"
#include "conv_common.h"
#include "kernels.h"

namespace agk {

// ----------------------------------------------------------------- forward
// STR (Cin % 64 == 32, e.g. the value net's 152 filters padded to 160): a
// 64-channel K-step may straddle two taps -- the 32-channel half h of every
// staged row comes from its own (tap, channel) source, selected per lane by
// the row piece's logical chunk, so no MFMA multiplies padding.  The last
// step's second half (K = taps * Cin is an odd multiple of 32) reads an extra
// all-zero weight tap (packed weights then hold K*K + 1 taps).
// BN whose per-wave weight rows are not a multiple of 8 (BN = 160) stage the
// weight tile as 8-row pieces dealt round-robin over the waves.
// CO (chunk outer): the K loop runs the 64-channel chunk in the outer loop and
// the taps inside it, instead of all chunks of one tap before the next tap.
// A tile's pixel rows for one chunk (BM + 2 halo rows x 128 B) are then re-read
// by the 9 taps while they are hot in the XCD's L2, where the tap-outer order
// cycles through every chunk of the tile (BM x Cin x 2 B per tile, ~5 MB for
// the 32 tiles of an XCD at Cin 192 -- more than its 4 MB L2).
template <int BN, int MODE, int BM, int MBW, bool EPF = true, bool PIPE = true, bool M32 = false, bool ILV = false,
          bool STR = false, bool CO = false>
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
  constexpr bool BDIST = (BN / NW) % 8 != 0;  // weight pieces dealt round-robin
  constexpr int B_ROWS_PW = BN / NW;   // weight rows staged per wave (contiguous layout)
  constexpr int B_INSTR = BDIST ? (BN / 8 + NW - 1) / NW : B_ROWS_PW / 8;  // glds instructions per wave
  static_assert(BN % 32 == 0 && BN % 8 == 0 && A_ROWS_PW % 8 == 0, "tile geometry");
  static_assert(!(BDIST && M32), "round-robin weight staging: not in the 32x32 loop");
  static_assert(!(STR && M32), "straddled K-steps: not in the 32x32 loop");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int lane = threadIdx.x & 63;
  const int wave = wave_id();
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int SS = a.S * a.S;
  const int CC = a.Cin >> 6;  // 64-channel chunks
  const int nK = STR ? (a.K * a.K * a.Cin + 63) >> 6 : a.K * a.K * CC;

  // --- staging addresses (element offsets)
  int arow[A_INSTR];
  bool ahi[A_INSTR], bhi[B_INSTR];  // STR: the piece's 32-channel half of the K-step
#pragma unroll
  for (int i = 0; i < A_INSTR; ++i) {
    const int r = wave * A_ROWS_PW + i * 8 + (lane >> 3);
    ahi[i] = (((lane & 7) ^ ((r >> 1) & 7)) >> 2) != 0;
    int m = m0 + r;
    m = m < a.M ? m : a.M - 1;
    const int b = fdiv(m, a.divSS);
    const int rem = m - b * SS;
    const int ii = fdiv(rem, a.divS);
    const int jj = rem - ii * a.S;
    const int logical = (lane & 7) ^ ((r >> 1) & 7);
    // STR: channel part (logical & 3) * 8 only; the half (logical >> 2) picks the source
    arow[i] = ((b * a.HPi + ii + a.offi) * a.HPi + jj + a.offi) * a.Cin + (STR ? (logical & 3) : logical) * 8;
  }
  int brow[B_INSTR], bldsrow[B_INSTR];
#pragma unroll
  for (int i = 0; i < B_INSTR; ++i) {
    const int piece = BDIST ? wave + i * NW : wave * (B_ROWS_PW / 8) + i;  // 8-row piece of the weight tile
    const int r = piece * 8 + (lane >> 3);
    const int logical = (lane & 7) ^ ((r >> 1) & 7);
    bhi[i] = (logical >> 2) != 0;
    brow[i] = (n0 + (r < BN ? r : BN - 1)) * a.Cin + (STR ? (logical & 3) : logical) * 8;
    bldsrow[i] = piece * 8;
  }

  const size_t wtap = (size_t)a.Cout * a.Cin;

  // staging cursor over (tap, 64-channel chunk), advanced incrementally with
  // scalar adds (no per-step integer divisions)
  int st_c0 = 0, st_kw = 0, st_a = 0, st_t = 0;
  size_t st_w = 0;
  // source offsets (without the lane's row/channel part) of the step's two
  // 32-channel halves; equal unless STR
  auto st_offsets = [&](int& xo0, int& xo1, size_t& wo0, size_t& wo1) {
    xo0 = st_a + st_c0;
    xo1 = xo0;
    wo0 = st_w + st_c0;
    wo1 = wo0;
    if constexpr (STR && CO) {
      // chunk outer: the 64-channel chunks run full steps tap by tap; the 32-channel tail chunk
      // (Cin % 64 == 32) pairs taps t and t+1 in one step (t = K*K: the all-zero extra tap)
      const bool part = st_c0 + 64 > a.Cin;
      const int a_next = st_a + (st_kw + 1 == a.K ? (a.HPi - a.K + 1) * a.Cin : a.Cin);
      xo1 = part ? (st_t + 1 < a.K * a.K ? a_next : st_a) + st_c0 : xo0 + 32;
      wo1 = part ? st_w + wtap + st_c0 : wo0 + 32;
    } else if constexpr (STR) {
      const int c1 = st_c0 + 32;
      const bool nx = c1 >= a.Cin;  // the second half opens the next tap
      const int a_next = st_a + (st_kw + 1 == a.K ? (a.HPi - a.K + 1) * a.Cin : a.Cin);
      // past the last tap: any in-range pixel rows (the weight tap there is all zero)
      xo1 = nx ? (st_t + 1 < a.K * a.K ? a_next : xo0) : st_a + c1;
      wo1 = nx ? st_w + wtap : st_w + c1;
    }
  };
  // DMA piece d of a stage: pixel pieces 0 .. A_INSTR-1, then weight pieces
  auto st_piece = [&](int d, char* base, int xo0, int xo1, size_t wo0, size_t wo1) {
    if (d < A_INSTR) {
      const int xo = arow[d] + ((STR && ahi[d]) ? xo1 : xo0);
#ifdef AGK_DEBUG
      const bool ok = AGK_DCHECK(xo >= 0 && (long long)xo + 8 <= a.x_elems, DBG_FWD_X);
      glds16(a.x + (ok ? xo : 0), base + (wave * A_ROWS_PW + d * 8) * 128);
#else
      glds16(a.x + xo, base + (wave * A_ROWS_PW + d * 8) * 128);
#endif
    } else {
      const int i = d - A_INSTR;
      if (BDIST && wave + i * NW >= BN / 8) return;  // wave-uniform: fewer pieces on the last waves
      const size_t wo = ((STR && bhi[i]) ? wo1 : wo0) + brow[i];
#ifdef AGK_DEBUG
      const bool ok = AGK_DCHECK((long long)wo + 8 <= a.w_elems, DBG_FWD_W);
      glds16(ok ? a.w + wo : a.w, base + A_BYTES + bldsrow[i] * 128);
#else
      glds16(a.w + wo, base + A_BYTES + bldsrow[i] * 128);
#endif
    }
  };
  // branch-free cursor advance (selects), so a caller can interleave the
  // DMA with MFMAs inside one basic block
  auto st_advance = [&]() {
    if constexpr (CO) {
      // one tap (two in the STR tail chunk, whose steps pair taps)
      const int nt = (STR && st_c0 + 64 > a.Cin) ? 2 : 1;
      st_t += nt;
      st_kw += nt;
      st_w += nt * wtap;
      st_a += nt * a.Cin;
      const bool wrap2 = st_kw >= a.K;
      st_kw = wrap2 ? st_kw - a.K : st_kw;
      st_a += wrap2 ? (a.HPi - a.K) * a.Cin : 0;
      const bool wrapt = st_t == a.K * a.K;  // all taps of the chunk done: next chunk, tap 0
      st_t = wrapt ? 0 : st_t;
      st_w = wrapt ? 0 : st_w;
      st_a = wrapt ? 0 : st_a;
      st_c0 += wrapt ? 64 : 0;
      return;
    }
    st_c0 += 64;
    const bool wrap = STR ? st_c0 >= a.Cin : st_c0 == a.Cin;
    st_c0 = wrap ? st_c0 - a.Cin : st_c0;
    st_w += wrap ? wtap : 0;
    st_t += wrap ? 1 : 0;
    st_kw += wrap ? 1 : 0;
    const bool wrap2 = st_kw == a.K;
    st_kw = wrap2 ? 0 : st_kw;
    st_a += (wrap ? a.Cin : 0) + (wrap2 ? (a.HPi - a.K) * a.Cin : 0);
  };
  auto stage = [&](int buf) {
    char* base = smem + buf * STAGE;
    int xo0, xo1;
    size_t wo0, wo1;
    st_offsets(xo0, xo1, wo0, wo1);
#pragma unroll
    for (int d = 0; d < A_INSTR + B_INSTR; ++d) st_piece(d, base, xo0, xo1, wo0, wo1);
    st_advance();
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
      int xo0, xo1;
      size_t wo0, wo1;
      st_offsets(xo0, xo1, wo0, wo1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int d = 0; d < NDMA; ++d) {
        mfma_range(d * MPD, (d + 1) * MPD);
        __builtin_amdgcn_sched_barrier(0);
        if (more) st_piece(d, nb, xo0, xo1, wo0, wo1);
        __builtin_amdgcn_sched_barrier(0);
      }
      mfma_range(NDMA * MPD, NMF);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      st_advance();
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


#ifdef AGK_KERNEL_LAB
// ------------------------------------ forward, pixel operand straight from L2
// Probe (scripts/probes/glds_rate.hip): LDS-DMA fills a CU at ~46 B/clk and
// serialises with ds_read traffic, so in the LDS-staged kernels the LDS port
// (pixel + weight DMA, plus fragment reads) is about as busy as the matrix
// pipe.  Here only the weights go through LDS; each wave loads its pixel
// fragments (16 B per lane, 8 channels of one pixel row) with ordinary
// global_load_dwordx4 into registers, one step ahead (register double
// buffer).  Waves own disjoint pixels (8 x 48 = 384 per workgroup) and all BN
// channels, so no pixel row is loaded twice in a workgroup; per 64-channel
// step a CU moves 24 KB through LDS-DMA instead of 72 KB.
// Epilogue and ReLU'-bitmask layout are those of conv_fwd_kernel (the wave's
// two channel halves are stored as wn = 0 and wn = 1).
template <int BN, int MODE>
__global__ __launch_bounds__(512, 1) void conv_fwd_ga_kernel(ConvFwdArgs a) {
  constexpr int MB = 3;          // 16-pixel blocks per wave (48 pixels)
  constexpr int NB = BN / 16;    // 16-channel blocks per wave (all BN channels)
  constexpr int NH = NB / 2;     // blocks per channel half
  constexpr int BM = 8 * 16 * MB;
  constexpr int W_BYTES = BN * 128;
  constexpr int WPIECES = BN / 8;       // 1-KB weight pieces per step
  constexpr int WPW = (WPIECES + 7) / 8;
  static_assert(NB % 2 == 0, "two channel halves");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int lane = threadIdx.x & 63;
  const int wave = wave_id();
  const int nwg = gridDim.x;
  const int xcd = blockIdx.x & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (blockIdx.x >> 3);
  const int m0 = tile * BM;
  const int n0 = blockIdx.y * BN;
  const int SS = a.S * a.S;
  const int CC = a.Cin >> 6;
  const int nK = a.K * a.K * CC;

  // Buffer resources: per-lane byte offsets stay fixed in one VGPR each, the
  // (wave-uniform) step cursor goes in the scalar offset, and loads past the
  // tensor return zero instead of faulting.
  const int nimg = a.M / SS;
  const long long xbytes = (long long)nimg * a.HPi * a.HPi * a.Cin * 2;
  const long long wbytes = (long long)a.K * a.K * a.Cout * a.Cin * 2;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.x, (short)0, (int)(xbytes < 0x7fffffffLL ? xbytes : 0x7fffffffLL), 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.w, (short)0, (int)(wbytes < 0x7fffffffLL ? wbytes : 0x7fffffffLL), 0x00020000);
  // pixel fragment sources: lane -> pixel (block j, row lane&15), 16-B chunk lane>>4 of the k-half
  int xrow[MB];
#pragma unroll
  for (int j = 0; j < MB; ++j) {
    int m = m0 + wave * 16 * MB + j * 16 + (lane & 15);
    m = m < a.M ? m : a.M - 1;
    const int b = fdiv(m, a.divSS);
    const int rem = m - b * SS;
    const int ii = fdiv(rem, a.divS);
    const int jj = rem - ii * a.S;
    xrow[j] = (((b * a.HPi + ii + a.offi) * a.HPi + jj + a.offi) * a.Cin + (lane >> 4) * 8) * 2;
  }
  // weight DMA: wave w stages pieces [w*WPW, ...) of the BN x 64-ch tile (128-B rows, swizzled)
  int wrow[WPW];
#pragma unroll
  for (int i = 0; i < WPW; ++i) {
    const int r = (wave * WPW + i) * 8 + (lane >> 3);
    wrow[i] = ((n0 + (r < BN ? r : 0)) * a.Cin + (((lane & 7) ^ ((r >> 1) & 7)) << 3)) * 2;
  }
  const int wtap = a.Cout * a.Cin;

  // step cursor in elements (branch-free advance; wave-uniform, lives in SGPRs)
  int c0 = 0, kw = 0, aoff = 0, woff = 0;
  auto advance = [&]() {
    c0 += 64;
    const bool wrap = c0 == a.Cin;
    c0 = wrap ? 0 : c0;
    woff += wrap ? wtap : 0;
    kw += wrap ? 1 : 0;
    const bool wrap2 = kw == a.K;
    kw = wrap2 ? 0 : kw;
    aoff += (wrap ? a.Cin : 0) + (wrap2 ? (a.HPi - a.K) * a.Cin : 0);
  };
  // Weights go global -> VGPR -> ds_write rather than by LDS-DMA: the compiler
  // does not count LDS-DMA in its vmcnt bookkeeping, and a DMA issued between
  // two register loads makes every later compiler wait over-strict.
  typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
  u32x4 wreg[WPW];
  auto load_w = [&]() {
#pragma unroll
    for (int i = 0; i < WPW; ++i) wreg[i] = __builtin_amdgcn_raw_buffer_load_b128(wr, wrow[i], (woff + c0) * 2, 0);
  };
  auto store_w = [&](int slot) {
#pragma unroll
    for (int i = 0; i < WPW; ++i)
      if (wave * WPW + i < WPIECES) *(u32x4*)(smem + slot * W_BYTES + (wave * WPW + i) * 1024 + lane * 16) = wreg[i];
  };
  auto load_x = [&](bf16x8 (&xf)[MB], int kk) {
#pragma unroll
    for (int j = 0; j < MB; ++j) {
      u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(xr, xrow[j], (aoff + c0 + kk * 32) * 2, 0);
      xf[j] = __builtin_bit_cast(bf16x8, v);
    }
  };

  f32x4 acc[NB][MB];
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int j = 0; j < MB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int swz = (lane & 15) >> 1;
  const int wr0 = (lane & 15) * 128;

  // Rolling register buffer: x[kk] is refilled with the next step's k-half as
  // soon as this step's MFMAs on it have issued, so a load has about one step
  // of matrix work to land in.  vmcnt order per step: W(next) (WPW), x[0], x[1].
  // The loads are unconditional (the last step's run past the tensors, where
  // the buffer range check returns zeros): with a conditional issue the
  // compiler's vmcnt bookkeeping merges the skip path and waits for loads that
  // are a whole step younger than the ones the MFMAs need.  Issue order per
  // step: W(next), x[0](next), x[1](next) -- each consumer waits for exactly
  // its own loads.
  bf16x8 x[2][MB];
  load_w();
  load_x(x[0], 0);
  __builtin_amdgcn_sched_barrier(0);
  load_x(x[1], 1);
  advance();
  store_w(0);
  __syncthreads();
  for (int ks = 0; ks < nK; ++ks) {
    const char* wb = smem + (ks & 1) * W_BYTES;
    load_w();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ch = ((kk << 2) + (lane >> 4)) ^ swz;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        bf16x8 wf[NH];
#pragma unroll
        for (int i = 0; i < NH; ++i) wf[i] = *(const bf16x8*)(wb + wr0 + (h * NH + i) * 16 * 128 + (ch << 4));
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < NH; ++i)
#pragma unroll
          for (int j = 0; j < MB; ++j) acc[h * NH + i][j] = mfma16x16x32(wf[i], x[kk][j], acc[h * NH + i][j]);
        __builtin_amdgcn_s_setprio(0);
      }
      __builtin_amdgcn_sched_barrier(0);
      load_x(x[kk], kk);
      __builtin_amdgcn_sched_barrier(0);
    }
    advance();
    store_w((ks + 1) & 1);
    __syncthreads();
  }
  wait_vmcnt0();

  const int mrow = m0 + wave * 16 * MB + (lane & 15);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    f32x4 ah[NH][MB];
#pragma unroll
    for (int i = 0; i < NH; ++i)
#pragma unroll
      for (int j = 0; j < MB; ++j) ah[i][j] = acc[h * NH + i][j];
    ConvEpilogue<NH, MB, MODE> ep;
    ep.load(a, mrow, n0 + h * (BN / 2) + ((lane >> 4) << 2), h);
    ep.store(a, ah, mrow);
  }
}

template <int BN, int MODE>
static void launch_fwd_ga(const ConvFwdArgs& a, hipStream_t st) {
  constexpr int smem = 2 * BN * 128;
  static const hipError_t attr = hipFuncSetAttribute((const void*)conv_fwd_ga_kernel<BN, MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, smem);  // once per instantiation (thread-safe static)
  hip_check(attr, "hipFuncSetAttribute(max dynamic LDS)");
  constexpr int BM = 8 * 16 * 3;
  dim3 grid((a.M + BM - 1) / BM, a.Cout / BN);
  hipLaunchKernelGGL((conv_fwd_ga_kernel<BN, MODE>), grid, dim3(512), smem, st, a);
}

#endif  // AGK_KERNEL_LAB

template <int BN, int MODE, int BM, int MBW, bool EPF = true, bool PIPE = true, bool M32 = false, bool ILV = false,
          bool STR = false, bool CO = false>
static void launch_fwd_bm(const ConvFwdArgs& a, hipStream_t st) {
  constexpr int smem = 2 * (BM * 128 + BN * 128);
  static const hipError_t attr = hipFuncSetAttribute(
      (const void*)conv_fwd_kernel<BN, MODE, BM, MBW, EPF, PIPE, M32, ILV, STR, CO>,
      hipFuncAttributeMaxDynamicSharedMemorySize, smem);  // once per instantiation (thread-safe static)
  hip_check(attr, "hipFuncSetAttribute(max dynamic LDS)");
  dim3 grid((a.M + BM - 1) / BM, a.Cout / BN);
  hipLaunchKernelGGL((conv_fwd_kernel<BN, MODE, BM, MBW, EPF, PIPE, M32, ILV, STR, CO>), grid, dim3(BM / MBW * 8),
                     smem, st, a);
}

// 160-wide output tile (value net: 152 filters padded to 160 instead of 192);
// Cin % 64 == 32 uses straddled K-steps
template <int MODE, bool STR>
static void launch_fwd_160(const ConvFwdArgs& a, int bm, hipStream_t st) {
  if (bm == 384) launch_fwd_bm<160, MODE, 384, 6, false, false, false, false, STR>(a, st);
  else if (bm == 385) launch_fwd_bm<160, MODE, 384, 6, false, false, false, true, STR>(a, st);
  else if (bm == 386) launch_fwd_bm<160, MODE, 384, 6, false, false, false, true, STR, true>(a, st);
  else if (bm == 387) launch_fwd_bm<160, MODE, 384, 6, false, false, false, false, STR, true>(a, st);
  else if (bm == 256) launch_fwd_bm<160, MODE, 256, 4, true, true, false, false, STR>(a, st);
  else if (bm == 128) launch_fwd_bm<160, MODE, 128, 4, true, true, false, false, STR>(a, st);
  else if (bm == 64) launch_fwd_bm<160, MODE, 64, 2, true, true, false, false, STR>(a, st);
  else throw std::invalid_argument("conv_fwd: 160-wide tiles support tile codes 64 / 128 / 256 / 384-387");
}


template <int BN, int MODE>
static void launch_fwd_t(const ConvFwdArgs& a, hipStream_t st) {
  int bm = a.tile;
  // forward and dgrad: 96x96-per-wave tiles (147 KB LDS).  dgrad used to keep
  // a 112-KB tile so that a wgrad workgroup (48 KB) could share its CU, but the
  // concurrent pair is bound by the same per-CU operand delivery either way;
  // the larger tile moves fewer bytes per MFMA (bench: 106.2k -> 108.5k pos/s,
  // scripts/bench_variants.sh).
  // automatic: 385 (the 384 tile with its DMA spread through the MFMAs);
  // alternating A/B, serial backward: SL 121.5-121.9k vs 120.0-120.7k pos/s,
  // value (160-wide, straddled K-steps) 140.1k vs 136.7k bf16 (profiles/r2_dma_spread.md)
  // automatic (round 3): 386 = 385 with the chunk-outer K order.  10 s power-limited runs at
  // B = 2176 (profiles/r3_chunk_outer.md): 3x3 forward 515 -> 480 us, bitmask dgrad 497 -> 463 us;
  // bench 120.8k -> 126.0k positions/s.  The 160-wide straddled tiles run the same order with the
  // 32-channel tail chunk's steps pairing two taps.
  // Small batches (round 3): below 128 x 256 pixels (B < 91 at 19 x 19) a 64-pixel tile on 4 waves
  // (32 x BN/2 per wave) -- B = 16 fills 91 workgroups instead of 46 (profiles/r3_small_batch.md)
  if (bm == 0) bm = (a.M >= 384 * 512) ? 386 : (a.M >= 256 * 512) ? 256 : (a.M >= 128 * 256) ? 128 : 64;
  if constexpr (BN == 160) {
    if (a.Cin % 64 == 32) launch_fwd_160<MODE, true>(a, bm, st);
    else launch_fwd_160<MODE, false>(a, bm, st);
  } else {
    if (a.Cin % 64 != 0) throw std::invalid_argument("conv_fwd: Cin % 64 == 32 needs the 160-wide tile");
    // production tile codes: 128 / 256 (64-pixel waves), 384 / 385 (96x96 per wave;
    // 385 = default, DMA spread through the MFMAs)
    if (bm == 384) launch_fwd_bm<BN, MODE, 384, 6, false, false>(a, st);
    else if (bm == 256) launch_fwd_bm<BN, MODE, 256, 4>(a, st);
    else if (bm == 128) launch_fwd_bm<BN, MODE, 128, 4>(a, st);
    else if (bm == 64) launch_fwd_bm<BN, MODE, 64, 2>(a, st);
    // 385: the 384 tile with the next stage's LDS-DMA spread through the first
    // k-half's MFMAs instead of issued as one burst (kernel-lab tile 9)
    else if (bm == 385) launch_fwd_bm<BN, MODE, 384, 6, false, false, false, true>(a, st);
    // 386 / 387: 385 / 384 with the chunk-outer K order (CO above)
    else if (bm == 386) launch_fwd_bm<BN, MODE, 384, 6, false, false, false, true, false, true>(a, st);
    else if (bm == 387) launch_fwd_bm<BN, MODE, 384, 6, false, false, false, false, false, true>(a, st);
#ifdef AGK_KERNEL_LAB
    // kernel-lab tile codes (profiles/r1_fwd_kernel_experiments.md):
    // conv_fwd_variants.hip (-1, 2, 4, 5, 6, 32), 2560 (epilogue loads after the loop),
    // 2568 (BM 256, 128-pixel waves), 11 (pixel operand from L2), 9 / 10 (DMA spread
    // through the MFMAs), 7 / 8 (32x32x16 MFMA)
    else if ((bm == -1 || bm == 2 || bm == 4 || bm == 5 || bm == 6 || bm == 32) &&
             launch_conv_fwd_variant(bm, a, MODE, st)) return;
    else if (bm == -1 || bm == 2 || bm == 4 || bm == 5 || bm == 6 || bm == 32) launch_fwd_bm<BN, MODE, 128, 4>(a, st);
    else if (bm == 2560) launch_fwd_bm<BN, MODE, 256, 4, false>(a, st);
    else if (bm == 2568) launch_fwd_bm<BN, MODE, 256, 8>(a, st);
    else if (bm == 11) launch_fwd_ga<BN, MODE>(a, st);
    else if (bm == 9) launch_fwd_bm<BN, MODE, 384, 6, false, false, false, true>(a, st);
    else if (bm == 10) launch_fwd_bm<BN, MODE, 256, 4, false, false, false, true>(a, st);
    else if (bm == 7) launch_fwd_bm<BN, MODE, 384, 6, false, false, true>(a, st);
    else if (bm == 8) launch_fwd_bm<BN, MODE, 256, 4, false, false, true>(a, st);
#endif
    else throw std::invalid_argument("conv_fwd: unknown tile code " + std::to_string(bm));
  }
}


template <int MODE>
static void launch_fwd_mode(const ConvFwdArgs& a, hipStream_t st) {
  if (a.Cout == 160) launch_fwd_t<160, MODE>(a, st);
  else if (a.Cout % 192 == 0) launch_fwd_t<192, MODE>(a, st);
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
// (lgkm_fence / ds_read_tr16_asm: conv_common.h)

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
  // workgroup -> (split, tap group, channel block).  xcd_group (tap-merged rows): the hardware
  // deals workgroups to the 8 XCDs round robin in launch order, which puts the K kernel-row
  // workgroups of a split -- all reading the same dZ rows -- on K different L2s, so every dZ
  // byte comes from the Infinity Cache K times (layer 0: 3 % L2 hits, profiles/r3_small_batch.md).
  // Grouped, each XCD runs a contiguous range of split-major work and a split's rows share an L2.
  int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  if (TAPS > 1 && a.xcd_group) {
    const int gyz = gridDim.y * gridDim.z;
    const int nwg = gridDim.x * gyz;
    const int lin = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    const int xcd = lin & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int l = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (lin >> 3);
    bx = l / gyz;
    const int rem = l - bx * gyz;
    by = rem / gridDim.z;
    bz = rem - by * gridDim.z;
  }
  const int split = bx;
  const int t = by * TAPS;  // first tap of the group
  const int ncb = a.Cin / WC;
  const int n0 = (bz / ncb) * WN;
  const int c0 = (bz % ncb) * WC;
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
#ifdef AGK_DEBUG
#pragma unroll
      for (int i = 0; i < IPW; ++i) {
        const int jj = wave * IPW + i - sub * (NINSTR / KSUB);
        if (jj >= 0 && jj < WN / 16) {
          const long long o = (long long)dzr[sub] + n0 + half + jj * 16;
          const bool ok = AGK_DCHECK(o >= 0 && o + 8 <= a.dz_elems, DBG_WG_DZ);
          glds16(ok ? dsrc + jj * 16 : a.dz, base + sub * SUB + jj * 1024);
        }
      }
#pragma unroll
      for (int i = 0; i < IPW; ++i) {
        const int jj = wave * IPW + i - sub * (NINSTR / KSUB);
        if (jj >= WN / 16 && jj < NINSTR / KSUB) {
          const int xj = jj - WN / 16;  // tap xj / XP, channel piece xj % XP
          const long long o = (long long)xr[sub] + half + (xj / XP) * a.Cin + (xj % XP) * 16;
          const bool ok = AGK_DCHECK(o >= 0 && o + 8 <= a.x_elems, DBG_WG_X);
          glds16(ok ? xsrc + (xj / XP) * a.Cin + (xj % XP) * 16 : a.x, base + sub * SUB + jj * 1024);
        }
      }
#else
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
#endif
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
// ConvWgradArgs::variant: 0 = production 2-buffer kernel (tap-merged rows for
// 64-wide c tiles); kernel-lab build only: 1 = one tap per workgroup,
// 2 = 256-thread tile, 3 / 4 = LDS ring with that many slots

#ifdef AGK_KERNEL_LAB
template <int WN, int WC, int NS>
static void launch_wgrad_ring(const ConvWgradArgs& a, dim3 grid, hipStream_t st) {
  constexpr int smem = NS * (WN + WC) * 64;
  static const hipError_t attr = hipFuncSetAttribute((const void*)conv_wgrad_ring_kernel<WN, WC, NS>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        smem);  // once per instantiation (thread-safe static)
  hip_check(attr, "hipFuncSetAttribute(max dynamic LDS)");
  hipLaunchKernelGGL((conv_wgrad_ring_kernel<WN, WC, NS>), grid, dim3(512), smem, st, a);
}
#endif

template <int WN, int TAPS>
static void launch_wgrad_taps(const ConvWgradArgs& a, hipStream_t st) {
  if (a.cin_real <= 48) {
    // thin first layer (48 real planes padded to 64): a 48-wide c tile on 6
    // waves (2 n x 3 c) skips the zero channels -- 25% fewer MFMAs and x bytes
    // on the backward's serial tail; the slab columns 48..63 stay unwritten
    // (the reduce reads only cin_real of them)
    constexpr int smem = 2 * (WN + 48 * TAPS) * 64 * kWgradKsub;
    static const hipError_t attr48 = hipFuncSetAttribute((const void*)conv_wgrad_kernel<WN, 48, kWgradKsub, 3, TAPS>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, smem);  // once per instantiation (thread-safe static)
  hip_check(attr48, "hipFuncSetAttribute(max dynamic LDS)");
    dim3 grid(a.nsplit, a.T / TAPS, a.Cout / WN);
    hipLaunchKernelGGL((conv_wgrad_kernel<WN, 48, kWgradKsub, 3, TAPS>), grid, dim3(384), smem, st, a);
    return;
  }
  constexpr int smem = 2 * (WN + 64 * TAPS) * 64 * kWgradKsub;
  static const hipError_t attr = hipFuncSetAttribute((const void*)conv_wgrad_kernel<WN, 64, kWgradKsub, 4, TAPS>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, smem);  // once per instantiation (thread-safe static)
  hip_check(attr, "hipFuncSetAttribute(max dynamic LDS)");
  dim3 grid(a.nsplit, a.T / TAPS, (a.Cout / WN) * (a.Cin / 64));
  hipLaunchKernelGGL((conv_wgrad_kernel<WN, 64, kWgradKsub, 4, TAPS>), grid, dim3(512), smem, st, a);
}

int wgrad_tap_group(int Cout, int Cin, int K, int variant) {
  const bool c64 = Cin != 160 && Cin % 192 != 0 && Cin % 128 != 0;
  (void)Cout;
  return (c64 && variant == 0 && (K == 3 || K == 5)) ? K : 1;
}

template <int WN, int WC>
static void launch_wgrad_t(const ConvWgradArgs& a, hipStream_t st) {
  dim3 grid(a.nsplit, a.T, (a.Cout / WN) * (a.Cin / WC));
  constexpr int KS = kWgradKsub;
  constexpr int smem = 2 * (WN + WC) * 64 * KS;
#ifdef AGK_KERNEL_LAB
  if (a.variant == 3 || a.variant == 4) {
    if (a.variant == 3) launch_wgrad_ring<WN, WC, 3>(a, grid, st);
    else launch_wgrad_ring<WN, WC, 4>(a, grid, st);
    return;
  }
  if (a.variant == 2 && WC % 32 == 0 && WC >= 64) {
    static const hipError_t attr2 = hipFuncSetAttribute((const void*)conv_wgrad_kernel<WN, WC, KS, 2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          smem);  // once per instantiation (thread-safe static)
  hip_check(attr2, "hipFuncSetAttribute(max dynamic LDS)");
    hipLaunchKernelGGL((conv_wgrad_kernel<WN, WC, KS, 2>), grid, dim3(256), smem, st, a);
    return;
  }
#else
  if (a.variant != 0) throw std::invalid_argument("conv_wgrad: variant " + std::to_string(a.variant) +
                                                  " is a kernel-lab variant");
#endif
  if constexpr (WC == 64) {
    // tap-merged kernel rows (see conv_wgrad_kernel); lab variant 1 forces one tap per workgroup
    if (a.variant != 1 && (a.K == 3 || a.K == 5)) {
      if (a.K == 3) launch_wgrad_taps<WN, 3>(a, st);
      else launch_wgrad_taps<WN, 5>(a, st);
      return;
    }
  }
  static const hipError_t attr = hipFuncSetAttribute((const void*)conv_wgrad_kernel<WN, WC, KS>, hipFuncAttributeMaxDynamicSharedMemorySize, smem);  // once per instantiation (thread-safe static)
  hip_check(attr, "hipFuncSetAttribute(max dynamic LDS)");
  hipLaunchKernelGGL((conv_wgrad_kernel<WN, WC, KS>), grid, dim3(512), smem, st, a);
}

// 160 x 160 tile on 4 waves (2 n x 2 c, 80 x 80 per wave): the value net's
// padded width; 40 KB of LDS, so several workgroups share a CU
static void launch_wgrad_160x160(const ConvWgradArgs& a, hipStream_t st) {
  if (a.variant != 0) throw std::invalid_argument("conv_wgrad: 160-wide tiles have no lab variants");
  constexpr int KS = kWgradKsub;
  constexpr int smem = 2 * (160 + 160) * 64 * KS;
  static const hipError_t attr = hipFuncSetAttribute((const void*)conv_wgrad_kernel<160, 160, KS, 2>,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, smem);
  hip_check(attr, "hipFuncSetAttribute(max dynamic LDS)");
  dim3 grid(a.nsplit, a.T, 1);
  hipLaunchKernelGGL((conv_wgrad_kernel<160, 160, KS, 2>), grid, dim3(256), smem, st, a);
}

int wgrad_stage_pixels() { return 32 * kWgradKsub; }

#ifdef AGK_DEBUG
unsigned debug_error_fetch_and_clear(hipStream_t st) {
  hip_check(hipStreamSynchronize(st), "debug: stream synchronize");
  unsigned code = 0, zero = 0;
  hip_check(hipMemcpyFromSymbol(&code, HIP_SYMBOL(g_dbg_err), sizeof(code)), "debug: read error word");
  if (code) hip_check(hipMemcpyToSymbol(HIP_SYMBOL(g_dbg_err), &zero, sizeof(zero)), "debug: clear error word");
  return code;
}
#endif

void wgrad_plan(int Cout, int Cin, int cin_real, int K, int variant, int out[3]) {
  const int code = variant == 5 ? wgrad_row_code(Cout, Cin, cin_real, K) : 0;
  if (code) {  // one kernel row per workgroup, one workgroup per CU (~170 VGPRs, 8 or 6 waves)
    out[0] = K;
    out[1] = wgrad_row_wgs_per_split(code, Cout, Cin, cin_real, K);
    out[2] = 1;
    return;
  }
  // per-tap kernel: tap-merged rows for 64-wide c tiles, else one tap; two workgroups per CU
  const int taps = wgrad_tap_group(Cout, Cin, K, variant == 5 ? 0 : variant);
  const bool c48 = cin_real <= 48 && Cin == 64;
  const int wn = Cout == 160 ? 160 : Cout % 192 == 0 ? 192 : Cout % 128 == 0 ? 128 : 64;
  const int wc = Cout == 160 && Cin == 160 ? 160 : Cin % 192 == 0 ? 192 : Cin % 128 == 0 ? 128 : 64;
  out[0] = taps;
  out[1] = (K * K / taps) * (Cout / wn) * (c48 ? 1 : Cin / wc);
  out[2] = 2;
}

static int wgrad_xcd_group() {
  static const int on = [] {
    const char* e = getenv("AGK_WGRAD_XCD");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  return on;
}

void launch_conv_wgrad(const ConvWgradArgs& a_in, hipStream_t st) {
  ConvWgradArgs a = a_in;
  a.divSS = make_fastdiv((uint32_t)(a.S * a.S));
  a.divS = make_fastdiv((uint32_t)a.S);
  a.xcd_group = wgrad_xcd_group();
  if (a.variant == 5) {
    // one-kernel-row wgrad (conv_wgrad_row.hip), opt-in: in the power-limited steady state it ran
    // 607-694 us per 192 -> 192 layer against 548-583 us for the per-tap kernel
    // (profiles/r3_wgrad_row.md); layers it does not cover run the per-tap kernel
    const int code = wgrad_row_code(a.Cout, a.Cin, a.cin_real, a.K);
    if (code) {
      wgrad_row_launch(code, a, st);
      return;
    }
    a.variant = 0;
  }
  const bool n192 = a.Cout % 192 == 0, c192 = a.Cin % 192 == 0;
  const bool n128 = a.Cout % 128 == 0, c128 = a.Cin % 128 == 0;
  if (a.Cout == 160) {  // value net (152 filters padded to 160)
    if (a.Cin == 160) launch_wgrad_160x160(a, st);
    else if (a.Cin % 64 == 0 && a.Cin % 128 != 0 && a.Cin % 192 != 0) launch_wgrad_t<160, 64>(a, st);
    else throw std::invalid_argument("conv_wgrad: Cout 160 supports Cin 160 or an odd multiple of 64");
  } else if (a.Cin == 160) {
    throw std::invalid_argument("conv_wgrad: Cin 160 needs Cout 160");
  } else if (n192 && c192) launch_wgrad_t<192, 192>(a, st);
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
// Fixed summation order per element (deterministic): four partial sums over
// the splits, s_k = sum of splits sp = k (mod 4) below the last multiple of 4
// in increasing order, the leftover splits added to s_0, then
// (s0 + s1) + (s2 + s3).  Wave k of a 256-thread block computes s_k for 64
// float4 elements (4 consecutive input channels of one tap and output
// channel), 4 16-B loads in flight; the four partials meet in LDS.  The OIHW
// write is strided but touches the (small) gradient once.
__global__ __launch_bounds__(256) void conv_wgrad_reduce_kernel(WgradReduceArgs a) {
  __shared__ f32x4 part[4][64];
  const int C4 = a.Cin >> 2;
  const int total = a.T * a.Cout_real * C4;
  const size_t tile = (size_t)a.Cout * a.Cin;
  const size_t sstride = (size_t)a.T * tile;
  const int k = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n4 = a.nsplit & ~3;
  for (int base = blockIdx.x * 64; base < total; base += gridDim.x * 64) {  // block-uniform trip count
    const int idx = base + lane;
    const int e = idx < total ? idx : total - 1;
    const int c = (e % C4) << 2;
    const int tn = e / C4;
    const int n = tn % a.Cout_real;
    const int t = tn / a.Cout_real;
    const float* s = a.slab + (size_t)t * tile + (size_t)n * a.Cin + c;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if (c < a.Cin_real) {
      int sp = k;
      for (; sp + 12 < n4; sp += 16) {
        const f32x4 v0 = *(const f32x4*)(s + (size_t)sp * sstride);
        const f32x4 v1 = *(const f32x4*)(s + (size_t)(sp + 4) * sstride);
        const f32x4 v2 = *(const f32x4*)(s + (size_t)(sp + 8) * sstride);
        const f32x4 v3 = *(const f32x4*)(s + (size_t)(sp + 12) * sstride);
        acc += v0;
        acc += v1;
        acc += v2;
        acc += v3;
      }
      for (; sp < n4; sp += 4) acc += *(const f32x4*)(s + (size_t)sp * sstride);
      if (k == 0)
        for (sp = n4; sp < a.nsplit; ++sp) acc += *(const f32x4*)(s + (size_t)sp * sstride);
    }
    part[k][lane] = acc;
    __syncthreads();
    if (k == 0 && idx < total && c < a.Cin_real) {
      const f32x4 sum = (part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane]);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (c + i >= a.Cin_real) break;
        float* g = a.grad_w + ((size_t)n * a.Cin_real + c + i) * a.T + t;
        *g = (a.beta != 0.f ? a.beta * *g : 0.f) + a.scale * sum[i];  // beta 0: no read of g
      }
    }
    __syncthreads();
  }
  if (blockIdx.x == gridDim.x - 1 && a.grad_b) {
    // bias: one sequential sum per channel (fixed order) with 8 loads in flight --
    // a load-add chain of nsplit dependent steps set this kernel's duration
    for (int n = threadIdx.x; n < a.Cout_real; n += blockDim.x) {
      const float* d = a.dbias_slab + n;
      float sum = 0.f;
      int sp = 0;
      for (; sp + 8 <= a.nsplit; sp += 8) {
        float v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = d[(size_t)(sp + k) * a.Cout];
#pragma unroll
        for (int k = 0; k < 8; ++k) sum += v[k];
      }
      for (; sp < a.nsplit; ++sp) sum += d[(size_t)sp * a.Cout];
      a.grad_b[n] = a.beta * a.grad_b[n] + a.scale * sum;
    }
  }
}

void launch_wgrad_reduce(const WgradReduceArgs& a, hipStream_t st) {
  const int total = a.T * a.Cout_real * (a.Cin >> 2);
  int blocks = (total + 63) / 64;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(conv_wgrad_reduce_kernel, dim3(blocks), dim3(256), 0, st, a);
}

}  // namespace agk
