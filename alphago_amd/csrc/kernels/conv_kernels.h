// Conv kernel templates shared by the production launchers (conv.hip) and the kernel lab
// (conv_lab.hip): the implicit-GEMM forward / dgrad kernel and the split-K wgrad kernel.  See conv.hip
// for the layout and the algorithm.
#pragma once
#include <hip/hip_runtime.h>

#include <stdexcept>

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
// NS > 2 (small batches): an NS-slot LDS ring, the DMA of step ks + NS - 1 issued while step ks
// computes.  With few workgroups per CU nothing else hides the global->LDS latency of a 2-buffer
// loop (~0.75 us per K-step at B = 16, 27 steps per 3x3 layer: profiles/r3_small_batch/).
// SK (split-K, small batches): blockIdx.z = split z of gridDim.z; the workgroup runs K-steps
// [nK z / nz, nK (z+1) / nz) and writes its raw fp32 partial tile to a.sk_ws[z][m][n];
// conv_splitk_finish_kernel sums the splits and applies the epilogue.  At B = 16 a 3x3 layer is 181
// 32-pixel tiles of 27 serial K-steps (~0.7 us each, whatever the DMA scheme): splitting K shortens
// that chain and fills the CUs.
template <int BN, int MODE, int BM, int MBW, bool EPF = true, bool PIPE = true, bool M32 = false, bool ILV = false,
          bool STR = false, bool CO = false, int NS = 2, bool SK = false>
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
  if constexpr (NS > 2) {
    static_assert(PIPE && !M32 && !ILV && !BDIST, "ring: the pipelined 16x16 loop");
    // DMA instructions per wave per stage (the vmcnt unit of one stage)
    constexpr int PW = A_INSTR + B_INSTR;
    static_assert(PW * (NS - 2) <= 63, "vmcnt range");
#pragma unroll
    for (int s = 0; s < NS - 1; ++s)
      if (s < nK) stage(s);  // workgroup-uniform
    for (int ks = 0; ks < nK; ++ks) {
      // step ks has landed once at most (stages issued after it) x PW DMAs are outstanding
      const int later = (nK - 1 - ks) < (NS - 2) ? (nK - 1 - ks) : (NS - 2);
      ring_wait<PW, NS - 2>(later);
      __syncthreads();  // every wave's DMA of step ks is visible; slot (ks - 1) % NS is free
      if (ks + NS - 1 < nK) stage((ks + NS - 1) % NS);
      const char* base = smem + (ks % NS) * STAGE;
      read_frags(base, 0, xa, wa);
      read_frags(base, 1, xb, wb);
      if (ks == ep_at) ep.load(a, ep_mrow, ep_nbase, wn);
      __builtin_amdgcn_s_setprio(1);
      mfmas(xa, wa);
      mfmas(xb, wb);
      __builtin_amdgcn_s_setprio(0);
    }
    ep.store(a, acc, ep_mrow);
    return;
  }
  if constexpr (SK) {
    static_assert(PIPE && !M32 && !ILV && !CO, "split-K: the pipelined 2-buffer loop, tap-outer order");
    const int z = blockIdx.z, nz = gridDim.z;
    const int kb = (int)((long)nK * z / nz), ke = (int)((long)nK * (z + 1) / nz);
    for (int i = 0; i < kb; ++i) st_advance();  // scalar cursor to step kb
    if (kb < ke) {  // workgroup-uniform
      stage(0);
      wait_vmcnt0();
      __syncthreads();
      read_frags(smem, 0, xa, wa);
      for (int ks = kb; ks < ke; ++ks) {
        const int cur = (ks - kb) & 1;
        const char* base = smem + cur * STAGE;
        if (ks + 1 < ke) stage(cur ^ 1);
        read_frags(base, 1, xb, wb);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
        mfmas(xa, wa);
        mfmas(xb, wb);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        wait_vmcnt0();
        __syncthreads();
        if (ks + 1 < ke) read_frags(smem + (cur ^ 1) * STAGE, 0, xa, wa);
      }
    }
    // raw partial sums: lane owns channels ep_nbase + 16 i + [0, 4) of pixel ep_mrow + 16 j
    float* ws = a.sk_ws + (size_t)z * a.M * a.Cout;
#pragma unroll
    for (int j = 0; j < MB; ++j) {
      const int m = ep_mrow + j * 16;
      if (m >= a.M) continue;
#pragma unroll
      for (int i = 0; i < NB; ++i) *(f32x4*)(ws + (size_t)m * a.Cout + ep_nbase + i * 16) = acc[i][j];
    }
    return;
  }
  int xo00, xo01;  // step 0's source offsets (ILV: the re-staged operands when nK == 1)
  size_t wo00, wo01;
  st_offsets(xo00, xo01, wo00, wo01);
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
    // The last step re-stages its own (in-range) operands into the idle buffer instead of
    // branching around each DMA piece: a uniform `if (more)` compiled to one s_cbranch per piece
    // inside the MFMA stream.
    int lxo0 = xo00, lxo1 = xo01;
    size_t lwo0 = wo00, lwo1 = wo01;
    for (int ks = 0; ks < nK; ++ks) {
      const int cur = ks & 1;
      const char* base = smem + cur * STAGE;
      const bool more = ks + 1 < nK;
      read_frags(base, 0, xa, wa);
      char* nb = smem + (cur ^ 1) * STAGE;
      int xo0, xo1;
      size_t wo0, wo1;
      st_offsets(xo0, xo1, wo0, wo1);
      xo0 = more ? xo0 : lxo0;
      xo1 = more ? xo1 : lxo1;
      wo0 = more ? wo0 : lwo0;
      wo1 = more ? wo1 : lwo1;
      lxo0 = xo0;
      lxo1 = xo1;
      lwo0 = wo0;
      lwo1 = wo1;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int d = 0; d < NDMA; ++d) {
        mfma_range(d * MPD, (d + 1) * MPD);
        __builtin_amdgcn_sched_barrier(0);
        st_piece(d, nb, xo0, xo1, wo0, wo1);
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

template <int BN, int MODE, int BM, int MBW, bool EPF = true, bool PIPE = true, bool M32 = false, bool ILV = false,
          bool STR = false, bool CO = false, int NS = 2>
static void launch_fwd_bm(const ConvFwdArgs& a, hipStream_t st) {
  constexpr int smem = NS * (BM * 128 + BN * 128);
  static_assert(smem <= 160 * 1024, "LDS");
  static const hipError_t attr = hipFuncSetAttribute(
      (const void*)conv_fwd_kernel<BN, MODE, BM, MBW, EPF, PIPE, M32, ILV, STR, CO, NS>,
      hipFuncAttributeMaxDynamicSharedMemorySize, smem);  // once per instantiation (thread-safe static)
  hip_check(attr, "hipFuncSetAttribute(max dynamic LDS)");
  dim3 grid((a.M + BM - 1) / BM, a.Cout / BN);
  hipLaunchKernelGGL((conv_fwd_kernel<BN, MODE, BM, MBW, EPF, PIPE, M32, ILV, STR, CO, NS>), grid,
                     dim3(BM / MBW * 8), smem, st, a);
}

// Split-K finish: one thread per (pixel, bitmask word); word w of a pixel covers the channels
// tn * BN + wn * BN/2 + 4 q + 16 i + r (tn = w / 8, wn = (w / 4) % 2, q = w % 4; i < NB = BN / 32,
// r < 4) -- the channels one lane of the conv epilogue owns, so the bitmask layout is the tile's.
template <int MODE, int NB>
__global__ __launch_bounds__(256) void conv_splitk_finish_kernel(ConvFwdArgs a) {
  constexpr int BN = 32 * NB;
  const int WPP = (a.Cout / BN) * 8;
  const long gid = (long)blockIdx.x * 256 + threadIdx.x;
  if (gid >= (long)a.M * WPP) return;
  const int m = (int)(gid / WPP), w = (int)(gid - (long)m * WPP);
  const int base = (w >> 3) * BN + ((w >> 2) & 1) * (BN / 2) + 4 * (w & 3);
  f32x4 v[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) v[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int z = 0; z < a.sk_nsplit; ++z) {
    const float* src = a.sk_ws + ((size_t)z * a.M + m) * a.Cout + base;
#pragma unroll
    for (int i = 0; i < NB; ++i) v[i] += *(const f32x4*)(src + 16 * i);
  }
  const int SS = a.S * a.S;
  const int b = fdiv(m, a.divSS);
  const int rem = m - b * SS;
  const int ii = fdiv(rem, a.divS);
  const int jj = rem - ii * a.S;
  const size_t pix = (size_t)(b * a.HPo + ii + a.Po) * a.HPo + jj + a.Po;
  uint32_t mw = 0u, bits = 0u;
  if constexpr (MODE == MODE_MASKBITS) mw = a.mbits_in[pix * WPP + w];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    float o4[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float x = v[i][r];
      if constexpr (MODE == MODE_BIAS_RELU) x = fmaxf(x + a.bias[base + 16 * i + r], 0.f);
      if constexpr (MODE == MODE_MASKBITS) x = ((mw >> (4 * i + r)) & 1u) ? x : 0.f;
      o4[r] = x;
    }
    bf16x4 o;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      o[r] = (__bf16)o4[r];
      if constexpr (MODE == MODE_BIAS_RELU) bits |= ((float)o[r] > 0.f ? 1u : 0u) << (4 * i + r);
    }
    *(bf16x4*)(a.y + pix * a.Cout + base + 16 * i) = o;
  }
  if constexpr (MODE == MODE_BIAS_RELU)
    if (a.mbits_out) a.mbits_out[pix * WPP + w] = bits;
}

// tile code 38: the 32-pixel tile (36) with split-K over a.sk_nsplit workgroups per tile, then the finish
// (BN = 160, the value width: STR straddled K-steps when Cin % 64 == 32, weight pieces dealt round-robin)
template <int BN, int MODE, bool STR = false>
static void launch_fwd_splitk(const ConvFwdArgs& a, hipStream_t st) {
  if constexpr (MODE == MODE_MASK) {
    throw std::invalid_argument("conv_fwd split-K: modes 0 (bias + ReLU), 2 (none) and 3 (bitmask dgrad)");
  } else {
    if (!a.sk_ws || a.sk_nsplit < 1 || a.y_bf8)
      throw std::invalid_argument("conv_fwd split-K (tile 38): needs a workspace and nsplit >= 1, no e5m2 copy");
    constexpr int BM = 32, MBW = 1;
    constexpr int smem = 2 * (BM * 128 + BN * 128);
    static const hipError_t attr = hipFuncSetAttribute(
        (const void*)conv_fwd_kernel<BN, MODE, BM, MBW, true, true, false, false, STR, false, 2, true>,
        hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    hip_check(attr, "hipFuncSetAttribute(max dynamic LDS)");
    dim3 grid((a.M + BM - 1) / BM, a.Cout / BN, a.sk_nsplit);
    hipLaunchKernelGGL((conv_fwd_kernel<BN, MODE, BM, MBW, true, true, false, false, STR, false, 2, true>), grid,
                       dim3(BM / MBW * 8), smem, st, a);
    const long threads = (long)a.M * (a.Cout / BN) * 8;
    hipLaunchKernelGGL((conv_splitk_finish_kernel<MODE, BN / 32>), dim3((unsigned)((threads + 255) / 256)), dim3(256),
                       0, st, a);
  }
}

// ----------------------------------------------------------------- packed-tap forward (thin first layer)
// The first layer's input has cin_real <= 64 real planes in a 64-channel padded tensor (48 policy,
// 49 value).  conv_fwd_kernel multiplies all 64 channels of every tap, so a quarter of the layer-0
// MACs are zeros.  Here the K loop runs over (tap, 8-channel chunk) pairs of the real channels only:
// cpt = ceil(cin_real / 8) chunks per tap, 8 chunks (one 64-wide K-step) per step, chunk j of step s
// is q = 8 s + j = (tap q / cpt, channels 8 (q % cpt) ..).  48 planes: 25 x 6 = 150 chunks in 19 steps
// instead of 25.  Weights packed [step][Cout][64] in the same chunk order (pack_weights_kernel with
// PackLayer::pk_cpt), zero past the last chunk.  Each lane's DMA source is its own (tap, chunk): the
// wave-uniform step state keeps the offsets of taps t0, t0 + 1, t0 + 2 (a step spans at most three
// taps when cpt >= 4) and a piece selects one of them.  The MFMA loop, LDS layout and epilogue are
// those of the 384-pixel tile (96 x 96 per wave, one DMA burst per step).
template <int BN, int BM, int MBW>
__global__ __launch_bounds__(BM / MBW * 8, 1) void conv_fwd_pk_kernel(ConvFwdArgs a, int cpt) {
  constexpr int NW = BM / (16 * MBW) * 2;
  constexpr int NB = BN / 32;
  constexpr int MB = MBW;
  constexpr int A_BYTES = BM * 128;
  constexpr int B_BYTES = BN * 128;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int A_ROWS_PW = BM / NW;
  constexpr int A_INSTR = A_ROWS_PW / 8;
  constexpr bool BDIST = (BN / NW) % 8 != 0;
  constexpr int B_ROWS_PW = BN / NW;
  constexpr int B_INSTR = BDIST ? (BN / 8 + NW - 1) / NW : B_ROWS_PW / 8;
  static_assert(BN % 32 == 0 && A_ROWS_PW % 8 == 0, "tile geometry");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int lane = threadIdx.x & 63;
  const int wave = wave_id();
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int SS = a.S * a.S;
  const int T = a.K * a.K;
  const int nK = (T * cpt + 7) >> 3;

  int arow[A_INSTR], alg[A_INSTR];
#pragma unroll
  for (int i = 0; i < A_INSTR; ++i) {
    const int r = wave * A_ROWS_PW + i * 8 + (lane >> 3);
    int m = m0 + r;
    m = m < a.M ? m : a.M - 1;
    const int b = fdiv(m, a.divSS);
    const int rem = m - b * SS;
    const int ii = fdiv(rem, a.divS);
    const int jj = rem - ii * a.S;
    alg[i] = (lane & 7) ^ ((r >> 1) & 7);
    arow[i] = ((b * a.HPi + ii + a.offi) * a.HPi + jj + a.offi) * a.Cin;
  }
  int brow[B_INSTR], bldsrow[B_INSTR];
#pragma unroll
  for (int i = 0; i < B_INSTR; ++i) {
    const int piece = BDIST ? wave + i * NW : wave * (B_ROWS_PW / 8) + i;
    const int r = piece * 8 + (lane >> 3);
    const int logical = (lane & 7) ^ ((r >> 1) & 7);
    brow[i] = (n0 + (r < BN ? r : BN - 1)) * 64 + logical * 8;
    bldsrow[i] = piece * 8;
  }

  // wave-uniform staging cursor: first chunk st_c of tap st_t = (st_kh, st_kw), weight step offset
  int st_c = 0, st_t = 0, st_kh = 0, st_kw = 0;
  size_t st_w = 0;
  const size_t wstep = (size_t)a.Cout * 64;
  auto stage = [&](int buf) {
    char* base = smem + buf * STAGE;
    // offsets of taps st_t, st_t + 1, st_t + 2 (past the last tap: the last tap's pixels, zero weights)
    int kh1 = st_kh, kw1 = st_kw + 1;
    if (kw1 == a.K) { kw1 = 0; ++kh1; }
    int kh2 = kh1, kw2 = kw1 + 1;
    if (kw2 == a.K) { kw2 = 0; ++kh2; }
    const int o0 = (st_kh * a.HPi + st_kw) * a.Cin;
    const int o1 = st_t + 1 < T ? (kh1 * a.HPi + kw1) * a.Cin : o0;
    const int o2 = st_t + 2 < T ? (kh2 * a.HPi + kw2) * a.Cin : o1;
#pragma unroll
    for (int i = 0; i < A_INSTR; ++i) {
      const int e = st_c + alg[i];
      const int dt = (e >= cpt ? 1 : 0) + (e >= 2 * cpt ? 1 : 0);
      const int off = (dt == 0 ? o0 : dt == 1 ? o1 : o2) + (e - dt * cpt) * 8;
#ifdef AGK_DEBUG
      const int xo = arow[i] + off;
      const bool ok = AGK_DCHECK(xo >= 0 && (long long)xo + 8 <= a.x_elems, DBG_FWD_X);
      glds16(a.x + (ok ? xo : 0), base + (wave * A_ROWS_PW + i * 8) * 128);
#else
      glds16(a.x + arow[i] + off, base + (wave * A_ROWS_PW + i * 8) * 128);
#endif
    }
#pragma unroll
    for (int i = 0; i < B_INSTR; ++i) {
      if (BDIST && wave + i * NW >= BN / 8) continue;  // wave-uniform
#ifdef AGK_DEBUG
      const bool ok = AGK_DCHECK((long long)(st_w + brow[i]) + 8 <= a.w_elems, DBG_FWD_W);
      glds16(ok ? a.w + st_w + brow[i] : a.w, base + A_BYTES + bldsrow[i] * 128);
#else
      glds16(a.w + st_w + brow[i], base + A_BYTES + bldsrow[i] * 128);
#endif
    }
    // advance by 8 chunks (at most two tap boundaries when cpt >= 4)
    st_w += wstep;
    st_c += 8;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      if (st_c >= cpt) {
        st_c -= cpt;
        ++st_t;
        if (++st_kw == a.K) { st_kw = 0; ++st_kh; }
      }
    }
  };

  f32x4 acc[NB][MB];
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int j = 0; j < MB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int swz = (lane & 15) >> 1;
  const int xrow0 = (wm * 16 * MB + (lane & 15)) * 128;
  const int wrow0 = A_BYTES + (wn * (BN / 2) + (lane & 15)) * 128;
  bf16x8 xf[MB], wf[NB];
  ConvEpilogue<NB, MB, MODE_BIAS_RELU> ep;
  const int ep_mrow = m0 + wm * 16 * MB + (lane & 15);
  const int ep_nbase = n0 + wn * (BN / 2) + ((lane >> 4) << 2);

  stage(0);
  wait_vmcnt0();
  __syncthreads();
  for (int ks = 0; ks < nK; ++ks) {
    const int cur = ks & 1;
    const char* base = smem + cur * STAGE;
    if (ks + 1 < nK) stage(cur ^ 1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int choff = (((kk << 2) + (lane >> 4)) ^ swz) << 4;
#pragma unroll
      for (int j = 0; j < MB; ++j) xf[j] = *(const bf16x8*)(base + xrow0 + j * 16 * 128 + choff);
#pragma unroll
      for (int i = 0; i < NB; ++i) wf[i] = *(const bf16x8*)(base + wrow0 + i * 16 * 128 + choff);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < NB; ++i)
#pragma unroll
        for (int j = 0; j < MB; ++j) acc[i][j] = mfma16x16x32(wf[i], xf[j], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
    }
    wait_vmcnt0();
    __syncthreads();
  }
  ep.load(a, ep_mrow, ep_nbase, wn);
  ep.store(a, acc, ep_mrow);
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
// the split's partial tile D[n][c] (lane owns n..n+3 at column c) and the bias partial
template <int WN, int WC, int NWC, int TAPS, int NWN = 2>
__device__ __forceinline__ void wgrad_store(const ConvWgradArgs& a,
                                            const f32x4 (&acc)[TAPS][WN / (16 * NWN)][WC / (16 * NWC)],
                                            const float (&dbs)[WN / (16 * NWN)], bool do_bias, int split, int t,
                                            int n0, int c0, int wn, int wc, int lane, int zero_split) {
  constexpr int NBn = WN / (16 * NWN), NBc = WC / (16 * NWC);
  const int nb0 = n0 + wn * (WN / NWN) + ((lane >> 4) << 2);
  const int cbase = c0 + wc * (WC / NWC) + (lane & 15);
  if (a.grad_w) {  // split-free plan: this workgroup holds the whole pixel sum -> the OIHW gradient
    const float sc = a.scale, be = a.beta;
#pragma unroll
    for (int tp = 0; tp < TAPS; ++tp)
#pragma unroll
      for (int i = 0; i < NBn; ++i)
#pragma unroll
        for (int j = 0; j < NBc; ++j) {
          const int c = cbase + j * 16;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int n = nb0 + i * 16 + r;
            if (n < a.cout_real && c < a.cin_real) {
              float* g = a.grad_w + ((size_t)n * a.cin_real + c) * a.T + t + tp;
              *g = (be != 0.f ? be * *g : 0.f) + sc * acc[tp][i][j][r];  // beta 0: no read of g
            }
          }
        }
    if (do_bias && a.grad_b) {
#pragma unroll
      for (int i = 0; i < NBn; ++i) {
        float s = dbs[i];
        s += __shfl_xor(s, 16, 64);
        s += __shfl_xor(s, 32, 64);
        const int n = n0 + wn * (WN / NWN) + i * 16 + lane;
        if (lane < 16 && n < a.cout_real) a.grad_b[n] = (be != 0.f ? be * a.grad_b[n] : 0.f) + sc * s;
      }
    }
    return;
  }
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
  if (zero_split >= 0) {  // PAIR's odd tap: the second split it covered contributes zeros
    float* out = a.slab + ((size_t)zero_split * a.T + t) * (size_t)a.Cout * a.Cin;
#pragma unroll
    for (int i = 0; i < NBn; ++i)
#pragma unroll
      for (int j = 0; j < NBc; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) out[(size_t)(nb0 + i * 16 + r) * a.Cin + cbase + j * 16] = 0.f;
  }
  if (do_bias) {
#pragma unroll
    for (int i = 0; i < NBn; ++i) {
      float s = dbs[i];
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      if (lane < 16) a.dbias_slab[(size_t)split * a.Cout + n0 + wn * (WN / NWN) + i * 16 + lane] = s;
    }
  }
}


// PAIR (3x3 only, with TAPS == 2, KSUB == 2): a workgroup owns two consecutive taps t, t+1 of
// any kernel rows (tstep = the element offset from tap t's x image to tap t+1's) and reuses each
// staged dz tile for both; per 64-pixel stage it moves 72 KB for 4.7 M MACs -- the forward's
// ratio and its one workgroup per CU -- instead of the per-tap kernel's 24 KB for 1.2 M.  The
// odd last tap (K*K = 9) runs the one-tap body over two splits' pixels, so every workgroup of
// the grid does the same MFMA work; it writes its sum into the first split's slab and zeros
// into the second's.
// NS > 2 (small batches): an NS-slot LDS ring instead of the double buffer (see conv_fwd_kernel);
// only for geometries whose waves each stage exactly IPW pieces per stage (the vmcnt unit).
// NWN: waves along n (2; the thin first layer's 12-wave variant has 4, see launch_wgrad_taps48).
// UP: unit pipelining inside a sub-step -- the x fragments of column unit u + 1 (a (tap, c block)
// pair) are read while the MFMAs of unit u run, instead of every fragment before the first MFMA;
// only the dz fragments and unit 0 stay exposed after the barrier.
template <int WN, int WC, int KSUB, int NWC, int TAPS, int NS = 2, int NWN = 2, bool UP = false>
__device__ __forceinline__ void wgrad_tile(const ConvWgradArgs& a, int split, int ks_begin, int ks_end, int t,
                                           int tstep, int n0, int c0, int zero_split) {
  // NWN (n) x NWC (c) waves; NWC = 2 gives each wave a 96x96 tile at 192x192
  // (a third fewer LDS fragment reads per MFMA than NWC = 4)
  constexpr int NWAVES = NWN * NWC;
  constexpr int NBn = WN / (16 * NWN);  // n blocks per wave (wave covers WN/NWN)
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
  const int kh = t / a.K, kw = t - (t / a.K) * a.K;
  const int toff = (kh * a.HPi + kw) * a.Cin + c0;
  const int SS = a.S * a.S;

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
        if constexpr (NS > 2) {  // see the release loop below
          if (jj >= NINSTR / KSUB) glds16(dsrc, base + sub * SUB);
        }
      }
#pragma unroll
      for (int i = 0; i < IPW; ++i) {
        const int jj = wave * IPW + i - sub * (NINSTR / KSUB);
        if (jj >= WN / 16 && jj < NINSTR / KSUB) {
          const int xj = jj - WN / 16;  // tap xj / XP, channel piece xj % XP
          const long long o = (long long)xr[sub] + half + (xj / XP) * tstep + (xj % XP) * 16;
          const bool ok = AGK_DCHECK(o >= 0 && o + 8 <= a.x_elems, DBG_WG_X);
          glds16(ok ? xsrc + (xj / XP) * tstep + (xj % XP) * 16 : a.x, base + sub * SUB + jj * 1024);
        }
      }
#else
      if constexpr (KSUB == 1 && (WN / 16) % IPW == 0 && NINSTR == NWAVES * IPW) {
        // every wave stages only dz pieces or only x pieces: one scalar branch per stage instead of
        // one per piece
        if (wave < (WN / 16) / IPW) {
#pragma unroll
          for (int i = 0; i < IPW; ++i) glds16(dsrc + (wave * IPW + i) * 16, base + (wave * IPW + i) * 1024);
        } else {
#pragma unroll
          for (int i = 0; i < IPW; ++i) {
            const int xj = wave * IPW + i - WN / 16;  // tap xj / XP, channel piece xj % XP
            glds16(xsrc + (xj / XP) * tstep + (xj % XP) * 16, base + (WN / 16 + xj) * 1024);
          }
        }
        continue;
      }
#pragma unroll
      for (int i = 0; i < IPW; ++i) {
        const int jj = wave * IPW + i - sub * (NINSTR / KSUB);
        if (jj >= 0 && jj < WN / 16) glds16(dsrc + jj * 16, base + sub * SUB + jj * 1024);
        // LDS ring with unequal piece counts: a wave past the last piece re-issues dz piece 0 (same
        // bytes to the same LDS address), so every wave has exactly IPW DMAs per stage -- the
        // vmcnt unit ring_wait counts in
        if constexpr (NS > 2) {
          if (jj >= NINSTR / KSUB) glds16(dsrc, base + sub * SUB);
        }
      }
#pragma unroll
      for (int i = 0; i < IPW; ++i) {
        const int jj = wave * IPW + i - sub * (NINSTR / KSUB);
        if (jj >= WN / 16 && jj < NINSTR / KSUB) {
          const int xj = jj - WN / 16;  // tap xj / XP, channel piece xj % XP
          glds16(xsrc + (xj / XP) * tstep + (xj % XP) * 16, base + sub * SUB + jj * 1024);
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

  constexpr bool RING = NS > 2;
  static_assert(!RING || KSUB == 1, "ring: one sub-step per stage");
  static_assert(!RING || IPW * (NS - 2) <= 63, "vmcnt range");
  if constexpr (RING) {
#pragma unroll
    for (int s = 0; s < NS - 1; ++s)
      if (ks_begin + s < ks_end) stage(ks_begin + s, s);
  } else if (ks_begin < ks_end) {
    stage(ks_begin, 0);
    wait_vmcnt0();
    __syncthreads();
  }
  for (int ks = ks_begin; ks < ks_end; ++ks) {
    int cur = (ks - ks_begin) & 1;
    if constexpr (RING) {
      const int later = (ks_end - 1 - ks) < (NS - 2) ? (ks_end - 1 - ks) : (NS - 2);
      ring_wait<IPW, (NS > 2 ? NS - 2 : 0)>(later);
      __syncthreads();  // stage ks visible to every wave; the slot read last step is free
      cur = (ks - ks_begin) % NS;
      if (ks + NS - 1 < ks_end) stage(ks + NS - 1, (ks - ks_begin + NS - 1) % NS);
    } else if (ks + 1 < ks_end) {
      stage(ks + 1, cur ^ 1);
    }
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
      if constexpr (UP) {
        constexpr int NU = TAPS * NBc;  // column units u = tp * NBc + j
        auto read_unit = [&](int u) {
          const char* cb = base + DZ_BYTES + ((u / NBc) * XP + wc * NBc + (u % NBc)) * 1024;
          tl[NBn + u] = ds_read_tr16_asm(cb + tr0);
          th[NBn + u] = ds_read_tr16_asm(cb + tr1);
        };
        read_unit(0);
        bf16x8 af[NBn];
#pragma unroll
        for (int u = 0; u < NU; ++u) {
          if (u + 1 < NU) read_unit(u + 1);
          // all but the two reads of unit u + 1 have returned (LDS reads complete in order)
          if (u == 0) {
#pragma unroll
            for (int i = 0; i < NBn; ++i) {
              if (NU > 1) lgkm_wait_pair<2>(tl[i], th[i]);
              else lgkm_wait_pair<0>(tl[i], th[i]);
              af[i] = bf16x8{tl[i][0], tl[i][1], tl[i][2], tl[i][3], th[i][0], th[i][1], th[i][2], th[i][3]};
            }
          }
          if (u + 1 < NU) lgkm_wait_pair<2>(tl[NBn + u], th[NBn + u]);
          else lgkm_wait_pair<0>(tl[NBn + u], th[NBn + u]);
          const bf16x8 bu = bf16x8{tl[NBn + u][0], tl[NBn + u][1], tl[NBn + u][2], tl[NBn + u][3],
                                   th[NBn + u][0], th[NBn + u][1], th[NBn + u][2], th[NBn + u][3]};
#pragma unroll
          for (int i = 0; i < NBn; ++i) acc[u / NBc][i][u % NBc] = mfma16x16x32(af[i], bu, acc[u / NBc][i][u % NBc]);
        }
        if (do_bias) {
#pragma unroll
          for (int i = 0; i < NBn; ++i) {
            float sb = 0.f;
#pragma unroll
            for (int e = 0; e < 8; ++e) sb += (float)af[i][e];
            dbs[i] += sb;
          }
        }
        continue;
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
    if constexpr (!RING) {
      wait_vmcnt0();
      __syncthreads();
    }
  }

  wgrad_store<WN, WC, NWC, TAPS, NWN>(a, acc, dbs, do_bias, split, t, n0, c0, wn, wc, lane, zero_split);
}

// LINE staging (wgrad variants 6 and 7): every DMA piece moves 8 whole 128-byte pixel lines (one
// 64-channel chunk of 8 pixels; lanes 8r..8r+7 fill line r, their 16-byte chunks XOR-swizzled by
// ((r >> 1) & 3) << 1) -- 8 cache lines per instruction instead of the 32 partial (32-byte) lines
// of wgrad_tile's [16 ch][32 px] pieces.  The LDS image of a sub-step is [64-ch chunk][32 px][128 B]
// and the transposed fragment reads address it directly (conflict-free: the 8 rows of a 32-lane
// group land on 8 distinct 8-bank column groups).  Piece gi = wave + NWAVES * d always has row
// group gi & 3 = wave & 3, so each lane stages one pixel per sub-step, as before.
template <int WN, int WC, int KSUB, int NWC, int TAPS, bool ILVW = false>
__device__ __forceinline__ void wgrad_tile_line(const ConvWgradArgs& a, int split, int ks_begin, int ks_end,
                                                int t, int tstep, int n0, int c0, int zero_split) {
  constexpr int NWAVES = 2 * NWC;
  static_assert(NWAVES % 4 == 0 && WN % 64 == 0 && WC % 64 == 0 && KSUB <= 2, "line staging geometry");
  constexpr int NBn = WN / 32;          // n blocks per wave (wave covers WN/2)
  constexpr int NBc = WC / (16 * NWC);  // c blocks per wave (wave covers WC/NWC)
  constexpr int NCN = WN / 64, NCC = WC / 64;  // 64-channel chunks of the two operands
  constexpr int DZ_BYTES = WN * 64;
  constexpr int X_BYTES = WC * 64 * TAPS;
  constexpr int SUB = DZ_BYTES + X_BYTES;
  constexpr int STAGE = SUB * KSUB;
  constexpr int DZP = WN / 16 * KSUB, XPS = WC / 16 * TAPS * KSUB;  // 1 KB pieces per stage
  static_assert((DZP + XPS) % NWAVES == 0, "pieces per wave");
  constexpr int NPW = (DZP + XPS) / NWAVES;  // piece gi = wave + NWAVES * d: dz pieces first, then x
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int lane = threadIdx.x & 63;
  const int wave = wave_id();
  const int wn = wave / NWC, wc = wave % NWC;
  const int kh = t / a.K, kw = t - (t / a.K) * a.K;
  const int toff = (kh * a.HPi + kw) * a.Cin + c0;
  const int SS = a.S * a.S;
  const int pp = wave & 3;                  // row group (8 pixels) of every piece this wave stages
  const int r_st = pp * 8 + (lane >> 3);    // the pixel (LDS row) this lane stages in a sub-step
  const int lchunk = ((lane & 7) ^ (((r_st >> 1) & 3) << 1)) * 8;  // its swizzled 16-B chunk (elements)

  int dzr[KSUB], xr[KSUB];
  auto stage_addr = [&](int ks) {
#pragma unroll
    for (int sub = 0; sub < KSUB; ++sub) {
      const int px = (ks * KSUB + sub) * 32 + r_st;
      const int pm = px < a.M ? px : a.M - 1;
      const int b = fdiv(pm, a.divSS);
      const int rem = pm - b * SS;
      const int ii = fdiv(rem, a.divS);
      const int jx = rem - ii * a.S;
      dzr[sub] = (px < a.M ? ((b * a.HPo + ii + a.Po) * a.HPo + jx + a.Po) * a.Cout : 0) + n0 + lchunk;
      xr[sub] = ((b * a.HPi + ii + a.offi) * a.HPi + jx + a.offi) * a.Cin + toff + lchunk;
    }
  };
  // DMA pieces d0 <= d < d1 of the stage whose addresses stage_addr computed.  dz and x pieces in
  // separate loops under wave-uniform conditions (see wgrad_tile: a per-piece select between the
  // two tensors makes hipcc drain vmcnt before the LDS reads)
  auto stage_pieces = [&](int buf, int d0, int d1) {
    char* base = smem + buf * STAGE + pp * 1024;
#pragma unroll
    for (int d = 0; d < NPW; ++d) {
      if (d < d0 || d >= d1) continue;
      const int idx = (wave >> 2) + (NWAVES / 4) * d;  // (sub, chunk) of a dz piece
      if (idx >= DZP / 4) continue;
      const int sub = idx / NCN, cc = idx - sub * NCN;
      const int o = (KSUB == 2 && sub ? dzr[KSUB - 1] : dzr[0]) + cc * 64;
#ifdef AGK_DEBUG
      const bool ok = AGK_DCHECK(o >= 0 && (long long)o + 8 <= a.dz_elems, DBG_WG_DZ);
      glds16(ok ? a.dz + o : a.dz, base + sub * SUB + cc * 4096);
#else
      glds16(a.dz + o, base + sub * SUB + cc * 4096);
#endif
    }
#pragma unroll
    for (int d = 0; d < NPW; ++d) {
      if (d < d0 || d >= d1) continue;
      const int idx = (wave >> 2) + (NWAVES / 4) * d - DZP / 4;  // (sub, tap, chunk) of an x piece
      if (idx < 0) continue;
      const int sub = idx / (TAPS * NCC), rem = idx - sub * (TAPS * NCC);
      const int tp = rem / NCC, cc = rem - tp * NCC;
      const int o = (KSUB == 2 && sub ? xr[KSUB - 1] : xr[0]) + tp * tstep + cc * 64;
#ifdef AGK_DEBUG
      const bool ok = AGK_DCHECK(o >= 0 && (long long)o + 8 <= a.x_elems, DBG_WG_X);
      glds16(ok ? a.x + o : a.x, base + sub * SUB + DZ_BYTES + (tp * NCC + cc) * 4096);
#else
      glds16(a.x + o, base + sub * SUB + DZ_BYTES + (tp * NCC + cc) * 4096);
#endif
    }
  };
  auto stage = [&](int ks, int buf) {
    stage_addr(ks);
    stage_pieces(buf, 0, NPW);
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

  // transposed reads: lane (g = lane>>4, q = (lane&15)>>2, p = lane&3) reads row 4g+q (16+4g+q),
  // channels 4p..4p+3 of a 16-channel block: byte 32 (blk & 3) + 8p of the row, swizzled
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int rr = 4 * g + q;
  const int swz = ((rr >> 1) & 3) << 1;
  const int roff0 = rr * 128 + (p & 1) * 8;
  const int roff1 = roff0 + 16 * 128;
  auto blk_off = [&](int blk) { return (blk >> 2) * 4096 + (((((blk & 3) << 1) | (p >> 1)) ^ swz) << 4); };
  int dzo[NBn], xo[NBc];
#pragma unroll
  for (int i = 0; i < NBn; ++i) dzo[i] = blk_off(wn * NBn + i);
#pragma unroll
  for (int j = 0; j < NBc; ++j) xo[j] = DZ_BYTES + blk_off(wc * NBc + j);
  constexpr int NF = NBn + TAPS * NBc;  // fragments read per sub-step

  if constexpr (TAPS == 2) {
    // tap pairs: the second tap's x fragments are read while the first tap's MFMAs run (counted
    // lgkmcnt); ILVW spreads the next stage's DMA pieces through the first sub-step's MFMAs (the
    // last iteration re-stages clamped in-range rows into the idle buffer: no branch among them)
    constexpr int N0 = NBn + NBc;  // dz + tap-0 fragments
    constexpr int NMF = NBn * NBc;
    if (ks_begin < ks_end) {
      stage(ks_begin, 0);
      wait_vmcnt0();
      __syncthreads();
    }
    for (int ks = ks_begin; ks < ks_end; ++ks) {
      const int cur = (ks - ks_begin) & 1;
      if constexpr (ILVW) stage_addr(ks + 1);
      else if (ks + 1 < ks_end) stage(ks + 1, cur ^ 1);
#pragma unroll
      for (int sub = 0; sub < KSUB; ++sub) {
        const char* base = smem + cur * STAGE + sub * SUB;
        bf16x4 tl[NF], th[NF];
#pragma unroll
        for (int i = 0; i < NBn; ++i) {
          tl[i] = ds_read_tr16_asm(base + dzo[i] + roff0);
          th[i] = ds_read_tr16_asm(base + dzo[i] + roff1);
        }
#pragma unroll
        for (int tp = 0; tp < 2; ++tp)
#pragma unroll
          for (int j = 0; j < NBc; ++j) {
            tl[NBn + tp * NBc + j] = ds_read_tr16_asm(base + tp * NCC * 4096 + xo[j] + roff0);
            th[NBn + tp * NBc + j] = ds_read_tr16_asm(base + tp * NCC * 4096 + xo[j] + roff1);
          }
#pragma unroll
        for (int f = 0; f < N0; ++f) lgkm_wait_pair<2 * NBc>(tl[f], th[f]);
        bf16x8 af[NBn], bfm[2 * NBc];
#pragma unroll
        for (int i = 0; i < NBn; ++i)
          af[i] = bf16x8{tl[i][0], tl[i][1], tl[i][2], tl[i][3], th[i][0], th[i][1], th[i][2], th[i][3]};
#pragma unroll
        for (int j = 0; j < NBc; ++j)
          bfm[j] = bf16x8{tl[NBn + j][0], tl[NBn + j][1], tl[NBn + j][2], tl[NBn + j][3],
                          th[NBn + j][0], th[NBn + j][1], th[NBn + j][2], th[NBn + j][3]};
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
        constexpr int MPD = ILVW ? (NMF / NPW > 0 ? NMF / NPW : 1) : NMF + 1;
#pragma unroll
        for (int f = 0; f < NMF; ++f) {
          acc[0][f / NBc][f % NBc] = mfma16x16x32(af[f / NBc], bfm[f % NBc], acc[0][f / NBc][f % NBc]);
          if (ILVW && sub == 0 && f % MPD == MPD - 1 && f / MPD < NPW) {
            __builtin_amdgcn_sched_barrier(0);
            stage_pieces(cur ^ 1, f / MPD, f / MPD + 1);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
        if (ILVW && sub == 0 && NMF / MPD < NPW) stage_pieces(cur ^ 1, NMF / MPD, NPW);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < NBc; ++j) lgkm_wait_pair<0>(tl[N0 + j], th[N0 + j]);
#pragma unroll
        for (int j = 0; j < NBc; ++j)
          bfm[NBc + j] = bf16x8{tl[N0 + j][0], tl[N0 + j][1], tl[N0 + j][2], tl[N0 + j][3],
                                th[N0 + j][0], th[N0 + j][1], th[N0 + j][2], th[N0 + j][3]};
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int f = 0; f < NMF; ++f)
          acc[1][f / NBc][f % NBc] = mfma16x16x32(af[f / NBc], bfm[NBc + f % NBc], acc[1][f / NBc][f % NBc]);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        if (do_bias) {
#pragma unroll
          for (int i = 0; i < NBn; ++i) {
            float sm = 0.f;
#pragma unroll
            for (int e = 0; e < 8; ++e) sm += (float)af[i][e];
            dbs[i] += sm;
          }
        }
      }
      wait_vmcnt0();
      __syncthreads();
    }
    wgrad_store<WN, WC, NWC, TAPS>(a, acc, dbs, do_bias, split, t, n0, c0, wn, wc, lane, zero_split);
    return;
  }
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
        tl[i] = ds_read_tr16_asm(base + dzo[i] + roff0);
        th[i] = ds_read_tr16_asm(base + dzo[i] + roff1);
      }
#pragma unroll
      for (int tp = 0; tp < TAPS; ++tp)
#pragma unroll
        for (int j = 0; j < NBc; ++j) {
          tl[NBn + tp * NBc + j] = ds_read_tr16_asm(base + tp * NCC * 4096 + xo[j] + roff0);
          th[NBn + tp * NBc + j] = ds_read_tr16_asm(base + tp * NCC * 4096 + xo[j] + roff1);
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
          float sm = 0.f;
#pragma unroll
          for (int e = 0; e < 8; ++e) sm += (float)af[i][e];
          dbs[i] += sm;
        }
      }
    }
    wait_vmcnt0();
    __syncthreads();
  }
  wgrad_store<WN, WC, NWC, TAPS>(a, acc, dbs, do_bias, split, t, n0, c0, wn, wc, lane, zero_split);
}

// LINE && !PAIR: two 8-wave workgroups per CU like the production per-tap kernel (<= 128 VGPRs)
// MW: minimum waves per SIMD the register allocation must allow (0: the default -- 4 for the line-staged
// lab kernel, else 1).  The thin first layer's tap-merged rows (48-wide c tile, 6 waves) take 180 VGPRs,
// which fits ONE workgroup per CU; MW = 3 caps them at 168 (11 dwords spilled) so that two share a CU
// (AGK_WGRAD0_OCC3=1, round 4 A/B).
template <int WN, int WC, int KSUB, int NWC = 4, int TAPS = 1, bool PAIR = false, bool LINE = false, bool ILVW = false,
          int NS = 2, int MW = 0, int NWN = 2, bool UP = false>
__global__ __launch_bounds__(64 * NWN * NWC, (MW > 0 ? MW : (LINE && !PAIR) ? 4 : 1)) void conv_wgrad_kernel(
    ConvWgradArgs a) {
  static_assert(!PAIR || TAPS == 2, "PAIR: two taps per workgroup");
  static_assert(NWN == 2 || (!PAIR && !LINE), "NWN != 2: the plain per-tap / tap-merged body only");
  // workgroup -> (split, tap group, channel block).  xcd_group (tap-merged rows): the hardware
  // deals workgroups to the 8 XCDs round robin in launch order, which puts the K kernel-row
  // workgroups of a split -- all reading the same dZ rows -- on K different L2s, so every dZ
  // byte comes from the Infinity Cache K times (layer 0: 3 % L2 hits, profiles/r3_small_batch.md).
  // Grouped, each XCD runs a contiguous range of split-major work and a split's rows share an L2.
  int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  if (TAPS > 1 && !PAIR && a.xcd_group) {
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
  const int ncb = a.Cin / WC;
  const int n0 = (bz / ncb) * WN;
  const int c0 = (bz % ncb) * WC;
  // a.ksteps_per_split is in units of one stage (KSUB*32 pixels)
  const int nks_total = (a.M + 32 * KSUB - 1) / (32 * KSUB);
  const int t = by * TAPS;  // first tap of the group
  if constexpr (PAIR) {
    if (t + 1 >= a.T) {  // the odd last tap: one tap over the pixels of splits 2 bx and 2 bx + 1
      const int s0 = 2 * split;
      if (s0 >= a.nsplit) return;  // workgroup-uniform: no barrier reached yet
      const int kb = s0 * a.ksteps_per_split;
      int ke = kb + 2 * a.ksteps_per_split;
      if (ke > nks_total) ke = nks_total;
      if constexpr (LINE) wgrad_tile_line<WN, WC, KSUB, NWC, 1>(a, s0, kb, ke, t, 0, n0, c0, s0 + 1 < a.nsplit ? s0 + 1 : -1);
      else wgrad_tile<WN, WC, KSUB, NWC, 1>(a, s0, kb, ke, t, 0, n0, c0, s0 + 1 < a.nsplit ? s0 + 1 : -1);
      return;
    }
  }
  const int ks_begin = split * a.ksteps_per_split;
  int ks_end = ks_begin + a.ksteps_per_split;
  if (ks_end > nks_total) ks_end = nks_total;
  int tstep = a.Cin;  // kernel rows: tap t+1 is one column right
  if constexpr (PAIR) {
    const int t1 = t + 1;
    tstep = ((t1 / a.K - t / a.K) * a.HPi + (t1 % a.K - t % a.K)) * a.Cin;
  }
  if constexpr (LINE) wgrad_tile_line<WN, WC, KSUB, NWC, TAPS, ILVW>(a, split, ks_begin, ks_end, t, tstep, n0, c0, -1);
  else wgrad_tile<WN, WC, KSUB, NWC, TAPS, NS, NWN, UP>(a, split, ks_begin, ks_end, t, tstep, n0, c0, -1);
}

constexpr int kWgradKsub = 1;
// ConvWgradArgs::variant: 0 = production 2-buffer kernel (tap-merged rows for
// 64-wide c tiles); kernel-lab build only: 1 = one tap per workgroup,
// 2 = 256-thread tile, 3 / 4 = LDS ring with that many slots

#ifdef AGK_KERNEL_LAB
// kernel-lab tile codes and wgrad variants (conv_lab.hip); true when the code was a lab code
bool launch_conv_fwd_lab(int bm, const ConvFwdArgs& a, int bn, int mode, hipStream_t st);
bool launch_conv_wgrad_lab(const ConvWgradArgs& a, int wn, int wc, dim3 grid, hipStream_t st);
bool launch_conv_wgrad_line_lab(const ConvWgradArgs& a, hipStream_t st);  // wgrad variants 6-8
#endif

}  // namespace agk
