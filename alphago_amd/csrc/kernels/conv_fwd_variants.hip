// Forward-conv kernel lab: alternative pipelines of the same implicit GEMM
// (same packed operands, padded NHWC geometry and epilogues as
// conv_fwd_kernel in conv.hip), selectable with set_conv_tile for A/B runs
// and covered by tests/test_hip_kernels.py.  Findings:
// profiles/r1_fwd_kernel_experiments.md.
//   -1  halo over padded positions (weights ring, counted vmcnt)
//    2  interior halo (A staged once per 64-channel chunk for all taps)
//   32  ring (4 LDS slots of 32-channel steps, DMA 3 steps ahead)
//    4  ping-pong: two wave groups one barrier apart
//    5  compact halo + ping-pong
//    6  compact halo + ping-pong on the 32x32x16 MFMA (3x3 and 5x5)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <numeric>

#include "common.h"
#include "conv_common.h"
#include "kernels.h"

namespace agk {

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

// diagnostic stamps: the lab op passes a buffer in ConvFwdArgs::dbg (scripts/conv_stamps.py)

template <int BN, int MODE>
static void launch_fwd_pp(const ConvFwdArgs& a_in, hipStream_t st) {
  constexpr int smem = PP_SLOTS * (PP_BM * 64 + BN * 64);
  if constexpr (BN == 192 && MODE == MODE_BIAS_RELU) {
    if (a_in.dbg) {  // diagnostic instantiation with segment stamps
      static const hipError_t attr_d = hipFuncSetAttribute((const void*)conv_fwd_pp_kernel<BN, MODE, true>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, smem);  // once per instantiation (thread-safe static)
  hip_check(attr_d, "hipFuncSetAttribute(max dynamic LDS)");
      ConvFwdArgs a = a_in;
      dim3 grid((a.M + PP_BM - 1) / PP_BM, a.Cout / BN);
      hipLaunchKernelGGL((conv_fwd_pp_kernel<BN, MODE, true>), grid, dim3(512), smem, st, a);
      return;
    }
  }
  const ConvFwdArgs& a = a_in;
  static const hipError_t attr = hipFuncSetAttribute((const void*)conv_fwd_pp_kernel<BN, MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, smem);  // once per instantiation (thread-safe static)
  hip_check(attr, "hipFuncSetAttribute(max dynamic LDS)");
  dim3 grid((a.M + PP_BM - 1) / PP_BM, a.Cout / BN);
  hipLaunchKernelGGL((conv_fwd_pp_kernel<BN, MODE>), grid, dim3(512), smem, st, a);
}

template <int BN, int MODE>
static void launch_fwd_ring(const ConvFwdArgs& a, hipStream_t st) {
  constexpr int smem = RING_SLOTS * (RING_BM * 64 + BN * 64);
  static const hipError_t attr = hipFuncSetAttribute((const void*)conv_fwd_ring_kernel<BN, MODE>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        smem);  // once per instantiation (thread-safe static)
  hip_check(attr, "hipFuncSetAttribute(max dynamic LDS)");
  dim3 grid((a.M + RING_BM - 1) / RING_BM, a.Cout / BN);
  hipLaunchKernelGGL((conv_fwd_ring_kernel<BN, MODE>), grid, dim3(512), smem, st, a);
}

template <int BN, int MODE>
static void launch_fwd_halo(const ConvFwdArgs& a_in, hipStream_t st) {
  constexpr int smem = 2 * HALO_ROWS * 128 + 3 * BN * 128;
  static const hipError_t attr = hipFuncSetAttribute((const void*)conv_fwd_halo_kernel<BN, MODE>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        smem);  // once per instantiation (thread-safe static)
  hip_check(attr, "hipFuncSetAttribute(max dynamic LDS)");
  ConvFwdArgs a = a_in;
  const int B = a.M / (a.S * a.S);
  a.M = B * a.HPo * a.HPo;  // padded positions
  a.divSS = make_fastdiv((uint32_t)(a.HPo * a.HPo));
  a.divS = make_fastdiv((uint32_t)a.HPo);
  dim3 grid((a.M + HALO_BM - 1) / HALO_BM, a.Cout / BN);
  hipLaunchKernelGGL((conv_fwd_halo_kernel<BN, MODE>), grid, dim3(512), smem, st, a);
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
  static const hipError_t attr = hipFuncSetAttribute((const void*)conv_fwd_halo2_kernel<BN, MODE>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        smem);  // once per instantiation (thread-safe static)
  hip_check(attr, "hipFuncSetAttribute(max dynamic LDS)");
  dim3 grid((a.M + H2_BM - 1) / H2_BM, a.Cout / BN);
  hipLaunchKernelGGL((conv_fwd_halo2_kernel<BN, MODE>), grid, dim3(512), smem, st, a);
}

template <int BN, int MODE>
static void launch_fwd_hpp(const ConvFwdArgs& a_in, hipStream_t st) {
  constexpr int smem = 2 * HC_ROWS * 128 + 3 * BN * 128;
  if constexpr (BN == 192 && MODE == MODE_BIAS_RELU) {
    if (a_in.dbg) {  // diagnostic instantiation with segment stamps
      static const hipError_t attr_d = hipFuncSetAttribute((const void*)conv_fwd_hpp_kernel<BN, MODE, true>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, smem);  // once per instantiation (thread-safe static)
  hip_check(attr_d, "hipFuncSetAttribute(max dynamic LDS)");
      ConvFwdArgs a = a_in;
      dim3 grid((a.M + H2_BM - 1) / H2_BM, a.Cout / BN);
      hipLaunchKernelGGL((conv_fwd_hpp_kernel<BN, MODE, true>), grid, dim3(512), smem, st, a);
      return;
    }
  }
  const ConvFwdArgs& a = a_in;
  static const hipError_t attr = hipFuncSetAttribute((const void*)conv_fwd_hpp_kernel<BN, MODE>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        smem);  // once per instantiation (thread-safe static)
  hip_check(attr, "hipFuncSetAttribute(max dynamic LDS)");
  dim3 grid((a.M + H2_BM - 1) / H2_BM, a.Cout / BN);
  hipLaunchKernelGGL((conv_fwd_hpp_kernel<BN, MODE>), grid, dim3(512), smem, st, a);
}

template <int BN, int MODE, int K>
static void launch_fwd_h32(const ConvFwdArgs& a_in, hipStream_t st) {
  constexpr int smem = (K == 3 ? 2 * (H32_DATA3 + 16) : (H32_DATA5 + 16)) * 128 + 3 * BN * 128;
  ConvFwdArgs a = a_in;
  dim3 grid((a.M + H2_BM - 1) / H2_BM, a.Cout / BN);
  if constexpr (BN == 192 && MODE == MODE_BIAS_RELU && K == 3) {
    if (a_in.dbg) {  // diagnostic instantiation with segment stamps
      static const hipError_t attr_d = hipFuncSetAttribute((const void*)conv_fwd_h32_kernel<BN, MODE, K, true>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, smem);  // once per instantiation (thread-safe static)
  hip_check(attr_d, "hipFuncSetAttribute(max dynamic LDS)");
      hipLaunchKernelGGL((conv_fwd_h32_kernel<BN, MODE, K, true>), grid, dim3(512), smem, st, a);
      return;
    }
  }
  static const hipError_t attr = hipFuncSetAttribute((const void*)conv_fwd_h32_kernel<BN, MODE, K>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        smem);  // once per instantiation (thread-safe static)
  hip_check(attr, "hipFuncSetAttribute(max dynamic LDS)");
  hipLaunchKernelGGL((conv_fwd_h32_kernel<BN, MODE, K>), grid, dim3(512), smem, st, a);
}

// the 32x32 halo kernel applies (3x3 any Cin; 5x5 with one 64-channel chunk)
static bool h32_ok(const ConvFwdArgs& a) {
  if (a.K == 3) return H2_BM + 2 * (a.S + 1) <= H32_DATA3;
  if (a.K == 5) return a.Cin == 64 && H2_BM + 4 * (a.S + 1) <= H32_DATA5;
  return false;
}


template <int BN, int MODE>
static bool launch_variant_t(int code, const ConvFwdArgs& a, hipStream_t st) {
  if (code == -1) {
    const bool halo_ok = a.K == 3 && a.HPi == a.HPo && a.offi == 0 && a.Po == 1 && a.HPo + 1 <= 32 &&
                         256 + 2 * (a.HPo + 1) <= HALO_ROWS && !a.mbits_out && MODE != MODE_MASKBITS;
    if (!halo_ok) return false;
    launch_fwd_halo<BN, MODE>(a, st);
    return true;
  }
  if (code == 2) {
    if (halo2_rows_needed(a.M, a.S, a.HPi, a.K, a.offi) > H2_ROWS || BN > 192) return false;
    launch_fwd_halo2<BN, MODE>(a, st);
    return true;
  }
  if (code == 5) {
    if (!(a.K == 3 && H2_BM + 2 * (a.S + 1) <= HC_DATA)) return false;
    launch_fwd_hpp<BN, MODE>(a, st);
    return true;
  }
  if (code == 6) {
    if (!h32_ok(a)) return false;
    if (a.K == 3) launch_fwd_h32<BN, MODE, 3>(a, st);
    else launch_fwd_h32<BN, MODE, 5>(a, st);
    return true;
  }
  if (code == 4) {
    launch_fwd_pp<BN, MODE>(a, st);
    return true;
  }
  if (code == 32) {
    launch_fwd_ring<BN, MODE>(a, st);
    return true;
  }
  return false;
}

template <int MODE>
static bool launch_variant_mode(int code, const ConvFwdArgs& a, hipStream_t st) {
  if (a.Cout % 192 == 0) return launch_variant_t<192, MODE>(code, a, st);
  if (a.Cout % 128 == 0) return launch_variant_t<128, MODE>(code, a, st);
  return launch_variant_t<64, MODE>(code, a, st);
}

bool launch_conv_fwd_variant(int code, const ConvFwdArgs& a, int mode, hipStream_t st) {
  if (mode == MODE_BIAS_RELU) return launch_variant_mode<MODE_BIAS_RELU>(code, a, st);
  if (mode == MODE_MASK) return launch_variant_mode<MODE_MASK>(code, a, st);
  if (mode == MODE_MASKBITS) return launch_variant_mode<MODE_MASKBITS>(code, a, st);
  return launch_variant_mode<MODE_NONE>(code, a, st);
}

}  // namespace agk
