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
template <int BN, int MODE, int BM, int MBW, bool EPF = true, bool PIPE = true>
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
    st_c0 += 64;
    if (st_c0 == a.Cin) {
      st_c0 = 0;
      st_w += wtap;
      st_a += a.Cin;
      if (++st_kw == a.K) {
        st_kw = 0;
        st_a += (a.HPi - a.K) * a.Cin;
      }
    }
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

template <int BN, int MODE, int BM, int MBW, bool EPF = true, bool PIPE = true>
static void launch_fwd_bm(const ConvFwdArgs& a, hipStream_t st) {
  constexpr int smem = 2 * (BM * 128 + BN * 128);
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)conv_fwd_kernel<BN, MODE, BM, MBW, EPF, PIPE>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr = true;
  }
  dim3 grid((a.M + BM - 1) / BM, a.Cout / BN);
  hipLaunchKernelGGL((conv_fwd_kernel<BN, MODE, BM, MBW, EPF, PIPE>), grid, dim3(BM / MBW * 8), smem, st, a);
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
static void launch_fwd_t(const ConvFwdArgs& a, hipStream_t st) {
  const bool halo_ok = a.K == 3 && a.HPi == a.HPo && a.offi == 0 && a.Po == 1 && a.HPo + 1 <= 32 &&
                       (a.S + 2) * (a.S + 2) * 0 + 256 + 2 * (a.HPo + 1) <= HALO_ROWS;
  if (halo_ok && g_fwd_bm == -1 && !a.mbits_out && MODE != MODE_MASKBITS) {  // opt-in: slower at S=19 (18% border work), see profiles/
    launch_fwd_halo<BN, MODE>(a, st);
    return;
  }
  int bm = g_fwd_bm;
  if (bm == 2) {  // interior-halo kernel when the tile's halo fits
    if (halo2_rows_needed(a.M, a.S, a.HPi, a.K, a.offi) <= H2_ROWS && BN <= 192) {
      launch_fwd_halo2<BN, MODE>(a, st);
      return;
    }
    bm = 0;
  }
  // forward: 96x96-per-wave tiles (147 KB LDS).  dgrad keeps the 112-KB tile:
  // it runs concurrently with wgrad (48 KB) on the other stream and the two
  // only share a CU when their LDS fits together.
  if (bm <= 0)
    bm = (MODE != MODE_MASK && MODE != MODE_MASKBITS && a.M >= 384 * 512) ? 384 : (a.M >= 256 * 512) ? 256 : 128;
  // tile codes: 128 / 256 (64-pixel waves), 2568 (BM 256, 128-pixel waves: 4 waves, 1 per SIMD)
  if (bm == 32) launch_fwd_ring<BN, MODE>(a, st);
  else if (bm == 256) launch_fwd_bm<BN, MODE, 256, 4>(a, st);
  else if (bm == 2560) launch_fwd_bm<BN, MODE, 256, 4, false>(a, st);  // epilogue loads after the loop
  else if (bm == 2568) launch_fwd_bm<BN, MODE, 256, 8>(a, st);
  else if (bm == 384) launch_fwd_bm<BN, MODE, 384, 6, false, false>(a, st);  // 96x96 per wave, 147 KB LDS
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
