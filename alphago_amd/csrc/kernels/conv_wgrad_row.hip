// Weight gradient of the 'same' convolutions, one kernel ROW of taps per
// workgroup, each pixel staged once (gfx950).
//
//   dW[kh][kw][n][c] = sum_m dZ[m][n] * X[m shifted by (kh, kw)][c]
//
// conv_wgrad_kernel (conv.hip) gives every tap its own workgroup, so each
// staged 32-pixel dz tile feeds 192 x 192 x 32 MACs: 24 KB of LDS-DMA per
// 1.18 M MACs, two workgroups per CU -> ~42 B/clk per CU at full MFMA rate,
// about what LDS-DMA delivers (profiles/r2_wgrad_variants.md: the kernel sits
// at ~0.92 PF in the power-limited steady state).  Here a workgroup owns the
// KW taps of one kernel row kh for a WN x WC (n x c) tile:
//
//   * the K loop runs over 32-pixel windows of COMPACT (unpadded) pixel
//     indices; window s stages its dz rows and the x rows of the same pixels
//     for the row's centre tap (column shift 0) into a ring slot (6 slots, the
//     LDS-DMA three windows ahead of the MFMAs, counted vmcnt waits);
//   * tap kw of pixel m needs x at compact pixel m + kw - KW/2 (same board
//     row): lanes read it from the window's own slot or a neighbour slot
//     (pixels -2..33 of the window live in slots s-1, s, s+1), or from an
//     all-zero LDS region when the tap leaves the board (column j + kw - KW/2
//     outside [0, S)).  ds_read_b64_tr_b16 takes a per-lane address, so the
//     redirect is per pixel; the zero rows keep the bank slot (row & 7) of the
//     row they replace (conflict-free like the data rows).
//
// Every x pixel is staged once for KW taps and every dz pixel once for KW taps:
// 18 KB per 32-pixel window for 192 x 96 x 3 x 32 MACs at the SL layer shape
// (96 MAC/B vs 49), one workgroup per CU.  The row shift kh needs no staging
// trick: rows leaving the board read the zero borders of the padded input.
// Output: the same per-split fp32 slab [split][tap][n][c] (+ bias slab) as
// conv_wgrad_kernel, summed by conv_wgrad_reduce_kernel.
#include <hip/hip_runtime.h>

#include "common.h"
#include "conv_common.h"
#include "kernels.h"

namespace agk {

// NWN x NWC waves; each wave owns (WN / NWN) n x (WC / NWC) c for all KW taps.
template <int WN, int WC, int KW, int NWN, int NWC>
__global__ __launch_bounds__(64 * NWN * NWC, 1) void conv_wgrad_row_kernel(ConvWgradArgs a) {
  constexpr int NW = NWN * NWC;
  constexpr int NBn = WN / NWN / 16;  // 16-wide n blocks per wave
  constexpr int NBc = WC / NWC / 16;  // 16-wide c blocks per wave
  static_assert(NBn * NWN * 16 == WN && NBc * NWC * 16 == WC, "tile geometry");
  constexpr int H = KW / 2;
  constexpr int DZ_BYTES = WN * 64;           // [WN/16][32 px][16 ch] bf16
  constexpr int SLOT = (WN + WC) * 64;        // dz tile + x tile of one window
  constexpr int RING = 6;                     // windows s-1, s, s+1 (read), s+2 (landing), s+3 (issued)
  constexpr int AHEAD = 3;                    // the DMA runs 3 windows ahead of the MFMAs
  constexpr int ZOFF = RING * SLOT;           // zero region, one KB per x block
  constexpr int NDZ = WN / 16;
  constexpr int NINSTR = (WN + WC) / 16;      // 1-KB LDS-DMA pieces per window
  constexpr int IPW = (NINSTR + NW - 1) / NW;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int lane = threadIdx.x & 63;
  const int wave = wave_id();
  const int wn = wave / NWC, wc = wave % NWC;
  const int split = blockIdx.x;
  const int kh = blockIdx.y;
  const int ncb = (a.cin_real + WC - 1) / WC;
  const int n0 = (blockIdx.z / ncb) * WN;
  const int c0 = (blockIdx.z % ncb) * WC;
  const int SS = a.S * a.S;
  const int nks_total = (a.M + 31) >> 5;
  const int ks_begin = split * a.ksteps_per_split;
  int ks_end = ks_begin + a.ksteps_per_split;
  if (ks_end > nks_total) ks_end = nks_total;
  // x element offset of the row's centre tap relative to the pixel's (offi, offi) corner
  const int xoff = (kh * a.HPi + H) * a.Cin + c0;

  // zero region (never a DMA target): written once, published by the prologue barrier
  for (int o = threadIdx.x * 16; o < WC * 64; o += 64 * NW * 16)
    *(uint4*)(smem + ZOFF + o) = make_uint4(0u, 0u, 0u, 0u);

  // window ks -> ring slot; with_dz false: halo window (x only)
  auto issue = [&](int ks, int slot, bool with_dz) {
    const int half = (lane & 1) * 8;
    char* base = smem + slot * SLOT;
    const int px = ks * 32 + (lane >> 1);
    const int pm = px < a.M ? px : a.M - 1;
    const int b = fdiv(pm, a.divSS);
    const int rem = pm - b * SS;
    const int ii = fdiv(rem, a.divS);
    const int jx = rem - ii * a.S;
    const int dzr = px < a.M ? ((b * a.HPo + ii + a.Po) * a.HPo + jx + a.Po) * a.Cout : 0;  // 0 = zero border
    const int xr = ((b * a.HPi + ii + a.offi) * a.HPi + jx + a.offi) * a.Cin + xoff;
    // dz and x pieces in separate loops (a per-piece select between the two
    // source tensors makes hipcc drain vmcnt before the following LDS reads)
    if (with_dz) {
#pragma unroll
      for (int i = 0; i < IPW; ++i) {
        const int jj = wave * IPW + i;
        if (jj < NDZ) {
#ifdef AGK_DEBUG
          const long long o = (long long)dzr + n0 + half + jj * 16;
          const bool ok = AGK_DCHECK(o >= 0 && o + 8 <= a.dz_elems, DBG_WG_DZ);
          glds16(ok ? a.dz + o : a.dz, base + jj * 1024);
#else
          glds16(a.dz + dzr + n0 + half + jj * 16, base + jj * 1024);
#endif
        }
      }
    }
#pragma unroll
    for (int i = 0; i < IPW; ++i) {
      const int jj = wave * IPW + i;
      if (jj >= NDZ && jj < NINSTR) {
#ifdef AGK_DEBUG
        const long long o = (long long)xr + half + (jj - NDZ) * 16;
        const bool ok = AGK_DCHECK(o >= 0 && o + 8 <= a.x_elems, DBG_WG_X);
        glds16(ok ? a.x + o : a.x, base + jj * 1024);
#else
        glds16(a.x + xr + half + (jj - NDZ) * 16, base + jj * 1024);
#endif
      }
    }
  };

  f32x4 acc[KW][NBn][NBc];
#pragma unroll
  for (int t = 0; t < KW; ++t)
#pragma unroll
    for (int i = 0; i < NBn; ++i)
#pragma unroll
      for (int j = 0; j < NBc; ++j) acc[t][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float dbs[NBn];
#pragma unroll
  for (int i = 0; i < NBn; ++i) dbs[i] = 0.f;
  const bool do_bias = (kh == 0) && (c0 == 0) && (wc == 0);

  // transposed-read geometry (conv_wgrad_kernel): lane reads pixel rows kA0 =
  // 4g + q and kA1 = 16 + 4g + q of its k-group, channel quad p
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int kA0 = 4 * g + q, kA1 = 16 + 4 * g + q;
  const int trA0 = wn * NBn * 1024 + kA0 * 32 + p * 8;
  const int trA1 = wn * NBn * 1024 + kA1 * 32 + p * 8;
  // per tap: which window holds pixel k + kw - H (-1: previous, 0: own, 1: next) and its row
  int dl0[KW], dl1[KW], rb0[KW], rb1[KW];
#pragma unroll
  for (int kw = 0; kw < KW; ++kw) {
    const int k0 = kA0 + kw - H, k1 = kA1 + kw - H;
    dl0[kw] = k0 < 0 ? -1 : 0;          // kA0 <= 15: never past the window
    dl1[kw] = k1 >= 32 ? 1 : 0;         // kA1 >= 16: never before it
    const int r0 = k0 - 32 * dl0[kw], r1 = k1 - 32 * dl1[kw];
    rb0[kw] = DZ_BYTES + wc * NBc * 1024 + r0 * 32 + p * 8;
    rb1[kw] = DZ_BYTES + wc * NBc * 1024 + r1 * 32 + p * 8;
  }
  const int zb0 = ZOFF + wc * NBc * 1024 + ((kA0 - H) & 7) * 32 + p * 8;  // + kw * 32 (mod 256) below
  const int zb1 = ZOFF + wc * NBc * 1024 + ((kA1 - H) & 7) * 32 + p * 8;

  // LDS-DMA pieces this wave issues per window (wave-uniform): counted vmcnt waits keep the
  // younger windows in flight
  int ndz_w = 0, nx_w = 0;
#pragma unroll
  for (int i = 0; i < IPW; ++i) {
    const int jj = wave * IPW + i;
    ndz_w += jj < NDZ ? 1 : 0;
    nx_w += (jj >= NDZ && jj < NINSTR) ? 1 : 0;
  }
  // window w lives in slot (w - ks_begin + 1) % RING; a window >= ks_end is x only (right halo)
  const int nst = ks_end - ks_begin;
  if (nst > 0) {
    // prologue: halo window ks_begin - 1 (x only), then windows ks_begin .. ks_begin + AHEAD - 1
    if (ks_begin > 0) issue(ks_begin - 1, 0, false);
    int last_p = 0;
#pragma unroll
    for (int d = 0; d < AHEAD; ++d) {
      if (ks_begin + d <= ks_end) {
        issue(ks_begin + d, d + 1, ks_begin + d < ks_end);
        last_p = nx_w + (ks_begin + d < ks_end ? ndz_w : 0);
      }
    }
    // windows ks_begin - 1 .. ks_begin + 1 must have landed; the last one issued may fly on
    if (nst + 1 >= AHEAD) vmcnt_wait_dyn(last_p);
    else wait_vmcnt0();
  }
  __syncthreads();  // zero region and prologue windows visible
  for (int s = ks_begin; s < ks_end; ++s) {
    const int rs = s - ks_begin;
    // window s+AHEAD into the slot window s+AHEAD-RING (read last by step s+AHEAD-RING+1 <= s-2)
    const bool more = s + AHEAD <= ks_end;
    if (more) issue(s + AHEAD, (rs + AHEAD + 1) % RING, s + AHEAD < ks_end);
    const int om1 = (rs % RING) * SLOT, o0 = ((rs + 1) % RING) * SLOT, op1 = ((rs + 2) % RING) * SLOT;
    // columns of the lane's two pixels (taps leaving the board read zeros)
    int m0 = s * 32 + kA0, m1 = s * 32 + kA1;
    m0 = m0 < a.M ? m0 : a.M - 1;
    m1 = m1 < a.M ? m1 : a.M - 1;
    const int j0 = m0 - fdiv(m0, a.divS) * a.S;  // SS is a multiple of S: m mod S is the column
    const int j1 = m1 - fdiv(m1, a.divS) * a.S;
    int ab0[KW], ab1[KW];
#pragma unroll
    for (int kw = 0; kw < KW; ++kw) {
      const bool v0 = (unsigned)(j0 + kw - H) < (unsigned)a.S;
      const bool v1 = (unsigned)(j1 + kw - H) < (unsigned)a.S;
      ab0[kw] = v0 ? (dl0[kw] < 0 ? om1 : o0) + rb0[kw] : zb0 + ((kw * 32) & 255);
      ab1[kw] = v1 ? (dl1[kw] > 0 ? op1 : o0) + rb1[kw] : zb1 + ((kw * 32) & 255);
    }
    // A = dz fragments (all taps), B = x fragments of tap 0
    bf16x4 tla[NBn], tha[NBn], tlb[2][NBc], thb[2][NBc];
    const char* ab = smem + o0;
#pragma unroll
    for (int i = 0; i < NBn; ++i) {
      tla[i] = ds_read_tr16_asm(ab + trA0 + i * 1024);
      tha[i] = ds_read_tr16_asm(ab + trA1 + i * 1024);
    }
#pragma unroll
    for (int j = 0; j < NBc; ++j) {
      tlb[0][j] = ds_read_tr16_asm(smem + ab0[0] + j * 1024);
      thb[0][j] = ds_read_tr16_asm(smem + ab1[0] + j * 1024);
    }
    lgkm_fence<NBn>(tla, tha);
    lgkm_fence<NBc>(tlb[0], thb[0]);
    bf16x8 af[NBn];
#pragma unroll
    for (int i = 0; i < NBn; ++i)
      af[i] = bf16x8{tla[i][0], tla[i][1], tla[i][2], tla[i][3], tha[i][0], tha[i][1], tha[i][2], tha[i][3]};
#pragma unroll
    for (int kw = 0; kw < KW; ++kw) {
      const int cb = kw & 1;
      if (kw + 1 < KW) {  // next tap's x fragments load under this tap's MFMAs
#pragma unroll
        for (int j = 0; j < NBc; ++j) {
          tlb[cb ^ 1][j] = ds_read_tr16_asm(smem + ab0[kw + 1] + j * 1024);
          thb[cb ^ 1][j] = ds_read_tr16_asm(smem + ab1[kw + 1] + j * 1024);
        }
      }
      bf16x8 bfm[NBc];
#pragma unroll
      for (int j = 0; j < NBc; ++j)
        bfm[j] = bf16x8{tlb[cb][j][0], tlb[cb][j][1], tlb[cb][j][2], tlb[cb][j][3],
                        thb[cb][j][0], thb[cb][j][1], thb[cb][j][2], thb[cb][j][3]};
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < NBn; ++i)
#pragma unroll
        for (int j = 0; j < NBc; ++j) acc[kw][i][j] = mfma16x16x32(af[i], bfm[j], acc[kw][i][j]);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      if (kw + 1 < KW) lgkm_fence<NBc>(tlb[cb ^ 1], thb[cb ^ 1]);
    }
    if (do_bias) {
#pragma unroll
      for (int i = 0; i < NBn; ++i) {
        float sm = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) sm += (float)af[i][e];
        dbs[i] += sm;
      }
    }
    // window s+2 landed before the barrier that precedes its first readers (step s+1); the
    // window issued in this step stays in flight
    if (more) vmcnt_wait_dyn(nx_w + (s + AHEAD < ks_end ? ndz_w : 0));
    else wait_vmcnt0();
    __syncthreads();
  }

  // --- the split's partial tiles: D[n][c], lane owns n..n+3 at column c
  const int nb0 = n0 + wn * (WN / NWN) + ((lane >> 4) << 2);
  const int cbase = c0 + wc * (WC / NWC) + (lane & 15);
#pragma unroll
  for (int kw = 0; kw < KW; ++kw) {
    float* out = a.slab + ((size_t)split * a.T + kh * KW + kw) * (size_t)a.Cout * a.Cin;
#pragma unroll
    for (int i = 0; i < NBn; ++i)
#pragma unroll
      for (int j = 0; j < NBc; ++j) {
        const int n = nb0 + i * 16;
        const int c = cbase + j * 16;
#pragma unroll
        for (int r = 0; r < 4; ++r) out[(size_t)(n + r) * a.Cin + c] = acc[kw][i][j][r];
      }
  }
  if (do_bias) {
#pragma unroll
    for (int i = 0; i < NBn; ++i) {
      float sm = dbs[i];
      sm += __shfl_xor(sm, 16, 64);
      sm += __shfl_xor(sm, 32, 64);
      if (lane < 16) a.dbias_slab[(size_t)split * a.Cout + n0 + wn * (WN / NWN) + i * 16 + lane] = sm;
    }
  }
}

template <int WN, int WC, int KW, int NWN, int NWC>
static void launch_row(const ConvWgradArgs& a, hipStream_t st) {
  constexpr int smem = (6 * (WN + WC) + WC) * 64;  // RING slots + the zero region
  static const hipError_t attr = hipFuncSetAttribute((const void*)conv_wgrad_row_kernel<WN, WC, KW, NWN, NWC>,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, smem);
  hip_check(attr, "hipFuncSetAttribute(max dynamic LDS)");
  const int ncb = (a.cin_real + WC - 1) / WC;
  dim3 grid(a.nsplit, a.K, (a.Cout / WN) * ncb);
  hipLaunchKernelGGL((conv_wgrad_row_kernel<WN, WC, KW, NWN, NWC>), grid, dim3(64 * NWN * NWC), smem, st, a);
}

// Row-kernel geometry for a layer, or 0 when it does not apply (the per-tap
// conv_wgrad_kernel then runs).  Returns the code used by wgrad_row_launch.
int wgrad_row_code(int Cout, int Cin, int cin_real, int K) {
  if (K == 3 && Cout % 192 == 0 && Cin % 192 == 0 && cin_real == Cin) return 1;  // 192 x 96, 8 waves
  if (K == 5 && Cout % 192 == 0 && Cin == 64 && cin_real <= 48) return 2;         // 192 x 48, 6 waves
  if (K == 3 && Cout % 128 == 0 && Cin % 128 == 0 && cin_real == Cin) return 3;  // 128 x 128, 8 waves
  if (K == 5 && Cout % 128 == 0 && Cin == 64 && cin_real <= 48) return 4;         // 128 x 48, 6 waves
  if (K == 3 && Cout == 160 && Cin == 160) return 5;                              // value net: 160 x 160, 4 waves
  if (K == 5 && Cout == 160 && Cin == 64) return 6;                               // value layer 0: 160 x 64
  return 0;
}

// workgroups per split (grid y * z) of the row kernel
int wgrad_row_wgs_per_split(int code, int Cout, int Cin, int cin_real, int K) {
  const int WN = (code == 1 || code == 2) ? 192 : (code == 5 || code == 6) ? 160 : 128;
  const int WC = code == 1 ? 96 : code == 3 ? 128 : code == 5 ? 160 : code == 6 ? 64 : 48;
  (void)Cin;
  return K * (Cout / WN) * ((cin_real + WC - 1) / WC);
}

void wgrad_row_launch(int code, const ConvWgradArgs& a, hipStream_t st) {
  switch (code) {
    case 1: launch_row<192, 96, 3, 4, 2>(a, st); break;
    case 2: launch_row<192, 48, 5, 2, 3>(a, st); break;
    case 3: launch_row<128, 128, 3, 4, 2>(a, st); break;
    case 4: launch_row<128, 48, 5, 2, 3>(a, st); break;
    case 5: launch_row<160, 160, 3, 2, 2>(a, st); break;  // 4 waves, 80 x 80 per wave (10 waves spill)
    case 6: launch_row<160, 64, 5, 2, 4>(a, st); break;
    default: throw std::invalid_argument("conv_wgrad: no row kernel for this geometry");
  }
}

}  // namespace agk
