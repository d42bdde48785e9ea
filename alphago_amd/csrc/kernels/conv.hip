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

#include "conv_kernels.h"

namespace agk {


// ----------------------------------------------------------------- forward launchers

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
#ifdef AGK_KERNEL_LAB  // LDS-ring tiles (round 4: slower or equal at small batches, kernel lab)
  else if (bm == 65) launch_fwd_bm<160, MODE, 64, 2, true, true, false, false, STR, false, 4>(a, st);
  else if (bm == 130) launch_fwd_bm<160, MODE, 128, 4, true, true, false, false, STR, false, 3>(a, st);
#endif
  else if (bm == 38) launch_fwd_splitk<160, MODE, STR>(a, st);  // split-K (small value-net batches)
  else if (bm == 36) launch_fwd_bm<160, MODE, 32, 1, true, true, false, false, STR>(a, st);  // 32 pixels, 4 waves
  else throw std::invalid_argument("conv_fwd: 160-wide tiles support tile codes 36 / 38 / 64 / 128 / 256 / 384-387");
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
  // round 4: below 64 x 256 pixels (B <= 45 at 19 x 19) the 32-pixel tile on 4 waves (tile 36) -- twice
  // the workgroups of the 64 tile; SL step at B = 16: 18.6k -> 19.7k positions/s (profiles/r4/README.md)
  if (BN != 160 && a.tile == 0 && a.M < 64 * 256) bm = 36;
  // the 160-wide value layers: 32-pixel tile below 8192 pixels (B <= 22); graph-timed per layer at
  // B = 1 / 16 15.0 / 16.1 us vs 16.4 / 17.0 (tile 64), but 18.9 vs 17.7 at B = 32
  // (profiles/r4/raw/tiles_160_graph.txt)
  if (BN == 160 && a.tile == 0 && a.M < 8192) bm = 36;
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
    // 32-pixel tiles (twice the workgroups of the 64 tile at small batches): 36 = 4 waves of 16 x BN/2,
    // 37 = 2 waves of 32 x BN/2; same ReLU' bitmask layout
    else if (bm == 36) launch_fwd_bm<BN, MODE, 32, 1>(a, st);
    else if (bm == 38) launch_fwd_splitk<BN, MODE>(a, st);  // 36 with split-K (conv_fwd_splitk op)
    else if (bm == 37) launch_fwd_bm<BN, MODE, 32, 2>(a, st);
#ifdef AGK_KERNEL_LAB
    // small batches: 65 / 130 = the 64 / 128-pixel tiles on a 4 / 3-slot LDS ring (NS above); measured
    // slower or equal (round 4), kernel lab only
    else if (bm == 65) launch_fwd_bm<BN, MODE, 64, 2, true, true, false, false, false, false, 4>(a, st);
    else if (bm == 130) launch_fwd_bm<BN, MODE, 128, 4, true, true, false, false, false, false, 3>(a, st);
#endif
    // 385: the 384 tile with the next stage's LDS-DMA spread through the first
    // k-half's MFMAs instead of issued as one burst (kernel-lab tile 9)
    else if (bm == 385) launch_fwd_bm<BN, MODE, 384, 6, false, false, false, true>(a, st);
    // 386 / 387: 385 / 384 with the chunk-outer K order (CO above)
    else if (bm == 386) launch_fwd_bm<BN, MODE, 384, 6, false, false, false, true, false, true>(a, st);
    else if (bm == 387) launch_fwd_bm<BN, MODE, 384, 6, false, false, false, false, false, true>(a, st);
#ifdef AGK_KERNEL_LAB
    // kernel-lab tile codes (conv_lab.hip, profiles/r1_fwd_kernel_experiments.md)
    else if (launch_conv_fwd_lab(bm, a, BN, MODE, st)) return;
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
  if (a.tile == 40) {  // weight-stationary small-batch kernel (conv_ws.hip)
    launch_conv_ws(a, mode, 0, st);
    return;
  }
#ifdef AGK_KERNEL_LAB
  if (a.tile > 1000 && a.tile < 1064) {  // its probes (which part sets the layer's time)
    launch_conv_ws(a, mode, 0, st, a.tile - 1000);
    return;
  }
#endif
  if (mode == MODE_BIAS_RELU) launch_fwd_mode<MODE_BIAS_RELU>(a, st);
  else if (mode == MODE_MASK) launch_fwd_mode<MODE_MASK>(a, st);
  else if (mode == MODE_MASKBITS) launch_fwd_mode<MODE_MASKBITS>(a, st);
  else launch_fwd_mode<MODE_NONE>(a, st);
}

#ifdef AGK_KERNEL_LAB
// packed-tap first layer (conv_fwd_pk_kernel): 384-pixel tile, 96 x 96 (or 96 x 80) per wave; equal to the
// 64-channel kernel in the step (399.5 vs 398.1 us, round 4), kernel lab only
template <int BN>
static void launch_fwd_pk_t(const ConvFwdArgs& a, int cpt, hipStream_t st) {
  constexpr int BM = 384, MBW = 6;
  constexpr int smem = 2 * (BM * 128 + BN * 128);
  static const hipError_t attr = hipFuncSetAttribute((const void*)conv_fwd_pk_kernel<BN, BM, MBW>,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, smem);
  hip_check(attr, "hipFuncSetAttribute(max dynamic LDS)");
  dim3 grid((a.M + BM - 1) / BM, a.Cout / BN);
  hipLaunchKernelGGL((conv_fwd_pk_kernel<BN, BM, MBW>), grid, dim3(BM / MBW * 8), smem, st, a, cpt);
}

void launch_conv_fwd_pk(const ConvFwdArgs& a_in, int cpt, hipStream_t st) {
  ConvFwdArgs a = a_in;
  a.divSS = make_fastdiv((uint32_t)(a.S * a.S));
  a.divS = make_fastdiv((uint32_t)a.S);
  if (cpt < 4 || cpt > 8 || a.Cin != 64) throw std::invalid_argument("conv_fwd_pk: 32 < cin_real <= 64 in a 64-channel input");
  if (a.Cout == 160) launch_fwd_pk_t<160>(a, cpt, st);
  else if (a.Cout % 192 == 0) launch_fwd_pk_t<192>(a, cpt, st);
  else if (a.Cout % 128 == 0) launch_fwd_pk_t<128>(a, cpt, st);
  else launch_fwd_pk_t<64>(a, cpt, st);
}
#endif  // AGK_KERNEL_LAB

// ----------------------------------------------------------------- wgrad launchers



// The thin first layer's kernel rows run one workgroup per CU (180 VGPRs on 6 waves): ~1.16 us per
// 32-pixel stage, 26-29 % MFMA busy (profiles/r3_final/pmc).  Round-4 variants, kernel lab only since
// round 5 (torch.ops.alphago_amd_lab.conv_wgrad variant argument; in-step times at B = 2176,
// profiles/r4/README.md):
//   10: 12 waves (4 n x 3 c, 48 x 48 per wave per tap, 104 VGPRs): 559 us vs 556 us;
//   11: the 6 waves with unit pipelining (wgrad_tile UP: the next tap's x fragments are read under
//       the current tap's MFMAs; after the barrier only the dz fragments and tap 0 are exposed): 557 us;
//   12: 12 waves with unit pipelining: 556 us.
// Measured and removed: the 6 waves on a 4-slot LDS ring (601 us), 12 waves + UP capped at 85 VGPRs
// for two workgroups per CU (56 B spilled, bench -4.5 %), UP on the 3x3 per-tap kernel (517 vs 500 us).
template <int WN, int TAPS, int MW, int NWN = 2, int NS = 2, bool UP = false>
static void launch_wgrad_taps48(const ConvWgradArgs& a_in, hipStream_t st) {
  constexpr int smem = NS * (WN + 48 * TAPS) * 64 * kWgradKsub;
  constexpr int threads = 64 * 3 * NWN;
  static const hipError_t attr48 = hipFuncSetAttribute(
      (const void*)conv_wgrad_kernel<WN, 48, kWgradKsub, 3, TAPS, false, false, false, NS, MW, NWN, UP>,
      hipFuncAttributeMaxDynamicSharedMemorySize, smem);  // once per instantiation (thread-safe static)
  hip_check(attr48, "hipFuncSetAttribute(max dynamic LDS)");
  const ConvWgradArgs& a = a_in;
  dim3 grid(a.nsplit, a.T / TAPS, a.Cout / WN);
  hipLaunchKernelGGL((conv_wgrad_kernel<WN, 48, kWgradKsub, 3, TAPS, false, false, false, NS, MW, NWN, UP>), grid,
                     dim3(threads), smem, st, a);
}

template <int WN, int TAPS>
static void launch_wgrad_taps(const ConvWgradArgs& a, hipStream_t st) {
  if (a.cin_real <= 48) {
    // thin first layer (48 real planes padded to 64): a 48-wide c tile on 6
    // waves (2 n x 3 c) skips the zero channels -- 25% fewer MFMAs and x bytes
    // on the backward's serial tail; the slab columns 48..63 stay unwritten
    // (the reduce reads only cin_real of them)
#ifdef AGK_KERNEL_LAB  // round-4 re-cuts of this kernel (equal or slower): variants 10-12, 13 = two per CU
    if (TAPS == 5 && a.variant == 13) {
      launch_wgrad_taps48<WN, TAPS, 3>(a, st);
      return;
    }
    if constexpr (TAPS == 5 && (WN / 16) % 4 == 0) {
      if (a.variant == 10) {
        launch_wgrad_taps48<WN, TAPS, 0, 4>(a, st);
        return;
      }
      if (a.variant == 12) {
        launch_wgrad_taps48<WN, TAPS, 0, 4, 2, true>(a, st);
        return;
      }

    }
    if constexpr (TAPS == 5) {
      if (a.variant == 11) {
        launch_wgrad_taps48<WN, TAPS, 0, 2, 2, true>(a, st);
        return;
      }
    }
#endif
    if constexpr (TAPS == 5 && WN == 192) {
      // round 5: the 5x5 first layer as 96-channel halves of the output rows -- half the accumulators
      // per wave (104 VGPRs instead of 180), so two workgroups share a CU and one resident round covers
      // the grid (51 splits instead of two rounds of 102): 552.9 -> 489.8 us in the B = 2176 step, its
      // split-K slab halved (reduce 205.5 -> 188.3 us per step), bench +0.6 % (profiles/r5/README.md)
      launch_wgrad_taps48<96, TAPS, 0>(a, st);
      return;
    }
    launch_wgrad_taps48<WN, TAPS, 0>(a, st);
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
  const bool c64 = (Cin != 160 && Cin % 192 != 0 && Cin % 128 != 0) || variant == kWgradSmall;
  (void)Cout;
  return (c64 && (variant == 0 || variant == kWgradSmall) && (K == 3 || K == 5)) ? K : 1;
}

#ifdef AGK_KERNEL_LAB
// variant 9 (small batches): the per-tap kernel on a 4-slot LDS ring, one workgroup per CU, for the
// tile geometries whose waves stage equal piece counts (192 x 192, 128 x 128, 160 x 160); the SL step at
// B = 16 measured 0.901 ms with it against 0.863 ms without (round 4): kernel lab only
template <int WN, int WC, int NWC>
static bool launch_wgrad_ring(const ConvWgradArgs& a, dim3 grid, hipStream_t st) {
  constexpr int KS = kWgradKsub;
  constexpr int NWAVES = 2 * NWC;
  constexpr int NINSTR = WN / 16 + WC / 16;
  constexpr int IPW = (NINSTR + NWAVES - 1) / NWAVES;
  if constexpr ((WN / 16) % IPW == 0 && NINSTR == NWAVES * IPW) {
    constexpr int NS = 4;
    constexpr int smem = NS * (WN + WC) * 64 * KS;
    static const hipError_t attr = hipFuncSetAttribute(
        (const void*)conv_wgrad_kernel<WN, WC, KS, NWC, 1, false, false, false, NS>,
        hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    hip_check(attr, "hipFuncSetAttribute(max dynamic LDS)");
    hipLaunchKernelGGL((conv_wgrad_kernel<WN, WC, KS, NWC, 1, false, false, false, NS>), grid, dim3(64 * NWAVES),
                       smem, st, a);
    return true;
  }
  return false;
}
#endif  // AGK_KERNEL_LAB

template <int WN, int WC>
static void launch_wgrad_t(const ConvWgradArgs& a, hipStream_t st) {
  dim3 grid(a.nsplit, a.T, (a.Cout / WN) * (a.Cin / WC));
  constexpr int KS = kWgradKsub;
  constexpr int smem = 2 * (WN + WC) * 64 * KS;
#ifdef AGK_KERNEL_LAB
  if (WC != 64 && a.variant == 9 && launch_wgrad_ring<WN, WC, 4>(a, grid, st)) return;
  if (a.variant != 9 && launch_conv_wgrad_lab(a, WN, WC, grid, st)) return;  // lab variants 2 / 3 / 4 (conv_lab.hip)
#else
  if (a.variant != 0)
    throw std::invalid_argument("conv_wgrad: variant " + std::to_string(a.variant) + " is a kernel-lab variant");
#endif
  if constexpr (WC == 64) {
    // tap-merged kernel rows (see conv_wgrad_kernel); lab variant 1 forces one tap per workgroup
    if (a.variant != 1 && (a.K == 3 || a.K == 5)) {
      if (a.K == 3) launch_wgrad_taps<WN, 3>(a, st);
      else launch_wgrad_taps<WN, 5>(a, st);
      return;
    }
  }
  static const hipError_t attr = hipFuncSetAttribute((const void*)conv_wgrad_kernel<WN, WC, KS>,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize,
                                                     smem);  // once per instantiation (thread-safe static)
  hip_check(attr, "hipFuncSetAttribute(max dynamic LDS)");
  hipLaunchKernelGGL((conv_wgrad_kernel<WN, WC, KS>), grid, dim3(512), smem, st, a);
}

// 160 x 160 tile on 4 waves (2 n x 2 c, 80 x 80 per wave): the value net's
// padded width; 40 KB of LDS, so several workgroups share a CU
static void launch_wgrad_160x160(const ConvWgradArgs& a, hipStream_t st) {
#ifdef AGK_KERNEL_LAB
  if (a.variant == 9 && launch_wgrad_ring<160, 160, 2>(a, dim3(a.nsplit, a.T, 1), st)) return;
#endif
  if (a.variant != 0) throw std::invalid_argument("conv_wgrad: 160-wide tiles have no production variants");
  constexpr int KS = kWgradKsub;
  constexpr int smem = 2 * (160 + 160) * 64 * KS;
  static const hipError_t attr = hipFuncSetAttribute((const void*)conv_wgrad_kernel<160, 160, KS, 2>,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, smem);
  hip_check(attr, "hipFuncSetAttribute(max dynamic LDS)");
  dim3 grid(a.nsplit, a.T, 1);
  hipLaunchKernelGGL((conv_wgrad_kernel<160, 160, KS, 2>), grid, dim3(256), smem, st, a);
}

int wgrad_stage_pixels() { return 32 * kWgradKsub; }

// Split-free small-batch wgrad (kWgradDirect).  At B <= 16 the split-K plan spends ~10 us per layer on
// its reduce launch beside a ~15 us wgrad (profiles/r5/README.md, B = 16 trace), and its one-round grid
// gives each split only a few hundred pixels.  Here every workgroup owns one 32 (n) x WC (c) tile of
// one tap over ALL B*S*S pixels: 6 x 4 x 9 = 216 workgroups for a 192 -> 192 3x3 layer (150 for the
// 5x5 first layer's 48 real input planes), at most one per CU.  Each streams (32 + WC) channels x M
// pixels through an LDS double buffer of KS 32-pixel sub-steps (one barrier per 32 KS pixels) and
// writes its fp32 sums straight into the OIHW gradient (wgrad_store, grad_w != nullptr): deterministic
// (one workgroup per output element, fixed pixel order), no slab and no reduce launch.
template <int WC, int NWC, int KS>
static void launch_wgrad_direct_t(const ConvWgradArgs& a, hipStream_t st) {
  constexpr int WN = 32;
  constexpr int smem = 2 * (WN + WC) * 64 * KS;
  static const hipError_t attr = hipFuncSetAttribute((const void*)conv_wgrad_kernel<WN, WC, KS, NWC>,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, smem);
  hip_check(attr, "hipFuncSetAttribute(max dynamic LDS)");
  dim3 grid(1, a.T, (a.Cout / WN) * (a.Cin / WC));
  hipLaunchKernelGGL((conv_wgrad_kernel<WN, WC, KS, NWC>), grid, dim3(64 * 2 * NWC), smem, st, a);
}

// c tile of the split-free plan: 48 (192-multiple widths; the first layer's 48 real planes of 64), else 32
int wgrad_direct_wc(int Cin, int cin_real) {
  if (Cin == 64 && cin_real <= 48) return 48;
  if (Cin % 48 == 0 && cin_real == Cin) return 48;
  if (Cin % 32 == 0) return 32;
  return 0;
}

bool wgrad_direct_supported(int Cout, int Cin, int cin_real, int K) {
  return Cout % 32 == 0 && wgrad_direct_wc(Cin, cin_real) > 0 && (K == 1 || K == 3 || K == 5);
}

void launch_conv_wgrad_direct(const ConvWgradArgs& a_in, int ksub, hipStream_t st) {
  ConvWgradArgs a = a_in;
  a.divSS = make_fastdiv((uint32_t)(a.S * a.S));
  a.divS = make_fastdiv((uint32_t)a.S);
  a.xcd_group = 0;
  a.nsplit = 1;
  if (!a.grad_w || !wgrad_direct_supported(a.Cout, a.Cin, a.cin_real, a.K))
    throw std::invalid_argument("conv_wgrad_direct: needs grad_w, Cout % 32 == 0 and a 48 / 32 c tile");
  const int wc = wgrad_direct_wc(a.Cin, a.cin_real);
  if (wc == 48) {
    if (ksub == 1) launch_wgrad_direct_t<48, 3, 1>(a, st);
    else if (ksub == 2) launch_wgrad_direct_t<48, 3, 2>(a, st);
    else if (ksub == 8) launch_wgrad_direct_t<48, 3, 8>(a, st);
    else launch_wgrad_direct_t<48, 3, 4>(a, st);
  } else {
    if (ksub == 1) launch_wgrad_direct_t<32, 2, 1>(a, st);
    else if (ksub == 2) launch_wgrad_direct_t<32, 2, 2>(a, st);
    else if (ksub == 8) launch_wgrad_direct_t<32, 2, 8>(a, st);
    else launch_wgrad_direct_t<32, 2, 4>(a, st);
  }
}

// tap-pair / line-staged wgrads (variants 6-8): kernel lab (conv_lab.hip, profiles/r3_wgrad_pair.md)
static bool wgrad_pair_applies(int Cout, int Cin, int cin_real, int K) {
  return K == 3 && Cout == 192 && Cin == 192 && cin_real == Cin;
}

#ifdef AGK_DEBUG
unsigned debug_error_fetch_and_clear(hipStream_t st) {
  hip_check(hipStreamSynchronize(st), "debug: stream synchronize");
  unsigned code = 0, zero = 0;
  hip_check(hipMemcpyFromSymbol(&code, HIP_SYMBOL(g_dbg_err), sizeof(code)), "debug: read error word");
  if (code) hip_check(hipMemcpyToSymbol(HIP_SYMBOL(g_dbg_err), &zero, sizeof(zero)), "debug: clear error word");
  return code;
}
#endif

void wgrad_plan(int Cout, int Cin, int cin_real, int K, int variant, int out[4]) {
  if ((variant == 6 || variant == 8) && wgrad_pair_applies(Cout, Cin, cin_real, K)) {
    // tap pairs: 4.5 workgroups per split (9 per two splits), one per CU -- reported as 9 per
    // split pair and 2 per CU so that nsplit = CUs * out[2] / out[1] stays an integer division
    out[0] = 2;
    out[1] = 9;
    out[2] = 2;
    out[3] = 512;
    return;
  }
#ifdef AGK_KERNEL_LAB
  const int code = variant == 5 ? wgrad_row_code(Cout, Cin, cin_real, K) : 0;
  if (code) {  // one kernel row per workgroup, one workgroup per CU (~170 VGPRs, 8 or 6 waves)
    out[0] = K;
    out[1] = wgrad_row_wgs_per_split(code, Cout, Cin, cin_real, K);
    out[2] = 1;
    out[3] = 256;
    return;
  }
#endif
  if (variant == kWgradSmall) {  // small batches: 64 x 64 tiles, tap-merged kernel rows (launch_conv_wgrad)
    out[0] = wgrad_tap_group(Cout, Cin, K, variant);
    out[1] = (K * K / out[0]) * (Cout / 64) * (Cin / 64);
    out[2] = 2;
    out[3] = 512;
    return;
  }
  // per-tap kernel: tap-merged rows for 64-wide c tiles, else one tap; two workgroups per CU
  const int taps = wgrad_tap_group(Cout, Cin, K, (variant >= 5 && variant <= 13) ? 0 : variant);
  const bool c48 = cin_real <= 48 && Cin == 64;
  int wn = Cout == 160 ? 160 : Cout % 192 == 0 ? 192 : Cout % 128 == 0 ? 128 : 64;
  if (c48 && taps == 5 && wn == 192) wn = 96;  // the first layer's 96-wide halves (launch_wgrad_taps)
  const int wc = Cout == 160 && Cin == 160 ? 160 : Cin % 192 == 0 ? 192 : Cin % 128 == 0 ? 128 : 64;
  out[0] = taps;
  out[1] = (K * K / taps) * (Cout / wn) * (c48 ? 1 : Cin / wc);
  // resident workgroups per CU: two, except the 5x5 tap-merged 160 x 64 kernel (value layer 0,
  // 49 planes), whose 154 VGPRs leave room for one 8-wave workgroup -- a grid sized for two ran
  // as two rounds (251 us per step, profiles/r3_fp8_wgrad.md)
  out[2] = (taps == 5 && wn == 160 && !c48) ? 1 : 2;
  if (variant == 9 && taps == 1) out[2] = 1;  // the 4-slot ring: one workgroup per CU
  // threads per workgroup
  out[3] = c48 ? 384 : (wn == 160 && wc == 160) ? 256 : 512;
}

void launch_conv_wgrad(const ConvWgradArgs& a_in, hipStream_t st) {
  ConvWgradArgs a = a_in;
  a.divSS = make_fastdiv((uint32_t)(a.S * a.S));
  a.divS = make_fastdiv((uint32_t)a.S);
  a.xcd_group = 1;  // kernel-row workgroups of a split on one XCD (conv_wgrad_kernel)
#ifdef AGK_KERNEL_LAB
  if (a.variant == 5) {
    // one-kernel-row wgrad (conv_wgrad_row.hip), kernel lab: in the power-limited steady state it ran
    // 607-694 us per 192 -> 192 layer against 548-583 us for the per-tap kernel
    // (profiles/r3_wgrad_row.md); layers it does not cover run the per-tap kernel
    const int code = wgrad_row_code(a.Cout, a.Cin, a.cin_real, a.K);
    if (code) {
      wgrad_row_launch(code, a, st);
      return;
    }
    a.variant = 0;
  }
#endif
#ifdef AGK_KERNEL_LAB
  if (a.variant >= 6 && a.variant <= 8) {  // tap pairs (8: DMA spread) / line-staged per-tap kernel
    if (wgrad_pair_applies(a.Cout, a.Cin, a.cin_real, a.K) && launch_conv_wgrad_line_lab(a, st)) return;
    a.variant = 0;
  }
#endif
  if (a.variant == kWgradSmall) {
    // small batches (ops.wgrad_config): 64 x 64 output tiles with the kernel row's taps merged -- three
    // times the workgroups per pixel split of a 192 -> 192 layer
    if (a.Cout % 64 || a.Cin % 64 || a.cin_real != a.Cin || (a.K != 3 && a.K != 5))
      throw std::invalid_argument("conv_wgrad: the small-batch tiles need 64-multiple widths and a 3x3 / 5x5 kernel");
    a.variant = 0;
    launch_wgrad_t<64, 64>(a, st);
    return;
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
// channel), up to 8 16-B loads in flight; the four partials meet in LDS.  The OIHW
// write is strided but touches the (small) gradient once.
__device__ __forceinline__ void wgrad_reduce_body(const WgradReduceArgs& a, int bid, int nblk) {
  __shared__ f32x4 part[4][64];
  const int C4 = a.Cin >> 2;
  const int total = a.T * a.Cout_real * C4;
  const size_t tile = (size_t)a.Cout * a.Cin;
  const size_t sstride = (size_t)a.T * tile;
  const int k = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n4 = a.nsplit & ~3;
  if (bid == 0 && a.grad_b) {
    // bias: one sequential sum per channel (fixed order).  The FIRST block issues it before its share
    // of the slab, so its dependent load-add rounds run under the other blocks; as the last block's
    // epilogue (up to round 6) they were the launch's tail.  16 loads in flight per round.
    for (int n = threadIdx.x; n < a.Cout_real; n += blockDim.x) {
      const float* d = a.dbias_slab + n;
      float sum = 0.f;
      int sp = 0;
      for (; sp + 16 <= a.nsplit; sp += 16) {
        float v[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = d[(size_t)(sp + i) * a.Cout];
#pragma unroll
        for (int i = 0; i < 16; ++i) sum += v[i];
      }
      for (; sp + 8 <= a.nsplit; sp += 8) {
        float v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = d[(size_t)(sp + i) * a.Cout];
#pragma unroll
        for (int i = 0; i < 8; ++i) sum += v[i];
      }
      for (; sp < a.nsplit; ++sp) sum += d[(size_t)sp * a.Cout];
      a.grad_b[n] = (a.beta != 0.f ? a.beta * a.grad_b[n] : 0.f) + a.scale * sum;  // beta 0: no read
    }
  }
  for (int base = bid * 64; base < total; base += nblk * 64) {  // block-uniform trip count
    const int idx = base + lane;
    const int e = idx < total ? idx : total - 1;
    const int c = (e % C4) << 2;
    const int tn = e / C4;
    const int n = tn % a.Cout_real;
    const int t = tn / a.Cout_real;
    const float* s = a.slab + (size_t)t * tile + (size_t)n * a.Cin + c;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if (c < a.Cin_real) {
      // up to 8 of this wave's splits loaded before they are added (round 5: 4 loads in flight left
      // the reduce latency-bound, ~4.4 TB/s); same order of additions as one split at a time
      for (int sp0 = k; sp0 < n4; sp0 += 32) {
        const int cnt = (n4 - sp0 + 3) >> 2;
        const float* p = s + (size_t)sp0 * sstride;
        f32x4 v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i)
          if (i < cnt) v[i] = *(const f32x4*)(p + (size_t)(4 * i) * sstride);
#pragma unroll
        for (int i = 0; i < 8; ++i)
          if (i < cnt) acc += v[i];
      }
      if (k == 0)
        for (int sp = n4; sp < a.nsplit; ++sp) acc += *(const f32x4*)(s + (size_t)sp * sstride);
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
}

__global__ __launch_bounds__(256) void conv_wgrad_reduce_kernel(WgradReduceArgs a) {
  wgrad_reduce_body(a, blockIdx.x, gridDim.x);
}

// Every layer's split-K reduce in ONE launch (the deferred small-batch backward, ops.conv_wgrad_reduce_multi):
// block b runs job j's reduce body as block b - first[j] of nblk[j], the same fixed summation order as
// the per-layer kernel, so the gradients are bitwise equal to twelve separate launches.
__global__ __launch_bounds__(256) void conv_wgrad_reduce_multi_kernel(WgradReduceMultiArgs m) {
  int j = 0;
  while (j + 1 < m.n && (int)blockIdx.x >= m.first[j + 1]) ++j;  // block-uniform
  wgrad_reduce_body(m.job[j], (int)blockIdx.x - m.first[j], m.nblk[j]);
}

static int wgrad_reduce_blocks(const WgradReduceArgs& a) {
  const int total = a.T * a.Cout_real * (a.Cin >> 2);
  int blocks = (total + 63) / 64;
  return blocks > 8192 ? 8192 : blocks;
}

void launch_wgrad_reduce_multi(const std::vector<WgradReduceArgs>& jobs, hipStream_t st) {
  if (jobs.empty()) return;
  if ((int)jobs.size() > kMaxReduceJobs) throw std::invalid_argument("conv_wgrad_reduce_multi: too many layers");
  WgradReduceMultiArgs m{};
  m.n = (int)jobs.size();
  int blocks = 0;
  for (int j = 0; j < m.n; ++j) {
    m.job[j] = jobs[j];
    m.first[j] = blocks;
    m.nblk[j] = wgrad_reduce_blocks(jobs[j]);
    blocks += m.nblk[j];
  }
  hipLaunchKernelGGL(conv_wgrad_reduce_multi_kernel, dim3(blocks), dim3(256), 0, st, m);
}

void launch_wgrad_reduce(const WgradReduceArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(conv_wgrad_reduce_kernel, dim3(wgrad_reduce_blocks(a)), dim3(256), 0, st, a);
}

}  // namespace agk
