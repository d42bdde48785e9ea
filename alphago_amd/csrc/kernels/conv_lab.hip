// Kernel-lab conv variants (built into _hip_kernels_lab.so only): the forward with the pixel
// operand straight from L2 (tile 11), the lab tile codes of the forward (conv_fwd_variants.hip and
// other instantiations of conv_fwd_kernel), and the wgrad variants (256-thread tile, LDS ring).
// Results: profiles/r1_fwd_kernel_experiments.md, profiles/r2_wgrad_variants.md.
#include <hip/hip_runtime.h>

#include "conv_kernels.h"

namespace agk {

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

template <int WN, int WC, int NS>
static void launch_wgrad_ring(const ConvWgradArgs& a, dim3 grid, hipStream_t st) {
  constexpr int smem = NS * (WN + WC) * 64;
  static const hipError_t attr = hipFuncSetAttribute((const void*)conv_wgrad_ring_kernel<WN, WC, NS>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        smem);  // once per instantiation (thread-safe static)
  hip_check(attr, "hipFuncSetAttribute(max dynamic LDS)");
  hipLaunchKernelGGL((conv_wgrad_ring_kernel<WN, WC, NS>), grid, dim3(512), smem, st, a);
}

template <int BN, int MODE>
static bool lab_fwd_t(int bm, const ConvFwdArgs& a, hipStream_t st) {
  // conv_fwd_variants.hip (-1, 2, 4, 5, 6, 32), 2560 (epilogue loads after the loop), 2568 (BM 256,
  // 128-pixel waves), 11 (pixel operand from L2), 9 / 10 (DMA spread through the MFMAs), 7 / 8
  // (32x32x16 MFMA)
  const bool var = bm == -1 || bm == 2 || bm == 4 || bm == 5 || bm == 6 || bm == 32;
  if (var && launch_conv_fwd_variant(bm, a, MODE, st)) return true;
  if (var) launch_fwd_bm<BN, MODE, 128, 4>(a, st);
  else if (bm == 2560) launch_fwd_bm<BN, MODE, 256, 4, false>(a, st);
  else if (bm == 2568) launch_fwd_bm<BN, MODE, 256, 8>(a, st);
  else if (bm == 11) launch_fwd_ga<BN, MODE>(a, st);
  else if (bm == 9) launch_fwd_bm<BN, MODE, 384, 6, false, false, false, true>(a, st);
  else if (bm == 10) launch_fwd_bm<BN, MODE, 256, 4, false, false, false, true>(a, st);
  else if (bm == 7) launch_fwd_bm<BN, MODE, 384, 6, false, false, true>(a, st);
  else if (bm == 8) launch_fwd_bm<BN, MODE, 256, 4, false, false, true>(a, st);
  else return false;
  return true;
}

template <int MODE>
static bool lab_fwd_m(int bm, const ConvFwdArgs& a, int bn, hipStream_t st) {
  if (bn == 192) return lab_fwd_t<192, MODE>(bm, a, st);
  if (bn == 128) return lab_fwd_t<128, MODE>(bm, a, st);
  if (bn == 64) return lab_fwd_t<64, MODE>(bm, a, st);
  return false;
}

bool launch_conv_fwd_lab(int bm, const ConvFwdArgs& a, int bn, int mode, hipStream_t st) {
  if (mode == MODE_BIAS_RELU) return lab_fwd_m<MODE_BIAS_RELU>(bm, a, bn, st);
  if (mode == MODE_MASK) return lab_fwd_m<MODE_MASK>(bm, a, bn, st);
  if (mode == MODE_MASKBITS) return lab_fwd_m<MODE_MASKBITS>(bm, a, bn, st);
  return lab_fwd_m<MODE_NONE>(bm, a, bn, st);
}

// wgrad variants: 2 = 256-thread tile, 3 / 4 = LDS ring with that many slots
template <int WN, int WC>
static bool lab_wgrad_t(const ConvWgradArgs& a, dim3 grid, hipStream_t st) {
  if (a.variant == 3 || a.variant == 4) {
    if (a.variant == 3) launch_wgrad_ring<WN, WC, 3>(a, grid, st);
    else launch_wgrad_ring<WN, WC, 4>(a, grid, st);
    return true;
  }
  if constexpr (WC % 32 == 0 && WC >= 64) {
    if (a.variant == 2) {
      constexpr int smem = 2 * (WN + WC) * 64 * kWgradKsub;
      static const hipError_t attr2 = hipFuncSetAttribute((const void*)conv_wgrad_kernel<WN, WC, kWgradKsub, 2>,
                                                          hipFuncAttributeMaxDynamicSharedMemorySize, smem);
      hip_check(attr2, "hipFuncSetAttribute(max dynamic LDS)");
      hipLaunchKernelGGL((conv_wgrad_kernel<WN, WC, kWgradKsub, 2>), grid, dim3(256), smem, st, a);
      return true;
    }
  }
  return false;
}

bool launch_conv_wgrad_lab(const ConvWgradArgs& a, int wn, int wc, dim3 grid, hipStream_t st) {
  if (wn == 192 && wc == 192) return lab_wgrad_t<192, 192>(a, grid, st);
  if (wn == 192 && wc == 128) return lab_wgrad_t<192, 128>(a, grid, st);
  if (wn == 192 && wc == 64) return lab_wgrad_t<192, 64>(a, grid, st);
  if (wn == 128 && wc == 128) return lab_wgrad_t<128, 128>(a, grid, st);
  if (wn == 128 && wc == 192) return lab_wgrad_t<128, 192>(a, grid, st);
  if (wn == 128 && wc == 64) return lab_wgrad_t<128, 64>(a, grid, st);
  if (wn == 64 && wc == 192) return lab_wgrad_t<64, 192>(a, grid, st);
  if (wn == 64 && wc == 128) return lab_wgrad_t<64, 128>(a, grid, st);
  if (wn == 64 && wc == 64) return lab_wgrad_t<64, 64>(a, grid, st);
  if (wn == 160 && wc == 64) return lab_wgrad_t<160, 64>(a, grid, st);
  return false;
}

// tap-pair wgrad (conv_wgrad_kernel PAIR): 192 x 192 x 2 taps per workgroup, 64-pixel stages,
// one workgroup per CU; grid y = ceil(T / 2), the last y runs the odd tap over split pairs

template <bool ILVW>
static void launch_wgrad_pair(ConvWgradArgs a, hipStream_t st) {
  constexpr int KS = 2;
  constexpr int smem = 2 * (192 + 2 * 192) * 64 * KS;  // 144 KB
  static const hipError_t attr = hipFuncSetAttribute(
      (const void*)conv_wgrad_kernel<192, 192, KS, 4, 2, true, true, ILVW>, hipFuncAttributeMaxDynamicSharedMemorySize,
      smem);
  hip_check(attr, "hipFuncSetAttribute(max dynamic LDS)");
  const int nks = (a.M + 32 * KS - 1) / (32 * KS);  // the op computed ksteps in 32-pixel units
  a.ksteps_per_split = (nks + a.nsplit - 1) / a.nsplit;
  dim3 grid(a.nsplit, (a.T + 1) / 2, 1);
  hipLaunchKernelGGL((conv_wgrad_kernel<192, 192, KS, 4, 2, true, true, ILVW>), grid, dim3(512), smem, st, a);
}

// per-tap kernel with line staging (variant 7): the production tile and grid, whole 128-byte
// pixel lines per DMA piece
static void launch_wgrad_line(const ConvWgradArgs& a, hipStream_t st) {
  constexpr int KS = kWgradKsub;
  constexpr int smem = 2 * (192 + 192) * 64 * KS;
  static const hipError_t attr = hipFuncSetAttribute((const void*)conv_wgrad_kernel<192, 192, KS, 4, 1, false, true>,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, smem);
  hip_check(attr, "hipFuncSetAttribute(max dynamic LDS)");
  dim3 grid(a.nsplit, a.T, 1);
  hipLaunchKernelGGL((conv_wgrad_kernel<192, 192, KS, 4, 1, false, true>), grid, dim3(512), smem, st, a);
}

// variants 6 (tap pairs), 7 (per tap, line staging), 8 (tap pairs, DMA spread); 192 x 192 3x3 only
bool launch_conv_wgrad_line_lab(const ConvWgradArgs& a, hipStream_t st) {
  if (a.variant == 6) launch_wgrad_pair<false>(a, st);
  else if (a.variant == 8) launch_wgrad_pair<true>(a, st);
  else if (a.variant == 7) launch_wgrad_line(a, st);
  else return false;
  return true;
}

}  // namespace agk
