// Winograd F(2x2, 3x3) forward convolution -- kernel lab ("settle Winograd on
// energy, with a kill criterion").  Reference layer: the 3x3 trunk of the policy net
// (/root/reference/AlphaGo/models/policy.py:132-142), 192 -> 192 channels on 19 x 19 boards.
//
// Y = A^T [ U (.) V ] A per 2 x 2 output tile, U = G g G^T (weights, transformed and packed once per
// step on the host side of the lab), V = B^T d B (the 4 x 4 input patch).  16 products (xi) per tile
// and channel pair instead of 36 MACs for 4 outputs: the 10 x 10 tiles of a 19 x 19 board do
// 16 * 100 / (9 * 361) = 0.49x the direct kernel's MFMA work.
//
// Workgroup: 32 tiles x 192 output channels, 8 waves = 2 tile blocks x 4 channel groups; every wave
// keeps all 16 xi of its 16 tiles x 48 channels in accumulators (192 fp32 per lane), so the output
// transform, bias and ReLU run in registers.  Per 32-channel K-step:
//   1. every thread transforms one (tile, channel pair): 16 dword loads of the patch, B^T d B in fp32 (row then column differences), 16 bf16x2 writes to LDS;
//   2. every wave runs 16 xi x 3 MFMA 16x16x32: A = V[xi] of its 16 tiles from LDS (one
//      ds_read_b128 per xi, XOR-swizzled 16-B units: conflict-free for the b128 lane groups), B =
//      the transformed weights straight from L2 (one 16-B load per lane and fragment, the next xi's
//      three fragments in flight while this xi multiplies).
// The packed weights hold 16 x Cin x Cout bf16 (1.18 MB at 192): every workgroup streams all of
// them, 16/9 of the direct kernel's weight bytes for a quarter of its output pixels per workgroup.
// That is the operand-traffic side of the trade this lab kernel exists to measure
// (profiles/r3_winograd.md).
#include <hip/hip_runtime.h>

#include <stdexcept>

#include "common.h"
#include "kernels.h"

namespace agk {

namespace {

constexpr int kWinoTiles = 32;                    // tiles per workgroup
constexpr int kWinoVBytes = 16 * kWinoTiles * 64;  // one K-step of V: [16 xi][32 tiles][32 ch] bf16

// 16-B unit swizzle of a V row (tile): unit u of tile t is stored at u ^ f((t >> 2) & 3),
// f = {0, 3, 2, 1}.  The four 16-lane groups of ds_read_b128 each read 16 tiles x one unit pattern
// (lanes 0-3 / 12-15 / 20-27 ...); with this f every group covers the 64 banks exactly once.
__device__ __forceinline__ int wino_swz(int t) { return (-((t >> 2) & 3)) & 3; }

__device__ __forceinline__ int wino_voff(int xi, int tile, int unit) {
  return (xi * kWinoTiles + tile) * 64 + ((unit ^ wino_swz(tile)) << 4);
}

__device__ __forceinline__ float bf_lo(unsigned v) { return __uint_as_float(v << 16); }
__device__ __forceinline__ float bf_hi(unsigned v) { return __uint_as_float(v & 0xffff0000u); }
__device__ __forceinline__ unsigned pack_bf2(float lo, float hi) {
  typedef __attribute__((ext_vector_type(2))) __bf16 bf2;
  bf2 v = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(unsigned, v);
}

template <int NG>
__global__ __launch_bounds__(512, 1) void wino_fwd_kernel(WinoArgs a) {
  constexpr int BNW = NG * 16;  // output channels per wave
  constexpr int BN = 4 * BNW;   // per workgroup
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
  const int mb = wave >> 2, ng = wave & 3;
  const int t0 = blockIdx.x * kWinoTiles;
  const int nw0 = blockIdx.y * BN + ng * BNW;  // first output channel of the wave
  const int HP = a.S + 2;
  const int TT = a.TS * a.TS;
  const int nks = a.Cin >> 5;
  const int nbs = a.Cout >> 4;

  // ---- transform role: thread -> (tile tt, channel pair cp)
  const int tt = tid >> 4, cp = tid & 15;
  int tg = t0 + tt;
  tg = tg < a.ntiles ? tg : a.ntiles - 1;
  int b = tg / TT;
  int rem = tg - b * TT;
  int ty = rem / a.TS;
  int tx = rem - ty * a.TS;
  // patch pixel (r, s) = padded (2ty + r, 2tx + s); for odd S the last tile row/column reaches row
  // HP, outside the image: zero (it only feeds outputs beyond the board)
  const int rlim = HP - 2 * ty, slim = HP - 2 * tx;
  const __bf16* xp = a.x + ((size_t)(b * HP + 2 * ty) * HP + 2 * tx) * a.Cin + 2 * cp;
  unsigned xr[16];
  auto load_x = [&](int ks) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        unsigned v = 0u;
        if (r < rlim && s < slim) v = *(const unsigned*)(xp + (r * HP + s) * a.Cin + ks * 32);
        xr[r * 4 + s] = v;
      }
  };
  auto transform_store = [&](char* vb) {
    // two channels (lo / hi bf16 halves of each dword) in fp32, one column j of V at a time
    const int unit = cp >> 2, sub = (cp & 3) * 4;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float t[4][2];  // (d B)[r][j]: column differences within each patch row
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const unsigned* d = xr + r * 4;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const float d0 = h ? bf_hi(d[0]) : bf_lo(d[0]), d1 = h ? bf_hi(d[1]) : bf_lo(d[1]);
          const float d2 = h ? bf_hi(d[2]) : bf_lo(d[2]), d3 = h ? bf_hi(d[3]) : bf_lo(d[3]);
          t[r][h] = j == 0 ? d0 - d2 : j == 1 ? d1 + d2 : j == 2 ? d2 - d1 : d1 - d3;
        }
      }
      float v[4][2];  // B^T (d B): row differences
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        v[0][h] = t[0][h] - t[2][h];
        v[1][h] = t[1][h] + t[2][h];
        v[2][h] = t[2][h] - t[1][h];
        v[3][h] = t[1][h] - t[3][h];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
        *(unsigned*)(vb + wino_voff(i * 4 + j, tt, unit) + sub) = pack_bf2(v[i][0], v[i][1]);
    }
  };

  // ---- multiply role
  f32x4 acc[16][NG];
#pragma unroll
  for (int x = 0; x < 16; ++x)
#pragma unroll
    for (int j = 0; j < NG; ++j) acc[x][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int arow = mb * 16 + (lane & 15);
  const int aunit = lane >> 4;
  typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
  const u32x4* up = reinterpret_cast<const u32x4*>(a.u);
  const int nb0 = nw0 >> 4;
  auto bfrag = [&](int xi, int ks, int j) {
    const u32x4 v = up[((size_t)(xi * nks + ks) * nbs + nb0 + j) * 64 + lane];
    return __builtin_bit_cast(bf16x8, v);
  };

  load_x(0);
  transform_store(smem);
  __syncthreads();
  for (int ks = 0; ks < nks; ++ks) {
    const char* vb = smem + (ks & 1) * kWinoVBytes;
    // B fragments: the next xi's three are in flight while this xi multiplies
    bf16x8 bc[NG], bn[NG];
#pragma unroll
    for (int j = 0; j < NG; ++j) bc[j] = bfrag(0, ks, j);
#pragma unroll
    for (int xi = 0; xi < 16; ++xi) {
      if (xi + 1 < 16) {
#pragma unroll
        for (int j = 0; j < NG; ++j) bn[j] = bfrag(xi + 1, ks, j);
      }
      const bf16x8 av = *(const bf16x8*)(vb + wino_voff(xi, arow, aunit));
#pragma unroll
      for (int j = 0; j < NG; ++j) acc[xi][j] = mfma16x16x32(av, bc[j], acc[xi][j]);
#pragma unroll
      for (int j = 0; j < NG; ++j) bc[j] = bn[j];
      __builtin_amdgcn_sched_barrier(0);
    }
    if (ks + 1 < nks) {  // the patch loads are not held across the multiplies (192 accumulators)
      load_x(ks + 1);
      transform_store(smem + ((ks + 1) & 1) * kWinoVBytes);
    }
    __syncthreads();
  }

  // ---- epilogue: Y = A^T M A per (tile, channel), bias + ReLU, bf16 stores
  const int HPo = a.S + 2;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    int tgo = t0 + mb * 16 + 4 * (lane >> 4) + r;
    const bool ok = tgo < a.ntiles;
    tgo = ok ? tgo : a.ntiles - 1;
    const int bo = tgo / TT;
    const int ro = tgo - bo * TT;
    const int tyo = ro / a.TS, txo = ro - (ro / a.TS) * a.TS;
#pragma unroll
    for (int j = 0; j < NG; ++j) {
      const int n = nw0 + j * 16 + (lane & 15);
      float m[4][4];
#pragma unroll
      for (int x = 0; x < 16; ++x) m[x >> 2][x & 3] = acc[x][j][r];
      float p[2][4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        p[0][c] = m[0][c] + m[1][c] + m[2][c];
        p[1][c] = m[1][c] - m[2][c] - m[3][c];
      }
      const float bb = a.bias ? a.bias[n] : 0.f;
#pragma unroll
      for (int aa = 0; aa < 2; ++aa) {
        const float y0 = p[aa][0] + p[aa][1] + p[aa][2];
        const float y1 = p[aa][1] - p[aa][2] - p[aa][3];
        const int oy = 2 * tyo + aa, ox = 2 * txo;
        if (ok && oy < a.S) {
          __bf16* yo = a.y + ((size_t)(bo * HPo + oy + 1) * HPo + ox + 1) * a.Cout + n;
          yo[0] = (__bf16)fmaxf(y0 + bb, 0.f);
          if (ox + 1 < a.S) yo[a.Cout] = (__bf16)fmaxf(y1 + bb, 0.f);
        }
      }
    }
  }
}

}  // namespace

void launch_wino_fwd(const WinoArgs& a, hipStream_t st) {
  if (a.Cout % 192 != 0 || a.Cin % 32 != 0)
    throw std::invalid_argument("wino_fwd: Cout % 192 == 0 and Cin % 32 == 0");
  constexpr int smem = 2 * kWinoVBytes;
  static const hipError_t attr =
      hipFuncSetAttribute((const void*)wino_fwd_kernel<3>, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
  hip_check(attr, "hipFuncSetAttribute(max dynamic LDS)");
  dim3 grid((a.ntiles + kWinoTiles - 1) / kWinoTiles, a.Cout / 192);
  hipLaunchKernelGGL(wino_fwd_kernel<3>, grid, dim3(512), smem, st, a);
}

}  // namespace agk
