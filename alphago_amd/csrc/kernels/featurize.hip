// GPU board featurizer: the reference's feature planes
// (AlphaGo/preprocessing/preprocessing.py:9-214) computed on the device from a
// compact per-board encoding, one workgroup (6 waves, one lane per point) per
// board.
//
// Input per board (written by the C++ engine, ~2 bytes per point):
//   board[p] in {-1, 0, +1};  ages[p] = turns_since plane (0..7) or 255;
//   meta = {ko point or -1, player to move};  optional ladder bits
//   (bit0 capture, bit1 escape) when a ladder plane is requested — ladder
//   reading is a sequential tree search and stays on the CPU.
// Steps, all in LDS: group labels by min-label propagation with pointer
// jumping (a label is the smallest point index of its chain); stone counts
// (LDS atomicAdd) and liberty bitsets per chain root (6 x u64, ds_or_b64);
// then each lane evaluates its point: legality (ko + suicide, go.py:181-216),
// capture size, self-atari size, liberties-after (incl. the 0-liberty ->
// plane 7 quirk) and the reference's recursive true-eye test
// (go.py:230-259) as an explicit DFS whose "stack" is the chain of ancestor
// frames, so sensibleness matches the CPU featurizer bit-for-bit.
// Outputs (each optional): uint8 planes [B][F][S][S]; the conv trunk's padded
// NHWC bf16 input [B][S+2P][S+2P][Cp] (interior written, borders untouched);
// the sensible-move mask [B][S*S] (policy renormalisation / MCTS priors);
// an overflow flag per board (eye recursion deeper than the frame stack:
// the caller recomputes that board on the CPU).
#include <hip/hip_runtime.h>

#include "common.h"
#include "kernels.h"

namespace agk {

constexpr int FZ_THREADS = 384;
constexpr int FZ_MAXP = 384;
constexpr int EYE_MAX_DEPTH = 40;
// The reference recursion re-explores shared sub-chains, so its cost is
// exponential in the length of a diagonal chain of eyeish points (a 9x9
// checkerboard takes ~30 s on the CPU).  The kernel bounds the frames it
// visits and flags the board instead; the host then recomputes it.
constexpr int EYE_MAX_FRAMES = 2048;

// feature ids (same numbering as the CPU featurizer, engine/featurize.h)
enum {
  FZ_BOARD = 0, FZ_ONES, FZ_TURNS, FZ_LIBS, FZ_CAPTURE, FZ_SELF_ATARI, FZ_LIBS_AFTER,
  FZ_LADDER_CAPTURE, FZ_LADDER_ESCAPE, FZ_SENSIBLE, FZ_ZEROS, FZ_COLOR, FZ_LEGAL, FZ_NUM
};

__device__ __forceinline__ int fz_nbrs(int p, int S, int* out) {
  const int x = p / S, y = p - x * S;
  int k = 0;
  if (x > 0) out[k++] = p - S;
  if (x < S - 1) out[k++] = p + S;
  if (y > 0) out[k++] = p - 1;
  if (y < S - 1) out[k++] = p + 1;
  return k;
}

__device__ __forceinline__ int fz_diags(int p, int S, int* out) {
  const int x = p / S, y = p - x * S;
  int k = 0;
  if (x > 0 && y > 0) out[k++] = p - S - 1;
  if (x < S - 1 && y < S - 1) out[k++] = p + S + 1;
  if (x < S - 1 && y > 0) out[k++] = p + S - 1;
  if (x > 0 && y < S - 1) out[k++] = p - S + 1;
  return k;
}

__device__ __forceinline__ bool fz_eyeish(const signed char* bd, int p, int owner, int S) {
  if (bd[p] != 0) return false;
  int nb[4];
  const int k = fz_nbrs(p, S, nb);
  for (int i = 0; i < k; ++i)
    if (bd[nb[i]] != owner) return false;
  return true;
}

// Iterative form of GameState::is_eye_rec.  Frame i's "stack" is the points
// of frames 0..i-1.  Returns 1 eye, 0 not an eye, -1 depth/work overflow.
__device__ int fz_is_eye(const signed char* bd, int p0, int owner, int S) {
  if (!fz_eyeish(bd, p0, owner, S)) return 0;
  short pt[EYE_MAX_DEPTH];
  unsigned char di[EYE_MAX_DEPTH], bad[EYE_MAX_DEPTH];
  int depth = 1;
  pt[0] = (short)p0;
  di[0] = 0;
  bad[0] = 0;
  int child = -1;  // pending result of the frame just popped (-1: none)
  int frames = 1;
  while (true) {
    const int f = depth - 1;
    const int cur = pt[f];
    int nb[4], dg[4];
    const int allow = (fz_nbrs(cur, S, nb) == 4) ? 1 : 0;
    const int nd = fz_diags(cur, S, dg);
    int ret = -1;  // -1 running, 0/1 returned, 2 descended
    if (child >= 0) {
      if (child == 0) bad[f]++;
      child = -1;
      if (bad[f] > allow) ret = 0;
    }
    while (ret == -1 && di[f] < nd) {
      const int d = dg[di[f]++];
      const int v = bd[d];
      if (v == -owner) {
        bad[f]++;
      } else if (v == 0) {
        bool on_stack = false;
        for (int a = 0; a < f; ++a) on_stack |= (pt[a] == d);
        if (!on_stack) {
          if (!fz_eyeish(bd, d, owner, S)) {
            bad[f]++;
          } else {
            if (depth >= EYE_MAX_DEPTH || ++frames > EYE_MAX_FRAMES) return -1;
            pt[depth] = (short)d;
            di[depth] = 0;
            bad[depth] = 0;
            ++depth;
            ret = 2;
            break;
          }
        }
      }
      if (bad[f] > allow) ret = 0;
    }
    if (ret == 2) continue;
    if (ret == -1) ret = 1;
    --depth;
    if (depth == 0) return ret;
    child = ret;
  }
}

__global__ __launch_bounds__(FZ_THREADS) void featurize_kernel(FeaturizeArgs a) {
  __shared__ signed char bd[FZ_MAXP];
  __shared__ short lab[FZ_MAXP];
  __shared__ int gsz[FZ_MAXP];
  __shared__ unsigned long long libs[FZ_MAXP][6];
  const int b = blockIdx.x;
  const int p = threadIdx.x;
  const int S = a.S, NP = S * S;
  const bool on = p < NP;
  const int ko = a.meta[2 * b], me = a.meta[2 * b + 1];
  int v = 0;
  if (on) {
    v = a.board[(size_t)b * NP + p];
    bd[p] = (signed char)v;
    lab[p] = v != 0 ? (short)p : (short)-1;
    gsz[p] = 0;
#pragma unroll
    for (int w = 0; w < 6; ++w) libs[p][w] = 0ull;
  }
  __syncthreads();

  int nb[4];
  const int nn = on ? fz_nbrs(p, S, nb) : 0;
  // ---- chain labels.  Labels only decrease and always name a stone of the
  // same chain, so unsynchronised reads within a sweep are benign.
  while (true) {
    int changed = 0;
    if (on && v != 0) {
      int m = lab[p];
      for (int i = 0; i < nn; ++i)
        if (bd[nb[i]] == v) m = min(m, (int)lab[nb[i]]);
      m = min(m, (int)lab[m]);
      if (m < lab[p]) {
        lab[p] = (short)m;
        changed = 1;
      }
    }
    if (!__syncthreads_or(changed)) break;
  }
  // ---- chain sizes and liberty sets, accumulated at the root
  if (on) {
    if (v != 0) {
      atomicAdd(&gsz[lab[p]], 1);
    } else {
      const unsigned long long bit = 1ull << (p & 63);
      for (int i = 0; i < nn; ++i) {
        const int r = lab[nb[i]];
        if (r >= 0) atomicOr(&libs[r][p >> 6], bit);
      }
    }
  }
  __syncthreads();

  // ---- per-point features
  // hot[f]: plane index (within feature f) that is 1 at this point, or -1.
  int hot[FZ_NUM];
#pragma unroll
  for (int f = 0; f < FZ_NUM; ++f) hot[f] = -1;
  int legal = 0, sensible = 0, overflow = 0;
  if (on) {
    hot[FZ_BOARD] = v == me ? 0 : (v == -me ? 1 : 2);
    hot[FZ_ONES] = 0;
    hot[FZ_COLOR] = me == 1 ? 0 : -1;
    const int age = a.ages[(size_t)b * NP + p];
    hot[FZ_TURNS] = age < 8 ? age : -1;
    if (v != 0) {
      const int r = lab[p];
      int lc = 0;
#pragma unroll
      for (int w = 0; w < 6; ++w) lc += __popcll(libs[r][w]);
      hot[FZ_LIBS] = lc >= 8 ? 7 : lc - 1;
    } else if (p != ko) {
      // distinct neighbouring chains
      int roots[4], nr = 0;
      bool has_empty = false;
      for (int i = 0; i < nn; ++i) {
        const int r = lab[nb[i]];
        if (r < 0) {
          has_empty = true;
          continue;
        }
        bool dup = false;
        for (int j = 0; j < nr; ++j) dup |= roots[j] == r;
        if (!dup) roots[nr++] = r;
      }
      int rlc[4];
      for (int j = 0; j < nr; ++j) {
        int c = 0;
#pragma unroll
        for (int w = 0; w < 6; ++w) c += __popcll(libs[roots[j]][w]);
        rlc[j] = c;
      }
      // suicide test (every neighbouring chain has p as a liberty)
      legal = has_empty;
      for (int j = 0; j < nr && !legal; ++j) {
        const int col = bd[roots[j]];
        if (col == me && rlc[j] > 1) legal = 1;
        if (col == -me && rlc[j] == 1) legal = 1;
      }
      if (legal) {
        int ncap = 0, own = 1;
        unsigned long long L[6];
#pragma unroll
        for (int w = 0; w < 6; ++w) L[w] = 0ull;
        for (int i = 0; i < nn; ++i)
          if (bd[nb[i]] == 0) L[nb[i] >> 6] |= 1ull << (nb[i] & 63);
        for (int j = 0; j < nr; ++j) {
          const int r = roots[j];
          if (bd[r] == me) {
            own += gsz[r];
#pragma unroll
            for (int w = 0; w < 6; ++w) L[w] |= libs[r][w];
          } else if (rlc[j] == 1) {
            ncap += gsz[r];
          }
        }
        L[p >> 6] &= ~(1ull << (p & 63));
        int nl = 0;
#pragma unroll
        for (int w = 0; w < 6; ++w) nl += __popcll(L[w]);
        hot[FZ_CAPTURE] = ncap > 7 ? 7 : ncap;
        if (nl == 1) hot[FZ_SELF_ATARI] = own - 1 > 7 ? 7 : own - 1;
        hot[FZ_LIBS_AFTER] = nl - 1 > 7 ? 7 : (nl - 1 < 0 ? 7 : nl - 1);
        hot[FZ_LEGAL] = 0;
        int eye = 0;
        if (a.need_eye) {
          eye = fz_is_eye(bd, p, me, S);
          if (eye < 0) overflow = 1;
        }
        sensible = eye == 0;
        hot[FZ_SENSIBLE] = sensible ? 0 : -1;
        if (a.ladder) {
          const int lb = a.ladder[(size_t)b * NP + p];
          hot[FZ_LADDER_CAPTURE] = (lb & 1) ? 0 : -1;
          hot[FZ_LADDER_ESCAPE] = (lb & 2) ? 0 : -1;
        }
      }
    }
  }
  if (a.overflow && __syncthreads_or(overflow) && p == 0) a.overflow[b] = 1;
  if (!on) return;
  if (a.sensible) a.sensible[(size_t)b * NP + p] = (uint8_t)sensible;
  if (a.legal) a.legal[(size_t)b * NP + p] = (uint8_t)legal;
  if (a.planes) {
    uint8_t* o = a.planes + (size_t)b * a.nplanes * NP + p;
    for (int i = 0, c = 0; i < a.nf; ++i) {
      const int f = a.fids[i];
      const int npl = a.fplanes[i];
      int h = -1;
#pragma unroll
      for (int g = 0; g < FZ_NUM; ++g)
        if (g == f) h = hot[g];
      for (int k = 0; k < npl; ++k, ++c) o[(size_t)c * NP] = (uint8_t)(h == k);
    }
  }
  if (a.nhwc) {
    const int x = p / S, y = p - x * S;
    const int HP = S + 2 * a.P;
    __bf16* o = a.nhwc + (((size_t)b * HP + x + a.P) * HP + y + a.P) * a.Cp;
    // channel c -> (feature slot, plane) through the per-launch table
    for (int c0 = 0; c0 < a.Cp; c0 += 8) {
      bf16x8 pk;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = c0 + j;
        float val = 0.f;
        if (c < a.nplanes) {
          const int f = a.chan_feat[c];
          int h = -1;
#pragma unroll
          for (int g = 0; g < FZ_NUM; ++g)
            if (g == f) h = hot[g];
          val = (h == a.chan_plane[c]) ? 1.f : 0.f;
        }
        pk[j] = (__bf16)val;
      }
      *reinterpret_cast<bf16x8*>(o + c0) = pk;
    }
  }
}

void launch_featurize(const FeaturizeArgs& a, hipStream_t st) {
  if (a.B <= 0) return;
  hipLaunchKernelGGL(featurize_kernel, dim3(a.B), dim3(FZ_THREADS), 0, st, a);
}

}  // namespace agk
