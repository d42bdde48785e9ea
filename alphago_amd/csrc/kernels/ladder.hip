// Ladder planes on the GPU (the reference's ladder_capture / ladder_escape are
// NotImplementedError, AlphaGo/preprocessing/preprocessing.py:147-152; our CPU
// reader is featurize.cpp).  The search code is ../engine/ladder_bb.h, the same
// bitboard reader the host tests check bit for bit against the CPU reader.
//
// ladder_prep_kernel: one wave per board.  Ballots turn the int8 board into
//   black / white bitboards (word k = ballot over points 64k + lane); every
//   lane then tests its points for candidacy (an empty liberty of an opponent
//   group with 2 liberties or of an own group in atari) and a ballot per word
//   gives the candidate set and its population.
// ladder_search_kernel: persistent grid; candidate tasks are enumerated through
//   the per-board exclusive offsets and claimed from a global counter; each
//   thread runs the iterative ladder search for its (board, point) with its
//   frame stack in a global workspace and writes bits (1 = ladder capture,
//   2 = ladder escape, 4 = step budget exhausted) into a zeroed (B, S*S) array.
//
// Measured (profiles/r2_gpu_ladders.md): bit-exact, but slower than the host
// reader -- a ladder search is a deep serial chain of dependent bitboard
// operations (up to ~4k plies of search for one root on random positions), a
// wave issues one VALU op per 4 cycles, and lanes of a wave walk unrelated
// searches.  A wave-per-task variant (wave-uniform scalar code, frame stack in
// LDS) was slower still.  The featurizer therefore reads ladders on the host
// by default (GpuFeaturizer(gpu_ladders=False)).
#include <hip/hip_runtime.h>

#include "../engine/ladder_bb.h"
#include "common.h"
#include "kernels.h"

namespace agk {

__global__ __launch_bounds__(64) void ladder_prep_kernel(LadderArgs a) {
  const int b = blockIdx.x;
  const int lane = threadIdx.x;
  lb::Geo g;
  lb::make_geo(g, a.S);
  const int np = a.S * a.S;
  const int8_t* brd = a.board + (size_t)b * np;
  lb::LState s;
#pragma unroll
  for (int k = 0; k < lb::W; ++k) {
    const int p = k * 64 + lane;
    const int v = p < np ? brd[p] : 0;
    s.black.w[k] = __ballot(v > 0);
    s.white.w[k] = __ballot(v < 0);
  }
  s.ko = a.meta[2 * b];
  const int me = a.meta[2 * b + 1];
  lb::BB cand;
  int count = 0;
#pragma unroll 1
  for (int k = 0; k < lb::W; ++k) {
    const int p = k * 64 + lane;
    const bool c = p < np && lb::is_candidate(s, p, me, g);
    cand.w[k] = __ballot(c);
    count += __popcll(cand.w[k]);
  }
  LadderBoard* out = a.boards + b;
  if (lane < lb::W) {  // one word per lane (vector stores)
    out->black[lane] = s.black.w[lane];
    out->white[lane] = s.white.w[lane];
    out->cand[lane] = cand.w[lane];
  }
  if (lane == lb::W) {
    out->ko = s.ko;
    out->me = me;
    a.counts[b] = count;
  }
}

// Thread per (board, point) task, frame stacks in a global workspace
// (kMaxFrames snapshots per thread).  Tasks are claimed from a global counter
// so long ladders do not hold up a statically assigned share; every thread
// leaves the loop once the counter passes the task total.
__global__ __launch_bounds__(64) void ladder_search_kernel(LadderArgs a) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  const int B = a.B;
  const int total = a.offsets[B - 1] + a.counts[B - 1];
  lb::Geo g;
  lb::make_geo(g, a.S);
  const int np = a.S * a.S;
  lb::Frame* stack = reinterpret_cast<lb::Frame*>(a.frames) + (size_t)tid * lb::kMaxFrames;
  while (true) {
    const int task = atomicAdd(a.counter, 1);
    if (task >= total) break;
    // board = last b with offsets[b] <= task
    int lo = 0, hi = B - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (a.offsets[mid] <= task) lo = mid;
      else hi = mid - 1;
    }
    const int b = lo;
    const LadderBoard& bd = a.boards[b];
    int idx = task - a.offsets[b];
    int p = -1;
    for (int k = 0; k < lb::W && p < 0; ++k) {
      uint64_t w = bd.cand[k];
      const int c = __popcll(w);
      if (idx >= c) {
        idx -= c;
        continue;
      }
      for (int t = 0; t < idx; ++t) w &= w - 1;  // drop the idx lowest set bits
      p = k * 64 + (__ffsll((long long)w) - 1);
    }
    if (p < 0 || p >= np) continue;
    lb::LState s;
    for (int k = 0; k < lb::W; ++k) {
      s.black.w[k] = bd.black[k];
      s.white.w[k] = bd.white[k];
    }
    s.ko = bd.ko;
    a.out[(size_t)b * np + p] = (uint8_t)lb::ladder_bits_at(s, p, bd.me, stack, g, a.budget);
  }
}

void launch_ladder_prep(const LadderArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(ladder_prep_kernel, dim3(a.B), dim3(64), 0, st, a);
}

void launch_ladder_search(const LadderArgs& a, int threads, hipStream_t st) {
  hipLaunchKernelGGL(ladder_search_kernel, dim3((threads + 63) / 64), dim3(64), 0, st, a);
}

size_t ladder_frame_bytes() { return sizeof(lb::Frame) * lb::kMaxFrames; }

}  // namespace agk
