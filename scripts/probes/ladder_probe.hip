// Stand-alone driver of the ladder kernels (no torch): reads boards written by
// scripts/probes/ladder_probe_data.py, runs prep + search, compares with the
// CPU bits in the same file: ./ladder_probe data/<set>.bin [threads].
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>


#include "../../alphago_amd/csrc/kernels/ladder.hip"

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                    \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

int main(int argc, char** argv) {
  FILE* f = fopen(argv[1], "rb");
  int hdr[2];
  if (!f || fread(hdr, 4, 2, f) != 2) return 2;
  const int B = hdr[0], S = hdr[1], np = S * S;
  const int threads = argc > 2 ? atoi(argv[2]) : 16384;
  std::vector<int8_t> board((size_t)B * np);
  std::vector<int> meta(2 * B);
  std::vector<uint8_t> ref((size_t)B * np);
  if (fread(board.data(), 1, board.size(), f) != board.size() || fread(meta.data(), 4, meta.size(), f) != meta.size() ||
      fread(ref.data(), 1, ref.size(), f) != ref.size())
    return 2;
  fclose(f);
  int8_t* d_board; int* d_meta; agk::LadderBoard* d_boards; int* d_counts; int* d_off; uint8_t* d_out;
  CK(hipMalloc(&d_board, board.size()));
  CK(hipMalloc(&d_meta, meta.size() * 4));
  CK(hipMalloc(&d_boards, B * sizeof(agk::LadderBoard)));
  CK(hipMalloc(&d_counts, (B + 1) * 4));
  CK(hipMalloc(&d_off, B * 4));
  CK(hipMalloc(&d_out, ref.size()));
  CK(hipMemcpy(d_board, board.data(), board.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(d_meta, meta.data(), meta.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemset(d_counts, 0, (B + 1) * 4));
  CK(hipMemset(d_out, 0, ref.size()));
  agk::LadderArgs a{};
  a.board = d_board; a.meta = d_meta; a.boards = d_boards; a.counts = d_counts; a.counter = d_counts + B;
  a.out = d_out; a.B = B; a.S = S;
  agk::launch_ladder_prep(a, 0);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  std::vector<int> counts(B), off(B);
  CK(hipMemcpy(counts.data(), d_counts, B * 4, hipMemcpyDeviceToHost));
  int tot = 0;
  for (int b = 0; b < B; ++b) { off[b] = tot; tot += counts[b]; }
  printf("prep done: %d tasks\n", tot);
  fflush(stdout);
  CK(hipMemcpy(d_off, off.data(), B * 4, hipMemcpyHostToDevice));
  a.offsets = d_off;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, 0));
  void* frames = nullptr;
  CK(hipMalloc(&frames, (size_t)threads * agk::ladder_frame_bytes()));
  a.frames = frames;
  agk::launch_ladder_search(a, threads, 0);
  CK(hipGetLastError());
  CK(hipEventRecord(e1, 0));
  CK(hipDeviceSynchronize());
  float ms = 0; CK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<uint8_t> got(ref.size());
  CK(hipMemcpy(got.data(), d_out, got.size(), hipMemcpyDeviceToHost));
  int bad = 0, shown = 0;
  for (size_t i = 0; i < got.size(); ++i)
    if (got[i] != ref[i]) { ++bad; if (shown++ < 8) printf("mismatch board %zu point %zu got %d ref %d\n", i / np, i % np, got[i], ref[i]); }
  printf("search %.3f ms, %d mismatches\n", ms, bad);
  return bad != 0;
}
