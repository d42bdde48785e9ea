// Native self-test driver for the C++ engine (rules, featurizer, encoder,
// batched MCTS forest), built standalone so it can run under host sanitizers:
//   python -m alphago_amd._build selftest --sanitize address,undefined
//   python -m alphago_amd._build selftest --sanitize thread
// (SURVEY.md §5 "Race detection / sanitizers".)  Every move of many random
// games is checked against a from-scratch recomputation of chains and
// liberties; featurizer planes are checked for one-hot structure and
// agreement with the rules; the threaded featurizer and the forest's threaded
// leaf featurization/encoding are exercised concurrently for TSAN.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <thread>
#include <vector>

#include "../engine/featurize.h"
#include "../engine/go.h"
#include "../engine/mcts.h"

using namespace ag;

static int g_fail = 0;
#define CHECK(c, ...)                                   \
  do {                                                  \
    if (!(c)) {                                         \
      std::fprintf(stderr, "CHECK failed %s:%d: %s  ", __FILE__, __LINE__, #c); \
      std::fprintf(stderr, __VA_ARGS__);                \
      std::fprintf(stderr, "\n");                       \
      if (++g_fail > 20) std::exit(1);                  \
    }                                                   \
  } while (0)

// Recompute chains and liberties by flood fill and compare with the
// incremental bookkeeping.
static void check_invariants(const GameState& s) {
  std::vector<int> comp(s.np, -1);
  for (int p = 0; p < s.np; ++p) {
    if (s.board[p] == EMPTY) {
      CHECK(s.head[p] == -1, "empty point %d has head %d", p, s.head[p]);
      continue;
    }
    if (comp[p] >= 0) continue;
    std::vector<int> st{p}, stones;
    comp[p] = p;
    Bits lib;
    lib.zero();
    while (!st.empty()) {
      int q = st.back();
      st.pop_back();
      stones.push_back(q);
      for (int i = 0; i < s.g->nnbr[q]; ++i) {
        int r = s.g->nbr[q][i];
        if (s.board[r] == EMPTY) lib.set(r);
        else if (s.board[r] == s.board[p] && comp[r] < 0) {
          comp[r] = p;
          st.push_back(r);
        }
      }
    }
    const int h = s.head[p];
    CHECK(h >= 0 && h < s.np, "bad head %d", h);
    if (h < 0 || h >= s.np) continue;
    for (int q : stones) CHECK(s.head[q] == h, "stone %d head %d != %d", q, s.head[q], h);
    CHECK(s.gsize[h] == (int)stones.size(), "group %d size %d != %d", h, s.gsize[h], (int)stones.size());
    CHECK(s.libc[h] == lib.count(), "group %d libc %d != %d", h, s.libc[h], lib.count());
    CHECK(s.libc[h] > 0, "group %d on board without liberties", h);
    for (int w = 0; w < BW; ++w) CHECK(s.libs[h].w[w] == lib.w[w], "group %d liberty word %d", h, w);
    // circular stone list covers exactly the group
    int cnt = 0, q = h;
    do {
      ++cnt;
      q = s.next[q];
    } while (q != h && cnt <= s.np);
    CHECK(cnt == (int)stones.size(), "stone list length %d != %d", cnt, (int)stones.size());
  }
  if (s.ko >= 0) CHECK(s.board[s.ko] == EMPTY, "ko point %d occupied", s.ko);
}

static void check_features(const GameState& s, const std::vector<int>& fids, int nplanes) {
  std::vector<uint8_t> out((size_t)nplanes * s.np);
  featurize(s, fids.data(), (int)fids.size(), out.data());
  const int np = s.np;
  // fids = all features in id order: offsets follow feature_planes()
  int off = 0;
  for (int f : fids) {
    const int k = feature_planes(f);
    for (int p = 0; p < np; ++p) {
      int hot = 0;
      for (int j = 0; j < k; ++j) hot += out[(size_t)(off + j) * np + p];
      if (f == F_BOARD || f == F_ONES) CHECK(hot == 1, "feature %d not one-hot at %d", f, p);
      else CHECK(hot <= 1, "feature %d multi-hot at %d", f, p);
      if (f == F_LEGAL) CHECK(hot == (s.is_legal(p) ? 1 : 0), "legal plane disagrees at %d", p);
      if (f == F_LIBERTIES) CHECK(hot == (s.board[p] != EMPTY ? 1 : 0), "liberties plane at %d", p);
    }
    off += k;
  }
  std::vector<int8_t> b(np);
  std::vector<uint8_t> ages(np), lad(np);
  int32_t meta[2];
  encode_state(s, b.data(), ages.data(), meta, lad.data());
  CHECK(meta[0] == s.ko && meta[1] == s.current_player, "encode meta");
  for (int p = 0; p < np; ++p) {
    CHECK(b[p] == s.board[p], "encode board at %d", p);
    if (ages[p] != 255) CHECK(ages[p] < 8 && s.board[p] != EMPTY, "encode age at %d", p);
    if (lad[p]) CHECK(s.is_legal(p), "ladder bit on illegal point %d", p);
  }
}

static GameState random_game(std::mt19937_64& rng, int n, int len, std::vector<GameState>* keep) {
  GameState s(n);
  std::vector<int> moves;
  for (int i = 0; i < len && !s.is_end_of_game; ++i) {
    s.legal_moves(moves, false);
    int mv = moves.empty() || rng() % 100 == 0 ? PASS : moves[rng() % moves.size()];
    bool ok = s.try_move(mv);
    CHECK(ok, "legal move %d rejected", mv);
    check_invariants(s);
    if (keep && rng() % 16 == 0) keep->push_back(s);
  }
  return s;
}

int main(int argc, char** argv) {
  const int games = argc > 1 ? std::atoi(argv[1]) : 40;
  std::mt19937_64 rng(12345);
  std::vector<int> fids;
  int nplanes = 0;
  for (int f = 0; f < F_NUM; ++f) {
    fids.push_back(f);
    nplanes += feature_planes(f);
  }
  std::vector<GameState> pool;
  const int sizes[4] = {7, 9, 13, 19};
  for (int g = 0; g < games; ++g) {
    int n = sizes[g % 4];
    random_game(rng, n, (int)(rng() % (n * n * 2)), n == 19 ? &pool : nullptr);
  }
  std::printf("rules: %d games ok\n", games);
  for (size_t i = 0; i < pool.size(); i += 3) check_features(pool[i], fids, nplanes);
  std::printf("features: %zu states ok\n", (pool.size() + 2) / 3);

  // concurrent featurization of shared const states (TSAN)
  {
    std::vector<std::thread> th;
    std::vector<std::vector<uint8_t>> outs(8, std::vector<uint8_t>((size_t)nplanes * MAXP));
    for (int t = 0; t < 8; ++t)
      th.emplace_back([&, t]() {
        for (size_t i = t; i < pool.size(); i += 2) featurize(pool[i], fids.data(), (int)fids.size(), outs[t].data());
      });
    for (auto& x : th) x.join();
  }
  // forest: gather / threaded leaf featurize + encode / apply / advance, run
  // with 1 and 4 worker threads: identical trees (workers own disjoint trees)
  {
    std::vector<int> pf;
    for (int f : {F_BOARD, F_ONES, F_TURNS_SINCE, F_LIBERTIES, F_SENSIBLENESS}) pf.push_back(f);
    std::vector<std::vector<int>> visits_by_threads;
    for (int nthreads : {1, 4}) {
      Forest forest(6, 5.0, 0.0, 60, 1000, 3, 7, pf);
      forest.set_threads(nthreads);
      for (int t = 0; t < 6; ++t) forest.set_root(t, pool[(t * 5) % pool.size()]);
      std::mt19937_64 prng(99);
      std::uniform_real_distribution<float> u(0.f, 1.f);
      for (int round = 0; round < 30; ++round) {
        int L = forest.gather(4);
        if (L == 0) continue;
        const int np = forest.leaf_state(0).np;
        std::vector<uint8_t> feat((size_t)L * forest.feature_planes() * np), masks((size_t)L * np);
        forest.leaf_features(feat.data(), 4);
        forest.leaf_masks(masks.data());
        std::vector<int8_t> b((size_t)L * np);
        std::vector<uint8_t> a((size_t)L * np), lad((size_t)L * np);
        std::vector<int32_t> m(2 * L);
        forest.leaf_encode(b.data(), a.data(), m.data(), lad.data(), 4);
        std::vector<float> pri((size_t)L * np), val(L);
        for (auto& x : pri) x = u(prng);
        for (auto& x : val) x = 2.f * u(prng) - 1.f;
        forest.apply(pri.data(), val.data(), (round & 1) ? masks.data() : nullptr);
      }
      std::vector<int> vis;
      for (int t = 0; t < 6; ++t) {
        std::vector<int> mv, vs;
        std::vector<float> q;
        forest.root_stats(t, mv, vs, q);
        vis.insert(vis.end(), vs.begin(), vs.end());
        int best = forest.best_move(t, 0.0);
        const GameState& r = forest.root_state(t);
        CHECK(best == PASS || r.is_legal(best), "best move %d illegal", best);
        forest.advance(t, best);
        check_invariants(forest.root_state(t));
      }
      visits_by_threads.push_back(vis);
      std::printf("forest (%d threads): ok (%lld evals)\n", nthreads, (long long)forest.total_evals());
    }
    CHECK(visits_by_threads[0] == visits_by_threads[1], "threaded search differs from serial search");
  }
  if (g_fail) {
    std::printf("FAILED (%d checks)\n", g_fail);
    return 1;
  }
  std::printf("ALL OK\n");
  return 0;
}
