#include "mcts.h"


#include <sys/mman.h>

#include <algorithm>
#include <cmath>
#include <new>
#include <thread>

#include "featurize.h"


namespace ag {

static_assert(sizeof(Node) == 32, "NodeStore block size assumes 32-byte nodes");

void NodeStore::grow() {
  const size_t bytes = sizeof(Node) * (size_t)kBlock;
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (p == MAP_FAILED) throw std::bad_alloc();
  // no populate: pages fault on first touch inside the apply() workers, in parallel
  // (MAP_POPULATE / MADV_POPULATE_WRITE of whole blocks measured 3x slower with 8 workers)
  blocks_.push_back(static_cast<Node*>(p));
}

NodeStore::~NodeStore() {
  for (Node* b : blocks_) munmap(b, sizeof(Node) * (size_t)kBlock);
}

static Node make_node(int parent, int move, float P) {
  Node n;
  n.parent = parent;
  n.first_child = -1;
  n.nchild = 0;
  n.move = (int16_t)move;
  n.P = P;
  n.N = 0;
  n.W = 0.f;
  n.vl = 0;
  n.v0 = 0.f;
  n.status = 0;
  return n;
}

Forest::Forest(int n_trees, double c_puct, double lmbda, int rollout_limit, int playout_depth, int virtual_loss,
               uint64_t seed, std::vector<int> feature_ids)
    : trees_(n_trees),
      c_puct_(c_puct),
      lmbda_(lmbda),
      rollout_limit_(rollout_limit),
      playout_depth_(playout_depth),
      vloss_(virtual_loss),
      rng_(seed),
      fids_(std::move(feature_ids)) {
  for (int f : fids_) nplanes_ += ag::feature_planes(f);
  for (auto& t : trees_) {
    t.nodes.clear();
    t.nodes.push_back(make_node(-1, PASS, 1.f));
    t.rng.seed(rng_());
  }
}

void Forest::set_root(int t, const GameState& s) {
  if (!pending_.empty() || !held_.empty()) throw std::runtime_error("set_root with pending evaluations");
  auto& tr = trees_.at(t);
  tr.root_state = s;
  tr.nodes.clear();
  tr.nodes.push_back(make_node(-1, PASS, 1.f));
  tr.sims = 0;
  lad_records_ -= (int64_t)tr.lad.size();
  lad_bytes_ -= tr.lad_bytes;
  tr.lad.clear();
  tr.lad_rep.clear();
  tr.lad_bytes = 0;
}

int Forest::select_child(const SearchTree& tr, int u) const {
  const Node& nu = tr.nodes[u];
  double nparent = (double)nu.N + (double)vloss_ * nu.vl;
  double sq = std::sqrt(std::max(nparent, 1.0));
  int best = -1;
  double bestv = -1e300;
  for (int i = 0; i < nu.nchild; ++i) {
    const Node& c = tr.nodes[nu.first_child + i];
    double n = (double)c.N + (double)vloss_ * c.vl;
    double q = n > 0 ? ((double)c.W - (double)vloss_ * c.vl) / n : 0.0;
    double v = q + c_puct_ * c.P * sq / (1.0 + n);
    if (v > bestv) {
      bestv = v;
      best = nu.first_child + i;
    }
  }
  return best;
}

int Forest::max_expanded_depth(int t) const {
  const SearchTree& tr = trees_.at(t);
  int best = -1;
  const int n = (int)tr.nodes.size();
  for (int i = 0; i < n; ++i) {
    if (tr.nodes[i].status != 2) continue;
    int d = 0;
    for (int x = tr.nodes[i].parent; x >= 0; x = tr.nodes[x].parent) ++d;
    best = std::max(best, d);
  }
  return best;
}

void Forest::backup(SearchTree& tr, int leaf, double v_leaf_to_move, bool remove_vl) {
  double val = -v_leaf_to_move;
  int x = leaf;
  while (x >= 0) {
    Node& nd = tr.nodes[x];
    nd.N += 1;
    nd.W += (float)val;
    if (remove_vl) nd.vl -= 1;
    val = -val;
    x = nd.parent;
  }
  tr.sims += 1;
}

void Forest::gather_trees(const int* trees, int ntrees, int leaves_per_tree, std::vector<Leaf>& pend,
                          std::vector<int>& slot_ids, int slot_base) {
  int next = slot_base;  // this worker owns slots [slot_base, slot_base + ntrees * leaves_per_tree)
  for (int ti = 0; ti < ntrees; ++ti) {
    const int t = trees[ti];
    SearchTree& tr = trees_.at(t);
    for (int k = 0; k < leaves_per_tree; ++k) {
      GameState& st = slots_[next];
      st = tr.root_state;
      int u = 0;
      tr.nodes[0].vl += 1;
      int depth = 0;
      bool stop_tree = false;
      while (true) {
        Node& nd = tr.nodes[u];
        if (nd.status == 3) {
          int w = st.get_winner();
          backup(tr, u, (double)(w * st.current_player), true);
          break;
        }
        if (nd.status == 1) {  // collision with a leaf already queued in this batch
          for (int x = u; x >= 0; x = tr.nodes[x].parent) tr.nodes[x].vl -= 1;
          stop_tree = true;
          break;
        }
        if (depth >= playout_depth_ && nd.status == 2) {
          // depth-limited playout (reference mcts.py _DFS(nDepth=L)): the tree does not grow
          // below L; the node at the cap is scored as a leaf again.  Its stored first
          // evaluation is backed up -- what re-evaluating the same position with the same
          // network returns (lambda = 0); with rollouts (lambda > 0) the first mix is reused.
          backup(tr, u, (double)nd.v0, true);
          break;
        }
        if (nd.status == 0 || depth >= playout_depth_) {
          if (st.is_end_of_game) {
            nd.status = 3;
            int w = st.get_winner();
            backup(tr, u, (double)(w * st.current_player), true);
            break;
          }
          if (nd.status == 0) {
            nd.status = 1;
            pend.push_back({t, u});
            slot_ids.push_back(next++);
            break;
          }
        }
        int c = select_child(tr, u);
        if (c < 0) {  // defensive: apply_range gives every expanded node >= 1 child (PASS when nothing is sensible)
          for (int x = u; x >= 0; x = tr.nodes[x].parent) tr.nodes[x].vl -= 1;
          stop_tree = true;
          break;
        }
        tr.nodes[c].vl += 1;
        st.try_move(tr.nodes[c].move, 0);
        u = c;
        ++depth;
      }
      if (stop_tree) break;
    }
  }
}

void Forest::discard() {
  for (const std::vector<Leaf>* batch : {&pending_, &held_}) {
    for (const Leaf& lf : *batch) {
      SearchTree& tr = trees_.at(lf.tree);
      if (tr.nodes[lf.node].status == 1) tr.nodes[lf.node].status = 0;
      for (int x = lf.node; x >= 0; x = tr.nodes[x].parent) tr.nodes[x].vl -= 1;
    }
  }
  pending_.clear();
  held_.clear();
  leaf_slot_.clear();
  held_slot_.clear();
}

int Forest::gather(int leaves_per_tree, const std::vector<int>* which) {
  if (!pending_.empty()) throw std::runtime_error("gather called with pending evaluations; call apply first");
  leaf_slot_.clear();
  std::vector<int> all;
  if (!which) {
    all.resize(trees_.size());
    for (size_t i = 0; i < trees_.size(); ++i) all[i] = (int)i;
    which = &all;
  }
  const int n = (int)which->size();
  const size_t need = (size_t)n * leaves_per_tree;
  if (slots_.size() < need) slots_.resize(need, GameState(trees_.empty() ? 19 : trees_[0].root_state.n));
  const int T = std::max(1, std::min(threads_, n));
  if (T == 1) {
    gather_trees(which->data(), n, leaves_per_tree, pending_, leaf_slot_, 0);
  } else {
    // contiguous blocks of trees per worker (each with its own slot range); concatenated in tree order
    std::vector<std::vector<Leaf>> pend(T);
    std::vector<std::vector<int>> ids(T);
    run_parts(T, [&](int w) {
      const int lo = (int)((int64_t)n * w / T), hi = (int)((int64_t)n * (w + 1) / T);
      pend[w].reserve((size_t)(hi - lo) * leaves_per_tree);
      ids[w].reserve((size_t)(hi - lo) * leaves_per_tree);
      gather_trees(which->data() + lo, hi - lo, leaves_per_tree, pend[w], ids[w], lo * leaves_per_tree);
    });
    for (int w = 0; w < T; ++w) {
      pending_.insert(pending_.end(), pend[w].begin(), pend[w].end());
      leaf_slot_.insert(leaf_slot_.end(), ids[w].begin(), ids[w].end());
    }
  }
  total_evals_ += (int64_t)pending_.size();
  return (int)pending_.size();
}

void Forest::leaf_features(uint8_t* out, int threads) const {
  int L = (int)pending_.size();
  if (L == 0) return;
  size_t stride = (size_t)nplanes_ * leaf_state(0).np;
  ensure_pool(threads);  // the forest's persistent pool (set_threads) runs the parts
  constexpr int kChunk = 8;
  run_parts((L + kChunk - 1) / kChunk, [&](int c) {
    for (int i = c * kChunk; i < std::min(L, (c + 1) * kChunk); ++i)
      featurize(leaf_state(i), fids_.data(), (int)fids_.size(), out + i * stride);
  });
}

// host bytes one cached record holds: the record, its entries (each with its read set) and the map node
static inline int64_t ladder_record_bytes(const LadderRecord& r) {
  return (int64_t)sizeof(LadderRecord) + (int64_t)r.e.capacity() * (int64_t)sizeof(LadderEntry) + 64;
}

void Forest::leaf_encode(int8_t* board, uint8_t* ages, int32_t* meta, uint8_t* ladder, int threads) {
  int L = (int)pending_.size();
  if (L == 0) return;
  const int np = leaf_state(0).np;
  ensure_pool(threads);  // the forest's persistent pool (set_threads) runs the parts
  // ladder cache: each leaf's candidate references (grandparent, encoded sibling), looked up before the
  // parallel encode (which only reads the maps) and the new records committed after it
  const bool cache = ladder && ladder_cache_;
  std::vector<const LadderRecord*> ref_gp, ref_sib;
  if (cache) {
    if ((int)lad_fresh_.size() < L) lad_fresh_.resize(L);
    ref_gp.assign(L, nullptr);
    ref_sib.assign(L, nullptr);
    for (int i = 0; i < L; ++i) {
      const SearchTree& tr = trees_[pending_[i].tree];
      const int pu = tr.nodes[pending_[i].node].parent;
      if (pu < 0) continue;
      const int gp = tr.nodes[pu].parent;
      if (gp >= 0) {
        auto it = tr.lad.find(gp);
        if (it != tr.lad.end()) ref_gp[i] = &it->second;
      }
      auto rs = tr.lad_rep.find(pu);
      if (rs != tr.lad_rep.end()) {
        auto it = tr.lad.find(rs->second);
        if (it != tr.lad.end()) ref_sib[i] = &it->second;
      }
    }
  }
  auto pick_ref = [&](int i) -> const LadderRecord* {
    const LadderRecord* a = ref_gp[i];
    const LadderRecord* b = ref_sib[i];
    if (!a || !b) return a ? a : b;
    // the reference whose board differs from the leaf's in fewer points
    const GameState& s = leaf_state(i);
    auto ndiff = [&](const LadderRecord* r) {
      int d = 0;
      for (int p = 0; p < s.np; ++p) {
        const int c = lb::btest(r->black, p) ? BLACK : lb::btest(r->white, p) ? WHITE : EMPTY;
        d += c != s.board[p];
      }
      return d;
    };
    return ndiff(b) < ndiff(a) ? b : a;
  };
  // small chunks claimed dynamically: ladder reads make a few boards far costlier than the rest.  A
  // single tree's leaf batch (tens of boards) goes one board per part so that every pool thread gets
  // work: with 4-board parts a 32-leaf batch kept 8 of 16 threads busy, and on positions with long
  // edge ladders the encode was 0.6 ms of each 1 ms search round (scripts/r4/genmove_diag.py)
  const int kChunk = L <= 256 ? 1 : 4;
  auto work = [&](int c) {
    for (int i = c * kChunk; i < std::min(L, (c + 1) * kChunk); ++i)
      encode_state(leaf_state(i), board + (size_t)i * np, ages + (size_t)i * np, meta + 2 * i,
                   ladder ? ladder + (size_t)i * np : nullptr, cache ? pick_ref(i) : nullptr,
                   cache ? &lad_fresh_[i] : nullptr);
  };
  const int nchunks = (L + kChunk - 1) / kChunk;
  if (!ladder) {  // without ladders this is a memcpy-class walk
    for (int c = 0; c < nchunks; ++c) work(c);
    return;
  }
  run_parts(nchunks, work);
  if (!cache) return;
  for (int i = 0; i < L; ++i) {
    SearchTree& tr = trees_[pending_[i].tree];
    const int u = pending_[i].node;
    lad_reused_ += lad_fresh_[i].reused;
    lad_read_ += lad_fresh_[i].read;
    const int64_t share = std::max<int64_t>(lad_budget_bytes_ / (int64_t)trees_.size(), 1 << 16);
    const int64_t rb = ladder_record_bytes(lad_fresh_[i]);
    if (tr.lad_bytes + rb > share && !tr.lad.empty()) {  // this tree's share is full: drop its records
      lad_records_ -= (int64_t)tr.lad.size();
      lad_bytes_ -= tr.lad_bytes;
      tr.lad.clear();
      tr.lad_rep.clear();
      tr.lad_bytes = 0;
      ++lad_evictions_;
    }
    auto ins = tr.lad.emplace(u, LadderRecord());
    if (ins.second) {
      ++lad_records_;
    } else {
      const int64_t old = ladder_record_bytes(ins.first->second);
      tr.lad_bytes -= old;
      lad_bytes_ -= old;
    }
    std::swap(ins.first->second, lad_fresh_[i]);  // (the fresh slot keeps a vector for the next batch)
    const int64_t nb = ladder_record_bytes(ins.first->second);
    tr.lad_bytes += nb;
    lad_bytes_ += nb;
    const int pu = tr.nodes[u].parent;
    if (pu >= 0) tr.lad_rep.emplace(pu, u);
  }
}

void Forest::leaf_masks(uint8_t* out) const {
  for (size_t i = 0; i < pending_.size(); ++i) {
    const GameState& s = leaf_state(i);
    for (int p = 0; p < s.np; ++p) out[i * s.np + p] = s.is_legal(p) && !s.is_eye(p, s.current_player);
  }
}

static inline bool sensible(const GameState& s, int p) {
  return p >= 0 && s.board[p] == EMPTY && s.is_legal(p) && !s.is_eye(p, s.current_player);
}

int Forest::rollout_move(const GameState& s, std::mt19937_64& rng, std::vector<int>& cand) const {
  const int me = s.current_player;
  const int last = s.history.empty() ? PASS : s.history.back();
  if (rollout_kind_ == ROLLOUT_HEURISTIC && last != PASS) {
    // 1) capture the group just played (or an enemy neighbour of it) when it is in atari;
    // 2) save an own group next to the last move that it put in atari, if the escape
    //    point gives it more than one liberty
    const Geometry& g = *s.g;
    for (int k = 0; k < g.nnbr[last] + 1; ++k) {
      const int q = k == 0 ? last : g.nbr[last][k - 1];
      if (s.board[q] == -me && s.libc[s.head[q]] == 1) {
        const int lib = s.libs[s.head[q]].first();
        if (sensible(s, lib)) return lib;
      }
    }
    for (int k = 0; k < g.nnbr[last]; ++k) {
      const int q = g.nbr[last][k];
      if (s.board[q] == me && s.libc[s.head[q]] == 1) {
        const int lib = s.libs[s.head[q]].first();
        if (!sensible(s, lib)) continue;
        int gain = 0;  // liberties of the escape point beyond the group's old one
        for (int j = 0; j < g.nnbr[lib]; ++j) gain += s.board[g.nbr[lib][j]] == EMPTY;
        if (gain >= 2) return lib;
      }
    }
    // 3) half of the remaining moves answer locally (8-neighbourhood of the last move)
    if (rng() & 1ull) {
      int loc[8], nl = 0;
      for (int k = 0; k < g.nnbr[last]; ++k)
        if (sensible(s, g.nbr[last][k])) loc[nl++] = g.nbr[last][k];
      for (int k = 0; k < g.ndiag[last]; ++k)
        if (sensible(s, g.diag[last][k])) loc[nl++] = g.diag[last][k];
      if (nl) return loc[rng() % (uint64_t)nl];
    }
  }
  for (int tries = 0; tries < 24; ++tries) {
    const int p = (int)(rng() % (uint64_t)s.np);
    if (sensible(s, p)) return p;
  }
  cand.clear();
  for (int p = 0; p < s.np; ++p)
    if (sensible(s, p)) cand.push_back(p);
  return cand.empty() ? PASS : cand[rng() % cand.size()];
}

double Forest::rollout(GameState& s, std::mt19937_64& rng) const {
  const int p0 = s.current_player;
  std::vector<int> cand;
  for (int it = 0; it < rollout_limit_ && !s.is_end_of_game; ++it) s.try_move(rollout_move(s, rng, cand), 0);
  return (double)(s.get_winner() * p0);
}

void Forest::apply_range(int i0, int i1, const float* priors, const float* values, const uint8_t* mask) {
  std::vector<int> moves;
  std::vector<float> ps;
  for (int i = i0; i < i1; ++i) {
    SearchTree& tr = trees_[pending_[i].tree];
    const int u = pending_[i].node;
    const GameState& st = leaf_state(i);
    const float* pr = priors + (size_t)i * st.np;
    const uint8_t* mk = mask ? mask + (size_t)i * st.np : nullptr;
    moves.clear();
    ps.clear();
    double sum = 0;
    for (int p = 0; p < st.np; ++p)
      if (mk ? (mk[p] != 0) : (st.is_legal(p) && !st.is_eye(p, st.current_player))) {
        moves.push_back(p);
        float v = std::max(pr[p], 0.f);
        ps.push_back(v);
        sum += v;
      }
    if (moves.empty()) {
      moves.push_back(PASS);
      ps.push_back(1.f);
      sum = 1.0;
    } else if (sum <= 0) {
      for (auto& v : ps) v = 1.f;
      sum = (double)ps.size();
    }
    int first = tr.nodes.size();
    for (size_t j = 0; j < moves.size(); ++j) tr.nodes.push_back(make_node(u, moves[j], (float)(ps[j] / sum)));
    Node& nd = tr.nodes[u];
    nd.first_child = first;
    nd.nchild = (int16_t)moves.size();
    nd.status = 2;
    double v = values ? (double)values[i] : 0.0;
    if (lmbda_ > 0) {
      GameState s2 = st;
      double z = rollout(s2, tr.rng);
      v = (1.0 - lmbda_) * v + lmbda_ * z;
    }
    nd.v0 = (float)v;
    backup(tr, u, v, true);
  }
}

void Forest::apply(const float* priors, const float* values, const uint8_t* mask) {
  const int L = (int)pending_.size();
  // rollouts draw from their tree's own stream, so they run on every worker (results are
  // independent of the worker count); without rollouts small batches stay on one thread
  const int T = std::max(1, std::min(threads_, lmbda_ > 0 ? L : L / 64));
  if (T == 1) {
    apply_range(0, L, priors, values, mask);
  } else {
    // split at tree boundaries (pending_ is grouped by tree): no two workers touch one tree
    std::vector<int> cut(T + 1, L);
    cut[0] = 0;
    for (int w = 1; w < T; ++w) {
      int c = (int)((int64_t)L * w / T);
      while (c < L && c > 0 && pending_[c].tree == pending_[c - 1].tree) ++c;
      cut[w] = std::max(c, cut[w - 1]);
    }
    run_parts(T, [&](int w) { apply_range(cut[w], cut[w + 1], priors, values, mask); });
  }
  pending_.clear();
  leaf_slot_.clear();
}

void Forest::add_root_noise(int t, double alpha, double eps) {
  SearchTree& tr = trees_.at(t);
  Node& r = tr.nodes[0];
  if (r.status != 2 || r.nchild == 0) return;
  std::gamma_distribution<double> gam(alpha, 1.0);
  std::vector<double> d(r.nchild);
  double s = 0;
  for (auto& x : d) {
    x = gam(tr.rng);
    s += x;
  }
  for (int i = 0; i < r.nchild; ++i) {
    Node& c = tr.nodes[r.first_child + i];
    c.P = (float)((1 - eps) * c.P + eps * (s > 0 ? d[i] / s : 1.0 / r.nchild));
  }
}

void Forest::root_stats(int t, std::vector<int>& moves, std::vector<int>& visits, std::vector<float>& q) const {
  const SearchTree& tr = trees_.at(t);
  const Node& r = tr.nodes[0];
  moves.clear();
  visits.clear();
  q.clear();
  for (int i = 0; i < r.nchild; ++i) {
    const Node& c = tr.nodes[r.first_child + i];
    moves.push_back(c.move);
    visits.push_back(c.N);
    q.push_back(c.N > 0 ? c.W / c.N : 0.f);
  }
}

int Forest::best_move(int t, double temperature) {
  const SearchTree& tr = trees_.at(t);
  const Node& r = tr.nodes[0];
  if (r.nchild == 0) return PASS;
  if (temperature <= 0) {
    int best = r.first_child;
    for (int i = 1; i < r.nchild; ++i)
      if (tr.nodes[r.first_child + i].N > tr.nodes[best].N) best = r.first_child + i;
    return tr.nodes[best].move;
  }
  std::vector<double> w(r.nchild);
  double s = 0;
  for (int i = 0; i < r.nchild; ++i) {
    w[i] = std::pow((double)tr.nodes[r.first_child + i].N, 1.0 / temperature);
    s += w[i];
  }
  if (s <= 0) return tr.nodes[r.first_child].move;
  double x = std::uniform_real_distribution<double>(0, s)(trees_[t].rng);
  for (int i = 0; i < r.nchild; ++i) {
    x -= w[i];
    if (x <= 0) return tr.nodes[r.first_child + i].move;
  }
  return tr.nodes[r.first_child + r.nchild - 1].move;
}

void Forest::advance(int t, int move) {
  if (!pending_.empty() || !held_.empty()) throw std::runtime_error("advance with pending evaluations");
  SearchTree& tr = trees_.at(t);
  int found = -1;
  const Node& r = tr.nodes[0];
  for (int i = 0; i < r.nchild; ++i)
    if (tr.nodes[r.first_child + i].move == move) found = r.first_child + i;
  tr.root_state.do_move(move, 0);
  if (found < 0 || tr.nodes[found].status == 1) {
    tr.nodes.clear();
    tr.nodes.push_back(make_node(-1, PASS, 1.f));
    lad_records_ -= (int64_t)tr.lad.size();
    lad_bytes_ -= tr.lad_bytes;
    tr.lad.clear();
    tr.lad_rep.clear();
    tr.lad_bytes = 0;
    return;
  }
  // BFS copy of the reused subtree (children stay contiguous)
  NodeStore& nn = tr.spare;
  nn.clear();
  Node root = tr.nodes[found];
  root.parent = -1;
  nn.push_back(root);
  std::vector<int> old_of;  // old index of each new node
  old_of.push_back(found);
  for (int k = 0; k < nn.size(); ++k) {
    int o = old_of[k];
    const Node& on = tr.nodes[o];
    if (on.nchild > 0 && on.first_child >= 0) {
      int first = nn.size();
      for (int i = 0; i < on.nchild; ++i) {
        Node c = tr.nodes[on.first_child + i];
        c.parent = k;
        nn.push_back(c);
        old_of.push_back(on.first_child + i);
      }
      nn[k].first_child = first;
    }
  }
  tr.nodes.swap(nn);
  // the ladder cache follows the kept subtree's renumbering; the rest is dropped
  if (!tr.lad.empty()) {
    std::unordered_map<int, LadderRecord> lad;
    std::unordered_map<int, int> rep;
    std::vector<int> new_of;  // old index -> new (-1: dropped)
    for (int k = 0; k < (int)old_of.size(); ++k) {
      if ((int)new_of.size() <= old_of[k]) new_of.resize(old_of[k] + 1, -1);
      new_of[old_of[k]] = k;
    }
    auto nw = [&](int o) { return o >= 0 && o < (int)new_of.size() ? new_of[o] : -1; };
    int64_t kept = 0;
    for (auto& kv : tr.lad) {
      const int k = nw(kv.first);
      if (k >= 0) {
        kept += ladder_record_bytes(kv.second);
        lad.emplace(k, std::move(kv.second));
      }
    }
    lad_bytes_ += kept - tr.lad_bytes;
    tr.lad_bytes = kept;
    for (auto& kv : tr.lad_rep) {
      const int a = nw(kv.first), b = nw(kv.second);
      if (a >= 0 && b >= 0) rep.emplace(a, b);
    }
    lad_records_ += (int64_t)lad.size() - (int64_t)tr.lad.size();
    tr.lad.swap(lad);
    tr.lad_rep.swap(rep);
  }
}

// ------------------------------------------------------------------ bindings

}  // namespace ag
