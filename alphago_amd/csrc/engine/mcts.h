// Batched PUCT Monte-Carlo tree search over many independent trees.
//
// Replaces the serial, batch-1 MCTS of the reference (AlphaGo/mcts.py:67-171,
// ParallelMCTS stub :174-175).  Each call to gather() descends every tree with
// virtual loss until it has collected up to `leaves_per_tree` unexpanded leaves;
// the caller evaluates all leaves of all trees in ONE batched network call on the
// GPU and returns priors+values through apply(), which expands and backs up.
//
// Fixes over the reference: the root's visit count is
// maintained and u = c·P·sqrt(ΣN)/(1+N) is evaluated at selection time (Q3);
// values are backed up negamax-style from the side-to-move perspective (Q4);
// rollouts are optional (λ = 0 is first class), sample from a cheap native
// rollout policy instead of printing a warning at the limit (Q5), and run in
// parallel over trees (one random stream per tree).
#pragma once

#include <cstdint>
#include <memory>
#include <random>
#include <stdexcept>
#include <unordered_map>
#include <vector>

#include "featurize.h"
#include "go.h"
#include "workpool.h"

namespace ag {

struct Node {
  int32_t parent;
  int32_t first_child;
  int16_t nchild;
  int16_t move;  // point index, PASS = -1
  float P;
  int32_t N;
  float W;      // sum of values from the perspective of the player who moved into this node
  float v0;     // the evaluation backed up when the node was expanded (side to move at the node)
  int16_t vl;   // pending virtual-loss count
  int8_t status;  // 0 unexpanded, 1 pending evaluation, 2 expanded, 3 terminal
};
static_assert(sizeof(Node) == 32, "Node stays 32 bytes (NodeStore blocks are 2 MiB)");

// Node storage in fixed 2-MiB blocks that are never moved or freed while the
// forest lives: growth never copies a tree (a vector doubling would), node
// references stay valid across appends, and clear() keeps the blocks (and
// their faulted-in pages) for the next search.
class NodeStore {
 public:
  static constexpr int kShift = 16;  // 65536 nodes x 32 B = 2 MiB per block
  static constexpr int kBlock = 1 << kShift;
  NodeStore() = default;
  NodeStore(const NodeStore&) = delete;
  NodeStore& operator=(const NodeStore&) = delete;
  NodeStore(NodeStore&& o) noexcept : blocks_(std::move(o.blocks_)), size_(o.size_) { o.size_ = 0; }
  ~NodeStore();
  int size() const { return size_; }
  void clear() { size_ = 0; }
  Node& operator[](int i) { return blocks_[i >> kShift][i & (kBlock - 1)]; }
  const Node& operator[](int i) const { return blocks_[i >> kShift][i & (kBlock - 1)]; }
  void push_back(const Node& n) {
    if ((size_ >> kShift) >= (int)blocks_.size()) grow();
    (*this)[size_++] = n;
  }
  void swap(NodeStore& o) {
    blocks_.swap(o.blocks_);
    std::swap(size_, o.size_);
  }

 private:
  void grow();
  std::vector<Node*> blocks_;
  int size_ = 0;
};

struct Leaf {
  int tree;
  int node;
};

struct SearchTree {
  NodeStore nodes;
  NodeStore spare;  // scratch for advance()'s subtree copy (keeps its blocks)
  GameState root_state;
  int64_t sims = 0;
  // per-tree stream (rollouts, root noise, temperature sampling): trees are
  // searched by different workers, and the results do not depend on the count
  std::mt19937_64 rng;
  // ladder cache (leaf_encode): each encoded node's ladder reads, and per expanded node the first of its
  // children that was encoded (the reference of its siblings)
  std::unordered_map<int, LadderRecord> lad;
  std::unordered_map<int, int> lad_rep;
  int64_t lad_bytes = 0;  // host bytes of lad (ladder_record_bytes)
  SearchTree() : root_state(19) {}
};

// rollout move choice (reference: any rollout_fn callable, mcts.py:128-140)
enum RolloutPolicy : int {
  ROLLOUT_RANDOM = 0,     // uniform over sensible moves (legal, not an own true eye)
  ROLLOUT_HEURISTIC = 1,  // capture / atari escape at the last move, else near it (p = 1/2), else uniform
};

class Forest {
 public:
  Forest(int n_trees, double c_puct, double lmbda, int rollout_limit, int playout_depth, int virtual_loss,
         uint64_t seed, std::vector<int> feature_ids);

  int n_trees() const { return (int)trees_.size(); }
  void set_root(int t, const GameState& s);
  const GameState& root_state(int t) const { return trees_[t].root_state; }
  // Descend all (or the listed) trees; returns number of leaves queued for evaluation.
  int gather(int leaves_per_tree, const std::vector<int>* which = nullptr);
  int n_pending() const { return (int)pending_.size(); }
  // Two batches of one forest in flight (single-tree search, round 4): hold() parks the pending batch
  // -- its leaves keep their virtual losses and queued status, its leaf states keep their slot bank --
  // so gather() can queue the next batch while the parked one is evaluated; swap_held() exchanges the
  // pending and the parked batch (apply() backs up whichever is pending).
  void hold() {
    if (!held_.empty()) throw std::runtime_error("hold: a batch is already held");
    held_.swap(pending_);
    held_slot_.swap(leaf_slot_);
    held_slots_.swap(slots_);
    pending_.clear();
    leaf_slot_.clear();
  }
  void swap_held() {
    held_.swap(pending_);
    held_slot_.swap(leaf_slot_);
    held_slots_.swap(slots_);
  }
  int n_held() const { return (int)held_.size(); }
  int n_held_tree(int t) const {
    int n = 0;
    for (const Leaf& lf : held_) n += lf.tree == t;
    return n;
  }
  // held leaves of every tree in one pass over the held batch (n_held_tree per tree is O(trees x held))
  std::vector<int> held_counts() const {
    std::vector<int> n(trees_.size(), 0);
    for (const Leaf& lf : held_) ++n[lf.tree];
    return n;
  }
  // Unwind an interrupted search: the pending and the held batch lose their virtual losses and
  // queued status (their leaves become unexpanded again) and both lists are cleared, so set_root /
  // advance work afterwards.
  void discard();
  const GameState& leaf_state(int i) const { return slots_[leaf_slot_[i]]; }
  int feature_planes() const { return nplanes_; }
  // uint8 features (L, F, n, n) and sensible-move masks (L, n*n); threaded.
  void leaf_features(uint8_t* out, int threads) const;
  void leaf_masks(uint8_t* out) const;
  // compact GPU-featurizer encoding of the pending leaves (see encode_state).  With ladders and the
  // ladder cache on, a leaf's reads are checked against its grandparent's or an encoded sibling's
  // (whichever board differs in fewer points; same player to move) and only the reads whose read set
  // the difference touches run again -- bit-exact (featurize.h LadderRecord).
  void leaf_encode(int8_t* board, uint8_t* ages, int32_t* meta, uint8_t* ladder, int threads);
  void set_ladder_cache(bool on) {
    ladder_cache_ = on;
    if (!on) clear_ladder_cache();
  }
  bool ladder_cache() const { return ladder_cache_; }
  void clear_ladder_cache() {
    for (SearchTree& tr : trees_) {
      tr.lad.clear();
      tr.lad_rep.clear();
      tr.lad_bytes = 0;
    }
    lad_records_ = 0;
    lad_bytes_ = 0;
  }
  // host-memory budget of the ladder cache, forest-wide: each tree may hold budget / n_trees bytes of
  // records; a tree that would exceed its share drops its own records (they are rebuilt as the search
  // goes on) instead of the cache freezing.  advance() already drops the records outside the kept subtree.
  void set_ladder_cache_bytes(int64_t bytes) { lad_budget_bytes_ = bytes < (1 << 20) ? (1 << 20) : bytes; }
  int64_t ladder_cache_bytes() const { return lad_budget_bytes_; }
  // records held, reads taken from a reference, reads run, bytes held, tree evictions
  void ladder_cache_stats(int64_t& records, int64_t& reused, int64_t& read, int64_t& bytes, int64_t& evictions) const {
    records = lad_records_;
    reused = lad_reused_;
    read = lad_read_;
    bytes = lad_bytes_;
    evictions = lad_evictions_;
  }
  // priors (L, n*n) float32 (any non-negative scores; renormalised over sensible moves), values (L,);
  // mask (L, n*n) optional sensible-move mask (e.g. from the GPU featurizer) — skips the legality/eye scan
  void apply(const float* priors, const float* values, const uint8_t* mask = nullptr);
  // worker threads for gather/apply (trees are independent; results are identical for any count)
  void set_threads(int n) {
    threads_ = n < 1 ? 1 : n;
    if (!pool_ || pool_->workers() != threads_ - 1) pool_.reset(threads_ > 1 ? new WorkPool(threads_ - 1) : nullptr);
  }
  // a pool for callers that pass a thread count without set_threads
  void ensure_pool(int threads) const {
    if (!pool_ && threads > 1) pool_.reset(new WorkPool(threads - 1));
  }
  // run fn(0..nparts-1) on the persistent workers (serially without a pool)
  void run_parts(int nparts, const std::function<void(int)>& fn) const {
    if (pool_) pool_->run(nparts, fn);
    else
      for (int p = 0; p < nparts; ++p) fn(p);
  }
  void add_root_noise(int t, double alpha, double eps);
  void set_rollout_policy(int kind) { rollout_kind_ = kind; }
  int rollout_policy() const { return rollout_kind_; }
  // Root statistics
  void root_stats(int t, std::vector<int>& moves, std::vector<int>& visits, std::vector<float>& q) const;
  int best_move(int t, double temperature);
  void advance(int t, int move);
  int64_t sims(int t) const { return trees_[t].sims; }
  // deepest expanded node below the root (root = 0); bounded by playout_depth
  int max_expanded_depth(int t) const;
  int64_t total_evals() const { return total_evals_; }

 private:
  int select_child(const SearchTree& tr, int u) const;
  double rollout(GameState& s, std::mt19937_64& rng) const;
  int rollout_move(const GameState& s, std::mt19937_64& rng, std::vector<int>& cand) const;
  void backup(SearchTree& tr, int leaf, double v_leaf_to_move, bool remove_vl);

  std::vector<SearchTree> trees_;
  std::vector<Leaf> pending_;
  std::vector<Leaf> held_;                // hold() / swap_held(): the parked batch,
  std::vector<int> held_slot_;            // its slot ids
  std::vector<GameState> held_slots_;     // and its slot bank
  // Leaf states live in a persistent slot pool (a GameState is ~20 KB of
  // inline arrays): each gather copies the root into a reused slot and plays
  // the path there, so a leaf costs one copy and no allocation.
  std::vector<GameState> slots_;
  std::vector<int> leaf_slot_;
  std::vector<std::vector<int>> leaf_paths_;
  double c_puct_, lmbda_;
  int rollout_limit_, playout_depth_, vloss_;
  std::mt19937_64 rng_;  // seeds the per-tree streams
  int rollout_kind_ = ROLLOUT_RANDOM;
  std::vector<int> fids_;
  int nplanes_ = 0;
  int64_t total_evals_ = 0;
  bool ladder_cache_ = true;
  int64_t lad_records_ = 0, lad_reused_ = 0, lad_read_ = 0, lad_bytes_ = 0, lad_evictions_ = 0;
  int64_t lad_budget_bytes_ = int64_t(256) << 20;  // forest-wide default (set_ladder_cache_bytes)
  std::vector<LadderRecord> lad_fresh_;
  int threads_ = 1;
  mutable std::unique_ptr<WorkPool> pool_;  // threads_ - 1 persistent workers (set_threads)
  void gather_trees(const int* trees, int ntrees, int lpt, std::vector<Leaf>& pend, std::vector<int>& slot_ids,
                    int slot_base);
  void apply_range(int i0, int i1, const float* priors, const float* values, const uint8_t* mask);
};



}  // namespace ag
