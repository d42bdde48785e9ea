#include "featurize.h"

#include <atomic>
#include <cstring>
#include <utility>
#include <vector>

#include "ladder_bb.h"

namespace ag {

static const char* kNames[F_NUM] = {"board", "ones", "turns_since", "liberties", "capture_size",
                                     "self_atari_size", "liberties_after", "ladder_capture",
                                     "ladder_escape", "sensibleness", "zeros", "color", "legal",
                                     "self_atari_size_exact", "liberties_after_exact"};
static const int kPlanes[F_NUM] = {3, 1, 8, 8, 8, 8, 8, 1, 1, 1, 1, 1, 1, 8, 8};

int feature_planes(int fid) { return (fid >= 0 && fid < F_NUM) ? kPlanes[fid] : 0; }
const char* feature_name(int fid) { return (fid >= 0 && fid < F_NUM) ? kNames[fid] : ""; }
int feature_id(const std::string& name) {
  for (int i = 0; i < F_NUM; ++i)
    if (name == kNames[i]) return i;
  return -1;
}

// ---------------------------------------------------------------- ladders
static constexpr int kLadderDepth = 96;  // plies; a corner-to-corner ladder is < 80

// Node budget per capture / escape test (lb::kLadderVisits, ladder_bb.h: the
// same rule in the bitboard and GPU readers): each prey_loses / hunter_wins
// call is one visit; past the budget a node gives up like one past
// kLadderDepth.  Runtime-settable for tests (set_ladder_budget).
static std::atomic<int> g_ladder_budget{lb::kLadderVisits};
static thread_local int t_ladder_visits = 0;

void set_ladder_budget(int visits) { g_ladder_budget.store(visits > 0 ? visits : lb::kLadderVisits); }
int ladder_budget() { return g_ladder_budget.load(std::memory_order_relaxed); }

static bool hunter_wins(const GameState& s, int prey, int depth);

// Per-thread scratch states, one per ladder ply: copy-assigning into a reused
// slot keeps the history vector's capacity, so reading a ladder allocates
// nothing (a fresh GameState copy per ply was a malloc + free each).
static GameState& ladder_slot(int depth) {
  thread_local std::vector<GameState> slots(kLadderDepth + 3, GameState(19));
  return slots[depth];
}

// prey to move, prey group in atari.  True if every prey reply loses.
static bool prey_loses(const GameState& s, int prey, int depth) {
  if (++t_ladder_visits > ladder_budget()) return false;
  if (depth > kLadderDepth) return false;
  const int pc = s.board[prey];
  int16_t cand[8];
  int nc = 0;
  int h = s.head[prey];
  cand[nc++] = (int16_t)s.libs[h].first();
  // captures of adjacent hunter groups in atari, in the order of each group's
  // lowest stone index next to the prey chain (the bitboard reader's order,
  // ladder_bb.h: the node budget then cuts both searches at the same node)
  int gkey[64], ghead[64], ng = 0;
  int st = prey;
  do {
    for (int i = 0; i < s.g->nnbr[st]; ++i) {
      int q = s.g->nbr[st][i];
      if (s.board[q] == -pc && s.libc[s.head[q]] == 1) {
        const int hq = s.head[q];
        int j = 0;
        while (j < ng && ghead[j] != hq) ++j;
        if (j < ng) gkey[j] = q < gkey[j] ? q : gkey[j];
        else if (ng < 64) { ghead[ng] = hq; gkey[ng] = q; ++ng; }
      }
    }
    st = s.next[st];
  } while (st != prey);
  for (int a = 1; a < ng; ++a)  // insertion sort by key (few groups)
    for (int b = a; b > 0 && gkey[b] < gkey[b - 1]; --b) {
      std::swap(gkey[b], gkey[b - 1]);
      std::swap(ghead[b], ghead[b - 1]);
    }
  for (int j = 0; j < ng; ++j) {
    const int l = s.libs[ghead[j]].first();
    bool dup = false;
    for (int k = 0; k < nc; ++k) dup |= (cand[k] == l);
    if (!dup && nc < 8) cand[nc++] = (int16_t)l;
  }
  for (int k = 0; k < nc; ++k) {
    int mv = cand[k];
    if (mv < 0 || !s.is_legal_for(mv, pc)) continue;
    GameState& s2 = ladder_slot(depth + 1);
    s2 = s;
    s2.try_move(mv, pc);
    if (s2.board[prey] != pc) continue;
    int lc = s2.libc[s2.head[prey]];
    if (lc >= 3) return false;
    if (lc == 2 && !hunter_wins(s2, prey, depth + 1)) return false;
  }
  return true;
}

// hunter to move against the prey group.
static bool hunter_wins(const GameState& s, int prey, int depth) {
  if (++t_ladder_visits > ladder_budget()) return false;
  if (depth > kLadderDepth) return false;
  const int pc = s.board[prey];
  int h = s.head[prey];
  int lc = s.libc[h];
  if (lc == 1) return true;
  if (lc >= 3) return false;
  Bits b = s.libs[h];
  for (int k = 0; k < 2; ++k) {
    int l = b.first();
    if (l < 0) break;
    b.clear(l);
    if (!s.is_legal_for(l, -pc)) continue;
    GameState& s2 = ladder_slot(depth + 1);
    s2 = s;
    s2.try_move(l, -pc);
    if (s2.board[prey] != pc) return true;  // captured outright
    if (s2.libc[s2.head[prey]] == 1 && prey_loses(s2, prey, depth + 1)) return true;
  }
  return false;
}

bool ladder_capture_at(const GameState& s, int m) {
  if (!s.is_legal(m)) return false;
  t_ladder_visits = 0;
  const int me = s.current_player;
  for (int i = 0; i < s.g->nnbr[m]; ++i) {
    int q = s.g->nbr[m][i];
    if (s.board[q] != -me || s.libc[s.head[q]] != 2) continue;
    GameState& s2 = ladder_slot(0);
    s2 = s;
    s2.try_move(m, me);
    if (s2.board[q] != -me) return true;  // captured
    if (s2.libc[s2.head[q]] == 1 && prey_loses(s2, q, 0)) return true;
  }
  return false;
}

bool ladder_escape_at(const GameState& s, int m) {
  if (!s.is_legal(m)) return false;
  t_ladder_visits = 0;
  const int me = s.current_player;
  for (int i = 0; i < s.g->nnbr[m]; ++i) {
    int q = s.g->nbr[m][i];
    if (s.board[q] != me || s.libc[s.head[q]] != 1) continue;
    GameState& s2 = ladder_slot(0);
    s2 = s;
    s2.try_move(m, me);
    if (s2.board[q] != me) continue;
    int lc = s2.libc[s2.head[q]];
    if (lc >= 3) return true;
    if (lc == 2 && !hunter_wins(s2, q, 0)) return true;
  }
  return false;
}

// ---------------------------------------------------------------- GPU encoding
void encode_state(const GameState& s, int8_t* board, uint8_t* ages, int32_t* meta, uint8_t* ladder,
                  const LadderRecord* ref, LadderRecord* rec) {
  const int np = s.np;
  for (int p = 0; p < np; ++p) board[p] = (int8_t)s.board[p];
  std::memset(ages, 255, np);
  int depth = 0;
  for (int k = (int)s.history.size() - 1; k >= 0; --k) {  // same walk as F_TURNS_SINCE
    int mv = s.history[k];
    if (mv != PASS && s.board[mv] != EMPTY && ages[mv] == 255) ages[mv] = (uint8_t)depth;
    if (depth < 7) ++depth;
  }
  meta[0] = s.ko;
  meta[1] = s.current_player;
  if (ladder) {
    // Only liberties of an opponent group in (pre-)atari with 2 liberties
    // (capture) or of an own group in atari (escape) can be non-zero: collect
    // them from the group roots' liberty sets instead of testing every point.
    std::memset(ladder, 0, np);
    const int me = s.current_player;
    Bits cand;
    cand.zero();
    for (int p = 0; p < np; ++p) {
      if (s.board[p] == EMPTY || s.head[p] != p) continue;
      if ((s.board[p] == -me && s.libc[p] == 2) || (s.board[p] == me && s.libc[p] == 1)) cand.orr(s.libs[p]);
    }
    // the searches run on the bitboard reader (ladder_bb.h: 100-byte states,
    // the prey chain tracked incrementally) -- bit-identical to
    // ladder_capture_at / ladder_escape_at, without a 20 KB GameState copy per
    // ply (tests/test_gpu_features.py compares the two at several budgets)
    static thread_local lb::Geo geo[20];
    static thread_local bool geo_ok[20] = {};
    if (!geo_ok[s.n]) {
      lb::make_geo(geo[s.n], s.n);
      geo_ok[s.n] = true;
    }
    const lb::Geo& g = geo[s.n];
    static thread_local std::vector<lb::Frame> stack(lb::kMaxFrames);
    lb::LState ls;
    lb::bzero(ls.black);
    lb::bzero(ls.white);
    for (int p = 0; p < np; ++p) {
      if (s.board[p] > 0) lb::bset(ls.black, p);
      else if (s.board[p] < 0) lb::bset(ls.white, p);
    }
    ls.ko = s.ko;
    const int budget = ladder_budget();
    if (rec) {
      rec->black = ls.black;
      rec->white = ls.white;
      rec->budget = budget;
      rec->e.clear();
      rec->reused = rec->read = 0;
    }
    // the points where this board and the reference's differ
    const bool use_ref = ref && ref->budget == budget && !ref->e.empty();
    lb::BB diff;
    if (use_ref)
      for (int i = 0; i < lb::W; ++i)
        diff.w[i] = (ref->black.w[i] ^ ls.black.w[i]) | (ref->white.w[i] ^ ls.white.w[i]);
    size_t ri = 0;
    for (int i = 0; i < BW; ++i)
      for (uint64_t w = cand.w[i]; w; w &= w - 1) {
        const int p = i * 64 + __builtin_ctzll(w);
        if (p >= np || s.board[p] != EMPTY || !s.is_legal(p)) continue;
        int bits = -1;
        lb::BB reads;
        if (use_ref) {  // candidates ascend, so does the reference's list
          while (ri < ref->e.size() && ref->e[ri].p < p) ++ri;
          if (ri < ref->e.size() && ref->e[ri].p == p) {
            const LadderEntry& en = ref->e[ri];
            uint64_t hit = 0;
            for (int k = 0; k < lb::W; ++k) hit |= en.reads.w[k] & diff.w[k];
            if (!hit) {
              bits = en.bits;
              reads = en.reads;
              if (rec) ++rec->reused;
            }
          }
        }
        if (bits < 0) {
          if (rec) {
            lb::bzero(reads);
            lb::trace_slot() = &reads;
          }
          bits = lb::ladder_bits_at(ls, p, me, stack, g, budget);
          lb::trace_slot() = nullptr;
          if (rec) ++rec->read;
        }
        ladder[p] = (uint8_t)(bits & 3);
        if (rec) rec->e.push_back({(int16_t)p, (uint8_t)bits, reads});
      }
  }
}

// ---------------------------------------------------------------- planes
int featurize(const GameState& s, const int* fids, int nf, uint8_t* out) {
  const int np = s.np;
  const int me = s.current_player;
  // legal mask computed once and shared (get_legal_moves, go.py:261-267)
  uint8_t legal[MAXP];
  bool need_legal = false;
  for (int i = 0; i < nf; ++i) {
    int f = fids[i];
    need_legal |= (f == F_CAPTURE_SIZE || f == F_SELF_ATARI_SIZE || f == F_LIBERTIES_AFTER ||
                   f == F_SENSIBLENESS || f == F_LADDER_CAPTURE || f == F_LADDER_ESCAPE || f == F_LEGAL ||
                   f == F_SELF_ATARI_SIZE_EXACT || f == F_LIBERTIES_AFTER_EXACT);
  }
  if (need_legal)
    for (int p = 0; p < np; ++p) legal[p] = s.is_legal(p) ? 1 : 0;

  int off = 0;
  for (int i = 0; i < nf; ++i) {
    const int f = fids[i];
    const int npl = feature_planes(f);
    uint8_t* o = out + (size_t)off * np;
    std::memset(o, 0, (size_t)npl * np);
    switch (f) {
      case F_BOARD:  // preprocessing.py:9-17
        for (int p = 0; p < np; ++p) {
          int b = s.board[p];
          if (b == me) o[p] = 1;
          else if (b == -me) o[np + p] = 1;
          else o[2 * np + p] = 1;
        }
        break;
      case F_ONES:
        std::memset(o, 1, np);
        break;
      case F_ZEROS:
        break;
      case F_COLOR:  // value.py:16's 49th plane ("player colour"), SURVEY Q18
        if (me == BLACK) std::memset(o, 1, np);
        break;
      case F_TURNS_SINCE: {  // preprocessing.py:20-43
        int depth = 0;
        uint8_t marked[MAXP];
        std::memset(marked, 0, sizeof(marked));
        for (int k = (int)s.history.size() - 1; k >= 0; --k) {
          int mv = s.history[k];
          if (mv != PASS && s.board[mv] != EMPTY && !marked[mv]) {
            o[depth * np + mv] = 1;
            marked[mv] = 1;
          }
          if (depth < 7) ++depth;
        }
        break;
      }
      case F_LIBERTIES:  // preprocessing.py:46-61
        for (int p = 0; p < np; ++p) {
          int lc = s.liberty_count(p);
          if (lc >= 1) o[(lc >= 8 ? 7 : lc - 1) * np + p] = 1;
        }
        break;
      case F_CAPTURE_SIZE:  // preprocessing.py:64-88
        for (int p = 0; p < np; ++p) {
          if (!legal[p]) continue;
          int16_t roots[4];
          int k = s.groups_around(p, roots);
          int ncap = 0;
          for (int j = 0; j < k; ++j)
            if (s.libc[roots[j]] == 1 && s.board[roots[j]] != me) ncap += s.gsize[roots[j]];
          o[(ncap > 7 ? 7 : ncap) * np + p] = 1;
        }
        break;
      case F_SELF_ATARI_SIZE:  // preprocessing.py:91-115
      case F_LIBERTIES_AFTER:  // preprocessing.py:118-144
        for (int p = 0; p < np; ++p) {
          if (!legal[p]) continue;
          Bits lib = s.liberty_set(p);
          int gsz = 1;
          int16_t roots[4];
          int k = s.groups_around(p, roots);
          for (int j = 0; j < k; ++j)
            if (s.board[roots[j]] == me) {
              lib.orr(s.libs[roots[j]]);
              gsz += s.gsize[roots[j]];
            }
          lib.clear(p);
          int nl = lib.count();
          if (f == F_SELF_ATARI_SIZE) {
            if (nl == 1) o[(gsz - 1 > 7 ? 7 : gsz - 1) * np + p] = 1;
          } else {
            int plane = nl - 1;
            if (plane > 7) plane = 7;
            if (plane < 0) plane = 7;  // python index -1
            o[plane * np + p] = 1;
          }
        }
        break;
      case F_SELF_ATARI_SIZE_EXACT:
      case F_LIBERTIES_AFTER_EXACT:
        // Capture-aware liberties after playing p (Q10): the merged group's
        // liberties plus the points of opponent groups that p captures and that
        // touch the merged group; 0 liberties cannot happen for a legal move.
        for (int p = 0; p < np; ++p) {
          if (!legal[p]) continue;
          Bits lib = s.liberty_set(p);
          int gsz = 1;
          int16_t roots[4];
          const int k = s.groups_around(p, roots);
          for (int j = 0; j < k; ++j)
            if (s.board[roots[j]] == me) {
              lib.orr(s.libs[roots[j]]);
              gsz += s.gsize[roots[j]];
            }
          lib.clear(p);
          for (int j = 0; j < k; ++j) {
            const int r = roots[j];
            if (s.board[r] != -me || s.libc[r] != 1) continue;  // not captured by p
            int q = r;
            do {  // captured stone q becomes a liberty if it touches p or the merged group
              for (int e = 0; e < s.g->nnbr[q]; ++e) {
                const int t = s.g->nbr[q][e];
                bool merged = t == p;
                for (int m = 0; m < k && !merged; ++m) merged = s.board[roots[m]] == me && s.board[t] == me &&
                                                                   s.head[t] == roots[m];
                if (merged) {
                  lib.set(q);
                  break;
                }
              }
              q = s.next[q];
            } while (q != r);
          }
          const int nl = lib.count();
          if (f == F_SELF_ATARI_SIZE_EXACT) {
            if (nl == 1) o[(gsz - 1 > 7 ? 7 : gsz - 1) * np + p] = 1;
          } else if (nl >= 1) {
            o[((nl > 8 ? 8 : nl) - 1) * np + p] = 1;  // planes 1..8+ liberties
          }
        }
        break;
      case F_LADDER_CAPTURE:
        for (int p = 0; p < np; ++p)
          if (legal[p] && ladder_capture_at(s, p)) o[p] = 1;
        break;
      case F_LADDER_ESCAPE:
        for (int p = 0; p < np; ++p)
          if (legal[p] && ladder_escape_at(s, p)) o[p] = 1;
        break;
      case F_SENSIBLENESS:  // preprocessing.py:155-161
        for (int p = 0; p < np; ++p)
          if (legal[p] && !s.is_eye(p, me)) o[p] = 1;
        break;
      case F_LEGAL:
        for (int p = 0; p < np; ++p) o[p] = legal[p];
        break;
      default:
        break;
    }
    off += npl;
  }
  return off;
}

}  // namespace ag
