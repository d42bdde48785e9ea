// Ladder reading on bitboards -- the same code runs on the host (engine,
// checked against the incremental-liberty reader in featurize.cpp) and on
// gfx950 (kernels/ladder.hip, the GPU featurizer's ladder planes).
//
// Semantics are those of featurize.cpp's ladder_capture_at / ladder_escape_at
// (the reference leaves ladder planes as NotImplementedError,
// AlphaGo/preprocessing/preprocessing.py:147-152):
//  * capture at m: m is legal for the player to move and, for an adjacent
//    opponent group with 2 liberties, playing m captures it outright or leaves
//    it in atari with every prey reply losing (prey_loses);
//  * escape at m: for an adjacent own group in atari, playing m leaves it with
//    >= 3 liberties, or with 2 and no winning hunter continuation.
//  prey_loses: prey to move, in atari: candidate replies are the prey's
//  liberty and the liberties of adjacent hunter groups in atari (capture
//  escapes, at most 8 candidates); the prey escapes if a legal reply leaves
//  >= 3 liberties, or 2 liberties and the hunter cannot win.  hunter_wins:
//  hunter to move, prey with 2 liberties: plays either liberty (ascending
//  index); wins if the prey is captured or left in atari with prey_loses.
//  Both give up (prey survives) beyond kLadderDepth plies.
// Rules (legality with simple ko and the reference's suicide rule, capture
// order, ko detection) follow go.cpp's GameState::is_legal_for / try_move with
// the neighbour order of go.py:91-96.  The search itself is iterative with an
// explicit frame stack (no recursion: on the GPU the frames live in a global
// workspace), and each frame holds a full bitboard snapshot.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define LB_HD __host__ __device__ __forceinline__
#else
#define LB_HD inline
#endif

namespace lb {

constexpr int W = 6;             // 64-bit words per 19x19 bitboard (>= 361 bits)
constexpr int kLadderDepth = 96;  // plies; a corner-to-corner ladder is < 80
constexpr int kMaxFrames = kLadderDepth + 3;
constexpr int kMaxCand = 8;
// Search-step budget per ladder_eval; reaching it returns kBudgetHit so a GPU
// wave always finishes.
#ifndef LB_MAX_STEPS
#define LB_MAX_STEPS (1 << 16)
#endif
constexpr int kMaxSteps = LB_MAX_STEPS;
constexpr int kBudgetHit = 4;  // ladder_bits_at bit: budget exhausted (result unknown)
// Node budget per root read (one capture or one escape test of a point): every
// prey_loses / hunter_wins node counts one visit; past the budget a node gives
// up like one past kLadderDepth (prey survives).  Same rule, and the same
// candidate order, in featurize.cpp.  No read of 3448 random positions (~62k
// roots) is cut at 4096 (one is at 2048); the budget bounds the rare
// exponential searches that stalled whole MCTS encode batches.
constexpr int kLadderVisits = 4096;

struct BB {
  uint64_t w[W];
};

// Read-set tracing (host only; the ladder cache of the MCTS encoder, featurize.cpp): while
// trace_slot() points at a set, every board point whose content a search reads is added to it --
// the points color_at tests, the dilation of every chain group_of fills or libs_of counts, and the
// neighbourhood of the hunter stones frame_init screens.  A search is a deterministic function of
// those points (plus the root's ko point, which only decides the root move's legality), so a board
// that differs from the traced one only outside the set gives the same result, bit for bit.
#if !defined(__HIP_DEVICE_COMPILE__)
inline BB*& trace_slot() {
  static thread_local BB* t = nullptr;
  return t;
}
#define LB_TRACE_PT(p)                                           \
  do {                                                           \
    if (::lb::BB* t_ = ::lb::trace_slot()) t_->w[(p) >> 6] |= 1ull << ((p) & 63); \
  } while (0)
#define LB_TRACE_SET(b)                                          \
  do {                                                           \
    if (::lb::BB* t_ = ::lb::trace_slot()) {                     \
      const ::lb::BB b_ = (b);                                   \
      for (int i_ = 0; i_ < ::lb::W; ++i_) t_->w[i_] |= b_.w[i_]; \
    }                                                            \
  } while (0)
#else
#define LB_TRACE_PT(p) \
  do {                 \
  } while (0)
#define LB_TRACE_SET(b) \
  do {                  \
  } while (0)
#endif

LB_HD int popc(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __popcll(x);
#else
  return __builtin_popcountll(x);
#endif
}
LB_HD int ctz(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __ffsll((long long)x) - 1;
#else
  return __builtin_ctzll(x);
#endif
}

LB_HD void bzero(BB& b) {
  for (int i = 0; i < W; ++i) b.w[i] = 0;
}
// Word selection: on the GPU by compare-and-select over the W words (a
// dynamically indexed register array would live in scratch memory); on the
// host by plain indexing.
#if defined(__HIP_DEVICE_COMPILE__)
LB_HD uint64_t bword(const BB& b, int i) {
  uint64_t r = 0;
  for (int k = 0; k < W; ++k) r |= b.w[k] & (0ull - (uint64_t)(i == k));
  return r;
}
LB_HD bool btest(const BB& b, int p) { return (bword(b, p >> 6) >> (p & 63)) & 1ull; }
LB_HD void bset(BB& b, int p) {
  const uint64_t m = 1ull << (p & 63);
  for (int k = 0; k < W; ++k) b.w[k] |= m & (0ull - (uint64_t)(k == (p >> 6)));
}
LB_HD void bclr(BB& b, int p) {
  const uint64_t m = 1ull << (p & 63);
  for (int k = 0; k < W; ++k) b.w[k] &= ~(m & (0ull - (uint64_t)(k == (p >> 6))));
}
#else
LB_HD uint64_t bword(const BB& b, int i) { return b.w[i]; }
LB_HD bool btest(const BB& b, int p) { return (b.w[p >> 6] >> (p & 63)) & 1ull; }
LB_HD void bset(BB& b, int p) { b.w[p >> 6] |= 1ull << (p & 63); }
LB_HD void bclr(BB& b, int p) { b.w[p >> 6] &= ~(1ull << (p & 63)); }
#endif
LB_HD int bcount(const BB& b) {
  int c = 0;
  for (int i = 0; i < W; ++i) c += popc(b.w[i]);
  return c;
}
LB_HD int bfirst(const BB& b) {
  for (int i = 0; i < W; ++i)
    if (b.w[i]) return i * 64 + ctz(b.w[i]);
  return -1;
}
LB_HD bool bany(const BB& b) {
  uint64_t o = 0;
  for (int i = 0; i < W; ++i) o |= b.w[i];
  return o != 0;
}
LB_HD bool beq(const BB& a, const BB& b) {
  uint64_t d = 0;
  for (int i = 0; i < W; ++i) d |= a.w[i] ^ b.w[i];
  return d == 0;
}

// Board geometry (size n, point p = x*n + y): masks for the +-1 (y) and +-n
// (x) shifts of a dilation.
struct Geo {
  int n, np;
  BB on;        // points of the board
  BB not_y0;    // destination of a +1 shift must not be y == 0
  BB not_ylast; // destination of a -1 shift must not be y == n-1
};

LB_HD void make_geo(Geo& g, int n) {
  g.n = n;
  g.np = n * n;
  bzero(g.on);
  bzero(g.not_y0);
  bzero(g.not_ylast);
  for (int p = 0; p < g.np; ++p) {
    bset(g.on, p);
    if (p % n != 0) bset(g.not_y0, p);
    if (p % n != n - 1) bset(g.not_ylast, p);
  }
}

// one-step dilation (4-neighbourhood) of b, including b
LB_HD BB dilate(const BB& b, const Geo& g) {
  const int n = g.n;
  BB o;
  for (int i = 0; i < W; ++i) {
    const uint64_t lo1 = i ? b.w[i - 1] >> 63 : 0;                 // carry for << 1
    const uint64_t hi1 = i + 1 < W ? b.w[i + 1] << 63 : 0;         // carry for >> 1
    const uint64_t lon = i ? b.w[i - 1] >> (64 - n) : 0;           // carry for << n
    const uint64_t hin = i + 1 < W ? b.w[i + 1] << (64 - n) : 0;   // carry for >> n
    const uint64_t up1 = ((b.w[i] << 1) | lo1) & g.not_y0.w[i];
    const uint64_t dn1 = ((b.w[i] >> 1) | hi1) & g.not_ylast.w[i];
    const uint64_t upn = (b.w[i] << n) | lon;
    const uint64_t dnn = (b.w[i] >> n) | hin;
    o.w[i] = (b.w[i] | up1 | dn1 | upn | dnn) & g.on.w[i];
  }
  return o;
}

struct LState {
  BB black, white;
  int ko;  // -1 = none
};

LB_HD int color_at(const LState& s, int p) {
  LB_TRACE_PT(p);
  return btest(s.black, p) ? 1 : (btest(s.white, p) ? -1 : 0);
}
// per-word selects (no reference to one of two register aggregates, which the
// GPU compiler would materialise in scratch)
LB_HD BB stones_copy(const LState& s, int c) {
  const uint64_t sel = 0ull - (uint64_t)(c > 0);
  BB r;
  for (int k = 0; k < W; ++k) r.w[k] = (s.black.w[k] & sel) | (s.white.w[k] & ~sel);
  return r;
}

// the chain through p (p must hold a stone)
LB_HD BB group_of(const LState& s, int p, const Geo& g) {
  const BB own = stones_copy(s, color_at(s, p));
  BB grp;
  bzero(grp);
  bset(grp, p);
  for (int it = 0; it < g.np; ++it) {  // converges in < np dilations; bounded loop
    BB d = dilate(grp, g);
    for (int i = 0; i < W; ++i) d.w[i] &= own.w[i];
    if (beq(d, grp)) break;
    grp = d;
  }
  LB_TRACE_SET(dilate(grp, g));
  return grp;
}

// group_of with the caller's known chain (the ladder's prey group, tracked
// incrementally): a long prey chain is never flood-filled again
LB_HD BB group_hint(const LState& s, int q, const Geo& g, const BB& known) {
  if (btest(known, q)) return known;
  return group_of(s, q, g);
}

// points with at least two empty 4-neighbours (e = empty points)
LB_HD BB two_empty_nbrs(const BB& e, const Geo& g) {
  const int n = g.n;
  BB r;
  for (int i = 0; i < W; ++i) {
    const uint64_t lo1 = i ? e.w[i - 1] >> 63 : 0;
    const uint64_t hi1 = i + 1 < W ? e.w[i + 1] << 63 : 0;
    const uint64_t lon = i ? e.w[i - 1] >> (64 - n) : 0;
    const uint64_t hin = i + 1 < W ? e.w[i + 1] << (64 - n) : 0;
    const uint64_t a = ((e.w[i] << 1) | lo1) & g.not_y0.w[i];     // empty at p - 1
    const uint64_t b = ((e.w[i] >> 1) | hi1) & g.not_ylast.w[i];  // empty at p + 1
    const uint64_t c = (e.w[i] << n) | lon;                        // empty at p - n
    const uint64_t d = (e.w[i] >> n) | hin;                        // empty at p + n
    r.w[i] = ((a & b) | (a & c) | (a & d) | (b & c) | (b & d) | (c & d)) & g.on.w[i];
  }
  return r;
}

LB_HD BB libs_of(const LState& s, const BB& grp, const Geo& g) {
  BB d = dilate(grp, g);
  LB_TRACE_SET(d);
  for (int i = 0; i < W; ++i) d.w[i] &= ~(s.black.w[i] | s.white.w[i]);
  return d;
}

// neighbours of p in go.py:91-96 order: (x-1, y), (x+1, y), (x, y-1), (x, y+1);
// off-board slots are -1 (fixed slots keep the array in registers on the GPU)
LB_HD void neighbours(int p, const Geo& g, int* out) {
  const int n = g.n, x = p / n, y = p - x * n;
  out[0] = x > 0 ? p - n : -1;
  out[1] = x + 1 < n ? p + n : -1;
  out[2] = y > 0 ? p - 1 : -1;
  out[3] = y + 1 < n ? p + 1 : -1;
}

// go.cpp GameState::is_suicide_for (go.py:181-202)
LB_HD bool is_suicide_for(const LState& s, int p, int color, const Geo& g, const BB& known) {
  int nb[4];
  neighbours(p, g, nb);
  for (int i = 0; i < 4; ++i)
    if (nb[i] >= 0 && color_at(s, nb[i]) == 0) return false;
  for (int i = 0; i < 4; ++i) {
    const int q = nb[i];
    if (q < 0) continue;
    const BB grp = group_hint(s, q, g, known);
    const BB lb = libs_of(s, grp, g);
    const int other = bcount(lb) - (btest(lb, p) ? 1 : 0);
    const int cq = color_at(s, q);
    if (cq == color && other > 0) return false;
    if (cq == -color && other == 0) return false;
  }
  return true;
}

// `known`: a chain of s whose membership the caller knows (or an empty set)
LB_HD bool is_legal_for(const LState& s, int p, int color, const Geo& g, const BB& known) {
  if (p < 0 || p >= g.np) return false;
  if (color_at(s, p) != 0) return false;
  if (p == s.ko) return false;
  return !is_suicide_for(s, p, color, g, known);
}

// go.cpp GameState::try_move for a legal non-pass move (capture order and ko
// detection in neighbour order, go.py:312-331)
LB_HD void play(LState& s, int p, int c, const Geo& g, const BB& known) {
  s.ko = -1;
  const uint64_t selb = 0ull - (uint64_t)(c > 0);  // all ones when black moves
  {
    const uint64_t m = 1ull << (p & 63);
    for (int k = 0; k < W; ++k) {
      const uint64_t mk = m & (0ull - (uint64_t)(k == (p >> 6)));
      s.black.w[k] |= mk & selb;
      s.white.w[k] |= mk & ~selb;
    }
  }
  int nb[4];
  neighbours(p, g, nb);
  for (int i = 0; i < 4; ++i) {
    const int q = nb[i];
    if (q < 0 || color_at(s, q) != -c) continue;
    // a stone with an empty neighbour keeps its chain alive: no flood fill
    int qn[4];
    neighbours(q, g, qn);
    bool open = false;
    for (int j = 0; j < 4; ++j) open |= qn[j] >= 0 && color_at(s, qn[j]) == 0;
    if (open) continue;
    const BB grp = group_hint(s, q, g, known);
    if (bany(libs_of(s, grp, g))) continue;
    for (int j = 0; j < W; ++j) {
      s.white.w[j] &= ~(grp.w[j] & selb);
      s.black.w[j] &= ~(grp.w[j] & ~selb);
    }
    if (bcount(grp) == 1) {
      const BB own = group_of(s, p, g);
      if (bcount(own) == 1 && bcount(libs_of(s, own, g)) == 1) s.ko = q;
    }
  }
}

LB_HD int prey_libcount(const LState& s, int prey, const Geo& g) {
  return bcount(libs_of(s, group_of(s, prey, g), g));
}

// the prey chain after the prey played p (pg: the chain before): if p touches
// it, p joins it with every own-colour chain next to p; a move elsewhere (a
// capture escape on a hunter's last liberty) leaves it as it was
LB_HD BB grow_chain(const LState& s, const BB& pg, int p, int color, const Geo& g) {
  int nb[4];
  neighbours(p, g, nb);
  bool touches = false;
  for (int i = 0; i < 4; ++i) touches |= nb[i] >= 0 && btest(pg, nb[i]);
  if (!touches) return pg;
  BB r = pg;
  bset(r, p);
  for (int i = 0; i < 4; ++i) {
    const int q = nb[i];
    if (q < 0 || color_at(s, q) != color || btest(r, q)) continue;
    const BB o = group_of(s, q, g);
    for (int k = 0; k < W; ++k) r.w[k] |= o.w[k];
  }
  return r;
}

enum : int { F_HUNTER = 0, F_PREY = 1 };

struct Frame {
  LState s;
  BB pg;  // the prey chain in s (tracked incrementally, never re-flood-filled)
  int prey, kind, depth, nc, k;
  int16_t cand[kMaxCand];
};

// Returns the first `res` of a new frame when it is decided without search
// (1 = hunter wins / prey loses, 0 = not), else -1 after filling the frame.
LB_HD int frame_init(Frame& f, const LState& st, const Geo& g, int& visits, int budget) {
  f.k = 0;
  f.nc = 0;
  if (++visits > budget) return 0;       // node budget spent: give up, prey survives
  if (f.depth > kLadderDepth) return 0;  // both give up: prey survives
  const int pc = color_at(st, f.prey);
  const BB& grp = f.pg;
  const BB lb = libs_of(st, grp, g);
  if (f.kind == F_HUNTER) {
    const int lc = bcount(lb);
    if (lc == 1) return 1;
    if (lc >= 3) return 0;
    BB b = lb;
    for (int t = 0; t < 2; ++t) {
      const int l = bfirst(b);
      if (l < 0) break;
      bclr(b, l);
      f.cand[f.nc++] = (int16_t)l;
    }
    return -1;
  }
  // prey: its liberty, then liberties of adjacent hunter groups in atari
  f.cand[f.nc++] = (int16_t)bfirst(lb);
  BB around = dilate(grp, g);
  LB_TRACE_SET(dilate(around, g));  // the hunter stones next to the chain and their neighbours
  BB hunters = stones_copy(st, -pc);
  for (int i = 0; i < W; ++i) hunters.w[i] &= around.w[i];
  // A chain holding a stone with two empty neighbours has two liberties: it is
  // not in atari, and none of its stones can be the key of an atari chain, so
  // dropping such stones keeps the candidate list and its order.
  {
    BB e;
    for (int i = 0; i < W; ++i) e.w[i] = g.on.w[i] & ~(st.black.w[i] | st.white.w[i]);
    const BB ge2 = two_empty_nbrs(e, g);
    for (int i = 0; i < W; ++i) hunters.w[i] &= ~ge2.w[i];
  }
  for (int it = 0; it < g.np && bany(hunters); ++it) {
    const int q = bfirst(hunters);
    const BB hg = group_of(st, q, g);
    for (int i = 0; i < W; ++i) hunters.w[i] &= ~hg.w[i];
    const BB hl = libs_of(st, hg, g);
    if (bcount(hl) == 1) {
      const int l = bfirst(hl);
      bool dup = false;
      for (int j = 0; j < f.nc; ++j) dup |= (f.cand[j] == l);
      if (!dup && f.nc < kMaxCand) f.cand[f.nc++] = (int16_t)l;
    }
  }
  return -1;
}

// Evaluate a root frame already placed in stack[0] (s, prey, kind, depth set).
// stack must hold kMaxFrames frames.  Returns 1/0.  The working state stays
// in registers; a frame's snapshot is written only when a child is pushed and
// read back only when the search returns to that frame.
template <class Stack>
LB_HD int ladder_eval(Stack& stack, const Geo& g, int& visits, int budget) {
  int top = 0;
  LState cur = stack[0].s;
  int res = frame_init(stack[0], cur, g, visits, budget);
  if (res >= 0) return res;
  res = -1;
  bool reload = false;
  for (int step = 0;; ++step) {
    if (step >= kMaxSteps) return -2;
    Frame& f = stack[top];
    if (reload) {
      cur = f.s;
      reload = false;
    }
    const int prey = f.prey, kind = f.kind;
    const int pc = color_at(cur, prey);
    int ret = -1;  // this frame's own result, once decided
    if (res >= 0) {  // a child returned
      if (kind == F_HUNTER && res == 1) ret = 1;      // prey_loses -> hunter wins
      else if (kind == F_PREY && res == 0) ret = 0;   // hunter fails -> prey escapes
      res = -1;
    }
    bool pushed = false;
    int k = f.k;
    const int nc = f.nc < kMaxCand ? f.nc : kMaxCand;
    LState ns;
    BB npg;
    while (ret < 0 && k < nc) {
      const int mv = f.cand[k++];
      const int mover = kind == F_HUNTER ? -pc : pc;
      if (mv < 0 || !is_legal_for(cur, mv, mover, g, f.pg)) continue;
      ns = cur;
      play(ns, mv, mover, g, f.pg);
      if (kind == F_HUNTER) {
        if (color_at(ns, prey) != pc) { ret = 1; break; }  // captured outright
        npg = f.pg;  // a hunter move leaves the prey chain as it was
        if (bcount(libs_of(ns, npg, g)) != 1) continue;
      } else {
        if (color_at(ns, prey) != pc) continue;
        npg = grow_chain(ns, f.pg, mv, pc, g);
        const int lc = bcount(libs_of(ns, npg, g));
        if (lc >= 3) { ret = 0; break; }
        if (lc != 2) continue;
      }
      Frame& c = stack[top + 1];
      c.pg = npg;
      c.prey = prey;
      c.kind = kind == F_HUNTER ? F_PREY : F_HUNTER;
      c.depth = f.depth + 1;
      const int r = frame_init(c, ns, g, visits, budget);
      if (r >= 0) {
        if (kind == F_HUNTER && r == 1) ret = 1;
        if (kind == F_PREY && r == 0) ret = 0;
        continue;
      }
      f.k = k;
      if (k < nc) f.s = cur;  // needed again only if this frame has candidates left
      c.s = ns;
      cur = ns;
      ++top;
      pushed = true;
      break;
    }
    if (pushed) continue;
    if (ret < 0) ret = (kind == F_HUNTER) ? 0 : 1;  // no candidate succeeded
    if (top == 0) return ret;
    --top;
    res = ret;
    reload = true;
  }
}

// featurize.cpp ladder_capture_at / ladder_escape_at on a root state whose
// player to move is `me`; bit 0 = capture, bit 1 = escape.
template <class Stack>
LB_HD int ladder_bits_at(const LState& s, int m, int me, Stack& stack, const Geo& g, int budget = kLadderVisits) {
  BB none;
  bzero(none);
  if (!is_legal_for(s, m, me, g, none)) return 0;
  int visits = 0;  // per capture test, then per escape test (featurize.cpp resets per call)
  int nb[4];
  neighbours(m, g, nb);
  int out = 0;
  for (int i = 0; i < 4 && !(out & 1); ++i) {  // capture
    const int q = nb[i];
    if (q < 0 || color_at(s, q) != -me) continue;
    const BB pg = group_of(s, q, g);
    if (bcount(libs_of(s, pg, g)) != 2) continue;
    Frame& f = stack[0];
    LState ns = s;
    play(ns, m, me, g, pg);
    if (color_at(ns, q) != -me) { out |= 1; break; }
    if (bcount(libs_of(ns, pg, g)) != 1) continue;
    f.s = ns;
    f.pg = pg;
    f.prey = q;
    f.kind = F_PREY;
    f.depth = 0;
    const int r = ladder_eval(stack, g, visits, budget);
    if (r == -2) return out | kBudgetHit;
    if (r == 1) out |= 1;
  }
  visits = 0;
  for (int i = 0; i < 4 && !(out & 2); ++i) {  // escape
    const int q = nb[i];
    if (q < 0 || color_at(s, q) != me) continue;
    const BB pg0 = group_of(s, q, g);
    if (bcount(libs_of(s, pg0, g)) != 1) continue;
    Frame& f = stack[0];
    LState ns = s;
    play(ns, m, me, g, pg0);
    if (color_at(ns, q) != me) continue;
    const BB pg = grow_chain(ns, pg0, m, me, g);
    const int lc = bcount(libs_of(ns, pg, g));
    if (lc >= 3) { out |= 2; break; }
    if (lc != 2) continue;
    f.s = ns;
    f.pg = pg;
    f.prey = q;
    f.kind = F_HUNTER;
    f.depth = 0;
    const int r = ladder_eval(stack, g, visits, budget);
    if (r == -2) return out | kBudgetHit;
    if (r == 0) out |= 2;
  }
  return out;
}

// Candidate points (the CPU encoder's filter): empty liberties of opponent
// groups with 2 liberties or own groups with 1 liberty.
LB_HD bool is_candidate(const LState& s, int p, int me, const Geo& g) {
  if (color_at(s, p) != 0) return false;
  int nb[4];
  neighbours(p, g, nb);
  for (int i = 0; i < 4; ++i) {
    const int q = nb[i];
    if (q < 0) continue;
    const int c = color_at(s, q);
    if (c == 0) continue;
    const int lc = prey_libcount(s, q, g);
    if ((c == -me && lc == 2) || (c == me && lc == 1)) return true;
  }
  return false;
}

}  // namespace lb
