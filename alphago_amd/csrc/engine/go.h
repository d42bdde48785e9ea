// alphago_amd native Go rules core.
//
// Semantics follow the reference rules engine (AlphaGo/go.py) — incremental
// group/liberty bookkeeping, simple-ko with the snapback exclusion
// (go.py:312-331), suicide test (go.py:181-202), recursive true-eye test
// (go.py:230-259), eyeish area scoring (go.py:269-293) and the "two passes with
// white to move" end-of-game rule (go.py:345-348) — but the data structures are
// designed for a native engine that is copied millions of times per second by
// the tree search: fixed-size arrays, one liberty *bitset* per group root and a
// circular stone list per group, so a state copy is one flat memcpy (~20 KB)
// and a liberty union is 6 OR + popcount instructions.
//
// Deliberate fixes over the reference:
//   Q2  copy() has value semantics (history, komi, passes, end flag copied).
//   Q14 bounds are checked before the board is indexed.
// Option (Q9): standard_two_pass ends the game after any two consecutive
// passes; the default keeps the reference rule (second pass by black).
#pragma once
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace ag {

constexpr int MAXN = 19;
constexpr int MAXP = MAXN * MAXN;  // 361
constexpr int BW = 6;              // 64-bit words per liberty bitset (>= 361 bits)
constexpr int8_t BLACK = 1, WHITE = -1, EMPTY = 0;
constexpr int PASS = -1;

struct Bits {
  uint64_t w[BW];
  inline void zero() { for (int i = 0; i < BW; ++i) w[i] = 0; }
  inline void set(int p) { w[p >> 6] |= (1ull << (p & 63)); }
  inline void clear(int p) { w[p >> 6] &= ~(1ull << (p & 63)); }
  inline bool test(int p) const { return (w[p >> 6] >> (p & 63)) & 1ull; }
  inline void orr(const Bits& o) { for (int i = 0; i < BW; ++i) w[i] |= o.w[i]; }
  inline int count() const {
    int c = 0;
    for (int i = 0; i < BW; ++i) c += __builtin_popcountll(w[i]);
    return c;
  }
  inline int first() const {
    for (int i = 0; i < BW; ++i)
      if (w[i]) return i * 64 + __builtin_ctzll(w[i]);
    return -1;
  }
};

// Precomputed board geometry; neighbour order matches go.py:91-102 so that
// order-dependent quirks (ko detection across multiple captures, eye recursion)
// reproduce exactly.
struct Geometry {
  int n = 0, np = 0;
  int16_t nbr[MAXP][4];
  int8_t nnbr[MAXP];
  int16_t diag[MAXP][4];
  int8_t ndiag[MAXP];
};
const Geometry& geometry(int n);

class IllegalMove : public std::runtime_error {
 public:
  explicit IllegalMove(const std::string& s) : std::runtime_error(s) {}
};

struct GameState {
  const Geometry* g;
  int n, np;
  int8_t board[MAXP];
  int16_t head[MAXP];  // group root of a stone, -1 for empty points
  int16_t next[MAXP];  // circular stone list of the group
  int16_t gsize[MAXP]; // stones in group (valid at root)
  int16_t libc[MAXP];  // liberty count (valid at root)
  Bits libs[MAXP];     // liberty set (valid at root)
  int8_t current_player;
  int turns_played;
  int ko;  // point index or -1
  double komi;
  int passes_white, passes_black;
  int num_black_prisoners, num_white_prisoners;
  bool is_end_of_game;
  bool standard_two_pass;  // Q9 option, see above
  std::vector<int16_t> history;  // PASS = -1

  explicit GameState(int size = 19, double komi_ = 7.5, bool standard_two_pass_ = false);

  inline int idx(int x, int y) const { return x * n + y; }
  inline bool on_board(int x, int y) const { return x >= 0 && y >= 0 && x < n && y < n; }

  inline int liberty_count(int p) const { return board[p] == EMPTY ? -1 : libc[head[p]]; }
  inline int group_size(int p) const { return board[p] == EMPTY ? 0 : gsize[head[p]]; }
  // liberty_sets[p] of the reference: the group's liberties for a stone, the
  // set of empty neighbours for an empty point (always exact, see go.cpp).
  Bits liberty_set(int p) const;
  std::vector<int> group_stones(int p) const;
  // unique adjacent groups (roots), in neighbour order (go.py:63-83)
  int groups_around(int p, int16_t* roots) const;

  bool is_suicide(int p) const;           // for current_player
  bool is_suicide_for(int p, int color) const;
  bool is_legal(int p) const;             // for current_player
  bool is_legal_for(int p, int color) const;
  bool is_eyeish(int p, int owner) const;
  bool is_eye(int p, int owner) const;
  void legal_moves(std::vector<int>& out, bool include_eyes = true) const;
  int get_winner() const;
  // returns is_end_of_game; throws IllegalMove
  bool do_move(int p, int color = 0);
  // Same as do_move but returns false instead of throwing.
  bool try_move(int p, int color = 0);

 private:
  bool is_eye_rec(int p, int owner, int16_t* stack, int depth) const;
  void place_stone(int p, int8_t color);
  int remove_group(int root);
};

}  // namespace ag
