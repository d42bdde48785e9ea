// Native Go rules core — see go.h for the design notes.
#include "go.h"

#include <mutex>

namespace ag {

static Geometry g_geoms[MAXN + 1];
static std::once_flag g_geom_once;

static void build_geometries() {
  for (int n = 1; n <= MAXN; ++n) {
    Geometry& g = g_geoms[n];
    g.n = n;
    g.np = n * n;
    for (int x = 0; x < n; ++x)
      for (int y = 0; y < n; ++y) {
        int p = x * n + y;
        // go.py:91-96 neighbour order
        const int nx[4] = {x - 1, x + 1, x, x};
        const int ny[4] = {y, y, y - 1, y + 1};
        int k = 0;
        for (int i = 0; i < 4; ++i)
          if (nx[i] >= 0 && ny[i] >= 0 && nx[i] < n && ny[i] < n) g.nbr[p][k++] = nx[i] * n + ny[i];
        g.nnbr[p] = k;
        // go.py:98-102 diagonal order
        const int dx[4] = {x - 1, x + 1, x + 1, x - 1};
        const int dy[4] = {y - 1, y + 1, y - 1, y + 1};
        k = 0;
        for (int i = 0; i < 4; ++i)
          if (dx[i] >= 0 && dy[i] >= 0 && dx[i] < n && dy[i] < n) g.diag[p][k++] = dx[i] * n + dy[i];
        g.ndiag[p] = k;
      }
  }
}

const Geometry& geometry(int n) {
  if (n < 1 || n > MAXN) throw std::invalid_argument("board size must be in [1, 19]");
  std::call_once(g_geom_once, build_geometries);
  return g_geoms[n];
}

GameState::GameState(int size, double komi_, bool standard_two_pass_) : standard_two_pass(standard_two_pass_) {
  g = &geometry(size);
  n = size;
  np = size * size;
  std::memset(board, 0, sizeof(board));
  for (int p = 0; p < MAXP; ++p) {
    head[p] = -1;
    next[p] = -1;
    gsize[p] = 0;
    libc[p] = 0;
    libs[p].zero();
  }
  current_player = BLACK;
  turns_played = 0;
  ko = -1;
  komi = komi_;
  passes_white = passes_black = 0;
  num_black_prisoners = num_white_prisoners = 0;
  is_end_of_game = false;
}

Bits GameState::liberty_set(int p) const {
  if (board[p] != EMPTY) return libs[head[p]];
  // For an empty point the reference keeps the set of empty neighbours.  It is
  // maintained incrementally there (go.py:109,148-152); it can never go stale
  // because a captured group has, by definition, no empty neighbour at capture
  // time, so recomputing it here is exact.
  Bits b;
  b.zero();
  for (int i = 0; i < g->nnbr[p]; ++i) {
    int q = g->nbr[p][i];
    if (board[q] == EMPTY) b.set(q);
  }
  return b;
}

std::vector<int> GameState::group_stones(int p) const {
  std::vector<int> out;
  if (board[p] == EMPTY) return out;
  int s = p;
  do {
    out.push_back(s);
    s = next[s];
  } while (s != p);
  return out;
}

int GameState::groups_around(int p, int16_t* roots) const {
  int k = 0;
  for (int i = 0; i < g->nnbr[p]; ++i) {
    int q = g->nbr[p][i];
    if (board[q] == EMPTY) continue;
    int h = head[q];
    bool seen = false;
    for (int j = 0; j < k; ++j) seen |= (roots[j] == h);
    if (!seen) roots[k++] = (int16_t)h;
  }
  return k;
}

bool GameState::is_suicide_for(int p, int color) const {
  // go.py:181-202
  for (int i = 0; i < g->nnbr[p]; ++i)
    if (board[g->nbr[p][i]] == EMPTY) return false;
  for (int i = 0; i < g->nnbr[p]; ++i) {
    int q = g->nbr[p][i];
    int h = head[q];
    int other = libc[h] - (libs[h].test(p) ? 1 : 0);
    if (board[q] == color && other > 0) return false;
    if (board[q] == -color && other == 0) return false;
  }
  return true;
}

bool GameState::is_suicide(int p) const { return is_suicide_for(p, current_player); }

bool GameState::is_legal_for(int p, int color) const {
  if (p == PASS) return true;
  if (p < 0 || p >= np) return false;
  if (board[p] != EMPTY) return false;
  if (p == ko) return false;
  return !is_suicide_for(p, color);
}

bool GameState::is_legal(int p) const { return is_legal_for(p, current_player); }

bool GameState::is_eyeish(int p, int owner) const {
  if (board[p] != EMPTY) return false;
  for (int i = 0; i < g->nnbr[p]; ++i)
    if (board[g->nbr[p][i]] != owner) return false;
  return true;
}

bool GameState::is_eye_rec(int p, int owner, int16_t* stack, int depth) const {
  // go.py:230-259.  `stack` holds the chain of callers; a diagonal that is on
  // the chain counts as good (breaks the mutual-support cycle).
  if (!is_eyeish(p, owner)) return false;
  int bad = 0;
  int allowable = (g->nnbr[p] == 4) ? 1 : 0;
  for (int i = 0; i < g->ndiag[p]; ++i) {
    int d = g->diag[p][i];
    if (board[d] == -owner) {
      ++bad;
    } else if (board[d] == EMPTY) {
      bool on_stack = false;
      for (int j = 0; j < depth; ++j) on_stack |= (stack[j] == d);
      if (!on_stack) {
        stack[depth] = (int16_t)p;
        if (!is_eye_rec(d, owner, stack, depth + 1)) ++bad;
      }
    }
    if (bad > allowable) return false;
  }
  return true;
}

bool GameState::is_eye(int p, int owner) const {
  int16_t stack[MAXP + 1];
  return is_eye_rec(p, owner, stack, 0);
}

void GameState::legal_moves(std::vector<int>& out, bool include_eyes) const {
  out.clear();
  for (int p = 0; p < np; ++p)
    if (is_legal(p) && (include_eyes || !is_eye(p, current_player))) out.push_back(p);
}

int GameState::get_winner() const {
  // go.py:269-293 — area = stones + eyeish empties, komi to white, -1 per pass
  double sw = 0, sb = 0;
  for (int p = 0; p < np; ++p) {
    if (board[p] == WHITE) sw += 1;
    else if (board[p] == BLACK) sb += 1;
    else if (is_eyeish(p, BLACK)) sb += 1;
    else if (is_eyeish(p, WHITE)) sw += 1;
  }
  sw += komi;
  sw -= passes_white;
  sb -= passes_black;
  if (sb > sw) return BLACK;
  if (sw > sb) return WHITE;
  return 0;
}

void GameState::place_stone(int p, int8_t color) {
  // go.py:104-136 (_update_neighbors) with bitset liberties
  board[p] = color;
  head[p] = (int16_t)p;
  next[p] = (int16_t)p;
  gsize[p] = 1;
  Bits lib;
  lib.zero();
  for (int i = 0; i < g->nnbr[p]; ++i) {
    int q = g->nbr[p][i];
    if (board[q] == EMPTY) lib.set(q);
  }
  libs[p] = lib;
  int root = p;
  for (int i = 0; i < g->nnbr[p]; ++i) {
    int q = g->nbr[p][i];
    if (board[q] == EMPTY) continue;
    int h = head[q];
    libs[h].clear(p);
    if (board[q] == -color) {
      libc[h] = (int16_t)libs[h].count();
    } else if (h != root) {
      // merge the smaller group into the larger one
      int big = root, small = h;
      if (gsize[h] > gsize[root]) { big = h; small = root; }
      int s = small;
      do { head[s] = (int16_t)big; s = next[s]; } while (s != small);
      // splice circular lists
      int16_t nb = next[big];
      next[big] = next[small];
      next[small] = nb;
      gsize[big] = (int16_t)(gsize[big] + gsize[small]);
      libs[big].orr(libs[small]);
      root = big;
    }
  }
  libs[root].clear(p);
  libc[root] = (int16_t)libs[root].count();
}

int GameState::remove_group(int root) {
  // go.py:138-157
  std::vector<int> stones = group_stones(root);
  for (int s : stones) board[s] = EMPTY;
  for (int s : stones) {
    head[s] = -1;
    next[s] = -1;
    gsize[s] = 0;
    libs[s].zero();
    libc[s] = 0;
  }
  for (int s : stones) {
    for (int i = 0; i < g->nnbr[s]; ++i) {
      int q = g->nbr[s][i];
      if (board[q] != EMPTY) {
        int h = head[q];
        libs[h].set(s);
        libc[h] = (int16_t)libs[h].count();
      }
    }
  }
  return (int)stones.size();
}

bool GameState::try_move(int p, int color) {
  // go.py:295-349
  int8_t c = color ? (int8_t)color : current_player;
  if (!is_legal_for(p, c)) return false;
  ko = -1;
  if (p != PASS) {
    place_stone(p, c);
    for (int i = 0; i < g->nnbr[p]; ++i) {
      int q = g->nbr[p][i];
      if (board[q] == -c && libc[head[q]] == 0) {
        int ncap = remove_group(head[q]);
        if (c == BLACK) num_white_prisoners += ncap;
        else num_black_prisoners += ncap;
        if (ncap == 1) {
          int h = head[p];
          if (libc[h] == 1 && gsize[h] == 1) ko = q;
        }
      }
    }
  } else {
    if (c == BLACK) passes_black += 1;
    else passes_white += 1;
  }
  current_player = (int8_t)(-c);
  turns_played += 1;
  history.push_back((int16_t)p);
  size_t hn = history.size();
  if (hn > 1 && history[hn - 1] == PASS && history[hn - 2] == PASS && (standard_two_pass || current_player == WHITE))
    is_end_of_game = true;
  return true;
}

bool GameState::do_move(int p, int color) {
  if (!try_move(p, color)) {
    if (p == PASS) throw IllegalMove("pass");
    throw IllegalMove("(" + std::to_string(p / n) + ", " + std::to_string(p % n) + ")");
  }
  return is_end_of_game;
}

}  // namespace ag
