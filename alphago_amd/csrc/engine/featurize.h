// Board featurizer (CPU/native path).  Plane semantics are those of the
// reference preprocessing (AlphaGo/preprocessing/preprocessing.py:9-214),
// including its quirks (liberties_after: 0 liberties -> plane 7).
// Output is uint8 one-hot planes laid out [plane][x][y] (x = SGF column,
// flattened move index x*size+y as util.py:6-8).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "go.h"
#include "ladder_bb.h"

namespace ag {

enum FeatureId : int {
  F_BOARD = 0,
  F_ONES,
  F_TURNS_SINCE,
  F_LIBERTIES,
  F_CAPTURE_SIZE,
  F_SELF_ATARI_SIZE,
  F_LIBERTIES_AFTER,
  F_LADDER_CAPTURE,
  F_LADDER_ESCAPE,
  F_SENSIBLENESS,
  F_ZEROS,
  F_COLOR,
  F_LEGAL,
  F_SELF_ATARI_SIZE_EXACT,  // capture-aware variants, CPU only
  F_LIBERTIES_AFTER_EXACT,
  F_NUM
};

int feature_planes(int fid);
int feature_id(const std::string& name);  // -1 if unknown
const char* feature_name(int fid);

// Write planes for one state; returns the number of planes written.
int featurize(const GameState& s, const int* fids, int nf, uint8_t* out);

// Compact encoding consumed by the GPU featurizer (kernels/featurize.hip):
// board[p] in {-1,0,1}; ages[p] = turns_since plane (0..7) or 255; meta =
// {ko or -1, player to move}; ladder (optional) bit0 = ladder capture,
// bit1 = ladder escape (only computed when requested: it is the expensive part).
//
// Ladder cache (the MCTS encoder, Forest::leaf_encode): with `rec`, every candidate point's read is
// recorded with its read set (ladder_bb.h trace_slot) next to the board; with `ref` -- the record of a
// state with the same player to move, e.g. the leaf's grandparent or an already encoded sibling -- a
// candidate whose recorded read set holds none of the points where the two boards differ takes the
// recorded result instead of reading again.  The reuse is exact: the read is a function of the board on
// its read set (the ko point only decides the root move's legality, which encode_state checks on the
// state itself first).
struct LadderEntry {
  int16_t p;
  uint8_t bits;  // lb::ladder_bits_at
  lb::BB reads;  // the board points the read looked at
};
struct LadderRecord {
  lb::BB black, white;
  int budget = -1;  // the node budget the reads ran with (ladder_budget())
  std::vector<LadderEntry> e;  // ascending p
  int reused = 0, read = 0;    // entries taken from the reference / read here
};
void encode_state(const GameState& s, int8_t* board, uint8_t* ages, int32_t* meta, uint8_t* ladder,
                  const LadderRecord* ref = nullptr, LadderRecord* rec = nullptr);

// Ladder reading (paper features; NotImplementedError in the reference
// preprocessing.py:147-152).  Exposed for tests.
bool ladder_capture_at(const GameState& s, int move);
bool ladder_escape_at(const GameState& s, int move);
// node budget of one capture / escape read (default lb::kLadderVisits); 0 restores the default
void set_ladder_budget(int visits);
int ladder_budget();

}  // namespace ag
