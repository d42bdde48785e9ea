// Native lock-step game driver: N games advanced together, one batched policy forward per side per
// ply (reference make_training_pairs, AlphaGo/training/reinforcement_policy_trainer.py:16-76, and the
// value-network position generator).  The Python loop of round 3 (search/selfplay.py) spent ~70 % of
// a ply on the host: per-game do_move calls through pybind, list comprehensions over the games, a
// fresh std::thread team per encode.  Here one call applies a group's sampled moves to all of its
// games, one call encodes a group into caller-owned (pinned) buffers for the GPU featurizer, and the
// active/turn bookkeeping comes back as numpy arrays -- all on a persistent worker pool with the GIL
// released, so the host work of one group overlaps the other group's forward on the device.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cstdint>
#include <memory>
#include <random>
#include <vector>

#include "featurize.h"
#include "go.h"
#include "workpool.h"

namespace py = pybind11;

namespace ag {

namespace {

template <typename T>
using carray = py::array_t<T, py::array::c_style | py::array::forcecast>;

template <typename T>
T* mut_ptr(py::array& a, ssize_t min_elems, const char* what) {
  if (!(a.flags() & py::array::c_style) || a.itemsize() != (ssize_t)sizeof(T) || a.size() < min_elems)
    throw py::value_error(std::string("lockstep: bad output buffer ") + what);
  return static_cast<T*>(a.mutable_data());
}

}  // namespace

class Lockstep {
 public:
  Lockstep(int n_games, int size, double komi, bool standard_two_pass, int threads)
      : pool_(std::max(0, threads - 1)), np_(size * size), size_(size) {
    if (n_games <= 0) throw py::value_error("lockstep: n_games must be positive");
    games_.reserve(n_games);
    for (int i = 0; i < n_games; ++i) games_.emplace_back(size, komi, standard_two_pass);
  }

  int n() const { return (int)games_.size(); }
  int size() const { return size_; }

  // (n,) uint8: 1 while the game is running
  py::array_t<uint8_t> active() const {
    py::array_t<uint8_t> a(n());
    auto* d = a.mutable_data();
    for (int i = 0; i < n(); ++i) d[i] = games_[i].is_end_of_game ? 0 : 1;
    return a;
  }

  // (n,) int8: the colour to move (+1 black, -1 white)
  py::array_t<int8_t> to_move() const {
    py::array_t<int8_t> a(n());
    auto* d = a.mutable_data();
    for (int i = 0; i < n(); ++i) d[i] = games_[i].current_player;
    return a;
  }

  // Active games split by whose turn it is: (colour[i] to move, the others), ascending indices.
  py::tuple groups(const carray<int8_t>& colors) const {
    if (colors.size() != n()) throw py::value_error("lockstep: colors must have one entry per game");
    const int8_t* c = colors.data();
    std::vector<int32_t> a, b;
    for (int i = 0; i < n(); ++i) {
      if (games_[i].is_end_of_game) continue;
      (games_[i].current_player == c[i] ? a : b).push_back(i);
    }
    return py::make_tuple(py::array_t<int32_t>((ssize_t)a.size(), a.data()),
                          py::array_t<int32_t>((ssize_t)b.size(), b.data()));
  }

  // Compact encoding of games idx into the first k rows of caller-owned buffers (the GPU featurizer's
  // inputs: board int8 (>=k, np), ages uint8 (>=k, np), meta int32 (>=k, 2), ladder uint8 or None).
  void encode(const carray<int32_t>& idx, py::array board, py::array ages, py::array meta, py::object ladder) {
    const int k = (int)idx.size();
    const int32_t* ix = idx.data();
    check_idx(ix, k);
    int8_t* pb = mut_ptr<int8_t>(board, (ssize_t)k * np_, "board");
    uint8_t* pa = mut_ptr<uint8_t>(ages, (ssize_t)k * np_, "ages");
    int32_t* pm = mut_ptr<int32_t>(meta, (ssize_t)k * 2, "meta");
    uint8_t* pl = nullptr;
    py::array lad;
    if (!ladder.is_none()) {
      lad = ladder.cast<py::array>();
      pl = mut_ptr<uint8_t>(lad, (ssize_t)k * np_, "ladder");
    }
    py::gil_scoped_release rel;
    parallel(k, [&](int r) {
      encode_state(games_[ix[r]], pb + (size_t)r * np_, pa + (size_t)r * np_, pm + 2 * r,
                   pl ? pl + (size_t)r * np_ : nullptr);
    });
  }

  // Host featurisation of games idx (records of the value-position generator, CPU fallbacks).
  py::array_t<uint8_t> featurize(const carray<int32_t>& idx, const std::vector<std::string>& names) {
    std::vector<int> ids;
    int nplanes = 0;
    for (auto& nm : names) {
      const int id = feature_id(nm);
      if (id < 0) throw py::value_error("unknown feature: " + nm);
      ids.push_back(id);
      nplanes += feature_planes(id);
    }
    const int k = (int)idx.size();
    const int32_t* ix = idx.data();
    check_idx(ix, k);
    py::array_t<uint8_t> out({(ssize_t)k, (ssize_t)nplanes, (ssize_t)size_, (ssize_t)size_});
    uint8_t* po = out.mutable_data();
    const size_t stride = (size_t)nplanes * np_;
    py::gil_scoped_release rel;
    parallel(k, [&](int r) { ag::featurize(games_[ix[r]], ids.data(), (int)ids.size(), po + r * stride); });
    return out;
  }

  // Apply flat move indices (-1 = pass) to games idx; a move the rules refuse becomes a pass (cannot
  // happen for samples from the sensible-move mask).  Returns the number of games still running.
  int play(const carray<int32_t>& idx, const carray<int64_t>& moves) {
    const int k = (int)idx.size();
    if (moves.size() < k) throw py::value_error("lockstep: one move per game");
    const int32_t* ix = idx.data();
    const int64_t* mv = moves.data();
    check_idx(ix, k);
    {
      py::gil_scoped_release rel;
      parallel(k, [&](int r) {
        GameState& g = games_[ix[r]];
        if (g.is_end_of_game) return;
        const int64_t m = mv[r];
        const int p = (m < 0 || m >= np_) ? PASS : (int)m;
        if (!g.try_move(p)) g.try_move(PASS);
      });
    }
    int alive = 0;
    for (auto& g : games_) alive += g.is_end_of_game ? 0 : 1;
    return alive;
  }

  // One uniformly random sensible move (legal, not filling an own eye) per game idx, applied; pass when
  // there is none.  Returns the flat moves (-1 = pass).  Seeded per call: deterministic.
  py::array_t<int64_t> play_random(const carray<int32_t>& idx, uint64_t seed) {
    const int k = (int)idx.size();
    const int32_t* ix = idx.data();
    check_idx(ix, k);
    py::array_t<int64_t> out(k);
    int64_t* po = out.mutable_data();
    py::gil_scoped_release rel;
    parallel(k, [&](int r) {
      GameState& g = games_[ix[r]];
      std::vector<int> cand;
      g.legal_moves(cand, false);
      std::mt19937_64 rng(seed * 0x9E3779B97F4A7C15ull + (uint64_t)ix[r]);
      int m = PASS;
      if (!cand.empty()) m = cand[rng() % cand.size()];
      if (!g.try_move(m)) {
        g.try_move(PASS);
        m = PASS;
      }
      po[r] = m;
    });
    return out;
  }

  py::array_t<int32_t> winners() const {
    py::array_t<int32_t> a(n());
    auto* d = a.mutable_data();
    for (int i = 0; i < n(); ++i) d[i] = games_[i].get_winner();
    return a;
  }

  py::array_t<int32_t> lengths() const {
    py::array_t<int32_t> a(n());
    auto* d = a.mutable_data();
    for (int i = 0; i < n(); ++i) d[i] = (int32_t)games_[i].history.size();
    return a;
  }

  GameState state(int i) const {
    if (i < 0 || i >= n()) throw py::index_error("lockstep: game index");
    return games_[i];
  }

 private:
  void check_idx(const int32_t* ix, int k) const {
    for (int r = 0; r < k; ++r)
      if (ix[r] < 0 || ix[r] >= n()) throw py::index_error("lockstep: game index out of range");
  }

  // parts of ~16 games per worker claim (one game per part is too fine for the pool's counter)
  template <typename F>
  void parallel(int k, const F& f) {
    constexpr int kChunk = 16;
    const int parts = (k + kChunk - 1) / kChunk;
    pool_.run(parts, [&](int part) {
      const int e = std::min(k, (part + 1) * kChunk);
      for (int r = part * kChunk; r < e; ++r) f(r);
    });
  }

  std::vector<GameState> games_;
  WorkPool pool_;
  int np_, size_;
};

void bind_lockstep(py::module_& m) {
  py::class_<Lockstep>(m, "Lockstep", "N games advanced in lock-step (native RL / value-generation driver)")
      .def(py::init<int, int, double, bool, int>(), py::arg("n_games"), py::arg("size") = 19, py::arg("komi") = 7.5,
           py::arg("standard_two_pass") = false, py::arg("threads") = 8)
      .def_property_readonly("n", &Lockstep::n)
      .def_property_readonly("size", &Lockstep::size)
      .def("active", &Lockstep::active)
      .def("to_move", &Lockstep::to_move)
      .def("groups", &Lockstep::groups, py::arg("colors"))
      .def("encode", &Lockstep::encode, py::arg("idx"), py::arg("board"), py::arg("ages"), py::arg("meta"),
           py::arg("ladder") = py::none())
      .def("featurize", &Lockstep::featurize, py::arg("idx"), py::arg("features"))
      .def("play", &Lockstep::play, py::arg("idx"), py::arg("moves"))
      .def("play_random", &Lockstep::play_random, py::arg("idx"), py::arg("seed"))
      .def("winners", &Lockstep::winners)
      .def("lengths", &Lockstep::lengths)
      .def("state", &Lockstep::state, py::arg("i"));
}

}  // namespace ag
