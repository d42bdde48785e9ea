// pybind11 bindings for the native engine: module alphago_amd._engine.
// Python-facing API keeps the reference's method names (AlphaGo/go.py) with
// (x, y) tuples for moves and None for pass.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

#include "ladder_bb.h"
#include <pybind11/stl.h>

#include <thread>

#include "featurize.h"
#include "go.h"
#include "mcts.h"

namespace py = pybind11;
using namespace ag;

namespace ag {
void bind_mcts(pybind11::module_& m);
void bind_lzf(py::module_& m);
void bind_lockstep(py::module_& m);
}

static int to_idx(const GameState& s, const py::object& a) {
  if (a.is_none()) return PASS;
  auto t = a.cast<std::pair<int, int>>();
  if (!s.on_board(t.first, t.second)) return -2;  // off-board sentinel
  return s.idx(t.first, t.second);
}
static py::object to_move(const GameState& s, int p) {
  if (p == PASS) return py::none();
  return py::make_tuple(p / s.n, p % s.n);
}
static py::set stones_to_set(const GameState& s, const std::vector<int>& v) {
  py::set out;
  for (int p : v) out.add(py::make_tuple(p / s.n, p % s.n));
  return out;
}

static std::vector<int> parse_features(const std::vector<std::string>& names) {
  std::vector<int> ids;
  for (auto& nm : names) {
    std::string low = nm;
    for (auto& c : low) c = (char)tolower(c);
    int id = feature_id(low);
    if (id < 0) throw py::value_error("unknown feature: " + nm);
    ids.push_back(id);
  }
  return ids;
}

PYBIND11_MODULE(_engine, m) {
  m.doc() = "alphago_amd native Go engine (rules, featurizer, batched MCTS)";
  static py::exception<IllegalMove> exc(m, "IllegalMove");
  py::register_exception_translator([](std::exception_ptr p) {
    try {
      if (p) std::rethrow_exception(p);
    } catch (const IllegalMove& e) {
      exc(e.what());
    }
  });
  m.attr("BLACK") = (int)BLACK;
  m.attr("WHITE") = (int)WHITE;
  m.attr("EMPTY") = (int)EMPTY;

  py::class_<GameState>(m, "GameState")
      .def(py::init<int, double, bool>(), py::arg("size") = 19, py::arg("komi") = 7.5,
           py::arg("standard_two_pass") = false)
      .def_readonly("size", &GameState::n)
      .def_property(
          "current_player", [](const GameState& s) { return (int)s.current_player; },
          [](GameState& s, int c) { s.current_player = (int8_t)c; })
      .def_readwrite("turns_played", &GameState::turns_played)
      .def_readwrite("komi", &GameState::komi)
      .def_readwrite("passes_white", &GameState::passes_white)
      .def_readwrite("passes_black", &GameState::passes_black)
      .def_readwrite("num_black_prisoners", &GameState::num_black_prisoners)
      .def_readwrite("num_white_prisoners", &GameState::num_white_prisoners)
      .def_readwrite("is_end_of_game", &GameState::is_end_of_game)
      .def_readwrite("standard_two_pass", &GameState::standard_two_pass)
      .def_property(
          "ko", [](const GameState& s) { return s.ko < 0 ? py::none() : to_move(s, s.ko); },
          [](GameState& s, py::object k) { s.ko = k.is_none() ? -1 : to_idx(s, k); })
      .def_property_readonly("board",
                             [](const GameState& s) {
                               py::array_t<double> a({s.n, s.n});
                               auto r = a.mutable_unchecked<2>();
                               for (int x = 0; x < s.n; ++x)
                                 for (int y = 0; y < s.n; ++y) r(x, y) = s.board[x * s.n + y];
                               return a;
                             })
      .def_property_readonly("liberty_counts",
                             [](const GameState& s) {
                               py::array_t<int64_t> a({s.n, s.n});
                               auto r = a.mutable_unchecked<2>();
                               for (int x = 0; x < s.n; ++x)
                                 for (int y = 0; y < s.n; ++y) r(x, y) = s.liberty_count(x * s.n + y);
                               return a;
                             })
      .def_property_readonly("history",
                             [](const GameState& s) {
                               py::list l;
                               for (auto p : s.history) l.append(to_move(s, p));
                               return l;
                             })
      .def("history_indices", [](const GameState& s) { return std::vector<int>(s.history.begin(), s.history.end()); })
      .def("board_array",
           [](const GameState& s) {
             py::array_t<int8_t> a({s.n, s.n});
             std::memcpy(a.mutable_data(), s.board, s.np);
             return a;
           })
      .def("copy", [](const GameState& s) { return GameState(s); })
      .def("__copy__", [](const GameState& s) { return GameState(s); })
      .def("__deepcopy__", [](const GameState& s, py::dict) { return GameState(s); })
      .def(
          "do_move",
          [](GameState& s, py::object action, py::object color) {
            int p = to_idx(s, action);
            int c = color.is_none() ? 0 : color.cast<int>();
            if (p == -2) throw IllegalMove(py::str(action).cast<std::string>());
            return s.do_move(p, c);
          },
          py::arg("action"), py::arg("color") = py::none())
      .def("is_legal",
           [](const GameState& s, py::object action) {
             int p = to_idx(s, action);
             return p != -2 && s.is_legal(p);
           })
      .def("is_suicide", [](const GameState& s, py::object a) { return s.is_suicide(to_idx(s, a)); })
      .def("is_eyeish",
           [](const GameState& s, py::object a, int owner) { return s.is_eyeish(to_idx(s, a), owner); })
      .def(
          "is_eye", [](const GameState& s, py::object a, int owner) { return s.is_eye(to_idx(s, a), owner); },
          py::arg("position"), py::arg("owner"))
      .def(
          "get_legal_moves",
          [](const GameState& s, bool include_eyes) {
            std::vector<int> v;
            s.legal_moves(v, include_eyes);
            py::list l;
            for (int p : v) l.append(to_move(s, p));
            return l;
          },
          py::arg("include_eyes") = true)
      .def("legal_mask",
           [](const GameState& s, bool include_eyes) {
             py::array_t<uint8_t> a(s.np);
             auto* d = a.mutable_data();
             for (int p = 0; p < s.np; ++p)
               d[p] = s.is_legal(p) && (include_eyes || !s.is_eye(p, s.current_player));
             return a;
           },
           py::arg("include_eyes") = true)
      .def("get_winner", &GameState::get_winner)
      .def("get_group", [](const GameState& s, py::object a) { return stones_to_set(s, s.group_stones(to_idx(s, a))); })
      .def("get_groups_around",
           [](const GameState& s, py::object a) {
             int16_t roots[4];
             int k = s.groups_around(to_idx(s, a), roots);
             py::list l;
             for (int i = 0; i < k; ++i) l.append(stones_to_set(s, s.group_stones(roots[i])));
             return l;
           })
      .def("ladder_capture", [](const GameState& s, py::object a) { return ladder_capture_at(s, to_idx(s, a)); })
      .def("ladder_escape", [](const GameState& s, py::object a) { return ladder_escape_at(s, to_idx(s, a)); });

  m.def("feature_planes", [](const std::string& name) {
    int id = feature_id(name);
    if (id < 0) throw py::value_error("unknown feature: " + name);
    return feature_planes(id);
  });
  m.def("featurize",
        [](const GameState& s, const std::vector<std::string>& names) {
          auto ids = parse_features(names);
          int nplanes = 0;
          for (int id : ids) nplanes += feature_planes(id);
          py::array_t<uint8_t> a({nplanes, s.n, s.n});
          featurize(s, ids.data(), (int)ids.size(), a.mutable_data());
          return a;
        });
  m.def(
      "featurize_batch",
      [](const std::vector<const GameState*>& states, const std::vector<std::string>& names, int threads) {
        auto ids = parse_features(names);
        int nplanes = 0;
        for (int id : ids) nplanes += feature_planes(id);
        if (states.empty()) return py::array_t<uint8_t>(std::vector<ssize_t>{0, nplanes, 0, 0});
        int n = states[0]->n;
        for (auto* s : states)
          if (s->n != n) throw py::value_error("all states must have the same size");
        py::array_t<uint8_t> a({(ssize_t)states.size(), (ssize_t)nplanes, (ssize_t)n, (ssize_t)n});
        uint8_t* base = a.mutable_data();
        size_t stride = (size_t)nplanes * n * n;
        {
          py::gil_scoped_release rel;
          int B = (int)states.size();
          int T = std::max(1, std::min(threads, B));
          std::vector<std::thread> pool;
          for (int t = 0; t < T; ++t)
            pool.emplace_back([&, t]() {
              for (int i = t; i < B; i += T) featurize(*states[i], ids.data(), (int)ids.size(), base + i * stride);
            });
          for (auto& th : pool) th.join();
        }
        return a;
      },
      py::arg("states"), py::arg("features"), py::arg("threads") = 8);

  m.def(
      "encode_batch",
      [](const std::vector<const GameState*>& states, bool ladder, int threads) -> py::tuple {
        const ssize_t B = (ssize_t)states.size();
        const int np = B ? states[0]->np : 0;
        for (auto* s : states)
          if (s->np != np) throw py::value_error("all states must have the same size");
        py::array_t<int8_t> board({B, (ssize_t)np});
        py::array_t<uint8_t> ages({B, (ssize_t)np});
        py::array_t<int32_t> meta({B, (ssize_t)2});
        py::array_t<uint8_t> lad({ladder ? B : (ssize_t)0, (ssize_t)np});
        int8_t* pb = board.mutable_data();
        uint8_t* pa = ages.mutable_data();
        int32_t* pm = meta.mutable_data();
        uint8_t* pl = ladder ? lad.mutable_data() : nullptr;
        {
          py::gil_scoped_release rel;
          int T = std::max(1, std::min(threads, (int)B));
          std::vector<std::thread> pool;
          for (int t = 0; t < T; ++t)
            pool.emplace_back([&, t]() {
              for (ssize_t i = t; i < B; i += T)
                encode_state(*states[i], pb + i * np, pa + i * np, pm + 2 * i, pl ? pl + i * np : nullptr);
            });
          for (auto& th : pool) th.join();
        }
        py::object l = ladder ? py::object(lad) : py::object(py::none());
        return py::make_tuple(board, ages, meta, l);
      },
      py::arg("states"), py::arg("ladder") = false, py::arg("threads") = 8);

  m.def(
      "ladder_bits_bb",
      [](py::array_t<int8_t, py::array::c_style> board, py::array_t<int32_t, py::array::c_style> meta, int n,
         int threads) {
        // host run of the bitboard ladder reader (ladder_bb.h, the code of the GPU kernel)
        // from the compact encoding: bit 0 capture, bit 1 escape, per point
        const ssize_t B = board.shape(0), np = board.shape(1);
        if (np != (ssize_t)n * n || meta.shape(0) != B) throw py::value_error("shape mismatch");
        py::array_t<uint8_t> out({B, np});
        const int8_t* pb = board.data();
        const int32_t* pm = meta.data();
        uint8_t* po = out.mutable_data();
        {
          py::gil_scoped_release rel;
          lb::Geo g;
          lb::make_geo(g, n);
          const int T = std::max(1, std::min(threads, (int)B));
          std::vector<std::thread> pool;
          for (int t = 0; t < T; ++t)
            pool.emplace_back([&, t]() {
              std::vector<lb::Frame> stack(lb::kMaxFrames);
              for (ssize_t i = t; i < B; i += T) {
                lb::LState s;
                lb::bzero(s.black);
                lb::bzero(s.white);
                for (int p = 0; p < np; ++p) {
                  if (pb[i * np + p] > 0) lb::bset(s.black, p);
                  if (pb[i * np + p] < 0) lb::bset(s.white, p);
                }
                s.ko = pm[2 * i];
                const int me = pm[2 * i + 1];
                const int budget = ladder_budget();
                for (int p = 0; p < np; ++p)
                  po[i * np + p] =
                      lb::is_candidate(s, p, me, g) ? (uint8_t)lb::ladder_bits_at(s, p, me, stack, g, budget) : 0;
              }
            });
          for (auto& th : pool) th.join();
        }
        return out;
      },
      py::arg("board"), py::arg("meta"), py::arg("n"), py::arg("threads") = 8);
  m.def("set_ladder_budget", &set_ladder_budget, py::arg("visits"),
        "node budget of one ladder capture / escape read (CPU, bitboard and GPU readers); 0 = default");
  m.def("ladder_budget", &ladder_budget);

  bind_mcts(m);
  bind_lzf(m);
  bind_lockstep(m);
}
