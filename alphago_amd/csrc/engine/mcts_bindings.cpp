// pybind11 bindings of the batched MCTS forest (module _engine.Forest).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "featurize.h"
#include "mcts.h"

namespace py = pybind11;

namespace ag {

static int tup_to_idx(const GameState& s, const py::object& a) {
  if (a.is_none()) return PASS;
  auto t = a.cast<std::pair<int, int>>();
  return s.idx(t.first, t.second);
}
static py::object idx_to_tup(const GameState& s, int p) {
  if (p == PASS) return py::none();
  return py::make_tuple(p / s.n, p % s.n);
}

void bind_mcts(py::module_& m) {
  py::class_<Forest>(m, "Forest")
      .def(py::init([](int n_trees, double c_puct, double lmbda, int rollout_limit, int playout_depth, int vl,
                       uint64_t seed, std::vector<std::string> features) {
             std::vector<int> ids;
             for (auto& f : features) {
               int id = feature_id(f);
               if (id < 0) throw py::value_error("unknown feature: " + f);
               ids.push_back(id);
             }
             return new Forest(n_trees, c_puct, lmbda, rollout_limit, playout_depth, vl, seed, ids);
           }),
           py::arg("n_trees"), py::arg("c_puct") = 5.0, py::arg("lmbda") = 0.0, py::arg("rollout_limit") = 500,
           py::arg("playout_depth") = 1000, py::arg("virtual_loss") = 3, py::arg("seed") = 0,
           py::arg("features") = std::vector<std::string>{})
      .def_property_readonly("n_trees", &Forest::n_trees)
      .def_property_readonly("feature_planes", &Forest::feature_planes)
      .def_property_readonly("n_pending", &Forest::n_pending)
      .def_property_readonly("total_evals", &Forest::total_evals)
      .def("set_root", &Forest::set_root)
      .def("root_state", [](const Forest& f, int t) { return GameState(f.root_state(t)); })
      .def(
          "gather",
          [](Forest& f, int lpt, py::object which) {
            if (which.is_none()) {
              py::gil_scoped_release r;
              return f.gather(lpt, nullptr);
            }
            std::vector<int> w = which.cast<std::vector<int>>();
            py::gil_scoped_release r;
            return f.gather(lpt, &w);
          },
          py::arg("leaves_per_tree") = 1, py::arg("which") = py::none())
      .def("leaf_state", [](const Forest& f, int i) { return GameState(f.leaf_state(i)); })
      .def(
          "leaf_features",
          [](const Forest& f, int threads) {
            int L = f.n_pending();
            int n = L ? f.leaf_state(0).n : 0;
            py::array_t<uint8_t> a({(ssize_t)L, (ssize_t)f.feature_planes(), (ssize_t)n, (ssize_t)n});
            uint8_t* d = a.mutable_data();
            {
              py::gil_scoped_release r;
              f.leaf_features(d, threads);
            }
            return a;
          },
          py::arg("threads") = 8)
      .def(
          "leaf_features_into",
          [](const Forest& f, uintptr_t ptr, size_t capacity, int threads) {
            int L = f.n_pending();
            if (L == 0) return 0;
            size_t need = (size_t)L * f.feature_planes() * f.leaf_state(0).np;
            if (need > capacity) throw py::value_error("leaf_features_into: buffer too small");
            py::gil_scoped_release r;
            f.leaf_features(reinterpret_cast<uint8_t*>(ptr), threads);
            return L;
          },
          py::arg("ptr"), py::arg("capacity"), py::arg("threads") = 8)
      .def("hold", &Forest::hold)
      .def("swap_held", &Forest::swap_held)
      .def("discard", &Forest::discard)
      .def("n_held_tree", &Forest::n_held_tree)
      .def("held_counts", &Forest::held_counts)
      .def_property_readonly("n_held", &Forest::n_held)
      .def(
          "leaf_encode_into",
          [](Forest& f, uintptr_t board, uintptr_t ages, uintptr_t meta, uintptr_t ladder, size_t capacity,
             int threads) {
            int L = f.n_pending();
            if (L == 0) return 0;
            if ((size_t)L > capacity) throw py::value_error("leaf_encode_into: buffer too small");
            py::gil_scoped_release r;
            f.leaf_encode(reinterpret_cast<int8_t*>(board), reinterpret_cast<uint8_t*>(ages),
                          reinterpret_cast<int32_t*>(meta), ladder ? reinterpret_cast<uint8_t*>(ladder) : nullptr,
                          threads);
            return L;
          },
          py::arg("board"), py::arg("ages"), py::arg("meta"), py::arg("ladder"), py::arg("capacity"),
          py::arg("threads") = 8)
      .def("leaf_masks",
           [](const Forest& f) {
             int L = f.n_pending();
             int np = L ? f.leaf_state(0).np : 0;
             py::array_t<uint8_t> a({(ssize_t)L, (ssize_t)np});
             f.leaf_masks(a.mutable_data());
             return a;
           })
      .def(
          "apply",
          [](Forest& f, py::array_t<float, py::array::c_style | py::array::forcecast> priors, py::object values,
             py::object mask) {
            int L = f.n_pending();
            if (L == 0) return;
            int np = f.leaf_state(0).np;
            if (priors.ndim() != 2 || priors.shape(0) != L || priors.shape(1) != np)
              throw py::value_error("priors must be (n_pending, size*size)");
            const float* pv = priors.data();
            const float* vv = nullptr;
            const uint8_t* mv = nullptr;
            py::array_t<float, py::array::c_style | py::array::forcecast> va;
            py::array_t<uint8_t, py::array::c_style | py::array::forcecast> ma;
            if (!values.is_none()) {
              va = values.cast<py::array_t<float, py::array::c_style | py::array::forcecast>>();
              if (va.size() != L) throw py::value_error("values must have n_pending entries");
              vv = va.data();
            }
            if (!mask.is_none()) {
              ma = mask.cast<py::array_t<uint8_t, py::array::c_style | py::array::forcecast>>();
              if (ma.size() != (ssize_t)L * np) throw py::value_error("mask must be (n_pending, size*size)");
              mv = ma.data();
            }
            py::gil_scoped_release r;
            f.apply(pv, vv, mv);
          },
          py::arg("priors"), py::arg("values") = py::none(), py::arg("mask") = py::none())
      .def("set_threads", &Forest::set_threads, py::arg("n"))
      .def_property("ladder_cache", &Forest::ladder_cache, &Forest::set_ladder_cache)
      .def("clear_ladder_cache", &Forest::clear_ladder_cache)
      .def("ladder_cache_stats",
           [](const Forest& f) {
             int64_t n, reused, read, bytes, ev;
             f.ladder_cache_stats(n, reused, read, bytes, ev);
             py::dict d;
             d["records"] = n;
             d["reused"] = reused;
             d["read"] = read;
             d["bytes"] = bytes;
             d["evictions"] = ev;
             d["budget_bytes"] = f.ladder_cache_bytes();
             return d;
           })
      .def("set_ladder_cache_bytes", &Forest::set_ladder_cache_bytes, py::arg("bytes"))
      .def_property("rollout_policy", &Forest::rollout_policy, &Forest::set_rollout_policy)
      .def("add_root_noise", &Forest::add_root_noise, py::arg("tree"), py::arg("alpha") = 0.03,
           py::arg("eps") = 0.25)
      .def("root_stats",
           [](const Forest& f, int t) {
             std::vector<int> mv, vis;
             std::vector<float> q;
             f.root_stats(t, mv, vis, q);
             py::list moves;
             for (int p : mv) moves.append(idx_to_tup(f.root_state(t), p));
             return py::make_tuple(moves, vis, q);
           })
      .def(
          "best_move",
          [](Forest& f, int t, double temp) { return idx_to_tup(f.root_state(t), f.best_move(t, temp)); },
          py::arg("tree"), py::arg("temperature") = 0.0)
      .def("advance", [](Forest& f, int t, py::object mv) { f.advance(t, tup_to_idx(f.root_state(t), mv)); })
      .def("sims", &Forest::sims)
      .def("max_expanded_depth", &Forest::max_expanded_depth, py::arg("tree"));
}

}  // namespace ag
