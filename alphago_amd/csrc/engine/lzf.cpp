// LZF block codec (HDF5 filter id 32000, used by the reference's training-data
// files: game_converter.py:71-86 compression="lzf").
//
// Format: a sequence of runs.  ctrl < 32: ctrl+1 literal bytes follow.
// Otherwise a back reference: len = ctrl>>5 (7 = extended by the next byte),
// offset = ((ctrl & 31) << 8 | next byte) + 1, copy len+2 bytes.
// The compressor is a greedy single-probe hash matcher (the same format any
// LZF decoder reads); lzf_decompress_many decodes a list of chunks on a thread
// pool with the GIL released (chunk-sliced dataset reads, data/dataset.py).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace py = pybind11;

namespace ag {

size_t lzf_decompress(const uint8_t* in, size_t in_len, uint8_t* out, size_t out_len) {
  const uint8_t* ip = in;
  const uint8_t* const in_end = in + in_len;
  uint8_t* op = out;
  uint8_t* const out_end = out + out_len;
  while (ip < in_end) {
    unsigned ctrl = *ip++;
    if (ctrl < (1 << 5)) {  // literal run of ctrl+1 bytes
      ctrl++;
      if (op + ctrl > out_end) throw std::runtime_error("lzf: output overflow");
      if (ip + ctrl > in_end) throw std::runtime_error("lzf: input overrun");
      std::memcpy(op, ip, ctrl);
      op += ctrl;
      ip += ctrl;
    } else {  // back reference
      unsigned len = ctrl >> 5;
      const uint8_t* ref = op - ((ctrl & 0x1f) << 8) - 1;
      if (ip >= in_end) throw std::runtime_error("lzf: input overrun");
      if (len == 7) {
        len += *ip++;
        if (ip >= in_end) throw std::runtime_error("lzf: input overrun");
      }
      ref -= *ip++;
      len += 2;
      if (op + len > out_end) throw std::runtime_error("lzf: output overflow");
      if (ref < out) throw std::runtime_error("lzf: invalid back reference");
      const size_t dist = (size_t)(op - ref);
      if (dist >= len) {  // non-overlapping: one block copy
        std::memcpy(op, ref, len);
        op += len;
      } else if (dist == 1) {  // run of one repeated byte
        std::memset(op, *ref, len);
        op += len;
      } else {  // periodic overlap: copy whole periods forward
        size_t left = len;
        while (left) {
          const size_t n = std::min(dist, left);
          std::memcpy(op, ref, n);
          op += n;
          ref += n;
          left -= n;
        }
      }
    }
  }
  return (size_t)(op - out);
}

// Returns the compressed size, or 0 when the output would not be smaller than
// out_cap (the HDF5 filter then stores the chunk raw with its mask bit set).
size_t lzf_compress(const uint8_t* in, size_t in_len, uint8_t* out, size_t out_cap) {
  constexpr int HBITS = 14;
  constexpr unsigned MAX_OFF = 1u << 13, MAX_REF = (1u << 8) + (1u << 3);
  std::vector<uint32_t> htab(1u << HBITS, 0xffffffffu);
  const uint8_t* ip = in;
  const uint8_t* const in_end = in + in_len;
  uint8_t* op = out;
  uint8_t* const out_end = out + out_cap;
  uint8_t* lit_ctrl = nullptr;  // position of the current literal run's control byte
  unsigned lit = 0;
  auto emit_lit = [&](uint8_t b) -> bool {
    if (lit == 0) {
      if (op >= out_end) return false;
      lit_ctrl = op++;
    }
    if (op >= out_end) return false;
    *op++ = b;
    *lit_ctrl = (uint8_t)lit;
    if (++lit == 32) lit = 0;
    return true;
  };
  while (ip < in_end) {
    if (ip + 2 < in_end) {
      const uint32_t v = (uint32_t)ip[0] << 16 | (uint32_t)ip[1] << 8 | ip[2];
      const uint32_t h = ((v >> (24 - HBITS)) ^ v) & ((1u << HBITS) - 1);
      const uint32_t cand = htab[h];
      htab[h] = (uint32_t)(ip - in);
      if (cand != 0xffffffffu) {
        const uint8_t* ref = in + cand;
        const size_t off = (size_t)(ip - ref) - 1;
        if (off < MAX_OFF && ref[0] == ip[0] && ref[1] == ip[1] && ref[2] == ip[2]) {
          size_t len = 3;
          const size_t maxlen = std::min<size_t>(MAX_REF, (size_t)(in_end - ip));
          while (len < maxlen && ref[len] == ip[len]) ++len;
          const size_t l = len - 2;
          if (op + 3 > out_end) return 0;
          lit = 0;
          if (l < 7) {
            *op++ = (uint8_t)((off >> 8) + (l << 5));
          } else {
            *op++ = (uint8_t)((off >> 8) + (7 << 5));
            *op++ = (uint8_t)(l - 7);
          }
          *op++ = (uint8_t)off;
          ip += len;
          continue;
        }
      }
    }
    if (!emit_lit(*ip++)) return 0;
  }
  return (size_t)(op - out);
}

void bind_lzf(py::module_& m) {
  m.def(
      "lzf_compress",
      [](py::bytes data) {
        std::string s = data;
        std::string out(s.size(), '\0');
        size_t n;
        {
          py::gil_scoped_release r;
          n = s.empty() ? 0 : lzf_compress((const uint8_t*)s.data(), s.size(), (uint8_t*)&out[0], out.size());
        }
        out.resize(n);
        return py::bytes(out);
      },
      py::arg("data"), "LZF-compress; returns b'' when the data does not shrink");
  m.def(
      "lzf_decompress_into",
      [](std::vector<py::bytes> chunks, py::buffer out, size_t out_len, int threads, std::vector<int64_t> slots) {
        // decode chunk i into out[s*out_len : (s+1)*out_len], s = slots[i] (default i), in a
        // writable contiguous buffer.  Reusing one long-lived buffer matters: first-touch page
        // faults of a fresh allocation serialise the decode threads in the kernel.
        py::buffer_info bi = out.request(true);
        const size_t n = chunks.size();
        if (!slots.empty() && slots.size() != n) throw std::runtime_error("lzf: slots/chunks length mismatch");
        const size_t cap = (size_t)(bi.size * bi.itemsize) / (out_len ? out_len : 1);
        for (size_t i = 0; i < n; ++i) {
          const size_t sl = slots.empty() ? i : (size_t)slots[i];
          if (slots.empty() ? n > cap : (slots[i] < 0 || sl >= cap))
            throw std::runtime_error("lzf: output buffer too small");
        }
        std::vector<std::pair<const char*, size_t>> src(n);
        std::vector<std::string> keep(n);
        for (size_t i = 0; i < n; ++i) {
          char* p;
          Py_ssize_t len;
          if (PyBytes_AsStringAndSize(chunks[i].ptr(), &p, &len) != 0) throw py::error_already_set();
          src[i] = {p, (size_t)len};
        }
        uint8_t* dst = (uint8_t*)bi.ptr;
        std::vector<std::string> err(n);
        {
          py::gil_scoped_release r;
          std::atomic<size_t> next{0};
          auto work = [&]() {
            for (size_t i = next++; i < n; i = next++) {
              try {
                const size_t sl = slots.empty() ? i : (size_t)slots[i];
                const size_t got = lzf_decompress((const uint8_t*)src[i].first, src[i].second, dst + sl * out_len,
                                                  out_len);
                if (got != out_len) err[i] = "lzf: short chunk";
              } catch (const std::exception& e) {
                err[i] = e.what();
              }
            }
          };
          const int nt = std::max(1, std::min<int>(threads, (int)n));
          std::vector<std::thread> pool;
          for (int t = 1; t < nt; ++t) pool.emplace_back(work);
          work();
          for (auto& t : pool) t.join();
        }
        for (size_t i = 0; i < n; ++i)
          if (!err[i].empty()) throw std::runtime_error(err[i] + " (chunk " + std::to_string(i) + ")");
      },
      py::arg("chunks"), py::arg("out"), py::arg("out_len"), py::arg("threads") = 8,
      py::arg("slots") = std::vector<int64_t>());
  m.def(
      "lzf_decompress_many",
      [](std::vector<std::string> chunks, size_t out_len, int threads) {
        // decode every chunk into one contiguous buffer (chunk i at i*out_len)
        const size_t n = chunks.size();
        std::string out(n * out_len, '\0');
        std::vector<std::string> err(n);
        {
          py::gil_scoped_release r;
          std::atomic<size_t> next{0};
          auto work = [&]() {
            for (size_t i = next++; i < n; i = next++) {
              try {
                const size_t got = lzf_decompress((const uint8_t*)chunks[i].data(), chunks[i].size(),
                                                  (uint8_t*)&out[i * out_len], out_len);
                if (got != out_len) err[i] = "lzf: short chunk";
              } catch (const std::exception& e) {
                err[i] = e.what();
              }
            }
          };
          const int nt = std::max(1, std::min<int>(threads, (int)n));
          std::vector<std::thread> pool;
          for (int t = 1; t < nt; ++t) pool.emplace_back(work);
          work();
          for (auto& t : pool) t.join();
        }
        for (size_t i = 0; i < n; ++i)
          if (!err[i].empty()) throw std::runtime_error(err[i] + " (chunk " + std::to_string(i) + ")");
        return py::bytes(out);
      },
      py::arg("chunks"), py::arg("out_len"), py::arg("threads") = 8);
  m.def(
      "lzf_decompress",
      [](py::bytes data, size_t out_len) {
        std::string s = data;
        std::string out(out_len, '\0');
        size_t n;
        {
          py::gil_scoped_release r;
          n = lzf_decompress((const uint8_t*)s.data(), s.size(), (uint8_t*)&out[0], out_len);
        }
        out.resize(n);
        return py::bytes(out);
      },
      py::arg("data"), py::arg("out_len"));
}

}  // namespace ag
