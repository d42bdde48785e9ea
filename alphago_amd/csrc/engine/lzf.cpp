// LZF block decompression (HDF5 filter id 32000, used by the reference's
// training-data files: game_converter.py:71-86 compression="lzf").
#include <pybind11/pybind11.h>

#include <cstdint>
#include <stdexcept>
#include <string>

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
      for (unsigned i = 0; i < ctrl; ++i) *op++ = *ip++;
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
      for (unsigned i = 0; i < len; ++i) *op++ = *ref++;
    }
  }
  return (size_t)(op - out);
}

void bind_lzf(py::module_& m) {
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
