// Python bindings of the native LMDB engine (csrc/lmdb_core.h): key lookup and
// a GIL-free multithreaded fixed-size record gather into a (pinned) tensor.
// Reference: /root/reference/torchbooster/lmdb.py (LMDBReader over py-lmdb).
#include "lmdb_core.h"

#include <torch/extension.h>


// ---------------------------------------------------------------- bindings
namespace {
namespace py = pybind11;

py::object env_get(const tbamd::LmdbEnv& e, py::bytes key) {
  std::string k = key;
  size_t n = 0;
  const uint8_t* v = e.find((const uint8_t*)k.data(), k.size(), &n);
  if (!v) return py::none();
  return py::bytes((const char*)v, n);
}

// Copy records idx[i] (keys str(idx)) into rows of `out` (uint8 [B, row_bytes],
// typically pinned).  Multi-threaded, GIL released.  Returns the number of
// bytes of each record (must all equal row_bytes unless `allow_short`).
void env_gather(const tbamd::LmdbEnv& e, std::vector<int64_t> idx, torch::Tensor out, int64_t threads) {
  TORCH_CHECK(out.dtype() == torch::kUInt8 && out.dim() == 2 && out.is_contiguous() && !out.is_cuda(),
              "gather: out must be a contiguous uint8 [B, bytes] host tensor");
  TORCH_CHECK((int64_t)idx.size() == out.size(0), "gather: batch mismatch");
  const int64_t row = out.size(1);
  uint8_t* dst = out.data_ptr<uint8_t>();
  std::atomic<int64_t> next{0};
  std::atomic<int> err{0};
  std::string errmsg;
  auto work = [&]() {
    char kb[32];
    for (;;) {
      const int64_t i = next.fetch_add(1);
      if (i >= (int64_t)idx.size() || err.load()) return;
      const int kl = std::snprintf(kb, sizeof(kb), "%lld", (long long)idx[i]);
      size_t n = 0;
      const uint8_t* v = nullptr;
      try {
        v = e.find((const uint8_t*)kb, (size_t)kl, &n);
      } catch (...) {
        err = 1;
        return;
      }
      if (!v || (int64_t)n != row) {
        err = v ? 2 : 3;
        return;
      }
      std::memcpy(dst + i * row, v, n);
    }
  };
  {
    py::gil_scoped_release nogil;
    int nt = (int)std::max<int64_t>(1, std::min<int64_t>(threads, (int64_t)idx.size()));
    std::vector<std::thread> pool;
    for (int t = 1; t < nt; ++t) pool.emplace_back(work);
    work();
    for (auto& th : pool) th.join();
  }
  TORCH_CHECK(err.load() == 0, err.load() == 2 ? "gather: record size != row bytes"
                                               : (err.load() == 3 ? "gather: missing key" : "gather: read error"));
}

}  // namespace

void register_lmdb(pybind11::module& m) {
  py::class_<tbamd::LmdbEnv>(m, "LmdbEnv")
      .def(py::init<const std::string&>())
      .def("get", &env_get)
      .def("gather", &env_gather, py::arg("indices"), py::arg("out"), py::arg("threads") = 8)
      .def("close", &tbamd::LmdbEnv::close)
      .def_property_readonly("is_open", &tbamd::LmdbEnv::is_open)
      .def_property_readonly("entries", &tbamd::LmdbEnv::entries)
      .def_property_readonly("page_size", &tbamd::LmdbEnv::page_size)
      .def_property_readonly("depth", &tbamd::LmdbEnv::depth);
  m.def("lmdb_write",
        [](const std::string& path, std::vector<std::pair<py::bytes, py::bytes>> items, uint64_t map_size,
           uint32_t psize) {
          std::vector<std::pair<std::string, std::string>> v;
          v.reserve(items.size());
          for (auto& it : items) v.emplace_back(std::string(it.first), std::string(it.second));
          py::gil_scoped_release nogil;
          tbamd::lmdb_write(path, std::move(v), map_size, psize);
        },
        py::arg("path"), py::arg("items"), py::arg("map_size") = (uint64_t)1 << 30, py::arg("psize") = 4096);
  py::class_<tbamd::LmdbStreamWriter>(m, "LmdbStreamWriter")
      .def(py::init<const std::string&, uint64_t, uint32_t>(), py::arg("path"),
           py::arg("map_size") = (uint64_t)1 << 30, py::arg("psize") = 4096)
      .def("add",
           [](tbamd::LmdbStreamWriter& w, py::bytes key, py::bytes value) {
             std::string k = key, v = value;
             py::gil_scoped_release nogil;
             w.add(k, v);
           })
      .def("close", &tbamd::LmdbStreamWriter::close)
      .def_property_readonly("entries", &tbamd::LmdbStreamWriter::entries);
}

void register_prefetch(pybind11::module& m) {}
