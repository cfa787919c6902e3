// Native read-only LMDB engine + bulk writer (no liblmdb / py-lmdb in this stack).
//
// Reference: /root/reference/torchbooster/lmdb.py (LMDBReader over py-lmdb,
// opened readonly / lock=False / readahead=False; key b"length" holds the
// dataset size; item i lives under str(i)).  SURVEY.md §7.4 hard part 5.
//
// The reader understands the LMDB on-disk format (64-bit, data version 1):
// two meta pages (the one with the larger txnid wins), B+tree branch/leaf
// pages, F_BIGDATA values on overflow pages, default lexicographic key order
// (memcmp, shorter-first on ties).  The file is mmap'ed read-only, lookups are
// lock-free and thread-safe, and `gather` copies many fixed-size records into
// one (pinned) host buffer from a C++ thread pool with the GIL released — the
// fast path of the pinned prefetcher (K24).
//
// The writer bulk-loads sorted (key, value) pairs into a fresh file in the same
// format (used by dataset `prepare` steps and the tests).
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include <torch/extension.h>

namespace tbamd {
namespace lmdbfmt {

constexpr uint32_t kMagic = 0xBEEFC0DE;
constexpr uint32_t kVersion = 1;
constexpr size_t kPageHdr = 16;
constexpr size_t kNodeHdr = 8;
constexpr uint16_t P_BRANCH = 0x01, P_LEAF = 0x02, P_OVERFLOW = 0x04, P_META = 0x08, P_LEAF2 = 0x20;
constexpr uint16_t F_BIGDATA = 0x01, F_SUBDATA = 0x02, F_DUPDATA = 0x04;
constexpr uint64_t P_INVALID = ~0ull;

struct DbRec {  // MDB_db, 48 bytes
  uint32_t pad;
  uint16_t flags;
  uint16_t depth;
  uint64_t branch_pages, leaf_pages, overflow_pages, entries, root;
};
static_assert(sizeof(DbRec) == 48, "MDB_db layout");

struct MetaRec {  // MDB_meta
  uint32_t magic, version;
  uint64_t address, mapsize;
  DbRec dbs[2];
  uint64_t last_pg, txnid;
};
static_assert(sizeof(MetaRec) == 136, "MDB_meta layout");

inline uint16_t rd16(const uint8_t* p) { uint16_t v; std::memcpy(&v, p, 2); return v; }
inline uint32_t rd32(const uint8_t* p) { uint32_t v; std::memcpy(&v, p, 4); return v; }
inline uint64_t rd64(const uint8_t* p) { uint64_t v; std::memcpy(&v, p, 8); return v; }

inline int keycmp(const uint8_t* a, size_t la, const uint8_t* b, size_t lb) {
  const size_t n = la < lb ? la : lb;
  int c = n ? std::memcmp(a, b, n) : 0;
  if (c) return c;
  return la < lb ? -1 : (la > lb ? 1 : 0);
}

}  // namespace lmdbfmt

class LmdbEnv {
 public:
  explicit LmdbEnv(const std::string& path) {
    struct stat st;
    std::string file = path;
    if (::stat(path.c_str(), &st) == 0 && S_ISDIR(st.st_mode)) file = path + "/data.mdb";
    fd_ = ::open(file.c_str(), O_RDONLY | O_CLOEXEC);
    if (fd_ < 0) throw std::runtime_error("lmdb: cannot open " + file);
    if (::fstat(fd_, &st) != 0) throw std::runtime_error("lmdb: stat failed");
    size_ = (size_t)st.st_size;
    if (size_ < 2 * 4096) {
      ::close(fd_);
      throw std::runtime_error("lmdb: file too small: " + file);
    }
    base_ = (const uint8_t*)::mmap(nullptr, size_, PROT_READ, MAP_SHARED, fd_, 0);
    if (base_ == MAP_FAILED) {
      ::close(fd_);
      throw std::runtime_error("lmdb: mmap failed");
    }
    ::madvise((void*)base_, size_, MADV_RANDOM);  // readahead=False
    using namespace lmdbfmt;
    MetaRec m0;
    std::memcpy(&m0, base_ + kPageHdr, sizeof(MetaRec));
    if (m0.magic != kMagic) throw std::runtime_error("lmdb: bad magic");
    if (m0.version != kVersion) throw std::runtime_error("lmdb: unsupported data version");
    psize_ = m0.dbs[0].pad ? m0.dbs[0].pad : 4096;
    MetaRec m1;
    std::memcpy(&m1, base_ + psize_ + kPageHdr, sizeof(MetaRec));
    meta_ = (m1.magic == kMagic && m1.txnid > m0.txnid) ? m1 : m0;
    main_ = meta_.dbs[1];
    if (main_.flags & 0x04 /*MDB_DUPSORT*/) throw std::runtime_error("lmdb: DUPSORT databases unsupported");
  }
  ~LmdbEnv() { close(); }
  void close() {
    if (base_ && base_ != MAP_FAILED) ::munmap((void*)base_, size_);
    base_ = nullptr;
    if (fd_ >= 0) ::close(fd_);
    fd_ = -1;
  }
  bool is_open() const { return base_ != nullptr; }
  uint64_t entries() const { return main_.entries; }
  uint32_t page_size() const { return psize_; }
  uint64_t depth() const { return main_.depth; }

  // Returns pointer/length of the value or nullptr if absent.
  const uint8_t* find(const uint8_t* key, size_t klen, size_t* vlen) const {
    using namespace lmdbfmt;
    if (!base_) throw std::runtime_error("lmdb: environment is closed");
    uint64_t pg = main_.root;
    if (pg == P_INVALID) return nullptr;
    for (int guard = 0; guard < 64; ++guard) {
      const uint8_t* p = page(pg);
      const uint16_t flags = rd16(p + 10);
      const uint16_t lower = rd16(p + 12);
      const int n = (int)((lower - kPageHdr) >> 1);
      if (flags & P_LEAF2) throw std::runtime_error("lmdb: LEAF2 pages unsupported");
      if (flags & P_BRANCH) {
        // last node whose key <= search key (node 0 acts as -inf)
        int lo = 1, hi = n - 1, pick = 0;
        while (lo <= hi) {
          const int mid = (lo + hi) >> 1;
          const uint8_t* nd = node(p, mid);
          const int c = keycmp(key, klen, nd + kNodeHdr, rd16(nd + 6));
          if (c >= 0) { pick = mid; lo = mid + 1; } else { hi = mid - 1; }
        }
        const uint8_t* nd = node(p, pick);
        pg = (uint64_t)rd16(nd) | ((uint64_t)rd16(nd + 2) << 16) | ((uint64_t)rd16(nd + 4) << 32);
        continue;
      }
      if (!(flags & P_LEAF)) throw std::runtime_error("lmdb: corrupt page type");
      int lo = 0, hi = n - 1;
      while (lo <= hi) {
        const int mid = (lo + hi) >> 1;
        const uint8_t* nd = node(p, mid);
        const uint16_t ks = rd16(nd + 6);
        const int c = keycmp(key, klen, nd + kNodeHdr, ks);
        if (c == 0) {
          const uint16_t nf = rd16(nd + 4);
          const size_t dsz = (size_t)rd16(nd) | ((size_t)rd16(nd + 2) << 16);
          const uint8_t* data = nd + kNodeHdr + ks;
          if (nf & (F_SUBDATA | F_DUPDATA)) throw std::runtime_error("lmdb: sub-databases unsupported");
          *vlen = dsz;
          if (nf & F_BIGDATA) {
            const uint64_t ov = rd64(data);
            const uint8_t* op = page(ov);
            if (op + kPageHdr + dsz > base_ + size_) throw std::runtime_error("lmdb: overflow out of range");
            return op + kPageHdr;
          }
          return data;
        }
        if (c < 0) hi = mid - 1; else lo = mid + 1;
      }
      return nullptr;
    }
    throw std::runtime_error("lmdb: tree too deep / cyclic");
  }

 private:
  const uint8_t* page(uint64_t pg) const {
    const uint64_t off = pg * (uint64_t)psize_;
    if (off + psize_ > size_) throw std::runtime_error("lmdb: page out of range");
    return base_ + off;
  }
  static const uint8_t* node(const uint8_t* p, int i) { return p + lmdbfmt::rd16(p + lmdbfmt::kPageHdr + 2 * i); }

  int fd_ = -1;
  size_t size_ = 0;
  const uint8_t* base_ = nullptr;
  uint32_t psize_ = 4096;
  lmdbfmt::MetaRec meta_{};
  lmdbfmt::DbRec main_{};
};

// ----------------------------------------------------------------- writer
void lmdb_write(const std::string& path, std::vector<std::pair<std::string, std::string>> items,
                uint64_t map_size, uint32_t psize) {
  using namespace lmdbfmt;
  std::sort(items.begin(), items.end(), [](const auto& a, const auto& b) {
    return keycmp((const uint8_t*)a.first.data(), a.first.size(), (const uint8_t*)b.first.data(),
                  b.first.size()) < 0;
  });
  for (size_t i = 1; i < items.size(); ++i)
    if (items[i].first == items[i - 1].first) throw std::invalid_argument("lmdb_write: duplicate key");
  const size_t nodemax = (((psize - kPageHdr) / 2) & ~(size_t)1) - 2;
  std::vector<std::vector<uint8_t>> pages;  // page images, pages[i] is page number i
  auto new_page = [&](uint16_t flags) {
    pages.emplace_back(psize, 0);
    auto& pg = pages.back();
    const uint64_t no = pages.size() - 1;
    std::memcpy(pg.data(), &no, 8);
    std::memcpy(pg.data() + 10, &flags, 2);
    uint16_t lower = kPageHdr, upper = (uint16_t)psize;
    std::memcpy(pg.data() + 12, &lower, 2);
    std::memcpy(pg.data() + 14, &upper, 2);
    return no;
  };
  new_page(P_META);
  new_page(P_META);
  // try to place a node into page `no`; returns false if it does not fit
  auto place = [&](uint64_t no, const std::string& key, const uint8_t* data, size_t dlen, uint16_t nflags,
                   uint32_t dsz_field, uint64_t pgno_field, bool branch) -> bool {
    auto& pg = pages[no];
    uint16_t lower = rd16(pg.data() + 12), upper = rd16(pg.data() + 14);
    size_t nsz = kNodeHdr + key.size() + (branch ? 0 : dlen);
    nsz = (nsz + 1) & ~(size_t)1;
    if ((size_t)upper < nsz + lower + 2) return false;
    upper = (uint16_t)(upper - nsz);
    uint8_t* nd = pg.data() + upper;
    uint16_t lo, hi, fl;
    if (branch) {
      lo = (uint16_t)(pgno_field & 0xffff);
      hi = (uint16_t)((pgno_field >> 16) & 0xffff);
      fl = (uint16_t)((pgno_field >> 32) & 0xffff);
    } else {
      lo = (uint16_t)(dsz_field & 0xffff);
      hi = (uint16_t)(dsz_field >> 16);
      fl = nflags;
    }
    const uint16_t ks = (uint16_t)key.size();
    std::memcpy(nd, &lo, 2);
    std::memcpy(nd + 2, &hi, 2);
    std::memcpy(nd + 4, &fl, 2);
    std::memcpy(nd + 6, &ks, 2);
    std::memcpy(nd + kNodeHdr, key.data(), key.size());
    if (!branch && dlen) std::memcpy(nd + kNodeHdr + key.size(), data, dlen);
    std::memcpy(pg.data() + lower, &upper, 2);
    lower = (uint16_t)(lower + 2);
    std::memcpy(pg.data() + 12, &lower, 2);
    std::memcpy(pg.data() + 14, &upper, 2);
    return true;
  };
  uint64_t leaf_pages = 0, branch_pages = 0, overflow_pages = 0;
  // level 0: leaves
  std::vector<std::pair<std::string, uint64_t>> level;  // (first key, page)
  uint64_t cur = 0;
  bool have = false;
  for (auto& kv : items) {
    if (kv.first.size() > 511) throw std::invalid_argument("lmdb_write: key longer than 511 bytes");
    const std::string& v = kv.second;
    const bool big = kNodeHdr + kv.first.size() + v.size() > nodemax;
    uint64_t ovno = 0;
    if (big) {
      const size_t npg = (kPageHdr - 1 + v.size()) / psize + 1;
      ovno = new_page(P_OVERFLOW);
      for (size_t i = 1; i < npg; ++i) pages.emplace_back(psize, 0);
      const uint32_t np32 = (uint32_t)npg;
      std::memcpy(pages[ovno].data() + 12, &np32, 4);
      // copy value across the contiguous overflow run
      size_t off = 0, pi = ovno, poff = kPageHdr;
      while (off < v.size()) {
        const size_t n = std::min(v.size() - off, (size_t)psize - poff);
        std::memcpy(pages[pi].data() + poff, v.data() + off, n);
        off += n;
        ++pi;
        poff = 0;
      }
      overflow_pages += npg;
    }
    const uint8_t* dptr = big ? (const uint8_t*)&ovno : (const uint8_t*)v.data();
    const size_t dlen = big ? 8 : v.size();
    const uint16_t nfl = big ? F_BIGDATA : 0;
    if (!have || !place(cur, kv.first, dptr, dlen, nfl, (uint32_t)v.size(), 0, false)) {
      cur = new_page(P_LEAF);
      ++leaf_pages;
      have = true;
      level.emplace_back(kv.first, cur);
      if (!place(cur, kv.first, dptr, dlen, nfl, (uint32_t)v.size(), 0, false))
        throw std::runtime_error("lmdb_write: record does not fit a page");
    }
  }
  uint64_t root = P_INVALID;
  uint16_t depth = 0;
  if (!level.empty()) {
    depth = 1;
    while (level.size() > 1) {
      std::vector<std::pair<std::string, uint64_t>> up;
      bool open = false;
      uint64_t bp = 0;
      for (size_t i = 0; i < level.size(); ++i) {
        // the first node of every branch page carries an empty key
        const std::string key = (!open) ? std::string() : level[i].first;
        if (!open || !place(bp, key, nullptr, 0, 0, 0, level[i].second, true)) {
          bp = new_page(P_BRANCH);
          ++branch_pages;
          open = true;
          up.emplace_back(level[i].first, bp);
          place(bp, std::string(), nullptr, 0, 0, 0, level[i].second, true);
        }
      }
      level.swap(up);
      ++depth;
    }
    root = level[0].second;
  }
  const uint64_t last_pg = pages.size() - 1;
  for (int mi = 0; mi < 2; ++mi) {
    MetaRec m{};
    m.magic = kMagic;
    m.version = kVersion;
    m.address = 0;
    m.mapsize = std::max<uint64_t>(map_size, (uint64_t)pages.size() * psize);
    m.dbs[0].pad = psize;
    m.dbs[0].root = P_INVALID;
    m.dbs[1].depth = depth;
    m.dbs[1].branch_pages = branch_pages;
    m.dbs[1].leaf_pages = leaf_pages;
    m.dbs[1].overflow_pages = overflow_pages;
    m.dbs[1].entries = items.size();
    m.dbs[1].root = root;
    m.last_pg = last_pg;
    m.txnid = (uint64_t)(mi + 1);
    std::memcpy(pages[mi].data() + kPageHdr, &m, sizeof(m));
  }
  struct stat st;
  std::string file = path;
  if (::stat(path.c_str(), &st) == 0 && S_ISDIR(st.st_mode)) file = path + "/data.mdb";
  const std::string tmp = file + ".tmp";
  FILE* f = std::fopen(tmp.c_str(), "wb");
  if (!f) throw std::runtime_error("lmdb_write: cannot create " + tmp);
  for (auto& pg : pages)
    if (std::fwrite(pg.data(), 1, psize, f) != psize) {
      std::fclose(f);
      throw std::runtime_error("lmdb_write: short write");
    }
  std::fclose(f);
  if (std::rename(tmp.c_str(), file.c_str()) != 0) throw std::runtime_error("lmdb_write: rename failed");
}

}  // namespace tbamd

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
}

void register_prefetch(pybind11::module& m) {}
