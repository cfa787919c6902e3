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
//
// Torch-free core (unit-tested standalone with host ASan: tests/cpp/test_runtime.cpp).
#pragma once

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <utility>
#include <vector>

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
// Streaming bulk loader: (key, value) pairs arrive in strictly increasing key order and leave for
// the file as soon as their page is full (leaf and overflow pages are written in place, only the
// (first key, page) list of the leaves stays in memory), so a dataset far larger than host RAM
// can be packed (data/readers.py pack_folder).  close() builds the branch levels, writes the two
// meta pages and renames <file>.tmp to the file (atomic); a writer destroyed unclosed removes its
// temporary file.
class LmdbStreamWriter {
 public:
  LmdbStreamWriter(const std::string& path, uint64_t map_size = (uint64_t)1 << 30, uint32_t psize = 4096);
  ~LmdbStreamWriter();
  LmdbStreamWriter(const LmdbStreamWriter&) = delete;
  LmdbStreamWriter& operator=(const LmdbStreamWriter&) = delete;
  void add(const std::string& key, const std::string& value);
  uint64_t close();  // number of records written
  uint64_t entries() const { return entries_; }

 private:
  void write_page(uint64_t no, const uint8_t* data, size_t npages);
  std::vector<uint8_t> blank(uint64_t no, uint16_t flags) const;
  FILE* f_ = nullptr;
  std::string file_, tmp_;
  uint64_t map_size_;
  uint32_t psize_;
  uint64_t next_pg_ = 2, entries_ = 0, leaf_pages_ = 0, overflow_pages_ = 0;
  std::vector<uint8_t> leaf_;
  uint64_t leaf_no_ = 0;
  bool have_leaf_ = false, have_key_ = false;
  std::string last_key_;
  std::vector<std::pair<std::string, uint64_t>> level_;  // (first key, page) of every leaf
};

// Bulk-load sorted or unsorted (key, value) pairs into a fresh LMDB file
// (atomic: written to <file>.tmp then renamed).
void lmdb_write(const std::string& path, std::vector<std::pair<std::string, std::string>> items,
                uint64_t map_size, uint32_t psize);

}  // namespace tbamd
