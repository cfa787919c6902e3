// LMDB writers (torch-free; see lmdb_core.h): a streaming loader that writes pages as they fill,
// and the in-memory bulk loader on top of it (sort, then stream).
#include "lmdb_core.h"

namespace tbamd {

namespace {
using namespace lmdbfmt;

// largest node that still goes on a leaf page (bigger values move to overflow pages)
size_t node_max(uint32_t psize) { return (((psize - kPageHdr) / 2) & ~(size_t)1) - 2; }

// Place a node into page image `pg`; false if it does not fit.  Leaf node: key + data (dlen bytes,
// dsz_field = the value size); branch node: key + child page number.
bool place(std::vector<uint8_t>& pg, const std::string& key, const uint8_t* data, size_t dlen, uint16_t nflags,
           uint32_t dsz_field, uint64_t pgno_field, bool branch) {
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
}
}  // namespace

LmdbStreamWriter::LmdbStreamWriter(const std::string& path, uint64_t map_size, uint32_t psize)
    : map_size_(map_size), psize_(psize) {
  struct stat st;
  file_ = path;
  if (::stat(path.c_str(), &st) == 0 && S_ISDIR(st.st_mode)) file_ = path + "/data.mdb";
  tmp_ = file_ + ".tmp";
  f_ = std::fopen(tmp_.c_str(), "w+b");
  if (!f_) throw std::runtime_error("lmdb_write: cannot create " + tmp_);
}

LmdbStreamWriter::~LmdbStreamWriter() {
  if (f_) {
    std::fclose(f_);
    std::remove(tmp_.c_str());
  }
}

std::vector<uint8_t> LmdbStreamWriter::blank(uint64_t no, uint16_t flags) const {
  std::vector<uint8_t> pg(psize_, 0);
  std::memcpy(pg.data(), &no, 8);
  std::memcpy(pg.data() + 10, &flags, 2);
  const uint16_t lower = kPageHdr, upper = (uint16_t)psize_;
  std::memcpy(pg.data() + 12, &lower, 2);
  std::memcpy(pg.data() + 14, &upper, 2);
  return pg;
}

void LmdbStreamWriter::write_page(uint64_t no, const uint8_t* data, size_t npages) {
  if (::fseeko(f_, (off_t)(no * psize_), SEEK_SET) != 0 ||
      std::fwrite(data, 1, npages * psize_, f_) != npages * psize_)
    throw std::runtime_error("lmdb_write: short write");
}

void LmdbStreamWriter::add(const std::string& key, const std::string& v) {
  if (!f_) throw std::runtime_error("lmdb_write: writer is closed");
  if (key.size() > 511) throw std::invalid_argument("lmdb_write: key longer than 511 bytes");
  if (have_key_) {
    const int c = keycmp((const uint8_t*)key.data(), key.size(), (const uint8_t*)last_key_.data(), last_key_.size());
    if (c == 0) throw std::invalid_argument("lmdb_write: duplicate key");
    if (c < 0) throw std::invalid_argument("lmdb_write: keys must arrive in increasing order");
  }
  last_key_ = key;
  have_key_ = true;
  const bool big = kNodeHdr + key.size() + v.size() > node_max(psize_);
  uint64_t ovno = 0;
  if (big) {  // contiguous overflow run, written now
    const size_t npg = (kPageHdr - 1 + v.size()) / psize_ + 1;
    ovno = next_pg_;
    next_pg_ += npg;
    std::vector<uint8_t> run((size_t)npg * psize_, 0);
    std::memcpy(run.data(), &ovno, 8);
    const uint16_t fl = P_OVERFLOW;
    std::memcpy(run.data() + 10, &fl, 2);
    const uint32_t np32 = (uint32_t)npg;
    std::memcpy(run.data() + 12, &np32, 4);
    std::memcpy(run.data() + kPageHdr, v.data(), v.size());
    write_page(ovno, run.data(), npg);
    overflow_pages_ += npg;
  }
  const uint8_t* dptr = big ? (const uint8_t*)&ovno : (const uint8_t*)v.data();
  const size_t dlen = big ? 8 : v.size();
  const uint16_t nfl = big ? F_BIGDATA : 0;
  if (!have_leaf_ || !place(leaf_, key, dptr, dlen, nfl, (uint32_t)v.size(), 0, false)) {
    if (have_leaf_) write_page(leaf_no_, leaf_.data(), 1);
    leaf_no_ = next_pg_++;
    leaf_ = blank(leaf_no_, P_LEAF);
    ++leaf_pages_;
    have_leaf_ = true;
    level_.emplace_back(key, leaf_no_);
    if (!place(leaf_, key, dptr, dlen, nfl, (uint32_t)v.size(), 0, false))
      throw std::runtime_error("lmdb_write: record does not fit a page");
  }
  ++entries_;
}

uint64_t LmdbStreamWriter::close() {
  if (!f_) throw std::runtime_error("lmdb_write: writer is closed");
  if (have_leaf_) write_page(leaf_no_, leaf_.data(), 1);
  uint64_t root = P_INVALID, branch_pages = 0;
  uint16_t depth = 0;
  std::vector<std::pair<std::string, uint64_t>> level = level_;
  if (!level.empty()) {
    depth = 1;
    while (level.size() > 1) {
      std::vector<std::pair<std::string, uint64_t>> up;
      std::vector<uint8_t> bp;
      uint64_t bno = 0;
      bool open = false;
      for (size_t i = 0; i < level.size(); ++i) {
        // the first node of every branch page carries an empty key
        if (!open || !place(bp, level[i].first, nullptr, 0, 0, 0, level[i].second, true)) {
          if (open) write_page(bno, bp.data(), 1);
          bno = next_pg_++;
          bp = blank(bno, P_BRANCH);
          ++branch_pages;
          open = true;
          up.emplace_back(level[i].first, bno);
          place(bp, std::string(), nullptr, 0, 0, 0, level[i].second, true);
        }
      }
      if (open) write_page(bno, bp.data(), 1);
      level.swap(up);
      ++depth;
    }
    root = level[0].second;
  }
  const uint64_t last_pg = next_pg_ - 1;
  for (int mi = 0; mi < 2; ++mi) {
    std::vector<uint8_t> pg = blank((uint64_t)mi, P_META);
    MetaRec m{};
    m.magic = kMagic;
    m.version = kVersion;
    m.address = 0;
    m.mapsize = std::max<uint64_t>(map_size_, next_pg_ * psize_);
    m.dbs[0].pad = psize_;
    m.dbs[0].root = P_INVALID;
    m.dbs[1].depth = depth;
    m.dbs[1].branch_pages = branch_pages;
    m.dbs[1].leaf_pages = leaf_pages_;
    m.dbs[1].overflow_pages = overflow_pages_;
    m.dbs[1].entries = entries_;
    m.dbs[1].root = root;
    m.last_pg = last_pg;
    m.txnid = (uint64_t)(mi + 1);
    std::memcpy(pg.data() + kPageHdr, &m, sizeof(m));
    write_page((uint64_t)mi, pg.data(), 1);
  }
  const bool ok = std::fflush(f_) == 0;
  std::fclose(f_);
  f_ = nullptr;
  if (!ok) {
    std::remove(tmp_.c_str());
    throw std::runtime_error("lmdb_write: flush failed");
  }
  if (std::rename(tmp_.c_str(), file_.c_str()) != 0) throw std::runtime_error("lmdb_write: rename failed");
  return entries_;
}

void lmdb_write(const std::string& path, std::vector<std::pair<std::string, std::string>> items,
                uint64_t map_size, uint32_t psize) {
  std::sort(items.begin(), items.end(), [](const auto& a, const auto& b) {
    return keycmp((const uint8_t*)a.first.data(), a.first.size(), (const uint8_t*)b.first.data(),
                  b.first.size()) < 0;
  });
  LmdbStreamWriter w(path, map_size, psize);
  for (auto& kv : items) w.add(kv.first, kv.second);
  w.close();
}

}  // namespace tbamd
