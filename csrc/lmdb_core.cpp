// LMDB bulk writer (torch-free; see lmdb_core.h).
#include "lmdb_core.h"

namespace tbamd {

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
