// Standalone unit tests of the torch-free host runtime (bucket planner, ready
// tracker, LMDB writer/reader).  Built and run by tests/test_native_host.py,
// with AddressSanitizer + UBSan on the host code:
//   g++ -std=c++17 -O1 -g -fsanitize=address,undefined -Icsrc tests/cpp/test_runtime.cpp
//       csrc/runtime_core.cpp csrc/lmdb_core.cpp -o /tmp/test_runtime
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <unistd.h>

#include "lmdb_core.h"
#include "runtime.h"

static int g_fail = 0;
#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      std::fprintf(stderr, "%s:%d CHECK failed: %s\n", __FILE__, __LINE__, #c); \
      ++g_fail;                                                         \
    }                                                                   \
  } while (0)

static void test_plan_buckets() {
  // 6 params registered 0..5, visited in reverse (backward order)
  std::vector<int64_t> numel{1000, 10, 300000, 7, 500000, 3};
  std::vector<int64_t> dtype{1, 0, 1, 0, 1, 1};  // mixed bf16 / f32
  std::vector<int64_t> esz{2, 4, 2, 4, 2, 2};
  std::vector<int64_t> order{5, 4, 3, 2, 1, 0};
  auto plan = tbamd::plan_buckets(numel, dtype, esz, order, 1 << 20, 1 << 10, 64);
  CHECK(plan.bucket_of.size() == 6 && plan.part_of.size() == 6);
  // every param in exactly one part of its bucket, offsets 64-aligned, parts single-dtype
  for (size_t i = 0; i < 6; ++i) {
    const int64_t b = plan.bucket_of[i], q = plan.part_of[i];
    CHECK(b >= 0 && b < (int64_t)plan.bucket_parts.size());
    CHECK(q >= 0 && q < (int64_t)plan.part_numel.size());
    CHECK(plan.part_bucket[q] == b);
    CHECK(plan.offset_of[i] % 64 == 0);
    CHECK(plan.offset_of[i] + numel[i] <= plan.part_numel[q]);
    CHECK(plan.part_dtype[q] == dtype[i]);
  }
  // params sharing a part never overlap
  for (size_t i = 0; i < 6; ++i)
    for (size_t j = i + 1; j < 6; ++j)
      if (plan.part_of[i] == plan.part_of[j])
        CHECK(plan.offset_of[i] + numel[i] <= plan.offset_of[j] || plan.offset_of[j] + numel[j] <= plan.offset_of[i]);
  // buckets are contiguous runs of `order`, numbered in order
  int64_t last = 0;
  for (size_t k = 0; k < 6; ++k) {
    CHECK(plan.bucket_of[order[k]] >= last);
    last = plan.bucket_of[order[k]];
  }
  // the f32 param 3 (between bf16 params 4 and 2) shares a bucket with a bf16 neighbour
  CHECK(plan.bucket_of[3] == plan.bucket_of[4] || plan.bucket_of[3] == plan.bucket_of[2]);
  // no bucket is closed below first_cap: bucket 0 = {5 (6 B), 4 (1 MB)} rather than {5} alone
  CHECK(plan.bucket_of[5] == plan.bucket_of[4]);
  bool threw = false;
  try {
    tbamd::plan_buckets({1, 2}, {0}, {4, 4}, {0, 1}, 1024, 1024, 64);
  } catch (const std::invalid_argument&) {
    threw = true;
  }
  CHECK(threw);
  threw = false;
  try {
    tbamd::plan_buckets({1, 2}, {0, 0}, {4, 4}, {0, 0}, 1024, 1024, 64);
  } catch (const std::invalid_argument&) {
    threw = true;
  }
  CHECK(threw);
}

static void test_ready_tracker() {
  // 5 params in 3 buckets; buckets must be released strictly in order
  tbamd::ReadyTracker t({0, 0, 1, 2, 2}, {2, 1, 2});
  CHECK(t.mark_ready(3).empty());  // bucket 2 half ready, bucket 0 not yet
  CHECK(t.mark_ready(2).empty());  // bucket 1 complete but 0 is not
  auto r = t.mark_ready(0);
  CHECK(r.empty());
  r = t.mark_ready(1);  // bucket 0 complete -> releases 0 and 1
  CHECK(r.size() == 2 && r[0] == 0 && r[1] == 1);
  CHECK(t.mark_ready(1).empty());  // duplicate hook is a no-op
  r = t.mark_ready(4);
  CHECK(r.size() == 1 && r[0] == 2);
  CHECK(t.drain().empty());
  t.reset();
  CHECK(!t.param_seen(0));
  t.mark_ready(4);
  r = t.drain();  // finalize: everything left, in order
  CHECK(r.size() == 3 && r[0] == 0 && r[2] == 2);
  bool threw = false;
  try {
    t.mark_ready(99);
  } catch (const std::out_of_range&) {
    threw = true;
  }
  CHECK(threw);
}

static void test_lmdb_roundtrip() {
  char tmpl[] = "/tmp/tbamd_lmdb_XXXXXX";
  const char* dir = mkdtemp(tmpl);
  CHECK(dir != nullptr);
  if (!dir) return;
  std::mt19937 rng(3);
  std::vector<std::pair<std::string, std::string>> items;
  const int n = 3000;
  for (int i = 0; i < n; ++i) {
    // values of mixed size: small (inline leaf nodes) and > page (overflow pages)
    const size_t len = (i % 97 == 0) ? 9000 + (rng() % 5000) : 1 + (rng() % 300);
    std::string v(len, '\0');
    for (auto& c : v) c = (char)(rng() & 0xff);
    items.emplace_back(std::to_string(i), std::move(v));
  }
  items.emplace_back("length", std::to_string(n));
  auto copy = items;
  tbamd::lmdb_write(dir, std::move(copy), 1ull << 30, 4096);
  const std::string dpath(dir);
  tbamd::LmdbEnv env{dpath};
  CHECK(env.entries() == (uint64_t)items.size());
  for (const auto& kv : items) {
    size_t vl = 0;
    const uint8_t* v = env.find((const uint8_t*)kv.first.data(), kv.first.size(), &vl);
    CHECK(v != nullptr && vl == kv.second.size() && std::memcmp(v, kv.second.data(), vl) == 0);
  }
  size_t vl = 0;
  CHECK(env.find((const uint8_t*)"nope", 4, &vl) == nullptr);
  env.close();
  std::remove((std::string(dir) + "/data.mdb").c_str());
  rmdir(dir);
}

// streaming writer: keys in order, values large enough to need overflow runs, out-of-order keys
// rejected, and an unclosed writer leaves no file behind
static void test_lmdb_stream() {
  char tmpl[] = "/tmp/tbamd_lmdbs_XXXXXX";
  const char* dir = mkdtemp(tmpl);
  CHECK(dir != nullptr);
  if (!dir) return;
  const std::string dpath(dir);
  std::vector<std::string> keys;
  for (int i = 0; i < 700; ++i) keys.push_back(std::to_string(i));
  std::sort(keys.begin(), keys.end());
  std::mt19937 rng(5);
  std::vector<std::string> vals;
  {
    tbamd::LmdbStreamWriter w(dpath, 1ull << 30, 4096);
    for (auto& k : keys) {
      std::string v(3 * 64 * 64 + 8, '\0');  // a packed 64x64 RGB record
      for (auto& c : v) c = (char)(rng() & 0xff);
      w.add(k, v);
      vals.push_back(std::move(v));
    }
    bool threw = false;
    try {
      w.add("0", "x");  // before the last key
    } catch (const std::invalid_argument&) {
      threw = true;
    }
    CHECK(threw);
    w.add("length", "700");
    CHECK(w.close() == 701);
  }
  tbamd::LmdbEnv env{dpath};
  CHECK(env.entries() == 701);
  for (size_t i = 0; i < keys.size(); ++i) {
    size_t vl = 0;
    const uint8_t* v = env.find((const uint8_t*)keys[i].data(), keys[i].size(), &vl);
    CHECK(v != nullptr && vl == vals[i].size() && std::memcmp(v, vals[i].data(), vl) == 0);
  }
  env.close();
  std::remove((dpath + "/data.mdb").c_str());
  {
    tbamd::LmdbStreamWriter w(dpath, 1ull << 30, 4096);
    w.add("a", "b");
  }  // destroyed unclosed
  struct stat st;
  CHECK(::stat((dpath + "/data.mdb.tmp").c_str(), &st) != 0);
  CHECK(::stat((dpath + "/data.mdb").c_str(), &st) != 0);
  rmdir(dir);
}

int main() {
  test_plan_buckets();
  test_ready_tracker();
  test_lmdb_roundtrip();
  test_lmdb_stream();
  if (g_fail) {
    std::fprintf(stderr, "%d check(s) failed\n", g_fail);
    return 1;
  }
  std::printf("test_runtime: all checks passed\n");
  return 0;
}
