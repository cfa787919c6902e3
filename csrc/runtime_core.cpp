// Reducer planning / readiness runtime (host C++, torch-free core).
//
// Reference: DDP's bucketed reducer used through EnvironementConfig.make ->
// to_env -> DistributedDataParallel (/root/reference/torchbooster/config.py:176-178);
// SURVEY.md §2.4 N5-N7 and §5.8 (design items a-d).  Unit-tested standalone
// with host ASan (tests/cpp/test_runtime.cpp).
#include "runtime.h"

#include <algorithm>
#include <stdexcept>

namespace tbamd {

BucketPlan plan_buckets(const std::vector<int64_t>& numel, const std::vector<int64_t>& dtype,
                        const std::vector<int64_t>& elem_size, const std::vector<int64_t>& order,
                        int64_t cap_bytes, int64_t first_cap_bytes, int64_t align_elems) {
  const size_t n = numel.size();
  if (dtype.size() != n || elem_size.size() != n || order.size() != n)
    throw std::invalid_argument("plan_buckets: size mismatch");
  if (align_elems < 1) align_elems = 1;
  // Pass 1: fill one open bucket per dtype, in `order`.  Mixed-dtype models
  // (bf16 conv weights + f32 norm params) thus get a few large buckets per
  // dtype instead of one bucket per dtype transition.
  std::vector<int64_t> bucket_of(n, -1), offset_of(n, 0);
  std::vector<int64_t> b_numel, b_dtype, b_last_pos, b_bytes;
  std::vector<std::pair<int64_t, int64_t>> open;  // (dtype, bucket)
  for (size_t k = 0; k < n; ++k) {
    const int64_t p = order[k];
    if (p < 0 || (size_t)p >= n) throw std::invalid_argument("plan_buckets: bad order index");
    int64_t cur = -1;
    for (auto& od : open)
      if (od.first == dtype[p]) cur = od.second;
    const int64_t bytes = numel[p] * elem_size[p];
    const int64_t cap = b_numel.empty() || cur == 0 ? first_cap_bytes : cap_bytes;
    if (cur < 0 || (b_bytes[cur] > 0 && b_bytes[cur] + bytes > cap)) {
      cur = (int64_t)b_numel.size();
      b_numel.push_back(0);
      b_dtype.push_back(dtype[p]);
      b_last_pos.push_back(0);
      b_bytes.push_back(0);
      bool found = false;
      for (auto& od : open)
        if (od.first == dtype[p]) { od.second = cur; found = true; }
      if (!found) open.emplace_back(dtype[p], cur);
    }
    int64_t off = (b_numel[cur] + align_elems - 1) / align_elems * align_elems;
    bucket_of[p] = cur;
    offset_of[p] = off;
    b_numel[cur] = off + numel[p];
    b_bytes[cur] = b_numel[cur] * elem_size[p];
    b_last_pos[cur] = (int64_t)k;
  }
  // Pass 2: number buckets by the position of their LAST param in `order`
  // (≈ when the bucket becomes ready), so in-order launching never makes an
  // early-ready bucket wait behind a late one.
  const size_t nb = b_numel.size();
  std::vector<int64_t> perm(nb);
  for (size_t i = 0; i < nb; ++i) perm[i] = (int64_t)i;
  std::sort(perm.begin(), perm.end(), [&](int64_t a, int64_t b) { return b_last_pos[a] < b_last_pos[b]; });
  std::vector<int64_t> rank(nb);
  for (size_t i = 0; i < nb; ++i) rank[perm[i]] = (int64_t)i;
  BucketPlan plan;
  plan.bucket_of.resize(n);
  plan.offset_of = offset_of;
  plan.bucket_numel.resize(nb);
  plan.bucket_dtype.resize(nb);
  plan.bucket_params.assign(nb, {});
  for (size_t i = 0; i < nb; ++i) {
    plan.bucket_numel[rank[i]] = (b_numel[i] + align_elems - 1) / align_elems * align_elems;
    plan.bucket_dtype[rank[i]] = b_dtype[i];
  }
  for (size_t k = 0; k < n; ++k) {
    const int64_t p = order[k];
    plan.bucket_of[p] = rank[bucket_of[p]];
    plan.bucket_params[rank[bucket_of[p]]].push_back(p);
  }
  return plan;
}

ReadyTracker::ReadyTracker(std::vector<int64_t> bucket_of, std::vector<int64_t> bucket_sizes)
    : bucket_of_(std::move(bucket_of)), sizes_(std::move(bucket_sizes)) {
  reset();
}

void ReadyTracker::reset() {
  pending_ = sizes_;
  seen_.assign(bucket_of_.size(), 0);
  next_launch_ = 0;
}

std::vector<int64_t> ReadyTracker::mark_ready(int64_t param) {
  std::vector<int64_t> out;
  if (param < 0 || (size_t)param >= bucket_of_.size()) throw std::out_of_range("mark_ready: bad param");
  if (seen_[param]) return out;  // a second hook in the same round is a no-op
  seen_[param] = 1;
  const int64_t b = bucket_of_[param];
  if (b < 0) return out;
  --pending_[b];
  while (next_launch_ < (int64_t)sizes_.size() && pending_[next_launch_] == 0) {
    out.push_back(next_launch_);
    ++next_launch_;
  }
  return out;
}

std::vector<int64_t> ReadyTracker::drain() {
  std::vector<int64_t> out;
  while (next_launch_ < (int64_t)sizes_.size()) out.push_back(next_launch_++);
  return out;
}

}  // namespace tbamd
