// Reducer planning / readiness runtime (host C++, torch-free core).
//
// Reference: DDP's bucketed reducer used through EnvironementConfig.make ->
// to_env -> DistributedDataParallel (/root/reference/torchbooster/config.py:176-178);
// SURVEY.md §2.4 N5-N7 and §5.8 (design items a-d).  Unit-tested standalone
// with host ASan (tests/cpp/test_runtime.cpp).
#include "runtime.h"

#include <algorithm>
#include <cstdint>
#include <stdexcept>

namespace tbamd {

BucketPlan plan_buckets(const std::vector<int64_t>& numel, const std::vector<int64_t>& dtype,
                        const std::vector<int64_t>& elem_size, const std::vector<int64_t>& order,
                        int64_t cap_bytes, int64_t first_cap_bytes, int64_t align_elems,
                        int64_t tail_cap_bytes) {
  const size_t n = numel.size();
  if (dtype.size() != n || elem_size.size() != n || order.size() != n)
    throw std::invalid_argument("plan_buckets: size mismatch");
  if (align_elems < 1) align_elems = 1;
  if (first_cap_bytes < 1) first_cap_bytes = 1;
  if (cap_bytes < first_cap_bytes) cap_bytes = first_cap_bytes;
  std::vector<uint8_t> visited(n, 0);
  BucketPlan plan;
  plan.bucket_of.assign(n, -1);
  plan.part_of.assign(n, -1);
  plan.offset_of.assign(n, 0);
  // first index of the tail bucket (n: none)
  size_t tail = n;
  if (tail_cap_bytes > 0) {
    int64_t tb = 0;
    for (size_t k = n; k-- > 1;) {  // never the whole order: at least one regular bucket
      const int64_t p = order[k];
      if (p < 0 || (size_t)p >= n) break;  // reported by the main loop
      const int64_t b = numel[p] * elem_size[p];
      if (tb + b > tail_cap_bytes) break;
      tb += b;
      tail = k;
    }
  }
  int64_t cur = -1;       // open bucket
  int64_t cur_bytes = 0;  // its payload bytes
  for (size_t k = 0; k < n; ++k) {
    const int64_t p = order[k];
    if (p < 0 || (size_t)p >= n) throw std::invalid_argument("plan_buckets: bad order index");
    if (visited[p]) throw std::invalid_argument("plan_buckets: order repeats a param");
    visited[p] = 1;
    const int64_t bytes = numel[p] * elem_size[p];
    const int64_t target = cur <= 0 ? first_cap_bytes : cap_bytes;
    const bool close = cur >= 0 && ((cur_bytes >= first_cap_bytes && cur_bytes + bytes > target) || k == tail);
    if (cur < 0 || close) {
      cur = (int64_t)plan.bucket_parts.size();
      plan.bucket_parts.emplace_back();
      plan.bucket_params.emplace_back();
      plan.bucket_bytes.push_back(0);
      cur_bytes = 0;
    }
    int64_t part = -1;
    for (int64_t q : plan.bucket_parts[cur])
      if (plan.part_dtype[q] == dtype[p]) part = q;
    if (part < 0) {
      part = (int64_t)plan.part_numel.size();
      plan.part_numel.push_back(0);
      plan.part_dtype.push_back(dtype[p]);
      plan.part_bucket.push_back(cur);
      plan.bucket_parts[cur].push_back(part);
    }
    const int64_t off = (plan.part_numel[part] + align_elems - 1) / align_elems * align_elems;
    plan.bucket_of[p] = cur;
    plan.part_of[p] = part;
    plan.offset_of[p] = off;
    plan.part_numel[part] = off + numel[p];
    plan.bucket_params[cur].push_back(p);
    cur_bytes += bytes;
    plan.bucket_bytes[cur] = cur_bytes;
  }
  for (auto& m : plan.part_numel) m = (m + align_elems - 1) / align_elems * align_elems;
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
