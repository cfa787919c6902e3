// Host-side C++ runtime pieces of torchbooster_amd (no device code):
//   * gradient bucket planning for the xGMI-aware reducer,
//   * the per-backward readiness tracker that releases buckets strictly in
//     order (every rank must issue its RCCL collectives in the same order),
//   * the read-only LMDB reader (lmdb_reader.cpp).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace tbamd {

// A bucket is a contiguous run of params in gradient-ready order; it holds one
// flat "part" buffer per dtype present in that run (bf16 conv weights and the
// f32 norm affine params of the SAME layers share a bucket and are reduced
// together, as one grouped collective per bucket).
struct BucketPlan {
  // per parameter
  std::vector<int64_t> bucket_of;
  std::vector<int64_t> part_of;    // flat buffer holding the param's gradient
  std::vector<int64_t> offset_of;  // element offset inside that part
  // per part
  std::vector<int64_t> part_numel;
  std::vector<int64_t> part_dtype;
  std::vector<int64_t> part_bucket;
  // per bucket
  std::vector<std::vector<int64_t>> bucket_parts;
  std::vector<std::vector<int64_t>> bucket_params;
  std::vector<int64_t> bucket_bytes;
};

// Params are visited in `order` (typically reverse registration order, which
// approximates gradient-ready order).  A bucket grows until adding the next
// param would take it past its target (first bucket: first_cap_bytes, then
// cap_bytes); a bucket is never closed while it holds less than
// first_cap_bytes, so no collective is issued for a few KiB (the classifier
// bias alone used to be a 2 KiB first bucket).  Offsets are aligned to
// `align_elems` so every gradient view is 16-B aligned.
// tail_cap_bytes > 0: the params at the END of `order` (the first layers of the model, whose
// gradients are the last ones ready) whose bytes sum to at most tail_cap_bytes form a bucket of
// their own, so the collective left exposed after the final weight gradient is that small one
// (ResNet-50: stem + layer1, < 1 MiB) instead of the tail of a 16 MiB bucket.
BucketPlan plan_buckets(const std::vector<int64_t>& numel, const std::vector<int64_t>& dtype,
                        const std::vector<int64_t>& elem_size, const std::vector<int64_t>& order,
                        int64_t cap_bytes, int64_t first_cap_bytes, int64_t align_elems,
                        int64_t tail_cap_bytes = 0);

class ReadyTracker {
 public:
  ReadyTracker() = default;
  ReadyTracker(std::vector<int64_t> bucket_of, std::vector<int64_t> bucket_sizes);
  // Marks a param ready; returns the buckets that may be launched now, in
  // order (a bucket is launched only once all earlier buckets launched).
  std::vector<int64_t> mark_ready(int64_t param);
  // Buckets not yet launched this round, in order (finalize path).
  std::vector<int64_t> drain();
  void reset();
  int64_t launched() const { return next_launch_; }
  int64_t num_buckets() const { return (int64_t)sizes_.size(); }
  bool param_seen(int64_t p) const { return seen_[p] != 0; }

 private:
  std::vector<int64_t> bucket_of_;
  std::vector<int64_t> sizes_;
  std::vector<int64_t> pending_;
  std::vector<uint8_t> seen_;
  int64_t next_launch_ = 0;
};

}  // namespace tbamd
