// Reducer planning / readiness runtime (host C++), exposed to Python.
//
// Reference: DDP's bucketed reducer used through EnvironementConfig.make ->
// to_env -> DistributedDataParallel (/root/reference/torchbooster/config.py:176-178);
// SURVEY.md §2.4 N5-N7 and §5.8 (design items a-d).
#include "runtime.h"

#include <torch/extension.h>

#include <stdexcept>

namespace tbamd {

BucketPlan plan_buckets(const std::vector<int64_t>& numel, const std::vector<int64_t>& dtype,
                        const std::vector<int64_t>& elem_size, const std::vector<int64_t>& order,
                        int64_t cap_bytes, int64_t first_cap_bytes, int64_t align_elems) {
  const size_t n = numel.size();
  if (dtype.size() != n || elem_size.size() != n || order.size() != n)
    throw std::invalid_argument("plan_buckets: size mismatch");
  if (align_elems < 1) align_elems = 1;
  BucketPlan plan;
  plan.bucket_of.assign(n, -1);
  plan.offset_of.assign(n, 0);
  int64_t cur = -1, cur_bytes = 0, cur_dtype = -1;
  for (size_t k = 0; k < n; ++k) {
    const int64_t p = order[k];
    if (p < 0 || (size_t)p >= n) throw std::invalid_argument("plan_buckets: bad order index");
    const int64_t cap = cur == 0 ? first_cap_bytes : cap_bytes;
    const int64_t bytes = numel[p] * elem_size[p];
    const bool need_new = cur < 0 || dtype[p] != cur_dtype || (cur_bytes > 0 && cur_bytes + bytes > cap);
    if (need_new) {
      cur = (int64_t)plan.bucket_numel.size();
      plan.bucket_numel.push_back(0);
      plan.bucket_dtype.push_back(dtype[p]);
      plan.bucket_params.emplace_back();
      cur_bytes = 0;
      cur_dtype = dtype[p];
    }
    int64_t off = plan.bucket_numel[cur];
    off = (off + align_elems - 1) / align_elems * align_elems;
    plan.bucket_of[p] = cur;
    plan.offset_of[p] = off;
    plan.bucket_numel[cur] = off + numel[p];
    plan.bucket_params[cur].push_back(p);
    cur_bytes = plan.bucket_numel[cur] * elem_size[p];
  }
  // round every bucket up to the alignment as well
  for (auto& b : plan.bucket_numel) b = (b + align_elems - 1) / align_elems * align_elems;
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

void register_lmdb(pybind11::module& m);
void register_prefetch(pybind11::module& m);

void register_runtime(pybind11::module& m) {
  namespace py = pybind11;
  py::class_<tbamd::BucketPlan>(m, "BucketPlan")
      .def_readonly("bucket_of", &tbamd::BucketPlan::bucket_of)
      .def_readonly("offset_of", &tbamd::BucketPlan::offset_of)
      .def_readonly("bucket_numel", &tbamd::BucketPlan::bucket_numel)
      .def_readonly("bucket_dtype", &tbamd::BucketPlan::bucket_dtype)
      .def_readonly("bucket_params", &tbamd::BucketPlan::bucket_params);
  m.def("plan_buckets", &tbamd::plan_buckets, py::arg("numel"), py::arg("dtype"), py::arg("elem_size"),
        py::arg("order"), py::arg("cap_bytes"), py::arg("first_cap_bytes"), py::arg("align_elems") = 64);
  py::class_<tbamd::ReadyTracker>(m, "ReadyTracker")
      .def(py::init<std::vector<int64_t>, std::vector<int64_t>>())
      .def("mark_ready", &tbamd::ReadyTracker::mark_ready)
      .def("drain", &tbamd::ReadyTracker::drain)
      .def("reset", &tbamd::ReadyTracker::reset)
      .def("param_seen", &tbamd::ReadyTracker::param_seen)
      .def_property_readonly("launched", &tbamd::ReadyTracker::launched)
      .def_property_readonly("num_buckets", &tbamd::ReadyTracker::num_buckets);
  register_lmdb(m);
  register_prefetch(m);
}
