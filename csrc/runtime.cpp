// Python bindings of the reducer runtime (csrc/runtime_core.cpp).
//
// Reference: DDP's bucketed reducer used through EnvironementConfig.make ->
// to_env -> DistributedDataParallel (/root/reference/torchbooster/config.py:176-178);
// SURVEY.md §2.4 N5-N7 and §5.8 (design items a-d).
#include "runtime.h"

#include <torch/extension.h>


void register_lmdb(pybind11::module& m);
void register_prefetch(pybind11::module& m);

void register_runtime(pybind11::module& m) {
  namespace py = pybind11;
  py::class_<tbamd::BucketPlan>(m, "BucketPlan")
      .def_readonly("bucket_of", &tbamd::BucketPlan::bucket_of)
      .def_readonly("part_of", &tbamd::BucketPlan::part_of)
      .def_readonly("offset_of", &tbamd::BucketPlan::offset_of)
      .def_readonly("part_numel", &tbamd::BucketPlan::part_numel)
      .def_readonly("part_dtype", &tbamd::BucketPlan::part_dtype)
      .def_readonly("part_bucket", &tbamd::BucketPlan::part_bucket)
      .def_readonly("bucket_parts", &tbamd::BucketPlan::bucket_parts)
      .def_readonly("bucket_params", &tbamd::BucketPlan::bucket_params)
      .def_readonly("bucket_bytes", &tbamd::BucketPlan::bucket_bytes);
  m.def("plan_buckets", &tbamd::plan_buckets, py::arg("numel"), py::arg("dtype"), py::arg("elem_size"),
        py::arg("order"), py::arg("cap_bytes"), py::arg("first_cap_bytes"), py::arg("align_elems") = 64,
        py::arg("tail_cap_bytes") = 0);
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
