// placeholder, replaced by the native LMDB reader
#include <torch/extension.h>
void register_lmdb(pybind11::module& m) {}
void register_prefetch(pybind11::module& m) {}
