// Native host-side runtime of torcheval_amd (C++): text-metric kernels that the reference
// runs as pure-Python loops (edit distance DP, n-gram counters).  Registered into the same
// extension module as the HIP ops.
#pragma once

#include <pybind11/pybind11.h>

void tea_register_runtime(pybind11::module_& m);
void tea_register_cpu_metrics(pybind11::module_& m);
void tea_register_rccl(pybind11::module_& m);  // csrc/runtime/rccl_direct.cpp
void tea_register_hostread(pybind11::module_& m);  // csrc/runtime/hostread.cpp
