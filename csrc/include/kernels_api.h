// Registration hook for the per-layer (generic path) HIP kernel ops.
#pragma once
#include <pybind11/pybind11.h>
void register_kernel_ops(pybind11::module_& m);
