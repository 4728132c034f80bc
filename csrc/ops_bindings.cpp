// Per-layer HIP kernel ops (generic Keras path).  Pointers in, pointers out; shapes are
// validated on the Python side (distributed_amd/ops/) before any launch.
#include <pybind11/pybind11.h>

#include "kernels_api.h"

namespace py = pybind11;

void register_kernel_ops(py::module_& m) {
  (void)m;
}
