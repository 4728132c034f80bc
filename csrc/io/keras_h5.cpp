// Python binding of the HDF5 tree I/O (module distributed_amd._h5).
//
// Reference: the Spark workers call `save_model_hdf5(model, "trained-<p>.hdf5")` and the
// chief ships the file back base64-encoded (reference README.md:234-247); upstream Keras
// writes it with h5py.  h5py is not available here, so the file is written natively
// (csrc/io/h5tree.cpp).  Python (distributed_amd/keras/saving.py) builds the Keras
// 2.2.4-tf layout as a tree
//   {"attrs": {name: value}, "groups": {name: tree}, "datasets": {name: ndarray}}
// which this file converts to / from damd::h5::Group: str/bytes -> fixed-length
// NULLPAD string attributes (what h5py stores for numpy 'S' values), lists of str ->
// 1-D string attributes, numbers / arrays -> native numeric attributes and datasets.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "h5tree.h"

namespace py = pybind11;
using damd::h5::Array;
using damd::h5::Attr;
using damd::h5::DType;
using damd::h5::Group;

namespace {

DType to_dtype(const py::dtype& dt) {
  const char k = dt.kind();
  const size_t sz = dt.itemsize();
  if (k == 'f' && sz == 4) return DType::F32;
  if (k == 'f' && sz == 8) return DType::F64;
  if (k == 'i' && sz == 8) return DType::I64;
  if (k == 'i' && sz == 4) return DType::I32;
  if ((k == 'u' || k == 'b') && sz == 1) return DType::U8;
  throw std::invalid_argument("unsupported numpy dtype for HDF5: " + std::string(py::str(dt)));
}

py::dtype to_numpy(DType t) {
  switch (t) {
    case DType::F32: return py::dtype("float32");
    case DType::F64: return py::dtype("float64");
    case DType::I32: return py::dtype("int32");
    case DType::I64: return py::dtype("int64");
    case DType::U8: return py::dtype("uint8");
  }
  throw std::invalid_argument("dtype");
}

std::string to_bytes(const py::handle& h) {
  if (py::isinstance<py::bytes>(h)) return std::string(py::reinterpret_borrow<py::bytes>(h));
  return py::str(h).cast<std::string>();
}

Array to_array(const py::handle& v) {
  py::array arr = py::array::ensure(v, py::array::c_style | py::array::forcecast);
  if (!arr) throw std::invalid_argument("value is not array-like");
  Array out;
  out.dtype = to_dtype(arr.dtype());
  out.shape.assign(arr.shape(), arr.shape() + arr.ndim());
  out.bytes.resize(arr.nbytes());
  if (arr.nbytes()) std::memcpy(out.bytes.data(), arr.data(), arr.nbytes());
  return out;
}

py::array from_array(const Array& a) {
  py::array arr(to_numpy(a.dtype), std::vector<ssize_t>(a.shape.begin(), a.shape.end()));
  if (!a.bytes.empty()) std::memcpy(arr.mutable_data(), a.bytes.data(), a.bytes.size());
  return arr;
}

Attr to_attr(const py::handle& v) {
  Attr a;
  if (py::isinstance<py::str>(v) || py::isinstance<py::bytes>(v)) {
    a.kind = Attr::Str;
    a.s = to_bytes(v);
  } else if (py::isinstance<py::list>(v) || py::isinstance<py::tuple>(v)) {
    a.kind = Attr::StrList;
    for (auto it : v) a.list.push_back(to_bytes(it));
  } else {
    a.kind = Attr::Num;
    a.num = to_array(v);
  }
  return a;
}

Group to_group(const py::dict& tree) {
  Group g;
  if (tree.contains("attrs"))
    for (auto kv : tree["attrs"].cast<py::dict>()) g.attrs.emplace_back(kv.first.cast<std::string>(), to_attr(kv.second));
  if (tree.contains("datasets"))
    for (auto kv : tree["datasets"].cast<py::dict>())
      g.datasets.emplace_back(kv.first.cast<std::string>(), to_array(kv.second));
  if (tree.contains("groups"))
    for (auto kv : tree["groups"].cast<py::dict>())
      g.groups.emplace_back(kv.first.cast<std::string>(), to_group(kv.second.cast<py::dict>()));
  return g;
}

py::dict from_group(const Group& g) {
  py::dict tree, attrs, groups, datasets;
  for (auto& kv : g.attrs) {
    const Attr& a = kv.second;
    if (a.kind == Attr::Str) {
      attrs[py::str(kv.first)] = py::str(a.s);
    } else if (a.kind == Attr::StrList) {
      py::list l;
      for (auto& s : a.list) l.append(py::str(s));
      attrs[py::str(kv.first)] = l;
    } else {
      attrs[py::str(kv.first)] = from_array(a.num);
    }
  }
  for (auto& kv : g.groups) groups[py::str(kv.first)] = from_group(kv.second);
  for (auto& kv : g.datasets) datasets[py::str(kv.first)] = from_array(kv.second);
  tree["attrs"] = attrs;
  tree["groups"] = groups;
  tree["datasets"] = datasets;
  return tree;
}

}  // namespace

PYBIND11_MODULE(_h5, m) {
  m.doc() = "HDF5 tree I/O (libhdf5 C API) for Keras-layout model files";
  m.def("version", &damd::h5::library_version);
  m.def("write", [](const std::string& path, py::dict tree) { damd::h5::write_file(path, to_group(tree)); },
        py::arg("path"), py::arg("tree"));
  m.def("read", [](const std::string& path) { return from_group(damd::h5::read_file(path)); }, py::arg("path"));
}
