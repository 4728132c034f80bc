// HDF5 tree reader/writer over the libhdf5 C API (module distributed_amd._h5).
//
// Reference: the Spark workers call `save_model_hdf5(model, "trained-<p>.hdf5")` and the
// chief ships the file back base64-encoded (reference README.md:234-247); upstream Keras
// writes it with h5py.  h5py is not available here, so this module writes/reads the
// same on-disk structure natively.  It is layout-agnostic: Python
// (distributed_amd/keras/saving.py) builds the Keras 2.2.4-tf layout as a tree
//   {"attrs": {name: value}, "groups": {name: tree}, "datasets": {name: ndarray}}
// with h5py-compatible encodings: str/bytes attributes -> fixed-length NULLPAD strings
// (what h5py stores for numpy 'S' values, e.g. `layer_names`, `weight_names`,
// `model_config`), numeric attributes/datasets -> native little-endian types.
#include <hdf5.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <stdexcept>
#include <string>
#include <vector>

namespace py = pybind11;

namespace {

struct H5Id {  // RAII for hid_t with a close function
  hid_t id;
  herr_t (*close)(hid_t);
  H5Id(hid_t i, herr_t (*c)(hid_t)) : id(i), close(c) {
    if (id < 0) throw std::runtime_error("HDF5 call failed");
  }
  ~H5Id() {
    if (id >= 0) close(id);
  }
  operator hid_t() const { return id; }
};

hid_t numpy_to_h5(const py::dtype& dt) {
  const char k = dt.kind();
  const size_t sz = dt.itemsize();
  if (k == 'f' && sz == 4) return H5T_NATIVE_FLOAT;
  if (k == 'f' && sz == 8) return H5T_NATIVE_DOUBLE;
  if (k == 'i' && sz == 8) return H5T_NATIVE_INT64;
  if (k == 'i' && sz == 4) return H5T_NATIVE_INT32;
  if (k == 'u' && sz == 1) return H5T_NATIVE_UINT8;
  if (k == 'b' && sz == 1) return H5T_NATIVE_UINT8;
  throw std::invalid_argument("unsupported numpy dtype for HDF5: " + std::string(py::str(dt)));
}

hid_t fixed_string_type(size_t n) {
  hid_t t = H5Tcopy(H5T_C_S1);
  H5Tset_size(t, n == 0 ? 1 : n);
  H5Tset_strpad(t, H5T_STR_NULLPAD);
  H5Tset_cset(t, H5T_CSET_ASCII);
  return t;
}

std::string to_bytes(const py::handle& h) {
  if (py::isinstance<py::bytes>(h)) return std::string(py::reinterpret_borrow<py::bytes>(h));
  return py::str(h).cast<std::string>();
}

void write_attr(hid_t obj, const std::string& name, const py::handle& v) {
  if (H5Aexists(obj, name.c_str()) > 0) H5Adelete(obj, name.c_str());
  if (py::isinstance<py::str>(v) || py::isinstance<py::bytes>(v)) {
    const std::string s = to_bytes(v);
    H5Id t(fixed_string_type(s.size()), H5Tclose);
    H5Id sp(H5Screate(H5S_SCALAR), H5Sclose);
    H5Id a(H5Acreate2(obj, name.c_str(), t, sp, H5P_DEFAULT, H5P_DEFAULT), H5Aclose);
    std::vector<char> buf(s.size() == 0 ? 1 : s.size(), 0);
    std::copy(s.begin(), s.end(), buf.begin());
    if (H5Awrite(a, t, buf.data()) < 0) throw std::runtime_error("H5Awrite failed for " + name);
    return;
  }
  if (py::isinstance<py::list>(v) || py::isinstance<py::tuple>(v)) {
    std::vector<std::string> items;
    size_t maxlen = 1;
    for (auto it : v) {
      items.push_back(to_bytes(it));
      maxlen = std::max(maxlen, items.back().size());
    }
    H5Id t(fixed_string_type(maxlen), H5Tclose);
    hsize_t dims[1] = {items.size()};
    H5Id sp(items.empty() ? H5Screate(H5S_NULL) : H5Screate_simple(1, dims, nullptr), H5Sclose);
    H5Id a(H5Acreate2(obj, name.c_str(), t, sp, H5P_DEFAULT, H5P_DEFAULT), H5Aclose);
    if (!items.empty()) {
      std::vector<char> buf(items.size() * maxlen, 0);
      for (size_t i = 0; i < items.size(); ++i) std::copy(items[i].begin(), items[i].end(), buf.begin() + i * maxlen);
      if (H5Awrite(a, t, buf.data()) < 0) throw std::runtime_error("H5Awrite failed for " + name);
    }
    return;
  }
  py::array arr = py::array::ensure(v);
  if (!arr) throw std::invalid_argument("unsupported attribute value for " + name);
  arr = py::array::ensure(arr, py::array::c_style | py::array::forcecast);
  const hid_t t = numpy_to_h5(arr.dtype());
  std::vector<hsize_t> dims(arr.shape(), arr.shape() + arr.ndim());
  H5Id sp(arr.ndim() == 0 ? H5Screate(H5S_SCALAR) : H5Screate_simple(arr.ndim(), dims.data(), nullptr), H5Sclose);
  H5Id a(H5Acreate2(obj, name.c_str(), t, sp, H5P_DEFAULT, H5P_DEFAULT), H5Aclose);
  if (H5Awrite(a, t, arr.data()) < 0) throw std::runtime_error("H5Awrite failed for " + name);
}

void write_tree(hid_t loc, const py::dict& tree) {
  if (tree.contains("attrs"))
    for (auto kv : tree["attrs"].cast<py::dict>()) write_attr(loc, kv.first.cast<std::string>(), kv.second);
  if (tree.contains("datasets")) {
    for (auto kv : tree["datasets"].cast<py::dict>()) {
      const std::string name = kv.first.cast<std::string>();
      py::array arr = py::array::ensure(kv.second, py::array::c_style | py::array::forcecast);
      const hid_t t = numpy_to_h5(arr.dtype());
      std::vector<hsize_t> dims(arr.shape(), arr.shape() + arr.ndim());
      H5Id sp(arr.ndim() == 0 ? H5Screate(H5S_SCALAR) : H5Screate_simple(arr.ndim(), dims.data(), nullptr),
              H5Sclose);
      H5Id lcpl(H5Pcreate(H5P_LINK_CREATE), H5Pclose);
      H5Pset_create_intermediate_group(lcpl, 1);  // "conv2d/kernel:0" creates group conv2d
      H5Id d(H5Dcreate2(loc, name.c_str(), t, sp, lcpl, H5P_DEFAULT, H5P_DEFAULT), H5Dclose);
      if (arr.size() > 0 && H5Dwrite(d, t, H5S_ALL, H5S_ALL, H5P_DEFAULT, arr.data()) < 0)
        throw std::runtime_error("H5Dwrite failed for " + name);
    }
  }
  if (tree.contains("groups")) {
    for (auto kv : tree["groups"].cast<py::dict>()) {
      const std::string name = kv.first.cast<std::string>();
      hid_t g = H5Lexists(loc, name.c_str(), H5P_DEFAULT) > 0 ? H5Gopen2(loc, name.c_str(), H5P_DEFAULT)
                                                              : H5Gcreate2(loc, name.c_str(), H5P_DEFAULT,
                                                                           H5P_DEFAULT, H5P_DEFAULT);
      H5Id gid(g, H5Gclose);
      write_tree(gid, kv.second.cast<py::dict>());
    }
  }
}

py::object read_attr(hid_t obj, const char* name) {
  H5Id a(H5Aopen(obj, name, H5P_DEFAULT), H5Aclose);
  H5Id t(H5Aget_type(a), H5Tclose);
  H5Id sp(H5Aget_space(a), H5Sclose);
  const int nd = H5Sget_simple_extent_ndims(sp);
  std::vector<hsize_t> dims(nd > 0 ? nd : 0);
  if (nd > 0) H5Sget_simple_extent_dims(sp, dims.data(), nullptr);
  hssize_t n = H5Sget_simple_extent_npoints(sp);
  if (H5Sget_simple_extent_type(sp) == H5S_NULL) n = 0;
  if (H5Tget_class(t) == H5T_STRING) {
    std::vector<std::string> out;
    if (H5Tis_variable_str(t) > 0) {
      std::vector<char*> ptrs(n > 0 ? n : 1, nullptr);
      H5Id mt(H5Tcopy(H5T_C_S1), H5Tclose);
      H5Tset_size(mt, H5T_VARIABLE);
      if (n > 0) H5Aread(a, mt, ptrs.data());
      for (hssize_t i = 0; i < n; ++i) out.emplace_back(ptrs[i] ? ptrs[i] : "");
      if (n > 0) H5Dvlen_reclaim(mt, sp, H5P_DEFAULT, ptrs.data());
    } else {
      const size_t sz = H5Tget_size(t);
      std::vector<char> buf(sz * (n > 0 ? n : 1), 0);
      if (n > 0) H5Aread(a, t, buf.data());
      for (hssize_t i = 0; i < n; ++i) {
        std::string s(buf.data() + i * sz, sz);
        s.erase(s.find_last_not_of('\0') == std::string::npos ? 0 : s.find_last_not_of('\0') + 1);
        out.push_back(s);
      }
    }
    if (nd == 0 && n == 1) return py::str(out[0]);
    py::list l;
    for (auto& s : out) l.append(py::str(s));
    return l;
  }
  hid_t mt;
  py::dtype dt;
  const H5T_class_t cls = H5Tget_class(t);
  const size_t sz = H5Tget_size(t);
  if (cls == H5T_FLOAT) {
    mt = sz == 4 ? H5T_NATIVE_FLOAT : H5T_NATIVE_DOUBLE;
    dt = sz == 4 ? py::dtype("float32") : py::dtype("float64");
  } else if (cls == H5T_INTEGER) {
    mt = H5T_NATIVE_INT64;
    dt = py::dtype("int64");
  } else {
    return py::none();
  }
  py::array arr(dt, std::vector<ssize_t>(dims.begin(), dims.end()));
  if (n > 0) H5Aread(a, mt, arr.mutable_data());
  return arr;
}

struct Collect {
  std::vector<std::string> names;
};
herr_t collect_link(hid_t, const char* name, const H5L_info_t*, void* op) {
  static_cast<Collect*>(op)->names.emplace_back(name);
  return 0;
}
herr_t collect_attr(hid_t, const char* name, const H5A_info_t*, void* op) {
  static_cast<Collect*>(op)->names.emplace_back(name);
  return 0;
}

py::array read_dataset(hid_t loc, const char* name) {
  H5Id d(H5Dopen2(loc, name, H5P_DEFAULT), H5Dclose);
  H5Id t(H5Dget_type(d), H5Tclose);
  H5Id sp(H5Dget_space(d), H5Sclose);
  const int nd = H5Sget_simple_extent_ndims(sp);
  std::vector<hsize_t> dims(nd > 0 ? nd : 0);
  if (nd > 0) H5Sget_simple_extent_dims(sp, dims.data(), nullptr);
  const H5T_class_t cls = H5Tget_class(t);
  const size_t sz = H5Tget_size(t);
  hid_t mt;
  py::dtype dt;
  if (cls == H5T_FLOAT) {
    mt = sz == 4 ? H5T_NATIVE_FLOAT : H5T_NATIVE_DOUBLE;
    dt = sz == 4 ? py::dtype("float32") : py::dtype("float64");
  } else if (cls == H5T_INTEGER && sz == 1) {
    mt = H5T_NATIVE_UINT8;
    dt = py::dtype("uint8");
  } else if (cls == H5T_INTEGER && sz <= 4) {
    mt = H5T_NATIVE_INT32;
    dt = py::dtype("int32");
  } else if (cls == H5T_INTEGER) {
    mt = H5T_NATIVE_INT64;
    dt = py::dtype("int64");
  } else {
    throw std::runtime_error(std::string("unsupported dataset type: ") + name);
  }
  py::array arr(dt, std::vector<ssize_t>(dims.begin(), dims.end()));
  if (arr.size() > 0 && H5Dread(d, mt, H5S_ALL, H5S_ALL, H5P_DEFAULT, arr.mutable_data()) < 0)
    throw std::runtime_error(std::string("H5Dread failed: ") + name);
  return arr;
}

py::dict read_tree(hid_t loc) {
  py::dict tree, attrs, groups, datasets;
  Collect ac;
  hsize_t idx = 0;
  H5Aiterate2(loc, H5_INDEX_CRT_ORDER, H5_ITER_INC, &idx, collect_attr, &ac);
  if (ac.names.empty()) {  // files without creation-order tracking
    idx = 0;
    H5Aiterate2(loc, H5_INDEX_NAME, H5_ITER_INC, &idx, collect_attr, &ac);
  }
  for (auto& n : ac.names) attrs[py::str(n)] = read_attr(loc, n.c_str());
  Collect lc;
  idx = 0;
  H5Literate(loc, H5_INDEX_NAME, H5_ITER_INC, &idx, collect_link, &lc);
  for (auto& n : lc.names) {
    H5O_info_t info;
    if (H5Oget_info_by_name2(loc, n.c_str(), &info, H5O_INFO_BASIC, H5P_DEFAULT) < 0) continue;
    if (info.type == H5O_TYPE_GROUP) {
      H5Id g(H5Gopen2(loc, n.c_str(), H5P_DEFAULT), H5Gclose);
      groups[py::str(n)] = read_tree(g);
    } else if (info.type == H5O_TYPE_DATASET) {
      datasets[py::str(n)] = read_dataset(loc, n.c_str());
    }
  }
  tree["attrs"] = attrs;
  tree["groups"] = groups;
  tree["datasets"] = datasets;
  return tree;
}

}  // namespace

PYBIND11_MODULE(_h5, m) {
  m.doc() = "HDF5 tree I/O (libhdf5 C API) for Keras-layout model files";
  m.def("version", []() {
    unsigned a, b, c;
    H5get_libversion(&a, &b, &c);
    return std::to_string(a) + "." + std::to_string(b) + "." + std::to_string(c);
  });
  m.def("write", [](const std::string& path, py::dict tree) {
    H5Eset_auto2(H5E_DEFAULT, nullptr, nullptr);
    H5Id fcpl(H5Pcreate(H5P_FILE_CREATE), H5Pclose);
    H5Pset_attr_creation_order(fcpl, H5P_CRT_ORDER_TRACKED);
    H5Id f(H5Fcreate(path.c_str(), H5F_ACC_TRUNC, fcpl, H5P_DEFAULT), H5Fclose);
    write_tree(f, tree);
    H5Fflush(f, H5F_SCOPE_GLOBAL);
  }, py::arg("path"), py::arg("tree"));
  m.def("read", [](const std::string& path) {
    H5Eset_auto2(H5E_DEFAULT, nullptr, nullptr);
    H5Id f(H5Fopen(path.c_str(), H5F_ACC_RDONLY, H5P_DEFAULT), H5Fclose);
    return read_tree(f);
  }, py::arg("path"));
}
