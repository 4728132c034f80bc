// HDF5 tree I/O over the libhdf5 C API (see h5tree.h).
#include "h5tree.h"

#include <algorithm>
#include <stdexcept>

namespace damd {
namespace h5 {
namespace {

struct Id {  // RAII for hid_t with its close function
  hid_t id;
  herr_t (*close)(hid_t);
  Id(hid_t i, herr_t (*c)(hid_t), const char* what) : id(i), close(c) {
    if (id < 0) throw std::runtime_error(std::string("HDF5 call failed: ") + what);
  }
  ~Id() {
    if (id >= 0) close(id);
  }
  Id(const Id&) = delete;
  Id& operator=(const Id&) = delete;
  operator hid_t() const { return id; }
};

hid_t mem_type(DType t) {
  switch (t) {
    case DType::F32: return H5T_NATIVE_FLOAT;
    case DType::F64: return H5T_NATIVE_DOUBLE;
    case DType::I32: return H5T_NATIVE_INT32;
    case DType::I64: return H5T_NATIVE_INT64;
    case DType::U8: return H5T_NATIVE_UINT8;
  }
  throw std::invalid_argument("dtype");
}

hid_t fixed_string_type(size_t n) {
  hid_t t = H5Tcopy(H5T_C_S1);
  H5Tset_size(t, n == 0 ? 1 : n);
  H5Tset_strpad(t, H5T_STR_NULLPAD);
  H5Tset_cset(t, H5T_CSET_ASCII);
  return t;
}

hid_t make_space(const std::vector<hsize_t>& shape) {
  return shape.empty() ? H5Screate(H5S_SCALAR) : H5Screate_simple((int)shape.size(), shape.data(), nullptr);
}

void write_attr(hid_t obj, const std::string& name, const Attr& a) {
  if (H5Aexists(obj, name.c_str()) > 0) H5Adelete(obj, name.c_str());
  if (a.kind == Attr::Str) {
    Id t(fixed_string_type(a.s.size()), H5Tclose, "string type");
    Id sp(H5Screate(H5S_SCALAR), H5Sclose, "scalar space");
    Id at(H5Acreate2(obj, name.c_str(), t, sp, H5P_DEFAULT, H5P_DEFAULT), H5Aclose, name.c_str());
    std::vector<char> buf(std::max<size_t>(a.s.size(), 1), 0);
    std::copy(a.s.begin(), a.s.end(), buf.begin());
    if (H5Awrite(at, t, buf.data()) < 0) throw std::runtime_error("H5Awrite failed for " + name);
    return;
  }
  if (a.kind == Attr::StrList) {
    size_t maxlen = 1;
    for (auto& s : a.list) maxlen = std::max(maxlen, s.size());
    Id t(fixed_string_type(maxlen), H5Tclose, "string type");
    hsize_t dims[1] = {a.list.size()};
    Id sp(a.list.empty() ? H5Screate(H5S_NULL) : H5Screate_simple(1, dims, nullptr), H5Sclose, "list space");
    Id at(H5Acreate2(obj, name.c_str(), t, sp, H5P_DEFAULT, H5P_DEFAULT), H5Aclose, name.c_str());
    if (!a.list.empty()) {
      std::vector<char> buf(a.list.size() * maxlen, 0);
      for (size_t i = 0; i < a.list.size(); ++i) std::copy(a.list[i].begin(), a.list[i].end(), buf.begin() + i * maxlen);
      if (H5Awrite(at, t, buf.data()) < 0) throw std::runtime_error("H5Awrite failed for " + name);
    }
    return;
  }
  if (a.num.bytes.size() != a.num.numel() * dtype_size(a.num.dtype))
    throw std::invalid_argument("attribute " + name + ": byte size does not match shape");
  const hid_t t = mem_type(a.num.dtype);
  Id sp(make_space(a.num.shape), H5Sclose, "attr space");
  Id at(H5Acreate2(obj, name.c_str(), t, sp, H5P_DEFAULT, H5P_DEFAULT), H5Aclose, name.c_str());
  if (H5Awrite(at, t, a.num.bytes.data()) < 0) throw std::runtime_error("H5Awrite failed for " + name);
}

void write_group(hid_t loc, const Group& g) {
  for (auto& kv : g.attrs) write_attr(loc, kv.first, kv.second);
  for (auto& kv : g.datasets) {
    const Array& arr = kv.second;
    if (arr.bytes.size() != arr.numel() * dtype_size(arr.dtype))
      throw std::invalid_argument("dataset " + kv.first + ": byte size does not match shape");
    const hid_t t = mem_type(arr.dtype);
    Id sp(make_space(arr.shape), H5Sclose, "dataset space");
    Id lcpl(H5Pcreate(H5P_LINK_CREATE), H5Pclose, "lcpl");
    H5Pset_create_intermediate_group(lcpl, 1);
    Id d(H5Dcreate2(loc, kv.first.c_str(), t, sp, lcpl, H5P_DEFAULT, H5P_DEFAULT), H5Dclose, kv.first.c_str());
    if (arr.numel() > 0 && H5Dwrite(d, t, H5S_ALL, H5S_ALL, H5P_DEFAULT, arr.bytes.data()) < 0)
      throw std::runtime_error("H5Dwrite failed for " + kv.first);
  }
  for (auto& kv : g.groups) {
    const char* n = kv.first.c_str();
    hid_t gid = H5Lexists(loc, n, H5P_DEFAULT) > 0 ? H5Gopen2(loc, n, H5P_DEFAULT)
                                                   : H5Gcreate2(loc, n, H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT);
    Id gi(gid, H5Gclose, n);
    write_group(gi, kv.second);
  }
}

bool dtype_of(hid_t t, DType& out) {
  const H5T_class_t cls = H5Tget_class(t);
  const size_t sz = H5Tget_size(t);
  if (cls == H5T_FLOAT) {
    out = sz == 4 ? DType::F32 : DType::F64;
    return true;
  }
  if (cls == H5T_INTEGER) {
    out = sz == 1 ? DType::U8 : (sz <= 4 ? DType::I32 : DType::I64);
    return true;
  }
  return false;
}

std::vector<hsize_t> shape_of(hid_t sp) {
  const int nd = H5Sget_simple_extent_ndims(sp);
  std::vector<hsize_t> dims(nd > 0 ? nd : 0);
  if (nd > 0) H5Sget_simple_extent_dims(sp, dims.data(), nullptr);
  return dims;
}

Attr read_attr(hid_t obj, const char* name) {
  Id a(H5Aopen(obj, name, H5P_DEFAULT), H5Aclose, name);
  Id t(H5Aget_type(a), H5Tclose, "attr type");
  Id sp(H5Aget_space(a), H5Sclose, "attr space");
  const std::vector<hsize_t> dims = shape_of(sp);
  hssize_t n = H5Sget_simple_extent_npoints(sp);
  if (H5Sget_simple_extent_type(sp) == H5S_NULL) n = 0;
  Attr out;
  if (H5Tget_class(t) == H5T_STRING) {
    std::vector<std::string> items;
    if (H5Tis_variable_str(t) > 0) {
      std::vector<char*> ptrs(n > 0 ? n : 1, nullptr);
      Id mt(H5Tcopy(H5T_C_S1), H5Tclose, "vlen type");
      H5Tset_size(mt, H5T_VARIABLE);
      if (n > 0 && H5Aread(a, mt, ptrs.data()) >= 0) {
        for (hssize_t i = 0; i < n; ++i) items.emplace_back(ptrs[i] ? ptrs[i] : "");
        H5Dvlen_reclaim(mt, sp, H5P_DEFAULT, ptrs.data());
      }
    } else {
      const size_t sz = H5Tget_size(t);
      std::vector<char> buf(sz * (n > 0 ? n : 1), 0);
      if (n > 0) H5Aread(a, t, buf.data());
      for (hssize_t i = 0; i < n; ++i) {
        std::string s(buf.data() + i * sz, sz);
        const size_t last = s.find_last_not_of('\0');
        s.erase(last == std::string::npos ? 0 : last + 1);
        items.push_back(s);
      }
    }
    if (dims.empty() && n == 1) {
      out.kind = Attr::Str;
      out.s = items[0];
    } else {
      out.kind = Attr::StrList;
      out.list = std::move(items);
    }
    return out;
  }
  out.kind = Attr::Num;
  DType dt;
  if (!dtype_of(t, dt)) throw std::runtime_error(std::string("unsupported attribute type: ") + name);
  if (dt == DType::I32 || dt == DType::U8) dt = DType::I64;  // numeric attributes come back as int64
  out.num.dtype = dt;
  out.num.shape = dims;
  out.num.bytes.assign(out.num.numel() * dtype_size(dt), 0);
  if (n > 0 && H5Aread(a, mem_type(dt), out.num.bytes.data()) < 0)
    throw std::runtime_error(std::string("H5Aread failed: ") + name);
  return out;
}

Array read_dataset(hid_t loc, const char* name) {
  Id d(H5Dopen2(loc, name, H5P_DEFAULT), H5Dclose, name);
  Id t(H5Dget_type(d), H5Tclose, "dataset type");
  Id sp(H5Dget_space(d), H5Sclose, "dataset space");
  Array arr;
  if (!dtype_of(t, arr.dtype)) throw std::runtime_error(std::string("unsupported dataset type: ") + name);
  arr.shape = shape_of(sp);
  arr.bytes.assign(arr.numel() * dtype_size(arr.dtype), 0);
  if (arr.numel() > 0 && H5Dread(d, mem_type(arr.dtype), H5S_ALL, H5S_ALL, H5P_DEFAULT, arr.bytes.data()) < 0)
    throw std::runtime_error(std::string("H5Dread failed: ") + name);
  return arr;
}

struct Names {
  std::vector<std::string> v;
};
herr_t on_link(hid_t, const char* name, const H5L_info_t*, void* op) {
  static_cast<Names*>(op)->v.emplace_back(name);
  return 0;
}
herr_t on_attr(hid_t, const char* name, const H5A_info_t*, void* op) {
  static_cast<Names*>(op)->v.emplace_back(name);
  return 0;
}

Group read_group(hid_t loc) {
  Group g;
  Names an;
  hsize_t idx = 0;
  H5Aiterate2(loc, H5_INDEX_CRT_ORDER, H5_ITER_INC, &idx, on_attr, &an);
  if (an.v.empty()) {  // files written without creation-order tracking
    idx = 0;
    H5Aiterate2(loc, H5_INDEX_NAME, H5_ITER_INC, &idx, on_attr, &an);
  }
  for (auto& n : an.v) g.attrs.emplace_back(n, read_attr(loc, n.c_str()));
  Names ln;
  idx = 0;
  H5Literate(loc, H5_INDEX_NAME, H5_ITER_INC, &idx, on_link, &ln);
  for (auto& n : ln.v) {
    H5O_info_t info;
    if (H5Oget_info_by_name2(loc, n.c_str(), &info, H5O_INFO_BASIC, H5P_DEFAULT) < 0) continue;
    if (info.type == H5O_TYPE_GROUP) {
      Id gi(H5Gopen2(loc, n.c_str(), H5P_DEFAULT), H5Gclose, n.c_str());
      g.groups.emplace_back(n, read_group(gi));
    } else if (info.type == H5O_TYPE_DATASET) {
      g.datasets.emplace_back(n, read_dataset(loc, n.c_str()));
    }
  }
  return g;
}

}  // namespace

size_t dtype_size(DType t) {
  switch (t) {
    case DType::F32: return 4;
    case DType::F64: return 8;
    case DType::I32: return 4;
    case DType::I64: return 8;
    case DType::U8: return 1;
  }
  return 0;
}

size_t Array::numel() const {
  size_t n = 1;
  for (auto d : shape) n *= (size_t)d;
  return n;
}

void write_file(const std::string& path, const Group& root) {
  H5Eset_auto2(H5E_DEFAULT, nullptr, nullptr);
  Id fcpl(H5Pcreate(H5P_FILE_CREATE), H5Pclose, "fcpl");
  H5Pset_attr_creation_order(fcpl, H5P_CRT_ORDER_TRACKED);
  Id f(H5Fcreate(path.c_str(), H5F_ACC_TRUNC, fcpl, H5P_DEFAULT), H5Fclose, path.c_str());
  write_group(f, root);
  H5Fflush(f, H5F_SCOPE_GLOBAL);
}

Group read_file(const std::string& path) {
  H5Eset_auto2(H5E_DEFAULT, nullptr, nullptr);
  Id f(H5Fopen(path.c_str(), H5F_ACC_RDONLY, H5P_DEFAULT), H5Fclose, path.c_str());
  return read_group(f);
}

std::string library_version() {
  unsigned a, b, c;
  H5get_libversion(&a, &b, &c);
  return std::to_string(a) + "." + std::to_string(b) + "." + std::to_string(c);
}

}  // namespace h5
}  // namespace damd
