// HDF5 tree model + file I/O over the libhdf5 C API, independent of Python.
//
// A file is a tree of groups; every group has ordered attributes, child groups and
// datasets.  Encodings follow what h5py writes for Keras model files (reference
// README.md:234-247, upstream keras hdf5_format): str attributes as fixed-length
// NULLPAD ASCII strings (scalar or 1-D), numeric attributes/datasets as native
// little-endian types.  Dataset names may contain '/' (intermediate groups are created,
// e.g. "conv2d/kernel:0").  Used by the Python binding (keras_h5.cpp) and by the
// sanitizer self-test (csrc/tests/h5_selftest.cpp).
#pragma once
#include <hdf5.h>

#include <cstdint>
#include <string>
#include <utility>
#include <vector>

namespace damd {
namespace h5 {

enum class DType { F32, F64, I32, I64, U8 };
size_t dtype_size(DType t);

struct Array {
  DType dtype = DType::F32;
  std::vector<hsize_t> shape;  // empty = scalar
  std::vector<uint8_t> bytes;  // C order, dtype_size * prod(shape)
  size_t numel() const;
};

struct Attr {
  enum Kind { Str, StrList, Num } kind = Str;
  std::string s;
  std::vector<std::string> list;
  Array num;
};

struct Group {
  std::vector<std::pair<std::string, Attr>> attrs;
  std::vector<std::pair<std::string, Group>> groups;
  std::vector<std::pair<std::string, Array>> datasets;
};

void write_file(const std::string& path, const Group& root);
Group read_file(const std::string& path);
std::string library_version();

}  // namespace h5
}  // namespace damd
