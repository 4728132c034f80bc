// Host-only self-test of the HDF5 tree writer/reader (csrc/io/h5tree.cpp), built with
// AddressSanitizer + UndefinedBehaviorSanitizer by tests/test_native_sanitizers.py
// (host C++ under ASan/UBSan in CPU tests).  Writes a Keras-layout-like
// tree, reads it back and compares every attribute, group and dataset byte for byte.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>

#include "h5tree.h"

using namespace damd::h5;

static int failures = 0;
#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                       \
    }                                                                   \
  } while (0)

static Array f32(std::vector<hsize_t> shape, float base) {
  Array a;
  a.dtype = DType::F32;
  a.shape = shape;
  a.bytes.resize(a.numel() * 4);
  for (size_t i = 0; i < a.numel(); ++i) {
    float v = base + 0.5f * (float)i - std::sin((float)i);
    std::memcpy(a.bytes.data() + 4 * i, &v, 4);
  }
  return a;
}

static Attr str(const std::string& s) {
  Attr a;
  a.kind = Attr::Str;
  a.s = s;
  return a;
}

static Attr strs(std::vector<std::string> v) {
  Attr a;
  a.kind = Attr::StrList;
  a.list = std::move(v);
  return a;
}

static const Attr* find_attr(const Group& g, const std::string& n) {
  for (auto& kv : g.attrs)
    if (kv.first == n) return &kv.second;
  return nullptr;
}
static const Group* find_group(const Group& g, const std::string& n) {
  for (auto& kv : g.groups)
    if (kv.first == n) return &kv.second;
  return nullptr;
}
static const Array* find_ds(const Group& g, const std::string& n) {
  for (auto& kv : g.datasets)
    if (kv.first == n) return &kv.second;
  return nullptr;
}

int main(int argc, char** argv) {
  const std::string path = argc > 1 ? argv[1] : "/tmp/damd_h5_selftest.h5";
  Group root;
  root.attrs.emplace_back("keras_version", str("2.2.4-tf"));
  root.attrs.emplace_back("backend", str("tensorflow"));
  std::string cfg(20000, 'x');  // a long model_config JSON
  root.attrs.emplace_back("model_config", str(cfg));
  Attr it;
  it.kind = Attr::Num;
  it.num.dtype = DType::I64;
  it.num.bytes.resize(8);
  int64_t iters = 1234567890123LL;
  std::memcpy(it.num.bytes.data(), &iters, 8);
  root.attrs.emplace_back("iterations", it);
  Group mw;
  mw.attrs.emplace_back("layer_names", strs({"conv2d", "max_pooling2d", "flatten", "dense", "dense_1"}));
  mw.attrs.emplace_back("empty_list", strs({}));
  Group conv;
  conv.attrs.emplace_back("weight_names", strs({"conv2d/kernel:0", "conv2d/bias:0"}));
  conv.datasets.emplace_back("conv2d/kernel:0", f32({3, 3, 1, 32}, 1.f));
  conv.datasets.emplace_back("conv2d/bias:0", f32({32}, -2.f));
  conv.datasets.emplace_back("empty", f32({0, 4}, 0.f));
  mw.groups.emplace_back("conv2d", conv);
  Group dense;
  dense.attrs.emplace_back("weight_names", strs({"dense/kernel:0"}));
  dense.datasets.emplace_back("dense/kernel:0", f32({5408, 64}, 3.f));
  mw.groups.emplace_back("dense", dense);
  root.groups.emplace_back("model_weights", mw);
  Array u8;
  u8.dtype = DType::U8;
  u8.shape = {7};
  u8.bytes = {0, 1, 2, 250, 251, 254, 255};
  root.datasets.emplace_back("bytes", u8);

  write_file(path, root);
  Group back = read_file(path);

  CHECK(find_attr(back, "keras_version") && find_attr(back, "keras_version")->s == "2.2.4-tf");
  CHECK(find_attr(back, "model_config") && find_attr(back, "model_config")->s == cfg);
  const Attr* ib = find_attr(back, "iterations");
  CHECK(ib && ib->kind == Attr::Num && ib->num.bytes.size() == 8);
  if (ib && ib->num.bytes.size() == 8) {
    int64_t v;
    std::memcpy(&v, ib->num.bytes.data(), 8);
    CHECK(v == iters);
  }
  // attribute order is creation order (Keras reads layer_names positionally)
  CHECK(back.attrs.size() == 4 && back.attrs[0].first == "keras_version" && back.attrs[3].first == "iterations");
  const Group* bmw = find_group(back, "model_weights");
  CHECK(bmw != nullptr);
  if (bmw) {
    const Attr* ln = find_attr(*bmw, "layer_names");
    CHECK(ln && ln->kind == Attr::StrList && ln->list.size() == 5 && ln->list[4] == "dense_1");
    const Attr* el = find_attr(*bmw, "empty_list");
    CHECK(el && el->kind == Attr::StrList && el->list.empty());
    const Group* bc = find_group(*bmw, "conv2d");
    CHECK(bc != nullptr);
    if (bc) {
      // "conv2d/kernel:0" created the intermediate group conv2d/conv2d
      const Group* inner = find_group(*bc, "conv2d");
      CHECK(inner != nullptr);
      if (inner) {
        const Array* k = find_ds(*inner, "kernel:0");
        const Array ref = f32({3, 3, 1, 32}, 1.f);
        CHECK(k && k->shape == ref.shape && k->bytes == ref.bytes);
      }
      const Array* e = find_ds(*bc, "empty");
      CHECK(e && e->numel() == 0 && e->shape.size() == 2);
    }
    const Group* bd = find_group(*bmw, "dense");
    const Group* bdi = bd ? find_group(*bd, "dense") : nullptr;
    const Array* dk = bdi ? find_ds(*bdi, "kernel:0") : nullptr;
    CHECK(dk && dk->bytes == f32({5408, 64}, 3.f).bytes);
  }
  const Array* bb = find_ds(back, "bytes");
  CHECK(bb && bb->dtype == DType::U8 && bb->bytes == u8.bytes);

  // failure paths raise, they do not crash
  bool threw = false;
  try {
    read_file(path + ".does-not-exist");
  } catch (const std::runtime_error&) {
    threw = true;
  }
  CHECK(threw);
  Group bad;
  Array wrong = f32({4}, 0.f);
  wrong.bytes.resize(3);
  bad.datasets.emplace_back("wrong", wrong);
  threw = false;
  try {
    write_file(path + ".bad", bad);
  } catch (const std::invalid_argument&) {
    threw = true;
  }
  CHECK(threw);
  std::remove((path + ".bad").c_str());
  std::remove(path.c_str());
  if (failures) {
    std::fprintf(stderr, "h5 selftest: %d failure(s)\n", failures);
    return 1;
  }
  std::printf("h5 selftest OK (libhdf5 %s)\n", library_version().c_str());
  return 0;
}
