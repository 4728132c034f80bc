// Python bindings of the native runtime (module distributed_amd._C).
//
// The extension deliberately does not link libtorch: tensors cross the boundary as raw
// device pointers (tensor.data_ptr()) and streams as hipStream_t integers, so the module
// only depends on the HIP runtime and RCCL that torch itself has already loaded.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "comm.h"
#include "convnet.h"
#include "damd_common.h"
#include "kernels_api.h"
#include "peer_comm.h"
#include "step_executor.h"

namespace py = pybind11;
using namespace damd;

#define HIP_CHECK(x)                                                                    \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess)                                                               \
      throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e_) +     \
                               " at " #x);                                              \
  } while (0)

template <typename T>
static T* P_(uintptr_t p) { return reinterpret_cast<T*>(p); }

// Fused MNIST-CNN trainer: every per-step buffer is preallocated by Python (torch
// tensors) and passed in as device pointers.
class ConvNetTrainer : public StepExecutor {
 public:
  ConvNetTrainer(int device, py::dict bufs, int B, int PP, int grad_allreduce)
      : StepExecutor(device), B_(B), PP_(PP), grad_allreduce_(grad_allreduce) {
    if (B <= 0) throw std::invalid_argument("batch must be > 0");
    if (B > 65535) throw std::invalid_argument("per-rank batch must be < 65536 (packed kernel argument)");
    if (PP < 1 || PP > 4) throw std::invalid_argument("positions per slice must be in [1,4]");
    auto g = [&](const char* k) -> uintptr_t { return bufs[k].cast<uintptr_t>(); };
    b_.X = nullptr; b_.labels = nullptr; b_.x_u8 = 0;
    b_.P = P_<float>(g("params")); b_.G = P_<float>(g("grads")); b_.V = P_<float>(g("velocity"));
    b_.ctrl = P_<Ctrl>(g("ctrl"));
    b_.pooled = P_<uint16_t>(g("pooled")); b_.code = P_<uint8_t>(g("code"));
    b_.W1alt = P_<float>(g("w1alt")); b_.V1alt = P_<float>(g("v1alt")); b_.w1bf = P_<uint16_t>(g("w1bf"));
    b_.stamps = bufs.contains("stamps") ? P_<unsigned long long>(g("stamps")) : nullptr;
    b_.eager_w1 = bufs.contains("eager_w1") ? (int)g("eager_w1") : 0;
    b_.hacc = P_<long long>(g("hacc"));
    b_.hconv = P_<long long>(g("hconv"));
    b_.calt = P_<float>(g("calt"));
    b_.ppb = bufs.contains("ppb") ? (int)g("ppb") : PP;
    // optional next-batch prefetch buffers (convnet.h): [B][784] x 4 bytes + one int64 tag
    b_.xnext = bufs.contains("xnext") ? P_<void>(g("xnext")) : nullptr;
    b_.xtag = bufs.contains("xtag") ? P_<long long>(g("xtag")) : nullptr;
    b_.xcur = bufs.contains("xcur") ? P_<void>(g("xcur")) : nullptr;
    b_.ycur = bufs.contains("ycur") ? P_<int>(g("ycur")) : nullptr;
    if ((b_.xnext == nullptr) != (b_.xtag == nullptr) || (b_.xcur == nullptr) != (b_.ycur == nullptr))
      throw std::invalid_argument("xnext / xtag and xcur / ycur go in pairs");
    // parity hints (convnet.h par_hint; DAMD_PAR_HINT=0: the kernels read ctrl.wpar)
    const char* ph = getenv("DAMD_PAR_HINT");
    hint_ = !(ph && ph[0] == '0');
    b_.par_hint = -1;
    if (b_.ppb < 1 || b_.ppb > 4) throw std::invalid_argument("bwd positions per slice must be in [1,4]");
    HIP_CHECK(convnet2_set_lds_limits());
  }
  // Phase timing: k eager steps of the 2-launch step with HIP events
  // between the forward launch, the backward launch and the gradient all-reduce; returns
  // per step [forward_ms, backward_ms, allreduce_ms] (the SGD update is fused into the
  // forward kernel: it applies the previous step's deferred update)
  std::vector<std::vector<float>> phase_times(int k) {
    if (!b_.X) throw std::runtime_error("ConvNetTrainer: set_data() not called");
    hipEvent_t ev[4];
    for (auto& e : ev) HIP_CHECK(hipEventCreate(&e));
    std::vector<std::vector<float>> out;
    for (int i = 0; i < k; ++i) {
      HIP_CHECK(hipEventRecord(ev[0], stream_));
      b_.par_hint = hint_ ? par_ : -1;
      HIP_CHECK(convnet2_launch_fwd(b_, B_, PP_, stream_));
      HIP_CHECK(hipEventRecord(ev[1], stream_));
      HIP_CHECK(convnet2_launch_bwd(b_, B_, PP_, stream_));
      par_ ^= 1;
      HIP_CHECK(hipEventRecord(ev[2], stream_));
      if (grad_allreduce_ && !sharded_) {
        if (peer_ && fold_)
          peer_->allreduce_staged((long)convnet_grad_count(PP_), 2 * kConvNetNConv, stream_, b_.hconv);
        else if (peer_) peer_->allreduce(b_.G, (long)convnet_grad_count(PP_), stream_, b_.hconv, 2 * kConvNetNConv);
        else if (comm_) comm_->allreduce_f32_i64(b_.G, convnet_grad_count(PP_), b_.hconv, 2 * kConvNetNConv, stream_);
      }
      HIP_CHECK(hipEventRecord(ev[3], stream_));
      HIP_CHECK(hipEventSynchronize(ev[3]));
      std::vector<float> r(3);
      for (int j = 0; j < 3; ++j) HIP_CHECK(hipEventElapsedTime(&r[j], ev[j], ev[j + 1]));
      out.push_back(r);
    }
    for (auto& e : ev) hipEventDestroy(e);
    return out;
  }
  // X [n][784] (fp32, or uint8 holding k for inputs k/255) and labels [n] int32:
  // epoch-permuted copies (stable pointers).
  void set_data(uintptr_t X, uintptr_t labels, int x_u8) {
    b_.X = P_<const void>(X); b_.labels = P_<const int>(labels); b_.x_u8 = x_u8;
    // a prefetched batch of the previous data must never match a tag again
    if (b_.xtag) HIP_CHECK(hipMemsetAsync(b_.xtag, 0, sizeof(long long), stream_));
    invalidate_graphs();
  }
  // Fold the per-step peer all-reduce into the step kernels: bwd writes its gradient
  // straight into the all-reduce's `in` staging (no copy-in pass), the next fwd / flush
  // read the reduced gradient from `out` (no copy-out pass); the peer kernel only
  // exchanges.  fold = false restores the engine's own buffers (copy-in / copy-out).
  void set_peer_fold(PeerAllreduce* p, bool fold) {
    if (!G_own_) { G_own_ = b_.G; hconv_own_ = b_.hconv; }
    set_peer(p);
    fold_ = fold && p && p->world() > 1;
    if (fold_) {
      const long n = (long)convnet_grad_count(PP_), nfp = (n + 3) / 4 * 4;
      if (PeerAllreduce::message_words(n, 2 * kConvNetNConv) > p->capacity())
        throw std::invalid_argument("peer all-reduce capacity too small for the folded step");
      b_.G = p->in_local();
      // the conv-gradient int64 sums stay in the engine's own (cached) buffer: bwd adds into
      // them with atomics, kept off the uncached staging; the peer kernel copies them in
      b_.hconv = hconv_own_;
      b_.Gr = p->out_local();
      b_.hconv_r = reinterpret_cast<long long*>(p->out_local() + nfp);
    } else {
      b_.G = G_own_; b_.hconv = hconv_own_; b_.Gr = nullptr; b_.hconv_r = nullptr;
    }
    invalidate_graphs();
  }
  bool folded() const { return fold_; }
  // Sharded multi-rank step (convnet.h XArgs): the gradient exchange runs inside the step
  // kernels through the peer all-reduce's mapped staging (its `in` holds the partial slots,
  // its `out` the reduced gradient, small messages and flags) -- no all-reduce launch.
  // hred: [2][320] int64 (the conv-gradient sums convnet2_launch_gather writes for flush)
  void set_sharded(PeerAllreduce* p, uintptr_t hred, int gbf16) {
    if (!p || p->world() < 2 || p->world() > kXMaxRanks) throw std::invalid_argument("sharded step: 2..8 ranks");
    const int NU = 4 * convnet_num_slices(b_.ppb);
    if (p->capacity() < convnet_xin_floats(p->world(), NU) || p->capacity() < convnet_xout_floats(NU))
      throw std::invalid_argument("sharded step: peer staging too small");
    const PeerArgs& a = p->args();
    XArgs x{};
    for (int r = 0; r < p->world(); ++r) {
      if (!a.in[r] || !a.out[r]) throw std::runtime_error("sharded step: peer staging not mapped");
      x.in[r] = a.in[r];
      x.out[r] = a.out[r];
    }
    x.status = a.status;
    x.timeout_ticks = a.timeout_ticks;
    x.world = p->world();
    x.rank = p->rank();
    x.gbf16 = gbf16;
    x.ppb = b_.ppb;
    xa_ = x;
    set_peer(p);
    sharded_ = true;
    fold_ = false;
    // the flags start at 0 (the self-test wrote over the whole staging): the caller joins a
    // barrier of all ranks after this returns, before any step
    HIP_CHECK(hipMemset(p->out_local() + kXFlags, 0,
                        (size_t)(convnet_xout_floats(NU) - kXFlags) * sizeof(float)));
    HIP_CHECK(hipDeviceSynchronize());
    b_.xa = &xa_;
    b_.Gr = p->out_local() + kXGred;
    b_.hconv_r = P_<long long>(hred);
    invalidate_graphs();
  }
  bool sharded() const { return sharded_; }
  // in-kernel wait deadline of the sharded exchange (follows the collective watchdog)
  void set_exchange_timeout(double s) { xa_.timeout_ticks = (unsigned long long)(s * 1e8); invalidate_graphs(); }
  // sharded step: the pending update's reduced small gradients / metric tail gathered into Gr
  void gather() {
    if (sharded_) HIP_CHECK(convnet2_launch_gather(b_, PP_, stream_));
  }
  // the reduced [loss, correct, count] tail of the last step (host copy, synchronizes)
  std::vector<float> metric_tail() {
    std::vector<float> t(3);
    gather();
    HIP_CHECK(hipStreamSynchronize(stream_));
    const float* g = b_.Gr ? b_.Gr : b_.G;
    HIP_CHECK(hipMemcpy(t.data(), g + kConvNetNParam, 3 * sizeof(float), hipMemcpyDeviceToHost));
    return t;
  }
  void flush() {
    gather();
    HIP_CHECK(convnet2_launch_flush(b_, B_, stream_));
    par_ = 0;  // flush resets ctrl.wpar
  }
  int parity() const { return par_; }
  // timed runs: k steps + the flush of the last deferred update as one graph
  void capture_final(int k) { StepExecutor::capture_final(k); }
  bool run_final(int k) { return StepExecutor::run_final(k); }
  bool warm_final(int k) { return StepExecutor::warm_final(k); }
  int num_slices() const { return convnet_num_slices(PP_); }
  int num_slices_bwd() const { return convnet_num_slices(b_.ppb); }
  int batch() const { return B_; }

 protected:
  void enqueue_tail() override { flush(); }
  int phase_value() const override { return par_; }
  void set_phase(int p) override { par_ = p; }
  int phase_after(int p, int k, bool tail) const override { return tail ? 0 : p ^ (k & 1); }
  void enqueue_one_step() override {
    if (!b_.X) throw std::runtime_error("ConvNetTrainer: set_data() not called");
    b_.par_hint = hint_ ? par_ : -1;
    HIP_CHECK(convnet2_launch_step(b_, B_, PP_, stream_));
    par_ ^= 1;  // bwd flips ctrl.wpar
    if (!grad_allreduce_ || sharded_) return;  // sharded: the exchange is inside the step kernels
    // the conv gradient is int64 fixed point (hconv): reduced exactly, in the same call as
    // the fp32 gradient + metric buffer; both parities (see convnet_step2.hip)
    long long* aux = b_.hconv;
    const long n64 = 2 * kConvNetNConv;
    if (peer_ && fold_)  // the message is already in the peer `in` staging: exchange only
      peer_->allreduce_staged((long)convnet_grad_count(PP_), n64, stream_, b_.hconv);
    else if (peer_)  // native xGMI two-shot all-reduce
      peer_->allreduce(b_.G, (long)convnet_grad_count(PP_), stream_, aux, n64);
    else if (comm_)  // comm set only when a reduction is wanted
      comm_->allreduce_f32_i64(b_.G, convnet_grad_count(PP_), aux, (size_t)n64, stream_);
  }

 private:
  ConvNetBuffers b_{};
  float* G_own_ = nullptr;         // the engine's gradient buffer (b_.G unless folded)
  long long* hconv_own_ = nullptr;
  bool fold_ = false;
  bool sharded_ = false;
  XArgs xa_{};  // b_.xa points here (kernels take it by value at launch)
  int par_ = 0;        // host shadow of ctrl.wpar (0 at construction and after every flush)
  bool hint_ = true;   // pass it to the kernels (par_hint)
  int B_, PP_, grad_allreduce_;
};

const char* damd_src_hash();  // build/obj/src_hash.cpp, generated by distributed_amd/_build.py

PYBIND11_MODULE(_C, m) {
  m.doc() = "distributed_amd native runtime (HIP/gfx950 kernels, RCCL, hipGraph executor)";
  m.def("src_hash", []() { return std::string(damd_src_hash()); });
  // structure of a captured (not yet destroyed) hipGraph: one (node type, kernel name or
  // "", [indices of the nodes it depends on]) per node -- what the tests use to check that
  // each gradient bucket's collective depends only on the backward work that wrote it
  m.def("graph_nodes", [](uintptr_t gp) {
    hipGraph_t g = reinterpret_cast<hipGraph_t>(gp);
    size_t n = 0;
    HIP_CHECK(hipGraphGetNodes(g, nullptr, &n));
    std::vector<hipGraphNode_t> nodes(n);
    if (n) HIP_CHECK(hipGraphGetNodes(g, nodes.data(), &n));
    std::unordered_map<hipGraphNode_t, int> idx;
    for (size_t i = 0; i < n; ++i) idx[nodes[i]] = (int)i;
    py::list out;
    for (size_t i = 0; i < n; ++i) {
      hipGraphNodeType t;
      HIP_CHECK(hipGraphNodeGetType(nodes[i], &t));
      std::string name;
      if (t == hipGraphNodeTypeKernel) {
        hipKernelNodeParams kp{};
        if (hipGraphKernelNodeGetParams(nodes[i], &kp) == hipSuccess && kp.func) {
          const char* nm = hipKernelNameRefByPtr(kp.func, nullptr);
          if (nm) name = nm;
        }
        (void)hipGetLastError();
      }
      size_t nd = 0;
      HIP_CHECK(hipGraphNodeGetDependencies(nodes[i], nullptr, &nd));
      std::vector<hipGraphNode_t> deps(nd);
      if (nd) HIP_CHECK(hipGraphNodeGetDependencies(nodes[i], deps.data(), &nd));
      std::vector<int> di;
      for (auto d : deps) di.push_back(idx.count(d) ? idx[d] : -1);
      out.append(py::make_tuple((int)t, name, di));
    }
    return out;
  });
  m.attr("CONVNET_NPARAM") = kConvNetNParam;
  m.attr("CONVNET_NGRAD") = kConvNetNGrad;
  m.attr("CONVNET_NCONV") = kConvNetNConv;
  m.def("convnet2_lds_bytes", [](int PP) { return py::make_tuple(convnet2_fwd_lds(PP, 4), convnet2_bwd_lds(PP)); });
  m.def("convnet_num_slices", &convnet_num_slices);
  m.def("convnet_hacc_elems", &convnet_hacc_elems);
  m.def("convnet_grad_count", &convnet_grad_count);

  m.def("device_count", []() { int n = 0; if (hipGetDeviceCount(&n) != hipSuccess) n = 0; return n; });
  m.def("rccl_unique_id", []() { return py::bytes(rccl_unique_id()); });
  m.def("rccl_version", []() { int v = 0; ncclGetVersion(&v); return v; });

  py::class_<RcclComm>(m, "RcclComm")
      .def(py::init([](int n, int r, py::bytes uid, int dev) {
             return new RcclComm(n, r, std::string(uid), dev);
           }),
           py::arg("nranks"), py::arg("rank"), py::arg("uid"), py::arg("device"),
           py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("nranks", &RcclComm::nranks)
      .def_property_readonly("rank", &RcclComm::rank)
      .def_property_readonly("comm_count", &RcclComm::comm_count)
      .def("allreduce",
           [](RcclComm& c, uintptr_t s, uintptr_t r, size_t n, int dt, int op, uintptr_t st) {
             c.allreduce(P_<void>(s), P_<void>(r), n, dt, op, P_<ihipStream_t>(st));
           })
      .def("broadcast",
           [](RcclComm& c, uintptr_t b, size_t n, int dt, int root, uintptr_t st) {
             c.broadcast(P_<void>(b), n, dt, root, P_<ihipStream_t>(st));
           })
      .def("allgather",
           [](RcclComm& c, uintptr_t s, uintptr_t r, size_t n, int dt, uintptr_t st) {
             c.allgather(P_<const void>(s), P_<void>(r), n, dt, P_<ihipStream_t>(st));
           })
      .def("reduce_scatter",
           [](RcclComm& c, uintptr_t s, uintptr_t r, size_t n, int dt, int op, uintptr_t st) {
             c.reduce_scatter(P_<const void>(s), P_<void>(r), n, dt, op, P_<ihipStream_t>(st));
           })
      .def("allreduce_f32_i64",
           [](RcclComm& c, uintptr_t d, size_t n, uintptr_t a, size_t n64, uintptr_t st) {
             c.allreduce_f32_i64(P_<float>(d), n, P_<long long>(a), n64, P_<ihipStream_t>(st));
           })
      .def("abort", &RcclComm::abort)
      .def_property_readonly("aborted", &RcclComm::aborted);

  m.def("stream_wait", [](uintptr_t st, double timeout_s) {
    py::gil_scoped_release nogil;
    return stream_wait_with_deadline(P_<ihipStream_t>(st), timeout_s, nullptr);
  });

  py::class_<PeerAllreduce>(m, "PeerAllreduce")
      .def(py::init<int, int, int, long, int, double>(), py::arg("world"), py::arg("rank"), py::arg("device"),
           py::arg("capacity"), py::arg("blocks") = 64, py::arg("timeout_s") = 120.0)
      .def("handles", [](PeerAllreduce& p) { return py::bytes(p.handles()); })
      .def("open",
           [](PeerAllreduce& p, std::vector<py::bytes> hs) {
             std::vector<std::string> v;
             for (auto& h : hs) v.emplace_back(std::string(h));
             p.open(v);
           })
      .def("allreduce",
           [](PeerAllreduce& p, uintptr_t data, long n, uintptr_t st, uintptr_t aux64, long n64) {
             p.allreduce(P_<float>(data), n, P_<ihipStream_t>(st), P_<long long>(aux64), n64);
           },
           py::arg("data"), py::arg("n"), py::arg("stream"), py::arg("aux64") = 0, py::arg("n64") = 0)
      .def_static("message_words", &PeerAllreduce::message_words)
      .def("link_local", &PeerAllreduce::link_local)
      .def("status", &PeerAllreduce::status)
      .def("clear_status", &PeerAllreduce::clear_status)
      .def("set_timeout", &PeerAllreduce::set_timeout)
      .def_property_readonly("ready", &PeerAllreduce::ready)
      .def_property_readonly("capacity", &PeerAllreduce::capacity)
      // diagnostics: n 32-bit words of this rank's `out` staging from word `off` (synchronizes)
      .def("peek_out",
           [](PeerAllreduce& p, long off, long n) {
             std::vector<uint32_t> v((size_t)n);
             HIP_CHECK(hipDeviceSynchronize());
             HIP_CHECK(hipMemcpy(v.data(), p.out_local() + off, (size_t)n * 4, hipMemcpyDeviceToHost));
             return v;
           })
      .def_property_readonly("world", &PeerAllreduce::world)
      .def_property_readonly("rank", &PeerAllreduce::rank);

  py::class_<ConvNetTrainer>(m, "ConvNetTrainer")
      .def(py::init<int, py::dict, int, int, int>(), py::arg("device"), py::arg("buffers"),
           py::arg("batch"), py::arg("positions_per_slice") = 4, py::arg("grad_allreduce") = 1)
      .def("set_data", &ConvNetTrainer::set_data, py::arg("x"), py::arg("labels"), py::arg("x_u8") = 0)
      .def("set_comm", [](ConvNetTrainer& t, RcclComm* c) { t.set_comm(c); },
           py::keep_alive<1, 2>())
      .def("set_peer", [](ConvNetTrainer& t, PeerAllreduce* p, bool fold) { t.set_peer_fold(p, fold); },
           py::arg("peer"), py::arg("fold") = false, py::keep_alive<1, 2>())
      .def_property_readonly("folded", &ConvNetTrainer::folded)
      .def("set_sharded", &ConvNetTrainer::set_sharded, py::arg("peer"), py::arg("hred"), py::arg("gbf16") = 0,
           py::keep_alive<1, 2>())
      .def_property_readonly("sharded", &ConvNetTrainer::sharded)
      .def("set_exchange_timeout", &ConvNetTrainer::set_exchange_timeout)
      .def("gather", &ConvNetTrainer::gather)
      .def("restrict_cus", &ConvNetTrainer::restrict_cus, py::arg("part"), py::arg("nparts"))
      .def("metric_tail", &ConvNetTrainer::metric_tail)
      .def("step", &ConvNetTrainer::step, py::call_guard<py::gil_scoped_release>())
      .def("capture", &ConvNetTrainer::capture)
      .def("step_graph_nodes", &ConvNetTrainer::step_graph_nodes, py::arg("steps"))
      .def("run", &ConvNetTrainer::run, py::call_guard<py::gil_scoped_release>())
      .def("capture_final", &ConvNetTrainer::capture_final, py::arg("steps"))
      .def("run_final", &ConvNetTrainer::run_final, py::arg("steps"), py::call_guard<py::gil_scoped_release>())
      .def("warm_final", &ConvNetTrainer::warm_final, py::arg("steps"), py::call_guard<py::gil_scoped_release>())
      .def("phase_times", &ConvNetTrainer::phase_times, py::arg("steps"), py::call_guard<py::gil_scoped_release>())
      .def("flush", &ConvNetTrainer::flush)
      .def("sync", &ConvNetTrainer::sync, py::arg("timeout_s") = 0.0,
           py::call_guard<py::gil_scoped_release>())
      .def("invalidate_graphs", &ConvNetTrainer::invalidate_graphs)
      .def_property_readonly("num_graphs", &ConvNetTrainer::num_graphs)
      .def_property_readonly("num_slices", &ConvNetTrainer::num_slices)
      .def_property_readonly("num_slices_bwd", &ConvNetTrainer::num_slices_bwd)
      .def_property_readonly("batch", &ConvNetTrainer::batch)
      .def_property_readonly("parity", &ConvNetTrainer::parity)
      .def_property_readonly("stream", [](ConvNetTrainer& t) { return reinterpret_cast<uintptr_t>(t.stream()); });

  register_kernel_ops(m);
}
