#include "step_executor.h"

#include <stdexcept>
#include <string>
#include <vector>

namespace damd {

#define HIP_CHECK(x)                                                                    \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess)                                                               \
      throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e_) +     \
                               " at " #x);                                              \
  } while (0)

StepExecutor::StepExecutor(int device) : device_(device) {
  HIP_CHECK(hipSetDevice(device));
  HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
}

StepExecutor::~StepExecutor() {
  invalidate_graphs();
  if (stream_) {
    hipStreamSynchronize(stream_);
    hipStreamDestroy(stream_);
  }
}

void StepExecutor::invalidate_graphs() {
  for (auto& kv : graphs_) hipGraphExecDestroy(kv.second);
  for (auto& kv : finals_) hipGraphExecDestroy(kv.second);
  for (auto& kv : final_graphs_) hipGraphDestroy(kv.second);
  graphs_.clear();
  finals_.clear();
  final_graphs_.clear();
}

void StepExecutor::step(int k) {
  for (int i = 0; i < k; ++i) enqueue_one_step();
}

hipGraphExec_t StepExecutor::capture_steps(int k, bool tail, hipGraph_t* keep) {
  hipGraph_t g = nullptr;
  const int p0 = phase_value();  // the captured steps do not run: the phase stays
  HIP_CHECK(hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal));
  try {
    for (int i = 0; i < k; ++i) enqueue_one_step();
    if (tail) enqueue_tail();
  } catch (...) {
    hipStreamEndCapture(stream_, &g);
    if (g) hipGraphDestroy(g);
    set_phase(p0);
    throw;
  }
  set_phase(p0);
  HIP_CHECK(hipStreamEndCapture(stream_, &g));
  hipGraphExec_t ge = nullptr;
  hipError_t e = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  if (keep && e == hipSuccess) *keep = g;
  else hipGraphDestroy(g);
  HIP_CHECK(e);
  // upload now, so the first replay inside a timed loop does not pay for it
  HIP_CHECK(hipGraphUpload(ge, stream_));
  HIP_CHECK(hipStreamSynchronize(stream_));
  return ge;
}

std::pair<int, int> StepExecutor::step_graph_nodes(int k) {
  hipGraph_t g = nullptr;
  const int p0 = phase_value();
  HIP_CHECK(hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal));
  try {
    for (int i = 0; i < k; ++i) enqueue_one_step();
  } catch (...) {
    hipStreamEndCapture(stream_, &g);
    if (g) hipGraphDestroy(g);
    set_phase(p0);
    throw;
  }
  set_phase(p0);
  HIP_CHECK(hipStreamEndCapture(stream_, &g));
  size_t n = 0;
  hipError_t e = hipGraphGetNodes(g, nullptr, &n);
  std::vector<hipGraphNode_t> nodes(n);
  if (e == hipSuccess && n) e = hipGraphGetNodes(g, nodes.data(), &n);
  int kern = 0;
  for (size_t i = 0; e == hipSuccess && i < n; ++i) {
    hipGraphNodeType t;
    e = hipGraphNodeGetType(nodes[i], &t);
    if (e == hipSuccess && t == hipGraphNodeTypeKernel) ++kern;
  }
  hipGraphDestroy(g);
  HIP_CHECK(e);
  return {kern, (int)n};
}

void StepExecutor::capture(int k) {
  if (k <= 0) return;
  const int p = phase_value();
  if (!graphs_.count(Key{k, p})) graphs_[Key{k, p}] = capture_steps(k, false);
  // a k that moves the phase (e.g. an odd step count of the fused trainer): the variant for
  // the phase a replay ends in is captured NOW too, not lazily inside run() -- which a timed
  // loop would otherwise pay for (capture + instantiate + upload) on its second replay
  const int q = phase_after(p, k, false);
  if (q != p && !graphs_.count(Key{k, q})) {
    set_phase(q);
    try {
      graphs_[Key{k, q}] = capture_steps(k, false);
    } catch (...) {
      set_phase(p);
      throw;
    }
    set_phase(p);
  }
}

void StepExecutor::capture_final(int k) {
  const Key key{k, phase_value()};
  if (k <= 0 || finals_.count(key)) return;
  hipGraph_t g = nullptr;
  finals_[key] = capture_steps(k, true, &g);
  final_graphs_[key] = g;
}

bool StepExecutor::warm_final(int k) {
  auto it = finals_.find(Key{k, phase_value()});
  auto gt = final_graphs_.find(Key{k, phase_value()});
  if (it == finals_.end() || gt == final_graphs_.end()) return false;
  size_t n = 0;
  if (hipGraphGetNodes(gt->second, nullptr, &n) != hipSuccess || n == 0) return false;
  std::vector<hipGraphNode_t> nodes(n);
  if (hipGraphGetNodes(gt->second, nodes.data(), &n) != hipSuccess) return false;
  // off = number of nodes actually disabled: a node whose type cannot be toggled stops the
  // walk, and only [0, off) is re-enabled (the failed node was never disabled)
  size_t off = 0;
  while (off < n && hipGraphNodeSetEnabled(it->second, nodes[off], 0) == hipSuccess) ++off;
  bool ok = off == n;
  if (ok) ok = hipGraphLaunch(it->second, stream_) == hipSuccess && hipStreamSynchronize(stream_) == hipSuccess;
  bool restored = true;
  for (size_t i = 0; i < off; ++i) restored = hipGraphNodeSetEnabled(it->second, nodes[i], 1) == hipSuccess && restored;
  (void)hipGetLastError();
  if (!restored) {  // a half-disabled graph must never be replayed: drop it
    hipGraphExecDestroy(it->second);
    finals_.erase(it);
    hipGraphDestroy(gt->second);
    final_graphs_.erase(gt);
    return false;
  }
  return ok;
}

bool StepExecutor::run_final(int k) {
  const int p = phase_value();
  auto it = finals_.find(Key{k, p});
  if (it == finals_.end()) return false;
  HIP_CHECK(hipGraphLaunch(it->second, stream_));
  set_phase(phase_after(p, k, true));
  return true;
}

void StepExecutor::run(int k) {
  while (k > 0) {
    // the longest captured step count <= k (any phase) ...
    int kk = 0;
    for (auto& kv : graphs_)
      if (kv.first.first <= k && kv.first.first > kk) kk = kv.first.first;
    if (kk == 0) break;
    // ... in the variant for the current phase (captured on first use)
    const int p = phase_value();
    auto it = graphs_.find(Key{kk, p});
    if (it == graphs_.end()) {
      graphs_[Key{kk, p}] = capture_steps(kk, false);
      it = graphs_.find(Key{kk, p});
    }
    HIP_CHECK(hipGraphLaunch(it->second, stream_));
    set_phase(phase_after(p, kk, false));
    k -= kk;
  }
  step(k);
}

void StepExecutor::restrict_cus(int part, int nparts) {
  if (nparts < 2) return;
  if (part < 0 || part >= nparts) throw std::invalid_argument("restrict_cus: bad part");
  hipDeviceProp_t prop;
  HIP_CHECK(hipGetDeviceProperties(&prop, device_));
  const int ncu = prop.multiProcessorCount;
  std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
  for (int cu = part; cu < ncu; cu += nparts) mask[cu / 32] |= 1u << (cu % 32);
  invalidate_graphs();
  HIP_CHECK(hipStreamSynchronize(stream_));
  HIP_CHECK(hipStreamDestroy(stream_));
  stream_ = nullptr;
  // (hipExtStreamCreateWithCUMask takes no flags: the new stream is a BLOCKING stream, i.e.
  // it synchronizes with the legacy null stream, unlike the constructor's non-blocking one.
  // Its users -- ranks sharing one device, one rank per process in the engine -- enqueue no
  // null-stream work between steps (host reads sync first); several ranks in ONE process
  // (tests/test_sharded_inproc_gpu.py) must not queue null-stream work while their steps
  // wait on each other, or the waits serialise until the in-kernel deadline.)
  HIP_CHECK(hipExtStreamCreateWithCUMask(&stream_, (uint32_t)mask.size(), mask.data()));
}

bool StepExecutor::sync(double timeout_s) { return stream_wait_with_deadline(stream_, timeout_s, comm_); }

}  // namespace damd
