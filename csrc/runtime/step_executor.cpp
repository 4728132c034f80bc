#include "step_executor.h"

#include <stdexcept>
#include <string>

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
  graphs_.clear();
}

void StepExecutor::step(int k) {
  for (int i = 0; i < k; ++i) enqueue_one_step();
}

void StepExecutor::capture(int k) {
  if (k <= 0 || graphs_.count(k)) return;
  hipGraph_t g = nullptr;
  HIP_CHECK(hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal));
  try {
    for (int i = 0; i < k; ++i) enqueue_one_step();
  } catch (...) {
    hipStreamEndCapture(stream_, &g);
    if (g) hipGraphDestroy(g);
    throw;
  }
  HIP_CHECK(hipStreamEndCapture(stream_, &g));
  hipGraphExec_t ge = nullptr;
  hipError_t e = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  hipGraphDestroy(g);
  HIP_CHECK(e);
  // upload now, so the first replay inside a timed loop does not pay for it
  HIP_CHECK(hipGraphUpload(ge, stream_));
  HIP_CHECK(hipStreamSynchronize(stream_));
  graphs_[k] = ge;
}

void StepExecutor::run(int k) {
  while (k > 0) {
    auto it = graphs_.upper_bound(k);  // first key > k
    if (it == graphs_.begin()) break;  // no graph <= k
    --it;
    HIP_CHECK(hipGraphLaunch(it->second, stream_));
    k -= it->first;
  }
  step(k);
}

bool StepExecutor::sync(double timeout_s) { return stream_wait_with_deadline(stream_, timeout_s, comm_); }

}  // namespace damd
