#include "comm.h"

#include <chrono>
#include <cstring>
#include <stdexcept>
#include <thread>

namespace damd {

#define RCCL_CHECK(x)                                                                   \
  do {                                                                                  \
    ncclResult_t r_ = (x);                                                              \
    if (r_ != ncclSuccess)                                                              \
      throw std::runtime_error(std::string("RCCL error: ") + ncclGetErrorString(r_) +  \
                               " at " #x);                                              \
  } while (0)
#define HIP_CHECK(x)                                                                    \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess)                                                               \
      throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e_) +     \
                               " at " #x);                                              \
  } while (0)

static ncclDataType_t to_nccl_dtype(int d) {
  switch (d) {
    case 0: return ncclFloat32;
    case 1: return ncclBfloat16;
    case 2: return ncclFloat16;
    case 3: return ncclInt32;
    case 4: return ncclFloat64;
    case 5: return ncclInt64;
    default: throw std::invalid_argument("unsupported dtype code");
  }
}
static ncclRedOp_t to_nccl_op(int o) {
  switch (o) {
    case 0: return ncclSum;
    case 1: return ncclMax;
    case 2: return ncclMin;
    case 3: return ncclAvg;
    default: throw std::invalid_argument("unsupported reduce op code");
  }
}

std::string rccl_unique_id() {
  ncclUniqueId id;
  RCCL_CHECK(ncclGetUniqueId(&id));
  return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
}

RcclComm::RcclComm(int nranks, int rank, const std::string& uid, int device)
    : nranks_(nranks), rank_(rank), device_(device) {
  if (uid.size() != sizeof(ncclUniqueId)) throw std::invalid_argument("bad RCCL unique id size");
  ncclUniqueId id;
  std::memcpy(&id, uid.data(), sizeof(id));
  HIP_CHECK(hipSetDevice(device));
  RCCL_CHECK(ncclCommInitRank(&comm_, nranks, id, rank));
}

RcclComm::~RcclComm() {
  if (comm_) {
    if (aborted_.load()) ncclCommAbort(comm_);
    else ncclCommDestroy(comm_);
    comm_ = nullptr;
  }
}

void RcclComm::allreduce(void* s, void* r, size_t n, int dt, int op, hipStream_t st) {
  RCCL_CHECK(ncclAllReduce(s, r, n, to_nccl_dtype(dt), to_nccl_op(op), comm_, st));
}
void RcclComm::broadcast(void* buf, size_t n, int dt, int root, hipStream_t st) {
  RCCL_CHECK(ncclBroadcast(buf, buf, n, to_nccl_dtype(dt), root, comm_, st));
}
void RcclComm::allgather(const void* s, void* r, size_t n, int dt, hipStream_t st) {
  RCCL_CHECK(ncclAllGather(s, r, n, to_nccl_dtype(dt), comm_, st));
}
void RcclComm::reduce_scatter(const void* s, void* r, size_t n, int dt, int op, hipStream_t st) {
  RCCL_CHECK(ncclReduceScatter(s, r, n, to_nccl_dtype(dt), to_nccl_op(op), comm_, st));
}
void RcclComm::abort() {
  if (!aborted_.exchange(true) && comm_) {
    ncclCommAbort(comm_);
    comm_ = nullptr;
  }
}

bool stream_wait_with_deadline(hipStream_t st, double timeout_s, RcclComm* comm) {
  // No deadline: the runtime's own wait returns as soon as the stream drains (a sleeping
  // poll overshoots a ~30 us training step by up to its sleep quantum).
  if (timeout_s <= 0) {
    HIP_CHECK(hipStreamSynchronize(st));
    return true;
  }
  auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    hipError_t q = hipStreamQuery(st);
    if (q == hipSuccess) return true;
    if (q != hipErrorNotReady) HIP_CHECK(q);
    double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (el > timeout_s) {
      if (comm) comm->abort();
      return false;
    }
    // busy-poll the first 2 ms (step-sized waits), then back off to 20 us sleeps
    if (el > 2e-3) std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}

void RcclComm::allreduce_f32_i64(float* data, size_t n, long long* aux, size_t n64, hipStream_t st) {
  RCCL_CHECK(ncclGroupStart());
  RCCL_CHECK(ncclAllReduce(data, data, n, ncclFloat32, ncclSum, comm_, st));
  if (n64) RCCL_CHECK(ncclAllReduce(aux, aux, n64, ncclInt64, ncclSum, comm_, st));
  RCCL_CHECK(ncclGroupEnd());
}

int RcclComm::comm_count() const {
  int n = 0;
  RCCL_CHECK(ncclCommCount(comm_, &n));
  return n;
}

}  // namespace damd
