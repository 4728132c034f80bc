// Native RCCL communicator (data plane of MultiWorkerMirroredStrategy on MI355X).
//
// The reference reduces gradients with TF's CPU ring over gRPC
// (reference README.md:395 rpc_layer='grpc', :398 CollectiveCommunication.AUTO,
// :403 "Collective batch_all_reduce: 6 all-reduces").  Here the same SUM all-reduce is
// one ncclAllReduce over xGMI on the trainer's HIP stream, so it can be captured into
// the per-step hipGraph.  Bootstrap (unique-id exchange) is done by the Python layer
// over the torch.distributed TCPStore, which is the only host-network crossing.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <string>
#include <vector>

namespace damd {

std::string rccl_unique_id();  // 128 raw bytes

class RcclComm {
 public:
  RcclComm(int nranks, int rank, const std::string& uid, int device);
  ~RcclComm();
  int nranks() const { return nranks_; }
  int rank() const { return rank_; }
  ncclComm_t comm() const { return comm_; }
  // ranks as RCCL itself counts them (ncclCommCount)
  int comm_count() const;
  // dtype: 0=f32 1=bf16 2=f16 3=i32 4=f64 5=i64 ; op: 0=sum 1=max 2=min 3=avg
  void allreduce(void* sendbuf, void* recvbuf, size_t count, int dtype, int op, hipStream_t st);
  // in-place SUM of n fp32 values and n64 int64 values as ONE grouped RCCL launch
  void allreduce_f32_i64(float* data, size_t n, long long* aux, size_t n64, hipStream_t st);
  void broadcast(void* buf, size_t count, int dtype, int root, hipStream_t st);
  void allgather(const void* sendbuf, void* recvbuf, size_t count, int dtype, hipStream_t st);
  void reduce_scatter(const void* sendbuf, void* recvbuf, size_t count, int dtype, int op,
                      hipStream_t st);
  void abort();
  bool aborted() const { return aborted_.load(); }

 private:
  int nranks_, rank_, device_;
  ncclComm_t comm_ = nullptr;
  std::atomic<bool> aborted_{false};
};

// Wait for all work queued on `st` with a deadline; on timeout abort `comm` (if any)
// and return false.  This is the collective watchdog (SURVEY.md §5 failure detection).
bool stream_wait_with_deadline(hipStream_t st, double timeout_s, RcclComm* comm);

}  // namespace damd
