#include "peer_comm.h"

#include <cstring>
#include <stdexcept>

namespace damd {

#define HIP_CHECK(x)                                                                    \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess)                                                               \
      throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e_) +     \
                               " at " #x);                                              \
  } while (0)

PeerAllreduce::PeerAllreduce(int world, int rank, int device, long capacity, int nblk, double timeout_s)
    : device_(device) {
  if (world < 1 || world > kPeerMaxRanks) throw std::invalid_argument("peer all-reduce: 1..8 ranks");
  if (rank < 0 || rank >= world) throw std::invalid_argument("peer all-reduce: bad rank");
  if (nblk < 1 || nblk > kPeerMaxBlocks) throw std::invalid_argument("peer all-reduce: 1..128 blocks");
  if (capacity < 1) throw std::invalid_argument("peer all-reduce: capacity must be > 0");
  HIP_CHECK(hipSetDevice(device));
  // chunk: floats per (shard, block), multiple of 4 (16-byte vectors)
  long per = (capacity + (long)world * nblk - 1) / ((long)world * nblk);
  a_.chunk = (per + 3) / 4 * 4;
  cap_ = (long)world * nblk * a_.chunk;
  a_.world = world;
  a_.rank = rank;
  a_.nblk = nblk;
  a_.timeout_ticks = (unsigned long long)(timeout_s * 1e8);  // s_memrealtime: 100 MHz
  const size_t bytes = (size_t)cap_ * sizeof(float);
  // staging buffers and flags are exchanged across devices inside one kernel: uncached
  // (MTYPE UC), so no cache holds a stale or dirty copy (see peer_allreduce.hip)
  HIP_CHECK(hipExtMallocWithFlags(reinterpret_cast<void**>(&in_), bytes, hipDeviceMallocUncached));
  HIP_CHECK(hipExtMallocWithFlags(reinterpret_cast<void**>(&out_), bytes, hipDeviceMallocUncached));
  const size_t fbytes = (size_t)2 * kPeerMaxRanks * kPeerMaxBlocks * sizeof(unsigned);
  HIP_CHECK(hipExtMallocWithFlags(reinterpret_cast<void**>(&flags_), fbytes, hipDeviceMallocUncached));
  HIP_CHECK(hipMalloc(&local_, (kPeerMaxBlocks + 1) * sizeof(unsigned)));
  HIP_CHECK(hipMemset(flags_, 0, fbytes));
  HIP_CHECK(hipMemset(local_, 0, (kPeerMaxBlocks + 1) * sizeof(unsigned)));
  HIP_CHECK(hipMemset(in_, 0, bytes));
  HIP_CHECK(hipMemset(out_, 0, bytes));
  HIP_CHECK(hipDeviceSynchronize());
  a_.epoch = local_;
  a_.status = local_ + kPeerMaxBlocks;
  for (int p = 0; p < kPeerMaxRanks; ++p) {
    a_.in[p] = nullptr;
    a_.out[p] = nullptr;
    a_.flags[p] = nullptr;
  }
  a_.in[rank] = in_;
  a_.out[rank] = out_;
  a_.flags[rank] = flags_;
  if (world == 1) opened_ = true;
}

PeerAllreduce::~PeerAllreduce() {
  hipSetDevice(device_);
  hipDeviceSynchronize();
  for (void* p : mapped_) hipIpcCloseMemHandle(p);
  if (in_) hipFree(in_);
  if (out_) hipFree(out_);
  if (flags_) hipFree(flags_);
  if (local_) hipFree(local_);
}

std::string PeerAllreduce::handles() const {
  std::string s;
  void* bufs[3] = {in_, out_, flags_};
  for (void* b : bufs) {
    hipIpcMemHandle_t h;
    HIP_CHECK(hipIpcGetMemHandle(&h, b));
    s.append(reinterpret_cast<const char*>(&h), sizeof(h));
  }
  return s;
}

void PeerAllreduce::open(const std::vector<std::string>& hs) {
  if ((int)hs.size() != a_.world) throw std::invalid_argument("peer all-reduce: one handle blob per rank");
  HIP_CHECK(hipSetDevice(device_));
  for (int p = 0; p < a_.world; ++p) {
    if (p == a_.rank) continue;
    if (hs[p].size() != 3 * sizeof(hipIpcMemHandle_t)) throw std::invalid_argument("peer all-reduce: bad handle");
    void* ptrs[3];
    for (int i = 0; i < 3; ++i) {
      hipIpcMemHandle_t h;
      std::memcpy(&h, hs[p].data() + i * sizeof(h), sizeof(h));
      HIP_CHECK(hipIpcOpenMemHandle(&ptrs[i], h, hipIpcMemLazyEnablePeerAccess));
      mapped_.push_back(ptrs[i]);
    }
    a_.in[p] = static_cast<float*>(ptrs[0]);
    a_.out[p] = static_cast<float*>(ptrs[1]);
    a_.flags[p] = static_cast<unsigned*>(ptrs[2]);
  }
  opened_ = true;
}

void PeerAllreduce::link_local(const std::vector<PeerAllreduce*>& peers) {
  if ((int)peers.size() != a_.world) throw std::invalid_argument("peer all-reduce: one instance per rank");
  for (int p = 0; p < a_.world; ++p) {
    const PeerAllreduce* q = peers[p];
    if (q->a_.rank != p || q->a_.world != a_.world || q->a_.chunk != a_.chunk || q->a_.nblk != a_.nblk)
      throw std::invalid_argument("peer all-reduce: mismatched local peer");
    a_.in[p] = q->in_;
    a_.out[p] = q->out_;
    a_.flags[p] = q->flags_;
  }
  opened_ = true;
}

void PeerAllreduce::allreduce(float* data, long n, hipStream_t st, long long* aux64, long n64) {
  if (!opened_) throw std::runtime_error("peer all-reduce: open() the peers' handles first");
  if (n64 < 0 || (n64 > 0 && !aux64)) throw std::invalid_argument("peer all-reduce: bad int64 segment");
  if (message_words(n, n64) > cap_) throw std::invalid_argument("peer all-reduce: message larger than the capacity");
  if (a_.world == 1) return;
  HIP_CHECK(peer_allreduce_launch(a_, data, n, aux64, n64, st));
}

void PeerAllreduce::allreduce_staged(long n, long n64, hipStream_t st, const long long* aux64) {
  if (!opened_) throw std::runtime_error("peer all-reduce: open() the peers' handles first");
  if (n64 < 0 || message_words(n, n64) > cap_) throw std::invalid_argument("peer all-reduce: bad staged message");
  if (a_.world == 1) {  // the result is the input
    const long nfp = (n + 3) / 4 * 4;
    HIP_CHECK(hipMemcpyAsync(out_, in_, (size_t)(aux64 ? nfp : message_words(n, n64)) * sizeof(float),
                             hipMemcpyDeviceToDevice, st));
    if (aux64)
      HIP_CHECK(hipMemcpyAsync(out_ + nfp, aux64, (size_t)n64 * sizeof(long long), hipMemcpyDeviceToDevice, st));
    return;
  }
  HIP_CHECK(peer_allreduce_staged_launch(a_, n, n64, st, aux64));
}

unsigned PeerAllreduce::status() const {
  unsigned s = 0;
  HIP_CHECK(hipMemcpy(&s, a_.status, sizeof(s), hipMemcpyDeviceToHost));
  return s;
}

void PeerAllreduce::clear_status() { HIP_CHECK(hipMemset(a_.status, 0, sizeof(unsigned))); }

}  // namespace damd
