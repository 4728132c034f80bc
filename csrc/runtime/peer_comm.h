// Native xGMI peer-to-peer all-reduce for the latency-bound per-step gradient reduction
// of the data-parallel trainers (MultiWorkerMirroredStrategy, reference README.md:403
// "Collective batch_all_reduce" -- there a TF CPU ring over gRPC, :395/:398).
//
// Why not RCCL for this message: the fused MNIST step all-reduces 1.39 MB per step
// (SURVEY.md §2.10), which is latency-bound on 8 GPUs; its cost sits on the critical
// path of a ~30 us step.  Every MI355X has a direct xGMI link to each of its 7 peers, so
// a two-shot algorithm over IPC-mapped peer buffers needs exactly one hop per phase:
//
//   block b of rank r (all ranks run the same grid of NB blocks):
//   A  copy its chunk set {(shard s, chunk b) : s < W} of the local gradient into the
//      exported `in` buffer; signal flag[0][r][b] on every peer
//   B  wait flag[0][p][b] from every peer p; reduce chunk (r, b) over all W peers' `in`
//      (fixed order p = 0..W-1, so the result is bitwise identical everywhere);
//      write it into chunk (r, b) of every peer's `out`; signal flag[1][r][b]
//   D  wait flag[1][p][b] from every peer; copy its chunk set of `out` back into the
//      local gradient.
//
// Blocks only synchronise with the same-index block of the peers (no intra-GPU grid
// barrier).  Buffer reuse across steps is safe without double buffering: a rank
// rewrites `in` chunk set b (step t+1, phase A) only after phase D's wait of step t,
// i.e. after every peer's block b has finished reading it in phase B of step t; `out`
// chunk (r, b) is rewritten in phase B of step t+1 only after every peer signalled
// phase A of t+1, i.e. finished phase D of t.  Flags carry a per-block epoch that lives
// in device memory, so the kernel is capturable into a hipGraph and replayable.
//
// All exchanged buffers are uncached device memory (coherent across devices without L2
// fences; see peer_allreduce.hip).  Every wait is bounded (s_memrealtime deadline): on expiry the block records an error
// in `status` and proceeds, so a missing peer can never hang the GPU; the host checks
// `status` (check()) and the engine falls back / raises.
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

namespace damd {

constexpr int kPeerMaxRanks = 8;
constexpr int kPeerMaxBlocks = 128;

struct PeerArgs {
  float* in[kPeerMaxRanks];          // rank p's exported input staging (mapped here)
  float* out[kPeerMaxRanks];         // rank p's exported result staging
  unsigned* flags[kPeerMaxRanks];    // rank p's flag words [2][kPeerMaxRanks][kPeerMaxBlocks]
  unsigned* epoch;                   // local per-block epoch [kPeerMaxBlocks]
  unsigned* status;                  // local error word (0 = ok)
  int world, rank, nblk;
  long chunk;                        // floats per (shard, block) chunk, multiple of 4
  unsigned long long timeout_ticks;  // s_memrealtime ticks (100 MHz)
};

// Message of one call: n fp32 values at `data`, then (optionally) n64 int64 values at
// `aux64` (fixed-point accumulators, summed exactly as integers) starting at the next
// 16-byte word boundary; every rank ends with the same bits.
hipError_t peer_allreduce_launch(const PeerArgs& a, float* data, long n, long long* aux64, long n64, hipStream_t st);
// staged: the fp32 part of the message is already in `in` of this rank, the result stays in
// `out`; aux64 (may be null: already staged too) is copied into `in` by the kernel itself
hipError_t peer_allreduce_staged_launch(const PeerArgs& a, long n, long n64, hipStream_t st,
                                        const long long* aux64 = nullptr);

class PeerAllreduce {
 public:
  // capacity: max floats per all-reduce; nblk: blocks per rank (<= kPeerMaxBlocks)
  PeerAllreduce(int world, int rank, int device, long capacity, int nblk, double timeout_s);
  ~PeerAllreduce();
  int world() const { return a_.world; }
  int rank() const { return a_.rank; }
  long capacity() const { return cap_; }
  // 3 x 64-byte IPC handles (in, out, flags) of this rank's exported buffers
  std::string handles() const;
  // map every peer's buffers (handles[p] from rank p, own entry ignored)
  void open(const std::vector<std::string>& handles);
  // test/benchmark only: peers that live in THIS process on the same device (no IPC)
  void link_local(const std::vector<PeerAllreduce*>& peers);
  bool ready() const { return opened_; }
  // in-place SUM all-reduce of n fp32 values at `data` (and n64 int64 values at `aux64`)
  // on `st` (capturable)
  void allreduce(float* data, long n, hipStream_t st, long long* aux64 = nullptr, long n64 = 0);
  // the same exchange for a message the caller has already written into this rank's `in`
  // staging (n fp32 words, then the int64 segment at the next 16-byte word); the result is
  // left in `out` (same layout) -- no copy-in / copy-out passes.  The caller writes `in`
  // only after this call's previous instance completed on its stream and reads `out` only
  // after this one did (stream order), which is what keeps the buffer reuse safe.
  // aux64: the int64 segment lives in the caller's own (cached) memory instead -- e.g.
  // accumulated there by atomics, which must not target the uncached staging -- and the
  // kernel copies it into `in` (n64 values, a few KB) before it signals.
  void allreduce_staged(long n, long n64, hipStream_t st, const long long* aux64 = nullptr);
  // the pointer table of every rank's mapped staging (for kernels that exchange through it
  // directly, e.g. the sharded MNIST step)
  const PeerArgs& args() const { return a_; }
  float* in_local() const { return in_; }
  float* out_local() const { return out_; }
  // message words (fp32 slots) of a call with n floats and n64 int64 values
  static long message_words(long n, long n64) { return (n + 3) / 4 * 4 + 2 * n64; }
  // 0 = every wait so far completed; otherwise a wait timed out (peer missing / wedged)
  unsigned status() const;
  void clear_status();
  void set_timeout(double timeout_s) { a_.timeout_ticks = (unsigned long long)(timeout_s * 1e8); }

 private:
  PeerArgs a_{};
  int device_;
  long cap_;
  bool opened_ = false;
  float* in_ = nullptr;
  float* out_ = nullptr;
  unsigned* flags_ = nullptr;
  unsigned* local_ = nullptr;  // epoch[kPeerMaxBlocks] + status
  std::vector<void*> mapped_;
};

}  // namespace damd
