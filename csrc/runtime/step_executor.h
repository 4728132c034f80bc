// Native step executor: owns a HIP stream, enqueues one training step (kernels +
// optional RCCL gradient all-reduce), and captures k back-to-back steps into a
// hipGraph that is replayed by the fit loop.  This replaces the reference's
// tf.function tracing (reference README.md:309 — epoch 1 pays tracing) with HIP graph
// capture: the host cost per k steps is one hipGraphLaunch.
#pragma once
#include <hip/hip_runtime.h>

#include <functional>
#include <map>
#include <utility>
#include <memory>

#include "comm.h"
#include "peer_comm.h"

namespace damd {

struct Ctrl;

class StepExecutor {
 public:
  explicit StepExecutor(int device);
  virtual ~StepExecutor();

  hipStream_t stream() const { return stream_; }
  void set_comm(RcclComm* comm) { comm_ = comm; invalidate_graphs(); }
  RcclComm* comm() const { return comm_; }
  // native xGMI all-reduce for the per-step gradient (takes precedence over RCCL)
  void set_peer(PeerAllreduce* p) { peer_ = p; invalidate_graphs(); }
  PeerAllreduce* peer() const { return peer_; }

  // Enqueue k steps eagerly (one host launch per kernel).
  void step(int k);
  // Capture k steps into a graph (cached by k).
  void capture(int k);
  // Run k steps: greedily replay the largest captured graph <= remaining, eager tail.
  void run(int k);
  // k steps followed by enqueue_tail() (e.g. the deferred-update flush) as ONE graph:
  // a timed run of k steps is then one replay (a graph boundary costs ~4.5 us, an eager
  // launch after a graph ~10 us).  run_final returns false if no such graph was captured.
  void capture_final(int k);
  bool run_final(int k);
  // One replay of the final graph with every node disabled (nothing executes): pays the
  // first-launch cost of the graph outside a timed window.  False if unsupported.
  bool warm_final(int k);
  // Block until the stream drains; false on watchdog timeout (comm aborted).
  bool sync(double timeout_s);
  // Several ranks sharing ONE device (the single-GPU rehearsal of a multi-GPU run): this
  // rank's step stream is limited to every nparts-th CU starting at `part`, so a rank's
  // blocks that spin on another rank's message can never occupy the CUs the other rank
  // needs to produce it.  (One rank per GPU -- the real deployment -- never calls this.)
  void restrict_cus(int part, int nparts);
  void invalidate_graphs();
  int num_graphs() const { return (int)graphs_.size(); }
  // host-side step phase (e.g. the fused trainer's parity): graphs are captured per (k,
  // phase) because their kernel arguments depend on it; a replay advances it
  int phase() const { return phase_value(); }
  // (kernel nodes, all nodes) of a k-step graph, captured and discarded: the launch contract
  // of a step (e.g. two kernels per step at any world size for the fused MNIST trainer)
  std::pair<int, int> step_graph_nodes(int k);

 protected:
  virtual void enqueue_one_step() = 0;
  virtual void enqueue_tail() {}
  // phase bookkeeping (default: a single phase): the phase before a step, restoring it after
  // a capture (capturing enqueues steps that do not run), and the phase after k steps (+ tail)
  virtual int phase_value() const { return 0; }
  virtual void set_phase(int) {}
  virtual int phase_after(int p, int, bool) const { return p; }
  hipStream_t stream_ = nullptr;
  RcclComm* comm_ = nullptr;
  PeerAllreduce* peer_ = nullptr;
  int device_;

 private:
  using Key = std::pair<int, int>;  // (steps, phase at the start)
  std::map<Key, hipGraphExec_t> graphs_;
  std::map<Key, hipGraphExec_t> finals_;
  std::map<Key, hipGraph_t> final_graphs_;  // kept for the node handles (warm_final)
  hipGraphExec_t capture_steps(int k, bool tail, hipGraph_t* keep = nullptr);
};

}  // namespace damd
