// Diagnostic kernels (scheduling probes, scripts/probe_graph_branches.py): a grid of blocks
// that each hold their CU for `ticks` s_memrealtime ticks (100 MHz), block 0 recording its
// start / end.  Used to see which captured-graph branches the HIP runtime lets run
// concurrently (e.g. a gradient all-reduce node beside the backward kernels).
#include <hip/hip_runtime.h>

namespace damd {
namespace {

__global__ __launch_bounds__(64) void spin_stamp_k(long long ticks, unsigned long long* __restrict__ out, int slot) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long t = t0;
  while ((long long)(t - t0) < ticks) {
    __builtin_amdgcn_s_sleep(2);
    t = __builtin_amdgcn_s_memrealtime();
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && out != nullptr) {
    out[2 * slot] = t0;
    out[2 * slot + 1] = t;
  }
}

}  // namespace

hipError_t spin_stamp(long long ticks, int blocks, unsigned long long* out, int slot, hipStream_t s) {
  if (blocks < 1 || ticks < 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(spin_stamp_k, dim3(blocks), dim3(64), 0, s, ticks, out, slot);
  return hipGetLastError();
}

}  // namespace damd
