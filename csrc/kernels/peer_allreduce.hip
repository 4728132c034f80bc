// xGMI peer-to-peer two-shot all-reduce kernel (algorithm and safety argument:
// csrc/runtime/peer_comm.h).
//
// Memory-model notes (gfx950):
//  - `in`, `out` and the flag words are allocated uncached (hipDeviceMallocUncached,
//    MTYPE UC): every access goes to the owning GPU's memory, nothing is held in any
//    L1/L2, so cross-device visibility needs no L2 write-back or invalidate (a
//    system-scope release/acquire costs a whole-L2 buffer_wbl2 / buffer_inv per block:
//    ~2-6 us each, measured as 21 us per call with them vs the UC form below).
//  - Publish: every wave drains its stores (s_waitcnt vmcnt(0)) -> workgroup barrier ->
//    thread 0 stores the flag (relaxed, system scope) into every rank's flag array.
//  - Consume: threads 0..W-1 poll one source each (relaxed system-scope loads + s_sleep)
//    -> workgroup barrier -> loads (the barrier also keeps the compiler from hoisting them).
//  - The local gradient itself is ordinary (cached) memory: it is only read and written
//    by this device, in stream order with the kernels around this one.
//  - Reductions are in a fixed peer order, so all ranks end bitwise identical.
#include "damd_common.h"
#include "peer_comm.h"

namespace damd {
namespace {

constexpr int NT = 256;

__device__ __forceinline__ unsigned* flag_slot(unsigned* base, int phase, int src, int blk) {
  return base + ((size_t)phase * kPeerMaxRanks + src) * kPeerMaxBlocks + blk;
}

// thread 0: publish this block's phase to every rank (own flags included: uniform waits)
__device__ __forceinline__ void signal_all(const PeerArgs& a, int phase, unsigned e) {
  damd_publish_drain();  // this wave's UC stores have landed
  __syncthreads();
  DAMD_PUBLISH_WG();
  if (threadIdx.x == 0) {
    for (int p = 0; p < a.world; ++p)
      __hip_atomic_store(flag_slot(a.flags[p], phase, a.rank, blockIdx.x), e, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// threads 0..world-1 each wait for one source rank's flag of this block
__device__ __forceinline__ void wait_all(const PeerArgs& a, int phase, unsigned e) {
  const int t = threadIdx.x;
  if (t < a.world) {
    unsigned* f = flag_slot(a.flags[a.rank], phase, t, blockIdx.x);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < e) {
      __builtin_amdgcn_s_sleep(2);
      const unsigned long long dt = __builtin_amdgcn_s_memrealtime() - t0;
      if (dt > a.timeout_ticks) {
        __hip_atomic_fetch_or(a.status, 1u << phase, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      // past 1 ms: give up at once when an earlier wait already expired (a broken exchange
      // then costs one deadline, not one per wait of every later call)
      if (dt > 100000ull && __hip_atomic_load(a.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) break;
    }
  }
  __syncthreads();
}

// Message word g (a multiple of 4): fp32 data below nfp = n rounded up to 4, then the
// int64 segment (two words per value) -- a 16-byte word is never mixed.
__device__ __forceinline__ float4 msg_load(const float* __restrict__ data, long n, const long long* __restrict__ aux,
                                           long n64, long nfp, long g) {
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  if (g < nfp) {
    if (g + 3 < n) {
      v = *reinterpret_cast<const float4*>(data + g);
    } else {
      v.x = g < n ? data[g] : 0.f;
      v.y = g + 1 < n ? data[g + 1] : 0.f;
      v.z = g + 2 < n ? data[g + 2] : 0.f;
    }
  } else {
    const long j = (g - nfp) / 2;
    const long long q0 = j < n64 ? aux[j] : 0, q1 = j + 1 < n64 ? aux[j + 1] : 0;
    v = make_float4(__int_as_float((int)(q0 & 0xffffffffLL)), __int_as_float((int)(q0 >> 32)),
                    __int_as_float((int)(q1 & 0xffffffffLL)), __int_as_float((int)(q1 >> 32)));
  }
  return v;
}
__device__ __forceinline__ void msg_store(float* __restrict__ data, long n, long long* __restrict__ aux, long n64,
                                          long nfp, long g, float4 v) {
  if (g < nfp) {
    if (g + 3 < n) {
      *reinterpret_cast<float4*>(data + g) = v;
    } else {
      if (g < n) data[g] = v.x;
      if (g + 1 < n) data[g + 1] = v.y;
      if (g + 2 < n) data[g + 2] = v.z;
    }
  } else {
    const long j = (g - nfp) / 2;
    if (j < n64) aux[j] = (long long)(((unsigned long long)__float_as_uint(v.y) << 32) | __float_as_uint(v.x));
    if (j + 1 < n64) aux[j + 1] = (long long)(((unsigned long long)__float_as_uint(v.w) << 32) | __float_as_uint(v.z));
  }
}
__device__ __forceinline__ float4 msg_add(float4 a, float4 b, bool i64) {
  if (i64) {
    const unsigned long long a0 = ((unsigned long long)__float_as_uint(a.y) << 32) | __float_as_uint(a.x);
    const unsigned long long a1 = ((unsigned long long)__float_as_uint(a.w) << 32) | __float_as_uint(a.z);
    const unsigned long long b0 = ((unsigned long long)__float_as_uint(b.y) << 32) | __float_as_uint(b.x);
    const unsigned long long b1 = ((unsigned long long)__float_as_uint(b.w) << 32) | __float_as_uint(b.z);
    const unsigned long long s0 = a0 + b0, s1 = a1 + b1;
    return make_float4(__uint_as_float((unsigned)s0), __uint_as_float((unsigned)(s0 >> 32)),
                       __uint_as_float((unsigned)s1), __uint_as_float((unsigned)(s1 >> 32)));
  }
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

// staged: the caller already wrote the message into own `in` and reads the result from own
// `out` (the fused trainer's folded step): phases A and D are skipped, the flags alone
// order the exchange (stream order covers the local side, see peer_comm.h).  With `aux`
// the int64 segment still lives in the caller's memory: phase A copies just that part.
__global__ __launch_bounds__(NT) void peer_allreduce_k(PeerArgs a, float* __restrict__ data, long n,
                                                       long long* __restrict__ aux, long n64, int staged) {
  const int b = blockIdx.x, t = threadIdx.x, W = a.world;
  const long chunk = a.chunk, shard = chunk * a.nblk;
  const unsigned e = a.epoch[b] + 1;
  const long c4 = chunk / 4;
  const long nfp = (n + 3) / 4 * 4;

  // A: local message -> own `in` (chunk set b), zero beyond the message
  float4* in_own = reinterpret_cast<float4*>(a.in[a.rank]);
  if (!staged) {
    for (int s = 0; s < W; ++s) {
      const long base = s * shard + (long)b * chunk;
      for (long i = t; i < c4; i += NT) in_own[base / 4 + i] = msg_load(data, n, aux, n64, nfp, base + 4 * i);
    }
  } else if (aux != nullptr) {  // the int64 words of this block's chunk set only
    const long a0 = nfp, a1 = nfp + (2 * n64 + 3) / 4 * 4;
    for (int s = 0; s < W; ++s) {
      const long base = s * shard + (long)b * chunk;
      const long lo = max(base, a0), hi = min(base + chunk, a1);
      for (long g = lo + 4 * t; g < hi; g += 4 * NT) in_own[g / 4] = msg_load(data, n, aux, n64, nfp, g);
    }
  }
  signal_all(a, 0, e);
  wait_all(a, 0, e);

  // B: reduce chunk (rank, b) over every rank's `in`, broadcast into every `out`
  {
    const long base4 = (a.rank * shard + (long)b * chunk) / 4;
    for (long i = t; i < c4; i += NT) {
      float4 v[kPeerMaxRanks];
#pragma unroll
      for (int p = 0; p < kPeerMaxRanks; ++p)
        if (p < W) v[p] = reinterpret_cast<const float4*>(a.in[p])[base4 + i];
      const bool i64 = 4 * (base4 + i) >= nfp;
      float4 acc = v[0];
#pragma unroll
      for (int p = 1; p < kPeerMaxRanks; ++p)
        if (p < W) acc = msg_add(acc, v[p], i64);
#pragma unroll
      for (int p = 0; p < kPeerMaxRanks; ++p)
        if (p < W) reinterpret_cast<float4*>(a.out[p])[base4 + i] = acc;
    }
  }
  signal_all(a, 1, e);
  wait_all(a, 1, e);

  // D: own `out` (chunk set b) -> local gradient
  const float4* out_own = reinterpret_cast<const float4*>(a.out[a.rank]);
  for (int s = 0; s < W && !staged; ++s) {
    const long base = s * shard + (long)b * chunk;
    for (long i = t; i < c4; i += NT) msg_store(data, n, aux, n64, nfp, base + 4 * i, out_own[base / 4 + i]);
  }
  if (t == 0) a.epoch[b] = e;
}

}  // namespace

hipError_t peer_allreduce_launch(const PeerArgs& a, float* data, long n, long long* aux64, long n64, hipStream_t st) {
  if (a.world < 1 || a.world > kPeerMaxRanks || a.nblk < 1 || a.nblk > kPeerMaxBlocks || a.chunk % 4)
    return hipErrorInvalidValue;
  if ((long)a.world * a.nblk * a.chunk < (n + 3) / 4 * 4 + 2 * n64) return hipErrorInvalidValue;
  if (reinterpret_cast<uintptr_t>(data) % 16) return hipErrorInvalidValue;
  hipLaunchKernelGGL(peer_allreduce_k, dim3(a.nblk), dim3(NT), 0, st, a, data, n, aux64, n64, 0);
  return hipGetLastError();
}

hipError_t peer_allreduce_staged_launch(const PeerArgs& a, long n, long n64, hipStream_t st, const long long* aux64) {
  if (a.world < 1 || a.world > kPeerMaxRanks || a.nblk < 1 || a.nblk > kPeerMaxBlocks || a.chunk % 4)
    return hipErrorInvalidValue;
  if ((long)a.world * a.nblk * a.chunk < (n + 3) / 4 * 4 + 2 * n64) return hipErrorInvalidValue;
  hipLaunchKernelGGL(peer_allreduce_k, dim3(a.nblk), dim3(NT), 0, st, a, nullptr, n,
                     const_cast<long long*>(aux64), n64, 1);
  return hipGetLastError();
}

}  // namespace damd
