// Probe: cost of one in-kernel hand-off of the MNIST step's h sums across 57 workgroups
// (1 per CU, 512 threads): every block adds 64x64 int64 partials (memory-side atomics),
// arrives at a counter, polls it, acquires, and reads the 32 KB sum back -- repeated for
// `iters` steps with double-buffered (parity) accumulators zeroed by atomic exchange.
// Every wait is bounded (s_memrealtime deadline), so a non-resident block cannot hang the
// GPU: the kernel records a timeout and exits.
//
// Build: hipcc --offload-arch=gfx950 -O3 scripts/probe_grid_barrier.hip -o /tmp/probe_gb
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

constexpr int NT = 512;

template <int MODE>  // 0: acquire fence + plain loads; 1: no fence, sc1 (relaxed atomic) loads; 2: barrier only
__global__ __launch_bounds__(NT) void probe(long long* acc, unsigned* ctr, int iters, int* err,
                                           unsigned long long* times, long long* out) {
  const int tid = threadIdx.x, nb = gridDim.x;
  __shared__ int ok;
  long long check = 0;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  const unsigned long long deadline = t0 + 200000000ull;  // 2 s at 100 MHz
  for (int it = 0; it < iters; ++it) {
    // three accumulators: step `it` adds into it % 3; after its barrier nobody reads
    // (it - 1) % 3 any more and nobody adds into it before barrier it + 1: zero it then
    long long* a = acc + (it % 3) * 4096;
    long long* dead = acc + ((it + 2) % 3) * 4096;
    if (MODE != 2)
      for (int j = 0; j < 8; ++j) {  // partials: 8 per thread, one 512-B row per wave instruction
        const int idx = j * NT + tid;
        __hip_atomic_fetch_add(reinterpret_cast<unsigned long long*>(a + idx), (unsigned long long)(blockIdx.x + 1),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned target = (unsigned)nb * (it + 1);
      int good = 1;
      while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memrealtime() > deadline) {
          good = 0;
          atomicOr(err, 1);
          break;
        }
      }
      if (MODE == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      ok = good;
    }
    __syncthreads();
    if (!ok) break;
    if (MODE != 2)
      for (int i = blockIdx.x * NT + tid; i < 4096; i += nb * NT)
        __hip_atomic_exchange(reinterpret_cast<unsigned long long*>(dead + i), 0ull, __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_AGENT);
    if (MODE == 2) continue;
    long long s = 0;
    for (int j = 0; j < 8; ++j) {
      const int idx = j * NT + tid;
      if (MODE == 0) s += a[idx];
      else s += (long long)__hip_atomic_load(reinterpret_cast<unsigned long long*>(a + idx), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
    }
    check += s;
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (tid == 0) times[blockIdx.x] = t1 - t0;
  out[blockIdx.x * NT + tid] = check;
}

int main(int argc, char** argv) {
  const int nb = argc > 1 ? atoi(argv[1]) : 57, iters = argc > 2 ? atoi(argv[2]) : 2000;
  long long *acc, *out;
  unsigned* ctr;
  int* err;
  unsigned long long* times;
  CK(hipMalloc(&acc, 3 * 4096 * 8));
  CK(hipMalloc(&out, (size_t)nb * NT * 8));
  CK(hipMalloc(&ctr, 4));
  CK(hipMalloc(&err, 4));
  CK(hipMalloc(&times, nb * 8));
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  if (nb > ncu) {
    printf("grid %d > %d CUs: refusing (blocks must be co-resident)\n", nb, ncu);
    return 1;
  }
  for (int mode = 0; mode < 3; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipMemset(acc, 0, 3 * 4096 * 8));
      CK(hipMemset(ctr, 0, 4));
      CK(hipMemset(err, 0, 4));
      CK(hipDeviceSynchronize());
      hipEvent_t e0, e1;
      CK(hipEventCreate(&e0));
      CK(hipEventCreate(&e1));
      CK(hipEventRecord(e0, 0));
      if (mode == 0) hipLaunchKernelGGL(probe<0>, dim3(nb), dim3(NT), 0, 0, acc, ctr, iters, err, times, out);
      else if (mode == 1) hipLaunchKernelGGL(probe<1>, dim3(nb), dim3(NT), 0, 0, acc, ctr, iters, err, times, out);
      else hipLaunchKernelGGL(probe<2>, dim3(nb), dim3(NT), 0, 0, acc, ctr, iters, err, times, out);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      int herr = 0;
      CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
      std::vector<long long> o((size_t)nb * NT);
      CK(hipMemcpy(o.data(), out, o.size() * 8, hipMemcpyDeviceToHost));
      // every read of a completed sum sees sum_{b=1..nb} b per element
      const long long per = (long long)nb * (nb + 1) / 2;
      long long bad = 0;
      for (size_t i = 0; i < o.size(); ++i) bad += o[i] != (mode == 2 ? 0 : per * 8 * iters);
      printf("mode %s grid %d iters %d: %.3f us per hand-off (kernel %.3f ms), timeout %d, wrong sums %lld\n",
             mode == 0 ? "acquire+plain" : (mode == 1 ? "sc1-loads" : "barrier-only"), nb, iters, ms * 1e3 / iters, ms, herr, bad);
    }
  }
  return 0;
}
