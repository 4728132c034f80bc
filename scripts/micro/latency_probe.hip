// Global-load latency on gfx950: one lane chases a dependent pointer chain (stride 4 KB,
// permuted) through a buffer of the given size; shader clocks (s_memtime) per load.  The
// first pass is cold (after a host write), later passes show the L2 / MALL / HBM level.
// Build here:  hipcc -O3 --offload-arch=gfx950 scripts/micro/latency_probe.hip -o build/latency_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#include <random>

__global__ void chase(const unsigned* __restrict__ next, int n, unsigned long long* t, unsigned* sink) {
  unsigned i = 0;
  const unsigned long long m0 = __builtin_amdgcn_s_memtime();
  for (int k = 0; k < n; ++k) i = __builtin_nontemporal_load(next + i) + 0u * k, i = next[i];
  const unsigned long long m1 = __builtin_amdgcn_s_memtime();
  t[0] = m1 - m0;
  sink[0] = i;
}

int main() {
  unsigned long long* t;
  unsigned* sink;
  (void)hipMalloc(&t, 8);
  (void)hipMalloc(&sink, 4);
  for (size_t mb : {1, 8, 64, 512, 4096}) {
    const size_t n = mb * 1024 * 1024 / 4, stride = 1024;  // 4 KB apart
    const size_t m = n / stride;
    std::vector<unsigned> h(n, 0);
    std::vector<unsigned> perm(m);
    for (size_t i = 0; i < m; ++i) perm[i] = (unsigned)i;
    std::shuffle(perm.begin() + 1, perm.end(), std::mt19937(7));
    for (size_t i = 0; i < m; ++i) h[perm[i] * stride] = perm[(i + 1) % m] * stride;
    unsigned* d;
    (void)hipMalloc(&d, n * 4);
    (void)hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice);
    const int loads = (int)std::min<size_t>(m, 2000);
    for (int pass = 0; pass < 3; ++pass) {
      hipLaunchKernelGGL(chase, dim3(1), dim3(1), 0, 0, d, loads / 2, t, sink);
      (void)hipDeviceSynchronize();
      unsigned long long c;
      (void)hipMemcpy(&c, t, 8, hipMemcpyDeviceToHost);
      printf("%5zu MB pass %d: %7.1f clk per load (%.0f ns at 2.4 GHz)\n", mb, pass, (double)c / loads,
             (double)c / loads / 2.4);
    }
    (void)hipFree(d);
  }
  return 0;
}
