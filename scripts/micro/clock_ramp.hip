// Does the shader clock ramp after idle?  After a host sleep, a chain of short kernels
// (each ~20 us of dependent FMAs) reports its own clock rate (s_memtime / s_memrealtime).
// Build here:  hipcc -O3 --offload-arch=gfx950 scripts/micro/clock_ramp.hip -o build/clock_ramp
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <thread>

__global__ void k(float* out, unsigned long long* t, int n, int slot) {
  float a = threadIdx.x * 1e-3f, b = 1.0001f;
  const unsigned long long m0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < n; ++i) asm volatile("v_fma_f32 %0, %0, %1, 1.0" : "+v"(a) : "v"(b));
  const unsigned long long m1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a;
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    t[2 * slot] = m1 - m0;
    t[2 * slot + 1] = r1 - r0;
  }
}

int main() {
  float* out;
  unsigned long long* t;
  (void)hipMalloc(&out, 256 * 512 * sizeof(float));
  (void)hipMalloc(&t, 2 * 64 * sizeof(unsigned long long));
  for (int idle_ms : {0, 5, 50, 500}) {
    (void)hipDeviceSynchronize();
    std::this_thread::sleep_for(std::chrono::milliseconds(idle_ms));
    for (int s = 0; s < 40; ++s) hipLaunchKernelGGL(k, dim3(256), dim3(512), 0, 0, out, t, 3000, s);
    (void)hipDeviceSynchronize();
    unsigned long long h[128];
    (void)hipMemcpy(h, t, sizeof(h), hipMemcpyDeviceToHost);
    printf("after %3d ms idle, MHz of kernels 0..39:", idle_ms);
    for (int s = 0; s < 40; s += 3) printf(" %4.0f", (double)h[2 * s] / (h[2 * s + 1] / 100.0));
    printf("\n");
  }
  return 0;
}
