// Per-wave instruction cadence on gfx950 (one block, W waves): shader clocks (s_memtime)
// per instruction for dependent / independent fp32 FMA chains, f32 and bf16 MFMA chains,
// DPP reductions, LDS round trips and SALU, plus the clock rate against s_memrealtime.
// Build here:  hipcc -O3 --offload-arch=gfx950 scripts/micro/clock_probe.hip -o build/clock_probe
// GPU box:     ./build/clock_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

enum Mode { FMA_DEP, FMA_IND, MFMA4_DEP, MFMA4_IND2, MFMA4_IND4, MFMA_BF16_DEP, DPP_MAX, LDS_DEP, SALU, NMODES };
static const char* names[] = {"fma dep", "fma indep x4", "mfma f32 16x16x4 dep", "mfma f32 16x16x4 2 chains",
                              "mfma f32 16x16x4 4 chains", "mfma bf16 16x16x32 dep", "dpp row_shr max dep",
                              "lds read dep", "salu add dep"};

template <int M>
__global__ void k(float* out, unsigned long long* t, int n) {
  __shared__ float lds[1024];
  lds[threadIdx.x % 1024] = (float)(threadIdx.x % 64);
  float a = threadIdx.x * 1e-3f, b = 1.0001f, c0 = 0.5f, c1 = 0.25f, c2 = 0.125f, c3 = 0.0625f;
  f32x4 q0 = {0.f, 0.f, 0.f, 0.f}, q1 = q0, q2 = q0, q3 = q0;
  bf16x8 hb;
  for (int i = 0; i < 8; ++i) hb[i] = (__bf16)(0.001f * i);
  int li = threadIdx.x % 64;
  int s = 0;
  __syncthreads();
  const unsigned long long m0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < n; ++i) {
    if constexpr (M == FMA_DEP) {
      for (int u = 0; u < 4; ++u) asm volatile("v_fma_f32 %0, %0, %1, 1.0" : "+v"(a) : "v"(b));
    } else if constexpr (M == FMA_IND) {
      asm volatile("v_fma_f32 %0, %0, %1, 1.0" : "+v"(c0) : "v"(b));
      asm volatile("v_fma_f32 %0, %0, %1, 1.0" : "+v"(c1) : "v"(b));
      asm volatile("v_fma_f32 %0, %0, %1, 1.0" : "+v"(c2) : "v"(b));
      asm volatile("v_fma_f32 %0, %0, %1, 1.0" : "+v"(c3) : "v"(b));
    } else if constexpr (M == MFMA4_DEP) {
      for (int u = 0; u < 4; ++u) q0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, q0, 0, 0, 0);
    } else if constexpr (M == MFMA4_IND2) {
      q0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, q0, 0, 0, 0);
      q1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, q1, 0, 0, 0);
      q0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, q0, 0, 0, 0);
      q1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, q1, 0, 0, 0);
    } else if constexpr (M == MFMA4_IND4) {
      q0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, q0, 0, 0, 0);
      q1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, q1, 0, 0, 0);
      q2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, q2, 0, 0, 0);
      q3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, q3, 0, 0, 0);
    } else if constexpr (M == MFMA_BF16_DEP) {
      for (int u = 0; u < 4; ++u) q0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(hb, hb, q0, 0, 0, 0);
    } else if constexpr (M == DPP_MAX) {
      for (int u = 0; u < 4; ++u)
        a = fmaxf(a, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(a), 0x111, 0xf, 0xf, false)));
    } else if constexpr (M == LDS_DEP) {
      for (int u = 0; u < 4; ++u) li = (int)lds[li];
    } else {
      for (int u = 0; u < 4; ++u) asm volatile("s_add_u32 %0, %0, 1" : "+s"(s));
    }
  }
  const unsigned long long m1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a + c0 + c1 + c2 + c3 + q0[0] + q1[1] + q2[2] + q3[3] + li + s;
  if (threadIdx.x % 64 == 0) {
    t[threadIdx.x / 64 * 2] = m1 - m0;
    t[threadIdx.x / 64 * 2 + 1] = r1 - r0;
  }
}

template <int M>
static void run(float* out, unsigned long long* t, int n) {
  for (int threads : {64, 256, 512}) {
    for (int rep = 0; rep < 2; ++rep) {
      hipLaunchKernelGGL(k<M>, dim3(1), dim3(threads), 0, 0, out, t, n);
      (void)hipDeviceSynchronize();
    }
    unsigned long long h[64];
    (void)hipMemcpy(h, t, sizeof(h), hipMemcpyDeviceToHost);
    const double cyc = (double)h[0], us = h[1] / 100.0;
    printf("%-28s waves %d: %6.2f clk per op (%4.0f MHz)\n", names[M], threads / 64, cyc / (4.0 * n), cyc / us);
  }
}

int main() {
  float* out;
  unsigned long long* t;
  (void)hipMalloc(&out, 1024 * sizeof(float));
  (void)hipMalloc(&t, 64 * sizeof(unsigned long long));
  const int n = 2048;
  run<FMA_DEP>(out, t, n);
  run<FMA_IND>(out, t, n);
  run<MFMA4_DEP>(out, t, n);
  run<MFMA4_IND2>(out, t, n);
  run<MFMA4_IND4>(out, t, n);
  run<MFMA_BF16_DEP>(out, t, n);
  run<DPP_MAX>(out, t, n);
  run<LDS_DEP>(out, t, n);
  run<SALU>(out, t, n);
  return 0;
}
