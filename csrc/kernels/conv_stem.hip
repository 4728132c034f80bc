// Direct packed-tap stem convolution, forward (gfx950 / MI355X): the ResNet 7x7 / stride-2
// stem over a 4-channel input (RGB + a zero channel), K = KH x (8 pixels x 4 channels).
//
// The implicit-GEMM path (conv_gemm.hip, A_CONV64 with Cin == 4) DMAs one filter row's
// 64-byte pixel run per output pixel and k-step: every input pixel crosses L2 -> LDS
// KH x 4 times (7 filter rows x the 4 output columns whose 8-pixel runs cover it at
// stride 2), ~360 MB of L2 -> LDS traffic for the 25.7 MB ResNet-18 input; the launch ran
// at ~6.5 TB/s of that traffic (54 us).  Here a block owns the same 256-pixel M-tile
// (consecutive NHWC output pixels = up to 4 output rows of one image), stages the input
// ROWS those pixels read ONCE (<= 13 rows x 230 pixels x 8 B) plus the whole filter
// (transposed to [Cout][K], ~29 KB), and reads every A fragment straight from the staged
// rows: the 8 consecutive k of a fragment (2 pixels x 4 channels) are 16 contiguous bytes
// of one input row, at pixel 2*ow + 2*chunk of the row (16-byte aligned: even pad / width).
//
// Same tiles, same fragments (lane & 15 = row, lane >> 4 = k chunk), same MFMA order (kh
// ascending, one v_mfma_f32_16x16x32_bf16 per (i, j) and k-step) and the same
// tile::epilogue as conv_gemm_kernel<256, 64, 32> -- so outputs and BatchNorm statistics
// partials (M-tile tm -> replica tm % reps) are bitwise those of the implicit-GEMM path
// (tests/test_conv_gemm_gpu.py::test_stem_direct_bitwise_equals_implicit_gemm).
#include "damd_common.h"
#include "gemm.h"
#include "gemm_tile.h"

#include <algorithm>
#include <cstdlib>

namespace damd {
namespace {

constexpr int NT = 256;
constexpr int SK_MAXU = 2 * 1536;  // 16-B window units: two buffers of 24 KiB (whole 1-KiB DMA pieces)
constexpr int SK_WPITCH = 232 * 2;  // [Cout][K <= 224] bf16 rows padded to 464 B (conflict-free)

__device__ __attribute__((aligned(64))) uint4 g_zero16_stem[4];
// diagnostics (stem_stamps_enable): s_memrealtime per block -- start, filter staged, then
// for its first two tiles: rows landed (after the barrier), MFMAs done, epilogue done
constexpr int kStemStampBlocks = 1024, kStemStamps = 8;
__device__ int g_stem_on;
__device__ unsigned long long g_stem_st[kStemStampBlocks][kStemStamps];

// Persistent blocks (two per CU), each over tiles blockIdx.x, + gridDim.x, ...: the filter
// is transposed into LDS once per block; a tile's input rows arrive by LDS-DMA into one of
// two window buffers -- the next tile's rows are in flight while this tile computes and
// stores.  Window layout: row r, 16-B unit c (pixels 2c, 2c + 1 of the staged row, staged
// pixel q = input column + pad) at unit r * upr + c (upr = Wo + 3): linear, so a wave's
// 64-unit DMA instruction fills 1 KiB contiguously.
template <int EPI>
__global__ __launch_bounds__(NT, 2) void stem_fwd_kernel(GemmArgs a) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  // (KH a compile-time 7: with a runtime filter height the k-step loop's conditional
  // fragment loads made the LDS wait counts conservative -- every k-step waited for the
  // NEXT step's reads too, 3.2 us of MFMA phase per tile instead of ~0.8)
  constexpr int KH = 7, K = KH * 32;
  const int H = a.H, W = a.W, Ho = a.Ho, Wo = a.Wo, N = a.N, pad = a.pad;
  char* wts = smem;                                  // [N = 64][K] bf16, pitch SK_WPITCH
  char* win = smem + 64 * SK_WPITCH;                 // two window buffers of SK_MAXU / 2 units
  float* red = reinterpret_cast<float*>(win + SK_MAXU * 16);
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int hw = Ho * Wo, ntiles = a.M / 256;
  const int upr = Wo + 3;  // 16-B units per staged row (2 Wo + 6 pixels)
  const void* zero = tile::pinned_addr(g_zero16_stem);
  // DMA of tile tt's input rows into buffer b (rows the tile does not read are left stale)
  auto issue = [&](int tt, int b) __attribute__((always_inline)) {
    const int m0 = tt * 256, img = m0 / hw;
    const int oh_a = (m0 - img * hw) / Wo, ih0 = oh_a * a.stride - pad;
    const int last = m0 + 255 - img * hw;
    const int nu = ((last / Wo - oh_a) * a.stride + KH) * upr;
    const uint16_t* x = (const uint16_t*)a.A + (long)img * H * W * 4;
    char* dst = win + b * (SK_MAXU / 2) * 16;
    for (int j = wave; j * 64 < nu; j += 4) {
      const int u = j * 64 + lane;
      const int r = u / upr, c2 = u - r * upr;
      const int ih = ih0 + r, iw = 2 * c2 - pad;
      const bool ok = u < nu && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
      tile::glds16(ok ? (const void*)(x + ((long)ih * W + iw) * 4) : zero, dst + j * 1024);
    }
  };
  const bool stamps = g_stem_on != 0 && blockIdx.x < kStemStampBlocks && t == 0;
  unsigned long long* stp = g_stem_st[stamps ? blockIdx.x : 0];
  if (stamps) stp[0] = __builtin_amdgcn_s_memrealtime();
  if ((int)blockIdx.x < ntiles) issue(blockIdx.x, 0);
  // filter [K][N] (row-major k) -> [N][K]: unit = 8 k x 8 n, 8 row loads, 8 row stores
  {
    const uint16_t* w = (const uint16_t*)a.B;
    for (int u = t; u < (K / 8) * (N / 8); u += NT) {
      const int k0 = 8 * (u / (N / 8)), n0 = 8 * (u % (N / 8));
      uint4 r[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) r[i] = *reinterpret_cast<const uint4*>(w + (long)(k0 + i) * a.ldb + n0);
#pragma unroll
      for (int c = 0; c < 8; ++c) {  // row n0 + c: the 8 k values of column c
        uint32_t o[4];
#pragma unroll
        for (int h = 0; h < 4; ++h) {
          const uint32_t* a0 = reinterpret_cast<const uint32_t*>(&r[2 * h]);
          const uint32_t* a1 = reinterpret_cast<const uint32_t*>(&r[2 * h + 1]);
          const uint32_t lo = (c & 1) ? (a0[c >> 1] >> 16) : (a0[c >> 1] & 0xffffu);
          const uint32_t hi = (c & 1) ? (a1[c >> 1] & 0xffff0000u) : (a1[c >> 1] << 16);
          o[h] = lo | hi;
        }
        *reinterpret_cast<uint4*>(wts + (n0 + c) * SK_WPITCH + k0 * 2) = uint4{o[0], o[1], o[2], o[3]};
      }
    }
  }
  if (stamps) stp[1] = __builtin_amdgcn_s_memrealtime();
  const int g = lane >> 4;
  int it = 0;
  for (int tm = blockIdx.x; tm < ntiles; tm += gridDim.x, ++it) {
    // this tile's rows landed (each wave waits for its own DMA; the epilogue stores of the
    // previous tile sit behind them in the in-order count and drain here too), and every
    // wave is done with the other buffer (the previous tile's fragments)
    // (after the first tile: vmcnt(16) -- the DMA is older than the 16 epilogue stores every
    // wave issued for the previous (always full) tile, so in the in-order count <= 16
    // outstanding means it landed, while those stores and wave 0's statistics atomics stay
    // in flight; vmcnt(0) waited out the atomics' memory-side round trip on every tile)
    if (it == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    __syncthreads();
    if (stamps && it < 2) stp[2 + 3 * it] = __builtin_amdgcn_s_memrealtime();
    if (tm + (int)gridDim.x < ntiles) issue(tm + gridDim.x, (it + 1) & 1);
    const char* cur = win + (it & 1) * (SK_MAXU / 2) * 16;
    const int m0 = tm * 256, img = m0 / hw, oh_a = (m0 - img * hw) / Wo;
    int aoff[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + wave * 64 + i * 16 + (lane & 15) - img * hw;
      const int oh = m / Wo, ow = m - oh * Wo;
      aoff[i] = (oh - oh_a) * a.stride * upr * 16 + (ow * a.stride + 2 * g) * 8;
    }
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 af[2][4], bfr[2][4];
    auto load = [&](int kh) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        af[kh & 1][i] = *reinterpret_cast<const bf16x8*>(cur + aoff[i] + kh * upr * 16);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        bfr[kh & 1][j] =
            *reinterpret_cast<const bf16x8*>(wts + (j * 16 + (lane & 15)) * SK_WPITCH + (kh * 32 + 8 * g) * 2);
    };
    load(0);
#pragma unroll
    for (int kh = 0; kh < KH; ++kh) {
      if (kh + 1 < KH) load(kh + 1);  // the next filter row's reads in flight during these MFMAs
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(bfr[kh & 1][j], af[kh & 1][i], acc[i][j]);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (stamps && it < 2) stp[3 + 3 * it] = __builtin_amdgcn_s_memrealtime();
    tile::epilogue<256, 64, EPI>(a, acc, m0, 0, tm, wave, 0, wave, lane, red);
    if (stamps && it < 2) stp[4 + 3 * it] = __builtin_amdgcn_s_memrealtime();
  }
}

template <int EPI>
hipError_t launch_stem(const GemmArgs& a, size_t lds, hipStream_t s) {
  auto k = stem_fwd_kernel<EPI>;
  static bool attr = false;  // once per instantiation (host-side, before any capture)
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    attr = true;
  }
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
  }
  const int blocks = std::min(a.M / 256, 2 * cus);  // persistent: two per CU
  hipLaunchKernelGGL(k, dim3(blocks), dim3(NT), lds, s, a);
  return hipGetLastError();
}

}  // namespace

hipError_t stem_stamps_enable(int on) {
  if (on) {
    static unsigned long long zeros[kStemStampBlocks][kStemStamps];
    const hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_stem_st), zeros, sizeof(zeros));
    if (e != hipSuccess) return e;
  }
  return hipMemcpyToSymbol(HIP_SYMBOL(g_stem_on), &on, sizeof(int));
}
hipError_t stem_stamps_read(unsigned long long* host, int blocks) {
  if (blocks > kStemStampBlocks) blocks = kStemStampBlocks;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stem_st), (size_t)blocks * kStemStamps * sizeof(unsigned long long));
}

// The stems this kernel takes (else the implicit-GEMM path runs): packed taps (Cin 4, KW'
// 8, K = KH x 32 <= 224), 64 outputs, stride 2, even pad / width, 2 Wo + 6 <= 232 staged
// pixels, whole 256-pixel tiles inside one image (Ho Wo % 256 == 0), at most 4 output rows
// per tile, no split-K, statistics (if any) into fixed-point accumulators, DAMD_STEM_DIRECT
// != 0.
int stem_direct_ok(const GemmArgs& a, int epi, int splits) {
  const char* e = getenv("DAMD_STEM_DIRECT");
  if (e && e[0] == '0') return 0;
  if (a.Cin != 4 || a.KW != 8 || a.KH != 7 || a.K != 7 * 32 || a.N != 64 || a.stride != 2 ||
      a.pad % 2 || a.pad < 0 || a.W % 2 || a.ldb != 64 || a.ldc != 64 || splits != 1)
    return 0;
  if ((a.Ho * a.Wo) % 256 || a.M % 256 || a.M % (a.Ho * a.Wo)) return 0;
  const int rows_max = (a.Wo - 1 + 255) / a.Wo + 1;  // output rows a 256-pixel tile can touch
  const int units = ((rows_max - 1) * a.stride + a.KH) * (a.Wo + 3);
  if (rows_max > 4 || (units + 63) / 64 * 64 > SK_MAXU / 2) return 0;
  if ((epi & (E_SLAB | E_ATOMIC | E_ADD | E_BNRED)) || ((epi & E_STATS) && !a.stats_acc)) return 0;
  return 1;
}

hipError_t stem_direct_launch(const GemmArgs& a, int epi, hipStream_t s) {
  if (!stem_direct_ok(a, epi, 1)) return hipErrorInvalidValue;
  const size_t lds = 64 * SK_WPITCH + SK_MAXU * 16 + 2 * 4 * 64 * sizeof(float);
  switch (epi) {
    case E_BF16: return launch_stem<E_BF16>(a, lds, s);
    case E_BIAS | E_BF16: return launch_stem<E_BIAS | E_BF16>(a, lds, s);
    case E_BIAS | E_RELU | E_BF16: return launch_stem<E_BIAS | E_RELU | E_BF16>(a, lds, s);
    case E_RELU | E_BF16: return launch_stem<E_RELU | E_BF16>(a, lds, s);
    case E_BF16 | E_STATS: return launch_stem<E_BF16 | E_STATS>(a, lds, s);
    case E_BIAS | E_BF16 | E_STATS: return launch_stem<E_BIAS | E_BF16 | E_STATS>(a, lds, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace damd
